# round-2 final profile: default bench (C2, 4 batches of 4096) and the C5 shard (131072 sets):
# kernel trace + PMC passes (VALU instructions / busy, LDS, HBM bytes), one pass per run
set -o pipefail
O=gpurun_out/prof_r2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $B > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- $B > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU -d $O/p2 -o run -- $B > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $B > $O/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run -- $B > $O/p4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/trace/*.db | head -1) > $O/c2_kernel_stats.csv &&
python3 tools/prof/pmc_table.py $O/c2_pmc.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) &&
python3 tools/prof/pmc_bytes.py $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) > $O/c2_pmc_bytes.csv &&
python3 tools/prof/timeline.py $(ls $O/trace/*.db | head -1) 3 k_mv_g1mul > $O/c2_timeline.txt &&
C5="python3 bench.py --config C5 --sets 131072 --steps 3 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace5 -o run -- $C5 > $O/trace5.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/q1 -o run -- $C5 > $O/q1.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/q3 -o run -- $C5 > $O/q3.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/q4 -o run -- $C5 > $O/q4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/trace5/*.db | head -1) > $O/c5_kernel_stats.csv &&
python3 tools/prof/pmc_table.py $O/c5_pmc.csv $(ls $O/q1/*.db | head -1) $(ls $O/q3/*.db | head -1) $(ls $O/q4/*.db | head -1) &&
python3 tools/prof/pmc_bytes.py $(ls $O/q3/*.db | head -1) $(ls $O/q4/*.db | head -1) > $O/c5_pmc_bytes.csv
