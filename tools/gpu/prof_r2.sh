# round-2 profile of the default bench (C2) and of C5: kernel trace + PMC passes
set -o pipefail
O=gpurun_out/prof_r2
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
C5="python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace5 -o run -- $C5 > $O/trace5.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/q1 -o run -- $C5 > $O/q1.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/trace5/*.db | head -1) > $O/c5_kernel_stats.csv &&
python3 tools/prof/pmc_table.py $O/c5_pmc.csv $(ls $O/q1/*.db | head -1)
