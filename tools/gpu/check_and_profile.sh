# GPU suite + default bench (with the CPU baseline) + C1 latency leg, then the rocprofv3
# evidence for the default bench command: kernel trace/stats and PMC passes (VALU instructions
# and busy, LDS bank conflicts, HBM bytes), one counter group per run.
# usage: bash tools/gpu/check_and_profile.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_b1.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $B > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- $B > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU -d $O/p2 -o run -- $B > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $B > $O/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run -- $B > $O/p4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/trace/*.db | head -1) > $O/c2_kernel_stats.csv &&
python3 tools/prof/pmc_table.py $O/c2_pmc.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) &&
python3 tools/prof/pmc_bytes.py $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) > $O/c2_pmc_bytes.csv &&
python3 tools/prof/timeline.py $(ls $O/trace/*.db | head -1) 3 k_mv_g1mul > $O/c2_timeline.txt
