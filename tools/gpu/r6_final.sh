# Round-6 final measurements on one GPU: the GPU suite and smoke, every config's bench line
# (the default command with its CPU baseline leg), C4 three times, the default command's
# kernel trace (stats, join delays) and PMC passes (instructions, LDS/waits, HBM bytes).
# usage: bash tools/gpu/r6_final.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu"
step() { echo "$1 $(date +%T)"; }
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
step bench
timeout -k 10 300 python bench.py > $O/bench_default.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_c2.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 > $O/bench_c3.txt 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/bench_c4_$i.txt 2>&1 || exit $?
done
timeout -k 10 400 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 > $O/bench_c5_shard.txt 2>&1 || exit $?
timeout -k 10 500 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1 || exit $?
for f in $O/bench_*.txt; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $B > $O/trace.log 2>&1 || exit $?
python3 tools/prof/db_stats.py $(ls $O/trace/*.db | head -1) > $O/c2_kernel_stats.csv &&
python3 tools/prof/join_wait.py $(ls $O/trace/*.db | head -1) 60000 > $O/c2_join_wait.txt &&
python3 tools/prof/timeline.py $(ls $O/trace/*.db | head -1) 3 k_mv_g1mul > $O/c2_timeline.txt || exit $?
tail -1 $O/c2_join_wait.txt
step pmc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- $B > $O/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU -d $O/p2 -o run -- $B > $O/p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $B > $O/p3.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run -- $B > $O/p4.log 2>&1 || exit $?
python3 tools/prof/pmc_table.py $O/c2_pmc.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) &&
python3 tools/prof/pmc_table.py --largest $O/c2_pmc_largest.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) &&
python3 tools/prof/pmc_bytes.py --largest $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) > $O/c2_pmc_bytes.csv || exit $?
step done
