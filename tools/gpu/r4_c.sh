# Round-4 main measurement pass.  Each GPU step has its own time limit; a step that fails
# ordinarily (exit 1: a test or assertion) lets the next one run, but a time limit, an abort
# or a fault (exit 124 / 134 / 137 / 139) ends the script at once.
# usage: bash tools/gpu/r4_c.sh TAG [quick]
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() {  # run LIMIT OUTFILE CMD...
  local lim=$1 out=$2
  shift 2
  timeout -k 10 $lim "$@" > $O/$out 2>&1
  local rc=$?
  echo "$out rc=$rc" >> $O/steps.txt
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $out"; exit $rc ;; esac
  return 0
}
B="python3 bench.py --steps 10 --warmup 2 --no-cpu --no-single"
run 900 pytest_gpu.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 bench_c2.txt python bench.py --steps 10 --warmup 2
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
run 300 bench_c3.txt python bench.py --config C3 --steps 5 --warmup 1 --no-cpu
run 300 bench_c4.txt python bench.py --config C4 --steps 10 --warmup 2 --no-cpu
run 400 bench_c5_shard.txt python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu
run 500 bench_c5.txt python bench.py --config C5 --steps 3 --warmup 1 --no-cpu
if [ "$2" = quick ]; then exit 0; fi
# block import under gossip load: reserved CUs (default 1 in 4) vs none
GBLS_BLOCK_RESERVE=0 run 300 bench_c1_noreserve.txt python bench.py --config C1 --steps 40 --warmup 5 --tuning
GBLS_BLOCK_RESERVE=8 run 300 bench_c1_reserve8.txt python bench.py --config C1 --steps 40 --warmup 5 --tuning
# line-buffer budget (n3): event slices small enough to stay in the Infinity Cache
for mb in 1024 256 128; do
  GBLS_LINE_BUDGET_MB=$mb run 300 bench_c2_budget$mb.txt $B --tuning
done
# kernel trace and counters of the default command without the one-batch leg
run 300 trace.log rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $B
run 120 p1.log rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- $B
run 120 p2.log rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU -d $O/p2 -o run -- $B
run 120 p3.log rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $B
run 120 p4.log rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run -- $B
python3 tools/prof/db_stats.py $(ls $O/trace/*.db | head -1) > $O/c2_kernel_stats.csv
python3 tools/prof/pmc_table.py $O/c2_pmc.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1)
python3 tools/prof/pmc_bytes.py $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) > $O/c2_pmc_bytes.csv
python3 tools/prof/timeline.py $(ls $O/trace/*.db | head -1) 3 k_mv_g1mul > $O/c2_timeline.txt
echo done >> $O/steps.txt
