# Row-distributed ml_reduce for small launches: headline + paths tests, C1 (+ kernel trace),
# C2 with the single-batch leg, all on lib_n.
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
export GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so
run 300 pytest.txt python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paths.py -m gpu -x -v --timeout 120 --timeout-method thread
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
run 300 trace_c1.log rocprofv3 --kernel-trace --stats -d $O/trace_c1 -o run -- python3 bench.py --config C1 --steps 20 --warmup 2 --no-cpu
python3 tools/prof/db_stats.py $(ls $O/trace_c1/*.db | head -1) > $O/c1_kernel_stats.csv
run 120 gossip.log python3 tools/gpu/gossip_load.py 3 16
run 300 bench_c2.txt python bench.py --steps 20 --warmup 4 --no-cpu
echo done >> $O/steps.txt
