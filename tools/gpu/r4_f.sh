# Cyclotomic final exponentiation (experiment build lib_n) against the r4 default build: the
# GPU suite on lib_n, C1/C2 bench lines of both builds, the pipeline / block-hold A/B on the
# default build, and a kernel trace of the C1 command on lib_n.
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
N=grandine_amd/lib_n/libgrandine_bls.so
GBLS_LIB=$N run 300 pytest_headline_n.txt python -u -m pytest tests/test_gpu_headline.py -m gpu -x -v --timeout 120 --timeout-method thread
GBLS_LIB=$N run 300 bench_c1_n.txt python bench.py --config C1 --steps 40 --warmup 5
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
GBLS_LIB=$N run 300 bench_c2_n.txt python bench.py --steps 20 --warmup 4 --no-cpu
run 300 bench_c2.txt python bench.py --steps 20 --warmup 4 --no-cpu
GBLS_PIPELINE=0 run 300 bench_c2_nopipe.txt python bench.py --steps 20 --warmup 4 --no-cpu --no-single --tuning
GBLS_BLOCK_HOLD=0 run 300 bench_c1_nohold.txt python bench.py --config C1 --steps 40 --warmup 5 --tuning
GBLS_LIB=$N run 300 trace_c1_n.log rocprofv3 --kernel-trace --stats -d $O/trace_c1_n -o run -- python3 bench.py --config C1 --steps 20 --warmup 2 --no-cpu
python3 tools/prof/db_stats.py $(ls $O/trace_c1_n/*.db | head -1) > $O/c1_n_kernel_stats.csv
GBLS_LIB=$N run 900 pytest_gpu_n.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done >> $O/steps.txt
