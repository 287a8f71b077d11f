# Wave-parallel easy-part inversion: final-verdict timing, the headline tests, C1 on lib_n.
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
GBLS_LIB=$N run 120 fexp_lib_n.log rocprofv3 --kernel-trace --stats -d $O/fexp_lib_n -o run -- python3 tools/gpu/fexp_time.py 1 40
python3 tools/prof/db_stats.py $(ls $O/fexp_lib_n/*.db | head -1) > $O/fexp_lib_n.csv
GBLS_LIB=$N run 300 pytest_headline_n.txt python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paths.py -m gpu -x -v --timeout 120 --timeout-method thread
GBLS_LIB=$N run 300 bench_c1_n.txt python bench.py --config C1 --steps 40 --warmup 5
echo done >> $O/steps.txt
