# Final-verdict kernel timing across builds (old generic/inversion-free, GS + inversion, GS
# without the inversion, generic squarings + inversion), then C1/C2 on lib_n (safegcd fp_inv
# everywhere, pipeline removed) and the GPU suite on it.
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
for b in lib lib_n lib_v1 lib_v2; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so run 120 fexp_$b.log rocprofv3 --kernel-trace --stats -d $O/fexp_$b -o run -- python3 tools/gpu/fexp_time.py 1 40
  python3 tools/prof/db_stats.py $(ls $O/fexp_$b/*.db | head -1) > $O/fexp_$b.csv
done
N=grandine_amd/lib_n/libgrandine_bls.so
GBLS_LIB=$N run 300 bench_c1_n.txt python bench.py --config C1 --steps 40 --warmup 5
GBLS_LIB=$N run 300 bench_c2_n.txt python bench.py --steps 20 --warmup 4 --no-cpu
GBLS_LIB=$N run 300 trace_c2_n.log rocprofv3 --kernel-trace --stats -d $O/trace_c2_n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-single
python3 tools/prof/db_stats.py $(ls $O/trace_c2_n/*.db | head -1) > $O/c2_n_kernel_stats.csv
GBLS_LIB=$N run 900 pytest_gpu_n.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done >> $O/steps.txt
