# Row product with two accumulator chains (lib_n) vs one (lib_oa): hash_to_G2 stages at 131
# messages, the final verdict, C1; then the headline + paths tests on lib_n.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib_oa; do
  export GBLS_LIB=grandine_amd/$b/libgrandine_bls.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/m_$b -o run -- python3 tools/gpu/maptime.py 131 30 > $O/m_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/m_$b/*.db | head -1) > $O/m_$b.csv
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/f_$b -o run -- python3 tools/gpu/fexp_time.py 1 40 > $O/f_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/f_$b/*.db | head -1) > $O/f_$b.csv
  timeout -k 10 300 python3 bench.py --config C1 --steps 30 --warmup 5 > $O/c1_$b.txt 2>&1 || exit $?
done
GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paths.py tests/test_gpu_w4.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
echo done > $O/steps.txt
