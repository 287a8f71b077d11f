# hash_to_G2 stage timing at C1's shape (131 messages): map with and without the row exponentiation.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib_np; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/m_$b -o run -- python3 tools/gpu/maptime.py 131 30 > $O/m_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/m_$b/*.db | head -1) > $O/m_$b.csv
done
GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so timeout -k 10 200 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -v -k "hash_to_g2_default or bad_segment" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
echo done > $O/steps.txt
