# Final-verdict phase breakdown by variant builds (timing only): full, no inversion, easy part
# only, doubled cyclotomic squarings.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib_v1 lib_v2 lib_v3; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/fexp_$b -o run -- python3 tools/gpu/fexp_time.py 1 40 > $O/fexp_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/fexp_$b/*.db | head -1) > $O/fexp_$b.csv
done
echo done >> $O/steps.txt
