# safegcd fp_inv (lib_n) vs the r03 binary extended Euclid (lib_bg): C4 and C2 lines, C4 kernel traces.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
for b in lib_n lib_bg; do
  export GBLS_LIB=grandine_amd/$b/libgrandine_bls.so
  timeout -k 10 300 $B > $O/c4_$b.txt 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/c2_$b.txt 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$b -o run -- $B > $O/tr_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/tr_$b/*.db | head -1) > $O/c4_stats_$b.csv
done
echo done > $O/steps.txt
