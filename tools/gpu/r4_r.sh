# C4 kernel traces of lib_old (9166118) and lib_n: per-kernel stats and one step's timeline each.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
for b in lib_old lib_n; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$b -o run -- $B > $O/tr_$b.log 2>&1 || exit $?
  python3 tools/prof/db_stats.py $(ls $O/tr_$b/*.db | head -1) > $O/stats_$b.csv
  python3 tools/prof/timeline.py $(ls $O/tr_$b/*.db | head -1) 8 k_h2c_field > $O/timeline_$b.txt || true
done
echo done >> $O/steps.txt
