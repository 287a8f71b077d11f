# SIMD-balanced cyclotomic rows (final verdict timing), the 16-thread gossip load alone with a
# kernel trace (how the coalescer merges), C1 and C2 on lib_n.
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
run 120 fexp.log rocprofv3 --kernel-trace --stats -d $O/fexp -o run -- python3 tools/gpu/fexp_time.py 1 40
python3 tools/prof/db_stats.py $(ls $O/fexp/*.db | head -1) > $O/fexp.csv
run 120 gossip.log python3 tools/gpu/gossip_load.py 3 16
run 120 gossip_trace.log rocprofv3 --kernel-trace -d $O/gtrace -o run -- python3 tools/gpu/gossip_load.py 2 16
python3 tools/prof/merge_sizes.py $(ls $O/gtrace/*.db | head -1) > $O/gossip_merges.txt
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
run 300 bench_c2.txt python bench.py --steps 20 --warmup 4 --no-cpu
echo done >> $O/steps.txt
