# C4 consistency (three bench lines in one call) and its kernel trace.
# usage: bash tools/gpu/c4_runs.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/bench_c4_$i.txt 2>&1 || exit $?
  echo "run $i $(grep -o '"value": [0-9.]*' $O/bench_c4_$i.txt | head -1)" >> $O/c4.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config C4 --steps 4 --warmup 1 --no-cpu > $O/trace_c4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/trace_c4/*.db | head -1) > $O/c4_kernel_stats.csv
