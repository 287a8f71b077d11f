# Timeline of one single-batch (4096-set) C2 step, 1 in flight.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run -- python3 bench.py --batches 1 --inflight 1 --steps 6 --warmup 2 --no-cpu --no-single > $O/tr.log 2>&1 || exit $?
python3 tools/prof/db_stats.py $(ls $O/tr/*.db | head -1) > $O/stats.csv
python3 tools/prof/timeline.py $(ls $O/tr/*.db | head -1) -3 k_h2c_field > $O/timeline.txt || true
tail -n1 $O/tr.log > $O/line.json
echo done > $O/steps.txt
