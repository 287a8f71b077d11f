# default shape sweep after restoring the 32768 lane thresholds
set -o pipefail
O=gpurun_out/r2x
mkdir -p $O
export TMPDIR=/tmp
for cfg in "1 12" "2 12" "1 10" "1 14" "2 6"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --inflight $1 --batches $2 > $O/bench_i$1_b$2.txt 2>&1 || exit 1
done
