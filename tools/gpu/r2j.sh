# hardware queues per process: 4 (default) vs 8 vs 16
set -o pipefail
O=gpurun_out/r2j
mkdir -p $O
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2_q$q.txt 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 8 > $O/bench_c2b8_q$q.txt 2>&1 || exit 1
done
