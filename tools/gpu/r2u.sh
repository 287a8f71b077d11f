# batches per submission at one submission in flight (the multi-GPU bench shape)
set -o pipefail
O=gpurun_out/r2u
mkdir -p $O
export TMPDIR=/tmp
for b in 12 16 24; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches $b > $O/bench_b$b.txt 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 16 --inflight 2 > $O/bench_i2_b16.txt 2>&1
