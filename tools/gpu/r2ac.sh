# batch-count sweep after the first-slice-before-join change; C1 without row clearing
set -o pipefail
O=gpurun_out/r2ac
mkdir -p $O
export TMPDIR=/tmp
for b in 12 16 20; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches $b > $O/bench_b$b.txt 2>&1 || exit 1
done &&
timeout -k 10 300 python3 bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1
