# per-kernel regime thresholds, first line slice before the join; default bench = 12 batches
set -o pipefail
O=gpurun_out/r2v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
for b in 1 4 8 16; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches $b > $O/bench_b$b.txt 2>&1 || exit 1
done &&
timeout -k 10 300 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu > $O/bench_c5_shard.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5.txt 2>&1
