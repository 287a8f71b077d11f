# lazy Karatsuba operand sums: GPU suite + default bench + single batch + C5 shard
set -o pipefail
O=gpurun_out/r2aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_b1.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu > $O/bench_c5_shard.txt 2>&1
