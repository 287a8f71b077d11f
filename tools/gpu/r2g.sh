# quad G1 products (no inversion), quad G2 chunk sums: GPU suite + C2 (default and 1 batch) + C5
set -o pipefail
O=gpurun_out/r2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu --batches 1 > $O/bench_c2_b1.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1
