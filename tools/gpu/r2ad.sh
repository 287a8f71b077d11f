# row clearing for tiny launches; default bench = 16 batches: GPU suite + default + C1 + single
set -o pipefail
O=gpurun_out/r2ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_b1.txt 2>&1
