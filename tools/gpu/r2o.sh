# lane variants of clear/lines for launches >= 32768: GPU suite, C2 B=4/B=8, C5
set -o pipefail
O=gpurun_out/r2o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 8 > $O/bench_c2b8.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5.txt 2>&1
