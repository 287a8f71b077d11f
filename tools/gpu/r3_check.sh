set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C1 --steps 200 --warmup 10 --no-cpu > $O/bench_c1.txt 2>&1
