# inversion-free final verdict: full GPU suite + C2 + C3
set -o pipefail
O=gpurun_out/r2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 1 > $O/bench_c3.txt 2>&1
