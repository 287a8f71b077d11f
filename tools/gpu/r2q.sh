# row aggregation (k_aggregate_rows): GPU suite + C3/C4 + C2
set -o pipefail
O=gpurun_out/r2q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_c2b1.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > $O/bench_c4.txt 2>&1
