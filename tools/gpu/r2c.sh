# map without GCD inversion; C2 at in-flight depth 1/2/4/8
set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_smoke.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
for d in 1 2 4 8; do timeout -k 10 200 python bench.py --steps 24 --warmup 3 --no-cpu --inflight $d > $O/bench_c2_d$d.txt 2>&1 || exit 1; done &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1
