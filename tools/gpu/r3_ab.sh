# correctness of the headline-regime kernels, then the default bench line (A/B iterations)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1
