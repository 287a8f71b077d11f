# bucket MSM: forced-MSM parity subprocess, C5 with MSM, C2 with/without forced MSM
set -o pipefail
O=gpurun_out/r2d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -x -v -k "msm or partials or zero_scalar" --timeout 200 --timeout-method thread > $O/pytest_msm.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_c2.txt 2>&1 &&
GBLS_MSM_MIN=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_c2_msm.txt 2>&1
