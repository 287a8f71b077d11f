# grouped single checks: the FAV parity tests (grouped vs per-check, C3 full size vs the C
# oracle), the whole GPU suite, the C3 bench leg and a kernel trace of one C3 step.
# usage: bash tools/gpu/r3_c3.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -k "fast_aggregate" tests/test_gpu_paths.py -x -v --timeout 240 --timeout-method thread -m gpu > $O/pytest_fav.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu > $O/bench_c3.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c3 -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu > $O/c3_prof.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
