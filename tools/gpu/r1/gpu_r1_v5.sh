set -o pipefail
mkdir -p gpurun_out/v5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v5/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 4096 > gpurun_out/v5/bench.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v5/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/v5/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/v5/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/v5/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/v5/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/v5/pmc_write.log 2>&1
