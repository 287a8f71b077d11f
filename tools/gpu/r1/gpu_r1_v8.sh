set -o pipefail
V=${V:-v8}
mkdir -p gpurun_out/$V
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$V/pytest_gpu.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$V/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/$V/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$V/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/$V/pmc_write.log 2>&1 &&
python tools/prof/pmc_bytes.py gpurun_out/$V/pmc_fetch/run_results.db gpurun_out/$V/pmc_write/run_results.db > profiles/r01/pmc_bytes.csv &&
cp profiles/r01/pmc_bytes.csv gpurun_out/$V/pmc_bytes.csv &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 4096 > gpurun_out/$V/bench.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$V/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/$V/prof.log 2>&1
