# round 2, first GPU pass: full GPU suite, then one bench line per config
set -o pipefail
V=${V:-r2a}
O=gpurun_out/$V
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 > $O/bench_c3.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 > $O/bench_c4.txt 2>&1 &&
timeout -k 10 400 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C1 --steps 20 --warmup 3 > $O/bench_c1.txt 2>&1
