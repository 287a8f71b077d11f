# C4 partials debug, then the GPU suite without the 2-rank C4 test, then the bench legs
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/gpu/dbg_c4.py 256 > $O/dbg_c4_256.txt 2>&1 &&
timeout -k 10 200 python tools/gpu/dbg_c4.py 2048 > $O/dbg_c4_2048.txt 2>&1 ;
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not c4_epoch" > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu > $O/bench_c3.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/bench_c4.txt 2>&1 &&
timeout -k 10 400 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu > $O/bench_c5_shard.txt 2>&1 &&
timeout -k 10 500 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5.txt 2>&1
