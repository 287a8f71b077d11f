# iteration check: GPU suite, then the latency-shape kernel traces (tools/gpu/r3_lat.sh) and
# the default C2 bench line.  usage: bash tools/gpu/r3_iter.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
bash tools/gpu/r3_lat.sh $T/lat &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C1 --steps 100 --warmup 10 --no-cpu > $O/bench_c1.txt 2>&1
