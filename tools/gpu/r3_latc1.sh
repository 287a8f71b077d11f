# latency traces (gossip 64 / 1024, C1 block) and the C1 bench only
set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
bash tools/gpu/r3_lat.sh $T/lat &&
timeout -k 10 300 python bench.py --config C1 --steps 100 --warmup 10 --no-cpu > gpurun_out/$T/bench_c1.txt 2>&1
