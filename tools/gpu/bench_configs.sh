# Bench legs of the other BASELINE configs on one GPU: C3, C4, C5 (2^20 sets) and the
# per-GPU C5 shard of an 8-GPU run (131072 sets).  usage: bash tools/gpu/bench_configs.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 > $O/bench_c3.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 > $O/bench_c4.txt 2>&1 &&
timeout -k 10 400 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 > $O/bench_c5_shard.txt 2>&1 &&
timeout -k 10 500 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1
