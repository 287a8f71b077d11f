# pipelining experiment: in-flight submissions x batches per submission
set -o pipefail
O=gpurun_out/r2n
mkdir -p $O
export TMPDIR=/tmp
for cfg in "1 2" "2 1" "2 2" "2 4" "3 2" "4 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 12 --warmup 3 --no-cpu --inflight $1 --batches $2 > $O/bench_i$1_b$2.txt 2>&1 || exit 1
done
