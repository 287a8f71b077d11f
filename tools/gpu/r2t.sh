# in-flight submissions x batches per submission (default bench shape choice)
set -o pipefail
O=gpurun_out/r2t
mkdir -p $O
export TMPDIR=/tmp
for cfg in "1 4" "2 4" "3 4" "2 2" "2 8" "1 8"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 12 --warmup 3 --no-cpu --inflight $1 --batches $2 > $O/bench_i$1_b$2.txt 2>&1 || exit 1
done
