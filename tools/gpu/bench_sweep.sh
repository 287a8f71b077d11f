# C2 bench sweep over (batches per step, submissions in flight, engine env knobs): one JSON
# line per point.  A point is B:I or B:I:K=V,K=V (e.g. 16:2:GBLS_LINE_BUDGET_MB=4096).
# usage: bash tools/gpu/bench_sweep.sh TAG "16:2 16:2:GBLS_ML_G=72 ..."  (gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
k=0
for p in ${2:?points}; do
  b=$(echo $p | cut -d: -f1); i=$(echo $p | cut -d: -f2); e=$(echo $p | cut -s -d: -f3 | tr , ' ')
  k=$((k + 1))
  echo "$p" > $O/point_$k.txt
  env $e timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --tuning --batches $b --inflight $i >> $O/point_$k.txt 2>&1 || exit 1
done
