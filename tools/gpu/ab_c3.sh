# A/B of engine knobs on the C3 leg (10 000 x 512-key fast_aggregate_verify), twice each.
# usage: bash tools/gpu/ab_c3.sh TAG "NAME=VALUE ..." ...
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
i=0
for rep in 1 2; do
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --tuning > $O/ab3_$i.txt 2>&1 || exit $?
  echo "$cfg :: C3 $(grep -o '"value": [0-9.]*' $O/ab3_$i.txt | head -1)" | tee -a $O/ab3.txt
done
done
