# A/B of engine knobs on the default C2 line (with its single-batch leg) and the C4 epoch:
# for each "NAME=VALUE ..." argument, `bench.py --tuning` runs of both.  usage:
# bash tools/gpu/ab_c2c4.sh TAG "GBLS_PREWARM=0" "GBLS_SYNC_ALLOC=1" ...   (one line per run in ab.txt)
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
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --tuning > $O/ab_$i.txt 2>&1 || exit $?
  env $cfg timeout -k 10 200 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/ab4_$i.txt 2>&1 || exit $?
  echo "$cfg :: C2 $(grep -o '"value": [0-9.]*' $O/ab_$i.txt | head -1) single $(grep -o '"single_batch": {[^}]*}' $O/ab_$i.txt | grep -o '"value": [0-9.]*') C4 $(grep -o '"value": [0-9.]*' $O/ab4_$i.txt | head -1)" | tee -a $O/ab.txt
done
done
