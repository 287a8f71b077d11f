# A/B of engine knobs over the bench legs: C2 (+ its single-batch leg), C1 (block p50 / p99, gossip),
# C3, C4 -- one line per knob set in ab_all.txt.  usage: bash tools/gpu/ab_all.sh TAG "NAME=VALUE ..." ...
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --tuning > $O/c2_$i.txt 2>&1 || exit $?
  env $cfg timeout -k 10 300 python bench.py --config C1 --steps 20 --warmup 5 --tuning > $O/c1_$i.txt 2>&1 || exit $?
  env $cfg timeout -k 10 200 python bench.py --config C3 --steps 3 --warmup 1 --tuning > $O/c3_$i.txt 2>&1 || exit $?
  env $cfg timeout -k 10 200 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_$i.txt 2>&1 || exit $?
  echo "$cfg :: C2 $(grep -o '"value": [0-9.]*' $O/c2_$i.txt | head -1) single $(grep -o '"single_batch": {[^}]*}' $O/c2_$i.txt | grep -o '"value": [0-9.]*') C1 $(grep -o '"value": [0-9.]*' $O/c1_$i.txt | head -1) C1p99 $(grep -o '"p99_ms": [0-9.]*' $O/c1_$i.txt | head -1) C3 $(grep -o '"value": [0-9.]*' $O/c3_$i.txt | head -1) C4 $(grep -o '"value": [0-9.]*' $O/c4_$i.txt | head -1)" | tee -a $O/ab_all.txt
done
