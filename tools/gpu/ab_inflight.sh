# Submissions in flight: C3 at 1 and 2, C2 at 2 and 3, twice each, one box.
# usage: bash tools/gpu/ab_inflight.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for d in 1 2; do
    timeout -k 10 200 python bench.py --config C3 --steps 4 --warmup 2 --inflight $d > $O/c3_d${d}_$r.txt 2>&1 || exit $?
    echo "C3 inflight $d run $r $(grep -o '"value": [0-9.]*' $O/c3_d${d}_$r.txt | head -1)" | tee -a $O/ab_inflight.txt
  done
  for d in 2 3; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --inflight $d > $O/c2_d${d}_$r.txt 2>&1 || exit $?
    echo "C2 inflight $d run $r $(grep -o '"value": [0-9.]*' $O/c2_d${d}_$r.txt | head -1)" | tee -a $O/ab_inflight.txt
  done
done
