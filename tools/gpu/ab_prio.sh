# Same-box A/B of the normal contexts' main-chain priority (GBLS_PRIO_MODE 0: highest, 3: middle
# level, leaving the highest to block import): the default C2 line (with its single batch) and the
# C1 leg (block under 16-thread gossip load).  usage: bash tools/gpu/ab_prio.sh TAG [reps]
set -o pipefail
T=${1:?tag}
R=${2:-2}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
python3 -c 'import torch; print("stream priority range", torch.cuda.Stream.priority_range())' > $O/range.txt 2>&1 || true
for r in $(seq 1 $R); do
  for m in 0 3; do
    GBLS_PRIO_MODE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $O/c2_m${m}_$r.txt 2>&1 || exit $?
    GBLS_PRIO_MODE=$m timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/c1_m${m}_$r.txt 2>&1 || exit $?
    echo "mode $m rep $r C2 $(grep -o '"value": [0-9.]*' $O/c2_m${m}_$r.txt | head -2 | tr '\n' ' ') C1 $(grep -o '"value": [0-9.]*' $O/c1_m${m}_$r.txt | head -1) $(grep -o '"block_under_gossip_load": {[^}]*}' $O/c1_m${m}_$r.txt) $(grep -o '"gossip64": {[^}]*}' $O/c1_m${m}_$r.txt)" | tee -a $O/summary.txt
  done
done
