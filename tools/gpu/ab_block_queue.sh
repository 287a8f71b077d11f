# (Needs the build that had the GBLS_BLOCK_QUEUE knob, removed after this A/B: profiles/r06/zz_ab_block_queue.txt.)
# Same-box A/B of GBLS_BLOCK_QUEUE (block import on one high-priority stream that keeps a hardware
# queue to itself; normal contexts created on demand take their main chain low): the C1 leg
# (idle block, block under 16-thread gossip load) R times per mode, the default C2 line once.
# usage: bash tools/gpu/ab_block_queue.sh TAG [reps]
set -o pipefail
T=${1:?tag}
R=${2:-3}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for m in 0 1; do
    GBLS_BLOCK_QUEUE=$m timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/c1_q${m}_$r.txt 2>&1 || exit $?
    echo "queue $m rep $r C1 $(grep -o '"value": [0-9.]*' $O/c1_q${m}_$r.txt | head -1) p99 $(grep -o '"p99_ms": [0-9.]*' $O/c1_q${m}_$r.txt | head -1) $(grep -o '"block_under_gossip_load": {[^}]*}' $O/c1_q${m}_$r.txt) $(grep -o '"gossip64_under_back_to_back_blocks": {[^}]*}' $O/c1_q${m}_$r.txt)" | tee -a $O/summary.txt
  done
done
for m in 0 1; do
  GBLS_BLOCK_QUEUE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $O/c2_q$m.txt 2>&1 || exit $?
  echo "queue $m C2 $(grep -o '"value": [0-9.]*' $O/c2_q$m.txt | head -2 | tr '\n' ' ')" | tee -a $O/summary.txt
done
