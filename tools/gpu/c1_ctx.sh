# Block under gossip load vs the contexts the C1 leg creates (GBLS_TRACE_STALLS=1 prints every
# context creation): is the slow mode (block p50 ~6.5 ms instead of ~3.7) a queue-sharing effect
# of extra contexts?  usage: bash tools/gpu/c1_ctx.sh TAG [runs]
set -o pipefail
T=${1:?tag}
N=${2:-4}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in $(seq 1 $N); do
  GBLS_TRACE_STALLS=1 timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/c1_$i.txt 2> $O/c1_$i.err || exit $?
  echo "run $i ctx_created $(grep -c 'creates ctx' $O/c1_$i.err) block $(grep -c 'class 1' $O/c1_$i.err) $(grep -o '"block_under_gossip_load": {[^}]*}' $O/c1_$i.txt)" | tee -a $O/summary.txt
  grep 'creates ctx' $O/c1_$i.err > $O/c1_${i}_ctx.txt || true
  rm -f $O/c1_$i.err
done
