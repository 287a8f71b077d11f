# Stream -> HW queue map of the default C2 command (16-batch leg + single-batch leg) under engine
# knob settings.  usage: bash tools/gpu/queue_map.sh TAG "GBLS_PREWARM=2,0" ...
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  for kv in $cfg; do export "$kv"; done
  timeout -s KILL 150 rocprofv3 --kernel-trace -d $O/t$i -o run -- python3 bench.py --tuning --steps 3 --warmup 2 --no-cpu > $O/t$i.log 2>&1 &&
  { echo "== $cfg"; python3 tools/prof/queues.py $(ls $O/t$i/*.db | head -1); } >> $O/queues.txt || exit $?
  for kv in $cfg; do unset "${kv%%=*}"; done
done
cat $O/queues.txt
