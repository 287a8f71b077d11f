# latency knob sweep: C1 leg (block, gossip64 serial and 16 threads) per env setting
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
k=0
for e in "GBLS_CU_SPLIT=0" "GBLS_CU_SPLIT=1" "GBLS_CU_SPLIT=2" "GBLS_LEADERS=4" "GBLS_LEADERS=8" "GBLS_LEADERS=8 GBLS_CU_SPLIT=2"; do
  k=$((k + 1))
  echo "$e" > $O/knob_$k.txt
  env $e timeout -k 10 200 python bench.py --config C1 --steps 60 --warmup 5 --no-cpu --tuning >> $O/knob_$k.txt 2>&1 || exit 1
done
