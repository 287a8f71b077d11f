# Cofactor clearing form for 2048-4096-point launches: rows (default) vs quad gangs
# (GBLS_ROW_CLEAR_MAX=1024): C2 with its single-batch leg, C4, C1 (unaffected), x2.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for m in 4096 1024; do
    GBLS_ROW_CLEAR_MAX=$m timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --tuning > $O/c2_${m}_$i.txt 2>&1 || exit $?
    GBLS_ROW_CLEAR_MAX=$m timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 2 --no-cpu --tuning > $O/c4_${m}_$i.txt 2>&1 || exit $?
    echo "rowmax $m C2 $(tail -n1 $O/c2_${m}_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["single_batch"]["value"])') C4 $(tail -n1 $O/c4_${m}_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')" >> $O/res.txt
  done
done
echo done >> $O/res.txt
