# Row product with two accumulator chains (lib_n) vs one (lib_oa), current tree: C2 x3 each, C1.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for b in lib_n lib_oa; do
    GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-cpu > $O/c2_${b}_$i.txt 2>&1 || exit $?
    echo "$b C2 $(tail -n1 $O/c2_${b}_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["single_batch"]["value"])')" >> $O/res.txt
  done
done
for b in lib_n lib_oa; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 python3 bench.py --config C1 --steps 30 --warmup 5 > $O/c1_$b.txt 2>&1 || exit $?
  echo "$b C1 $(tail -n1 $O/c1_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["gossip64"])')" >> $O/res.txt
done
echo done >> $O/res.txt
