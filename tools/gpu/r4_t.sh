# Lane-form extra-pair lines in the throughput regime + MSM threshold 4096 (lib_n) vs lib:
# C2 x2, C5 shard, C4 x2.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib lib_n lib; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-cpu > $O/c2_$b.txt 2>&1 || exit $?
  echo "$b C2 $(tail -n1 $O/c2_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["single_batch"]["value"])')" >> $O/res.txt
done
for b in lib_n lib; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 python3 bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu > $O/c5s_$b.txt 2>&1 || exit $?
  echo "$b C5 shard $(tail -n1 $O/c5s_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/res.txt
done
for i in 1 2; do
  GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 2 --no-cpu > $O/c4_$i.txt 2>&1 || exit $?
  echo "lib_n C4 $(tail -n1 $O/c4_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/res.txt
done
echo done >> $O/res.txt
