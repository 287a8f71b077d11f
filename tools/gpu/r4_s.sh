# C4 bisection: current tree with the 9166118 final-verdict kernel (lib_of) vs lib_n vs lib_old.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
for b in lib_of lib_n lib_old lib_of; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 $B > $O/c4_$b.txt 2>&1 || exit $?
  echo "$b $(tail -n1 $O/c4_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/res.txt
done
echo done >> $O/res.txt
