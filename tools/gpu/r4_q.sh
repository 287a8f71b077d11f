# C4 bisection: commit 9166118's build (lib_old) against lib_n, same box.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
for b in lib_old lib_n lib_old; do
  GBLS_LIB=grandine_amd/$b/libgrandine_bls.so timeout -k 10 300 $B > $O/c4_$b.txt 2>&1 || exit $?
  echo "$b $(tail -n1 $O/c4_$b.txt | cut -c1-150)" >> $O/res.txt
done
echo done >> $O/res.txt
