# C4 repeatability: default x3 and bucket-MSM-off x2 on lib_n, default x1 on lib.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
for i in 1 2 3; do GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so timeout -k 10 300 $B > $O/c4_$i.txt 2>&1 || exit $?; done
for i in 1 2; do GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so GBLS_MSM_MIN=4097 timeout -k 10 300 $B --tuning > $O/c4_nomsm_$i.txt 2>&1 || exit $?; done
timeout -k 10 300 $B > $O/c4_lib.txt 2>&1 || exit $?
echo done > $O/steps.txt
