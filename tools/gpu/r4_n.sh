# C4 (one epoch, 2048 committees) variants: default, bucket MSM off below 4097 sets, 3 in flight;
# C1 with the time-window gossip measurement and merge target 768.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
export GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so
B="python bench.py --config C4 --steps 10 --warmup 2 --no-cpu"
timeout -k 10 300 $B > $O/c4.txt 2>&1 || exit $?
GBLS_MSM_MIN=4097 timeout -k 10 300 $B --tuning > $O/c4_nomsm.txt 2>&1 || exit $?
timeout -k 10 300 $B --inflight 3 > $O/c4_inflight3.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/c1.txt 2>&1 || exit $?
echo done > $O/steps.txt
