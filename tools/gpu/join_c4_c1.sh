# Kernel traces of C4 and of the idle C1 block: does the signature-side stream (per-set r.sigma,
# the G2 sum with its 2^32 shift) delay the join?  usage: bash tools/gpu/join_c4_c1.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o run -- python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/c4.log 2>&1 || exit $?
python3 tools/prof/join_wait.py $(ls $O/c4/*.db | head -1) > $O/c4_join.txt || exit $?
tail -3 $O/c4_join.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/c1 -o run -- python3 bench.py --config C1 --steps 20 --warmup 3 > $O/c1.log 2>&1 || exit $?
python3 tools/prof/join_wait.py $(ls $O/c1/*.db | head -1) > $O/c1_join.txt || exit $?
tail -3 $O/c1_join.txt
