# The GPU suite on the current build,
# then a same-box A/B against the previous build (grandine_amd/libprev, GBLS_LIB): C4 and C1
# alternating three times, and C4's join waits on the new build.  usage: bash tools/gpu/ab_lib.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
PREV=$PWD/grandine_amd/libprev/libgrandine_bls.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
for r in 1 2 3; do
  for m in new prev; do
    if [ $m = prev ]; then export GBLS_LIB=$PREV; else unset GBLS_LIB; fi
    timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/c4_${m}_$r.txt 2>&1 || exit $?
    timeout -k 10 400 python bench.py --config C1 --steps 40 --warmup 5 > $O/c1_${m}_$r.txt 2>&1 || exit $?
    echo "$m rep $r C4 $(grep -o '"value": [0-9.]*' $O/c4_${m}_$r.txt | head -1) g2sum $(grep -o '"k_g2sum": [0-9.]*' $O/c4_${m}_$r.txt | head -1) C1 $(grep -o '"value": [0-9.]*' $O/c1_${m}_$r.txt | head -1) $(grep -o '"gossip64": {[^,]*' $O/c1_${m}_$r.txt)" | tee -a $O/summary.txt
  done
done
unset GBLS_LIB
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o run -- python3 bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/c4_trace.log 2>&1 || exit $?
python3 tools/prof/join_wait.py $(ls $O/c4/*.db | head -1) > $O/c4_join.txt || exit $?
tail -1 $O/c4_join.txt
