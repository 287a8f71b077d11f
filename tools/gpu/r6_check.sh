# Round-6 check: the GPU suite, the default C2 line, C4 five times in one call (consistency of the
# host-stall fix: host_enqueue_ms in every line).  usage: bash tools/gpu/r6_check.sh TAG [-k expr]
set -o pipefail
T=${1:?tag}
K=${2:-}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
echo "suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
echo "c2 $(date +%T)"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $O/bench_c2.txt 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/bench_c2.txt | head -1
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/bench_c4_$i.txt 2>&1 || exit $?
  echo "c4 run $i $(grep -o '"value": [0-9.]*' $O/bench_c4_$i.txt | head -1) $(grep -o '"host_enqueue_ms": {[^}]*}' $O/bench_c4_$i.txt | head -1)" | tee -a $O/c4.txt
done
if [ -n "$PMC" ]; then
  B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-single"
  echo "pmc $(date +%T)"
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/p2 -o run -- $B > $O/p2.log 2>&1 &&
  python3 tools/prof/pmc_table.py --largest $O/c2_pmc_lds.csv $(ls $O/p2/*.db | head -1) || exit $?
fi
