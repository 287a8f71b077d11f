# Round-4 final pass B: kernel trace and PMC counters of the default command without the
# one-batch leg (16-batch launches only), their tables, and the GPU idle gaps.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() {  # run LIMIT OUTFILE CMD...
  local lim=$1 out=$2
  shift 2
  timeout -k 10 $lim "$@" > $O/$out 2>&1
  local rc=$?
  echo "$out rc=$rc" >> $O/steps.txt
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $out"; exit $rc ;; esac
  return 0
}
B="python3 bench.py --steps 10 --warmup 2 --no-cpu --no-single"
run 300 trace.log rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $B
run 120 p1.log rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run -- $B
run 120 p2.log rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU -d $O/p2 -o run -- $B
run 120 p3.log rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $B
run 120 p4.log rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run -- $B
python3 tools/prof/db_stats.py $(ls $O/trace/*.db | head -1) > $O/c2_kernel_stats.csv
python3 tools/prof/pmc_table.py $O/c2_pmc.csv $(ls $O/p1/*.db | head -1) $(ls $O/p2/*.db | head -1) $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1)
python3 tools/prof/pmc_bytes.py $(ls $O/p3/*.db | head -1) $(ls $O/p4/*.db | head -1) > $O/c2_pmc_bytes.csv
tail -n1 $O/trace.log > $O/trace_line.json
echo done >> $O/steps.txt
