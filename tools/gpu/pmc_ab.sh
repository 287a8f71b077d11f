# Per-kernel instruction counts and durations of the default C2 command under different engine
# knobs: for each "NAME=VALUE ..." argument, one rocprofv3 PMC pass (VALU instructions, INT64
# instructions, waves, VALU-active quad cycles) and one kernel-trace pass of
# `bench.py --tuning --steps 3 --warmup 1 --no-cpu --no-single`.  The knobs reach the engine
# through bench.py's --tuning (GBLS_INIT_TUNING), the profiler launches python itself.
# usage: bash tools/gpu/pmc_ab.sh TAG "GBLS_LANE_R28=0" "GBLS_LANE_R28=1"
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --tuning --steps 3 --warmup 1 --no-cpu --no-single"
i=0
for cfg in "$@"; do
  i=$((i + 1))
  for kv in $cfg; do export "$kv"; done
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 &&
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/t$i -o run -- $B > $O/t$i.log 2>&1 &&
  python3 tools/prof/pmc_table.py $O/pmc_$i.csv $(ls $O/p$i/*.db | head -1) &&
  python3 tools/prof/db_stats.py $(ls $O/t$i/*.db | head -1) > $O/stats_$i.csv || exit $?
  for kv in $cfg; do unset "${kv%%=*}"; done
  echo "$i: $cfg" >> $O/configs.txt
done
