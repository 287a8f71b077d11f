# C3 kernel traces of two library builds in one box (per-kernel totals per step).
# usage: bash tools/gpu/c3_trace_ab.sh TAG LIB_A   (LIB_A: a GBLS_LIB path, traced beside the default)
set -o pipefail
T=${1:?tag}
A=${2:?lib}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
GBLS_LIB=$A timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ta -o run -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu > $O/ta.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tb -o run -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu > $O/tb.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/ta/*.db | head -1) > $O/stats_a.csv &&
python3 tools/prof/db_stats.py $(ls $O/tb/*.db | head -1) > $O/stats_b.csv && grep -o '"value": [0-9.]*' $O/ta.log $O/tb.log
