# one-batch (4096-set) regime check: GPU suite (headline + parity + paths), a kernel trace of
# the 4096-set submission, then the default bench line (C2 + single_batch).
# usage: bash tools/gpu/r3_single.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
PROBE_N=4096 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/g4096 -o run -- python3 tools/prof/lat_probe.py gossip 20 > $O/g4096.log 2>&1 &&
python3 tools/prof/timeline.py $(ls $O/g4096/*.db | head -1) -2 k_h2c_field > $O/g4096_timeline.txt &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1
