# other configs (C3, C4, C5 shard, C5), the 4096-set latency trace, and the coalescer knobs
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O/lat
export TMPDIR=/tmp
bash tools/gpu/bench_configs.sh $T &&
PROBE_N=4096 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/lat/g4096 -o run -- python3 tools/prof/lat_probe.py gossip 20 > $O/lat/g4096.log 2>&1 &&
python3 tools/prof/timeline.py $(ls $O/lat/g4096/*.db | head -1) -2 k_h2c_field > $O/lat/g4096_timeline.txt &&
bash tools/gpu/r3_knobs.sh $T/knobs
