# kernel traces of the latency shapes (gossip 64, 1024 sets; C1 block)
set -o pipefail
O=gpurun_out/${1:-r3lat}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/g64 -o run -- python3 tools/prof/lat_probe.py gossip 30 > $O/g64.log 2>&1 &&
PROBE_N=1024 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/g1024 -o run -- python3 tools/prof/lat_probe.py gossip 30 > $O/g1024.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/blk -o run -- python3 tools/prof/lat_probe.py block 30 > $O/blk.log 2>&1 &&
for k in g64 g1024 blk; do python3 tools/prof/timeline.py $(ls $O/$k/*.db | head -1) -2 k_h2c_field > $O/${k}_timeline.txt || exit 1; done
