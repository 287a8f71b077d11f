set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out/$T
timeout -k 10 300 python bench.py --config C1 --steps 100 --warmup 10 --no-cpu > gpurun_out/$T/bench_c1.txt 2>&1 &&
PROBE_N=1024 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$T/g1024 -o run -- python3 tools/prof/lat_probe.py gossip 30 > gpurun_out/$T/g1024.log 2>&1 &&
python3 tools/prof/timeline.py $(ls gpurun_out/$T/g1024/*.db | head -1) -2 k_h2c_field > gpurun_out/$T/g1024_timeline.txt
