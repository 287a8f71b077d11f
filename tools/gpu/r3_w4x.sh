# A/B of the wave-per-point threshold (lib_w4x: GBLS_W4_MAX=4096): 4096-set latency trace and
# the one-batch C2 leg with the default library and with the experiment build
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
X=$PWD/grandine_amd/xlib/libgrandine_bls.so
for n in 2048 4096; do
  PROBE_N=$n GBLS_LIB=$X timeout -k 10 200 rocprofv3 --kernel-trace -d $O/x$n -o run -- python3 tools/prof/lat_probe.py gossip 20 > $O/x$n.log 2>&1 || exit 1
  python3 tools/prof/timeline.py $(ls $O/x$n/*.db | head -1) -2 k_h2c_field > $O/x${n}_timeline.txt || exit 1
  PROBE_N=$n timeout -k 10 200 python3 tools/prof/lat_probe.py gossip 20 > $O/d$n.log 2>&1 || exit 1
done
GBLS_LIB=$X timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_b1_x.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_b1_d.txt 2>&1
