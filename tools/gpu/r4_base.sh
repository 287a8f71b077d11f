# Round-4 baseline on the current build: GPU suite, then every bench leg (C2 default with the
# CPU baseline, C1, C3 grouped, C4, C5 shard, C5) and a kernel trace of one C3 step.
# usage: bash tools/gpu/r4_base.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_c2.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu > $O/bench_c3.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/bench_c4.txt 2>&1 &&
timeout -k 10 400 python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu > $O/bench_c5_shard.txt 2>&1 &&
timeout -k 10 500 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c3 -o run -- python3 bench.py --config C3 --steps 2 --warmup 1 --no-cpu > $O/c3_prof.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/c3/*.db | head -1) > $O/c3_kernel_stats.csv
