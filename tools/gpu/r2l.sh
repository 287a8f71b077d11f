# fused line evaluation groups (k_ml_group), MSM flags folded into k_msm_count
# and a kernel trace of B=4
set -o pipefail
O=gpurun_out/r2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_c2b1.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 8 > $O/bench_c2b8.txt 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > $O/bench_c5.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b4 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/b4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/b4/*.db | head -1) > $O/b4_stats.csv
