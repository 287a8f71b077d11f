# kernel trace of the default bench (12 batches) and the C1 leg
set -o pipefail
O=gpurun_out/r2w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t12 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/t12.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/t12/*.db | head -1) > $O/t12_stats.csv &&
python3 tools/prof/timeline.py $(ls $O/t12/*.db | head -1) 3 k_mv_g1mul > $O/t12_timeline.txt &&
timeout -k 10 300 python3 bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1
