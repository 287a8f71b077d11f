set -o pipefail
O=gpurun_out/prof_msm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --batches 1 > $O/b1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b4 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --batches 4 > $O/b4.log 2>&1 &&
python3 tools/prof/db_stats.py $(ls $O/b1/*.db | head -1) > $O/b1_stats.csv &&
python3 tools/prof/db_stats.py $(ls $O/b4/*.db | head -1) > $O/b4_stats.csv
