# Split Horner (4 parts + combine) on lib_n: headline + paths tests, C1 (+ trace), C2.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
export GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paths.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config C1 --steps 40 --warmup 5 > $O/c1.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run -- python3 bench.py --config C1 --steps 20 --warmup 2 --no-cpu > $O/tr.log 2>&1 || exit $?
python3 tools/prof/db_stats.py $(ls $O/tr/*.db | head -1) > $O/c1_stats.csv
timeout -k 10 300 python3 bench.py --steps 20 --warmup 4 --no-cpu > $O/c2.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 2 --no-cpu > $O/c4.txt 2>&1 || exit $?
echo done > $O/steps.txt
