# The driver's default bench command on the final build, plus C1 and C4.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench_c2.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 2 --no-cpu > $O/bench_c4.txt 2>&1 || exit $?
echo done > $O/steps.txt
