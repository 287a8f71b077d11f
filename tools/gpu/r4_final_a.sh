# Round-4 final pass A (default build grandine_amd/lib): GPU suite, smoke, every config's bench line.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() {  # run LIMIT OUTFILE CMD...
  local lim=$1 out=$2
  shift 2
  timeout -k 10 $lim "$@" > $O/$out 2>&1
  local rc=$?
  echo "$out rc=$rc" >> $O/steps.txt
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $out"; exit $rc ;; esac
  return 0
}
run 600 pytest_gpu.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 300 bench_c2.txt python bench.py
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
run 300 bench_c3.txt python bench.py --config C3 --steps 5 --warmup 1 --no-cpu
run 300 bench_c4.txt python bench.py --config C4 --steps 20 --warmup 2 --no-cpu
run 300 bench_c4b.txt python bench.py --config C4 --steps 20 --warmup 2 --no-cpu
run 400 bench_c5_shard.txt python bench.py --config C5 --sets 131072 --steps 5 --warmup 1 --no-cpu
run 500 bench_c5.txt python bench.py --config C5 --steps 3 --warmup 1 --no-cpu
echo done >> $O/steps.txt
