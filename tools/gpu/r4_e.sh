# A/B of the cross-submission pipeline (C2, C5) and of the block hold (C1), then the GPU suite
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
run 300 bench_c2.txt python bench.py --steps 20 --warmup 4 --no-cpu
GBLS_PIPELINE=0 run 300 bench_c2_nopipe.txt python bench.py --steps 20 --warmup 4 --no-cpu --no-single --tuning
run 300 bench_c2_inflight3.txt python bench.py --steps 20 --warmup 4 --no-cpu --no-single --inflight 3
run 300 bench_c1.txt python bench.py --config C1 --steps 40 --warmup 5
GBLS_BLOCK_HOLD=0 run 300 bench_c1_nohold.txt python bench.py --config C1 --steps 40 --warmup 5 --tuning
run 400 bench_c5_shard.txt python bench.py --config C5 --sets 131072 --steps 5 --warmup 2 --no-cpu
run 300 trace.log rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-single
run 900 pytest_gpu.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done >> $O/steps.txt
