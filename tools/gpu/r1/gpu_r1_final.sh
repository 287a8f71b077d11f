set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/final/bench_default.txt 2>&1
