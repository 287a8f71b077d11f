# Round-4 last check on the final build: the whole GPU suite as the driver runs it, and smoke().
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo "pytest rc=$?" >> $O/steps.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo "smoke rc=$?" >> $O/steps.txt
