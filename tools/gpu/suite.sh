# The GPU test suite (or a subset), then the default C2 bench line and the C1 latency leg.
# usage: bash tools/gpu/suite.sh TAG [pytest -k expression]   (outputs under gpurun_out/TAG)
set -o pipefail
T=${1:?tag}
K=${2:-}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 400 python bench.py --config C1 --steps 40 --warmup 5 > $O/bench_c1.txt 2>&1
