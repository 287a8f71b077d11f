# main chain on the high-priority context stream for device calls too
set -o pipefail
O=gpurun_out/r2z
mkdir -p $O
export TMPDIR=/tmp
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > $O/prio.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 4 > $O/bench_b4.txt 2>&1
