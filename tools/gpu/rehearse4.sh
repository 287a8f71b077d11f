# The C5 full-size test (oracle accept on a clean slice), then the N-rank bench flow with 4 ranks
# on the box's one GPU (gloo rehearsal, GBLS_BENCH_ONE_DEVICE): C2 weak and C4 strong.
# usage: bash tools/gpu/rehearse4.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread -k "c5_full" > $O/pytest_c5.txt 2>&1 || { tail -20 $O/pytest_c5.txt; exit 1; }
tail -2 $O/pytest_c5.txt
for cfg in C2 C4; do
  GBLS_BENCH_ONE_DEVICE=1 OMP_NUM_THREADS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr=127.0.0.1 --master-port=29531 bench.py --gpus 4 --config $cfg --steps 3 --warmup 1 > $O/bench4_$cfg.txt 2>&1 || { tail -20 $O/bench4_$cfg.txt; exit 1; }
  grep '^{' $O/bench4_$cfg.txt | head -1 | cut -c1-400
done
