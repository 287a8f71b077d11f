# The 2-rank C4 bench (tests/test_gpu_dist.py) repeated, with the bench's warm-up diagnostics.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
export GBLS_BENCH_ONE_DEVICE=1 OMP_NUM_THREADS=1
for i in $(seq 1 14); do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$((29600 + i)) bench.py --config C4 --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/run_$i.txt 2>&1
  rc=$?
  echo "run $i rc=$rc $(grep -h 'rank .* slot\|WRONG' $O/run_$i.txt | tr '\n' ' ' | cut -c1-600)" >> $O/res.txt
  case $rc in 124|134|137|139) exit $rc ;; esac
done
echo done >> $O/res.txt
