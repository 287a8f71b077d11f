# the 2-rank C4 debug flow, then the main measurement pass (r4_c.sh)
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp GBLS_BENCH_ONE_DEVICE=1
for cfg in "65536 256" "1048576 2048"; do
  set -- $cfg
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=29533 tools/gpu/dbg_c4_dist.py $1 $2 > $O/dbg_c4_dist_$2.txt 2>&1
  rc=$?; echo "dbg $cfg rc=$rc" >> $O/steps.txt
  case $rc in 124|134|137|139) exit $rc ;; esac
done
unset GBLS_BENCH_ONE_DEVICE
bash tools/gpu/r4_c.sh $T
