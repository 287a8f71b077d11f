# Block under gossip load: the C1 leg with 16 / 8 / 4 loader threads (is the slow mode host CPU
# contention?), plus the box's CPU share.  usage: bash tools/gpu/c1_load.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP $OMP_NUM_THREADS"; } > $O/cpu.txt 2>&1
for th in 16 8 4 16; do
  timeout -k 10 300 python bench.py --config C1 --steps 40 --warmup 5 --load-threads $th > $O/c1_t$th.txt 2>&1 || exit $?
  echo "threads $th $(grep -o '"block_under_gossip_load": {[^}]*}' $O/c1_t$th.txt)" | tee -a $O/summary.txt
done
