# C4 shard shapes on one GPU (VERDICT r05 "next 5"): rank 0's committees of a 2/4/8-way split of
# the 2048-committee epoch, and the whole epoch, each twice.  usage: bash tools/gpu/c4_shards.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for nsh in 1 2 4 8; do
    if [ $nsh = 1 ]; then E=""; else E="--emulate-shard $nsh"; fi
    timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu $E > $O/c4_s${nsh}_$rep.txt 2>&1 || exit $?
    echo "shard $nsh rep $rep: $(grep -o '"value": [0-9.]*' $O/c4_s${nsh}_$rep.txt | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c4_s${nsh}_$rep.txt | head -1) $(grep -o '"predicted_node_sets_per_s": [0-9.]*' $O/c4_s${nsh}_$rep.txt)" | tee -a $O/shards.txt
  done
done
