# C4 shard shapes on one GPU (bench --emulate-shard N: rank 0's share of an N-way split, 2048/N-set
# segments) with the bucket MSM for those segments (GBLS_MSM_MIN=256) against the default threshold
# (2048: per-set r.sigma products below it), alternating twice, bench --tuning.
# usage: bash tools/gpu/ab_c4_shard_msm.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for sh in 2 4; do
    for m in 2048 256; do
      GBLS_MSM_MIN=$m timeout -k 10 300 python bench.py --config C4 --emulate-shard $sh --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_s${sh}_m${m}_$r.txt 2>&1 || exit $?
      echo "shard $sh msm_min $m rep $r $(grep -o '"value": [0-9.]*' $O/c4_s${sh}_m${m}_$r.txt | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c4_s${sh}_m${m}_$r.txt | head -1) ok $(grep -o '"committees_verified": [0-9]*' $O/c4_s${sh}_m${m}_$r.txt)" | tee -a $O/summary.txt
    done
  done
done
