# Same-box A/B on C4: the bucket MSM for its 2048-set segments (GBLS_MSM_MIN=2048) against the
# per-set r.sigma products (default threshold 4096), alternating three times, bench --tuning.
# usage: bash tools/gpu/ab_c4_msm.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for m in 4096 2048; do
    GBLS_MSM_MIN=$m timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_m${m}_$r.txt 2>&1 || exit $?
    echo "msm_min $m rep $r C4 $(grep -o '"value": [0-9.]*' $O/c4_m${m}_$r.txt | head -1) msm $(grep -o '"k_msm": [0-9.]*' $O/c4_m${m}_$r.txt | head -1) ok $(grep -o '"committees_verified": [0-9]*' $O/c4_m${m}_$r.txt)" | tee -a $O/summary.txt
  done
done
