# C4 (2048-set segments through the bucket MSM) per MSM chunk size K (GBLS_MSM_K), alternating
# three times, bench --tuning.  usage: bash tools/gpu/ab_c4_msm_k.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for k in 16 8 4; do
    GBLS_MSM_K=$k timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_k${k}_$r.txt 2>&1 || exit $?
    echo "msm_k $k rep $r C4 $(grep -o '"value": [0-9.]*' $O/c4_k${k}_$r.txt | head -1) msm $(grep -o '"k_msm": [0-9.]*' $O/c4_k${k}_$r.txt | head -1) ok $(grep -o '"committees_verified": [0-9]*' $O/c4_k${k}_$r.txt)" | tee -a $O/summary.txt
  done
done
