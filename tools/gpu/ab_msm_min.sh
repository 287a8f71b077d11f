# Same-box confirmation of the bucket-MSM threshold: C4 (2048-set segments) four alternations of
# GBLS_MSM_MIN 4096 / 2048, then the default C2 line and the C1 leg once per threshold (bench
# --tuning).  usage: bash tools/gpu/ab_msm_min.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for m in 2048 4096; do
    GBLS_MSM_MIN=$m timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_m${m}_$r.txt 2>&1 || exit $?
    echo "msm_min $m rep $r C4 $(grep -o '"value": [0-9.]*' $O/c4_m${m}_$r.txt | head -1) ok $(grep -o '"committees_verified": [0-9]*' $O/c4_m${m}_$r.txt)" | tee -a $O/summary.txt
  done
done
for m in 2048 4096; do
  GBLS_MSM_MIN=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --tuning > $O/c2_m$m.txt 2>&1 || exit $?
  GBLS_MSM_MIN=$m timeout -k 10 400 python bench.py --config C1 --steps 40 --warmup 5 --tuning > $O/c1_m$m.txt 2>&1 || exit $?
  echo "msm_min $m C2 $(grep -o '"value": [0-9.]*' $O/c2_m$m.txt | head -2 | tr '\n' ' ') C1 $(grep -o '"value": [0-9.]*' $O/c1_m$m.txt | head -1) $(grep -o '"gossip64": {[^,]*' $O/c1_m$m.txt)" | tee -a $O/summary.txt
done
