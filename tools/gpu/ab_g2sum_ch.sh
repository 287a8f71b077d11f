# Same-box A/B of the signature sum's level-1 chunk size (GBLS_G2SUM_CH: sets per k_g2sum_chunks
# workgroup; 256 = WGR, the default) on C4, alternating three times (bench --tuning so the engine
# reads the knob).  usage: bash tools/gpu/ab_g2sum_ch.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for ch in 256 128 64; do
    GBLS_G2SUM_CH=$ch timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu --tuning > $O/c4_ch${ch}_$r.txt 2>&1 || exit $?
    echo "ch $ch rep $r C4 $(grep -o '"value": [0-9.]*' $O/c4_ch${ch}_$r.txt | head -1) g2sum $(grep -o '"k_g2sum": [0-9.]*' $O/c4_ch${ch}_$r.txt | head -1) ok $(grep -o '"committees_verified": [0-9]*' $O/c4_ch${ch}_$r.txt)" | tee -a $O/summary.txt
  done
done
