# Same-box A/B: the signature-side stream at high priority (GBLS_SIDE2_HIGH=1) on C4 (2048-set
# segments: per-set r.sigma products and the G2 tree sum on that stream), three alternations.
# usage: bash tools/gpu/ab_c4_side2.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for h in 0 1; do
    GBLS_SIDE2_HIGH=$h timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $O/c4_h${h}_$r.txt 2>&1 || exit $?
    echo "side2_high $h rep $r $(grep -o '"value": [0-9.]*' $O/c4_h${h}_$r.txt | head -1) $(grep -o '"k_g2sum": [0-9.]*' $O/c4_h${h}_$r.txt | head -1) $(grep -o '"k_h2c_clear": [0-9.]*' $O/c4_h${h}_$r.txt | head -1)" | tee -a $O/summary.txt
  done
done
