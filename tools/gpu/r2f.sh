# C2 with B coalesced batches per submission
set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
export TMPDIR=/tmp
for b in 1 2 4 8 16; do timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches $b > $O/bench_c2_b$b.txt 2>&1 || exit 1; done
