# Regime thresholds for single 4096-set submissions: W4 forms up to 4096 points (w4k), the
# row map up to 8192 field elements (m8k), both; C2 (+ single batch) and C4 per build, then
# the headline tests on the combined build.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib_w4k lib_m8k lib_both; do
  export GBLS_LIB=grandine_amd/$b/libgrandine_bls.so
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/c2_$b.txt 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --config C4 --steps 20 --warmup 2 --no-cpu > $O/c4_$b.txt 2>&1 || exit $?
  echo "$b C2 $(tail -n1 $O/c2_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["single_batch"])') C4 $(tail -n1 $O/c4_$b.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')" >> $O/res.txt
done
GBLS_LIB=grandine_amd/lib_both/libgrandine_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_both.txt 2>&1 || exit $?
echo done >> $O/res.txt
