# A/B of engine tuning knobs on the default C2 bench line: for each "NAME=VALUE ..." argument
# after the tag, one `bench.py --tuning` run with those variables set (outputs gpurun_out/TAG/ab_<i>.txt,
# one line per run in ab.txt).  usage: bash tools/gpu/ab_env.sh TAG "GBLS_MSM_K=16" "GBLS_MSM_K=8" ...
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --tuning > $O/ab_$i.txt 2>&1 || exit $?
  echo "$cfg :: $(grep -o '"value": [0-9.]*' $O/ab_$i.txt | head -1) single $(grep -o '"single_batch": {[^}]*}' $O/ab_$i.txt | grep -o '"value": [0-9.]*')" >> $O/ab.txt
done
