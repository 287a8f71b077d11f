# Latency-form threshold (GBLS_W4_MAX 1024 / 512 / 256 builds) x gossip merge target: the
# 16-thread gossip load, C1 and the C2 line (with its single-batch leg) per build.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for b in lib_n lib_w512 lib_w256; do
  export GBLS_LIB=grandine_amd/$b/libgrandine_bls.so
  for mt in 512 768 1024; do
    GBLS_MERGE_TARGET=$mt timeout -k 10 120 python3 tools/gpu/gossip_load.py 3 16 --tuning > $O/g_${b}_$mt.log 2>&1 || exit $?
    echo "$b target $mt: $(tail -n1 $O/g_${b}_$mt.log)" >> $O/sweep.txt
  done
  timeout -k 10 300 python bench.py --config C1 --steps 30 --warmup 5 > $O/c1_$b.txt 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/c2_$b.txt 2>&1 || exit $?
  echo "$b C1: $(tail -n1 $O/c1_$b.txt | cut -c1-200)" >> $O/sweep.txt
done
echo done >> $O/sweep.txt
