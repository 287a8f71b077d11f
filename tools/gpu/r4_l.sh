# Gossip coalescer sweep: 16-thread 64-set load under merge targets / leaders / windows.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
export GBLS_LIB=grandine_amd/lib_n/libgrandine_bls.so
for cfg in "512 2 300" "256 2 300" "1024 2 300" "1024 1 300" "1024 2 1000" "2048 1 1000" "768 2 600"; do
  set -- $cfg
  GBLS_MERGE_TARGET=$1 GBLS_LEADERS=$2 GBLS_MERGE_WINDOW_US=$3 timeout -k 10 120 python3 tools/gpu/gossip_load.py 3 16 --tuning > $O/g_$1_$2_$3.log 2>&1 || exit $?
  echo "target $1 leaders $2 window $3: $(tail -n1 $O/g_$1_$2_$3.log)" >> $O/sweep.txt
done
echo done >> $O/sweep.txt
