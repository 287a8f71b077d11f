# W4 engine checks, then the iteration check (GPU suite, latency traces, C2 + C1 benches)
set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out/$T
timeout -k 10 60 tools/ubench/_bin/w4_prim gpurun_out/$T/prim.bin > gpurun_out/$T/w4_prim.txt 2>&1 &&
python3 tools/ubench/w4_prim.py gpurun_out/$T/prim.bin >> gpurun_out/$T/w4_prim.txt &&
timeout -k 10 120 tools/ubench/_bin/w4_check > gpurun_out/$T/w4_check.txt 2>&1 &&
bash tools/gpu/r3_iter.sh $T
