# instruction-cache experiment: out-of-line fp_mul build (lib_call) vs inline, and
# icache PMC counters of the default bench
set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2.txt 2>&1 &&
GBLS_LIB=$PWD/grandine_amd/lib_call/libgrandine_bls.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_c2_call.txt 2>&1 &&
GBLS_LIB=$PWD/grandine_amd/lib_call/libgrandine_bls.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batches 1 > $O/bench_c2b1_call.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/pmc_ic -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_ic.log 2>&1
