"""CPU: the engine's host-compiled arithmetic under AddressSanitizer + UndefinedBehaviorSanitizer
(VERDICT r02 "next 8"; the reference keeps overflow checks in release builds,
/root/reference/Cargo.toml:485-490).

tests/native/host_harness.cpp compiles the engine's __host__ __device__ formulas (field, tower,
curve, hash_to_G2, the serial pipeline including the inversion-free verdict) for the CPU.  Here
it is rebuilt with -fsanitize=address,undefined -fno-sanitize-recover=all and the golden-fixture
tests of tests/test_host_harness.py run against it in a child interpreter that preloads libasan:
any out-of-bounds access, use-after-scope, signed overflow, misaligned or oversized shift aborts
the child.  (The GPU kernels themselves cannot be sanitized on this pool: GPU ASan and XNACK
builds are refused.)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SUBSET = ("test_fp_mul_random or test_g1_decode_fixtures or test_g2_decode_fixtures or "
          "test_hash_to_g2_fixtures or test_verify_fixtures or test_multi_verify_fixtures or "
          "test_inversion_free_final_verdict or test_fp_inv or test_fp_inv_var_safegcd or r28")


def test_host_harness_under_asan_ubsan():
    libasan = subprocess.check_output(["g++", "-print-file-name=libasan.so"], text=True).strip()
    assert os.path.exists(libasan), libasan
    env = dict(os.environ, GBLS_HARNESS_SAN="1", LD_PRELOAD=libasan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",  # the interpreter's own allocations
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                          os.path.join(ROOT, "tests", "test_host_harness.py"), "-k", SUBSET],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    log = out.stdout[-3000:] + out.stderr[-3000:]
    assert out.returncode == 0, log
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, log
    assert " passed" in out.stdout, log


def test_scheduling_under_tsan(tmp_path):
    """VERDICT r03 "next 7" / ADVICE r03 (high): the context pool and the coalescer
    (grandine_amd/csrc/gbls_sched.h, the code gbls_capi.hip runs) under ThreadSanitizer with stub
    contexts and a stub verifier: 48 threads leasing both context classes, a block-import lease
    while every normal slot is held (and the reverse), and 32 threads of coalesced calls mixing
    block and gossip classes, four key kinds, random sizes and segment counts, each checking its
    own verdicts and signature statuses (tests/native/sched_tsan.cpp)."""
    exe = str(tmp_path / "sched_tsan")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", "-Wall", "-Wextra",
                           "-Werror", "-I", os.path.join(ROOT, "grandine_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "sched_tsan.cpp"), "-o", exe])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    out = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    log = out.stdout[-3000:] + out.stderr[-3000:]
    assert out.returncode == 0, log
    assert "ThreadSanitizer" not in out.stderr, log
    assert "sched_tsan: OK" in out.stdout, log


def test_miller_tables_under_asan(tmp_path):
    """the Miller product tables (grandine_amd/csrc/gbls_tables.h, built by
    every pipeline) keep the line buffer within 1.25x the event-slice budget also for uneven
    segment mixes (one large segment beside thousands of one- and two-set segments), never put a
    whole large segment in one lane, list every pair once and give each its column
    (tests/native/tables_check.cpp, under ASan/UBSan)."""
    exe = str(tmp_path / "tables_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-Wall", "-Wextra", "-Werror",
                           "-I", os.path.join(ROOT, "grandine_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "tables_check.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    log = out.stdout[-3000:] + out.stderr[-3000:]
    assert out.returncode == 0, log
    assert "tables_check: OK" in out.stdout, log
