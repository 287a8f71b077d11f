"""CPU: the drop-in boundary as a maintainer would bind it (VERDICT r02 "next 7").

* rust/bls_gpu_sys/src/lib.rs declares every prototype of include/grandine_bls_gpu.h with the
  same argument count and the C types mapped to their Rust FFI equivalents, and the same
  constants (status codes, error codes, flags);
* the sys crate does not inherit the workspace's `unsafe_code = 'forbid'`
  (/root/reference/Cargo.toml:66) and its build script builds the engine in-tree;
* tests/native/abi_c99.c includes the header in a -std=c99 -Wall -Wextra -Werror -pedantic
  translation unit, calls every entry point and links against the built library; without a GPU
  every call fails closed (GBLS_VERIFY_FAIL, failure-filled outputs, GBLS_ERR_NO_DEVICE).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "grandine_bls_gpu.h")
RS = os.path.join(ROOT, "rust", "bls_gpu_sys", "src", "lib.rs")
LIBDIR = os.path.join(ROOT, "grandine_amd", "lib")

SCALAR = {"size_t": "usize", "int": "c_int", "uint32_t": "u32", "int32_t": "i32", "uint64_t": "u64",
          "uint8_t": "u8", "double": "f64", "void": "c_void", "char": "c_char"}


def c_prototypes():
    txt = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^([a-z][\w \*]*?\b)(gbls_\w+)\s*\(([^;]*?)\);", txt, flags=re.M | re.S):
        args = " ".join(args.split())
        types = [] if args == "void" else [c_type(a) for a in split_args(args)]
        out[name] = (c_ret(ret.strip()), types)
    return out


def split_args(args):
    parts, depth, cur = [], 0, ""
    for ch in args:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    parts.append(cur.strip())
    return parts


def c_type(arg):
    """C parameter declaration -> the Rust FFI type it must be bound as."""
    m = re.match(r"(const\s+)?(\w+)\s*\(\*\s*\w+\)\[(\d+)\]$", arg)  # const uint8_t (*in)[48]
    if m:
        return "*%s [%s; %s]" % ("const" if m.group(1) else "mut", SCALAR[m.group(2)], m.group(3))
    m = re.match(r"(const\s+)?(\w+)\s*(\*?)\s*\w+$", arg)
    assert m, arg
    base = SCALAR.get(m.group(2), m.group(2))
    if m.group(3):
        return "*%s %s" % ("const" if m.group(1) else "mut", base)
    return base


def c_ret(ret):
    return {"int": "c_int", "size_t": "usize", "double": "f64", "const char *": "*const c_char", "void": None}[ret]


def rust_prototypes():
    txt = open(RS).read()
    block = txt[txt.index('extern "C" {'):]
    out = {}
    for name, args, ret in re.findall(r"pub fn (gbls_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        args = " ".join(args.split()).rstrip(",")
        types = [] if not args.strip() else [a.split(":", 1)[1].strip() for a in split_args(args) if a]
        out[name] = (ret.strip() if ret else None, [" ".join(t.split()) for t in types])
    return out


def test_every_prototype_bound_with_matching_types():
    c, r = c_prototypes(), rust_prototypes()
    assert len(c) >= 40
    assert sorted(c) == sorted(r), set(c) ^ set(r)
    for name in c:
        assert c[name] == r[name], (name, c[name], r[name])


def test_constants_agree():
    hdr = open(HDR).read()
    rs = open(RS).read()
    consts = dict(re.findall(r"\b(GBLS_[A-Z0-9_]+)\s*=\s*(\d+),", hdr))
    consts.update({k: str(int(v, 16)) for k, v in re.findall(r"#define (GBLS_[A-Z_]+) (0x[0-9a-f]+)u", hdr)})
    assert len(consts) >= 14
    for k, v in consts.items():
        m = re.search(r"pub const %s: \w+ = (0x[0-9a-f]+|\d+);" % k, rs)
        assert m, k
        assert int(m.group(1), 0) == int(v), k


def test_sys_crate_manifest_and_build_script():
    toml = open(os.path.join(ROOT, "rust", "bls_gpu_sys", "Cargo.toml")).read()
    body = "\n".join(line.split("#")[0] for line in toml.splitlines())  # comments aside
    assert "[lints]" not in body and "workspace" not in body
    assert 'links = "grandine_bls"' in toml
    build = open(os.path.join(ROOT, "rust", "bls_gpu_sys", "build.rs")).read()
    assert 'join("grandine_amd")' in build and "rustc-link-lib=dylib=grandine_bls" in build
    for f in ("gpu.rs", "signature.rs", "public_key.rs", "verifier_finish.rs"):
        assert os.path.getsize(os.path.join(ROOT, "rust", "bls_patch", f)) > 500, f


@pytest.fixture(scope="module")
def c99_run(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libgrandine_bls.so")):
        pytest.skip("library not built")
    exe = str(tmp_path_factory.mktemp("abi") / "abi_c99")
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "abi_c99.c"),
                           "-L", LIBDIR, "-lgrandine_bls", "-Wl,-rpath," + LIBDIR, "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout


def test_c99_consumer_calls_every_entry_point(c99_run):
    called = set(re.findall(r"^(gbls_\w+)", c99_run, flags=re.M)) | {"gbls_last_error", "gbls_profile_reset"}
    assert called == set(c_prototypes()), set(c_prototypes()) ^ called


def test_c99_consumer_fails_closed_without_device(c99_run):
    rows = {line.split()[0]: line.split()[1:] for line in c99_run.splitlines()}
    if rows["gbls_init"][0] == "0":
        pytest.skip("a device is present: the fail-closed leg is for GPU-less hosts")
    info = {"gbls_device_count", "gbls_registry_size", "gbls_version", "gbls_measure_mad64_peak", "gbls_profile",
            "gbls_profile_read", "gbls_stage_name", "status", "verdict"}
    for name, vals in rows.items():
        if name in info:
            continue
        assert vals == ["5", "100"], (name, vals)  # GBLS_VERIFY_FAIL, GBLS_ERR_NO_DEVICE
    assert rows["status"] == ["1"] and rows["verdict"] == ["5"]
    assert rows["gbls_device_count"][0] == "0" and rows["gbls_registry_size"][0] == "0"
