"""CPU: the drop-in boundary as a maintainer would bind it (VERDICT r02 "next 7").

* rust/bls_gpu_sys/src/ffi.rs declares every prototype of include/grandine_bls_gpu.h with the
  same argument count and the C types mapped to their Rust FFI equivalents, and the same
  constants (status codes, error codes, flags);
* every `unsafe` block of the drop-in is in the sys crate: the patched `bls` / `helper_functions`
  bodies (rust/bls_patch) and INTEGRATION.md's code for those crates contain no unsafe code
  (Grandine forbids it workspace-wide, /root/reference/Cargo.toml:65-66, bls/Cargo.toml:6-7);
* each safe wrapper of rust/bls_gpu_sys/src/lib.rs calls the header entry point it names with
  the header's argument count, and each patched body has a blst branch for engine errors;
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
RS = os.path.join(ROOT, "rust", "bls_gpu_sys", "src", "ffi.rs")
SAFE = os.path.join(ROOT, "rust", "bls_gpu_sys", "src", "lib.rs")
PATCH = os.path.join(ROOT, "rust", "bls_patch")
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
    return {"int": "c_int", "size_t": "usize", "double": "f64", "const char *": "*const c_char", "void": None,
            "uint32_t": "u32"}[ret]


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
    for f in ("gpu.rs", "signature.rs", "public_key.rs", "verifier.rs"):
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
            "gbls_set_policy",
            "gbls_profile_read", "gbls_stage_name", "status", "verdict"}
    for name, vals in rows.items():
        if name in info:
            continue
        assert vals == ["5", "100"], (name, vals)  # GBLS_VERIFY_FAIL, GBLS_ERR_NO_DEVICE
    assert rows["status"] == ["1"] and rows["verdict"] == ["5"]
    assert rows["gbls_device_count"][0] == "0" and rows["gbls_registry_size"][0] == "0"


def _strip_comments(txt):
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return "\n".join(line.split("//")[0] for line in txt.splitlines())


def test_no_unsafe_outside_the_sys_crate():
    """VERDICT r03 "next 1": nothing unsafe in the bls / helper_functions patch."""
    for f in sorted(os.listdir(PATCH)):
        if f.endswith(".rs"):
            code = _strip_comments(open(os.path.join(PATCH, f)).read())
            assert not re.search(r"\bunsafe\b", code), f
            assert "unsafe_code" not in code, f
            assert "transmute" not in code, f
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```rust\n(.*?)```", md, flags=re.S)
    assert len(blocks) >= 4
    for b in blocks:
        if b.startswith("// bls_gpu_sys/"):
            continue  # the sys crate may hold unsafe blocks
        code = _strip_comments(b)
        assert not re.search(r"\bunsafe\b", code), b[:80]
        assert "unsafe_code" not in code, b[:80]


def _rust_fns(txt):
    """name -> body of every top-level `pub fn` in a Rust file (brace matching)."""
    out = {}
    for m in re.finditer(r"\bpub fn (\w+)", txt):
        i = txt.index("{", m.end())
        depth, j = 0, i
        while True:
            if txt[j] == "{":
                depth += 1
            elif txt[j] == "}":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        out[m.group(1)] = txt[m.start():j + 1]
    return out


def test_safe_wrappers_call_the_header_entry_points():
    c = c_prototypes()
    fns = _rust_fns(open(SAFE).read())
    wrappers = {"g1_decompress": "gbls_g1_decompress", "g2_decompress": "gbls_g2_decompress",
                "g1_aggregate": "gbls_g1_aggregate", "g2_aggregate": "gbls_g2_aggregate",
                "verify": "gbls_verify", "fast_aggregate_verify": "gbls_fast_aggregate_verify",
                "multi_verify": "gbls_multi_verify", "multi_verify_compressed": "gbls_multi_verify_compressed_ex",
                "multi_verify_bisect": "gbls_multi_verify_bisect", "engine": "gbls_init",
                "verify_batch_compressed": "gbls_verify_batch_compressed", "set_policy": "gbls_set_policy",
                "g2_decompress_many": "gbls_g2_decompress", "g2_aggregate_segments": "gbls_g2_aggregate_segments"}
    for w, entry in wrappers.items():
        body = fns[w]
        m = re.search(r"ffi::%s\((.*?)\)\s*\}?;?\n" % entry, body, flags=re.S)
        assert m, (w, entry)
        args = [a for a in split_args(" ".join(m.group(1).split()).rstrip(",")) if a.strip()]
        assert len(args) == len(c[entry][1]), (w, entry, args)
        # every pointer/length pair comes from a slice checked in the wrapper: no raw pointer
        # parameters in the safe signature
        sig = body[:body.index("{")]
        assert "*const" not in sig and "*mut" not in sig, w
        # engine errors are read back from gbls_last_error
        if w not in ("engine", "set_policy"):
            assert "verdict(rc)" in body or "status(rc)" in body or "last_error()" in body, w
    # every unsafe block of the safe layer carries a SAFETY note
    safe = open(SAFE).read()
    assert safe.count("unsafe {") == safe.count("// SAFETY:"), "undocumented unsafe block"


def test_patched_bodies_fall_back_to_blst():
    sig = open(os.path.join(PATCH, "signature.rs")).read()
    pk = open(os.path.join(PATCH, "public_key.rs")).read()
    fin = open(os.path.join(PATCH, "verifier.rs")).read()
    gpu = open(os.path.join(PATCH, "gpu.rs")).read()
    # the routing helper runs the cpu closure when the engine is absent or returns Err
    route = _rust_fns(gpu.replace("pub(crate) fn route", "pub fn route"))["route"]
    assert "available()" in route and "if let Ok(value) = gpu()" in route and route.rstrip("}\n ").endswith("cpu()")
    for body, n in ((sig, 5), (pk, 2)):
        assert body.count("crate::gpu::route(") + body.count("crate::gpu::route_single(") >= n - 1
    # lone single checks: blst unless GBLS_SINGLE_CHECKS=engine, then the same engine route
    single = _rust_fns(gpu.replace("pub(crate) fn route_single", "pub fn route_single"))["route_single"]
    assert "single_checks_on_engine()" in single and "route(gpu, cpu)" in single
    assert sig.split("\nmod cpu {")[0].count("crate::gpu::route_single(") == 3
    for name in ("decompress", "verify", "fast_aggregate_verify", "multi_verify", "aggregate_in_place"):
        assert re.search(r"fn %s\b" % name, sig.split("\nmod cpu {")[1]), name
        assert "cpu::%s" % name in sig.split("\nmod cpu {")[0], name
    assert "verify_multiple_aggregate_signatures" in sig.split("\nmod cpu {")[1]
    for name in ("decompress_validate", "aggregate_in_place", "sum"):
        assert "cpu::%s" % name in pk.split("\nmod cpu {")[0], name
    assert "validate()" in pk.split("\nmod cpu {")[1]
    # finish: no engine verdict -> the reference body (rayon decompression + multi_verify)
    assert "None => self.finish_on_cpu()" in fin and "par_iter()" in fin.split("fn finish_on_cpu")[1]
    # a multi_verify message that is not 32 bytes is not a panic: it takes the blst branch
    assert "expect(" not in sig and "EngineError::Argument" in sig
    # aggregate_in_place never keeps self on a failure: it is the blst addition itself
    for body in (sig, pk):
        m = re.search(r"pub fn aggregate_in_place\(&mut self, other: Self\) \{(.*?)\n    \}", body, flags=re.S)
        assert m and m.group(1).strip() == "cpu::aggregate_in_place(self, other);"


def test_triples_defer_key_aggregation_to_the_engine():
    """VERDICT r04 "next 1": Triple::verify_aggregate keeps the key list (no rayon reduce, no
    AggregatePublicKey::aggregate on the engine path); finish and SingleVerifier::extend hand the
    lists to the engine with per-set offsets; the blst sums are only in the fallbacks."""
    ver = open(os.path.join(PATCH, "verifier.rs")).read()
    code = _strip_comments(ver)
    body = lambda name: code.rsplit("fn %s(" % name, 1)[1].split("\nfn ", 1)[0]  # the top-level one
    va = code.split("fn verify_aggregate", 1)[1].split("fn extend", 1)[0]
    assert "reduce" not in va and "aggregate(" not in va.replace("verify_aggregate(", "") and "deferred: Some(keys)" in va
    for name in ("finish", "extend"):
        engine_branch = body(name).split("None =>")[0]
        assert "AggregatePublicKey" not in engine_branch and ".public_key()" not in engine_branch, name
        assert "engine_sets(" in engine_branch, name
    assert "bls::gpu::multi_verify_compressed(&messages, &signature_bytes, &points, &offsets" in body("finish")
    assert "bls::gpu::verify_batch_compressed(&messages, &signature_bytes, &points, &offsets)" in body("extend")
    # fallbacks form the sums with blst and run the reference bodies
    assert "None => self.finish_on_cpu()" in body("finish") and "None => extend_on_cpu(" in body("extend")
    assert "Triple::public_key" in body("finish_on_cpu") and "triple.public_key()" in body("extend_on_cpu")
    # the sys wrappers pass the offsets as pk_off (points + per-set ranges)
    fns = _rust_fns(open(SAFE).read())
    assert "key_offsets.as_ptr()" in fns["multi_verify_compressed"]
    assert "key_ranges_ok(keys, key_offsets, n)" in fns["multi_verify_compressed"]
    assert "key_ranges_ok(keys, key_offsets, n)" in fns["verify_batch_compressed"]
    # blst -> engine conversion: by default a limb copy through blst's From impls (no
    # serialisation round trip per key); feature `serialized-points` (the From impls
    # are unverified in this image) decodes blst's own serialisation instead
    safe = open(SAFE).read()
    for name, de in (("p1_of_public_key", "blst_p1_deserialize"), ("p2_of_signature", "blst_p2_deserialize")):
        defs = re.findall(r'(#\[cfg\((not\()?feature = "serialized-points"\)?\)\]\n#\[must_use\]\npub fn %s\(.*?\n\})'
                          % name, safe, flags=re.S)
        assert len(defs) == 2, name
        default = [d[0] for d in defs if d[1]][0]
        alt = [d[0] for d in defs if not d[1]][0]
        assert "serialize()" not in default and "::from(" in default, name
        assert "serialize()" in alt and de in alt and "// SAFETY:" in alt, name
    cargo = open(os.path.join(ROOT, "rust", "bls_gpu_sys", "Cargo.toml")).read()
    assert "[features]" in cargo and "serialized-points = []" in cargo


def test_gossip_fallback_names_failing_items_in_one_submission():
    """VERDICT r05 "next 4" (f2 as code): the patched Err arms of the gossip batch tasks
    (p2p/src/attestation_verifier.rs:231-238, 379-384) send only the items with a failing set to
    the singular path, decided by ONE MultiVerifier::verify_each submission, and keep the
    reference loops when the engine gives no verdict."""
    av = open(os.path.join(PATCH, "attestation_verifier.rs")).read()
    code = _strip_comments(av)
    for kind in ("attestation", "aggregate"):
        arm = code.split("match self.failing_%ss(" % kind, 1)[1].split("fn failing_", 1)[0]
        some, none = arm.split("None =>", 1)
        # Some: per item, singular only when failed, else the batch result is kept and sent
        assert "if failed {" in some and "self.process_singular_%s(%s_wo);" % (kind, kind) in some
        assert "passed.push(result);" in some and "self.send_results_to_fork_choice(passed);" in some
        # None: the reference loop over every accepted item
        assert "for %s_wo in accepted_%ss_wo {" % (kind, kind) in none
        assert "self.process_singular_%s(%s_wo);" % (kind, kind) in none
    # the sets are built in item order (slice par_iter keeps order; par_bridge would not)
    assert code.count(".par_iter()") == 2 and "par_bridge" not in code
    fi = code.split("fn failing_items(", 1)[1]
    assert "verifier.verify_each()?" in fi and "failing.push(sets.is_none());" in fi
    # an aggregate contributes its three sets: selection proof, aggregate-and-proof, attestation
    agg = code.split("fn failing_aggregates(", 1)[1].split("fn failing_items", 1)[0]
    assert agg.count("Triple::new(") == 2 and "attestation_triple," in agg
    # verify_each is one verify_batch_compressed submission over the verifier's sets
    ver = _strip_comments(open(os.path.join(PATCH, "verifier.rs")).read())
    ve = ver.split("pub fn verify_each(&self)", 1)[1].split("\n}", 1)[0]
    assert "engine_sets(&self.triples)" in ve
    assert "bls::gpu::verify_batch_compressed(&messages, &signature_bytes, &points, &offsets)" in ve
    assert "matches!(outcome, Ok(true))" in ve


def test_registry_mirror_names_slots_in_finish():
    """VERDICT r05 "next 4" (f1 as code): the attestation predicate passes the attesting indices
    (verify_aggregate_indexed), Triple keeps them beside the keys, finish names registry slots
    only when every set has indices and the registry mirrors them (else the key points), the
    mirror loads only a finalized validator list's new tail, and the sys crate's indexed wrapper
    passes indices + offsets with no key points."""
    pred = _strip_comments(open(os.path.join(PATCH, "predicates.rs")).read())
    assert "verifier.verify_aggregate_indexed(" in pred and "&validator_indices," in pred
    assert "accessors::public_key(state, validator_index)?" in pred and ".decompress()" in pred
    ver = _strip_comments(open(os.path.join(PATCH, "verifier.rs")).read())
    assert "indices: Option<Vec<u32>>," in ver
    tvai = ver.split("fn verify_aggregate_indexed<'keys>(", 1)[1].split("\n    }", 1)[0]
    assert "self.verify_aggregate(message, signature_bytes, public_keys, signature_kind)?;" in tvai
    assert "u32::try_from(index).ok()" in tvai
    ei = ver.split("fn engine_indices(", 1)[1].split("\n}", 1)[0]
    assert "triple.indices.as_deref()?" in ei and "bls::gpu::registry::covers(&indices)" in ei
    fin = ver.rsplit("fn finish(", 1)[1].split("\nfn ", 1)[0]
    assert "match engine_indices(&self.triples)" in fin
    assert "bls::gpu::multi_verify_compressed_indexed(" in fin and "bls::gpu::multi_verify_compressed(" in fin
    assert "None => self.finish_on_cpu()" in fin
    gpu = _strip_comments(open(os.path.join(PATCH, "gpu.rs")).read())
    reg = gpu.split("pub mod registry {", 1)[1]
    assert "keys[*mirrored..]" in reg and "bls_gpu_sys::registry_set(*mirrored, &tail)" in reg
    assert "index < mirrored" in reg
    fns = _rust_fns(open(SAFE).read())
    body = fns["multi_verify_compressed_indexed"]
    m = re.search(r"ffi::gbls_multi_verify_compressed_ex\((.*?)\)\s*\};", body, flags=re.S)
    args = [a.strip() for a in m.group(1).split(",") if a.strip()]
    assert args[2] == "ptr::null()" and args[3] == "indices.as_ptr()" and args[4] == "index_offsets.as_ptr()"
    assert "status(rc)?" in fns["registry_set"] and "ffi::gbls_registry_set(first, keys.as_ptr()" in fns["registry_set"]


def test_sync_pool_aggregates_in_one_submission():
    """f4 (VERDICT r05 "missing 1"): the sync-committee pool's message loops
    (operation_pools/src/sync_committee_agg_pool/pool.rs:90-115, 159-192) plan their additions and
    hand them to bls::gpu::aggregate_into (one batched decode + one segmented sum); the reference
    loops stay as the no-verdict fallback; a decode failure stops the sums where the reference's
    `try_into()?` returns."""
    pool = _strip_comments(open(os.path.join(PATCH, "sync_committee_pool.rs")).read())
    gpu = _strip_comments(open(os.path.join(PATCH, "gpu.rs")).read())
    agg = _rust_fns(gpu)["aggregate_into"]
    assert "bls_gpu_sys::g2_decompress_many(" in agg and "bls_gpu_sys::g2_aggregate_segments(" in agg
    assert "position(Result::is_err)" in agg and "additions[..upto]" in agg
    # bases are replaced only after every sum converted
    assert agg.index("collect::<Option<Vec<_>>>()?") < agg.index("*base = Signature::from(raw)")
    for fn in ("add_sync_committee_contribution", "aggregate_messages"):
        body = _rust_fns(pool.replace("pub async fn", "pub fn"))[fn]
        assert "plan_additions(" in body and "add_on_engine(" in body, fn
        # the reference loop, with its per-message decode, is the fallback
        assert ".aggregate_in_place(message.signature.try_into()?)" in body, fn
        assert "lookup_error" in body, fn
    eng = pool.split("fn add_on_engine", 1)[1].split("\npub async fn", 1)[0]
    assert "bls::gpu::aggregate_into(" in eng
    # no verdict: every planned bit cleared; a failure: the bits after it cleared
    assert "for a in plan {" in eng and "&plan[i + 1..]" in eng
