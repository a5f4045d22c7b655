"""The Rust FFI crate (crates/dtgpu-sys) and the static archive it links.

cargo / rustc are not in this image, so the crate is checked structurally: every `extern "C"`
declaration in src/lib.rs must name a function of include/dtgpu.h with the same parameter and
return types (C types mapped to their Rust FFI spellings), and build.rs must link the static
archive plus the HIP runtime.  The archive itself (diamond-types_amd/lib/libdtgpu.a) must define
every symbol the header declares; tests/ffi/checkout_tip.c, linked against it with gcc the way
rustc links a staticlib, is run on the GPU against the golden text."""
import gzip
import json
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "dtgpu.h")
CRATE = os.path.join(ROOT, "crates", "dtgpu-sys")
LIB = os.path.join(ROOT, "diamond-types_amd", "lib")

BASE = {"uint8_t": "u8", "char": "c_char", "size_t": "usize", "int": "c_int", "int32_t": "i32", "int64_t": "i64",
        "uint32_t": "u32", "uint64_t": "u64", "float": "f32", "void": "c_void", "dtgpu_status": "dtgpu_status"}


def c_to_rust(t):
    """`const uint8_t *const *` -> `*const *const u8` (a pointer is *const when what it points
    to is const)."""
    t = t.replace("*", " * ").split()
    levels, base = [False], None
    for tok in t:
        if tok == "const":
            levels[-1] = True
        elif tok == "*":
            levels.append(False)
        else:
            base = BASE.get(tok, tok)
    out = base
    for i in range(len(levels) - 1):
        out = ("*const " if levels[i] else "*mut ") + out
    return out


def header_protos():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    src = re.sub(r"#.*", "", src)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(dtgpu_\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, params = " ".join(m.group(1).split()), m.group(2), m.group(3).strip()
        if ret.startswith("typedef"):
            continue
        plist = []
        if params and params != "void":
            for p in params.split(","):
                p = " ".join(p.split())
                arr = "[" in p
                p = re.sub(r"\[.*?\]", "", p)
                ty = re.sub(r"\b\w+$", "", p).strip()   # drop the parameter name
                plist.append(c_to_rust(ty + (" *" if arr else "")))
        protos[name] = (None if ret == "void" else c_to_rust(ret), plist)
    return protos


def rust_externs():
    src = open(os.path.join(CRATE, "src", "lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    out = {}
    for m in re.finditer(r"pub fn (dtgpu_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        params = [p.split(":", 1)[1].strip() for p in re.split(r",\s*(?![^()]*\))", " ".join(m.group(2).split())) if p.strip()]
        out[m.group(1)] = (m.group(3).strip() if m.group(3) else None, params)
    return out


def test_rust_externs_match_the_header():
    h, r = header_protos(), rust_externs()
    assert len(r) >= 25
    for name, (ret, params) in r.items():
        assert name in h, f"{name} is not in include/dtgpu.h"
        assert (ret, params) == h[name], f"{name}: rust {ret} {params} != header {h[name]}"
    for core in ("dtgpu_oplog_load", "dtgpu_checkout_tip", "dtgpu_batch_checkout", "dtgpu_xf_operations_from",
                 "dtgpu_oplog_decode_and_add"):
        assert core in r


def test_build_rs_links_static_archive_and_hip_runtime():
    b = open(os.path.join(CRATE, "build.rs")).read()
    assert "rustc-link-lib=static=dtgpu" in b and "rustc-link-lib=dylib=amdhip64" in b
    cargo = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'links = "dtgpu"' in cargo and 'build = "build.rs"' in cargo


def test_static_archive_defines_every_header_symbol():
    a = os.path.join(LIB, "libdtgpu.a")
    assert os.path.exists(a), "run `make -C diamond-types_amd static` (build() does)"
    syms = subprocess.run(["nm", "-g", "--defined-only", a], capture_output=True, text=True, check=True).stdout
    defined = set(re.findall(r" T (dtgpu_\w+)", syms))
    missing = set(header_protos()) - defined
    assert not missing, missing
    assert os.access(os.path.join(LIB, "checkout_tip_static"), os.X_OK)


@pytest.mark.gpu
def test_static_linked_c_program_checks_out_friendsforever(tmp_path):
    out = tmp_path / "ff.txt"
    dt = os.path.join(ROOT, "tests", "golden", "benchmark_data", "friendsforever.dt")
    r = subprocess.run([os.path.join(LIB, "checkout_tip_static"), dt, str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    gold = json.load(gzip.open(os.path.join(ROOT, "tests", "golden", "benchmark_data",
                                            "friendsforever_flat.json.gz")))["endContent"].encode()
    assert out.read_bytes() == gold
    assert int(r.stdout.split()[0]) == len(gold)
