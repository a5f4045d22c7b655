"""The build record of libdtgpu (lib/build_info.json, tools/build_info.py): it names the flags and
the hash of every source, it matches the sources in the tree, and the loader refuses a library
whose record names other sources (a stale prebuilt binary)."""
import hashlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "diamond-types_amd")
sys.path.insert(0, PKG)
import dt_amd  # noqa: E402

INFO = os.path.join(os.path.dirname(dt_amd.LIB_PATH), "build_info.json")


def test_record_matches_the_sources():
    if not os.path.exists(INFO):
        pytest.skip("library built without a record (experiment build directory)")
    rec = json.load(open(INFO))
    assert "gfx950" in " ".join(rec["flags"])
    assert any("amdgpu-atomic-optimizer-strategy" in f for f in rec["flags"])   # the replay's own flags
    srcs = rec["sources"]
    for name in ("csrc/dt_replay.hip", "csrc/dt_prep.hip", "csrc/dt_plan.hip", "csrc/dtgpu_api.cpp", "../include/dtgpu.h"):
        assert name in srcs
    for rel, h in srcs.items():
        with open(os.path.join(PKG, rel), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == h, rel
    with open(dt_amd.LIB_PATH, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == rec["library"]["sha256"]


def test_loader_refuses_other_sources(tmp_path, monkeypatch):
    lib_dir = tmp_path / "pkg" / "lib"
    lib_dir.mkdir(parents=True)
    (tmp_path / "pkg" / "csrc").mkdir()
    (tmp_path / "pkg" / "csrc" / "x.hip").write_bytes(b"edited after the build")
    (lib_dir / "build_info.json").write_text(json.dumps({"sources": {"csrc/x.hip": "0" * 64}}))
    monkeypatch.setattr(dt_amd, "LIB_PATH", str(lib_dir / "libdtgpu.so"))
    with pytest.raises(RuntimeError, match="other sources"):
        dt_amd._check_build_record()
    (lib_dir / "build_info.json").write_text(json.dumps(
        {"sources": {"csrc/x.hip": hashlib.sha256(b"edited after the build").hexdigest()}}))
    dt_amd._check_build_record()
