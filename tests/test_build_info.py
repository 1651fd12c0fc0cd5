"""Build provenance of the native extension: csrc/build.py writes a source digest at link time,
ops/_ext.build_info() compares it with the tree it runs from (bench.py / smoke() report it)."""
import importlib.util
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "learning-deep-neural-network-in-distributed-computing-environment_amd")


def _load_build(path):
    spec = importlib.util.spec_from_file_location("_ldnn_build_t", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_source_digest_covers_every_source_and_changes_with_any(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(os.path.join(PKG, "csrc"), csrc, ignore=shutil.ignore_patterns("__pycache__"))
    b = _load_build(str(csrc / "build.py"))
    names = {os.path.relpath(f, str(csrc)) for f in b.sources()}
    assert "bindings.cpp" in names
    assert {os.path.join("kernels", f) for f in os.listdir(csrc / "kernels") if f.endswith(".hip")} <= names
    assert {os.path.join("include", f) for f in os.listdir(csrc / "include") if f.endswith(".h")} <= names
    d0 = b.source_digest()
    assert len(d0) == 64 and d0 == b.source_digest()
    k = sorted((csrc / "kernels").glob("*.hip"))[0]
    k.write_text(k.read_text() + "\n// edit\n")
    assert b.source_digest() != d0


def test_build_info_reports_whether_the_record_matches_this_tree():
    sys.path.insert(0, ROOT)
    from ldnn.ops import _ext

    info = _ext.build_info()
    assert "loaded" in info and "matches_sources" in info
    rec = os.path.join(PKG, "_C.build.json")
    if os.path.exists(rec):
        with open(rec) as f:
            sha = json.load(f)["sources_sha256"]
        b = _load_build(os.path.join(PKG, "csrc", "build.py"))
        assert info["matches_sources"] == (sha == b.source_digest())
        assert info["sources_sha16"] == sha[:16]
    else:
        assert info["matches_sources"] is None
