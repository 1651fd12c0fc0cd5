"""Loader of the native gfx950 extension (`_C.so`, built in-tree by csrc/build.py).

Policy: on a machine with a GPU the native kernels are THE compute path -- if
the extension is missing there, importing it raises instead of silently
falling back to PyTorch/MIOpen.  On a CPU-only host (CI, the orchestration
tests) the ops run their plain PyTorch fp32 reference implementation.
Set LDNN_DISABLE_NATIVE=1 only to run the stock-PyTorch comparison baseline.
"""
from __future__ import annotations

import os

import torch

_C = None
_IMPORT_ERROR: Exception | None = None
try:  # the .so sits next to this package's __init__.py
    from .. import _C as _C  # type: ignore[attr-defined,no-redef]
except Exception as e:  # pragma: no cover - depends on build state
    _IMPORT_ERROR = e

_DISABLED = os.environ.get("LDNN_DISABLE_NATIVE", "0") == "1"


def native_available() -> bool:
    return _C is not None and not _DISABLED


def C():
    """Return the native module or raise a loud, actionable error."""
    if _C is None:
        raise RuntimeError(
            "ldnn native extension (_C.so) is not built/loadable: "
            f"{_IMPORT_ERROR!r}. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `python learning-deep-neural-network-in-distributed-computing-environment_amd/csrc/build.py`."
        )
    return _C


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on the GPU and must take the native HIP path."""
    if not t.is_cuda:
        return False
    if _DISABLED:
        return False
    C()  # raises if the extension is missing on a GPU box
    return True


def build_info() -> dict:
    """Provenance of the loaded `_C.so`: the record csrc/build.py wrote at link time and
    whether its source digest equals the sources in this tree (`matches_sources`)."""
    import importlib.util
    import json

    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    info: dict = {"loaded": _C is not None, "so": getattr(_C, "__file__", None)}
    try:
        with open(os.path.join(pkg, "_C.build.json")) as f:
            info.update(json.load(f))
        spec = importlib.util.spec_from_file_location("_ldnn_build", os.path.join(pkg, "csrc", "build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        info["matches_sources"] = info.get("sources_sha256") == mod.source_digest()
    except OSError as e:
        info["matches_sources"] = None
        info["error"] = f"no build record: {e.__class__.__name__}"
    if "sources_sha256" in info:
        info["sources_sha16"] = info.pop("sources_sha256")[:16]
    return info


def check_gpu_native() -> None:
    """Fail loudly on a GPU host without the native extension."""
    if torch.cuda.is_available() and not _DISABLED:
        C()
