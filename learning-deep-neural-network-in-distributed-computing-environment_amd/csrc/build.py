"""In-tree build of the ldnn native extension (`_C.so`) for gfx950.

No hipify and no torch JIT cache: every `.hip` kernel file is compiled by
`hipcc --offload-arch=gfx950` straight from CDNA4 source, the pybind layer
(`bindings.cpp`) is compiled against the installed torch headers, and the
objects are linked into `<package>/_C.so`, which travels with the repo
snapshot to the GPU box.  Rebuilds are incremental (mtime based).  Every link
also writes `<package>/_C.build.json` (sha256 over the sources it was built
from, arch, hipcc version); `ops/_ext.build_info()` compares it with the tree
it is imported from, and `bench.py` / `smoke()` report the result, so a stale
`_C.so` is visible in every record.

Usage:  python -m <pkg>.csrc.build   or   python <pkg>/csrc/build.py [-v] [--force]
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(HERE)
REPO = os.path.dirname(PKG_DIR)
BUILD_DIR = os.path.join(REPO, "build", "ldnn_C")
OUT = os.path.join(PKG_DIR, "_C.so")
INFO = os.path.join(PKG_DIR, "_C.build.json")
ARCH = os.environ.get("LDNN_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch

    inc = ce.include_paths()
    lib = ce.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _deps(path):
    headers = glob.glob(os.path.join(HERE, "include", "*.h"))
    return [path] + headers


def sources() -> list[str]:
    """Every file the extension is compiled from (kernels, bindings, headers)."""
    return sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip")) + glob.glob(os.path.join(HERE, "include", "*.h"))
                  + [os.path.join(HERE, "bindings.cpp")])


def source_digest() -> str:
    h = hashlib.sha256()
    for f in sources():
        h.update(os.path.relpath(f, HERE).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def _write_info():
    try:
        ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout
        ver = next((ln.strip() for ln in ver.splitlines() if "HIP version" in ln), ver.strip()[:80])
    except OSError:
        ver = "unknown"
    import datetime

    info = {"sources_sha256": source_digest(), "n_sources": len(sources()), "arch": ARCH, "hipcc": ver,
            "built_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")}
    with open(INFO + ".tmp", "w") as f:
        json.dump(info, f)
    os.replace(INFO + ".tmp", INFO)


def _stale(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(verbose: bool = False, force: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    inc, lib, abi = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{os.path.join(HERE, 'include')}", "-Wno-unused-result"]
    kern_flags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    py_inc = sysconfig.get_paths()["include"]
    import pybind11

    bind_flags = common + [
        "-x", "c++",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_C",
        f"-I{py_inc}",
        f"-I{pybind11.get_include()}",
        f"-I{os.path.join(ROCM, 'include')}",
    ] + [f"-I{p}" for p in inc]

    jobs_list = []
    for src in sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))):
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        jobs_list.append((src, obj, [HIPCC] + kern_flags + ["-c", src, "-o", obj]))
    bsrc = os.path.join(HERE, "bindings.cpp")
    bobj = os.path.join(BUILD_DIR, "bindings.o")
    jobs_list.append((bsrc, bobj, [HIPCC] + bind_flags + ["-c", bsrc, "-o", bobj]))

    todo = [(s, o, c) for (s, o, c) in jobs_list if force or _stale(o, _deps(s))]
    if todo:
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 4)), 16)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            futs = [ex.submit(_run, c, verbose) for (_, _, c) in todo]
            for f in futs:
                f.result()
    objs = [o for (_, o, _) in jobs_list]
    if force or todo or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT + ".tmp"] + objs
        for p in lib:
            link += [f"-L{p}", f"-Wl,-rpath,{p}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64",
                 f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lrocprofiler-sdk-roctx"]
        _run(link, verbose)
        os.replace(OUT + ".tmp", OUT)
        _write_info()
    elif not os.path.exists(INFO):
        _write_info()   # (an up-to-date .so from before the provenance file existed)
    return OUT


if __name__ == "__main__":
    out = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(out)
