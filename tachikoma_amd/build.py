"""Build the in-tree HIP library ``tachikoma_amd/libtachikoma.so`` for gfx950.

Plain hipcc, no cmake: each translation unit is compiled to an object in
``tachikoma_amd/_build/`` (in parallel) and linked into one shared library whose
exported symbols are exactly the ``extern "C"`` entry points of
``include/tachikoma.h``.

Rebuilds are decided by content, not by file times: ``source_hash()`` digests every
source, header and the compile flags and is compiled into the library (``tk_build_info()``,
tk_host.cc only), so ``_lib.load()`` can refuse a library that does not match the tree it is
imported from (a stale binary pushed to a GPU box).  Each object carries a stamp of what it was
built from -- its own source, the shared headers, the flags (and, for tk_host.cc, the tree
digest) -- so an edit to one kernel file recompiles that file, not the whole library.
"""
from __future__ import annotations

import concurrent.futures
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libtachikoma.so")
ARCH = "gfx950"

SOURCES = ["tk_host.cc", "tk_calibrate.cc", "tk_format.cc", "tk_runtime.cc", "tk_elementwise.hip", "tk_gemm.hip",
           "tk_residual.hip", "tk_realize.hip", "tk_conv_img.hip", "tk_conv_pf.hip", "tk_qnn_ops.hip", "tk_dense.hip", "tk_dw.hip"]
HEADERS = ["tk_common.h", "tk_conv.h"]
BASE_FLAGS = ["-std=c++20", "-O3", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", "-Wall",
              "-Wno-unused-function"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the tachikoma HIP library cannot be built")


def _hash_inputs():
    return ([os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS] +
            [os.path.join(ROOT, "include", "tachikoma.h")])


def source_hash() -> str:
    """Digest of everything the library is compiled from (sources, headers, flags)."""
    h = hashlib.sha256()
    h.update(" ".join(BASE_FLAGS).encode())
    for path in _hash_inputs():
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


RESOURCES = os.path.join(BUILD, "kernel_resources.json")
_REMARK = re.compile(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                     r"LDS Size \[bytes/block\]):\s*(\S+)")


def _resources(stderr: str):
    """Per-kernel register / scratch / LDS / occupancy from -Rpass-analysis=kernel-resource-usage."""
    out, cur = {}, None
    for key, val in _REMARK.findall(stderr):
        if key == "Function Name":
            cur = out.setdefault(val, {})
        elif cur is not None:
            cur[key.split(" [")[0]] = int(val) if val.lstrip("-").isdigit() else val
    return out


def _compile(src: str, obj: str, extra):
    cmd = [_hipcc()] + BASE_FLAGS + ["-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj] + extra
    if src.endswith(".cc"):
        cmd[1:1] = ["-x", "hip"]
    else:
        cmd += ["-Rpass-analysis=kernel-resource-usage", "-fno-caret-diagnostics"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    noise = [ln for ln in r.stderr.splitlines() if "kernel-resource-usage" not in ln and ln.strip()]
    if noise:
        sys.stderr.write("\n".join(noise) + "\n")
    if r.returncode != 0:
        raise subprocess.CalledProcessError(r.returncode, cmd)
    return _resources(r.stderr)


def _stamp(obj: str) -> str:
    return obj + ".stamp"


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


def _write(path: str, text: str) -> None:
    with open(path, "w") as f:
        f.write(text)


def _object_stamp(src: str, defines, build_id: str) -> str:
    """What one object is compiled from: its source, the shared headers, the flags; tk_host.cc
    also embeds the tree digest (tk_build_info)."""
    h = hashlib.sha256()
    h.update(" ".join(BASE_FLAGS + list(defines)).encode())
    for path in [os.path.join(CSRC, src)] + [p for p in _hash_inputs() if not p.endswith(tuple(SOURCES))]:
        with open(path, "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read() + b"\0")
    if src == "tk_host.cc":
        h.update(build_id.encode())
    return h.hexdigest()[:16]


def _build_into(obj_dir: str, lib: str, defines, tag: str, force: bool, verbose: bool) -> str:
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    digest = source_hash()
    build_id = digest + tag
    if not force and os.path.exists(lib) and _read(_stamp(lib)) == build_id:
        return lib  # up to date (objects are only consulted when something must be rebuilt)
    jobs, objs = [], []
    for s in SOURCES:
        obj = os.path.join(obj_dir, s + ".o")
        objs.append(obj)
        stamp = _object_stamp(s, list(defines), build_id)
        if force or not os.path.exists(obj) or _read(_stamp(obj)) != stamp:
            extra = list(defines) + ([f'-DTK_SOURCE_HASH="{build_id}"'] if s == "tk_host.cc" else [])
            jobs.append((os.path.join(CSRC, s), obj, extra, stamp))
    if jobs:
        workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")))
        res = {}
        if os.path.exists(RESOURCES):
            with open(RESOURCES) as f:
                res = json.load(f)
        with concurrent.futures.ThreadPoolExecutor(max_workers=workers) as ex:
            futs = [(os.path.basename(s), o, st, ex.submit(_compile, s, o, extra)) for s, o, extra, st in jobs]
            for name, o, st, f in futs:
                r = f.result()
                _write(_stamp(o), st)
                if name.endswith(".hip") and not tag:
                    res[name] = r
        if not tag:
            with open(RESOURCES, "w") as f:
                json.dump(res, f, indent=1, sort_keys=True)
            # a kernel that spills to scratch (or copies its arguments there) runs several times
            # slower: fail the build instead of shipping it
            bad = [k for unit in res.values() for k, v in unit.items() if v.get("ScratchSize", 0)]
            if bad:
                raise RuntimeError(f"kernels using scratch memory: {bad[:5]} (see {RESOURCES})")
    if force or jobs or not os.path.exists(lib) or _read(_stamp(lib)) != build_id:
        tmp = lib + ".tmp"
        subprocess.run([_hipcc(), "-shared", "-fPIC", "-pthread", f"--offload-arch={ARCH}", "-o", tmp] + objs,
                       check=True)
        os.replace(tmp, lib)
        _write(_stamp(lib), build_id)
        if verbose:
            print(f"[tachikoma] built {lib} ({build_id})")
    return lib


def build_ablation(verbose: bool = True) -> str:
    """Profiling variant with the kernel-selection and main-loop ablation switches read from
    the environment (TK_ABLATE, TK_XCD, TK_RING, ...; see tune_env in csrc/tk_gemm.hip):
    tachikoma_amd/_ab/libtachikoma_ablate.so, loaded by the tools through TK_LIB_PATH.  The
    product library has them compiled out."""
    return _build_into(os.path.join(BUILD, "ablate"), os.path.join(HERE, "_ab", "libtachikoma_ablate.so"),
                       ["-DTK_ABLATION_BUILD"], "+ablation", False, verbose)


def build(force: bool = False, verbose: bool = True) -> str:
    return _build_into(BUILD, LIB, [], "", force, verbose)


if __name__ == "__main__":
    if "--ablation" in sys.argv:
        build_ablation()
    else:
        build(force="--force" in sys.argv)
