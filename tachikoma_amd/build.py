"""Build the in-tree HIP library ``tachikoma_amd/libtachikoma.so`` for gfx950.

Plain hipcc, no cmake: each translation unit is compiled to an object in
``tachikoma_amd/_build/`` (in parallel) and linked into one shared library whose
exported symbols are exactly the ``extern "C"`` entry points of
``include/tachikoma.h``.
"""
from __future__ import annotations

import concurrent.futures
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
ARCH = os.environ.get("TK_OFFLOAD_ARCH", "gfx950")

SOURCES = ["tk_host.cc", "tk_calibrate.cc", "tk_format.cc", "tk_runtime.cc", "tk_elementwise.hip", "tk_gemm.hip", "tk_residual.hip", "tk_realize.hip"]
HEADERS = ["tk_common.h"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the tachikoma HIP library cannot be built")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


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
    hipcc = _hipcc()
    cmd = [hipcc, "-std=c++17", "-O3", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}",
           "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function", "-c", src, "-o", obj] + extra
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


def build_ablation(verbose: bool = True) -> str:
    """Profiling variant with the main-loop ablation switches compiled in (TK_ABLATE env, see
    GemmArgs::ablate): tachikoma_amd/_ab/libtachikoma_ablate.so, loaded by the tools through
    TK_LIB_PATH.  The product library has them compiled out."""
    out_dir = os.path.join(HERE, "_ab")
    obj_dir = os.path.join(BUILD, "ablate")
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(obj_dir, exist_ok=True)
    objs = []
    for s in SOURCES:
        obj = os.path.join(obj_dir, s + ".o")
        _compile(os.path.join(CSRC, s), obj, ["-DTK_ABLATION_BUILD"])
        objs.append(obj)
    lib = os.path.join(out_dir, "libtachikoma_ablate.so")
    subprocess.run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs, check=True)
    if verbose:
        print(f"[tachikoma] built {lib}")
    return lib


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "tachikoma.h")]
    jobs = []
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD, s + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + hdrs + [__file__]):
            jobs.append((src, obj))
    if jobs:
        workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")))
        res = {}
        if os.path.exists(RESOURCES):
            with open(RESOURCES) as f:
                res = json.load(f)
        with concurrent.futures.ThreadPoolExecutor(max_workers=workers) as ex:
            futs = [(os.path.basename(s), ex.submit(_compile, s, o, [])) for s, o in jobs]
            for name, f in futs:
                r = f.result()
                if name.endswith(".hip"):
                    res[name] = r
        with open(RESOURCES, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
        # a kernel that spills to scratch (or copies its arguments there) runs several times
        # slower: fail the build instead of shipping it
        bad = [k for unit in res.values() for k, v in unit.items() if v.get("ScratchSize", 0)]
        if bad:
            raise RuntimeError(f"kernels using scratch memory: {bad[:5]} (see {RESOURCES})")
    if force or jobs or not _newer(LIB, objs):
        tmp = LIB + ".tmp"
        subprocess.run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs, check=True)
        os.replace(tmp, LIB)
        if verbose:
            print(f"[tachikoma] built {LIB}")
    return LIB


if __name__ == "__main__":
    if "--ablation" in sys.argv:
        build_ablation()
    else:
        build(force="--force" in sys.argv)
