"""Parity oracle — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's algorithms on the trace path:
  * qnn_ref.py      numpy restatement of the integer QNN semantics (pinned to the
                    reference's literal KATs in tests/golden/qnn_kats.json)
  * qnn_ref.c       OpenMP C restatement of conv/dense (CPU baseline + full-size checker)
  * graph_ref.py    per-op record-and-run over a Relay-style graph (mrt Trace.calibrate)
  * ndarray_list.py restatement of SaveParams/LoadParams (the trace tensor encoding)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker.  The product (tachikoma_amd) never calls it.
"""
import ctypes
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
C_LIB = os.path.join(HERE, "libqnnref.so")
_c = None


def build_c(force: bool = False) -> str:
    src = os.path.join(HERE, "qnn_ref.c")
    if not force and os.path.exists(C_LIB) and os.path.getmtime(C_LIB) >= os.path.getmtime(src):
        return C_LIB
    cc = shutil.which("gcc") or "gcc"
    tmp = C_LIB + ".tmp"
    subprocess.run([cc, "-O3", "-march=x86-64-v3", "-fopenmp", "-fwrapv", "-shared", "-fPIC", "-o", tmp, src],
                   check=True)
    os.replace(tmp, C_LIB)
    return C_LIB


def c_lib():
    global _c
    if _c is None:
        if not os.path.exists(C_LIB):
            build_c()
        lib = ctypes.CDLL(C_LIB)
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        lib.oracle_qnn_conv2d.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp] + [ctypes.c_int] * 16 + \
            [i32, i32, vp, ctypes.c_int]
        lib.oracle_qnn_conv2d.restype = ctypes.c_int
        lib.oracle_qnn_dense.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, i32, i32, vp, ctypes.c_int]
        lib.oracle_qnn_dense.restype = ctypes.c_int
        lib.oracle_num_threads.restype = ctypes.c_int
        _c = lib
    return _c
