"""Teardown order of the native module (CPU, no GPU): the device is synchronised before
tk_module_destroy, destroy runs once, never from a finaliser during interpreter shutdown, and the
atexit hook closes modules left open before the interpreter finalises (the
exit SIGSEGV inside __cxa_finalize)."""
import ctypes
import os
import subprocess
import sys

import pytest

from tachikoma_amd.relay import device_module as dm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeLib:
    def __init__(self, log):
        self.log = log

    def tk_module_destroy(self, h):
        self.log.append(("destroy", h.value, sys.is_finalizing()))
        return 0


def _fake_module(log):
    m = object.__new__(dm.DeviceModule)
    m.lib = _FakeLib(log)
    m.handle = ctypes.c_void_p(0x1234)
    m.device = "cuda:0"
    m.buffers = {"x": object()}
    m._keep = [object()]
    dm._LIVE.add(m)
    return m


@pytest.fixture
def sync_log(monkeypatch):
    import torch
    log = []
    monkeypatch.setattr(torch.cuda, "synchronize", lambda device=None: log.append(("sync", str(device))))
    return log


def test_close_synchronises_then_destroys_once(sync_log):
    m = _fake_module(sync_log)
    assert not m.closed
    m.close()
    assert sync_log == [("sync", "cuda:0"), ("destroy", 0x1234, False)]
    assert m.closed and m.buffers == {} and m._keep == [] and m not in dm._LIVE
    m.close()
    m.__del__()
    assert len(sync_log) == 2


def test_del_during_finalisation_makes_no_native_call(sync_log, monkeypatch):
    m = _fake_module(sync_log)
    monkeypatch.setattr(sys, "is_finalizing", lambda: True)
    m.__del__()
    assert sync_log == []
    monkeypatch.undo()
    dm._LIVE.discard(m)


def test_close_all_closes_every_live_module(sync_log):
    a, b = _fake_module(sync_log), _fake_module(sync_log)
    dm.close_all()
    assert a.closed and b.closed
    assert [e[0] for e in sync_log] == ["sync", "destroy", "sync", "destroy"]


def test_atexit_hook_runs_before_finalisation():
    """A module left open at exit is destroyed by the atexit hook, i.e. while the interpreter (and
    the HIP runtime under it) is still up -- not by a finaliser and not after static destructors."""
    code = f"""
import ctypes, sys
sys.path.insert(0, {ROOT!r})
import torch
torch.cuda.synchronize = lambda device=None: print("sync", flush=True)
from tachikoma_amd.relay import device_module as dm
class L:
    def tk_module_destroy(self, h):
        print("destroy", hex(h.value), "finalizing" if sys.is_finalizing() else "live", flush=True)
        return 0
m = object.__new__(dm.DeviceModule)
m.lib, m.handle, m.device, m.buffers, m._keep = L(), ctypes.c_void_p(0xbeef), "cuda:0", {{}}, []
dm._LIVE.add(m)
keep = m  # still referenced at exit
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split("\n")[:2] == ["sync", "destroy 0xbeef live"], r.stdout


def test_rocprof_one_hsa_wrapper(tmp_path):
    """tools/rocprof_one_hsa.sh (the exit SIGSEGV's cause: two HSA runtimes under rocprofv3, DESIGN.md
    §8) offers torch's bundled runtime under the soname the profiler's libraries ask for, first on
    LD_LIBRARY_PATH, and hands every argument to rocprofv3 unchanged (a stand-in rocprofv3 here)."""
    import torch
    fake = tmp_path / "bin"
    fake.mkdir()
    (fake / "rocprofv3").write_text('#!/bin/bash\necho "LDP=$LD_LIBRARY_PATH"\nfor a in "$@"; do echo "ARG=$a"; done\n')
    (fake / "rocprofv3").chmod(0o755)
    env = dict(os.environ, PATH=f"{fake}:{os.environ['PATH']}", TMPDIR=str(tmp_path), LD_LIBRARY_PATH="/x")
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "rocprof_one_hsa.sh"), "--memory-copy-trace", "-d",
                          "a b", "--", "python3", "bench.py"], env=env, capture_output=True, text=True, check=True).stdout
    lines = out.splitlines()
    ldp = next(x for x in lines if x.startswith("LDP="))[4:].split(":")
    assert ldp[0] == str(tmp_path / "tk_one_hsa") and ldp[1:] == ["/x"]
    link = tmp_path / "tk_one_hsa" / "libhsa-runtime64.so.1"
    want = os.path.join(os.path.dirname(torch.__file__), "lib", "libhsa-runtime64.so")
    assert os.path.realpath(link) == os.path.realpath(want)
    assert [x[4:] for x in lines if x.startswith("ARG=")] == ["--memory-copy-trace", "-d", "a b", "--", "python3",
                                                             "bench.py"]
