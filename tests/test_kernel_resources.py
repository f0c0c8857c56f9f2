"""Static checks on the compiled gfx950 kernels (no GPU): the build's
-Rpass-analysis=kernel-resource-usage report (tachikoma_amd/_build/kernel_resources.json).

A kernel that uses scratch memory (a register spill, or a local array / the kernel arguments
forced into memory by an escaping address) runs several times slower; the hot block kernel
must also keep the occupancy its LDS budget was sized for."""
import json
import os

import pytest

from tachikoma_amd import build

pytestmark = pytest.mark.skipif(not os.path.exists(build.RESOURCES), reason="library not built here")


def _report():
    with open(build.RESOURCES) as f:
        return json.load(f)


def test_every_hip_unit_reported():
    rep = _report()
    for src in build.SOURCES:
        if src.endswith(".hip"):
            assert rep.get(src), f"no resource report for {src}"


def test_no_kernel_uses_scratch():
    bad = [(u, k) for u, ks in _report().items() for k, v in ks.items() if v.get("ScratchSize", 0)]
    assert not bad, bad


def test_block_kernel_occupancy():
    """The fused conv-block kernels (64-row tiles, 64-byte stages) keep 4 workgroups per CU:
    16 waves, i.e. 4 waves per SIMD at <= 128 VGPRs and ~38 KB of LDS."""
    ks = _report()["tk_gemm.hip"]
    blk = {k: v for k, v in ks.items() if k.startswith("_ZN2tk14gemm_i8_kernelILi1ELb1ELb1ELi0ELi3ELb0ELi128E")}
    assert blk, "block kernel not found"
    for k, v in blk.items():
        assert v["Occupancy"] >= 4 and v["VGPRs"] <= 128 and v["LDS Size"] <= 40960, (k, v)


def test_block_kernel_256_column_occupancy():
    """The 256-column image-tile block kernel (14x14 expand layers) keeps 2 workgroups per CU:
    <= 80 KB of LDS (3-stage ring of 20 KB stages, 64 x 260-dword epilogue tile) and 2 waves per SIMD."""
    ks = _report()["tk_gemm.hip"]
    blk = {k: v for k, v in ks.items() if k.startswith("_ZN2tk14gemm_i8_kernelILi1ELb1ELb1ELi0ELi3ELb0ELi256E")}
    assert blk, "256-column block kernel not found"
    for k, v in blk.items():
        assert v["Occupancy"] >= 2 and v["LDS Size"] <= 81920, (k, v)
