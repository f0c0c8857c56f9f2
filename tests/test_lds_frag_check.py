"""tools/check_lds_frags.py (the round-5 advisor's check on the image-tile kernel's inline-asm
fragment reads) finds a use of a pending inline-asm ds_read_b128 destination and accepts the
counted-wait pattern; its run on the real gfx950 assembly is profiles/r06_lds_fragment_check.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_lds_frags  # noqa: E402

HEAD = "_ZN2tk15conv_img_kernelILi3E_test:\n"
TAIL = ".Lfunc_end0:\n"


def _run(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text(HEAD + body + TAIL)
    return check_lds_frags.main(str(p), "conv_img_kernel")


def test_counted_wait_pattern_passes(tmp_path):
    body = """\t;;#ASMSTART
\tds_read_b128 v[0:3], v10
\t;;#ASMEND
\t;;#ASMSTART
\tds_read_b128 v[4:7], v11
\t;;#ASMEND
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(1)
\t;;#ASMEND
\tv_mfma_i32_32x32x32_i8 a[0:15], v[0:3], v[20:23], a[0:15]
\ts_waitcnt lgkmcnt(0)
\tv_mov_b32_e32 v30, v5
"""
    assert _run(tmp_path, body) == 0


def test_use_before_the_wait_is_reported(tmp_path):
    body = """\t;;#ASMSTART
\tds_read_b128 v[0:3], v10
\t;;#ASMEND
\tds_read_b32 v40, v12
\tv_mov_b32_e32 v30, v2
\ts_waitcnt lgkmcnt(1)
"""
    assert _run(tmp_path, body) == 1


def test_loop_carried_read_is_checked(tmp_path):
    body = """.LBB0_1:
\tv_mov_b32_e32 v31, v1
\t;;#ASMSTART
\tds_read_b128 v[0:3], v10
\t;;#ASMEND
\ts_cbranch_scc1 .LBB0_1
\ts_waitcnt lgkmcnt(0)
"""
    assert _run(tmp_path, body) == 1
