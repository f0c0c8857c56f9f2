"""Round-5 ablations of the 3x3 image-tile kernels (ablation build, tools/bench_block.py): the
hand-pipelined K steps against the compiler-scheduled ones (TK_ABLATE 1<<22), and what is left when
the epilogue (4), the MFMAs (512), the LDS-DMA (128), the fragment reads (1<<20) and the stage
waits (1<<21) are removed.  Usage: python tools/abl_r05.py <layer substring> <ipt>"""
import json
import sys

OLD, NOREAD, NOWAIT = 1 << 22, 1 << 20, 1 << 21


def configs(ipt: str):
    base = {"TK_IMG_R": "32", "TK_IMG_CC": "64", "TK_IMG_IPT": ipt, "TK_IMG_TWO": "2", "TK_IMG_SPLIT": "0"}
    out = []
    for abl in (0, OLD, 4, OLD | 4, 512, NOREAD, NOREAD | 512, 128 | NOWAIT, 4 | 512 | 128, 4 | 512 | 128 | NOREAD,
                4 | 512 | 128 | NOREAD | NOWAIT):
        out.append(dict(base, TK_ABLATE=str(abl)) if abl else dict(base))
    out.append({"TK_IMG": "0"})
    return out


if __name__ == "__main__":
    print(json.dumps(configs(sys.argv[1])))
