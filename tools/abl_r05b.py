"""Where the 3x3 image-tile kernels' fixed time goes (ablation build): return at wave start (1<<23),
after the prologue (1<<24), the K-loop skeleton (no epilogue / MFMA / DMA / fragment reads / stage
waits), the skeleton with the stage waits, and the full kernel.  Usage: python tools/abl_r05b.py <ipt>"""
import json
import sys

if __name__ == "__main__":
    base = {"TK_IMG_R": "32", "TK_IMG_CC": "64", "TK_IMG_IPT": sys.argv[1], "TK_IMG_TWO": "2", "TK_IMG_SPLIT": "0"}
    abls = [1 << 23, 1 << 24, 4 | 512 | 128 | (1 << 20) | (1 << 21), 4 | 512 | 128 | (1 << 20), 4, 0]
    cfgs = [dict(base, TK_ABLATE=str(a)) if a else dict(base) for a in abls]
    cfgs += [dict(base, TK_IMG_TWO="0", TK_ABLATE=str(1 << 23)), dict(base, TK_IMG_CC="32", TK_ABLATE=str(1 << 23))]
    print(json.dumps(cfgs))
