"""Check, on the gfx950 assembly of the image-tile kernel, that no instruction touches the
destination VGPRs of an LDS read before a counted `s_waitcnt lgkmcnt` has retired that read.

Why: `compute_asm` in csrc/tk_conv_img.hip issues its fragment reads as inline-asm
`ds_read_b128` two K steps ahead and retires them with counted `s_waitcnt lgkmcnt(N)`; the
compiler does not know those registers are still being written by the LDS, so a register copy,
spill or reuse of them before the wait would read stale data.  The empty "+v" pins after each
wait cannot prevent a copy made before it (round-5 advisor finding).  This tool models the LGKM
counter: LDS operations retire in issue order, `s_waitcnt lgkmcnt(N)` retires the oldest until
N remain; an instruction reading or writing a VGPR of a not-yet-retired `ds_read*` is a
violation.  Only the reads inside inline-asm regions (`;;#ASMSTART` .. `;;#ASMEND`) are tracked as
pending -- the compiler's own LDS reads are covered by its waitcnt insertion -- but every LDS
operation counts against lgkmcnt.  Scalar memory loads share the counter and retire out of order,
so while one is in flight only `lgkmcnt(0)` is trusted (the stage loop has none).  Straight-line
scan of each function (the dead fall-through after an unconditional branch starts empty) plus one
extra pass around every backward branch (loop-carried reads).

usage: python tools/check_lds_frags.py <gfx950 .s> [symbol substring]
  (the .s: hipcc -std=c++20 -O3 --offload-arch=gfx950 --cuda-device-only -S -Iinclude
   tachikoma_amd/csrc/tk_conv_img.hip -o conv_img.s)
exit status 1 if a violation is found.
"""
import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
WAIT = re.compile(r"lgkmcnt\((\d+)\)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add(f"{m.group(1)}{m.group(2)}")
        else:
            out.update(f"{m.group(3)}{i}" for i in range(int(m.group(4)), int(m.group(5)) + 1))
    return out


def split_ops(line):
    """mnemonic, destination VGPR/AGPR set, source set (the first operand is the destination of a
    VALU / LDS read / MFMA; stores and s_* have no vector destination)."""
    code = line.split(";")[0].strip()
    if not code or code.endswith(":") or code.startswith("."):
        return None, set(), set()
    parts = code.split(None, 1)
    mn = parts[0]
    ops = parts[1] if len(parts) > 1 else ""
    operands = [o.strip() for o in ops.split(",")]
    if not operands or not operands[0]:
        return mn, set(), set()
    stores = ("ds_write", "ds_store", "buffer_store", "global_store", "flat_store", "scratch_store")
    if mn.startswith(stores) or mn.startswith("s_") or mn.startswith("v_cmp") or mn.startswith("v_readfirstlane") \
            or mn.startswith("v_readlane"):
        return mn, set(), regs(ops)
    return mn, regs(operands[0]), regs(",".join(operands[1:]))


def scan(lines, start, stop, queue, report, func):
    """Scan lines[start:stop] from LGKM queue `queue` (list of (is_lds_read, dst regs))."""
    q = [list(e) for e in queue]
    smem = sum(1 for e in q if e[0] == "smem")
    back = []
    in_asm = False
    for i in range(start, stop):
        line = lines[i]
        if ";;#ASMSTART" in line:
            in_asm = True
            continue
        if ";;#ASMEND" in line:
            in_asm = False
            continue
        mn, dst, src = split_ops(line)
        if mn is None:
            continue
        if mn.startswith("s_waitcnt"):
            m = WAIT.search(line)
            if m:
                n = int(m.group(1))
                if smem and n > 0:
                    n = len(q)  # out-of-order scalar loads in flight: nothing is known retired
                while len(q) > n:
                    e = q.pop(0)
                    smem -= e[0] == "smem"
            continue
        pending = set()
        for e in q:
            if e[0] == "lds":
                pending |= e[1]
        bad = (src | dst) & pending
        if bad:
            report.append((func, i + 1, line.strip(), sorted(bad)))
        if mn.startswith("ds_"):
            q.append(["lds", dst if in_asm and mn.startswith(("ds_read", "ds_load")) else set()])
        elif mn.startswith(("s_load", "s_buffer_load")):
            q.append(["smem", set()])
            smem += 1
        if mn.startswith("s_cbranch") or mn.startswith("s_branch"):
            back.append((i, line.split()[-1], [list(e) for e in q]))
        if mn in ("s_branch", "s_endpgm", "s_setpc_b64"):
            q, smem = [], 0  # the fall-through is reached from elsewhere
    return back


def main(path, want="conv_img_kernel"):
    lines = open(path).read().split("\n")
    funcs = []
    for i, line in enumerate(lines):
        m = re.match(r"^(_Z\S+):", line)
        if m and want in m.group(1):
            end = next(j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end"))
            funcs.append((m.group(1), i, end))
    report, nreads, nasm = [], 0, 0
    for name, a, b in funcs:
        labels = {lines[k].split(":")[0]: k for k in range(a, b) if re.match(r"^\.LBB\S*:", lines[k])}
        nreads += sum(1 for k in range(a, b) if "ds_read_b128" in lines[k])
        inside = False
        for k in range(a, b):
            inside = (inside or ";;#ASMSTART" in lines[k]) and ";;#ASMEND" not in lines[k]
            nasm += inside and "ds_read_b128" in lines[k]
        back = scan(lines, a, b, [], report, name)
        for at, target, q in back:  # loop-carried: from the branch target to the branch, with its queue
            if target in labels and labels[target] < at:
                scan(lines, labels[target], at, q, report, name)
    print(f"{len(funcs)} functions, {nreads} ds_read_b128 ({nasm} in inline asm), {len(report)} violations")
    for func, ln, text, bad in report[:20]:
        print(f"  {func[:60]} line {ln}: {text}  (pending {bad})")
    return 1 if report else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
