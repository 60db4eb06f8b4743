"""Static hazard check for the asm LDS reads (csrc/common.h
lds_read_tr16_async / lds_read_b128_async).

hipcc treats an asm statement's output register as ready the moment the
statement ends; the kernels retire those reads themselves (s_waitcnt
lgkmcnt) before the MFMAs use them.  Any other instruction that reads such
a register in between -- typically a spill store or a register copy the
compiler inserts under register pressure -- reads it before the LDS data has
landed (seen once: a spilled fp8 B fragment).  This walks a gfx950 .s in
program order per function and reports every instruction that reads a
register written by a ds_read which no s_waitcnt lgkmcnt has retired yet
(LDS operations retire in order; a write to the register ends the hazard).
Branches are followed linearly, so a report is a candidate to inspect, not a
proof; none is expected in the GEMM k-loops.

    python tools/lgkm_check.py build/gemm-hip-amdgcn-amd-amdhsa-gfx950.s [kernel-substring]
"""
import re
import sys


def _regs(tok):
    tok = tok.strip()
    m = re.match(r"^([va])\[(\d+):(\d+)\]$", tok)
    if m:
        return {m.group(1) + str(i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    if re.match(r"^[va]\d+$", tok):
        return {tok}
    return set()


_NO_DST = ("ds_write", "global_store", "buffer_store", "scratch_store", "flat_store", "global_atomic",
           "s_", "global_load_lds", "buffer_load_dword lds")


def check(path, only=None):
    """Returns {function: [(line, instruction, registers)]}."""
    bad = {}
    fn = None
    q = []  # register sets of in-flight LDS ops, oldest first
    for ln, line in enumerate(open(path)):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            fn = m.group(1)
            q = []
            continue
        if fn is None or (only and only not in fn):
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        parts = t.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                q = q[len(q) - n:] if n < len(q) else q
            continue
        has_dst = not op.startswith(_NO_DST) and bool(ops)
        dst = _regs(ops[0]) if has_dst else set()
        srcs = set()
        for o in (ops[1:] if has_dst else ops):
            srcs |= _regs(o)
        pending = set().union(*q) if q else set()
        hit = srcs & pending
        if hit:
            bad.setdefault(fn, []).append((ln + 1, t[:80], sorted(hit)[:4]))
        if dst and not op.startswith("ds_read"):
            q = [r - dst for r in q]
        if op.startswith("ds_read"):
            q.append(dst)
        elif op.startswith("ds_"):
            q.append(set())
    return bad


if __name__ == "__main__":
    res = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for f, v in res.items():
        print(len(v), f[:90])
        for x in v[:4]:
            print("    ", x)
    sys.exit(1 if res else 0)
