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
Branches are followed linearly, except that every loop body is walked again
seeded with the reads pending at its back-edge (cross-iteration prefetch);
scalar-memory loads count toward lgkmcnt out of order, so while one is in
flight only lgkmcnt(0) retires anything.  A report is a candidate to
inspect, not a proof; none is expected in the GEMM k-loops.

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


_SMEM = "smem"  # marker entry: a scalar-memory load in flight (counts toward lgkmcnt, out of order)


def _parse(path, only):
    """{function: [(line, op, operands-text)]} for the instructions of each function."""
    fns = {}
    fn = None
    for ln, line in enumerate(open(path)):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            fn = m.group(1)
            fns[fn] = []
            continue
        if fn is None or (only and only not in fn):
            continue
        t = line.split(";")[0].strip()
        if not t or (t.startswith(".") and not t.endswith(":")):
            continue
        fns[fn].append((ln + 1, t))
    return fns


def _walk(body, q, bad, fn, backedges=None):
    """Walks body in order from pending queue q; appends hazards to bad[fn].
    With backedges given, records (label index, queue) at every branch back to
    an earlier label of the function."""
    labels = {}
    for i, (ln, t) in enumerate(body):
        if t.endswith(":"):
            labels[t[:-1]] = i
            continue
        parts = t.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                if n == 0:
                    q = []
                elif _SMEM not in q:
                    q = q[len(q) - n:] if n < len(q) else q
                # an SMEM load in flight may be any of the n outstanding: nothing is retired for sure
            continue
        if backedges is not None and op.startswith(("s_branch", "s_cbranch")) and ops:
            tgt = ops[-1]
            if tgt in labels:
                backedges.append((labels[tgt], i, list(q)))
        if op.startswith(("s_load", "s_buffer_load")):
            q = q + [_SMEM]
            continue
        has_dst = not op.startswith(_NO_DST) and bool(ops)
        dst = _regs(ops[0]) if has_dst else set()
        srcs = set()
        for o in (ops[1:] if has_dst else ops):
            srcs |= _regs(o)
        pending = set().union(*[r for r in q if r is not _SMEM]) if q else set()
        hit = srcs & pending
        if hit:
            bad.setdefault(fn, []).append((ln, t[:80], tuple(sorted(hit)[:4])))
        if dst and not op.startswith("ds_read"):
            q = [r if r is _SMEM else r - dst for r in q]
        if op.startswith("ds_read"):
            q = q + [dst]
        elif op.startswith("ds_"):
            q = q + [set()]
    return q


def check(path, only=None):
    """Returns {function: [(line, instruction, registers)]}.  Each loop body
    (a label with a later branch back to it) is walked a second time seeded
    with the reads still pending at its back-edge, so reads issued at the end
    of one iteration and consumed at the top of the next are covered."""
    bad = {}
    for fn, body in _parse(path, only).items():
        backedges = []
        _walk(body, [], bad, fn, backedges)
        for li, bi, q in backedges:
            if any(r is _SMEM or r for r in q):
                _walk(body[li:bi + 1], q, bad, fn)
    for fn in bad:
        bad[fn] = sorted(set(bad[fn]))
    return bad


if __name__ == "__main__":
    res = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for f, v in res.items():
        print(len(v), f[:90])
        for x in v[:4]:
            print("    ", x)
    sys.exit(1 if res else 0)
