"""Pure-Python mirror of csrc/decode_ops.hip grammar_greedy_kernel (test
infrastructure): one request's state vector, one step of masked argmax +
commit + next feed, so the CPU suite can check the kernel's state machine
against the host `_Span` (generation.py:528-687 restated)."""
import numpy as np

F_SEP, F_CONT, F_PITCH, F_REST = 1, 2, 4, 8
C_CONT, C_PITCH, C_DUR, C_SEPSTR, C_RESTSTR, C_CTRL = 1, 2, 4, 8, 16, 32


def state_code(flags, ln, target, no_whole):
    if flags & F_SEP:
        return 0
    if flags & F_CONT:
        return 1
    if flags & F_PITCH:
        return 2 + no_whole
    if flags & F_REST:
        return 4 + no_whole
    if ln == 1:
        return 10 if target == 0 else 5 + target
    return 11 + no_whole


def step(st, targets, keep, cls, logit, *, eos, m0, trash_pos, src_len, max_span=100):
    """st: dict(pos, flags, len, midx, nmask, done, no_whole, count, err).
    Returns (idx, rows) with rows = [(id, pos, nks, nkc)] for slots 2r, 2r+1."""
    code = state_code(st["flags"], st["len"], targets[st["midx"]], st["no_whole"])
    x = np.where(keep[code].astype(bool), logit.astype(np.float32), np.float32(-100.0))
    idx = int(np.argmax(x))
    c = int(cls[idx])
    f = st["flags"]
    if c & C_CONT:
        f = (f | F_CONT) & ~F_SEP
    if c & C_PITCH:
        f = (f | F_PITCH) & ~(F_SEP | F_CONT)
    if c & C_DUR:
        f &= ~(F_REST | F_PITCH)
    if c & C_SEPSTR:
        f |= F_SEP
    if c & C_RESTSTR:
        f |= F_REST
    st["count"] += 1
    pos = st["pos"]
    if c & C_CTRL:
        end, feed = True, [idx, m0]
    elif idx == eos or st["len"] + 1 >= max_span:
        end, feed = True, [m0]
    else:
        end, feed = False, [idx]
    done = False
    if end:
        st["midx"] += 1
        if st["midx"] >= st["nmask"]:
            done, feed = True, []
        else:
            f = 0
            st["len"] = 1
    else:
        st["len"] += 1
    st["flags"] = f
    if not done and pos + len(feed) > trash_pos:
        st["err"], done = 1, True
    rows = []
    nf = len(feed)
    for k in range(2):
        j = k - (2 - nf)
        real = not done and j >= 0
        rows.append((feed[j], pos + j, pos + j + 1, max(src_len, 1)) if real
                    else (0, trash_pos, 1, 1))
    if done:
        st["done"] = 1
    else:
        st["pos"] = pos + nf
    return idx, rows
