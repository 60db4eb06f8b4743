"""Instruction mix of a kernel's main loop (the longest backward branch) in a
gfx950 .s, per category and per basic block.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ismer_music_generation_amd/csrc \\
          --cuda-device-only -S smer_music_generation_amd/csrc/attention.hip -o /tmp/attn.s
    python3 tools/isa_loop_stats.py /tmp/attn.s attn_fwd_bf16ILi64ELi2ELb1ELb0ELb0E

The second argument is a substring of the mangled kernel name.  Counts are
static (both sides of a branch); the per-block lines show which blocks a
common-case iteration skips."""
import collections
import re
import sys


def category(op, line):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp"):
        return "v_exp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch->" + line.split()[-1]
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, pat):
    s = open(path).read().split("\n")
    start = [i for i, l in enumerate(s) if re.match(r"^_Z\S*" + pat + r"\S*:", l)][0]
    end = start
    while not s[end].startswith(".Lfunc_end"):
        end += 1
    body = s[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    a, b = max(loops, key=lambda x: x[1] - x[0])
    total = collections.Counter()
    blocks, cur, c = [], "(loop head)", collections.Counter()
    for l in body[a:b + 1]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        t = l.strip()
        if m:
            blocks.append((cur, c))
            cur, c = m.group(1), collections.Counter()
            continue
        if not t or t.startswith((".", ";")):
            continue
        k = category(t.split()[0], t)
        c[k] += 1
        if not k.startswith("branch"):
            total[k] += 1
    blocks.append((cur, c))
    print("loop lines %d..%d: %s" % (a, b, dict(total)))
    for name, cnt in blocks:
        if cnt:
            print("  %-12s %s" % (name, dict(cnt)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
