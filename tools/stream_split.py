"""Per-stream busy time of a rocprofv3 kernel trace over the last N steps
(which stream is the critical path of the overlapped train step).
    python tools/stream_split.py run_kernel_trace.csv [steps] [step_kernel_regex]"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
marker = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"^embed_bwd_reduce")  # once per step, at the end of backward
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if marker.search(r["Kernel_Name"])]
if len(ends) < steps + 1:
    sys.exit("not enough steps (%d markers)" % len(ends))
sel = rows[ends[-steps - 1] + 1: ends[-1] + 1]
t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
busy = defaultdict(float)
top = defaultdict(lambda: defaultdict(float))
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    q = r["Stream_Id"] + "/" + r["Queue_Id"]
    busy[q] += d
    top[q][r["Kernel_Name"][:60]] += d
# union of all kernel intervals (GPU busy) vs wall
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel)
union, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
print("wall per step %.3f ms, GPU busy (union) %.3f ms" % ((t1 - t0) / 1e6 / steps, union / 1e6 / steps))
for q, b in sorted(busy.items(), key=lambda x: -x[1]):
    print("stream/queue %-8s busy %.3f ms/step" % (q, b / 1e3 / steps))
    for k, v in sorted(top[q].items(), key=lambda x: -x[1])[:8]:
        print("     %8.3f  %s" % (v / 1e3 / steps, k))
