"""Timeline of a rocprofv3 kernel trace: busy time vs wall time over the
last N kernels (graph-replayed decode: launch gaps between kernels)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
wall = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
gaps.sort()
print("kernels %d  busy %.1f us  wall %.1f us  busy/wall %.2f" % (len(rows), busy / 1e3, wall / 1e3, busy / wall))
print("gap us: p10 %.2f p50 %.2f p90 %.2f max %.1f" % tuple(gaps[int(q * (len(gaps) - 1))] / 1e3 for q in (0.1, 0.5, 0.9, 1.0)))
