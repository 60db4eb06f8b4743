"""Per-kernel HBM traffic from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half
the bytes of a wide coalesced stream -> doubled; WRITE_SIZE (KiB) is exact for
16-B stores.  Prints per-kernel average bytes per launch.

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write ...csv> [filter]
"""
import collections
import csv
import sys


def load(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def summary(fetch_csv, write_csv, filt=None):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    out = {}
    for name in sorted(set(f) | set(w)):
        if filt and filt not in name:
            continue
        fv, wv = f.get(name, []), w.get(name, [])
        fb = 2.0 * 1024 * sum(fv) / max(1, len(fv))
        wb = 1024 * sum(wv) / max(1, len(wv))
        out[name] = {"launches": max(len(fv), len(wv)), "fetch_bytes": fb, "write_bytes": wb,
                     "hbm_bytes": fb + wb}
    return out


if __name__ == "__main__":
    s = summary(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    for name, v in sorted(s.items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"])[:20]:
        print("%-70s %5d  fetch %9.2f MB  write %9.2f MB  per launch"
              % (name.replace("void ", "")[:70], v["launches"], v["fetch_bytes"] / 1e6,
                 v["write_bytes"] / 1e6))
