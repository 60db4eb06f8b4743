"""Per-kernel SQ / GRBM counter summary from rocprofv3 --pmc passes.

Each pass is a separate rocprofv3 run (counter_collection.csv); values are
summed over the dimensions of one dispatch, then averaged over launches.
Derived (MI355X_MICROARCH.md, rocprofv3 PMC section):
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
               (GRBM_GUI_ACTIVE is reported summed over the 8 XCDs)
  lds_conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per
               LDS-array cycle)
  wait_*     = SQ_WAIT_* / SQ_WAVE_CYCLES (quad-cycle units on both sides)

    python tools/pmc_sq.py out.json <pass1.csv> [<pass2.csv> ...] [--filter gemm]
"""
import collections
import csv
import json
import sys


def load(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> ctr
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (r["Kernel_Name"].replace("void ", ""), p, r.get("Dispatch_Id", r.get("Correlation_Id")))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (name, _, _), ctr in per.items():
        for c, v in ctr.items():
            agg[name][c].append(v)
    out = {}
    for name, ctrs in agg.items():
        d = {c: sum(v) / len(v) for c, v in ctrs.items()}
        d["launches"] = max(len(v) for v in ctrs.values())
        g = d.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            d["mfma_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * g / 8.0)
        if d.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conf"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
        if d.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
                if c in d:
                    d["frac_" + c[3:].lower()] = d[c] / d["SQ_WAVE_CYCLES"]
        out[name] = d
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--filter")]
    filt = None
    for a in sys.argv[1:]:
        if a.startswith("--filter="):
            filt = a.split("=", 1)[1]
    res = load(args[1:])
    if filt:
        res = {k: v for k, v in res.items() if filt in k}
    json.dump(res, open(args[0], "w"), indent=1, sort_keys=True)
    cols = ("launches", "mfma_busy", "lds_conf", "frac_wait_any", "frac_wait_inst_any",
            "frac_wait_inst_lds")
    print("%-64s " % "kernel" + " ".join("%10s" % c[-10:] for c in cols))
    for name, d in sorted(res.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0) * kv[1]["launches"]):
        print("%-64s " % name[:64] + " ".join(
            ("%10.3f" % d[c]) if isinstance(d.get(c), float) else "%10s" % d.get(c, "-") for c in cols))
