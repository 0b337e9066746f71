"""Average per-dispatch PMC counters of one kernel from rocprofv3 --pmc passes (tools only).
  python tools/pmc_kernel_summary.py KERNEL_SUBSTRING DIR [DIR ...] [--first N] [--label L]
Prints a JSON object: per counter the mean over the kernel's dispatches (and the dispatch count),
plus the derived HBM bytes with the gfx950 correction of MI355X_MICROARCH.md's HBM section
(FETCH_SIZE reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE exact; both KiB),
the L2 hit rate and the MFMA-busy fraction of the kernel's SQ busy cycles."""
import collections
import csv
import glob
import json
import os
import sys

args = [a for a in sys.argv[1:]]
label = None
if "--label" in args:
    i = args.index("--label")
    label = args[i + 1]
    del args[i:i + 2]
kern, dirs = args[0], args[1:]
vals = collections.defaultdict(list)
names = set()
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if kern not in r.get("Kernel_Name", ""):
                continue
            names.add(r["Kernel_Name"])
            per[int(r.get("Dispatch_Id", 0))][r["Counter_Name"]] = float(r["Counter_Value"])
        for did, cs in per.items():
            for c, v in cs.items():
                vals[c].append(v)
out = {"kernel": sorted(names), "label": label, "counters": {}}
for c, v in sorted(vals.items()):
    out["counters"][c] = {"mean": sum(v) / len(v), "dispatches": len(v)}
m = {c: d["mean"] for c, d in out["counters"].items()}
if "FETCH_SIZE" in m:
    out["fetch_bytes_per_dispatch"] = 2 * m["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in m:
    out["write_bytes_per_dispatch"] = m["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    out["hbm_bytes_per_dispatch"] = out["fetch_bytes_per_dispatch"] + out["write_bytes_per_dispatch"]
if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
    out["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"] > 0:
    out["mfma_busy_over_sq_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_BUSY_CYCLES"]
print(json.dumps(out, indent=1))
