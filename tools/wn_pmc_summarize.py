"""Per-launch HBM bytes of the WaveNet step kernels from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; KiB) over tools/wn_pmc.py.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide coalesced
streaming reads -> doubled; WRITE_SIZE is exact.  Averages per kernel name, and the sum
over one sample step (every wn_layer_kernel + tail + head launch)."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            for k in ("wn_layer_kernel", "wn_tail_kernel", "wn_head_kernel", "wn_layer2_kernel", "wn_step_kernel"):
                if k in name:
                    key = k + ("<L0>" if "true" in name.split(k, 1)[1][:40] else "")
                    acc[key].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


f, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
w, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 256
out = {"kernels": {}, "correction": "FETCH_SIZE doubled (gfx950 reports half of wide streaming reads); WRITE_SIZE as is",
       "source": "tools/wn_pmc.py under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)"}
step_bytes = 0.0
for k in sorted(f):
    b = (2 * f[k] + w.get(k, 0.0)) * 1024
    out["kernels"][k] = {"launches": nf[k], "fetch_kib_raw": round(f[k], 1), "write_kib": round(w.get(k, 0.0), 1),
                         "hbm_bytes_per_launch": int(b)}
    step_bytes += b * nf[k] / steps
out["hbm_bytes_per_sample_step"] = int(step_bytes)
print(json.dumps(out, indent=1))
