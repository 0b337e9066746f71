"""Per-0.5-ms queue occupancy of the last training step in a rocprofv3 kernel trace (tools
only): python tools/queue_timeline.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
seg = rows[adam[-2] + 1:adam[-1] + 1]
t0 = int(seg[0]["Start_Timestamp"])
W = 500_000
win = collections.defaultdict(lambda: collections.defaultdict(int))
names = collections.defaultdict(collections.Counter)
queues = sorted({r["Queue_Id"] for r in seg})
for r in seg:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r["Queue_Id"]
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    n = (n[:n.find("(")] if "(" in n else n)[:28]
    k = s // W
    while s < e:
        nxt = min(e, (k + 1) * W)
        win[k][q] += nxt - s
        names[k][(q, n)] += nxt - s
        s = nxt
        k += 1
span = (int(seg[-1]["End_Timestamp"]) - t0) / 1e6
print(f"step span {span:.2f} ms, queues {queues}")
for k in sorted(win):
    occ = " ".join(f"q{q} {win[k].get(q, 0) / W * 100:5.1f}%" for q in queues)
    top = "; ".join(f"{q}:{n}" for (q, n), _ in names[k].most_common(3))
    print(f"{k * 0.5:5.1f}ms {occ}  {top}")
