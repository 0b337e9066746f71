"""Timeline summary of a rocprofv3 kernel trace (tools only): GPU-busy union, idle gaps and
per-queue busy time over the fp32 phase of `bench.py` (kernels before the first bf16 GEMM)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first_bf16 = next((i for i, r in enumerate(rows) if "bf16" in r["Kernel_Name"]), len(rows))
fp = rows[:first_bf16]
# skip warmup: last 5 steps = from the 5th-last adam_kernel onward
adam = [i for i, r in enumerate(fp) if "adam_kernel" in r["Kernel_Name"]]
start = adam[-6] + 1 if len(adam) >= 6 else 0
fp = fp[start:adam[-1] + 1]
nsteps = min(5, len(adam) - 1)
t0, t1 = int(fp[0]["Start_Timestamp"]), int(fp[-1]["End_Timestamp"])
busy, cur_s, cur_e = 0, None, None
gaps = []
qbusy = defaultdict(int)
for r in fp:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    qbusy[r.get("Queue_Id", r.get("Stream_Id", "?"))] += e - s
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, r["Kernel_Name"][:60]))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print(f"steps {nsteps} span/step {span/nsteps/1e6:.3f} ms busy-union/step {busy/nsteps/1e6:.3f} ms idle/step {(span-busy)/nsteps/1e6:.3f} ms")
for q, b in sorted(qbusy.items()):
    print(f"queue {q}: kernel time/step {b/nsteps/1e6:.3f} ms")
gaps.sort(reverse=True)
hist = defaultdict(lambda: [0, 0])
for g, _ in gaps:
    k = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">20us"
    hist[k][0] += 1
    hist[k][1] += g
for k, (n, t) in hist.items():
    print(f"gaps {k}: {n/nsteps:.0f}/step total {t/nsteps/1e6:.3f} ms/step")
for g, name in gaps[:15]:
    print(f"  gap {g/1e3:8.1f} us before {name}")
tot = defaultdict(lambda: [0, 0, set()])  # per kernel name: time, calls, queues
for r in fp:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]
    q = r.get("Queue_Id", "?")
    tot[k + " q" + q][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[k + " q" + q][1] += 1
for k, (t, n, _) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:45]:
    print(f"{t/nsteps/1e6:7.3f} ms/step {n/nsteps:6.0f}/step {t/n/1e3:8.1f} us {k}")
