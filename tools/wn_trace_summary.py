"""Per-hop summary of a tools/wn_pipe_trace.py timeline (per role: first poll after the previous
role's last publish, poll spread, sync, compute + butterfly, epilogue).  Not part of the product."""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
blocks, cur = [], None
for ln in lines:
    if ln.startswith("==="):
        if cur is not None:
            blocks.append(cur)
        cur = []
    elif cur is not None and ln.strip():
        cur.append(ln)
blocks.append(cur)
order = [f"L{i:02d}" for i in range(24)] + ["tail", "head"]
for bi, b in enumerate(blocks):
    roles = {}
    for ln in b:
        name = ln.split()[0]
        vals = {k: float(v) for k, v in re.findall(r"(\w+)\s+(-?[\d.]+)", ln[len(name):])}
        roles.setdefault(name.split(".")[0], []).append(vals)
    prev, tot = None, {"hop": 0.0, "spread": 0.0, "sync": 0.0, "compute": 0.0, "epi": 0.0}
    print(f"step block {bi}")
    for r in order:
        vs = roles.get(r)
        if not vs:
            continue
        g = lambda k, f=max: f(v.get(k, 0.0) for v in vs)
        pol, pmin, syn, red, pub = g("polled"), g("polled", min), g("synced"), g("reduced"), g("published")
        hop = pmin - prev if prev is not None else float("nan")
        line = f"  {r:5s} hop {hop:5.2f} spread {pol - pmin:5.2f}"
        if syn > 0:
            line += f" sync {syn - pol:5.2f}"
        if red > 0 and syn > 0:
            line += f" compute {red - syn:5.2f} epi {pub - red:5.2f}"
        line += f"  last pub {pub:7.2f}"
        print(line)
        prev = pub
