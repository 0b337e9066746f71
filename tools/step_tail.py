"""When the step's last main-stream kernel ends vs the side (gradient) stream's last kernel
before the final Adam launch, from a rocprofv3 kernel trace (tools only):
    python tools/step_tail.py run_kernel_trace.csv
Prints, for the last step, each queue's last kernel end relative to the step start, and the
main-stream gaps (sum of idle time between consecutive main-stream kernels)."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need two Adam launches")
    seg = rows[adam[-2] + 1:adam[-1]]
    t0 = int(rows[adam[-2]]["End_Timestamp"])
    tA = int(rows[adam[-1]]["Start_Timestamp"])
    queues = {}
    for r in seg:
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        queues.setdefault(q, []).append(r)
    print(f"step: {(tA - t0) / 1e3:.1f} us from the previous Adam's end to this Adam's start")
    for q, rs in sorted(queues.items(), key=lambda kv: -len(kv[1])):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        last = max(int(r["End_Timestamp"]) for r in rs)
        gaps = 0
        prev_end = None
        for r in rs:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if prev_end is not None and s > prev_end:
                gaps += s - prev_end
            prev_end = max(prev_end or 0, e)
        tail = rs[-1]["Kernel_Name"][:60]
        print(f"queue {q}: {len(rs)} kernels, busy {busy / 1e3:.1f} us, idle between them {gaps / 1e3:.1f} us, "
              f"last end at {(last - t0) / 1e3:.1f} us ({tail})")


if __name__ == "__main__":
    main(sys.argv[1])
