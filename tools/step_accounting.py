"""Kernel-time accounting of ONE training step from a rocprofv3 kernel trace (tools only):
the segment after the second-to-last Adam launch up to the last one, kernel time per
category and per queue, and the step's span.   python tools/step_accounting.py run_kernel_trace.csv
(rocprof kernel tracing serialises the gradient side stream behind the main stream, so the
span reads longer than the unprofiled ms/step; the per-category sums are what this is for.)"""
import collections
import csv
import re
import sys

CATS = [
    ("lstm2 fwd (persistent)", r"lstm_persist_kernel<1024|lstm2_rs_kernel"),
    ("lstm2 fwd (per step)", r"lstm2_fwd_step"),
    ("lstm2 bwd (fused step / products)", r"lstm2_bwd_rec|lstm2_bwd_fused"),
    ("lstm2 bwd pointwise", r"lstm2_bwd_pointwise"),
    ("lstm1 fwd", r"lstm_fwd_step|lstm_persist_kernel<512|lstm_xcd_fwd"),
    ("lstm1 bwd", r"lstm_bwd_(rec|pointwise|fused)|lstm_xcd_bwd"),
    ("encoder BLSTM", r"blstm_"),
    ("GEMM fp32", r"gemm_kernel<"),
    ("GEMM fp32 on bf16 planes (X6)", r"gemm_bf16_kernel<.*, true>\("),
    ("GEMM bf16", r"gemm_bf16_kernel<"),
    ("split-K reduce", r"splitk_reduce|splitk_stats"),
    ("Winograd transforms", r"wino_"),
    ("BatchNorm", r"stats_(partial|finalize)|apply_kernel|bwd_partial|bwd_finalize|bwd_apply|bn_dy"),
    ("bias column sums", r"colsum_"),
    ("conv pack/unpack", r"conv_pack|conv_unpack|transpose_kernel|conv_weights_batched"),
    ("losses", r"loss_"),
    ("Adam", r"adam_kernel"),
    ("frame/code glue", r"frame_concat|code_gather|zero_words"),
]


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    # --adam N: the step ending at the N-th Adam launch (0-based; default the last one) — a bench
    # trace holds the fp32 steps first, then the bf16 ones
    n = int(sys.argv[sys.argv.index("--adam") + 1]) if "--adam" in sys.argv else len(adam) - 1
    seg = rows[adam[n - 1] + 1:adam[n] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    cat = collections.Counter()
    calls = collections.Counter()
    queue = collections.Counter()
    for r in seg:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c = next((name for name, pat in CATS if re.search(pat, n)), "other (torch / copies)")
        cat[c] += d
        calls[c] += 1
        queue[r["Queue_Id"]] += d
    tot = sum(cat.values())
    print(f"one step: span {(t1 - t0) / 1e6:.2f} ms, kernel time {tot / 1e6:.2f} ms, {len(seg)} launches")
    for q, d in sorted(queue.items()):
        print(f"  queue {q}: {d / 1e6:.2f} ms busy")
    for c, d in cat.most_common():
        print(f"  {c:24s} {d / 1e6:7.3f} ms  {100 * d / tot:5.1f} %  {calls[c]:5d} launches")
    if "--kernels" in sys.argv:
        per, n = collections.Counter(), collections.Counter()
        for r in seg:
            k = "q" + r["Queue_Id"] + " " + r["Kernel_Name"].replace("(anonymous namespace)::", "")[:57]
            per[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            n[k] += 1
        print("per kernel:")
        for k, d in per.most_common(40):
            print(f"  {k:60s} {d / 1e6:7.3f} ms {n[k]:5d} x {d / n[k] / 1e3:7.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
