"""Per-queue timeline summary of a rocprofv3 kernel trace: for the last N seconds of kernels, each queue's
kernels in order with start offset / duration (ms), and the busy fraction of the GPU (any kernel running)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t_from = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5  # fraction of the trace to skip (warmup)
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"].split("(")[0][-40:],
       int(r["Grid_Size_X"])) for r in rows]
ks.sort()
t0, t1 = ks[0][0], max(k[1] for k in ks)
cut = t0 + (t1 - t0) * t_from
ks = [k for k in ks if k[0] >= cut]
base = ks[0][0]
busy, cur_end = 0, base
for s, e, *_ in ks:
    if s > cur_end:
        cur_end = s
    if e > cur_end:
        busy += e - cur_end
        cur_end = e
span = max(k[1] for k in ks) - base
print(f"span {span/1e6:.3f} ms, GPU busy {busy/span:.3f}")
for s, e, q, n, g in ks:
    if (e - s) > 50_000 or "splat" in n or "merge" in n or "pack" in n:
        print(f"q{q:>3} {(s-base)/1e6:9.3f} +{(e-s)/1e6:7.3f}  {n} grid {g}")
