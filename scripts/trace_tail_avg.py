"""Average duration of the last N dispatches of a kernel in a rocprofv3 kernel_trace.csv.

bench.py times the roofline kernel in a serialized pass that runs after the timed region, so the
kernel's last `launches` dispatches in the trace are exactly the ones the bench line's
`roofline.avg_launch_ms` averages (HIP events on the kernel's stream).
usage: python scripts/trace_tail_avg.py run_kernel_trace.csv KERNEL_SUBSTRING N
"""
import csv
import sys

path, pat, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        if pat in name:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), name))
rows.sort()
tail = rows[-n:]
avg = sum(d for _, d, _ in tail) / len(tail)
allavg = sum(d for _, d, _ in rows) / len(rows)
print(f"kernel {pat}: {len(rows)} dispatches in trace, avg {allavg / 1e6:.4f} ms (all, incl. overlapping pools); "
      f"last {len(tail)} (serialized roofline pass) avg {avg / 1e6:.4f} ms")
