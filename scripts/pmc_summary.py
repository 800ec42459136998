"""Per-kernel PMC summary from scripts/pmc.sh output: counter sums per dispatch, averaged over the
kernel's dispatches, with the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md, HBM section)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))   # (kernel) -> counter -> sum over dispatches
disp = defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
print(f"{'kernel':60s} {'counter':22s} {'per_dispatch':>16s} {'dispatches':>10s}")
for k in sorted(per):
    for c, v in sorted(per[k].items()):
        n = len(disp[(k, c)])
        val = v / max(n, 1)
        note = ""
        if c == "FETCH_SIZE":  # KB; x2 on gfx950
            note = f"  -> HBM read bytes/dispatch (x2, KB->B): {val * 2 * 1024:.4g}"
        if c == "WRITE_SIZE":
            note = f"  -> HBM write bytes/dispatch (KB->B): {val * 1024:.4g}"
        print(f"{k[:60]:60s} {c:22s} {val:16.6g} {n:10d}{note}")
