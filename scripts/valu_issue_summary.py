"""Summary of scripts/valu_issue.sh's PMC pass: per (kind, waves/SIMD) the VALU instructions per CU-cycle from the
counters (SQ_INSTS_VALU over GRBM_GUI_ACTIVE cycles x CUs, GRBM_GUI_ACTIVE normalised by the kernel-trace duration at
the peak clock to undo a per-XCD sum), SQ_ACTIVE_INST_VALU per instruction (quad-cycles per VALU instruction as the
SQ counts them) and the event-timed rate of the same sweep (events.jsonl)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
events = [json.loads(x) for x in open(os.path.join(root, "events.jsonl")) if x.startswith("{")]
dev = events[0]
n_cu, clock_mhz = dev["cus"], dev["peak_clock_mhz"]
runs = events[1:]
ctr = defaultdict(dict)
names = {}
for f in glob.glob(os.path.join(root, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        ctr[d][r["Counter_Name"]] = ctr[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
dur = {}
for f in glob.glob(os.path.join(root, "pmc", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
disp = sorted(ctr)
# the sweep: for each kind, for W in 1, 2, 4, 8: one warm-up + 5 timed dispatches
print(f"device {dev['device']}, {n_cu} CUs, peak clock {clock_mhz:.0f} MHz; per (kind, waves/SIMD): mean over the 5 timed "
      "dispatches")
print(f"{'kind':32s} {'W':>2s} {'ev insts/CU-cyc':>16s} {'pmc insts/CU-cyc':>17s} {'ACTIVE_VALU/inst':>17s} "
      f"{'GRBM/trace-cyc':>15s}")
i = 0
for run in runs:
    ds = disp[i + 1:i + 6]
    i += 6
    vals = defaultdict(float)
    for d in ds:
        for k, v in ctr[d].items():
            vals[k] += v / len(ds)
    tcyc = sum(dur.get(d, 0) for d in ds) / len(ds) * 1e-9 * clock_mhz * 1e6
    grbm = vals.get("GRBM_GUI_ACTIVE", 0.0)
    scale = grbm / tcyc if tcyc else 1.0  # > 1 when GRBM_GUI_ACTIVE is summed over several XCDs
    cyc = grbm / max(round(scale), 1) if grbm else tcyc
    insts = vals.get("SQ_INSTS_VALU", 0.0)
    act = vals.get("SQ_ACTIVE_INST_VALU", 0.0)
    print(f"{run['kind'][:32]:32s} {run['waves_per_simd']:2d} {run['insts_per_cu_cycle_at_peak_clock']:16.3f} "
          f"{insts / (cyc * n_cu) if cyc else 0:17.3f} {act / insts if insts else 0:17.3f} {scale:15.2f}")
