"""Record HBM bytes per launch of one kernel from a scripts/pmc.sh run into profiles/pmc_traffic.json.

usage: python scripts/pmc_traffic.py gpurun_out/pmc_TAG WORKLOAD_KEY KERNEL_SUBSTRING
FETCH_SIZE (KB) is doubled (gfx950 reports half the bytes of wide coalesced reads,
MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) is taken as is. Both are averaged over the
kernel's dispatches, like the bench's achieved bytes per launch.
The record names the full kernel instantiation the counters came from (one distinct kernel name must match
KERNEL_SUBSTRING) and the build it ran: lib_sha16, the first 16 hex digits of the SHA-256 of the library the passes
loaded (NH_LIB_PATH, else optix-renderer_amd/lib/libnori_hip.so). bench.py uses a record only for that same build.
"""
import hashlib
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, key, pat = sys.argv[1:4]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = os.environ.get("NH_LIB_PATH") or os.path.join(REPO, "optix-renderer_amd", "lib", "libnori_hip.so")
lib_sha16 = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
vals = defaultdict(list)
names = set()
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            names.add(r["Kernel_Name"])
        if pat in r["Kernel_Name"] and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU",
                                                             "GRBM_GUI_ACTIVE", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
                                                             "SQ_ACTIVE_INST_VALU", "VALUBusy", "VALUUtilization",
                                                             "TCC_HIT_sum", "TCC_MISS_sum"):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
if len(names) != 1:
    sys.exit(f"pmc_traffic: {len(names)} distinct kernels match {pat!r}: {sorted(names)}")
kernel = names.pop()
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 2 * 1024  # x2: gfx950 FETCH_SIZE (HBM section)
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
data = json.load(open(out)) if os.path.exists(out) else {}
data[key] = {"kernel": kernel, "lib_sha16": lib_sha16, "hbm_bytes_per_launch": int(fetch + write), "read_bytes_per_launch": int(fetch),
             "write_bytes_per_launch": int(write), "dispatches": len(vals["FETCH_SIZE"]),
             "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {os.path.basename(root)}"}
avg = lambda k: sum(vals[k]) / len(vals[k]) if vals[k] else None  # noqa: E731
if avg("SQ_INSTS_VALU") and avg("GRBM_GUI_ACTIVE"):
    # VALU issue: one wave64 VALU instruction per cycle per CU -- each takes its SIMD one quad-cycle
    # (SQ_ACTIVE_INST_VALU, in quad-cycles, ~ SQ_INSTS_VALU: recorded below), 4 SIMDs per CU;
    # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
    cycles = avg("GRBM_GUI_ACTIVE") / 8
    data[key]["valu_insts_per_launch"] = int(avg("SQ_INSTS_VALU"))
    data[key]["valu_issue_frac"] = round(avg("SQ_INSTS_VALU") / (cycles * 256), 3)
if avg("SQ_ACTIVE_INST_VALU") and avg("SQ_INSTS_VALU"):
    data[key]["quad_cycles_per_valu_inst"] = round(avg("SQ_ACTIVE_INST_VALU") / avg("SQ_INSTS_VALU"), 3)
if avg("VALUBusy") is not None:
    data[key]["valu_busy_pct"] = round(avg("VALUBusy"), 1)
if avg("VALUUtilization") is not None:
    data[key]["valu_utilization_pct"] = round(avg("VALUUtilization"), 1)
if avg("TCC_HIT_sum") is not None and avg("TCC_MISS_sum") is not None:
    data[key]["l2_hit_rate"] = round(avg("TCC_HIT_sum") / max(avg("TCC_HIT_sum") + avg("TCC_MISS_sum"), 1.0), 3)
if avg("SQ_WAIT_ANY") and avg("SQ_WAVE_CYCLES"):
    data[key]["wait_frac"] = round(avg("SQ_WAIT_ANY") / avg("SQ_WAVE_CYCLES"), 3)
json.dump(data, open(out, "w"), indent=1, sort_keys=True)
print(key, data[key])
