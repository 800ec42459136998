"""Summarise a rocprofv3 rocpd database: per-kernel count/total/avg, and optionally a per-dispatch listing."""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, duration, grid_x, workgroup_x from kernels order by start").fetchall()
agg = defaultdict(lambda: [0, 0, 0, 1e30])
for n, d, gx, wx in rows:
    a = agg[n]
    a[0] += 1
    a[1] += d
    a[2] = max(a[2], d)
    a[3] = min(a[3], d)
tot = sum(a[1] for a in agg.values())
print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{n[:70]:70s} {a[0]:6d} {a[1]/1e6:10.3f} {a[1]/a[0]/1e3:10.2f} {a[3]/1e3:9.2f} {a[2]/1e3:9.2f} {100*a[1]/tot:6.2f}")
if len(sys.argv) > 2:
    pat = sys.argv[2]
    for n, d, gx, wx in rows:
        if pat in n:
            print(f"{n[:40]:40s} items={gx:10d} us={d/1e3:9.2f}")
