"""Per-dispatch table of a rocprofv3 kernel trace: (kernel, grid) -> count, avg us, and the
time share of the run; the gaps between consecutive dispatches on the queue."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: [0, 0.0])
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    k = (r["Kernel_Name"].split("(")[0][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r.get("Workgroup_Size_X", ""))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"dispatches {len(rows)}  busy {tot/1e3:.2f} ms  span {span/1e3:.2f} ms")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t/1e3:8.3f} ms {100*t/tot:5.1f}%  n={n:4d} avg {t/n:9.1f} us  grid {k[1]}x{k[2]}x{k[3]} wg {k[4]}  {k[0]}")
