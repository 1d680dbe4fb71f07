"""Aggregate algorithmic HBM rate over the last bench step of a two-stream trace, split by how
many streaming kernels run at once (each kernel's bytes spread evenly over its duration)."""
import csv, sys
from collections import defaultdict
BPE = {"rowproj_efh3": 10, "colproj_efh3": 10, "colproj_h3": 4, "rowproj_h3": 4, "rank_stream": 8}
SHAPE_ELEMS = None  # from grid: not recoverable; use the Llama group sizes by kernel + duration order
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
upd = [i for i, r in enumerate(rows) if "rank_stream" in r["Kernel_Name"]]
prev_end = max(int(rows[i]["End_Timestamp"]) for i in upd[: len(upd) - 8])
step = [r for r in rows if int(r["Start_Timestamp"]) >= prev_end]
# bytes of each streaming dispatch: elements from grid (Llama shapes) -> match by grid dims
def elems(r):
    k = r["Kernel_Name"]; gx, gy = int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])
    table = {  # (kernel, grid x, grid y) -> rows x cols of the 16 matrices
        ("rowproj_efh3", 57344): 28672 * 4096, ("rowproj_efh3", 12288): 6144 * 4096, ("rowproj_efh3", 8192): 4096 * 4096,
        ("colproj_efh3", 28672): 4096 * 14336, ("rowproj_h3", 8192): 4096 * 14336,
    }
    for (name, x), v in table.items():
        if name in k and gx == x:
            return 16 * v
    if "colproj_h3" in k or "rank_stream" in k:
        return None
    return None
ev = []
for r in step:
    k = next((n for n in BPE if n in r["Kernel_Name"]), None)
    if k is None:
        continue
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r))
t0 = min(e[0] for e in ev); t1 = max(e[1] for e in ev)
print(f"streaming dispatches {len(ev)}, span {(t1-t0)/1e3:.1f} us")
# concurrency histogram with kernel pairs
pts = sorted({e[0] for e in ev} | {e[1] for e in ev})
acc = defaultdict(float)
for a, b in zip(pts, pts[1:]):
    act = [e[2] for e in ev if e[0] <= a and e[1] >= b]
    acc[tuple(sorted(act))] += (b - a) / 1e3
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f} us  {k}")
