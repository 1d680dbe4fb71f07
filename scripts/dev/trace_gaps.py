"""Dev: busy/idle accounting of a rocprofv3 kernel trace (run_kernel_trace.csv).
Per kernel name: launches, total and mean duration; over the whole trace window after
the first `--skip` seconds: union of busy intervals vs wall time (the launch gaps)."""
import csv
import sys
from collections import defaultdict


def main(path, skip_frac=0.5):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    cut = t0 + int((t1 - t0) * skip_frac)
    tail = [r for r in rows if r[0] >= cut]
    per = defaultdict(lambda: [0, 0])
    for s, e, n in tail:
        per[n.split("(")[0][:70]][0] += 1
        per[n.split("(")[0][:70]][1] += e - s
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in tail:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = max(e for _, e, _ in tail) - tail[0][0]
    print(f"window {wall/1e6:.2f} ms, busy(union) {busy/1e6:.2f} ms, idle {(wall-busy)/1e6:.2f} ms, kernels {len(tail)}")
    for n, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{d/1e6:9.3f} ms  {c:5d}x  {d/c/1e3:9.1f} us  {n}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
