"""Dev: where a multi-stream step is not streaming.  From a rocprofv3 kernel trace, over the
last `--frac` of the trace: time with no streaming kernel (the HBM passes) active, split by
which other kernels were running then (or none: a launch / host gap), and the longest such
intervals.  Usage: python scripts/dev/trace_uncovered.py run_kernel_trace.csv [frac]"""
import csv
import sys
from collections import defaultdict

STREAMING = ("rowproj_efh3", "colproj_efh3", "colproj_h3", "rowproj_h3", "rank_stream", "rowproj_ef_",
             "colproj_ef_", "rowproj_x6", "colproj_x6", "rowproj_fast", "colproj_fast")


def main(path, frac=0.5):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[5:] if name.startswith("void ") else name))
    rows.sort()
    # the timed steps: the last cluster of kernels with no gap over 2 ms that lasts > 50 ms
    clusters, cs, ce = [], rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s - ce > 2_000_000:
            clusters.append((cs, ce))
            cs = s
        ce = max(ce, e)
    clusters.append((cs, ce))
    long = [c for c in clusters if c[1] - c[0] > 50_000_000] or clusters
    c0, c1 = long[-1]
    cut = c0 + int((c1 - c0) * (1 - frac))
    t1 = c1
    rows = [r for r in rows if r[1] > cut and r[0] < t1]
    events = sorted({cut, t1} | {max(s, cut) for s, _, _ in rows} | {min(e, t1) for _, e, _ in rows})
    uncovered = defaultdict(int)
    intervals = []
    total = 0
    for a, b in zip(events, events[1:]):
        active = [n for s, e, n in rows if s <= a and e >= b]
        total += b - a
        if any(n.startswith(STREAMING) for n in active):
            continue
        key = " + ".join(sorted({n[:40] for n in active})) or "(idle)"
        uncovered[key] += b - a
        if intervals and intervals[-1][1] == a:
            intervals[-1] = (intervals[-1][0], b, intervals[-1][2] | set(active))
        else:
            intervals.append((a, b, set(active)))
    unc = sum(uncovered.values())
    print(f"window {total / 1e6:.2f} ms, no streaming kernel active {unc / 1e6:.2f} ms ({100 * unc / total:.1f} %)")
    for k, v in sorted(uncovered.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v / 1e6:8.3f} ms  {k}")
    print("longest uncovered intervals:")
    for a, b, act in sorted(intervals, key=lambda x: x[0] - x[1])[:10]:
        print(f"  {(b - a) / 1e3:8.1f} us at +{(a - cut) / 1e6:.2f} ms: {', '.join(sorted(n[:30] for n in act)) or '(idle)'}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
