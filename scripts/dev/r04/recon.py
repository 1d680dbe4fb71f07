"""Per-kernel average launch time: the bench's probe (HIP events around each codec call) against
the rocprofv3 kernel trace of the same process; and the kernels each probed call launches."""
import csv, json, sys
from collections import defaultdict
bench = json.load(open(sys.argv[1]))
rows = list(csv.DictReader(open(sys.argv[2])))
dur = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print("kernel  probe_ms  rocprof_ms  ratio")
for k, v in bench["roofline"]["kernels"].items():
    t = dur.get(k)
    rp = sum(t) / len(t) if t else float("nan")
    print(f"{k:45s} {v['avg_launch_ms']:8.4f} {rp:8.4f} {v['avg_launch_ms'] / rp:6.3f}  n={len(t or [])}")
# every kernel's average, for the calls' extra launches
print("all kernels (rocprof avg ms, count):")
for k, t in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {sum(t) / len(t):8.4f} n={len(t):4d} total={sum(t):8.2f}  {k[:90]}")
