"""Timeline of the last bench step in a rocprofv3 kernel trace: the time with no streaming kernel
active, with one, with two; and what runs in the no-streaming gaps."""
import csv, sys
from collections import defaultdict
STREAM = ("rowproj_efh3", "colproj_efh3", "colproj_h3", "rowproj_h3", "rank_stream", "b16_", "rowproj_fast", "colproj_fast")
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
upd = [i for i, r in enumerate(rows) if "rank_stream" in r["Kernel_Name"] or "b16_stream" in r["Kernel_Name"]]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 8
# last step: after the end of the (len/per - 1)-th step's last update
nsteps = len(upd) // per
first = upd[(nsteps - 1) * per - 1] + 1
# step start = first dispatch after the previous step's final update (by end time)
prev_end = max(int(rows[i]["End_Timestamp"]) for i in upd[: (nsteps - 1) * per])
step = [r for r in rows if int(r["Start_Timestamp"]) >= prev_end]
t0 = min(int(r["Start_Timestamp"]) for r in step)
t1 = max(int(r["End_Timestamp"]) for r in step)
ev = []
for r in step:
    s = any(k in r["Kernel_Name"] for k in STREAM)
    ev.append((int(r["Start_Timestamp"]), 1, s, r))
    ev.append((int(r["End_Timestamp"]), -1, s, r))
ev.sort(key=lambda e: (e[0], e[1]))
act_s = 0; act_o = 0; last = t0
dur = defaultdict(float)
gaps = []
for t, d, s, r in ev:
    key = (min(act_s, 2), act_o > 0)
    dur[key] += (t - last) / 1e3
    if act_s == 0 and t > last:
        gaps.append((last, t))
    last = t
    if s: act_s += d
    else: act_o += d
print(f"step span {(t1 - t0)/1e3:.1f} us, dispatches {len(step)}")
for k in sorted(dur):
    print(f"  streaming={k[0]} other={'y' if k[1] else 'n'}: {dur[k]:9.1f} us")
big = sorted(gaps, key=lambda g: g[0])
print("gaps with no streaming kernel (>= 20 us):")
for a, b in big:
    if b - a >= 20e3 / 1e3 * 1e3:
        names = sorted({r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "") for r in step
                        if int(r["Start_Timestamp"]) < b and int(r["End_Timestamp"]) > a})
        print(f"  at {(a - t0)/1e3:8.1f} us: {(b - a)/1e3:7.1f} us  {names}")
# per-stream order
qs = defaultdict(list)
for r in step:
    qs[r["Queue_Id"]].append(r)
for q, lst in qs.items():
    print(f"queue {q}: " + " ".join(
        f"{r['Kernel_Name'].split('(')[0].split('<')[0].replace('void ', '')[:14]}@{(int(r['Start_Timestamp'])-t0)/1e3:.0f}+{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:.0f}"
        for r in lst if any(k in r["Kernel_Name"] for k in STREAM)))
# per-family duration sums over the step (non-streaming families are the ortho chain and glue)
fam = defaultdict(lambda: [0, 0.0])
for r in step:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    n = n.split("<")[0] + ("<" + n.split("<")[1][:12] if "<" in n else "")
    fam[n][0] += 1
    fam[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("per-kernel sums over the step:")
for n, (c, d) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    print(f"  {d:9.1f} us  n={c:3d}  {n}")
