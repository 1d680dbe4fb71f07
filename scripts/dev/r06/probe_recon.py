"""Dev: reconcile bench.py's probe (HIP events around each codec call) with a rocprofv3 kernel
trace of the same single-stream bench run.  For every streaming kernel ("main" kernels) the
call is the main kernel plus the small launches that follow it before the next main or chain
kernel (split-K reduction, fix-up partials, column norm); printed per kernel: the main kernel's
average, the whole call's kernel time (start of the main kernel to the end of its last trailing
launch), and the probe's average call from the bench JSON line.
Usage: python scripts/dev/r06/probe_recon.py <run_kernel_trace.csv> <bench json line file>"""
import csv
import json
import re
import sys
from collections import defaultdict

MAIN = ("rowproj_efh3_kernel", "colproj_efh3_kernel", "rowproj_efgl_kernel", "colproj_efgl_kernel",
        "colproj_h3_kernel", "rowproj_h3_kernel", "rowproj_h3gl_kernel", "colproj_h3gl_kernel",
        "rank_stream_kernel", "rowproj_fast_kernel", "colproj_fast_kernel")
TRAIL = ("reduce_slabs_kernel", "reduce_fix_partial_kernel", "fixup_partial_kernel", "colnorm_apply_kernel",
         "absmax_kernel", "presplit16_kernel")


def short(name):
    m = re.match(r"(?:void\s+)?([A-Za-z_0-9]+(?:<[^()]*>)?)", name.strip())
    return m.group(1) if m else name


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
main_t, call_t = defaultdict(list), defaultdict(list)
cur = None
for r in rows:
    n = short(r["Kernel_Name"])
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    base = n.split("<")[0]
    if base in MAIN:
        if cur:
            call_t[cur[0]].append(cur[2] - cur[1])
        cur = [n, s, e]
        main_t[n].append(e - s)
    elif cur and base in TRAIL:
        cur[2] = e
    elif cur:
        call_t[cur[0]].append(cur[2] - cur[1])
        cur = None
if cur:
    call_t[cur[0]].append(cur[2] - cur[1])
probe = {}
try:
    line = next(l for l in open(sys.argv[2]) if l.startswith('{"metric'))
    for k, v in json.loads(line)["roofline"]["kernels"].items():
        probe[k] = v["avg_launch_ms"]
except (OSError, StopIteration, IndexError):
    pass
print(f"{'kernel':45s} {'kernel us':>10s} {'call us':>9s} {'probe us':>9s} {'probe/kernel':>12s} {'probe/call':>10s}")
for n in sorted(main_t, key=lambda k: -sum(main_t[k])):
    km = sum(main_t[n]) / len(main_t[n]) / 1e3
    cm = sum(call_t[n]) / len(call_t[n]) / 1e3
    p = probe.get(n)
    ps = f"{p * 1e3:9.1f} {p * 1e3 / km:12.3f} {p * 1e3 / cm:10.3f}" if p else ""
    print(f"{n[:45]:45s} {km:10.1f} {cm:9.1f} {ps}")
