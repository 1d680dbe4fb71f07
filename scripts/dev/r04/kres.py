"""Kernel resources from hipcc -S output: name, VGPR, AGPR, SGPR, LDS, scratch (the amdhsa metadata)."""
import re, sys, subprocess
s = open(sys.argv[1]).read()
meta = s[s.find("amdhsa.kernels:"):]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in meta.split("  - .agpr_count:")[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = g("name")
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if pat and pat not in dem:
        continue
    agpr = blk.split("\n", 1)[0].strip()
    print(f"vgpr {g('vgpr_count'):>4} agpr {agpr:>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4}  {dem}")
