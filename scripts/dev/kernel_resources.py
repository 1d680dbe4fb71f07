"""Dev: VGPR/AGPR, LDS and scratch of the codec's kernels from a -save-temps gfx950 .s file.
Usage: python scripts/dev/kernel_resources.py <file.s> [substring ...]"""
import re
import sys

s = open(sys.argv[1]).read()
keys = sys.argv[2:]
for m in re.finditer(r'\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel', s, re.S):
    name, body = m.group(1), m.group(2)
    if keys and not any(k in name for k in keys):
        continue
    g = lambda k: (re.search(r'\.amdhsa_' + k + r'\s+(\d+)', body) or [None, None])[1]
    print(f"{name[:80]:80s} regs {g('next_free_vgpr'):>4} accoff {g('accum_offset'):>4} "
          f"lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size')}")
