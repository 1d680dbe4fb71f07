"""Per-kernel MFMA / VALU / wait summary from the rocprofv3 --pmc passes of scripts/gpu_pmc_sq.sh.

MFMA utilisation = SIMD-cycles the matrix pipe is busy / (1024 SIMDs x kernel cycles):
  * mfma_util       SQ_VALU_MFMA_BUSY_CYCLES / (1024 * cycles)
  * mfma_util_insts SQ_INSTS_MFMA * 16 / (1024 * cycles)   (v_mfma_f32_16x16x32_bf16 = 16 cycles,
                    MI355X_MICROARCH.md "Per-instruction cycle constants"; every product MFMA here
                    is that instruction)
  kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MICROARCH "DVFS give-back").
Wave-time fractions (all per-wave quad-cycle counts): active_inst_any, active_valu, active_lds,
wait_any (parked at s_waitcnt / barrier), wait_inst_any (issue stall).
Usage: python scripts/pmc_sq_summary.py <dir containing pmcsq_<op>_<group>/>  (prints JSON)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short_name(name):
    m = re.match(r"(?:void\s+)?([A-Za-z_0-9]+(?:<[^()]*>)?)", name.strip())
    return m.group(1) if m else name


def main():
    root = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmcsq_*", "**", "*counter_collection.csv"), recursive=True):
        op = os.path.relpath(f, root).split(os.sep)[0][len("pmcsq_"):].rsplit("_", 1)[0]
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short_name(row["Kernel_Name"])
                if k.startswith("at::") or "elementwise_kernel" in k or "distribution" in k:
                    continue
                acc[(op, k)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"source": "rocprofv3 --pmc, one pass per counter group (scripts/gpu_pmc_sq.sh)", "kernels": {}}
    for (op, k), d in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        cyc = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        rec = {"op": op, "launches_sampled": max(len(v) for v in d.values()), "counters": avg}
        if cyc > 0:
            rec["kernel_cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                rec["mfma_util"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
            if "SQ_INSTS_MFMA" in avg:
                rec["mfma_util_insts"] = avg["SQ_INSTS_MFMA"] * 16 / (1024 * cyc)
        if wc > 0:
            for key, c in (("active_inst_any", "SQ_ACTIVE_INST_ANY"), ("active_valu", "SQ_ACTIVE_INST_VALU"),
                           ("active_lds", "SQ_ACTIVE_INST_LDS"), ("active_vmem", "SQ_ACTIVE_INST_VMEM"),
                           ("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY")):
                if c in avg:
                    rec[key] = avg[c] / wc
        out["kernels"][f"{op}:{k}"] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
