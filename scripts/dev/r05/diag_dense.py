"""Dev: re-run tests/test_gpu_configs.py's W = 2 dense-branch case and print, per (rank, step,
matrix), Q's error against the oracle codec with and without per-column sign alignment."""
import os
import sys
import tempfile

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from tests import test_gpu_configs as T
    with tempfile.TemporaryDirectory() as tmp:
        check = {n for n, _, _ in T.DENSE}
        mp.start_processes(T._worker, args=(2, T._port(), tmp, T.DENSE, 32, 3, False, check, None), nprocs=2,
                           join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{q}.pt"), weights_only=True) for q in range(2)]
    for rank in range(2):
        R = res[rank]
        for key in sorted(k for k in R if k.startswith("hip_s") and k.endswith("_Q") and "sinit" not in k):
            h, o = R[key].double(), R["oracle" + key[3:]].double()
            err = (h - o).abs().max().item() / o.abs().max().item()
            sgn = torch.where((h * o).sum(0) < 0, -1.0, 1.0).double()
            err_al = (h * sgn - o).abs().max().item() / o.abs().max().item()
            colerr = ((h - o).abs().amax(0) / o.abs().amax(0)).tolist()
            bad = [i for i, e in enumerate(colerr) if e > 1e-4]
            print(f"rank{rank} {key:24s} err {err:.3e} aligned {err_al:.3e} flipped {int((sgn < 0).sum())} "
                  f"bad cols {bad[:8]} norms {[round(float(o[:, i].norm()), 4) for i in bad[:4]]}", flush=True)
