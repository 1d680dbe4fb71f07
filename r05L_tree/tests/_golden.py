"""Helpers to read the golden fixtures captured from the reference (make_golden.py)."""
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def manifest(name="manifest.json"):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def case_names():
    return [c["name"] for c in manifest()["cases"]]


class Case:
    MANIFEST = "manifest.json"

    def __init__(self, name):
        man = manifest(self.MANIFEST)
        self.hyper = man["hyper"]
        self.entry = next(c for c in man["cases"] if c["name"] == name)
        self.name = name
        self.world = int(self.entry["world"])
        self.steps = int(self.entry["steps"])
        self.r = int(self.entry.get("r", 0))  # FS captures carry r per matrix (shards)
        self.mats = [(n, int(m), int(k)) for n, m, k, *_ in self.entry["mats"]]
        with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
            self.arr = {k: z[k] for k in z.files}

    @property
    def rank_fraction(self):
        _, m, n = self.mats[0]
        return self.r / min(m, n)

    def t(self, rank, step, key):
        return torch.from_numpy(self.arr[f"r{rank}_s{step}_{key}"].copy())

    def has(self, rank, step, key):
        return f"r{rank}_s{step}_{key}" in self.arr

    def batches(self, rank, step):
        return self.entry["rank_meta"][rank]["steps"][step]["batches"]

    def ortho_calls(self, rank, step):
        meta = self.entry["rank_meta"][rank]["steps"][step]["ortho"]
        out = []
        for i, om in enumerate(meta):
            out.append(dict(
                p_in=self.t(rank, step, f"ortho{i}_pin"),
                p_out=self.t(rank, step, f"ortho{i}_pout"),
                S=self.t(rank, step, f"ortho{i}_S") if om["has_sketch"] else None,
            ))
        return out

    def sketch_for(self, rank, step, p_in):
        """Return the sketch the reference drew for the ortho call whose input matches p_in."""
        best, best_err = None, float("inf")
        for call in self.ortho_calls(rank, step):
            if call["p_in"].shape != p_in.shape:
                continue
            err = (call["p_in"] - p_in).abs().max().item()
            if err < best_err:
                best, best_err = call, err
        assert best is not None, "no ortho call with matching shape"
        scale = max(p_in.abs().max().item(), 1e-30)
        assert best_err <= 1e-4 * scale, f"closest ortho input differs by {best_err}"
        return best["S"]


def fs_case_names():
    return [c["name"] for c in manifest("manifest_fs.json")["cases"]]


class FsCase(Case):
    """An FS ("fsdp") capture (make_golden_fs.py): per-rank local shards of each matrix."""
    MANIFEST = "manifest_fs.json"

    @property
    def rank_fraction(self):
        return float(self.entry["rf"])

    def shard(self, rank, name):
        return self.entry["rank_meta"][rank]["shards"][name]

    def fs_dim(self, name):
        return next(int(d) for n, _, _, d in self.entry["mats"] if n == name)


def tp_case_names():
    return [c["name"] for c in manifest("manifest_tp.json")["cases"]]


class TpCase(FsCase):
    """A TP ("fsdp_tp") capture (make_golden_tp.py): per-rank row shards of the P side and
    column shards of Q; shard() also carries the rank's Q columns (c0, c1)."""
    MANIFEST = "manifest_tp.json"

    def tp_dim(self, name):
        return self.fs_dim(name)

    def global_rows(self, name):
        """m_P of the global matrix: rows (tp_shard_dim 0) or columns (1) -- the sharded side."""
        _, m, n, dim = next(e for e in self.entry["mats"] if e[0] == name)
        return int(m) if int(dim) == 0 else int(n)
