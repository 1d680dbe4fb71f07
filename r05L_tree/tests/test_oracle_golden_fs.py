"""Pin the oracle's FS ("fsdp") restatement against the reference's own FS=2 captures.

tests/golden/make_golden_fs.py ran the reference's MegatronDion.step over its
build_dion_batches with every matrix sharded over a 2-rank FS group (the default Megatron
Dion topology, FS = DP, RP = 1) and recorded each rank's shards before and after every
step plus the sketch of every orthogonalize call.  The oracle's FS generator
(oracle/dion_oracle.py `_fs_batch_gen`) replays the captured schedule with those sketches:
W1 / M1 / Q1 of every shard on every rank within 1e-6 max-relative.
"""
import pytest
import torch

from oracle import dion_oracle as O
from tests._golden import FsCase, fs_case_names


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def fs_oracle_steps(case):
    """Yield (step, rank, name, state) after every step of the oracle replay of `case`."""
    h = case.hyper
    hyper = O.DionHyper(lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"], epsilon=h["epsilon"],
                        rcqr_oversample=h["rcqr_oversample"], scale_mode=h["scale_mode"],
                        extra_scale_factor=h["extra_scale_factor"], rank_fraction=case.rank_fraction)
    names = [n for n, _, _ in case.mats]
    gshape = {n: (m, k) for n, m, k in case.mats}
    W = case.world
    sdt = torch.bfloat16 if case.entry.get("bf16") else torch.float32  # the speedrun's bf16 M and Q
    st = {(k, n): O.DionMatrix(W=case.t(k, 0, f"{n}_W0"), M=case.t(k, 0, f"{n}_M0").to(sdt),
                               Q=case.t(k, 0, f"{n}_Q0").to(sdt), G=None, transposed=case.fs_dim(n) == 0,
                               rank_fraction=case.rank_fraction)
          for k in range(W) for n in names}
    for step in range(case.steps):
        for k in range(W):
            for n in names:
                st[(k, n)].G = case.t(k, step, f"{n}_G")
        batches = []
        for b in case.batches(0, step):
            assert b["kind"] == "fsdp" and b["q_norm"] and b["fs_indices"] == list(range(W))
            real = int(b["real"])
            members = b["members"]
            per_rank = []
            for k in range(W):
                row = []
                for i, n in enumerate(members):
                    if i < real:
                        row.append(st[(k, n)])
                    else:  # padding: zero G / M / Q of the batch's local shape (batches.py:903-968)
                        t = st[(k, members[0])]
                        row.append(O.DionMatrix(W=torch.zeros_like(t.W), M=torch.zeros_like(t.M),
                                                Q=torch.zeros_like(t.Q), G=torch.zeros_like(t.M),
                                                transposed=t.transposed, rank_fraction=t.rank_fraction))
                per_rank.append(row)
            batches.append((per_rank, real, gshape[members[0]]))
        O.dion_step_fs(batches, hyper, sketch_fn=lambda k, i, P, _s=step: case.sketch_for(k, _s, P))
        for k in range(W):
            for n in names:
                yield step, k, n, st[(k, n)]


@pytest.mark.parametrize("name", fs_case_names())
def test_fs_oracle_matches_reference_capture(name):
    case = FsCase(name)
    seen = 0
    for step, k, n, s in fs_oracle_steps(case):
        for key, got in (("W1", s.W), ("M1", s.M), ("Q1", s.Q)):
            err = _maxrel(got, case.t(k, step, f"{n}_{key}"))
            assert err <= 1e-6, (name, step, k, n, key, err)
        seen += 1
    assert seen == case.steps * case.world * len(case.mats)


def test_fs_shards_cover_the_global_matrix():
    """The captured shard ranges tile the sharded dim exactly (uneven split: 26 + 25)."""
    case = FsCase("f3_fs2_uneven_mixed")
    for n, m, k, dim in case.entry["mats"]:
        split = m if dim == 0 else k
        ranges = sorted((case.shard(r, n)["start"], case.shard(r, n)["end"]) for r in range(case.world))
        assert ranges[0][0] == 0 and ranges[-1][1] == split
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert case.shard(0, "u")["end"] - case.shard(0, "u")["start"] == 26
