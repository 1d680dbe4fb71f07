"""Pin the oracle's TP ("fsdp_tp") restatement against the reference's own TP=2 captures.

tests/golden/make_golden_tp.py ran the reference's MegatronDion.step over its
build_dion_batches with every matrix sharded over a 2-rank TP group on the P-row side and Q
sharded by columns, and recorded each rank's shards before and after every step plus every
distributed orthogonalize call with its sketch slice.  Checked here:
  - the sketch restatement: each rank's captured sketch slice is exactly the rows-slice of the
    seeded draw keyed ("distributed", step, param_uid, param_name) (ortho.py:126-177, 575-640);
  - the oracle's TP step (oracle/dion_oracle.py dion_batch_step_tp) replays the captured
    schedule: W1 / M1 / Q1 of every shard on every rank within 1e-6 max-relative.
"""
import pytest
import torch

from oracle import dion_oracle as O
from tests._golden import TpCase, tp_case_names


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def _hyper(case):
    h = case.hyper
    return O.DionHyper(lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"], epsilon=h["epsilon"],
                       rcqr_oversample=h["rcqr_oversample"], scale_mode=h["scale_mode"],
                       extra_scale_factor=h["extra_scale_factor"], rank_fraction=case.rank_fraction)


def tp_sketch_fn(case, step, members):
    """Rank k's slice of entry i's reference sketch, regenerated from the seed rule
    (the optimizer's step count is step + 1 inside MegatronDion.step)."""
    def fn(k, i, rows):
        n = members[i]
        sh = case.shard(k, n)
        r = int(sh["r"])
        ks = O.sketch_rows(r, case.hyper["rcqr_oversample"])
        seed = O.distributed_sketch_seed(step + 1, (n,), n)
        return O.reference_sharded_sketch(seed, ks, case.global_rows(n), int(sh["start"]), rows)
    return fn


def tp_oracle_steps(case):
    hyper = _hyper(case)
    names = [n for n, _, _ in case.mats]
    gshape = {n: (m, k) for n, m, k in case.mats}
    W = case.world
    sdt = torch.bfloat16 if case.entry.get("bf16") else torch.float32  # the speedrun's bf16 M and Q
    st = {(k, n): O.DionMatrix(W=case.t(k, 0, f"{n}_W0"), M=case.t(k, 0, f"{n}_M0").to(sdt),
                               Q=case.t(k, 0, f"{n}_Q0").to(sdt), G=None, transposed=case.tp_dim(n) == 1,
                               rank_fraction=case.rank_fraction)
          for k in range(W) for n in names}
    for step in range(case.steps):
        for k in range(W):
            for n in names:
                st[(k, n)].G = case.t(k, step, f"{n}_G")
        for b in case.batches(0, step):
            assert b["kind"] == "fsdp_tp"
            real = int(b["real"])
            members = b["members"][:real]
            per_rank = [[st[(k, n)] for n in members] for k in range(W)]
            O.dion_batch_step_tp(per_rank, hyper, *gshape[members[0]],
                                 sketch_fn=tp_sketch_fn(case, step, members))
        for k in range(W):
            for n in names:
                yield step, k, n, st[(k, n)]


@pytest.mark.parametrize("name", tp_case_names())
def test_tp_sketch_restatement_matches_capture(name):
    case = TpCase(name)
    checked = 0
    for k in range(case.world):
        for step in range(case.steps):
            calls = case.ortho_calls(k, step)
            batches = [b for b in case.batches(k, step)]
            for call, b in zip(calls, batches):
                if call["S"] is None:
                    continue
                members = b["members"][:int(b["real"])]
                fn = tp_sketch_fn(case, step, members)
                for i in range(len(members)):
                    want = fn(k, i, call["S"].shape[-1])
                    assert torch.equal(call["S"][i], want), (name, k, step, i)
                    checked += 1
    if name != "t4_tp2_plain_qr":
        assert checked > 0


@pytest.mark.parametrize("name", tp_case_names())
def test_tp_oracle_matches_reference_capture(name):
    case = TpCase(name)
    seen = 0
    for step, k, n, s in tp_oracle_steps(case):
        for key, got in (("W1", s.W), ("M1", s.M), ("Q1", s.Q)):
            err = _maxrel(got, case.t(k, step, f"{n}_{key}"))
            assert err <= 1e-6, (name, step, k, n, key, err)
        seen += 1
    assert seen == case.steps * case.world * len(case.mats)
