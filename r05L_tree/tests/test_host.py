"""CPU tests of the host side: C-ABI library loading/exports, state rules, batching, runtime."""
import ctypes
import os
import re

import pytest
import torch

import megatron_dion_amd as mda
from megatron_dion_amd import _lib
from megatron_dion_amd.batches import build_dion_batches
from megatron_dion_amd.runtime import AsyncRuntime
from megatron_dion_amd.types import DionDistMeta, DionStepParam
from oracle import dion_oracle as O
from tests._golden import Case, case_names

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "dion_codec.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(dion_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) == 24
    assert sorted(_lib.EXPORTED) == syms
    for s in syms:
        assert getattr(lib, s) is not None
    assert lib.dion_abi_version() == _lib.ABI_VERSION


def test_deferred_ef_query_names_the_fused_shapes():
    lib = _lib.load()
    nbytes = ctypes.c_size_t(0)
    # (shape, fp32 momentum supported, bf16 momentum supported)
    for (m, n, r, tr), ok, ok16 in (((4096, 4096, 64, 0), True, True), ((28672, 4096, 64, 0), True, True),
                                    ((4096, 14336, 64, 1), True, True), ((6144, 4096, 32, 0), True, True),
                                    ((64, 48, 8, 0), False, False), ((4096, 4096, 128, 0), True, False),
                                    ((4096, 4096, 128, 1), True, False), ((4096, 14300, 64, 1), False, False)):
        d = _lib.DionBatchDesc(batch=16, m=m, n=n, r=r, transposed=tr, g_dtype=_lib.DTYPE_BF16,
                               m_dtype=_lib.DTYPE_F32, w_dtype=_lib.DTYPE_F32)
        rc = lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P_EF, ctypes.byref(nbytes))
        assert (rc == _lib.DION_OK) == ok, (m, n, r, tr, rc)
        if not ok:
            assert rc == _lib.DION_E_UNSUPPORTED
        # bf16 momentum (case viii): the fused pass A of the bf16 streaming kernels (r = 32 / 64,
        # whole blocks); elsewhere the eager schedule runs
        d.m_dtype = _lib.DTYPE_BF16
        rc16 = lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P_EF, ctypes.byref(nbytes))
        assert rc16 == (_lib.DION_OK if ok16 else _lib.DION_E_UNSUPPORTED), (m, n, r, tr, rc16)
        for op in (_lib.OP_PROJECT_P, _lib.OP_PROJECT_R, _lib.OP_ORTHONORMALIZE, _lib.OP_FIXUP_COLNORM):
            assert lib.dion_workspace_bytes(ctypes.byref(d), op, ctypes.byref(nbytes)) == _lib.DION_OK


def test_abi_rejects_bad_descriptors_without_gpu():
    lib = _lib.load()
    d = _lib.DionBatchDesc(batch=1, m=64, n=48, r=8, transposed=0, g_dtype=_lib.DTYPE_BF16,
                           m_dtype=_lib.DTYPE_F32, w_dtype=_lib.DTYPE_F32)
    nbytes = ctypes.c_size_t(123)
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P, ctypes.byref(nbytes)) == _lib.DION_OK
    d.r = 0
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P, ctypes.byref(nbytes)) == \
        _lib.DION_E_UNSUPPORTED
    assert b"rank" in lib.dion_last_error()
    d.r = 8
    d.m_dtype = _lib.DTYPE_BF16     # the bf16 state mode (case viii) is supported ...
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P, ctypes.byref(nbytes)) == _lib.DION_OK
    d.m_dtype = 7                   # ... other state dtypes are not
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P, ctypes.byref(nbytes)) == \
        _lib.DION_E_UNSUPPORTED
    d.m_dtype = _lib.DTYPE_F32
    d.r = 100   # r > min(m, n): a TP row shard may have fewer rows than r, a whole matrix may not
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P, ctypes.byref(nbytes)) == _lib.DION_OK
    assert lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_ORTHONORMALIZE, ctypes.byref(nbytes)) == \
        _lib.DION_E_INVALID
    assert b"whole matrix" in lib.dion_last_error()
    d.r = 8
    assert lib.dion_workspace_bytes(ctypes.byref(d), 99, ctypes.byref(nbytes)) == _lib.DION_E_INVALID
    # null pointers are rejected before any device work
    assert lib.dion_project_p(ctypes.byref(d), None, None, None, None, None, None, 0, None) == _lib.DION_E_INVALID


def test_workspace_sizes_cover_llama_batches():
    lib = _lib.load()
    for (m, n) in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)):
        for batch in (1, 8, 32, 100):
            d = _lib.DionBatchDesc(batch=batch, m=m, n=n, r=64, transposed=int(m < n), g_dtype=_lib.DTYPE_BF16,
                                   m_dtype=_lib.DTYPE_F32, w_dtype=_lib.DTYPE_F32)
            for op in (_lib.OP_PROJECT_P, _lib.OP_ORTHONORMALIZE, _lib.OP_PROJECT_R):
                nbytes = ctypes.c_size_t(0)
                assert lib.dion_workspace_bytes(ctypes.byref(d), op, ctypes.byref(nbytes)) == 0
                assert nbytes.value < 8 << 30


def test_rules_match_oracle_and_reference():
    for m, n in ((64, 48), (48, 96), (28672, 4096), (4096, 14336), (17, 19), (5, 3)):
        for rf in (1 / 64, 0.25, 0.5, 1.0):
            assert mda.rank_for_shape(m, n, rf) == O.rank_for_shape(m, n, rf)
            r = mda.rank_for_shape(m, n, rf)
            assert mda.should_use_low_rank_sync(global_shape=(m, n), r_global=r, rank_fraction=rf) == \
                O.use_low_rank_sync(m, n, r, rf)
        assert mda.is_transposed_shape(m, n) == (m < n)
    assert mda.scaled_lr_for_shape(lr=1.0, m_global=16, n_global=4, scale_mode="spectral",
                                   rank_fraction=0.25) == pytest.approx(0.8)
    with pytest.raises(RuntimeError, match="DION_INVALID_SCALE_MODE"):
        mda.scaled_lr_for_shape(lr=1.0, m_global=4, n_global=4, scale_mode="x", rank_fraction=0.25)


def test_q_init_is_seeded_and_topology_invariant():
    # dion/state.py:233-260 + :86-88: the seed depends only on the parameter key
    s1 = mda.q_seed_from_param_key(base_seed=0, param_uid=("w",), param_name="w", q_global_shape=(48, 8),
                                   is_transposed=False)
    s2 = mda.q_seed_from_param_key(base_seed=0, param_uid=("w",), param_name="other", q_global_shape=(48, 8),
                                   is_transposed=False)
    s3 = mda.q_seed_from_param_key(base_seed=1, param_uid=("w",), param_name="w", q_global_shape=(48, 8),
                                   is_transposed=False)
    assert s1 == s2 and s1 != s3 and 0 <= s1 < 2 ** 63
    p = torch.zeros(64, 48)
    st_a, cfg = mda.init_dion_state(p, rank_fraction=1 / 6, param_uid=("w",))
    st_b, _ = mda.init_dion_state(p, rank_fraction=1 / 6, param_uid=("w",))
    assert torch.equal(st_a["Q"], st_b["Q"]) and st_a["Q"].shape == (48, 8)
    gen = torch.Generator().manual_seed(s1)
    assert torch.equal(st_a["Q"], torch.randn((48, 8), generator=gen))
    assert cfg.is_transposed is False and cfg.use_low_rank_sync is True


@pytest.mark.parametrize("name", [n for n in case_names() if Case(n).world == 1])
def test_batch_schedule_matches_reference_w1(name):
    case = Case(name)
    group = {"lr": 0.01, "mu": 0.95, "weight_decay": 0.01, "rank_fraction": case.rank_fraction}
    steps = []
    for n, m, k in case.mats:
        p = torch.nn.Parameter(torch.zeros(m, k))
        st, cfg = mda.init_dion_state(p, rank_fraction=case.rank_fraction, param_uid=(n,), param_name=n)
        steps.append(DionStepParam(param=p, grad=torch.zeros(m, k), optimizer_state=st, optim_group=group,
                                   config=cfg, dist_meta=DionDistMeta(global_shape=(m, k), param_uid=(n,),
                                                                      param_name=n)))
    steps.sort(key=lambda s: s.dist_meta.param_uid)
    batches = build_dion_batches(dion_params=steps, get_replicate_group=lambda: None)
    got = [([e.dist_meta.param_name for e in b.entries], b.real_batch_size) for b in batches]
    want = [(b["members"], b["real"]) for b in case.batches(0, 0)]
    assert got == want


def test_async_runtime_interleave_matches_reference_emulation():
    trace_a, trace_b = [], []

    def gen(tag, n, trace):
        for i in range(n):
            trace.append((tag, i))
            yield
        trace.append((tag, "done"))

    tasks = [("t0", 3), ("t1", 1), ("t2", 4), ("t3", 2), ("t4", 0)]
    AsyncRuntime((gen(t, n, trace_a) for t, n in tasks), 3).run()
    O.run_async_runtime((gen(t, n, trace_b) for t, n in tasks), 3)
    assert trace_a == trace_b


def test_step_requires_distributed_mode_and_checks_elementwise_items():
    from megatron_dion_amd.types import ElementwiseStepParam
    p = torch.nn.Parameter(torch.zeros(8, 8))
    opt = mda.MegatronDion([p], codec=object(), elementwise_optimizer="sgd")
    with pytest.raises(RuntimeError, match="DION_STEP_REQUIRES_DISTRIBUTED_MODE"):
        opt.step()
    item = ElementwiseStepParam(param=p, grad=torch.zeros(8, 8), optimizer_state=opt.state[p],
                                optim_group=opt.param_groups[0])
    opt.enable_distributed_mode(route_step_params=lambda: ([], [item]))
    with pytest.raises(RuntimeError, match="DION_INVALID_ELEMENTWISE_OPT"):  # algorithm.py:276-280
        opt.step()
    assert opt.param_groups[0]["step"] == 2 and opt._step_count == 2
    opt.state[p]["first_moment"] = torch.zeros(8, 8)
    opt.state[p]["exp_avg"] = torch.zeros(8, 8)
    opt.param_groups[0]["elementwise_optimizer"] = "adamw"
    with pytest.raises(RuntimeError, match="DION_SCALAR_STATE_LAYOUT_CONFLICT"):  # algorithm.py:296-299
        opt.step()


def test_optimizer_defaults_match_reference_keys():
    p = torch.nn.Parameter(torch.zeros(8, 8))
    opt = mda.MegatronDion([p], codec=object())
    # dion/algorithm.py:82-105
    for k in ("lr", "mu", "weight_decay", "rank_fraction", "rank_multiple_of", "epsilon", "rcqr_oversample",
              "betas", "elementwise_eps", "rp_average_in_collective", "use_fs_collectives", "enable_async",
              "use_low_rank_sync", "elementwise_optimizer", "elementwise_lr_scale", "scale_mode",
              "extra_scale_factor", "split_qkv", "split_linear", "algorithm", "step"):
        assert k in opt.defaults
    assert opt.defaults["mu"] == 0.95 and opt.defaults["epsilon"] == 1e-8


def test_product_path_fails_loudly_without_library(tmp_path):
    with pytest.raises(_lib.DionLibraryError, match="DION_HIP_LIBRARY_MISSING"):
        _lib.load(str(tmp_path / "missing.so"))


@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_local_path_end_to_end_with_oracle_codec(deferred):
    """Host runtime (W = 1, coalesced launch groups) reproduces the golden c7 (3 matrices, both
    orientations, 2 steps) when the test-only oracle codec stands in for the kernels.  With the
    deferred error feedback the weights and Q match every step and the momentum matches once
    the pending update is flushed (what state_dict() does)."""
    from megatron_dion_amd.optimizer import attach_dp_routing
    from megatron_dion_amd.runtime import _PENDING_EF
    from tests._cpu_codec import OracleCodec

    case = Case("c7_two_steps_mixed")
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    params = {n: torch.nn.Parameter(case.t(0, 0, f"{n}_W0").clone()) for n in names}
    cur = {"step": 0}
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction,
                           codec=OracleCodec(sketch_lookup=lambda P: case.sketch_for(0, cur["step"], P),
                                             deferred=deferred),
                           defer_error_feedback=deferred)
    attach_dp_routing(opt, [(n, params[n]) for n in names])
    for n in names:
        opt.state[params[n]]["Q"].copy_(case.t(0, 0, f"{n}_Q0"))
    for step in range(case.steps):
        cur["step"] = step
        for n in names:
            params[n].grad = case.t(0, step, f"{n}_G").clone()
        opt.step()
        if deferred:
            assert all(_PENDING_EF in opt.state[params[n]] for n in names)
            if step == case.steps - 1:
                assert opt.flush_error_feedback() == len(names)
        for n in names:
            checks = [(params[n], "W1"), (opt.state[params[n]]["Q"], "Q1")]
            if not deferred or step == case.steps - 1:
                checks.append((opt.state[params[n]]["momentum"], "M1"))
            for got, key in checks:
                ref = case.t(0, step, f"{n}_{key}")
                assert (got.detach() - ref).abs().max().item() <= 1e-6 * ref.abs().max().item()


@pytest.mark.parametrize("name", ["c11_bf16_two_steps_mixed", "c13_m32_q16_two_steps", "c14_m16_q32_two_steps"])
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_state_dtype_goldens_through_the_runtime(name, deferred):
    """DionMixedPrecisionConfig with bf16 states, and with independent momentum / Q dtypes
    (dion/types.py:10-17, state.py:502-547: fp32 M with bf16 Q, bf16 M with fp32 Q): the
    product runtime (the Q state cast to the momentum's dtype for the batch and committed back
    in its own) with the oracle codec reproduces the reference's captures."""
    from megatron_dion_amd.optimizer import attach_dp_routing
    from tests._cpu_codec import OracleCodec

    case = Case(name)
    h = case.hyper
    bf = torch.bfloat16 if case.entry.get("bf16") else torch.float32
    mdt = getattr(torch, case.entry["m_dtype"]) if "m_dtype" in case.entry else bf
    qdt = getattr(torch, case.entry["q_dtype"]) if "q_dtype" in case.entry else bf
    names = [n for n, _, _ in case.mats]
    params = {n: torch.nn.Parameter(case.t(0, 0, f"{n}_W0").clone()) for n in names}
    cur = {"step": 0}
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction,
                           codec=OracleCodec(sketch_lookup=lambda P: case.sketch_for(0, cur["step"], P),
                                             deferred=deferred),
                           defer_error_feedback=deferred,
                           mixed_precision_config=mda.DionMixedPrecisionConfig(momentum_dtype=mdt, q_dtype=qdt))
    attach_dp_routing(opt, [(n, params[n]) for n in names])
    for n in names:
        st = opt.state[params[n]]
        assert st["momentum"].dtype == mdt and st["Q"].dtype == qdt
        st["Q"].copy_(case.t(0, 0, f"{n}_Q0"))
    for step in range(case.steps):
        cur["step"] = step
        for n in names:
            params[n].grad = case.t(0, step, f"{n}_G").clone()
        opt.step()
        opt.flush_error_feedback()
        for n in names:
            st = opt.state[params[n]]
            assert st["Q"].dtype == qdt
            for got, key in ((params[n], "W1"), (st["Q"], "Q1"), (st["momentum"], "M1")):
                ref = case.t(0, step, f"{n}_{key}")
                err = (got.detach().float() - ref).abs().max().item() / ref.abs().max().item()
                assert err <= 1e-6, (name, step, n, key, err)


# ---------------------------------------------------------------------------------------------- boundary guard
def _one_batch(kind="ddp", shard=False, collectives=None):
    from megatron_dion_amd.types import (DionBatch, DionBatchCollectives, DionBatchEntry, DionBatchGroup,
                                         DionParamConfig)
    from tests._cpu_codec import OracleCodec

    p = torch.nn.Parameter(torch.randn(64, 48) * 0.02)
    opt = mda.MegatronDion([p], rank_fraction=0.25, codec=OracleCodec())
    local = (32, 48) if shard else (64, 48)
    st = {"momentum": torch.zeros(*local), "Q": torch.randn(48, 12), "r": 12, "local_shape": local,
          "global_shape": (64, 48)}
    opt.state[p].update(st)
    entry = DionBatchEntry(param=p, grad=torch.zeros(*local), optimizer_state=opt.state[p],
                           optim_group=opt.param_groups[0], config=DionParamConfig(use_low_rank_sync=True),
                           dist_meta=DionDistMeta(global_shape=(64, 48)), momentum=st["momentum"],
                           q_tensor=st["Q"], param_shape=local)
    batch = DionBatch(batch_key=(), entries=(entry,), real_batch_size=1,
                      batch_group=DionBatchGroup(kernel_kind=kind, batch_world_size=1),
                      batch_collectives=collectives or DionBatchCollectives())
    return opt, batch


@pytest.mark.parametrize("case", ["fsdp", "fsdp_tp", "shard", "fs_collective"])
def test_unsupported_kernel_kinds_are_refused_before_any_work(case):
    """FS/TP batches must not run as whole matrices (distrib_dion/batches.py:571-584)."""
    from megatron_dion_amd.runtime import run_dion_batch_async
    from megatron_dion_amd.types import DionBatchCollectives

    kind = case if case.startswith("fsdp") else "ddp"
    coll = DionBatchCollectives(fs_collective=object()) if case == "fs_collective" else None
    opt, batch = _one_batch(kind=kind, shard=case == "shard", collectives=coll)
    M0 = batch.momentums[0].clone()
    with pytest.raises(RuntimeError, match=r"\[DION_UNSUPPORTED_KERNEL_KIND\]"):
        for _ in run_dion_batch_async(opt, batch):
            pass
    assert torch.equal(batch.momentums[0], M0)  # nothing ran


def test_ddp_batch_passes_the_guard():
    from megatron_dion_amd.runtime import run_dion_batch_async

    opt, batch = _one_batch()
    opt._step_count = 1
    with torch.no_grad():
        for _ in run_dion_batch_async(opt, batch):
            pass
    assert torch.isfinite(batch.params[0]).all()


# ---------------------------------------------------------------------------------------------- drop-in defaults
def test_deferred_error_feedback_is_the_drop_in_default():
    """INTEGRATION.md's Megatron kwargs construct exactly the benchmarked optimizer."""
    p = torch.nn.Parameter(torch.zeros(8, 8))
    opt = mda.MegatronDion([p], codec=object())
    assert opt._defer_ef is True
    assert isinstance(opt._buffer_cache, dict)  # cleared by DionDistributedOptimizer.offload_to_cpu


def _ckpt_run(steps_before, steps_after, interrupt, via_load_state_dict=True):
    """Deferred-EF run over two matrices with a Megatron-style save / restore in the middle:
    save = reading optimizer.state without '_' keys (checkpoint_io.py:247-268
    build_persistent_param_state, which iterates `state.items()` and does NOT call
    state_dict() first); restore = optionally optimizer.load_state_dict()
    (distrib_optimizer.py:740), then new tensors for every persistent key, keeping the live
    '_' keys (checkpoint_io.py:271-336)."""
    from megatron_dion_amd.optimizer import attach_dp_routing
    from megatron_dion_amd.runtime import _PENDING_EF
    from tests._cpu_codec import OracleCodec

    torch.manual_seed(0)
    named = [("a", torch.nn.Parameter(torch.randn(64, 48) * 0.02)),
             ("b", torch.nn.Parameter(torch.randn(40, 96) * 0.02))]
    sk = {}

    def sketch(P):
        key = tuple(P.shape)
        if key not in sk:
            sk[key] = torch.randn(1, 128, P.shape[-2], generator=torch.Generator().manual_seed(P.shape[-2])) / 128 ** .5
        return sk[key]

    opt = mda.MegatronDion([p for _, p in named], rank_fraction=0.25,
                           codec=OracleCodec(sketch_lookup=sketch, deferred=True))
    attach_dp_routing(opt, named)

    def step(i):
        g = torch.Generator().manual_seed(10 + i)
        for _, p in named:
            p.grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).float()
        opt.step()

    for i in range(steps_before):
        step(i)
    if interrupt:
        assert all(_PENDING_EF in dict.keys(opt.state[p]) for _, p in named)  # deferred after a step
        # the save reads the state directly: the read applies the pending error feedback
        saved = {n: {k: (v.clone() if torch.is_tensor(v) else v) for k, v in opt.state[p].items()
                     if not k.startswith("_")} for n, p in named}
        assert all(_PENDING_EF not in dict.keys(opt.state[p]) for _, p in named)
        step(steps_before)  # the run goes on, then is rolled back to the checkpoint
        live = {n: {k: v for k, v in dict.items(opt.state[p]) if k.startswith("_")} for n, p in named}
        assert all(_PENDING_EF in live[n] for n in live)  # the live run holds a pending EF
        if via_load_state_dict:
            opt.load_state_dict(opt.state_dict())  # drops pending; the adapter then restores tensors
            live = {n: {k: v for k, v in dict.items(opt.state[p]) if k.startswith("_")} for n, p in named}
        for n, p in named:
            restored = dict(live[n])  # the live '_' keys (a stale pending EF, without load_state_dict)
            for k, v in saved[n].items():
                restored[k] = v.clone() if torch.is_tensor(v) else v
            opt.state[p] = restored
        return opt, named, step, saved
    return opt, named, step, None


@pytest.mark.parametrize("via_load_state_dict", [True, False])
def test_checkpoint_round_trip_with_deferred_error_feedback(via_load_state_dict):
    """Save through a direct read of optimizer.state, restore that replaces the momentum
    while keeping the live '_' keys: the saved momentum carries the pending EF and the
    restored one never receives the live run's stale pending EF."""
    ref_opt, ref_named, ref_step, _ = _ckpt_run(3, 0, False)
    ref_opt.flush_error_feedback()
    # interrupted run: 3 steps, save, 1 more step, restore params + state from the checkpoint
    opt, named, step, saved = _ckpt_run(3, 0, True, via_load_state_dict)
    for (n, p), (_, q) in zip(named, ref_named):
        p.data.copy_(q.data)  # the weights of the checkpointed step (the payload's "param")
        assert torch.equal(opt.state[p]["momentum"], ref_opt.state[q]["momentum"])
    for i in range(3, 5):
        step(i)
        ref_step(i)
    opt.flush_error_feedback()
    ref_opt.flush_error_feedback()
    for (_, p), (_, q) in zip(named, ref_named):
        assert torch.allclose(p, q, rtol=0, atol=1e-7)
        assert torch.allclose(opt.state[p]["momentum"], ref_opt.state[q]["momentum"], rtol=0, atol=1e-9)


def test_state_read_inside_the_step_keeps_the_deferral(monkeypatch):
    """The batch builder reads state['momentum'] inside step(): no flush there, so the
    deferred error feedback still rides on the next pass A (no late eager application)."""
    import megatron_dion_amd.runtime as rt
    from megatron_dion_amd.runtime import _PENDING_EF

    calls = []
    real = rt._apply_pending
    monkeypatch.setattr(rt, "_apply_pending", lambda *a: (calls.append(1), real(*a)))
    opt, named, step, _ = _ckpt_run(2, 0, False)
    step(2)
    assert calls == []
    assert all(_PENDING_EF in dict.keys(opt.state[p]) for _, p in named)
    _ = opt.state[named[1][1]]["momentum"]  # a read from outside the step applies it
    assert calls == [1] and _PENDING_EF not in dict.keys(opt.state[named[1][1]])
    assert type(opt.state[named[0][1]]).__name__ == "DionParamState"
    opt.state[named[0][1]] = dict(dict.items(opt.state[named[0][1]]))  # a restore's plain dict
    assert type(opt.state[named[0][1]]).__name__ == "DionParamState"


def test_standalone_routing_sends_non_dion_params_to_the_elementwise_branch():
    """bootstrap.py:565-576 via attach_dp_routing: 1D / embedding / output params -> ElementwiseStepParam."""
    from megatron_dion_amd.optimizer import attach_dp_routing, is_dion_param

    named = [("layers.0.linear_fc1.weight", torch.nn.Parameter(torch.zeros(64, 32))),
             ("layers.0.norm.weight", torch.nn.Parameter(torch.ones(32))),
             ("embedding.word_embeddings.weight", torch.nn.Parameter(torch.zeros(100, 32))),
             ("output_layer.weight", torch.nn.Parameter(torch.zeros(100, 32)))]
    for _, p in named:
        p.grad = torch.zeros_like(p)
    opt = mda.MegatronDion([p for _, p in named], rank_fraction=0.25, codec=object())
    attach_dp_routing(opt, named)
    batches, ew = opt._route_step_params()
    assert [b.dist_metas[0].param_name for b in batches] == ["layers.0.linear_fc1.weight"]
    assert sorted(id(e.param) for e in ew) == sorted(id(p) for _, p in named[1:])
    assert "Q" not in opt.state[named[1][1]]
    assert is_dion_param(named[0][1], named[0][0]) and not is_dion_param(named[2][1], named[2][0])
