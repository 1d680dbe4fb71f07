"""Batch runtime of the Dion data-parallel step on MI355X.

Device-side counterpart of /root/reference/megatron/core/optimizer/dion/runtime.py:
  AsyncRuntime                 :140-171   (<= max_concurrent batch generators, round robin)
  validate_update_contract     :196-291
  batch_dion_update_async      :1499-1911 (the hot path; ddp low-rank branch :1379-1496)
Each batch is a generator that enqueues HIP kernels (through the codec backend)
on the current stream and yields right after launching an asynchronous RCCL
collective (reduce-scatter of P, all-gather of P, all-reduce of R), so the
next batch's kernels are enqueued while the collective runs -- the same
overlap structure as the reference, with per-batch buffers (the reference's
unscoped "replicated_p_ortho_full" buffer, runtime.py:1419-1424, lets
concurrent same-shape batches read each other's P).
"""
from __future__ import annotations

import collections
import math
import time
import weakref
from typing import Callable, Generator, Iterable, List, Optional

import torch
import torch.distributed as dist

from ._lib import DionUnsupportedError
from .codec import factor_rows
from .dense_grad_cache import consume_if_reduced
from .kernels import scaled_lr_for_shape


class PhaseClock:
    """DION_PROFILE_SPLIT: the reference's per-phase step profile (dion/runtime.py:67-99,
    dion/algorithm.py:170-218), timed with HIP events instead of a device synchronise at every
    mark (which would serialise the streams).  `mark(label)` charges the time since the
    previous mark of this batch to `label`; MegatronDion.step sums the records per label after
    one synchronise.  Labels are the reference's: grad_momentum, q_unshard, p_matmul, p_reduce,
    ortho_r, error_feedback, q_normalize, apply_update.  Fused kernels charge their phase
    where they end: M += G (and a deferred error feedback) to p_matmul (pass A), the fix-up to
    q_normalize, an eager error feedback to apply_update; the fused phases are listed with 0 s."""

    def __init__(self, optimizer, device, desc: str):
        self.records = getattr(optimizer, "_phase_records", None)
        self.cuda = self.records is not None and getattr(device, "type", "cpu") == "cuda"
        self.desc = desc
        self.last = self._now() if self.records is not None else None

    def _now(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def mark(self, label: str) -> None:
        if self.records is None:
            return
        now = self._now()
        self.records.append((label, self.last, now, self.desc))
        self.last = now


def phase_seconds(start, end) -> float:
    """Seconds between two PhaseClock stamps (HIP events after a synchronise, or host times)."""
    if isinstance(start, float):
        return float(end) - start
    return start.elapsed_time(end) / 1e3


def _batch_desc(batch_group, dist_metas, real, shape) -> str:
    """runtime.py:48-64 (_profile_desc)."""
    meta = dist_metas[0] if dist_metas else None
    return (f"kernel={getattr(batch_group, 'kernel_kind', '')} real={int(real)} shape={tuple(shape)} "
            f"name={getattr(meta, 'param_name', '')}")


class AsyncRuntime:
    """Round-robin driver of batch generators with bounded width."""

    def __init__(self, tasks: Iterable[Generator], max_concurrent_tasks: int = 3, streams=None):
        if int(max_concurrent_tasks) <= 0:
            raise ValueError(f"Invalid max_concurrent_tasks={max_concurrent_tasks}")
        self.tasks = tasks
        self.width = int(max_concurrent_tasks)
        # optional HIP streams: the k-th admitted task always runs on streams[k % len], so a
        # batch's latency-bound orthonormalisation overlaps the other batches' streaming passes
        self.streams = list(streams) if streams else None

    @staticmethod
    def _advance(gen, stream=None) -> bool:
        try:
            if stream is None:
                next(gen)
            else:
                with torch.cuda.stream(stream):
                    next(gen)
            return True
        except StopIteration:
            return False

    def run(self) -> None:
        pending = iter(self.tasks)
        more = True
        admitted = 0
        live: List[tuple] = []
        while more or live:
            nxt: List[tuple] = []
            if more and len(live) < self.width:
                gen = next(pending, None)
                if gen is None:
                    more = False
                else:
                    stream = self.streams[admitted % len(self.streams)] if self.streams else None
                    admitted += 1
                    if self._advance(gen, stream):
                        nxt.append((gen, stream))
            for gen, stream in live:
                if self._advance(gen, stream):
                    nxt.append((gen, stream))
            live = nxt


def _group_world(group) -> int:
    if group is None:
        return 1
    return int(dist.get_world_size(group))


def is_replicated(batch) -> bool:
    """True when the batch exchanges factors with other ranks: replicas (replicate group size > 1)
    or FS / TP shards (the "fsdp" and "fsdp_tp" kinds)."""
    bg = getattr(batch, "batch_group", None)
    return (_group_world(getattr(bg, "replicate_group", None)) > 1
            or str(getattr(bg, "kernel_kind", "ddp")) in ("fsdp", "fsdp_tp"))


def validate_update_contract(optimizer, *, optim_groups, optimizer_states, dist_metas, param_shapes,
                             real_batch_size: int) -> None:
    """All real entries of a batch must share shape, lr, rank_fraction, wd, mu and r."""
    rows = []
    for i in range(int(real_batch_size)):
        st = optimizer_states[i] or {}
        grp = optim_groups[i] or {}
        meta = dist_metas[i]
        gshape = st.get("per_expert_global_shape") or st.get("global_shape") \
            or getattr(meta, "global_shape", None) or param_shapes[i]
        wd_mult = float(grp.get("wd_mult", 1.0))
        rows.append((
            tuple(int(d) for d in gshape),
            float(grp.get("lr", optimizer.defaults["lr"])),
            float(grp.get("rank_fraction", optimizer.defaults.get("rank_fraction", 0.25))),
            float(grp.get("weight_decay", optimizer.defaults["weight_decay"] * wd_mult)),
            float(grp.get("mu", optimizer.defaults["mu"])),
            int(st.get("r", -1)),
        ))
    bad = [i for i, row in enumerate(rows) if row != rows[0]]
    if bad:
        raise RuntimeError(
            "[DION_BATCH_UPDATE_CONTRACT_MISMATCH] "
            f"step={optimizer._step_count} expected={rows[0]} mismatched={[rows[i] for i in bad]}")


def _shape_of(meta, state, fallback):
    st = state or {}
    shape = st.get("per_expert_global_shape") or st.get("global_shape") \
        or getattr(meta, "per_expert_global_shape", None) or getattr(meta, "global_shape", None) or fallback
    return tuple(int(d) for d in shape)


def replicate_op(optimizer):
    """runtime.py:361-364: AVG when rp_average_in_collective, else SUM."""
    return dist.ReduceOp.AVG if optimizer.defaults.get("rp_average_in_collective", True) else dist.ReduceOp.SUM


def dense_replica_all_reduce(optimizer, grads, group) -> Generator[None, None, None]:
    """runtime.py:439-491: all-reduce the dense gradients across the replicas, unless this
    step's grad norm already did (dense_grad_cache, runtime.py:387-435)."""
    op = replicate_op(optimizer)
    if consume_if_reduced(optimizer, grads, group=group, op=op):
        return
    works = [dist.all_reduce(g, op=op, group=group, async_op=True) for g in grads]
    yield
    for w in works:
        w.wait()


def check_supported_batch(optimizer, *, batch_group, batch_collectives, configs, dist_metas, optimizer_states,
                          param_shapes, real_batch_size: int) -> None:
    """Refuse the batches this codec cannot compute, before any kernel runs.

    The reference's adapter emits "fsdp" / "fsdp_tp" batches (distrib_dion/batches.py:571-584)
    whose entries are FS row/column shards or TP shards, with FS/TP collectives attached
    (types.py:149-158) and a q_norm / ortho group.  Treating those shards as whole matrices
    would orthonormalise and normalise a local piece while scaling the LR by the global
    shape: wrong updates with no error.  Computed here: the whole-matrix data-parallel kind
    ("ddp", runtime.py:1379-1496), the FS kind ("fsdp", runtime.py:1201-1293, 1729-1795) and the
    TP kind with TP on the P-row side and FS, if any, on the contraction side ("fsdp_tp",
    runtime.py:680-962, 1328-1377); anything else (another kind, TP on the contraction side, P
    sharded on both axes, a batch without the collectives its kind needs) raises
    [DION_UNSUPPORTED_KERNEL_KIND]."""
    def world(g):
        try:
            return int(dist.get_world_size(g))
        except Exception:  # a stand-in group object (the reference's unit-test fakes)
            return len(tuple(getattr(g, "ranks", ()) or ())) or 2

    kind = str(getattr(batch_group, "kernel_kind", "ddp"))
    why = None
    tp_colls = batch_collectives is not None and any(
        len(tuple(getattr(batch_collectives, f, None) or ())) for f in ("tp_q_gathers", "tp_r_collectives",
                                                                         "tp_q_reshards"))
    reals = configs[:int(real_batch_size)]
    if kind not in ("ddp", "fsdp", "fsdp_tp"):
        why = f"kernel_kind={kind!r}"
    elif kind == "fsdp_tp":
        og = getattr(batch_group, "ortho_group", None)
        gathers = tuple(getattr(batch_collectives, "tp_q_gathers", None) or ()) if batch_collectives else ()
        rsums = tuple(getattr(batch_collectives, "tp_r_collectives", None) or ()) if batch_collectives else ()
        every = set(range(len(param_shapes)))
        if og is None or world(og) <= 1:
            why = "an fsdp_tp batch without its TP ortho group"
        elif not all(is_p_tp_sharded(c) for c in reals):
            why = "an fsdp_tp batch whose entries are not TP-sharded on the P-row side"
        elif len(gathers) != 1 or set(int(i) for i in gathers[0].indices) != every:
            why = "an fsdp_tp batch without one Q all-gather over all its entries"
        elif len(rsums) != 1 or set(int(i) for i in rsums[0].indices) != every:
            why = "an fsdp_tp batch without one R all-reduce over all its entries"
        elif any(bool(getattr(c, "use_fs_shard", False)) and not reduces_p_over_fs(c) for c in reals):
            why = "FS shards on the P-row side together with TP (P sharded on both axes)"
        elif any(bool(getattr(c, "use_fs_shard", False)) for c in reals) and (
                not len(tuple(getattr(batch_collectives, "fs_p_collectives", None) or ()))
                or getattr(batch_group, "q_norm_group", None) is None):
            why = "an FS-sharded fsdp_tp batch without its FS P reduction and q_norm group"
    elif getattr(batch_group, "ortho_group", None) is not None and world(batch_group.ortho_group) > 1:
        why = "a distributed ortho_group (TP-sharded P)"
    elif tp_colls or any(bool(getattr(c, "use_tp_shard", False)) for c in configs[:int(real_batch_size)]):
        why = "TP-sharded entries / TP batch collectives"
    elif kind == "fsdp":
        fs = getattr(batch_collectives, "fs_collective", None) if batch_collectives is not None else None
        if fs is None or int(getattr(fs, "world_size", 1)) <= 1:
            why = "an fsdp batch without its FS collective"
        elif not all(bool(getattr(c, "use_fs_shard", False)) for c in configs[:int(real_batch_size)]):
            why = "an fsdp batch with entries that are not FS shards"
        elif len(param_shapes) != int(fs.world_size) or len(tuple(fs.indices)) != len(param_shapes):
            why = f"fsdp batch size {len(param_shapes)} != FS world {fs.world_size} ([DION_FSONLY_BATCH_SIZE_MISMATCH])"
    else:
        if getattr(batch_group, "q_norm_group", None) is not None and world(batch_group.q_norm_group) > 1:
            why = "a q_norm_group on a ddp batch (FS-sharded column norm)"
        elif batch_collectives is not None and (
                getattr(batch_collectives, "fs_collective", None) is not None
                or len(tuple(getattr(batch_collectives, "fs_p_collectives", None) or ()))):
            why = "FS batch collectives on a ddp batch"
        else:
            for i in range(int(real_batch_size)):
                local = tuple(int(d) for d in param_shapes[i])
                glob = _shape_of(dist_metas[i], optimizer_states[i], local)
                if local != glob:
                    why = f"entry {i} is a shard: local shape {local} != global shape {glob}"
                    break
    if why is not None:
        raise RuntimeError(
            f"[DION_UNSUPPORTED_KERNEL_KIND] step={optimizer._step_count}: {why}; this codec computes "
            "whole-matrix data-parallel ('ddp') batches, FS-sharded ('fsdp') batches, and TP-sharded "
            "('fsdp_tp') batches with TP on the P-row side (FS, if any, on the contraction side)")


def is_p_tp_sharded(config) -> bool:
    """dion/state.py:407-416: TP shards the P-row side (tp_shard_dim 0 not transposed, 1 transposed)."""
    if not (bool(getattr(config, "use_tp_shard", False)) and bool(getattr(config, "has_tp_shard", True))):
        return False
    dim, tr = int(getattr(config, "tp_shard_dim", -1)), bool(config.is_transposed)
    return (not tr and dim == 0) or (tr and dim == 1)


def reduces_p_over_fs(config) -> bool:
    """dion/state.py:399-404: FS shards the contraction side, so P = X Q is a partial sum over FS."""
    if not bool(getattr(config, "use_fs_shard", False)):
        return False
    dim, tr = int(getattr(config, "fs_shard_dim", -1)), bool(config.is_transposed)
    return (not tr and dim == 1) or (tr and dim == 0)


def split_range(size: int, world: int, rank: int):
    """dion/ortho.py:247-259: contiguous shard [start, end) of `rank`, remainder on the first ranks."""
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _sketch_seed(optimizer, batch_cache_key: int, entry: int) -> int:
    """Per (step, matrix) sketch seed; the reference's sketch is unseeded (ortho.py:659-661)."""
    base = int(getattr(optimizer, "_sketch_seed", 0))
    return (base * 0x9E3779B97F4A7C15 + optimizer._step_count * 0xBF58476D1CE4E5B9
            + (int(batch_cache_key) + entry) * 0x94D049BB133111EB) & ((1 << 64) - 1)


def batch_dion_update_async(optimizer, params, momentums, Qs, configs, dist_metas, optim_groups, grads=None,
                            optimizer_states=None, param_shapes=None, real_batch_size=None,
                            batch_cache_key: int = 0, batch_group=None, batch_collectives=None,
                            commit_updates: Optional[List[Optional[Callable]]] = None,
                            sketches: Optional[dict] = None, chunks: int = 0,
                            phase_marks: bool = False) -> Generator[None, None, None]:
    """One batch of same-shape matrices: project, exchange, orthonormalise, update.

    `sketches` (tests only) maps an entry index to an explicit (k, m_P) sketch so
    parity runs can reuse the sketch the reference drew.  `chunks` > 1 marks a
    coalesced group of full W-entry batches (coalesce_replicated_batches).
    `phase_marks` (world size 1 only): yield "ortho" after pass A and "stream" after
    the orthonormalisation, so a scheduler can run the latency-bound phase on another
    HIP stream (MegatronDion._run_local_pipelined).
    """
    codec = optimizer.codec
    B = len(params)
    real = B if real_batch_size is None else int(real_batch_size)
    if batch_group is None:
        raise RuntimeError(f"[DION_MISSING_BATCH_GROUPS] step={optimizer._step_count}")
    if real <= 0:
        return
    param_shapes = list(param_shapes) if param_shapes else [tuple(p.shape) for p in params]
    check_supported_batch(optimizer, batch_group=batch_group, batch_collectives=batch_collectives, configs=configs,
                          dist_metas=dist_metas, optimizer_states=optimizer_states, param_shapes=param_shapes,
                          real_batch_size=real)
    validate_update_contract(optimizer, optim_groups=optim_groups, optimizer_states=optimizer_states,
                             dist_metas=dist_metas, param_shapes=param_shapes, real_batch_size=real)
    group = getattr(batch_group, "replicate_group", None)
    W = _group_world(group)
    use_low_rank = bool(optimizer.use_low_rank_sync) and W > 1 and any(
        bool(c.use_low_rank_sync) for c in configs)
    real_grads = [g for g in (grads or [])[:real]] if grads is not None else []
    if str(getattr(batch_group, "kernel_kind", "ddp")) == "fsdp_tp":
        yield from _tp_batch_update(optimizer, params, momentums, Qs, configs, dist_metas, optim_groups, real_grads,
                                    optimizer_states, param_shapes, real, batch_cache_key, batch_group,
                                    batch_collectives, commit_updates, use_low_rank, sketches)
        return
    if str(getattr(batch_group, "kernel_kind", "ddp")) == "fsdp":
        yield from _fs_batch_update(optimizer, params, momentums, Qs, configs, dist_metas, optim_groups, real_grads,
                                    optimizer_states, param_shapes, real, batch_cache_key, batch_group,
                                    batch_collectives, commit_updates, use_low_rank, sketches)
        return

    if W > 1 and not use_low_rank and real_grads:
        yield from dense_replica_all_reduce(optimizer, real_grads, group)

    kch = int(chunks) if (W > 1 and int(chunks) > 1 and B == real == int(chunks) * W) else 0
    if kch:
        # rank-major layout: position r k + c holds entry c W + r, so a single reduce-scatter
        # gives rank r exactly the entries the per-chunk exchange would (runtime.py:1435)
        order = [c * W + r for r in range(W) for c in range(kch)]
        pick = lambda seq: [seq[i] for i in order] if seq is not None else None  # noqa: E731
        params, momentums, Qs, configs, dist_metas = (pick(list(params)), pick(list(momentums)), pick(list(Qs)),
                                                      pick(list(configs)), pick(list(dist_metas)))
        optim_groups, optimizer_states, param_shapes = (pick(list(optim_groups)), pick(list(optimizer_states)),
                                                        pick(list(param_shapes)))
        real_grads = pick(real_grads) if real_grads else real_grads
        commit_updates = pick(list(commit_updates)) if commit_updates is not None else None
        if sketches is not None:
            sketches = {order.index(e): S for e, S in sketches.items()}
    m, n = (int(d) for d in param_shapes[0])
    transposed = bool(configs[0].is_transposed)
    r = int(Qs[0].shape[1])
    mp, nq = factor_rows(m, n, transposed)
    dev = momentums[0].device
    oversample = float(optimizer.defaults["rcqr_oversample"])
    Qs, commit_qs = _qs_in_state_dtype(list(Qs), real, momentums[0].dtype)
    # bf16 momentum and Q (the speedrun's DionMixedPrecisionConfig): P and R stay fp32
    # buffers of bf16 values; the kernels round where the reference's bf16 tensors round,
    # and an averaging collective is followed by the same rounding (round_bf16)
    sdt = momentums[0].dtype
    bf16_state = sdt == torch.bfloat16

    # padded entries (and the W > 1 exchange buffers) must read as zero; a full
    # world-size-1 batch is written completely by the kernels
    alloc = torch.empty if ((W == 1 or kch) and real == B) else torch.zeros
    P = alloc((B, mp, r), dtype=torch.float32, device=dev)
    nonzero = torch.zeros((B,), dtype=torch.int32, device=dev)
    # deferred error feedback: the previous step's M += -(1-mu) P R^T rides on this pass A
    defer = (getattr(optimizer, "_defer_ef", False) and hasattr(codec, "supports_deferred_ef")
             and (commit_updates is None or all(c is None for c in commit_updates[:real]))
             and codec.supports_deferred_ef(m, n, r, transposed, state_dtype=momentums[0].dtype,
                                           grad_dtype=real_grads[0].dtype if real_grads else None))
    clock = PhaseClock(optimizer, dev, _batch_desc(batch_group, dist_metas, real, (m, n)))
    _project_with_pending(codec, real_grads, momentums, Qs, P, nonzero, optimizer_states, real, m, n, transposed,
                          defer)
    clock.mark("p_matmul")

    def ortho(P_slice, entry):
        S = None if sketches is None else sketches.get(entry)
        codec.orthonormalize(P_slice, m, n, transposed, _sketch_seed(optimizer, batch_cache_key, entry),
                             oversample, sketch=None if S is None else S.reshape(1, *S.shape[-2:]).contiguous(),
                             state_dtype=sdt)

    p_fixed = False
    r_fixed = False  # W = 1: pass B also did the fix-up and column norm (project_r_fixup)
    if W > 1 and kch:
        rank = dist.get_rank(group)
        mine = P[rank * kch:(rank + 1) * kch]
        P_own = torch.empty((kch, mp, r), dtype=torch.float32, device=dev)
        if use_low_rank:
            work = dist.reduce_scatter_tensor(P_own, P, op=dist.ReduceOp.AVG, group=group, async_op=True)
            yield
            work.wait()
            if bf16_state:
                codec.round_bf16(P_own)
        else:
            P_own.copy_(mine)
        clock.mark("p_reduce")
        if sketches is None:
            codec.orthonormalize(P_own, m, n, transposed,
                                 _sketch_seed(optimizer, batch_cache_key, rank * kch), oversample, state_dtype=sdt)
        else:
            for c in range(kch):
                S = sketches.get(rank * kch + c)
                codec.orthonormalize(P_own[c:c + 1], m, n, transposed,
                                     _sketch_seed(optimizer, batch_cache_key, rank * kch + c), oversample,
                                     sketch=None if S is None else S.reshape(1, *S.shape[-2:]).contiguous(),
                                     state_dtype=sdt)
        work = dist.all_gather_into_tensor(P, P_own, group=group, async_op=True)
        yield
        work.wait()
        R = torch.empty((B, nq, r), dtype=torch.float32, device=dev)
        codec.project_r(list(momentums[:real]), P, R, transposed, nonzero=nonzero)
        if use_low_rank:
            work = dist.all_reduce(R, op=dist.ReduceOp.AVG, group=group, async_op=True)
            yield
            work.wait()
            if bf16_state:
                codec.round_bf16(R)
    elif W > 1:
        rank = dist.get_rank(group)
        padded = (B + W - 1) // W * W
        if padded != B:
            P = torch.cat([P, P.new_zeros((padded - B, mp, r))], dim=0)
        for start in range(0, padded, W):
            chunk = P[start:start + W]
            P_single = torch.empty((1, mp, r), dtype=torch.float32, device=dev)
            if use_low_rank:
                # runtime.py:1428-1434: reduce-scatter(avg) hands entry start+rank to this rank
                work = dist.reduce_scatter_tensor(P_single, chunk, op=dist.ReduceOp.AVG, group=group,
                                                  async_op=True)
                yield
                work.wait()
                if bf16_state:
                    codec.round_bf16(P_single)
            else:
                P_single.copy_(chunk[rank:rank + 1])
            idx = start + rank
            if idx < real:
                ortho(P_single, idx)
            else:
                P_single.zero_()  # padded entries stay inert (runtime.py:1436-1441)
            work = dist.all_gather_into_tensor(chunk, P_single, group=group, async_op=True)
            yield
            work.wait()
        P = P[:B]
        R = torch.zeros((B, nq, r), dtype=torch.float32, device=dev)
        codec.project_r(list(momentums[:real]), P, R, transposed, nonzero=nonzero)
        if use_low_rank:
            work = dist.all_reduce(R, op=dist.ReduceOp.AVG, group=group, async_op=True)
            yield
            work.wait()
            if bf16_state:
                codec.round_bf16(R)
    else:
        # W = 1, fp32 state: the last solve of the orthonormalisation also fixes P (the fix-up's
        # P half, kernels.py:185-188: an orthonormalised P is NaN only in whole columns, whose R
        # column is zero either way) and writes pass B's split of P, so pass B needs no absmax /
        # presplit of P and the fix-up no pass over P.  The split is allocated here, on the
        # stream of the batch's streaming passes (as P is), before a pipelined schedule moves
        # the orthonormalisation to its latency stream.
        fused = real == B and not bf16_state and getattr(codec, "fuses_p_fixup", False)
        split = codec.psplit_buffer(B, m, n, r, transposed) if fused and hasattr(codec, "psplit_buffer") else None
        fix = nonzero if fused else None
        p_fixed = fused
        if phase_marks:
            yield "ortho"
        if sketches is None:
            codec.orthonormalize(P[:real], m, n, transposed, _sketch_seed(optimizer, batch_cache_key, 0),
                                 oversample, state_dtype=sdt, **_fused_kw(fix, split, 0, real))
        else:
            for i in range(real):
                S = sketches.get(i)
                codec.orthonormalize(P[i:i + 1], m, n, transposed, _sketch_seed(optimizer, batch_cache_key, i),
                                     oversample, sketch=None if S is None else S.reshape(1, *S.shape[-2:]).contiguous(),
                                     state_dtype=sdt, **_fused_kw(fix, split, i, i + 1))
        if phase_marks:
            yield "stream"
        R = torch.empty((B, nq, r), dtype=torch.float32, device=dev)
        if p_fixed and getattr(codec, "fuses_r_fixup", False):
            # pass B with the fix-up and column norm (R's half) riding on its reduction
            r_fixed = True
            codec.project_r_fixup(list(momentums[:real]), P, R, list(Qs[:real]), nonzero,
                                  float(optimizer.defaults["epsilon"]), transposed,
                                  **({} if split is None else {"p_split": split}))
        else:
            codec.project_r(list(momentums[:real]), P, R, transposed, nonzero=nonzero,
                            **({} if split is None else {"p_split": split}))

    clock.mark("ortho_r")
    eps = float(optimizer.defaults["epsilon"])
    if not r_fixed:
        codec.fixup_colnorm(None if (W == 1 and p_fixed) else P, R, list(Qs[:real]), nonzero, eps, m, n, transposed)
    clock.mark("q_normalize")

    grp = optim_groups[0] or {}
    st0 = optimizer_states[0] or {}
    gshape = st0.get("per_expert_global_shape") or st0.get("global_shape") \
        or getattr(dist_metas[0], "global_shape", None) or (m, n)
    lr = float(grp.get("lr", optimizer.defaults["lr"]))
    mu = float(grp.get("mu", optimizer.defaults["mu"]))
    wd = float(grp.get("weight_decay", optimizer.defaults["weight_decay"] * float(grp.get("wd_mult", 1.0))))
    rank_fraction = float(grp.get("rank_fraction", optimizer.defaults.get("rank_fraction", 0.25)))
    scaled = scaled_lr_for_shape(lr=lr, m_global=int(gshape[0]), n_global=int(gshape[1]),
                                 scale_mode=optimizer.defaults.get("scale_mode", "spectral"),
                                 rank_fraction=rank_fraction,
                                 extra_scale_factor=optimizer.defaults.get("extra_scale_factor", 0.2))
    if defer:
        # weights now; this step's error feedback waits for the next pass A (or a flush)
        codec.ef_apply(None, list(params[:real]), P, R, list(Qs[:real]), nonzero, mu, lr, wd, scaled, transposed)
        for i in range(real):
            _record_pending(optimizer_states[i], P[i], R[i], -(1.0 - mu), transposed)
    else:
        codec.ef_apply(list(momentums[:real]), list(params[:real]), P, R, list(Qs[:real]), nonzero, mu, lr, wd,
                       scaled, transposed)
    clock.mark("apply_update")
    commit_qs()
    if commit_updates is not None:
        for i in range(real):
            if commit_updates[i] is not None:
                commit_updates[i](params[i], momentums[i])
    optimizer._last_batch_factors = (P, R) if getattr(optimizer, "_keep_factors", False) else None
    sink = getattr(optimizer, "_factor_sink", None)
    if sink is not None:  # the compressed factors leaving the device (scripts/e2e_pcie.py)
        sink(P[:real], R[:real], list(params[:real]))


def _fs_batch_update(optimizer, params, momentums, Qs, configs, dist_metas, optim_groups, real_grads,
                     optimizer_states, param_shapes, real, batch_cache_key, batch_group, batch_collectives,
                     commit_updates, use_low_rank, sketches):
    """One FS ("fsdp") batch: the reference's default Dion topology (FS = DP,
    megatron/training/initialize.py:79-81).  Entry i of the batch is this rank's shard of
    matrix i, sharded along fs_shard_dim, and the orientation puts the sharded dim on the
    contraction side (dion/state.py:304-310), so P_local = X_local Q_local is a partial sum:

      M += G (the local shard); P = X Q (partial)                      pass A, local
      reduce-scatter(sum) over the FS group -> this rank's entry      runtime.py:1201-1216 / :1751-1757
        (+ all-reduce(avg) over the replicate group with low-rank sync, :1218-1228)
      orthonormalise it (zero for a padded entry), all-gather          :1229-1293 / :1758-1795
      R = X^T P (this shard's rows of R)                               pass B, local
        (+ all-reduce(avg) over the replicate group with low-rank sync, :1284-1291)
      fix-up with this shard's zero test; local column sums of R^2, all-reduced (sum) over
        the q_norm group (the FS group), Q = R / (sqrt(sum) + eps)     kernels.py:157-210, runtime.py:965-1013
      error feedback on the shard; weight update with the GLOBAL shape's scaled LR  runtime.py:1015-1113
    """
    codec = optimizer.codec
    fs = batch_collectives.fs_collective
    fs_group, fs_world, fs_rank = fs.process_group, int(fs.world_size), int(fs.rank)
    indices = tuple(int(i) for i in fs.indices)
    if sorted(indices) != list(range(len(params))):
        raise RuntimeError(f"[DION_FSONLY_GATHER_PERMUTATION_INVALID] batch_size={len(params)} indices={indices}")
    rgroup = getattr(batch_group, "low_rank_replicate_group", None)
    rworld = _group_world(rgroup)
    group = getattr(batch_group, "replicate_group", None)
    if not use_low_rank and _group_world(group) > 1 and real_grads:
        # runtime.py:1553-1558 -> :439-491: dense all-reduce of the shard gradients across replicas
        yield from dense_replica_all_reduce(optimizer, real_grads, group)
    B = len(params)
    m, n = (int(d) for d in param_shapes[0])
    transposed = bool(configs[0].is_transposed)
    r = int(Qs[0].shape[1])
    mp, nq = factor_rows(m, n, transposed)
    dev = momentums[0].device
    oversample = float(optimizer.defaults["rcqr_oversample"])
    Qs, commit_qs = _qs_in_state_dtype(list(Qs), real, momentums[0].dtype)
    # bf16 momentum and Q (the speedrun's FS = 4 recipe): P and R stay fp32 buffers of bf16
    # values, rounded where the reference's bf16 tensors round (after each reduction)
    bf16_state = momentums[0].dtype == torch.bfloat16
    P = torch.zeros((B, mp, r), dtype=torch.float32, device=dev)
    nonzero = torch.zeros((B,), dtype=torch.int32, device=dev)
    defer = (getattr(optimizer, "_defer_ef", False) and hasattr(codec, "supports_deferred_ef")
             and (commit_updates is None or all(c is None for c in commit_updates[:real]))
             and codec.supports_deferred_ef(m, n, r, transposed, state_dtype=momentums[0].dtype,
                                           grad_dtype=real_grads[0].dtype if real_grads else None))
    clock = PhaseClock(optimizer, dev, _batch_desc(batch_group, dist_metas, real, (m, n)))
    _project_with_pending(codec, real_grads, momentums, Qs, P, nonzero, optimizer_states, real, m, n, transposed,
                          defer)
    clock.mark("p_matmul")
    # reduce-scatter(sum): this rank receives entry fs_rank summed over the FS shards
    P_own = torch.empty((1, mp, r), dtype=torch.float32, device=dev)
    work = dist.reduce_scatter_tensor(P_own, P, op=dist.ReduceOp.SUM, group=fs_group, async_op=True)
    yield
    work.wait()
    if bf16_state:
        codec.round_bf16(P_own)
    if use_low_rank and rworld > 1:
        work = dist.all_reduce(P_own, op=dist.ReduceOp.AVG, group=rgroup, async_op=True)  # runtime.py:367-369
        yield
        work.wait()
        if bf16_state:
            codec.round_bf16(P_own)
    clock.mark("p_reduce")
    own = indices[fs_rank]
    if own >= real or dist_metas[own] is None:
        P_own.zero_()  # a padded entry stays inert (runtime.py:1242-1248)
    else:
        S = None if sketches is None else sketches.get(own)
        codec.orthonormalize(P_own, m, n, transposed, _sketch_seed(optimizer, batch_cache_key, own), oversample,
                             sketch=None if S is None else S.reshape(1, *S.shape[-2:]).contiguous(),
                             state_dtype=momentums[0].dtype)
    gathered = torch.empty_like(P)
    work = dist.all_gather_into_tensor(gathered, P_own, group=fs_group, async_op=True)
    yield
    work.wait()
    if indices == tuple(range(B)):
        P = gathered
    else:
        for k, idx in enumerate(indices):
            P[idx].copy_(gathered[k])
    R = torch.zeros((B, nq, r), dtype=torch.float32, device=dev)
    codec.project_r(list(momentums[:real]), P, R, transposed, nonzero=nonzero)
    if use_low_rank and rworld > 1:
        work = dist.all_reduce(R, op=dist.ReduceOp.AVG, group=rgroup, async_op=True)
        yield
        work.wait()
        if bf16_state:
            codec.round_bf16(R)
    clock.mark("ortho_r")
    colsum = torch.empty((real, r), dtype=torch.float32, device=dev)
    codec.fixup_colsum(P, R, list(Qs[:real]), nonzero, colsum, m, n, transposed)
    qgroup = getattr(batch_group, "q_norm_group", None)
    if qgroup is not None:
        work = dist.all_reduce(colsum, op=dist.ReduceOp.SUM, group=qgroup, async_op=True)
        yield
        work.wait()
    codec.colnorm_apply(R, list(Qs[:real]), colsum, float(optimizer.defaults["epsilon"]), m, n, transposed)
    clock.mark("q_normalize")
    _apply_updates(optimizer, codec, params, momentums, Qs, P, R, nonzero, optim_groups, optimizer_states,
                   dist_metas, real, m, n, transposed, defer, commit_updates, commit_qs)
    clock.mark("apply_update")


def _tp_batch_update(optimizer, params, momentums, Qs, configs, dist_metas, optim_groups, real_grads,
                     optimizer_states, param_shapes, real, batch_cache_key, batch_group, batch_collectives,
                     commit_updates, use_low_rank, sketches):
    """One TP ("fsdp_tp") batch: every entry is this rank's TP shard of a matrix, sharded on the
    P-row side (dion/state.py:304-310, 407-416), and its Q holds this rank's columns of Q
    (resolve_q_state_layout, state.py:159-217).  The reference's order:

      dense all-reduce of G across replicas without low-rank sync     runtime.py:1553-1558
      Q all-gathered over TP (columns in rank order)                  runtime.py:680-873
      M += G; P = X Q_full (this rank's rows of P)                    pass A, local
      FS on the contraction side: all-reduce(sum) of P over FS        runtime.py:876-920
      with low-rank sync over replicas: all-reduce(avg) of P          runtime.py:1339-1345
      row-sharded randomised Cholesky QR over the TP group            ortho.py:682-834
      R = X^T P, all-reduce(sum) over TP (+ avg over replicas)        runtime.py:923-962, 1361-1376
      fix-up with the local zero test and the gathered Q; column norm (summed over the FS
        q_norm group when FS shards the rows of R); error feedback on the shard; weight
        update with the GLOBAL shape's LR                              runtime.py:1838-1901
      Q <- this rank's columns of the new Q                           ortho.py:837-871, runtime.py:1101-1132
    `sketches` (tests): entry -> this rank's (k, local rows) slice of the sketch."""
    codec = optimizer.codec
    group = getattr(batch_group, "replicate_group", None)
    W = _group_world(group)
    if W > 1 and not use_low_rank and real_grads:
        yield from dense_replica_all_reduce(optimizer, real_grads, group)
    B = len(params)
    m, n = (int(d) for d in param_shapes[0])
    transposed = bool(configs[0].is_transposed)
    mp, nq = factor_rows(m, n, transposed)
    dev = momentums[0].device
    bf16_state = momentums[0].dtype == torch.bfloat16  # P, R round after reductions
    qdt = momentums[0].dtype  # Q computes in the momentum's dtype (runtime.py:1576-1590), commits in its own
    # Q unshard: all-gather this rank's columns (padded to the widest rank) over TP
    gath = batch_collectives.tp_q_gathers[0]
    tp_group, T, tp_rank = gath.process_group, int(gath.world_size), int(gath.rank)
    r = int((optimizer_states[0] or {}).get("r", -1))
    if r <= 0:
        raise RuntimeError(f"[DION_INVALID_Q_UNSHARD_RANK] step={optimizer._step_count} r={r}")
    cols = [split_range(r, T, k) for k in range(T)]
    widest = max(c1 - c0 for c0, c1 in cols)
    c0, c1 = cols[tp_rank]
    for i in range(B):
        if tuple(Qs[i].shape) != (nq, c1 - c0):
            raise RuntimeError(f"[DION_Q_UNSHARD_LOCAL_RANK_MISMATCH] step={optimizer._step_count} entry={i} "
                               f"local_shape={tuple(Qs[i].shape)} expected={(nq, c1 - c0)} r={r} tp={T}")
    clock = PhaseClock(optimizer, dev, _batch_desc(batch_group, dist_metas, real, (m, n)))
    local = torch.zeros((B, nq, widest), dtype=qdt, device=dev)
    for i in range(B):
        local[i, :, :c1 - c0].copy_(Qs[i])
    gathered = torch.empty((T * B, nq, widest), dtype=qdt, device=dev)
    work = dist.all_gather_into_tensor(gathered, local, group=tp_group, async_op=True)
    yield
    work.wait()
    gathered = gathered.view(T, B, nq, widest)
    Qfull = torch.empty((B, nq, r), dtype=qdt, device=dev)
    for k, (a, b) in enumerate(cols):
        Qfull[:, :, a:b].copy_(gathered[k, :, :, :b - a])
    del local, gathered
    qviews = [Qfull[i] for i in range(B)]
    clock.mark("q_unshard")
    P = torch.zeros((B, mp, r), dtype=torch.float32, device=dev)
    nonzero = torch.zeros((B,), dtype=torch.int32, device=dev)
    defer = (getattr(optimizer, "_defer_ef", False) and hasattr(codec, "supports_deferred_ef")
             and (commit_updates is None or all(c is None for c in commit_updates[:real]))
             and codec.supports_deferred_ef(m, n, r, transposed, state_dtype=momentums[0].dtype,
                                           grad_dtype=real_grads[0].dtype if real_grads else None))
    _project_with_pending(codec, real_grads, momentums, qviews, P, nonzero, optimizer_states, real, m, n, transposed,
                          defer)
    clock.mark("p_matmul")
    for coll in tuple(getattr(batch_collectives, "fs_p_collectives", None) or ()):
        if coll.process_group is not None and int(coll.world_size) > 1:
            idx = [int(i) for i in coll.indices]
            work = (dist.all_reduce(P, op=dist.ReduceOp.SUM, group=coll.process_group, async_op=True)
                    if idx == list(range(B)) else
                    dist.all_reduce_coalesced([P[i] for i in idx], op=dist.ReduceOp.SUM, group=coll.process_group,
                                              async_op=True))
            yield
            work.wait()
            if bf16_state:
                codec.round_bf16(P)
    if use_low_rank and W > 1:
        work = dist.all_reduce(P, op=dist.ReduceOp.AVG, group=group, async_op=True)
        yield
        work.wait()
        if bf16_state:
            codec.round_bf16(P)
    clock.mark("p_reduce")
    yield from distributed_orthonormalize(optimizer, P, real, m, n, transposed, batch_group.ortho_group, dist_metas,
                                          batch_cache_key, sketches)
    if bf16_state:
        codec.round_bf16(P)  # ortho.py:829 P_local.to(original_dtype)
    R = torch.empty((B, nq, r), dtype=torch.float32, device=dev)
    codec.project_r(list(momentums[:real]), P[:real], R[:real], transposed, nonzero=nonzero)
    if real < B:
        R[real:].zero_()
    rsum = batch_collectives.tp_r_collectives[0]
    work = dist.all_reduce(R, op=dist.ReduceOp.SUM, group=rsum.process_group, async_op=True)
    yield
    work.wait()
    if bf16_state:
        codec.round_bf16(R)
    if use_low_rank and W > 1:
        work = dist.all_reduce(R, op=dist.ReduceOp.AVG, group=group, async_op=True)
        yield
        work.wait()
        if bf16_state:
            codec.round_bf16(R)
    clock.mark("ortho_r")
    eps = float(optimizer.defaults["epsilon"])
    qgroup = getattr(batch_group, "q_norm_group", None)
    if qgroup is not None and _group_world(qgroup) > 1:
        colsum = torch.empty((real, r), dtype=torch.float32, device=dev)
        codec.fixup_colsum(P, R, qviews[:real], nonzero, colsum, m, n, transposed)
        work = dist.all_reduce(colsum, op=dist.ReduceOp.SUM, group=qgroup, async_op=True)
        yield
        work.wait()
        codec.colnorm_apply(R, qviews[:real], colsum, eps, m, n, transposed)
    else:
        codec.fixup_colnorm(P, R, qviews[:real], nonzero, eps, m, n, transposed)
    clock.mark("q_normalize")
    _apply_updates(optimizer, codec, params, momentums, qviews, P, R, nonzero, optim_groups, optimizer_states,
                   dist_metas, real, m, n, transposed, defer, commit_updates)
    clock.mark("apply_update")
    for i in range(real):  # reshard_q_along_tp: keep this rank's columns
        Qs[i].copy_(Qfull[i][:, c0:c1])


def _tp_row_sizes(dist_metas, real, T, global_rows):
    """ortho.py:270-380: explicit row_shard_sizes from the metadata, else the canonical split."""
    meta = next((d for d in dist_metas[:real] if d is not None), None)
    explicit = getattr(meta, "row_shard_sizes", None) if meta is not None else None
    if explicit is not None:
        sizes = [int(x) for x in explicit]
        if len(sizes) != T or sum(sizes) != global_rows:
            raise RuntimeError(f"[DION_ORTHO_ROW_SIZES_MISMATCH] row_shard_sizes={tuple(sizes)} ortho_world={T} "
                               f"global_rows={global_rows}")
        return sizes
    return [b - a for a, b in (split_range(global_rows, T, k) for k in range(T))]


def distributed_orthonormalize(optimizer, P, real, m, n, transposed, ortho_group, dist_metas, batch_cache_key,
                               sketches=None):
    """Randomised Cholesky QR of the first `real` entries of a row-sharded P (this rank's rows,
    in place), dion/ortho.py:682-834.  The small products run on the device (dion_dortho_*);
    the reductions over the ortho group follow the reference's partition: reduce-scatter
    (sum) over batch shards, the owner factors its entries, all-gather of the factors."""
    codec = optimizer.codec
    T, rank = _group_world(ortho_group), int(dist.get_rank(ortho_group))
    B, rows, r = (int(x) for x in P.shape)
    dev = P.device
    meta0 = next((d for d in dist_metas[:real] if d is not None), None)
    gshape = getattr(meta0, "global_shape", None) if meta0 is not None else None
    if gshape is None:
        raise RuntimeError("[DION_MISSING_ORTHO_GLOBAL_SHAPE] distributed orthonormalisation needs global_shape")
    global_rows = int(gshape[1]) if transposed else int(gshape[0])
    sizes = _tp_row_sizes(dist_metas, real, T, global_rows)
    if sizes[rank] != rows:
        raise RuntimeError(f"[DION_ORTHO_ROW_LAYOUT_MISMATCH] local rows {rows} != {sizes[rank]} "
                           f"(row sizes {tuple(sizes)}, rank {rank})")
    offset = sum(sizes[:rank])
    Pa = P[:real]
    if global_rows <= r:
        # ortho.py:752-775: the whole P is a short matrix; every rank gathers the rows and
        # takes the Q factor of the same Householder QR (the reference gives each rank a share
        # of the batch instead: the same numbers)
        widest = max(sizes)
        buf = torch.zeros((real, widest, r), dtype=torch.float32, device=dev)
        buf[:, :rows].copy_(Pa)
        allrows = torch.empty((T * real, widest, r), dtype=torch.float32, device=dev)
        work = dist.all_gather_into_tensor(allrows, buf, group=ortho_group, async_op=True)
        yield
        work.wait()
        allrows = allrows.view(T, real, widest, r)
        full = torch.cat([allrows[k, :, :sizes[k]] for k in range(T)], dim=1).contiguous()
        codec.orthonormalize(full, global_rows, max(r, 1), False, 0, float(optimizer.defaults["rcqr_oversample"]))
        Pa.copy_(full[:, offset:offset + rows])
        return
    oversample = float(optimizer.defaults["rcqr_oversample"])
    k = int(math.ceil(oversample * r / 128.0) * 128)  # ortho.py:595
    shares = [b - a for a, b in (split_range(real, T, q) for q in range(T))]
    most = max(shares)
    starts = [sum(shares[:q]) for q in range(T)]

    def exchange(local_full, width):
        """Reduce-scatter (sum) the (real, width, r) products by batch shards; return this rank's
        (most, width, r) sums (ortho.py:529-572)."""
        padded = torch.zeros((T * most, width, r), dtype=torch.float32, device=dev)
        for q in range(T):
            if shares[q]:
                padded[q * most:q * most + shares[q]].copy_(local_full[starts[q]:starts[q] + shares[q]])
        mine = torch.empty((most, width, r), dtype=torch.float32, device=dev)
        work = dist.reduce_scatter_tensor(mine, padded, op=dist.ReduceOp.SUM, group=ortho_group, async_op=True)
        return mine, work

    def gather(mine_inv):
        """All-gather the owners' (most, r, r) factors back to (real, r, r) (ortho.py:383-419)."""
        allf = torch.empty((T * most, r, r), dtype=torch.float32, device=dev)
        work = dist.all_gather_into_tensor(allf, mine_inv, group=ortho_group, async_op=True)
        return allf, work

    def unpack(allf):
        return torch.cat([allf[q * most:q * most + shares[q]] for q in range(T) if shares[q]], dim=0).contiguous()

    SP = torch.empty((real, k, r), dtype=torch.float32, device=dev)
    if sketches is not None:
        S = torch.stack([sketches[i].to(device=dev, dtype=torch.float32) for i in range(real)], dim=0).contiguous()
    else:
        S = None
    seed = _sketch_seed(optimizer, batch_cache_key, 0)
    codec.dortho_sketch(Pa, m, n, transposed, seed, offset, oversample, SP, sketch=S)
    mine, work = exchange(SP, k)
    yield
    work.wait()
    inv = torch.zeros((most, r, r), dtype=torch.float32, device=dev)
    if shares[rank]:
        codec.dortho_qr_inv(mine[:shares[rank]].contiguous(), inv[:shares[rank]])
    allf, work = gather(inv)
    yield
    work.wait()
    P1 = torch.empty_like(Pa)
    codec.dortho_apply(Pa, unpack(allf), P1, m, n, transposed)
    gram = torch.empty((real, r, r), dtype=torch.float32, device=dev)
    codec.dortho_gram(P1, gram, m, n, transposed)
    mine, work = exchange(gram, r)
    yield
    work.wait()
    inv.zero_()
    if shares[rank]:
        codec.dortho_chol_inv(mine[:shares[rank]].contiguous(), inv[:shares[rank]])
    allf, work = gather(inv)
    yield
    work.wait()
    codec.dortho_apply(P1, unpack(allf), Pa, m, n, transposed)


def _qs_in_state_dtype(Qs, real, dtype):
    """Q states in the momentum's dtype, as the reference computes with them: Q_batch is cast to
    M_batch.dtype for P = M Q (runtime.py:1576-1590), Q_new keeps R's dtype for the update
    (kernels.py:229-276) and is cast into the Q state on commit (runtime.py:1132).  With
    independent momentum / Q dtypes (DionMixedPrecisionConfig, types.py:10-17) the batch runs on
    a cast copy; `commit()` writes the new Q back in the state's own dtype."""
    if all(q.dtype == dtype for q in Qs):
        return list(Qs), (lambda: None)
    work = [q if q.dtype == dtype else q.to(dtype) for q in Qs]

    def commit():
        for i in range(real):
            if work[i] is not Qs[i]:
                Qs[i].copy_(work[i])
    return work, commit


def _project_with_pending(codec, real_grads, momentums, Qs, P, nonzero, optimizer_states, real, m, n, transposed,
                          defer):
    """Pass A: M (+ the pending error feedback of the previous step) += G; P = X Q."""
    pending = [_take_pending(optimizer_states[i]) for i in range(real)]
    if any(p is not None for p in pending):
        alphas = {p[2] for p in pending if p is not None}
        if defer and len(alphas) == 1:
            try:
                codec.project_p_ef(real_grads or None, list(momentums[:real]), list(Qs[:real]), P, nonzero,
                                   transposed, [p[0] if p is not None else None for p in pending],
                                   [p[1] if p is not None else None for p in pending], alphas.pop())
                return
            except DionUnsupportedError:
                # refused before any launch (e.g. a momentum or gradient view whose layout the
                # fused kernel cannot stream): the popped error feedback goes on eagerly
                pass
        for i, p in enumerate(pending):
            if p is not None:
                _apply_pending(codec, momentums[i], Qs[i], p, m, n, transposed)
    codec.project_p(real_grads or None, list(momentums[:real]), list(Qs[:real]), P, nonzero, transposed)


def _apply_updates(optimizer, codec, params, momentums, Qs, P, R, nonzero, optim_groups, optimizer_states,
                   dist_metas, real, m, n, transposed, defer, commit_updates, commit_qs=None):
    """Error feedback (now, or pending for the next pass A) and the weight update with the
    global shape's scaled LR (runtime.py:1015-1113, kernels.py:25-51)."""
    grp = optim_groups[0] or {}
    st0 = optimizer_states[0] or {}
    gshape = st0.get("per_expert_global_shape") or st0.get("global_shape") \
        or getattr(dist_metas[0], "global_shape", None) or (m, n)
    lr = float(grp.get("lr", optimizer.defaults["lr"]))
    mu = float(grp.get("mu", optimizer.defaults["mu"]))
    wd = float(grp.get("weight_decay", optimizer.defaults["weight_decay"] * float(grp.get("wd_mult", 1.0))))
    rank_fraction = float(grp.get("rank_fraction", optimizer.defaults.get("rank_fraction", 0.25)))
    scaled = scaled_lr_for_shape(lr=lr, m_global=int(gshape[0]), n_global=int(gshape[1]),
                                 scale_mode=optimizer.defaults.get("scale_mode", "spectral"),
                                 rank_fraction=rank_fraction,
                                 extra_scale_factor=optimizer.defaults.get("extra_scale_factor", 0.2))
    if defer:
        codec.ef_apply(None, list(params[:real]), P, R, list(Qs[:real]), nonzero, mu, lr, wd, scaled, transposed)
        for i in range(real):
            _record_pending(optimizer_states[i], P[i], R[i], -(1.0 - mu), transposed)
    else:
        codec.ef_apply(list(momentums[:real]), list(params[:real]), P, R, list(Qs[:real]), nonzero, mu, lr, wd,
                       scaled, transposed)
    if commit_qs is not None:
        commit_qs()
    if commit_updates is not None:
        for i in range(real):
            if commit_updates[i] is not None:
                commit_updates[i](params[i], momentums[i])
    optimizer._last_batch_factors = (P, R) if getattr(optimizer, "_keep_factors", False) else None
    sink = getattr(optimizer, "_factor_sink", None)
    if sink is not None:
        sink(P[:real], R[:real], list(params[:real]))


# optimizer-state key of a pending (deferred) error feedback: (P_b, R_b, alpha, M ref,
# transposed).  The orientation is recorded with the factors: it cannot be told from the
# shapes (a square FS or TP shard has m_P == m in either orientation).
# The leading underscore keeps it out of the reference's persistent checkpoint state
# (distrib_dion/checkpoint_io.py:247-266), so the momentum must carry it before anything
# outside the step reads it: DionParamState applies it on such a read, and
# MegatronDion.flush_error_feedback() applies all of them.  The weak reference names the
# momentum tensor the factors belong to: a restore that replaces the momentum
# (checkpoint_io.py:300-330 keeps the live underscore keys) orphans the entry, and an
# orphan is dropped, never applied to the restored value.
_PENDING_EF = "_dion_pending_ef"


def _record_pending(state, P_b, R_b, alpha, transposed: bool) -> None:
    M = dict.get(state, "momentum")
    dict.__setitem__(state, _PENDING_EF, (P_b, R_b, alpha, weakref.ref(M) if M is not None else None,
                                          bool(transposed)))


def _fused_kw(fix, split, i0, i1) -> dict:
    """orthonormalize's fused fix-up / pass-B split arguments for entries [i0, i1)."""
    kw = {}
    if fix is not None:
        kw["fix_nonzero"] = fix[i0:i1]
    if split is not None:
        kw["p_split"] = split[i0:i1]
    return kw


def _take_pending(state):
    """Pop one state's pending error feedback as (P_b, R_b, alpha, transposed); None when there
    is none or when it was recorded for a momentum tensor the state no longer holds."""
    if state is None:
        return None
    pend = dict.pop(state, _PENDING_EF, None)
    if pend is None:
        return None
    ref = pend[3]
    if ref is not None and ref() is not dict.get(state, "momentum"):
        return None
    return pend[0], pend[1], pend[2], pend[4]


class DionParamState(dict):
    """A Dion parameter's optimizer state that applies its pending error feedback before
    any read of the momentum from outside the step (`state["momentum"]`, `.get`,
    `.items()`, `.values()`, copies, pickling): checkpoint writers such as the reference's
    build_persistent_param_state (checkpoint_io.py:247-266, which iterates `state.items()`
    and skips underscore keys) then save the eager momentum.  Inside MegatronDion.step
    the read is plain, so the deferral is kept."""

    __slots__ = ("_owner",)

    def __init__(self, *args, owner=None, **kwargs):
        super().__init__(*args, **kwargs)
        self._owner = owner

    def _sync(self):
        if not dict.__contains__(self, _PENDING_EF):
            return
        opt = self._owner() if self._owner is not None else None
        if opt is None or getattr(opt, "_dion_in_step", False):
            return
        pend = _take_pending(self)
        if pend is not None:
            M = dict.__getitem__(self, "momentum")
            _apply_pending(opt.codec, M, dict.__getitem__(self, "Q"), pend, int(M.shape[0]), int(M.shape[1]),
                           pend[3])

    def __getitem__(self, key):
        if key == "momentum":
            self._sync()
        return dict.__getitem__(self, key)

    def get(self, key, default=None):
        if key == "momentum":
            self._sync()
        return dict.get(self, key, default)

    def items(self):
        self._sync()
        return dict.items(self)

    # dict(state), {**state} and dict.update(other, state) copy a dict subclass through
    # CPython's fast path (no __getitem__) unless its type overrides __iter__: with these
    # overrides they go through keys() / __getitem__ and see the eager momentum
    def __iter__(self):
        self._sync()
        return dict.__iter__(self)

    def keys(self):
        self._sync()
        return dict.keys(self)

    def values(self):
        self._sync()
        return dict.values(self)

    def copy(self):
        self._sync()
        return dict(dict.items(self))

    def __reduce__(self):
        self._sync()
        return (dict, (dict(dict.items(self)),))


class DionStateMap(collections.defaultdict):
    """`optimizer.state` of MegatronDion: new entries, and plain dicts assigned by a
    restore (checkpoint_io.py:351 `optimizer_state[param] = new_state`), become
    DionParamState."""

    def __init__(self, owner, *args):
        super().__init__(None, *args)
        self._owner_ref = weakref.ref(owner)
        for k in list(dict.keys(self)):
            dict.__setitem__(self, k, self._wrap(dict.__getitem__(self, k)))

    def _wrap(self, v):
        if type(v) is dict:
            return DionParamState(v, owner=self._owner_ref)
        return v

    def __missing__(self, key):
        v = DionParamState(owner=self._owner_ref)
        dict.__setitem__(self, key, v)
        return v

    def __setitem__(self, key, value):
        dict.__setitem__(self, key, self._wrap(value))

    def __reduce__(self):
        return (dict, (dict(dict.items(self)),))


def _apply_pending(codec, M, Q, pending, m, n, transposed):
    """M += alpha P R^T (or alpha R P^T) for one matrix: the eager error feedback, late."""
    Pb, Rb, alpha = pending[:3]
    mu = 1.0 + float(alpha)
    Q = Q if Q.dtype == M.dtype else Q.to(M.dtype)  # independent Q dtype: only its dtype is read here
    ones = torch.ones((1,), dtype=torch.int32, device=M.device)
    codec.ef_apply([M], None, Pb.unsqueeze(0), Rb.unsqueeze(0), [Q], ones, mu, 0.0, 0.0, 0.0, transposed)


def flush_pending_error_feedback(optimizer, get_codec) -> int:
    """Apply every deferred error feedback held in `optimizer.state`; returns how many."""
    count = 0
    codec = None
    for p, st in dict.items(optimizer.state):
        pend = _take_pending(st) if isinstance(st, dict) else None
        if pend is None:
            continue
        codec = codec or get_codec()
        M, Q = dict.__getitem__(st, "momentum"), dict.__getitem__(st, "Q")
        _apply_pending(codec, M, Q, pend, int(M.shape[0]), int(M.shape[1]), pend[3])
        count += 1
    return count


def drop_pending_error_feedback(optimizer) -> int:
    """Forget every deferred error feedback (the momentum is about to be replaced)."""
    count = 0
    for st in dict.values(optimizer.state):
        if isinstance(st, dict) and dict.pop(st, _PENDING_EF, None) is not None:
            count += 1
    return count


def run_dion_batch_async(optimizer, batch, sketches=None, phase_marks=False) -> Generator[None, None, None]:
    """Unpack a DionBatch (ours or the reference's) into batch_dion_update_async."""
    if batch is None or not batch.params:
        return
    entries = getattr(batch, "entries", ())
    commit = [getattr(e, "commit_update", None) for e in entries[:int(batch.real_batch_size)]]
    yield from batch_dion_update_async(
        optimizer, list(batch.params), list(batch.momentums), list(batch.q_tensors), list(batch.configs),
        list(batch.dist_metas), list(batch.optim_groups), list(batch.grads), list(batch.optimizer_states),
        list(batch.param_shapes), int(batch.real_batch_size), int(batch.batch_cache_key), batch.batch_group,
        batch.batch_collectives, commit_updates=commit, sketches=sketches,
        chunks=int(getattr(batch, "_chunks", 0) or 0), phase_marks=phase_marks)


def coalesce_replicated_batches(batches, max_entries: int = 16):
    """Merge consecutive full same-key W > 1 batches into one launch group of k chunks.

    The merged batch keeps the reference's assignment of entries to ranks: entry
    c W + r of the group (chunk c) is orthonormalised by rank r (runtime.py:1428-1435).
    `batch_dion_update_async` lays the group out rank-major (position r k + c), so ONE
    reduce-scatter hands rank r its k entries, one batched orthonormalisation runs on
    them and ONE all-gather restores the group; R is all-reduced in one call.  Same
    per-entry arithmetic, k times fewer launches and collectives.
    """
    from .types import DionBatch

    out = []
    for b in batches:
        W = _group_world(getattr(getattr(b, "batch_group", None), "replicate_group", None))
        full = W > 1 and int(b.real_batch_size) == len(b.params) == W
        prev = out[-1] if out else None
        if full and prev is not None and getattr(prev, "_chunks", 0) > 0 and prev.batch_key == b.batch_key \
                and prev.batch_group is b.batch_group and len(prev.entries) + W <= max(max_entries, W):
            merged = DionBatch(batch_key=prev.batch_key, entries=tuple(prev.entries) + tuple(b.entries),
                               real_batch_size=prev.real_batch_size + b.real_batch_size,
                               batch_cache_key=prev.batch_cache_key, batch_group=prev.batch_group,
                               batch_collectives=prev.batch_collectives)
            merged._chunks = prev._chunks + 1
            out[-1] = merged
        elif full:
            nb = DionBatch(batch_key=b.batch_key, entries=tuple(b.entries), real_batch_size=b.real_batch_size,
                           batch_cache_key=b.batch_cache_key, batch_group=b.batch_group,
                           batch_collectives=b.batch_collectives)
            nb._chunks = 1
            out.append(nb)
        else:
            out.append(b)
    return out


def coalesce_local_batches(batches, max_entries: int = 64):
    """Merge consecutive same-key batches of a world-size-1 schedule into one launch group.

    At batch_world_size 1 every DionBatch holds one matrix (batches.py:1001-1036)
    and the matrices are independent, so running k of them through one set of
    kernel launches is the same computation with k times fewer launches.
    """
    from .types import DionBatch

    out = []
    for b in batches:
        bg = b.batch_group
        if is_replicated(b) or int(b.real_batch_size) != len(b.params):
            out.append(b)
            continue
        if out and isinstance(out[-1], DionBatch) and getattr(out[-1], "_coalesced", False) \
                and out[-1].batch_key == b.batch_key and len(out[-1].entries) + len(b.entries) <= max_entries:
            prev = out[-1]
            merged = DionBatch(batch_key=prev.batch_key, entries=tuple(prev.entries) + tuple(b.entries),
                               real_batch_size=prev.real_batch_size + b.real_batch_size,
                               batch_cache_key=prev.batch_cache_key, batch_group=prev.batch_group,
                               batch_collectives=prev.batch_collectives)
            merged._coalesced = True
            out[-1] = merged
        else:
            nb = DionBatch(batch_key=b.batch_key, entries=tuple(b.entries), real_batch_size=b.real_batch_size,
                           batch_cache_key=b.batch_cache_key, batch_group=b.batch_group,
                           batch_collectives=b.batch_collectives)
            nb._coalesced = True
            out.append(nb)
    return out
