"""Batch assembly for the data-parallel (replicate) Dion path.

Follows /root/reference/megatron/core/optimizer/distrib_dion/batches.py:
  build_batch_key            :76-107   (shape/shard/orientation/low-rank/dtype key)
  update-contract key        :52-73    (lr, weight_decay, wd_mult, mu, rank_fraction, r)
  group key                  :233-242  (kernel kind, batch world size, group ranks)
  ordering                   :115-117, :195 (sorted by repr of the key; identical on every rank)
  chunk + pad                :903-1067 (chunks of batch_world_size; padding entries carry
                                        zero grad/momentum/Q, dist_meta=None, the first param)
The reference agrees the order across ranks with a (cached) all_gather_object;
replicas of a data-parallel model hold identical parameter sets, so the locally
sorted order is already global.  `verify_schedule_across_ranks` performs the
same agreement check once when asked.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .types import DionAxisCollective, DionBatch, DionBatchCollectives, DionBatchEntry, DionBatchGroup


def _norm_dim(dim, has_axis: bool) -> int:
    if dim is None and not has_axis:
        return -1
    if dim is None:
        raise RuntimeError("[Dion] missing shard tensor dim for active sharded axis in batch key construction")
    return int(dim)


def _norm_shape(shape) -> tuple:
    return () if shape is None else tuple(int(d) for d in shape)


def build_batch_key(shape, cfg, dtype, *, global_shape=None, per_expert_global_shape=None,
                    tensor_row_shard_sizes=None, row_shard_sizes=None) -> tuple:
    key_shape = per_expert_global_shape or global_shape or shape
    return (
        tuple(int(d) for d in key_shape),
        bool(cfg.has_fs_shard),
        bool(getattr(cfg, "use_fs_shard", cfg.has_fs_shard)),
        bool(cfg.has_tp_shard),
        bool(getattr(cfg, "use_tp_shard", cfg.has_tp_shard)),
        bool(cfg.is_transposed),
        bool(cfg.use_low_rank_sync),
        _norm_dim(cfg.tp_shard_dim, cfg.has_tp_shard),
        _norm_dim(cfg.fs_shard_dim, cfg.has_fs_shard),
        dtype,
        _norm_shape(global_shape),
        _norm_shape(per_expert_global_shape),
        _norm_shape(tensor_row_shard_sizes),
        _norm_shape(row_shard_sizes),
    )


def _contract_key(group: Optional[dict], state: Optional[dict]) -> tuple:
    def f(name):
        return float(group[name]) if group is not None and name in group else None
    r = int(state.get("r", -1)) if state is not None else -1
    return (f("lr"), f("weight_decay"), f("wd_mult"), f("mu"), f("rank_fraction"), r)


def _ranks(group) -> tuple:
    if group is None:
        return ()
    try:
        return tuple(int(x) for x in dist.get_process_group_ranks(group))
    except Exception:  # fake groups in unit tests
        return tuple(getattr(group, "ranks", ()))


def _group_key(bg: DionBatchGroup) -> tuple:
    return (str(bg.kernel_kind), int(bg.batch_world_size), _ranks(bg.replicate_group), _ranks(bg.ortho_group),
            _ranks(bg.q_norm_group), _ranks(bg.low_rank_replicate_group),
            tuple(_ranks(g) for g in bg.sync_groups))


def resolve_dp_batch_group(config, *, replicate_group, group_size: Callable, fs_group=None,
                           tp_group=None) -> DionBatchGroup:
    """resolve_batch_group (batches.py:496-603) for the DP/RP, FS and TP axes.

    A TP-sharded entry (P-row side, state.py:407-416) with a TP group of size > 1 gets the
    "fsdp_tp" kind: batch size = TP world, ortho group = TP group (sharding.py:194-209).  An
    FS-sharded entry with an FS group of size > 1 gets the "fsdp" kind: batch size = FS
    world, q_norm group = FS group, and with low-rank sync over replicas the
    low_rank_replicate_group (:571-603).  Everything else is "ddp" over the replicate group."""
    world = group_size(replicate_group) if replicate_group is not None else 1
    sync = [replicate_group] if (config.use_low_rank_sync and replicate_group is not None and world > 1) else []
    if getattr(config, "use_tp_shard", False):
        if tp_group is None:
            raise RuntimeError("[DION_MISSING_BATCH_TP_GROUP] a TP-sharded Dion param needs its TP group")
        tp_world = group_size(tp_group)
        dim, tr = int(getattr(config, "tp_shard_dim", -1)), bool(config.is_transposed)
        if not ((not tr and dim == 0) or (tr and dim == 1)):
            raise RuntimeError("[DION_UNSUPPORTED_SHARDING] TP on the contraction side of P is not built")
        if tp_world > 1:
            sync.append(tp_group)
            # FS x TP (the speedrun's topology): FS shards the contraction side; its group
            # normalises Q's columns (q_norm_group, batches.py:562-569) and sums P (:703-715)
            qn = None
            if bool(getattr(config, "use_fs_shard", False)):
                if fs_group is None:
                    raise RuntimeError("[DION_MISSING_BATCH_FS_GROUP] an FS-sharded Dion param needs its FS group")
                if group_size(fs_group) > 1:
                    sync.append(fs_group)
                    qn = fs_group
            return DionBatchGroup(kernel_kind="fsdp_tp", replicate_group=replicate_group, ortho_group=tp_group,
                                  q_norm_group=qn, batch_world_size=int(tp_world), sync_groups=tuple(sync))
    if bool(getattr(config, "use_fs_shard", False)):
        if fs_group is None:
            raise RuntimeError("[DION_MISSING_BATCH_FS_GROUP] an FS-sharded Dion param needs its FS group")
        fs_world = group_size(fs_group)
        if fs_world > 1:
            sync.append(fs_group)
            low = replicate_group if (config.use_low_rank_sync and replicate_group is not None and world > 1) else None
            return DionBatchGroup(kernel_kind="fsdp", replicate_group=replicate_group, q_norm_group=fs_group,
                                  low_rank_replicate_group=low, batch_world_size=int(fs_world),
                                  sync_groups=tuple(sync))
    return DionBatchGroup(kernel_kind="ddp", replicate_group=replicate_group, batch_world_size=int(world),
                          sync_groups=tuple(sync))


def build_dion_batches(*, dion_params: Sequence, get_replicate_group: Callable,
                       group_size: Callable = None, batch_key_cache: Optional[dict] = None,
                       resolve_fs_group_from_meta: Optional[Callable] = None,
                       resolve_tp_group: Optional[Callable] = None, **_unused) -> List[DionBatch]:
    """Group, order, chunk and pad routed Dion params into DionBatch objects.

    FS-sharded params (config.use_fs_shard) take their FS group from
    `resolve_fs_group_from_meta(dist_meta, expect_group=True)` (batches.py:971 takes the same
    callback) and form "fsdp" batches of FS-world entries with an FS collective covering every
    entry (build_batch_collectives, batches.py:606-770)."""
    group_size = group_size or (lambda g: dist.get_world_size(g))
    replicate_group = get_replicate_group()
    grouped: Dict[tuple, list] = {}
    groups: Dict[tuple, DionBatchGroup] = {}
    sync_of: Dict[tuple, list] = {}
    for sp in dion_params:
        state = sp.optimizer_state
        meta = sp.dist_meta
        cfg = sp.config
        local_shape = state.get("local_shape") or tuple(sp.param.shape)
        global_shape = state.get("global_shape") or getattr(meta, "global_shape", None)
        per_expert = state.get("per_expert_global_shape") or getattr(meta, "per_expert_global_shape", None)
        fs_group = None
        if bool(getattr(cfg, "use_fs_shard", False)):
            fs_group = resolve_fs_group_from_meta(meta, expect_group=True) if resolve_fs_group_from_meta \
                else getattr(meta, "fs_group", None)
        tp_group = None
        if bool(getattr(cfg, "use_tp_shard", False)):
            tp_group = resolve_tp_group(meta, expect_group=True) if resolve_tp_group \
                else getattr(meta, "tp_group", None)
        bg = resolve_dp_batch_group(cfg, replicate_group=replicate_group, group_size=group_size, fs_group=fs_group,
                                    tp_group=tp_group)
        key = (build_batch_key(local_shape, cfg, sp.grad.dtype, global_shape=global_shape,
                               per_expert_global_shape=per_expert,
                               tensor_row_shard_sizes=getattr(meta, "tensor_row_shard_sizes", None),
                               row_shard_sizes=getattr(meta, "row_shard_sizes", None)),
               _contract_key(sp.optim_group, state), _group_key(bg))
        grouped.setdefault(key, []).append(sp)
        groups.setdefault(key, bg)
        if key not in sync_of:  # resolve_batch_group's sync groups (batches.py:519-551)
            sync = []
            for g, on in ((replicate_group, cfg.use_low_rank_sync), (tp_group, getattr(cfg, "use_tp_shard", False)),
                          (fs_group, getattr(cfg, "use_fs_shard", False))):
                if on and g is not None and group_size(g) > 1 and all(g is not x for x in sync):
                    sync.append(g)
            sync_of[key] = sync

    # batches.py:855-884: keys listed per sync group in first-seen group order (keys with no sync
    # group form one more group), each group's keys sorted by repr, a key's first listing wins
    per_group: Dict[object, list] = {}
    for key in grouped:
        for g in sync_of[key] or [None]:
            per_group.setdefault(None if g is None else id(g), []).append(key)
    ordered = list(dict.fromkeys(k for keys in per_group.values() for k in sorted(keys, key=repr)))
    batches: List[DionBatch] = []
    cache_key = 0
    for key in ordered:
        items = grouped[key]
        bg = groups[key]
        size = max(1, int(bg.batch_world_size))
        for start in range(0, len(items), size):
            chunk = items[start:start + size]
            entries = []
            for sp in chunk:
                shape = tuple(int(d) for d in sp.optimizer_state["momentum"].shape)
                entries.append(DionBatchEntry(
                    param=sp.param, grad=sp.grad.view(*shape), optimizer_state=sp.optimizer_state,
                    optim_group=sp.optim_group, config=sp.config, dist_meta=sp.dist_meta,
                    momentum=sp.optimizer_state["momentum"].view(*shape), q_tensor=sp.optimizer_state["Q"],
                    param_shape=shape, commit_update=sp.commit_update))
            real = len(entries)
            tmpl = entries[0]
            while len(entries) < size:
                entries.append(DionBatchEntry(
                    param=tmpl.param, grad=torch.zeros_like(tmpl.grad), optimizer_state=None,
                    optim_group=tmpl.optim_group, config=tmpl.config, dist_meta=None,
                    momentum=torch.zeros_like(tmpl.momentum), q_tensor=torch.zeros_like(tmpl.q_tensor),
                    param_shape=tmpl.param_shape))
            coll = DionBatchCollectives()
            if bg.kernel_kind == "fsdp_tp":
                # build_batch_collectives (batches.py:659-771): Q gather, R sum and Q reshard over TP
                tp = bg.ortho_group
                ax = DionAxisCollective(indices=tuple(range(size)), process_group=tp, world_size=int(group_size(tp)),
                                        rank=int(dist.get_rank(tp)))
                fsp = ()
                if bg.q_norm_group is not None:  # should_reduce_p_over_fs: P = X Q sums over the FS shards
                    fs = bg.q_norm_group
                    fsp = (DionAxisCollective(indices=tuple(range(size)), process_group=fs,
                                              world_size=int(group_size(fs)), rank=int(dist.get_rank(fs))),)
                coll = DionBatchCollectives(tp_q_gathers=(ax,), tp_r_collectives=(ax,), tp_q_reshards=(ax,),
                                            fs_p_collectives=fsp)
            elif bg.kernel_kind == "fsdp":
                fs = bg.q_norm_group
                coll = DionBatchCollectives(fs_collective=DionAxisCollective(
                    indices=tuple(range(size)), process_group=fs, world_size=int(group_size(fs)),
                    rank=int(dist.get_rank(fs))))
            batches.append(DionBatch(batch_key=key, entries=tuple(entries), real_batch_size=real,
                                     batch_cache_key=cache_key, batch_group=bg, batch_collectives=coll))
            cache_key += real
    return batches


def verify_schedule_across_ranks(batches: Sequence[DionBatch], group) -> None:
    """Check every rank built the same (key, real size) schedule (batches.py:185-216)."""
    if group is None or dist.get_world_size(group) <= 1:
        return
    mine = [(repr(b.batch_key), int(b.real_batch_size)) for b in batches]
    gathered: List = [None] * dist.get_world_size(group)
    dist.all_gather_object(gathered, mine, group=group)
    if any(g != mine for g in gathered):
        raise RuntimeError("[DION_BATCH_KEY_MULTIPLICITY_MISMATCH] ranks built different Dion batch schedules")


def _sync_groups_of(batch: DionBatch) -> List[object]:
    """The process groups whose members must agree on this batch's place in the schedule: its
    sync groups (resolve_batch_group, batches.py:519-551: the replicate group under low-rank
    sync, the TP group, the FS group)."""
    out = []
    for g in tuple(getattr(batch.batch_group, "sync_groups", ()) or ()):
        if g is not None and dist.get_world_size(g) > 1 and all(g is not x for x in out):
            out.append(g)
    return out


def _collective_signature(batch: DionBatch) -> tuple:
    """What a batch's collectives look like to the other members of its groups: the kind, the
    batch / real sizes, the matrices' global shape, the global rank r and the orientation (the
    P / R / Q buffers' sizes follow from them).  Local shapes, local Q columns (TP) and group
    handles differ between the members of an FS or TP group, so the batch key itself is not
    comparable across ranks."""
    e = batch.entries[0]
    st = e.optimizer_state or {}
    gshape = st.get("per_expert_global_shape") or st.get("global_shape") or \
        getattr(e.dist_meta, "global_shape", None) or e.param_shape
    return (str(getattr(batch.batch_group, "kernel_kind", "ddp")), len(batch.entries), int(batch.real_batch_size),
            tuple(int(d) for d in gshape), int(st.get("r", -1)), bool(e.config.is_transposed))


def verify_sync_group_order(batches: Sequence[DionBatch]) -> None:
    """Every member of a process group must issue that group's collectives in the same order
    (batches.py:855-884 _sync_group_batch_metadata agrees on the order with an all_gather).  The
    local listing above is canonical for whole-group batches; a split child owned by part of its
    row group (split.split_child_layouts) gives the members of one parent group different key
    sets, so the order is checked once: per group, in one global order of groups (sorted member
    ranks, so the checks cannot wait on each other), all_gather the sequence of batch
    signatures (`_collective_signature`) this rank will issue on it and compare."""
    seqs: Dict[tuple, list] = {}
    handle: Dict[tuple, object] = {}
    for b in batches:
        for g in _sync_groups_of(b):
            ranks = tuple(int(r) for r in dist.get_process_group_ranks(g))
            handle.setdefault(ranks, g)
            seqs.setdefault(ranks, []).append(_collective_signature(b))
    for ranks in sorted(seqs):
        g, mine = handle[ranks], seqs[ranks]
        gathered: List = [None] * dist.get_world_size(g)
        dist.all_gather_object(gathered, mine, group=g)
        if any(x != mine for x in gathered):
            bad = [ranks[i] for i, x in enumerate(gathered) if x != mine]
            raise RuntimeError(f"[DION_SYNC_GROUP_ORDER_MISMATCH] group ranks={ranks}: ranks {bad} issue another "
                               f"batch order ({len(mine)} batches here)")

