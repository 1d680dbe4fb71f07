"""`MegatronDion`: the optimizer Megatron's DistributedOptimizer selects, MI355X edition.

Mirrors /root/reference/megatron/core/optimizer/dion/algorithm.py:29-221:
same constructor keywords and `defaults` keys (:48-105), the same
`enable_distributed_mode(route_step_params=...)` hook (runtime.py:632-644) and
the same `step()` contract (:149-221): bump `param_group['step']` and
`_step_count`, ask the adapter for `(List[DionBatch], List[ElementwiseStepParam])`,
run the batches through a width-limited AsyncRuntime.  The per-batch work runs
in HIP kernels (`codec=` backend, default `HipDionCodec`); there is no CPU
fallback.

The elementwise branch (AdamW / Lion for the ElementwiseStepParam items,
algorithm.py:247-429) runs after the Dion batches in one multi-tensor HIP launch per
update contract.  The batch kinds are the reference's: whole-matrix data parallel ("ddp"),
FS-sharded ("fsdp") and TP-sharded ("fsdp_tp", FS on the contraction side when both are on: the
speedrun's topology), fp32 or bf16 momentum / Q (independent dtypes); split QKV / QKVG /
linear children of whole or sharded parents come from the stand-alone adapter
(`attach_dp_routing`, split.py) or from the reference's own adapter.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch.optim.optimizer import Optimizer

from .batches import build_dion_batches, verify_sync_group_order
from .runtime import (AsyncRuntime, DionStateMap, coalesce_local_batches, coalesce_replicated_batches,
                      drop_pending_error_feedback, flush_pending_error_feedback, is_replicated,
                      run_dion_batch_async)
from .split import child_uid, gather_rows, make_commit, split_child_layouts, split_plan, state_key
from .state import init_dion_state
from .types import DionDistMeta, DionMixedPrecisionConfig, DionStepParam, ElementwiseStepParam


class MegatronDion(Optimizer):
    def __init__(self, params, lr: float = 0.01, mu: float = 0.95, weight_decay: float = 0.01,
                 rank_fraction: float = 1.0, rank_multiple_of: int = 1, epsilon: float = 1e-8,
                 rcqr_oversample: float = 1.25, betas: tuple = (0.9, 0.95), elementwise_eps: float = 1e-8,
                 rp_average_in_collective: bool = True, use_fs_collectives: bool = True,
                 mixed_precision_config: Optional[DionMixedPrecisionConfig] = None, enable_async: bool = True,
                 use_low_rank_sync: bool = True, elementwise_optimizer: str = "adam",
                 elementwise_lr_scale: float = 1.0, scale_mode: str = "spectral",
                 extra_scale_factor: float = 0.2, split_qkv: bool = False, split_linear: bool = False,
                 max_concurrent_tasks: Optional[int] = None, *, codec=None, sketch_seed: int = 0,
                 coalesce_local: bool = True, local_streams: int = 2, coalesce_max_entries: int = 16,
                 defer_error_feedback: bool = True, pipeline_lookahead: int = 0):
        if isinstance(params, (list, tuple)):
            for pg in params:
                if isinstance(pg, dict) and "wd_mult" in pg:
                    pg["weight_decay"] = float(pg.get("weight_decay", weight_decay)) * float(pg.get("wd_mult", 1.0))
        if scale_mode not in ("spectral", "unit_rms_norm", "shape_scaling"):
            raise RuntimeError(f"[DION_INVALID_SCALE_MODE] got {scale_mode!r}")
        if float(elementwise_lr_scale) < 0.0:
            raise RuntimeError(f"[DION_INVALID_ELEMENTWISE_LR_SCALE] elementwise_lr_scale={elementwise_lr_scale}")
        defaults = dict(lr=lr, mu=mu, weight_decay=weight_decay, rank_fraction=rank_fraction,
                        rank_multiple_of=rank_multiple_of, epsilon=epsilon, rcqr_oversample=rcqr_oversample,
                        betas=betas, elementwise_eps=elementwise_eps,
                        rp_average_in_collective=rp_average_in_collective, use_fs_collectives=use_fs_collectives,
                        enable_async=enable_async, use_low_rank_sync=use_low_rank_sync,
                        elementwise_optimizer=elementwise_optimizer, elementwise_lr_scale=elementwise_lr_scale,
                        scale_mode=scale_mode, extra_scale_factor=extra_scale_factor, split_qkv=bool(split_qkv),
                        split_linear=bool(split_linear), algorithm="dion", step=0)
        super().__init__(params, defaults)
        # states apply a deferred error feedback before any read of the momentum from
        # outside the step (DionParamState), whoever creates or restores them
        self.state = DionStateMap(self, self.state)
        self._dion_in_step = False
        self._global_rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.is_distributed_mode = False
        self.use_fs_collectives = use_fs_collectives
        self.use_low_rank_sync = use_low_rank_sync
        self.enable_async = enable_async
        self.max_concurrent_tasks = max_concurrent_tasks
        self._mixed_precision_config = mixed_precision_config or DionMixedPrecisionConfig()
        self._route_step_params = None
        self._dion_update_count = 0
        self._elementwise_update_count = 0
        self._step_count = 0
        self._sketch_seed = int(sketch_seed)
        self._coalesce_local = bool(coalesce_local)
        self._local_streams = max(1, int(local_streams))
        self._coalesce_max = max(1, int(coalesce_max_entries))
        self._streams = None
        self._rstreams = None
        self._pstreams = None
        self._pipeline_lookahead = max(0, int(pipeline_lookahead))
        self._codec = codec
        self._defer_ef = bool(defer_error_feedback)
        self._profile_records: List[Tuple[str, float]] = []
        # algorithm.py:146: per-step scratch the reference's adapter clears on offload
        # (dion_distrib_optimizer.py:4284-4306 calls optimizer._buffer_cache.clear())
        self._buffer_cache: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ backend
    @property
    def codec(self):
        if self._codec is None:
            from .codec import HipDionCodec
            self._codec = HipDionCodec()
        return self._codec

    # ------------------------------------------------------------------ deferred error feedback
    @torch.no_grad()
    def flush_error_feedback(self) -> int:
        """Apply every deferred error feedback now, so `state[p]['momentum']` is the eager value.

        With `defer_error_feedback=True` the step-t update M += -(1-mu) P R^T is
        carried by the step-(t+1) pass A (dion_project_p_ef): same sums in the same
        order, one M read/write less per step.  Anything that reads the momentum
        between steps (checkpointing, inspection) calls this first; `state_dict()`
        does so itself."""
        return flush_pending_error_feedback(self, lambda: self.codec)

    def zero_grad(self, set_to_none: bool = True):
        """torch's zero_grad, plus: the gradients about to be repopulated invalidate the
        grad norm's dense-reduction marks (dense_grad_cache.invalidate), so a norm computed
        before a skipped step can never vouch for the next iteration's gradients."""
        from .dense_grad_cache import invalidate
        invalidate(self)
        return super().zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        self.flush_error_feedback()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """Drop every pending error feedback, then load.

        The loaded momentum is an eager value (state_dict() flushed it before saving), so a
        pending factor pair of the live run must not ride on it.  Megatron's Dion restore
        keeps the live state's underscore keys (distrib_dion/checkpoint_io.py:308) but calls
        this method first (distrib_optimizer.py:740 inside DionDistributedOptimizer.
        load_state_dict, dion_distrib_optimizer.py:4218-4260), so the pending key is gone by
        then."""
        drop_pending_error_feedback(self)
        out = super().load_state_dict(state_dict)
        self.state = DionStateMap(self, self.state)
        return out

    # ------------------------------------------------------------------ plugin surface
    def enable_distributed_mode(self, *, route_step_params=None) -> None:
        """runtime.py:632-644: install the adapter's routing callback."""
        if route_step_params is None:
            raise RuntimeError(f"[DION_MISSING_DIST_STEP_ITEMS_CALLBACK] step={self._step_count}")
        self.is_distributed_mode = True
        self._route_step_params = route_step_params

    def _batches(self):
        batches, elementwise = self._route_step_params()
        self._dion_update_count += sum(int(b.real_batch_size) for b in batches)
        self._elementwise_update_count += len(elementwise)
        if self._coalesce_local:
            batches = coalesce_local_batches(batches, max_entries=self._coalesce_max)
            batches = coalesce_replicated_batches(batches, max_entries=self._coalesce_max)
        return batches, list(elementwise)

    # ------------------------------------------------------------------ elementwise branch
    def _apply_elementwise_batches(self, elementwise_params) -> None:
        """algorithm.py:247-429: group the elementwise items by their update contract
        (algorithm, group, device, dtypes, lr, wd, eps, betas, step) in first-seen order and
        run one multi-tensor AdamW / Lion launch per group (elementwise_opts.py)."""
        default_opt = self.defaults.get("elementwise_optimizer", "adam")
        default_scale = float(self.defaults.get("elementwise_lr_scale", 1.0))
        default_betas = self.defaults.get("betas", (0.9, 0.95))
        default_eps = self.defaults.get("elementwise_eps", 1e-8)
        mpc = self._mixed_precision_config
        groups: "OrderedDict[tuple, dict]" = OrderedDict()
        for item in elementwise_params:
            p, grad, state, grp = item.param, item.grad, item.optimizer_state, item.optim_group
            algo = grp.get("algorithm", None)
            opt_name = grp.get("elementwise_optimizer", default_opt) if algo in (None, "dion") else algo
            if opt_name == "adam":
                opt_name = "adamw"
            if opt_name not in ("adamw", "lion"):
                raise RuntimeError(f"[DION_INVALID_ELEMENTWISE_OPT] elementwise_optimizer={opt_name}")
            lr_scale = float(grp.get("elementwise_lr_scale", default_scale))
            if lr_scale < 0.0:
                raise RuntimeError(f"[DION_INVALID_ELEMENTWISE_LR_SCALE] elementwise_lr_scale={lr_scale}")
            lr = float(grp.get("lr", self.defaults["lr"])) * lr_scale
            wd = float(grp.get("weight_decay", self.defaults["weight_decay"] * grp.get("wd_mult", 1.0)))
            step = int(grp.get("step", 0))
            eps = float(grp.get("elementwise_eps", grp.get("eps", grp.get("epsilon", default_eps))))
            if "betas" in grp:
                b1, b2 = (float(x) for x in grp["betas"])
            else:
                b1 = float(grp.get("beta1", default_betas[0]))
                b2 = float(grp.get("beta2", default_betas[1]))
            if step <= 0:
                raise RuntimeError(f"[DION_INVALID_ELEMENTWISE_STEP] step={step}")
            m1 = _elementwise_moment(state, p, "first_moment", ("exp_avg", "momentum"), mpc.momentum_dtype)
            state["step"] = step
            m2 = None
            if opt_name == "adamw":
                m2 = _elementwise_moment(state, p, "second_moment", ("exp_avg_sq", "variance"), mpc.variance_dtype)
            key = (opt_name, id(grp), str(p.device), str(p.dtype), str(m1.dtype),
                   str(m2.dtype if m2 is not None else torch.float32), lr, wd, eps, b1, b2, step)
            g = groups.setdefault(key, dict(opt=opt_name, params=[], grads=[], m1=[], m2=[], lr=lr, wd=wd,
                                            eps=eps, step=step, b1=b1, b2=b2))
            g["params"].append(p.data if isinstance(p, torch.nn.Parameter) else p)
            g["grads"].append(grad)
            g["m1"].append(m1)
            if m2 is not None:
                g["m2"].append(m2)
        codec = self.codec
        for g in groups.values():
            if g["opt"] == "lion":
                codec.elementwise_lion(g["params"], g["grads"], g["m1"], lr=g["lr"], beta1=g["b1"], beta2=g["b2"],
                                       weight_decay=g["wd"])
            else:
                codec.elementwise_adamw(g["params"], g["grads"], g["m1"], g["m2"], lr=g["lr"], beta1=g["b1"],
                                        beta2=g["b2"], weight_decay=g["wd"], step=g["step"], epsilon=g["eps"])

    def _run_local_overlapped(self, batches, sketches) -> bool:
        """World-size-1 schedule: independent batches alternate over HIP streams, so one
        batch's latency-bound orthonormalisation overlaps the next batch's streaming passes."""
        if self._local_streams <= 1 or not torch.cuda.is_available() or not batches:
            return False
        if any(is_replicated(b) for b in batches):
            return False
        if not all(getattr(b.params[0], "is_cuda", False) for b in batches):
            return False
        dev = batches[0].params[0].device
        if self._streams is None or self._streams[0].device != dev:
            self._streams = [torch.cuda.Stream(device=dev) for _ in range(self._local_streams)]
        main = torch.cuda.current_stream(dev)
        for s in self._streams:
            s.wait_stream(main)
        for b, si in self._stream_plan(batches):
            with torch.cuda.stream(self._streams[si]):
                for _ in run_dion_batch_async(self, b, sketches=sketches(b) if sketches else None):
                    raise RuntimeError("[DION_INTERNAL] a world-size-1 batch yielded")
        for s in self._streams:
            main.wait_stream(s)
        return True

    def _stream_plan(self, batches):
        """(batch, stream index) in issue order.  "rr": round robin in the reference's batch
        order.  "stagger": largest launch groups first, each to the stream with the least
        queued work (elements), except that stream 1 opens with the smallest group, so the
        streams' latency-bound orthonormalisations do not fall together."""
        n = len(self._streams)
        order = os.environ.get("DION_LOCAL_ORDER", "stagger")
        if order == "rr" or n < 2 or len(batches) < 3:
            return [(b, i % n) for i, b in enumerate(batches)]

        def work(b):
            m, k = b.params[0].shape[-2:]
            return int(b.real_batch_size) * int(m) * int(k)

        rest = sorted(range(len(batches)), key=lambda i: -work(batches[i]))
        first_small = rest.pop()  # the smallest group opens stream 1
        load = [0] * n
        plan = [(rest[0], 0), (first_small, 1)]
        load[0] += work(batches[rest[0]])
        load[1] += work(batches[first_small])
        for i in rest[1:]:
            si = min(range(n), key=lambda k: load[k])
            plan.append((i, si))
            load[si] += work(batches[i])
        return [(batches[i], si) for i, si in plan]

    def _run_local_pipelined(self, batches, sketches) -> bool:
        """World-size-1 schedule, software-pipelined over two HIP streams.

        Stream S runs every streaming pass (pass A, pass B, fix-up, the updates) one
        launch group after another; stream L runs each group's latency-bound
        orthonormalisation as soon as its pass A is done.  S enqueues group k's pass B
        only after the pass A of groups k+1 .. k+lookahead, so L's work always has
        streaming work beside it and the streaming kernels never share the memory
        system with each other.  Events carry the two hand-offs (A_k -> ortho_k on L,
        ortho_k -> B_k on S); per-group buffers live until the group's last kernel
        on S."""
        if self._local_streams <= 1 or self._pipeline_lookahead <= 0 or not torch.cuda.is_available() \
                or not batches:
            return False
        if any(is_replicated(b) for b in batches):
            return False
        if not all(getattr(b.params[0], "is_cuda", False) for b in batches):
            return False
        dev = batches[0].params[0].device
        ns = max(1, self._local_streams - 1)  # streaming streams; the last one is the latency stream
        if self._pstreams is None or len(self._pstreams) != ns + 1 or self._pstreams[0].device != dev:
            self._pstreams = [torch.cuda.Stream(device=dev) for _ in range(ns + 1)]
        Ss, L = self._pstreams[:ns], self._pstreams[ns]
        main = torch.cuda.current_stream(dev)
        for s in self._pstreams:
            s.wait_stream(main)

        def advance(gen, stream):
            with torch.cuda.stream(stream):
                try:
                    return next(gen)
                except StopIteration:
                    return None

        def finish(entry):
            g0, e0, s0 = entry
            s0.wait_event(e0)
            if advance(g0, s0) is not None:
                raise RuntimeError("[DION_INTERNAL] pipelined batch yielded after its phases")

        # group k streams on Ss[k % ns]; each streaming stream keeps `lookahead` groups' pass A
        # ahead of their pass B, so it never waits for its own group's orthonormalisation
        pending = [[] for _ in range(ns)]
        for k, b in enumerate(batches):
            S = Ss[k % ns]
            gen = run_dion_batch_async(self, b, sketches=sketches(b) if sketches else None, phase_marks=True)
            if advance(gen, S) != "ortho":
                continue
            ev = torch.cuda.Event()
            ev.record(S)
            L.wait_event(ev)
            if advance(gen, L) != "stream":
                raise RuntimeError("[DION_INTERNAL] pipelined batch lost its phase marks")
            done = torch.cuda.Event()
            done.record(L)
            q = pending[k % ns]
            q.append((gen, done, S))
            while len(q) > self._pipeline_lookahead:
                finish(q.pop(0))
        for q in pending:
            for entry in q:
                finish(entry)
        for s in self._pstreams:
            main.wait_stream(s)
        return True

    def _replica_streams(self, batches, width):
        """One HIP stream per AsyncRuntime slot for replicated (W > 1) batches on the GPU."""
        if self._local_streams <= 1 or not torch.cuda.is_available() or not batches:
            return None
        if not all(getattr(b.params[0], "is_cuda", False) for b in batches if b.params):
            return None
        dev = batches[0].params[0].device
        if self._rstreams is None or len(self._rstreams) != width or self._rstreams[0].device != dev:
            self._rstreams = [torch.cuda.Stream(device=dev) for _ in range(width)]
        return self._rstreams

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._dion_update_count = 0
        self._elementwise_update_count = 0
        for group in self.param_groups:
            group["step"] = group.get("step", 0) + 1
        self._step_count += 1
        if not self.is_distributed_mode:
            raise RuntimeError(f"[DION_STEP_REQUIRES_DISTRIBUTED_MODE] step={self._step_count}")
        profile = os.environ.get("DION_PROFILE_SPLIT", "").lower() in ("1", "true", "yes")
        self._profile_enabled = profile
        self._phase_records = [] if profile else None
        if profile and torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter() if profile else None
        self._dion_in_step = True
        try:
            self._step_batches(profile, t0)
        except BaseException:
            self._phase_records = None  # a failed step reports nothing (its events may never complete)
            raise
        finally:
            self._dion_in_step = False
        if profile:
            self._report_profile(t0)
        return loss

    # phases the fused kernels fold into another phase's record (PhaseClock)
    _FUSED_PHASES = {"grad_momentum": "p_matmul", "error_feedback": "apply_update or the next p_matmul",
                     "q_normalize": "ortho_r"}

    def _report_profile(self, t0) -> None:
        """algorithm.py:170-218 with HIP-event phase times: one synchronise, then the per-label sums
        (the reference's [DION_PROFILE] line) and the slowest batches ([DION_PROFILE_BATCH]).
        Phase times of batches on concurrent streams overlap, so their sum can exceed `total`."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        from .runtime import phase_seconds
        self._profile_records = [(label, phase_seconds(a, b), desc) for label, a, b, desc in
                                 (self._phase_records or [])]
        self._phase_records = None
        if self._global_rank != 0:
            return
        by_label, by_desc = OrderedDict(), {}
        for label in ("grad_momentum", "q_unshard", "p_matmul", "p_reduce", "ortho_r", "error_feedback",
                      "q_normalize", "apply_update"):
            by_label[label] = 0.0
        for label, sec, desc in self._profile_records:
            by_label[label] = by_label.get(label, 0.0) + sec
            by_desc[desc] = by_desc.get(desc, 0.0) + sec
        summary = ", ".join(f"{k}={v:.3f}s" + (f" (fused: {self._FUSED_PHASES[k]})" if k in self._FUSED_PHASES and
                                              v == 0.0 else "") for k, v in by_label.items())
        print(f"[DION_PROFILE] step={self._step_count} total={elapsed:.3f}s {summary}", flush=True)
        for desc, sec in sorted(by_desc.items(), key=lambda kv: kv[1], reverse=True)[:12]:
            print(f"[DION_PROFILE_BATCH] step={self._step_count} time={sec:.3f}s {desc}", flush=True)

    def _step_batches(self, profile, t0):
        width = 3 if self.max_concurrent_tasks is None else int(self.max_concurrent_tasks)
        sketches = getattr(self, "_sketch_override", None)
        batches, elementwise = self._batches()
        if not (self._run_local_pipelined(batches, sketches) or self._run_local_overlapped(batches, sketches)):
            streams = self._replica_streams(batches, width)
            main = torch.cuda.current_stream(streams[0].device) if streams else None
            for s in streams or ():
                s.wait_stream(main)
            AsyncRuntime((run_dion_batch_async(self, b, sketches=sketches(b) if sketches else None)
                          for b in batches), width, streams=streams).run()
            for s in streams or ():
                main.wait_stream(s)
        if elementwise:
            # runtime.py:314-315: the elementwise task runs after the Dion batches
            self._apply_elementwise_batches(elementwise)
        self._buffer_cache.clear()  # algorithm.py:219


def _elementwise_moment(state, param, key, legacy, dtype):
    """algorithm.py:295-331: the moment under `key`, migrated from a legacy key or zero-initialised."""
    if key in state and legacy[0] in state:
        raise RuntimeError(f"[DION_SCALAR_STATE_LAYOUT_CONFLICT] found both {key} and {legacy[0]}")
    if key not in state:
        for old in legacy:
            if old in state:
                state[key] = state.pop(old)
                break
        else:
            state[key] = torch.zeros_like(param, dtype=_as_dtype(dtype) or param.dtype)
    return state[key]


def _as_dtype(d):
    """DionMixedPrecisionConfig fields may be torch dtypes or their names (state.py str_to_dtype)."""
    if d is None or isinstance(d, torch.dtype):
        return d
    name = str(d).replace("torch.", "")
    return {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float32": torch.float32,
            "fp32": torch.float32, "float": torch.float32}[name]


# ---------------------------------------------------------------------------- standalone routing
def is_dion_param(param: torch.Tensor, name: str = "") -> bool:
    """distrib_dion/parameter.py:34-57 for a stand-alone model: 2D, not opted out
    (`use_dion=False`), not sequence-parallel, not an embedding / output / LM-head table.
    Everything else takes the elementwise branch (bootstrap.py:565-576)."""
    if getattr(param, "use_dion", None) is False or param.dim() != 2:
        return False
    for flag in ("sequence_parallel", "average_gradients_across_tp_domain", "is_embedding_or_output_parameter",
                 "is_lm_head_parameter"):
        if getattr(param, flag, False):
            return False
    return not any(k in name for k in ("embedding", "output_layer", "lm_head"))


# owner groups of split children, by global ranks; valid for one default process group only
_CHILD_ROW_GROUPS: Dict[Tuple[int, ...], object] = {}
_CHILD_ROW_GROUPS_WORLD: List[object] = [None]


def _child_group_cache() -> Dict[Tuple[int, ...], object]:
    """The owner-group cache of the current default process group.  After
    destroy_process_group() and a new init_process_group() the cached handles belong to the
    destroyed world, and a rank that still held them would skip the new_group calls its peers
    make (unmatched collective group creation): a new WORLD starts an empty cache."""
    world = dist.group.WORLD if dist.is_initialized() else None
    if _CHILD_ROW_GROUPS_WORLD[0] is not world:
        _CHILD_ROW_GROUPS.clear()
        _CHILD_ROW_GROUPS_WORLD[0] = world
    return _CHILD_ROW_GROUPS


def _child_ranks(parent_group, members: Sequence[int]) -> Tuple[int, ...]:
    ranks = tuple(int(r) for r in dist.get_process_group_ranks(parent_group))
    return tuple(ranks[k] for k in members)


def _prepare_child_row_groups(needed: Sequence[Tuple[int, ...]]) -> None:
    """Create every split child's owner group on every rank, in one order (row_child.py:94-101,
    dion_distrib_optimizer.py:260-284 _ensure_child_group).  The ranks of the job exchange the
    owner sets they need (another FS group's children have other global ranks) and all create
    the union, sorted, so each new_group call is matched on every rank; the reference's
    group-local creation is not used because gloo's group-local rendezvous does not line up when
    ranks create different groups."""
    want = sorted(set(tuple(int(r) for r in t) for t in needed))
    if dist.get_world_size() > 1:
        every = [None] * dist.get_world_size()
        dist.all_gather_object(every, want)
        want = sorted(set(t for lst in every for t in lst))
    cache = _child_group_cache()
    for ranks in want:
        if ranks not in cache:
            cache[ranks] = dist.new_group(list(ranks))


def _child_row_group(parent_group, members: Sequence[int]):
    """The prepared process group of a split child's owners; one owner needs none."""
    child = _child_ranks(parent_group, members)
    if len(child) <= 1:
        return None
    cache = _child_group_cache()
    if child not in cache:
        raise RuntimeError(f"[DION_SPLIT_CHILD_GROUP_NOT_PREPARED] ranks={child}")
    return cache[child]


def _row_axis_group(spec, tspec, fs_group, tp_group, fs_world: int, tp_world: int):
    """The group a split parent's rows are sharded over (TP on dim 0, else FS on dim 0)."""
    if tspec is not None and int(tspec[1]) == 0 and tp_world > 1:
        return tp_group
    if spec is not None and int(spec[1]) == 0 and fs_world > 1:
        return fs_group
    return None


def attach_dp_routing(optimizer: MegatronDion, named_params: Sequence[Tuple[str, torch.Tensor]],
                      replicate_group=None, base_seed: int = 0, dion_predicate=None, fs_group=None,
                      fs_shards: Optional[Dict[str, tuple]] = None, tp_group=None,
                      tp_shards: Optional[Dict[str, tuple]] = None,
                      q_stream: str = "device") -> Dict[str, torch.Tensor]:
    """Stand-alone adapter: state init + `route_step_params` for plain data parallelism.

    `q_stream`: "device" draws each Q0 on the parameter's device exactly as the reference
    does there (per-row Philox offsets, state.init_q: two small launches per Q row); "cpu"
    draws the reference's CPU stream and copies it over (the values a CPU run gets; the
    benchmark uses it to keep its startup and profiler traces free of ~10^5 init launches).

    Plays the part of the reference's DionDistributedOptimizer routing
    (distrib_dion/bootstrap.py:519-606 -> batches.py:971 build_dion_batches) for
    users outside Megatron and for the benchmark: 2D Dion params (`dion_predicate`,
    default `is_dion_param`) sorted by uid, one batch per `batch_world_size` same-key
    matrices; every other param with a gradient becomes an ElementwiseStepParam
    (AdamW / Lion).  As in Megatron, elementwise gradients arrive already reduced across
    replicas (only Dion buckets skip the replica all-reduce,
    param_and_grad_buffer.py:649-698).  G of each step is taken from `param.main_grad` (Megatron's grad
    buffer view, bf16 or fp32) when present, else from `param.grad`.

    FS sharding (the reference's default topology, FS = DP): `fs_shards[name] =
    (global_shape, fs_shard_dim, start, end)` marks `param` as this rank's shard of a matrix
    sharded over `fs_group` (distrib_dion/parameter.py:424-466); those params form "fsdp"
    batches of FS-world entries.

    TP sharding: `tp_shards[name] = (global_shape, tp_shard_dim, start, end)` marks `param` as
    this rank's TP shard over `tp_group` (rows for dim 0, columns for dim 1); Q then holds this
    rank's columns of r and those params form "fsdp_tp" batches of TP-world entries.
    """
    group = optimizer.param_groups[0]
    rf = float(group.get("rank_fraction", optimizer.defaults["rank_fraction"]))
    mult = int(optimizer.defaults.get("rank_multiple_of", 1))
    pred = dion_predicate or is_dion_param
    metas = {}
    # shard param -> its DionDistMeta, where the reference's helpers look it up
    # (distrib_dion/grad_norm.py:27-34; split parents stay out: their children are the Dion params)
    dist_metas = optimizer.__dict__.setdefault("dist_metas", {})
    group_of = {id(p): g for g in optimizer.param_groups for p in g["params"]}
    dion_named, ew_named = [], []
    # split children owned by part of their parent's row group need owner groups, created on every
    # rank before any state (row_child.py:94-101); all ranks hold the same split parents, so they
    # agree on whether to exchange
    layouts, needed, sharded_split = {}, [], False
    for name, p in named_params:
        spec, tspec = (fs_shards or {}).get(name), (tp_shards or {}).get(name)
        if not pred(p, name) or (spec is None and tspec is None):
            continue
        plan = split_plan(p, optimizer.defaults, global_rows=int((tspec or spec)[0][0]))
        if plan is None:
            continue
        if tspec is not None and tp_group is None:
            raise RuntimeError(f"[DION_MISSING_BATCH_TP_GROUP] {name}: tp_shards given without tp_group")
        fs_world = int(dist.get_world_size(fs_group)) if (spec is not None and fs_group is not None) else 1
        tp_world = int(dist.get_world_size(tp_group)) if tspec is not None else 1
        tp_rank = int(dist.get_rank(tp_group)) if tspec is not None else 0
        layout = split_child_layouts(p, plan, fs_spec=spec, tp_spec=tspec, fs_world=fs_world,
                                     fs_rank=int(dist.get_rank(fs_group)) if fs_world > 1 else 0,
                                     tp_world=tp_world, tp_rank=tp_rank)
        row_group = _row_axis_group(spec, tspec, fs_group, tp_group, fs_world, tp_world)
        layouts[name] = layout
        if row_group is not None:
            sharded_split = True
            size = int(dist.get_world_size(row_group))
            needed += [_child_ranks(row_group, lay["members"]) for lay in layout.values()
                       if 1 < len(lay["members"]) < size]
    if sharded_split:
        _prepare_child_row_groups(needed)
    for name, p in named_params:
        if not pred(p, name):
            ew_named.append((name, p))
            continue
        dion_named.append((name, p))
        mpc = optimizer._mixed_precision_config
        spec = (fs_shards or {}).get(name)
        fs_world = int(dist.get_world_size(fs_group)) if (spec is not None and fs_group is not None) else 1
        tspec = (tp_shards or {}).get(name)
        if tspec is not None and tp_group is None:
            raise RuntimeError(f"[DION_MISSING_BATCH_TP_GROUP] {name}: tp_shards given without tp_group")
        plan = split_plan(p, optimizer.defaults, global_rows=None if (spec is None and tspec is None)
                          else int((tspec or spec)[0][0]))
        if plan is not None:
            family, kinds, _, flags = plan
            pstate = optimizer.state[p]
            pstate.update(flags)
            pstate["momentum"] = torch.zeros_like(p, dtype=_as_dtype(getattr(mpc, "momentum_dtype", None)) or p.dtype)
            tp_world = int(dist.get_world_size(tp_group)) if tspec is not None else 1
            tp_rank = int(dist.get_rank(tp_group)) if tspec is not None else 0
            layout = layouts.get(name) or split_child_layouts(p, plan, fs_spec=spec, tp_spec=tspec)
            row_axis_group = _row_axis_group(spec, tspec, fs_group, tp_group, fs_world, tp_world)
            for kind in kinds:
                lay = layout[kind]
                c_fs_group, c_fs_world, c_tp_group, c_tp_world, c_tp_rank = fs_group, fs_world, tp_group, tp_world, tp_rank
                if row_axis_group is not None and len(lay["members"]) < dist.get_world_size(row_axis_group):
                    # owners short of the whole row group: the child's own owner group
                    sub = _child_row_group(row_axis_group, lay["members"])
                    if row_axis_group is tp_group and tspec is not None and int(tspec[1]) == 0:
                        c_tp_group, c_tp_world, c_tp_rank = sub, lay["child_world"], max(lay["child_rank"], 0)
                    else:
                        c_fs_group, c_fs_world = sub, lay["child_world"]
                if lay["child_rank"] < 0:
                    metas[(name, kind)] = None  # no rows of this child here (row_child.py:105-106)
                    continue
                rows = lay["local_rows"]
                cname = f"{name}::{kind}"
                cuid = child_uid((name,), family, kind)
                cstate, ccfg = init_dion_state(p.narrow(0, 0, rows), rank_fraction=rf, rank_multiple_of=mult,
                                               base_seed=base_seed, param_uid=cuid, param_name=cname,
                                               q_dtype=_as_dtype(getattr(mpc, "q_dtype", None)),
                                               use_low_rank_sync=optimizer.use_low_rank_sync, with_momentum=False,
                                               fs_shard=None if lay["fs"] is None else (*lay["fs"], c_fs_world),
                                               tp_shard=None if lay["tp"] is None else (*lay["tp"], c_tp_world,
                                                                                        c_tp_rank),
                                               q_stream=q_stream)
                for field in ("Q", "r", "local_shape", "global_shape"):
                    pstate[state_key(family, field, kind)] = cstate[field]
                cmeta = DionDistMeta(shape=(rows, int(p.shape[1])), global_shape=tuple(cstate["global_shape"]),
                                     rank_fraction=rf, is_transposed=ccfg.is_transposed, param_uid=cuid,
                                     is_dion_param=True, param_name=cname, param_config=ccfg,
                                     local_shape=(rows, int(p.shape[1])),
                                     tensor_row_shard_sizes=lay["row_sizes"],
                                     row_shard_sizes=lay["row_sizes"] if lay["row_axis"] == "tp" else None)
                if lay["fs"] is not None:
                    cmeta.extra.update(fs_group=c_fs_group, fs_shard_dim=int(lay["fs"][1]),
                                       fs_start_idx=int(lay["fs"][2]), fs_end_idx=int(lay["fs"][3]),
                                       fs_world_size=c_fs_world)
                if lay["tp"] is not None:
                    cmeta.extra.update(tp_group=c_tp_group, tp_shard_dim=int(lay["tp"][1]),
                                       tp_start_idx=int(lay["tp"][2]), tp_end_idx=int(lay["tp"][3]),
                                       tp_world_size=c_tp_world)
                metas[(name, kind)] = (ccfg, cmeta, lay["segments"])
            metas[name] = (None, plan)
            continue
        state, cfg = init_dion_state(p, rank_fraction=rf, rank_multiple_of=mult, base_seed=base_seed,
                                     param_uid=(name,), param_name=name,
                                     momentum_dtype=_as_dtype(getattr(mpc, "momentum_dtype", None)),
                                     q_dtype=_as_dtype(getattr(mpc, "q_dtype", None)),
                                     use_low_rank_sync=optimizer.use_low_rank_sync,
                                     fs_shard=None if spec is None else (tuple(spec[0]), spec[1], spec[2], spec[3],
                                                                         fs_world),
                                     tp_shard=None if tspec is None else (tuple(tspec[0]), tspec[1], tspec[2], tspec[3],
                                                                          int(dist.get_world_size(tp_group)),
                                                                          int(dist.get_rank(tp_group))),
                                     q_stream=q_stream)
        optimizer.state[p].update(state)
        meta = DionDistMeta(shape=tuple(p.shape), global_shape=tuple(state["global_shape"]), rank_fraction=rf,
                            is_transposed=cfg.is_transposed, param_uid=(name,), is_dion_param=True,
                            param_name=name, param_config=cfg, local_shape=tuple(p.shape))
        if spec is not None:
            meta.extra.update(fs_group=fs_group, fs_shard_dim=int(spec[1]), fs_start_idx=int(spec[2]),
                              fs_end_idx=int(spec[3]), fs_world_size=fs_world)
        if tspec is not None:
            meta.extra.update(tp_group=tp_group, tp_shard_dim=int(tspec[1]), tp_start_idx=int(tspec[2]),
                              tp_end_idx=int(tspec[3]), tp_world_size=int(dist.get_world_size(tp_group)))
        metas[name] = (cfg, meta)
        dist_metas[p] = meta
    ordered = sorted(dion_named, key=lambda kv: kv[0])

    def grad_of(p):
        g = getattr(p, "main_grad", None)
        return p.grad if g is None else g

    checked = [False]

    def route():
        steps = []
        for name, p in ordered:
            g = grad_of(p)
            if g is None:
                continue
            cfg, meta = metas[name]
            if cfg is None:  # a split parent: one step param per child (split.py)
                family, kinds, _, _ = meta
                pstate = optimizer.state[p]
                M = dict.__getitem__(pstate, "momentum")
                for kind in kinds:
                    if metas[(name, kind)] is None:
                        continue
                    ccfg, cmeta, segs = metas[(name, kind)]
                    cstate = {"momentum": gather_rows(M, segs)}
                    for field in ("Q", "r", "local_shape", "global_shape"):
                        cstate[field] = pstate[state_key(family, field, kind)]
                    steps.append(DionStepParam(param=gather_rows(p.data, segs), grad=gather_rows(g, segs),
                                               optimizer_state=cstate, optim_group=group_of.get(id(p), group),
                                               config=ccfg, dist_meta=cmeta,
                                               commit_update=make_commit(p, M, segs)))
                continue
            steps.append(DionStepParam(param=p, grad=g, optimizer_state=optimizer.state[p],
                                       optim_group=group_of.get(id(p), group), config=cfg, dist_meta=meta))
        batches = build_dion_batches(
            dion_params=steps, get_replicate_group=lambda: replicate_group,
            group_size=lambda g: dist.get_world_size(g),
            resolve_fs_group_from_meta=lambda meta, expect_group=True: meta.extra.get("fs_group"),
            resolve_tp_group=lambda meta, expect_group=True: meta.extra.get("tp_group"))
        if not checked[0]:
            # once: the members of every sync group issue its collectives in one order
            verify_sync_group_order(batches)
            checked[0] = True
        elementwise = []
        for _, p in ew_named:
            g = grad_of(p)
            if g is not None:
                elementwise.append(ElementwiseStepParam(param=p, grad=g, optimizer_state=optimizer.state[p],
                                                        optim_group=group_of.get(id(p), group)))
        return batches, elementwise

    optimizer.enable_distributed_mode(route_step_params=route)
    return {name: p for name, p in named_params}
