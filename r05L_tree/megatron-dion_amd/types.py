"""Data contracts of the Dion batch interface.

Field names follow the reference's contracts
(/root/reference/megatron/core/optimizer/dion/types.py:9-252) so that objects
built by the reference's Megatron adapter (`route_step_params()` ->
`(List[DionBatch], List[ElementwiseStepParam])`, runtime.py:294-315) are
accepted unchanged; the runtime reads them duck-typed (getattr with defaults),
so either these classes or the reference's own can be passed.  Only the fields
the data-parallel (replicate) path reads are modelled here; FS/TP/split-child
metadata is carried through untouched (`extra`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch


@dataclass
class DionMixedPrecisionConfig:
    """State dtypes (None: the parameter's dtype).  types.py:9-19."""
    momentum_dtype: Optional[torch.dtype] = None
    q_dtype: Optional[torch.dtype] = None
    variance_dtype: Optional[torch.dtype] = None


@dataclass
class DionParamConfig:
    """Per-matrix configuration.  types.py:21-32.

    `is_transposed` is the orientation rule (m < n, state.py:304-310);
    `use_low_rank_sync` selects the compressed replica exchange.
    """
    fs_shard_dim: Optional[int] = None
    tp_shard_dim: Optional[int] = None
    has_fs_shard: bool = False
    use_fs_shard: bool = False
    has_tp_shard: bool = False
    use_tp_shard: bool = False
    is_transposed: bool = False
    use_low_rank_sync: bool = False


@dataclass
class DionDistMeta:
    """The metadata the DP path reads (types.py:94-135 has the full FS/TP set)."""
    shape: Optional[Tuple[int, ...]] = None
    global_shape: Optional[Tuple[int, int]] = None
    rank_fraction: float = 0.25
    is_transposed: bool = False
    param_uid: Optional[Tuple] = None
    is_dion_param: bool = False
    param_name: str = ""
    param_config: Optional[DionParamConfig] = None
    per_expert_global_shape: Optional[Tuple[int, int]] = None
    local_shape: Optional[Tuple[int, int]] = None
    # uneven row layouts of split children of row-sharded parents (split_child.py:10-52):
    # every member's rows of the sharded side; row_shard_sizes when they shard P's rows
    tensor_row_shard_sizes: Optional[Tuple[int, ...]] = None
    row_shard_sizes: Optional[Tuple[int, ...]] = None
    extra: Dict[str, Any] = field(default_factory=dict)


@dataclass
class ElementwiseStepParam:
    """A non-2D parameter routed to the scalar optimizer (types.py:35-42); not on this path."""
    param: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None
    optimizer_state: Optional[dict] = None
    optim_group: Optional[dict] = None


@dataclass
class DionStepParam:
    """One routed Dion parameter (types.py:45-56)."""
    param: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None
    optimizer_state: Optional[dict] = None
    optim_group: Optional[dict] = None
    config: Optional[DionParamConfig] = None
    dist_meta: Any = None
    post_q_sync: Optional[Callable[[], None]] = None
    commit_update: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None


@dataclass
class DionBatchEntry:
    """One entry of a batch (types.py:59-72); padded entries carry zero grad/momentum/Q."""
    param: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None
    optimizer_state: Optional[dict] = None
    optim_group: Optional[dict] = None
    config: Optional[DionParamConfig] = None
    dist_meta: Any = None
    momentum: Optional[torch.Tensor] = None
    q_tensor: Optional[torch.Tensor] = None
    param_shape: Tuple[int, ...] = ()
    commit_update: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None


@dataclass
class DionBatchGroup:
    """Execution groups of a batch (types.py:75-92).

    `replicate_group` is the RP (inter distributed-optimizer instance) group
    whose ranks exchange P/R; `batch_world_size` is the batch size it implies.
    """
    kernel_kind: str = "ddp"
    replicate_group: Any = None
    ortho_group: Any = None
    q_norm_group: Any = None
    low_rank_replicate_group: Any = None
    batch_world_size: int = 1
    sync_groups: Tuple[Any, ...] = ()


@dataclass
class DionAxisCollective:
    """One grouped FS/TP collective over a shared axis (types.py:140-147): the process group,
    its size, this rank's index in it, and the batch entries it covers."""
    indices: Tuple[int, ...] = ()
    process_group: Any = None
    world_size: int = 1
    rank: int = 0


@dataclass
class DionBatchCollectives:
    """TP/FS collectives of a batch (types.py:149-158); empty on the pure DP path."""
    tp_q_gathers: Tuple[Any, ...] = ()
    fs_p_collectives: Tuple[Any, ...] = ()
    tp_r_collectives: Tuple[Any, ...] = ()
    tp_q_reshards: Tuple[Any, ...] = ()
    fs_collective: Any = None


@dataclass
class DionBatch:
    """A ready batch of same-shape matrices (types.py:161-226)."""
    batch_key: tuple = ()
    entries: Tuple[DionBatchEntry, ...] = ()
    real_batch_size: int = 0
    batch_cache_key: int = 0
    batch_group: Optional[DionBatchGroup] = None
    batch_collectives: Optional[DionBatchCollectives] = None

    def _col(self, name):
        return tuple(getattr(e, name) for e in self.entries)

    params = property(lambda self: self._col("param"))
    grads = property(lambda self: self._col("grad"))
    momentums = property(lambda self: self._col("momentum"))
    q_tensors = property(lambda self: self._col("q_tensor"))
    configs = property(lambda self: self._col("config"))
    dist_metas = property(lambda self: self._col("dist_meta"))
    optim_groups = property(lambda self: self._col("optim_group"))
    optimizer_states = property(lambda self: self._col("optimizer_state"))
    param_shapes = property(lambda self: self._col("param_shape"))


def batch_columns(batch) -> Dict[str, List]:
    """Unpack any DionBatch-like object (ours or the reference's) into lists."""
    names = ("params", "grads", "momentums", "q_tensors", "configs", "dist_metas", "optim_groups",
             "optimizer_states", "param_shapes")
    return {n: list(getattr(batch, n) or []) for n in names}
