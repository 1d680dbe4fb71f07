"""MI355X-native Dion gradient codec (import as `megatron_dion_amd`).

Drop-in for the data-parallel Dion hot path of krafton-ai/Megatron-Dion
(/root/reference/megatron/core/optimizer/dion/runtime.py:1499-1911): the device
work runs in hand-written HIP kernels for gfx950 (csrc/dion_codec.hip, C ABI in
include/dion_codec.h); the host side mirrors the reference's optimizer and
batch interfaces.
"""
from .types import (  # noqa: F401
    DionBatch,
    DionBatchCollectives,
    DionBatchEntry,
    DionBatchGroup,
    DionDistMeta,
    DionMixedPrecisionConfig,
    DionParamConfig,
    DionStepParam,
    ElementwiseStepParam,
)
from .state import (  # noqa: F401
    init_dion_state,
    is_transposed_shape,
    q_seed_from_param_key,
    rank_for_shape,
    should_use_low_rank_sync,
)
from .kernels import scaled_lr_for_shape  # noqa: F401
from .batches import build_dion_batches  # noqa: F401
from .runtime import AsyncRuntime, batch_dion_update_async  # noqa: F401
from .optimizer import MegatronDion  # noqa: F401
from .grad_norm import dion_grad_norm, dion_grad_norm_sq  # noqa: F401

__all__ = [
    "MegatronDion",
    "DionBatch",
    "DionBatchEntry",
    "DionBatchGroup",
    "DionBatchCollectives",
    "DionDistMeta",
    "DionMixedPrecisionConfig",
    "DionParamConfig",
    "DionStepParam",
    "ElementwiseStepParam",
    "build_dion_batches",
    "batch_dion_update_async",
    "AsyncRuntime",
    "scaled_lr_for_shape",
    "rank_for_shape",
    "should_use_low_rank_sync",
    "is_transposed_shape",
    "q_seed_from_param_key",
    "init_dion_state",
    "dion_grad_norm_sq",
    "dion_grad_norm",
]
