"""The speedrun's FS x TP topology on the GPU (`pytest -m gpu`): four processes share cuda:0 and
form FS = 2 x TP = 2 over gloo; the Dion work is the product path (HIP kernels through the C
ABI), the batches come from the product adapter with split QKV children of the TP/FS-sharded
parent, fp32 and the speedrun's bf16 momentum and Q.  Checked against the reference's own
captures (tests/golden/make_golden_fstp.py) with the reference's seeded sketch slices.
Tolerance: max |a - b| / max |b| <= 1e-5; bf16 state: BF16_GPU_TOLS.
"""
import pytest
import torch

from tests.test_dist_gloo_fs import BF16_GPU_TOLS
from tests.test_dist_gloo_fstp import CASES, check_fstp_results, run_fstp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_hip_fs2tp2_speedrun_matches_reference(name, deferred):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = run_fstp(name, deferred=deferred, device="cuda:0")
    worst = check_fstp_results(res, name, deferred, 1e-5, bf16_tols=BF16_GPU_TOLS)
    print(f"{name} deferred={deferred}: worst {worst:.2e}")
