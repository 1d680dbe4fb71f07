"""GPU parity of the elementwise AdamW / Lion kernel (`pytest -m gpu`) against the
reference's golden vectors (tests/golden/make_golden_elementwise.py).

The kernel performs the reference's foreach chain per element in fp32, in the same
order and with torch's lerp formula; it differs from the captured CPU results only
where a CPU library routine (sqrt, division) rounds differently from the GPU's
correctly rounded ones.  Bar: max |a - b| / max |b| <= 1e-6 for W and the moments
(observed: printed).  With a bf16 moment (the speedrun's mixed precision, or a bf16
first or second moment beside an fp32 one: cases e6 / e7) such a
difference can flip one bf16 rounding: moments <= 2^-7 (one ulp of the largest
element), W <= 2e-3 (one flipped bf16 update is about 1e-3 of max |W| here).
"""
import pytest
import torch

from tests.test_elementwise import _cases, _maxrel, run_through_optimizer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", _cases())
def test_hip_elementwise_matches_reference(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tests.test_elementwise import _load
    case = _load(name)[1]
    bf16 = "bfloat16" in (case.get("state_dtype"), case.get("variance_dtype"))
    worst = 0.0
    for step, n, k, ours, ref in run_through_optimizer(name, torch.device("cuda", 0)):
        err = _maxrel(ours, ref)
        worst = max(worst, err)
        tol = (2e-3 if k == "W" else 2 ** -7) if bf16 else 1e-6
        assert err <= tol, (name, step, n, k, err)
    print(name, "worst maxrel", worst)


def test_hip_elementwise_llama_embedding_size():
    """One Llama-3-8B embedding-sized tensor (128256 x 4096, fp32 moments, bf16 grad) against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import megatron_dion_amd as mda
    from oracle import dion_oracle as O
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    shape = (128256 // 8, 4096)  # an eighth of the table keeps the CPU oracle quick
    W = torch.randn(shape) * 0.02
    G = (torch.randn(shape) * 1e-2).to(torch.bfloat16)
    m1, m2 = torch.randn(shape) * 1e-3, torch.rand(shape) * 1e-5
    Wd, Gd, m1d, m2d = W.to(dev), G.to(dev), m1.to(dev), m2.to(dev)
    codec = mda.MegatronDion([torch.nn.Parameter(torch.zeros(2, 2, device=dev))]).codec
    codec.elementwise_adamw([Wd], [Gd], [m1d], [m2d], lr=3e-4, beta1=0.9, beta2=0.95, weight_decay=0.1, step=7,
                            epsilon=1e-8)
    torch.cuda.synchronize()
    O.elementwise_adamw([W], [G], [m1], [m2], lr=3e-4, beta1=0.9, beta2=0.95, weight_decay=0.1, step=7,
                        epsilon=1e-8)
    for ours, ref in ((Wd, W), (m1d, m1), (m2d, m2)):
        assert _maxrel(ours, ref) <= 1e-6
