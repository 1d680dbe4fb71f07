"""Dev: the cause of the flipped Q column in
test_bf16_matches_oracle_three_steps[wide_T_bf16G] (round 5, call L: Q 1.55 raw at step 2).
Runs the test's case (bf16 state, two 384 x 1024 matrices, r = 64, explicit sketches) with every
orthonormalize call recorded on both sides -- the HIP codec through the optimizer, the oracle's
orthogonalize through dion_batch_step_local -- and prints per call the input difference, the
flipped columns of the output and, for each flipped column, the sketch-QR Householder pivot
|alpha_j| / ||x_j|| (LAPACK's sign rule: a column's sign is -sign(alpha_j), so a pivot within
rounding of zero lets two correct implementations disagree).  Writes the record as JSON to argv[1]."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

import megatron_dion_amd as mda  # noqa: E402
from megatron_dion_amd.optimizer import attach_dp_routing  # noqa: E402
from oracle import dion_oracle as O  # noqa: E402
from tests.test_gpu_bf16 import BF16, CASES, _seeded  # noqa: E402


def pivots(sk, pin):
    """|alpha_j| / ||x_j|| of the Householder QR of S P (fp64), every column."""
    A = sk.double().reshape(-1, sk.shape[-1]) @ pin.double().reshape(pin.shape[-2], -1)
    out = []
    for j in range(A.shape[1]):
        x = A[j:, j].clone()
        out.append(abs(x[0].item()) / max(x.norm().item(), 1e-300))
        v = x.clone()
        v[0] -= -math.copysign(x.norm().item(), x[0].item())
        v = v / v.norm()
        A[j:, :] -= 2 * torch.outer(v, v @ A[j:, :])
    return out


def pivot_signs(sk, pin):
    """sign(alpha_j) of the Householder QR of S P (fp64), every column."""
    A = sk.double().reshape(-1, sk.shape[-1]) @ pin.double().reshape(pin.shape[-2], -1)
    out = []
    for j in range(A.shape[1]):
        x = A[j:, j].clone()
        out.append(1 if x[0].item() >= 0 else -1)
        v = x.clone()
        v[0] -= -math.copysign(x.norm().item(), x[0].item())
        v = v / v.norm()
        A[j:, :] -= 2 * torch.outer(v, v @ A[j:, :])
    return out


def main(out_path):
    dev = torch.device("cuda", 0)
    label, shapes, r, gdt, zero = next(c for c in CASES if c[0] == "wide_T_bf16G")
    mats = _seeded(shapes, r, 11, gdt, zero)
    hyper = O.DionHyper(rank_fraction=r / min(shapes[0]))
    names = [f"w{i}" for i in range(len(mats))]
    params = {n: torch.nn.Parameter(W.to(dev)) for n, (W, _, _) in zip(names, mats)}
    opt = mda.MegatronDion([params[n] for n in names], lr=hyper.lr, mu=hyper.mu, weight_decay=hyper.weight_decay,
                           rank_fraction=hyper.rank_fraction, epsilon=hyper.epsilon, coalesce_local=False,
                           mixed_precision_config=BF16)
    attach_dp_routing(opt, [(n, params[n]) for n in names])
    hip_calls, ora_calls = [], []
    codec = opt.codec
    orig = codec.orthonormalize

    def hooked(P, m, n, transposed, seed, oversample=1.25, sketch=None, **kw):
        pin = P.detach().cpu().clone()
        orig(P, m, n, transposed, seed, oversample, sketch=sketch, **kw)
        torch.cuda.synchronize()
        hip_calls.append((pin, P.detach().cpu().clone()))
    codec.orthonormalize = hooked
    o_orth = O.orthogonalize

    def o_hooked(P, oversample=1.25, sketch=None, generator=None):
        out = o_orth(P, oversample, sketch=sketch, generator=generator)
        ora_calls.append((P.detach().clone(), sketch.detach().clone(), out.detach().clone()))
        return out
    O.orthogonalize = o_hooked
    cpu = {}
    for n, (W, Q, _) in zip(names, mats):
        st = opt.state[params[n]]
        st["Q"].copy_(Q.to(dev))
        m, k = W.shape
        cpu[n] = O.DionMatrix(W=W.clone(), M=torch.zeros(m, k, dtype=torch.bfloat16), Q=Q.clone(), G=None,
                              transposed=m < k, rank_fraction=hyper.rank_fraction)
    name_of = {id(params[n]): n for n in names}
    kk = O.sketch_rows(r, hyper.rcqr_oversample)
    rec = []
    for step in range(3):
        gen = torch.Generator().manual_seed(100 + step)
        sk = {}
        for n, (W, _, Gs) in zip(names, mats):
            m, k = W.shape
            sk[n] = torch.randn(1, kk, k if m < k else m, generator=gen) * (1.0 / kk) ** 0.5
            params[n].main_grad = Gs[step].to(dev)
            cpu[n].G = Gs[step].float()
        opt._sketch_override = lambda batch, _sk=sk: {0: _sk[name_of[id(batch.params[0])]][0].to(dev)}
        h0 = len(hip_calls)
        opt.step()
        torch.cuda.synchronize()
        for n in names:
            O.dion_batch_step_local([cpu[n]], hyper, sketch_fn=lambda i, p, _s=sk[n]: _s)
        for (hin, hout), (oin, osk, oout), n in zip(hip_calls[h0:], ora_calls[len(ora_calls) - len(names):], names):
            ein = ((hin.float() - oin.float()).abs().max() / oin.float().abs().max()).item()
            dots = (hout.double() * oout.double()).sum(-2).flatten()
            flips = [int(i) for i in torch.nonzero(dots < 0).flatten()]
            piv = pivots(osk, oin)
            # the sign each side's own input gives the Householder pivot of column j (fp64): a
            # column whose two pivots differ in sign comes out negated
            sh, so = pivot_signs(osk, hin), pivot_signs(osk, oin)
            sign_diff = [j for j in range(len(sh)) if sh[j] != so[j]]
            entry = dict(step=step, matrix=n, input_maxrel=ein, flipped_columns=flips,
                         flipped_pivots={str(j): piv[j] for j in flips},
                         pivot_sign_differs_from_inputs=sign_diff,
                         smallest_pivot=min(piv), smallest_pivot_column=int(min(range(len(piv)), key=piv.__getitem__)))
            rec.append(entry)
            print(json.dumps(entry), flush=True)
    with open(out_path, "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "bf16_flip.json")
