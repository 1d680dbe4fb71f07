"""Dev: HIP orthonormalize (explicit sketch) against the oracle on many random P, per column:
sign agreement and aligned error; also P's column-sign flips relative to the oracle."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from megatron_dion_amd.codec import HipDionCodec
    from oracle import dion_oracle as O
    dev = torch.device("cuda", 0)
    codec = HipDionCodec(dev)
    for mp_, r, B, kind in ((512, 64, 32, "randn"), (1024, 64, 32, "randn"), (512, 64, 32, "lowrankish"),
                            (512, 32, 32, "randn")):
        g = torch.Generator().manual_seed(mp_ + r)
        if kind == "randn":
            P = torch.randn(B, mp_, r, generator=g)
        else:
            P = torch.randn(B, mp_, r, generator=g) @ torch.diag(torch.logspace(0, -3, r))
        k = O.sketch_rows(r)
        S = torch.randn(B, k, mp_, generator=g) / k ** 0.5
        Ph = P.clone().to(dev)
        for b in range(B):
            codec.orthonormalize(Ph[b:b + 1], mp_, 4 * r, False, 0, 1.25, sketch=S[b:b + 1].to(dev).contiguous())
        torch.cuda.synchronize()
        flips, worst = 0, 0.0
        for b in range(B):
            Po = O.orthogonalize(P[b:b + 1], 1.25, sketch=S[b:b + 1])[0].double()
            h = Ph[b].double().cpu()
            sgn = torch.where((h * Po).sum(0) < 0, -1.0, 1.0).double()
            flips += int((sgn < 0).sum())
            worst = max(worst, ((h * sgn - Po).abs().max() / Po.abs().max()).item())
        print(f"mp {mp_} r {r} {kind}: {B} matrices, flipped columns {flips}, aligned worst {worst:.3e}", flush=True)
