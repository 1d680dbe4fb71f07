"""Scores shared by the parity tests."""
import torch


def dw_err(w_prev_hip, w_hip, w_prev_or, w_or, decay):
    """Update-only score of a weight step (tests/test_gpu_fullsize.py's docstring):
    max(|dW_a - dW_b| - ulp(W(t))) / max |dW_b|,  dW_x = W_x(t) - fp32(W_x(t-1) decay)."""
    d = torch.tensor(decay, dtype=torch.float32)
    dh = w_hip.double() - (w_prev_hip.float() * d).double()
    do = w_or.double() - (w_prev_or.float() * d).double()
    big = torch.maximum(w_hip.abs(), w_or.abs()).float()
    ulp = (torch.nextafter(big, torch.full_like(big, float("inf"))) - big).double()
    excess = ((dh - do).abs() - ulp).clamp_min(0.0)
    return excess.max().item() / max(do.abs().max().item(), 1e-30)


def q_err(q, ref):
    """max |q D - ref| / max |ref| with D the per-column sign that aligns q to ref.

    The sign of an orthonormalised column is -sign(alpha_j), alpha_j the sketch QR's Householder
    pivot (ortho.py:71-123, LAPACK dlarfg convention).  When |alpha_j| is within fp32 rounding of
    zero, two correct implementations -- or the reference on two machines -- can take opposite
    signs: tests/test_gpu_configs.py's W = 2 dense case hit alpha_56 = 2.7e-7 of its column's
    norm at step 2 (profiles/r05/h_dense_branch_sign_flip.log).  Q and P columns are therefore
    compared up to sign; W, M and the update dW are sign-invariant (P Q^T, P R^T) and keep their
    unaligned bars."""
    q, ref = q.detach().double().cpu(), ref.detach().double().cpu()
    d = torch.where((q * ref).sum(dim=-2, keepdim=True) < 0, -1.0, 1.0).double()
    return (q * d - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
