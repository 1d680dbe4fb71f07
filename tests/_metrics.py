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
