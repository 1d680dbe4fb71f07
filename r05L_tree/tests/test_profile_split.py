"""DION_PROFILE_SPLIT: the reference's phase-labelled step profile (dion/algorithm.py:170-218,
dion/runtime.py:67-99) -- same [DION_PROFILE] / [DION_PROFILE_BATCH] lines and phase labels,
timed per batch phase (HIP events on the GPU, host clock here)."""
import re

import torch


def test_profile_split_reports_the_reference_phase_labels(monkeypatch, capsys):
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from tests._cpu_codec import OracleCodec

    torch.manual_seed(0)
    named = [(f"w{i}", torch.nn.Parameter(torch.randn(m, n) * 0.02)) for i, (m, n) in
             enumerate([(64, 48), (64, 48), (40, 96)])]
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, rank_fraction=0.25, codec=OracleCodec())
    attach_dp_routing(opt, named)
    monkeypatch.setenv("DION_PROFILE_SPLIT", "1")
    for _ in range(2):
        for _, p in named:
            p.grad = torch.randn_like(p) * 1e-3
        opt.step()
    out = capsys.readouterr().out
    lines = [ln for ln in out.splitlines() if ln.startswith("[DION_PROFILE] step=2 ")]
    assert lines, out
    labels = re.findall(r" ([a-z_]+)=[0-9.]+s", lines[0])[1:]  # after total=
    assert labels == ["grad_momentum", "q_unshard", "p_matmul", "p_reduce", "ortho_r", "error_feedback",
                      "q_normalize", "apply_update"], labels
    assert "(fused: p_matmul)" in lines[0]
    assert any(ln.startswith("[DION_PROFILE_BATCH] step=2 time=") and "kernel=ddp" in ln for ln in out.splitlines())
    recs = {label for label, _, _ in opt._profile_records}
    assert {"p_matmul", "ortho_r", "q_normalize", "apply_update"} <= recs
    assert all(sec >= 0.0 for _, sec, _ in opt._profile_records)
    # off again: no records, no lines
    monkeypatch.delenv("DION_PROFILE_SPLIT")
    opt.step()
    assert "[DION_PROFILE]" not in capsys.readouterr().out
