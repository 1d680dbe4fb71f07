"""Full-size GPU parity of the bench configurations (`pytest -m gpu`).

The optimizer runs EXACTLY as bench.py runs it -- MegatronDion's defaults (deferred
error feedback), launch groups of up to 16 matrices (`coalesce_max_entries=16`), two
alternating HIP streams (`local_streams=2`) -- on the BASELINE configs' real shapes, and
its W, M (after flush_error_feedback) and Q are compared with the CPU oracle
(oracle/dion_oracle.py, pinned to the reference's golden captures) step by step, with
explicit sketches (Q up to column signs, tests/_metrics.q_err: a sketch-QR pivot within rounding
of zero decides a column's sign either way) -- and configs 3 and 5 once more with the
sketch generated on the device exactly as bench.py times it (Rademacher, sketch_rad_kernel)
against the oracle's own Gaussian sketch, Q and P compared after column-sign alignment:

  config 2  single 4096 x 4096, r = 64
  config 3  the four Llama-3-8B 2D shapes (qkv 6144x4096, proj 4096x4096, fc1 28672x4096,
            fc2 4096x14336 transposed), r = 64, two matrices each (8 matrices, 4 launch groups)
  config 5  Mixtral-8x7B experts at r = 128: 8 x fc1 28672x4096 + 8 x fc2 4096x14336 in two
            launch groups of 8; the oracle checks the first and the last expert of each
            group (the indexing ends of a launch), and every expert's Q columns have unit norm
  config 4  (multi-rank schedule) a world-size-2 run on the GPU over gloo with rank-major
            launch groups of k = 2 and 3 chunks (coalesce_replicated_batches), deferred EF,
            two slot streams, against the same runtime driven by the CPU oracle codec

Tolerance: max |a - b| / max |b| <= 1e-5 for W, M and Q.  W0 (0.02 N(0,1))
dwarfs one step's update (~1e-3 of it), so W is also scored on the update alone ("dW"):

  dW_x(t) = W_x(t) - fp32(W_x(t-1) (1 - lr wd))       (fp64 arithmetic, x = hip | oracle)
  err_dW  = max(|dW_hip - dW_or| - ulp(W(t))) / max |dW_or|    <= TOL_DW

(the ulp is the two final fp32 roundings of W(t)).  dW also carries the P / Q differences
between the two runs (~1e-6), so TOL_DW = 5e-6; the isolated weight update is held to 1e-6
of its own scale in tests/test_gpu_update_precision.py.  The measured errors are written to
gpurun_out/fullsize_errors.json when that directory exists.
"""
import json
import math
import os
import socket
import tempfile
import zlib

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import megatron_dion_amd as mda
from megatron_dion_amd.optimizer import attach_dp_routing
from oracle import dion_oracle as O
from tests._metrics import dw_err, q_err

pytestmark = pytest.mark.gpu

TOL = 1e-5
TOL_DW = 5e-6
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ERRORS = {}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _record(key, errs):
    _ERRORS[key] = errs
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "fullsize_errors.json"), "w") as f:
            json.dump(_ERRORS, f, indent=1)


def _sketch(seed, k, mp_):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(k, mp_, generator=g) * math.sqrt(1.0 / k)


def _col_signs(a, b):
    """D (+-1 per column) with a D ~ b: the sign of each column pair's inner product."""
    d = (a.double() * b.double()).sum(dim=-2)
    return torch.where(d < 0, -1.0, 1.0).to(torch.float64)


def _run_vs_oracle(label, shapes, r, steps, check=None, generated=False):
    """shapes: list of (name, m, n).  Runs the bench-configured optimizer on the GPU and the
    oracle on the CPU for the matrices in `check` (default: all); returns worst errors.

    generated=True runs the HIP side exactly as bench.py does: no explicit sketch, so
    sketch_rad_kernel generates its Rademacher S (+-1/sqrt(k)) in the slab-reduced sketch
    product, while the oracle draws its own Gaussian N(0, 1/k) sketch (the reference's
    distribution, dion/ortho.py:643-662).  RCQR's P is the Q factor of M Q whatever the
    sketch, up to column signs, so W, M and dW keep their bars, and Q (= R / |R|, R = M^T P)
    and P are compared after aligning each column's sign: Q every step for every checked
    matrix, P for the first checked matrix of each shape."""
    dev = _dev()
    check = set(check) if check is not None else {n for n, _, _ in shapes}
    k = O.sketch_rows(r)
    named, host = [], {}
    for idx, (name, m, n) in enumerate(shapes):
        g = torch.Generator(device=dev).manual_seed(1000 + idx)
        p = torch.nn.Parameter(torch.randn(m, n, generator=g, device=dev) * 0.02)
        named.append((name, p))
        if name in check:
            host[name] = p.detach().cpu().clone()
    rf = r / min(min(m, n) for _, m, n in shapes)
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=rf,
                           coalesce_max_entries=16, local_streams=2)
    assert opt._defer_ef, "the bench configuration is the default: deferred error feedback"
    attach_dp_routing(opt, named)
    hyper = O.DionHyper(rank_fraction=rf)
    mats = {}
    for name, p in named:
        st = opt.state[p]
        assert st["r"] == r
        if name in check:
            m, n = p.shape
            mats[name] = O.DionMatrix(W=host[name].clone(), M=torch.zeros(m, n), Q=st["Q"].cpu().clone(), G=None,
                                      transposed=m < n, rank_fraction=rf)
    name_of = {id(p): name for name, p in named}
    cur = {"step": 0}

    def sk(name, m, n):
        return _sketch(7919 * cur["step"] + zlib.crc32(name.encode()), k, max(m, n))

    def override(batch):
        out = {}
        for i, bp in enumerate(batch.params):
            m, n = bp.shape
            out[i] = sk(name_of[id(bp)], m, n).to(dev)
        return out

    p_hip = {}
    first_of_shape = {}
    for name, p in named:
        if name in check:
            first_of_shape.setdefault(tuple(p.shape), name)
    watch = {id(p): name for name, p in named if first_of_shape.get(tuple(p.shape)) == name}
    if generated:
        def sink(P, R, params):
            for i, bp in enumerate(params):
                if id(bp) in watch:
                    p_hip[watch[id(bp)]] = P[i].detach().cpu().clone()
        opt._factor_sink = sink
    else:
        opt._sketch_override = override
    worst = {"W": 0.0, "dW": 0.0, "M": 0.0, "Q": 0.0}
    if generated:
        worst["P"] = 0.0
    decay = 1.0 - 0.01 * 0.01
    for step in range(steps):
        cur["step"] = step
        prev = {name: (p.detach().cpu().clone(), mats[name].W.clone()) for name, p in named if name in mats}
        grads = {}
        for idx, (name, p) in enumerate(named):
            g = torch.Generator(device=dev).manual_seed(99 + 17 * step + 131 * idx)
            p.main_grad = (torch.randn(p.shape, generator=g, device=dev) * 1e-3).to(torch.bfloat16)
            if name in check:
                grads[name] = p.main_grad.float().cpu()
        opt.step()
        if step == steps - 1:
            opt.flush_error_feedback()
        torch.cuda.synchronize()
        for name, mt in mats.items():
            m, n = mt.W.shape
            mt.G = grads[name]
            S = sk(name, m, n)
            O.dion_batch_step_local([mt], hyper, sketch_fn=lambda j, P, _S=S: _S[None])
        for name, p in named:
            if name not in mats:
                continue
            mt = mats[name]
            st = opt.state[p]
            errs = {"W": maxrel(p, mt.W), "Q": q_err(st["Q"], mt.Q),
                    "dW": dw_err(prev[name][0], p.detach().cpu(), prev[name][1], mt.W, decay)}
            if generated and name in watch.values():
                assert name in p_hip, f"no P of {name} reached the factor sink"
                ph, po = p_hip.pop(name), mt.trace["P"]
                errs["P"] = maxrel(ph.double() * _col_signs(ph, po), po)
            if step == steps - 1:
                errs["M"] = maxrel(st["momentum"], mt.M)
            for key, v in errs.items():
                worst[key] = max(worst[key], v)
            assert all(v <= (TOL_DW if key == "dW" else TOL) for key, v in errs.items()), (label, step, name, errs)
        assert not generated or not p_hip, f"P of {sorted(p_hip)} was never compared"
    for name, p in named:
        Q = opt.state[p]["Q"].double()
        assert torch.isfinite(p).all() and torch.isfinite(opt.state[p]["momentum"]).all()
        assert (Q.norm(dim=0) - 1).abs().max().item() <= 1e-5, (label, name)
    _record(label, worst)
    return worst


def test_config2_single_4096_r64():
    _run_vs_oracle("config2_4096x4096_r64", [("w", 4096, 4096)], 64, steps=3)


def test_config3_llama_shapes_bench_settings():
    _run_vs_oracle("config3_llama_shapes_r64", _llama_set(), 64, steps=3)


def _llama_set():
    shapes = []
    for layer in range(2):
        for name, m, n in (("linear_qkv", 6144, 4096), ("linear_proj", 4096, 4096),
                           ("linear_fc1", 28672, 4096), ("linear_fc2", 4096, 14336)):
            shapes.append((f"layers.{layer}.{name}.weight", m, n))
    return shapes


def _mixtral_set():
    shapes = [(f"layers.0.experts.{e}.linear_fc1.weight", 28672, 4096) for e in range(8)] + \
             [(f"layers.0.experts.{e}.linear_fc2.weight", 4096, 14336) for e in range(8)]
    return shapes, [shapes[0][0], shapes[7][0], shapes[8][0], shapes[15][0]]


def test_config5_mixtral_experts_r128():
    shapes, check = _mixtral_set()
    _run_vs_oracle("config5_mixtral_experts_r128", shapes, 128, steps=2, check=check)


def test_config3_llama_generated_sketch():
    """The timed path itself: bench.py's generated Rademacher sketch (sketch_rad_kernel at
    m_P = 6144 / 4096 / 28672 / 14336, its many-chunk slab-reduced configuration) against the
    oracle's Gaussian-sketch step."""
    _run_vs_oracle("config3_llama_generated_sketch", _llama_set(), 64, steps=3, generated=True)


def test_config5_mixtral_generated_sketch():
    """r = 128, k = 256 sketch rows, generated as bench.py runs it, against the oracle."""
    shapes, check = _mixtral_set()
    _run_vs_oracle("config5_mixtral_generated_sketch", shapes, 128, steps=2, check=check, generated=True)


# ---------------------------------------------------------------------------------------------- W = 2, k > 1
def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


W2_SHAPES = [(f"a{i}", 512, 384) for i in range(8)] + [(f"t{i}", 384, 1024) for i in range(6)] + \
            [("odd", 512, 384)]


def _w2_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle.cpu_codec import OracleCodec

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    r, steps = 64, 3
    k = O.sketch_rows(r)
    res = {}
    q0 = {}
    for backend in ("hip", "oracle"):
        on = dev if backend == "hip" else torch.device("cpu")
        named = [(n, torch.nn.Parameter((torch.randn(m, c, generator=torch.Generator().manual_seed(i)) * 0.02)
                                        .to(on))) for i, (n, m, c) in enumerate(W2_SHAPES)]
        kw = dict(codec=OracleCodec(deferred=True)) if backend == "oracle" else {}
        opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=r / 384,
                               coalesce_max_entries=6, local_streams=2, **kw)
        attach_dp_routing(opt, named, replicate_group=dist.group.WORLD)
        # one Q0 for both backends: the device stream (HIP) and the CPU stream (oracle) of
        # the seeded Q init differ (state.py init_q), the runs must start from the same Q
        if backend == "hip":
            q0 = {n: opt.state[p]["Q"].detach().cpu().clone() for n, p in named}
        else:
            for n, p in named:
                opt.state[p]["Q"].copy_(q0[n])
        name_of = {id(p): n for n, p in named}
        cur = {"s": 0}

        def override(batch, _on=on, _name_of=name_of, _cur=cur):
            # one sketch per (step, matrix), whichever rank owns the matrix; padded entries
            # (the batch's first param repeated) are never orthonormalised
            out = {}
            for i, bp in enumerate(batch.params):
                m, c = bp.shape
                out[i] = _sketch(7919 * _cur["s"] + zlib.crc32(_name_of[id(bp)].encode()), k, max(m, c)).to(_on)
            return out

        opt._sketch_override = override
        for n, p in named:
            res[f"{backend}_sinit_{n}_W"] = p.detach().cpu().clone()
        chunks = []
        for s in range(steps):
            cur["s"] = s
            for i, (n, p) in enumerate(named):
                g = torch.Generator().manual_seed(100 * s + 10 * rank + i)
                p.main_grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).to(on)
            chunks.append([int(getattr(b, "_chunks", 0) or 0) for b in opt._batches()[0]])
            opt.step()
            if s == steps - 1:
                opt.flush_error_feedback()
            if backend == "hip":
                torch.cuda.synchronize()
            for n, p in named:
                res[f"{backend}_s{s}_{n}_W"] = p.detach().cpu().clone()
                res[f"{backend}_s{s}_{n}_Q"] = opt.state[p]["Q"].detach().cpu().clone()
                if s == steps - 1:
                    res[f"{backend}_s{s}_{n}_M"] = opt.state[p]["momentum"].detach().cpu().clone()
        res[f"{backend}_chunks"] = torch.tensor(chunks[0])
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_w2_rank_major_groups_k_gt_1_on_gpu():
    """coalesce_replicated_batches with k = 3 (512x384: 8 full batches of 2 -> groups of
    3 + 1 + a padded batch) and k = 3 (384x1024 transposed: 3 full batches), deferred EF,
    two slot streams: the HIP path over gloo against the CPU oracle codec over gloo."""
    _dev()
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_w2_worker, args=(2, _port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    worst = {"W": 0.0, "dW": 0.0, "M": 0.0, "Q": 0.0}
    decay = 1.0 - 0.01 * 0.01
    for rank in range(2):
        R = res[rank]
        for s in range(3):
            for n, _, _ in W2_SHAPES:
                before = "sinit" if s == 0 else f"s{s - 1}"
                e = dw_err(R[f"hip_{before}_{n}_W"], R[f"hip_s{s}_{n}_W"], R[f"oracle_{before}_{n}_W"],
                           R[f"oracle_s{s}_{n}_W"], decay)
                worst["dW"] = max(worst["dW"], e)
                assert e <= TOL_DW, (rank, s, n, e)
    for rank in range(2):
        assert max(res[rank]["hip_chunks"].tolist()) == 3, res[rank]["hip_chunks"]
        assert res[rank]["hip_chunks"].tolist() == res[rank]["oracle_chunks"].tolist()
        for key, v in res[rank].items():
            if not key.startswith("hip_s") or key.startswith("hip_sinit"):
                continue
            ref = res[rank]["oracle" + key[3:]]
            e = q_err(v, ref) if key.endswith("_Q") else maxrel(v, ref)
            worst[key[-1]] = max(worst[key[-1]], e)
            assert e <= TOL, (rank, key, e)
    for key in res[0]:
        if key.startswith("hip_s") and (key.endswith("_W") or key.endswith("_Q")):
            assert torch.equal(res[0][key], res[1][key]), key
    _record("w2_rank_major_k3", worst)
