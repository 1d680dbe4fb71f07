"""Codec backend built from the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Lets the multi-process (gloo) tests -- and bench.py's `cpu_baseline` leg -- drive the
product's batch runtime and collective schedule (megatron_dion_amd/runtime.py) on
CPU tensors with the oracle's arithmetic (oracle/dion_oracle.py).  It is injected
explicitly (`MegatronDion(..., codec=OracleCodec())`); the product never constructs
it and has no CPU fallback of its own.
"""
import torch

from . import dion_oracle as O


class OracleCodec:
    name = "oracle-cpu"
    fuses_p_fixup = True  # orthonormalize(fix_nonzero=...) + fixup_colnorm(P=None)
    fuses_r_fixup = True  # project_r_fixup = project_r + fixup_colnorm(P=None)

    def __init__(self, sketch_lookup=None, hyper_eps=1e-8, deferred=False):
        self.sketch_lookup = sketch_lookup  # fn(P (1, m_P, r)) -> sketch (1, k, m_P) or None
        self.deferred = deferred            # offer the deferred-EF pass A (host-logic tests)

    def supports_deferred_ef(self, m, n, r, transposed, state_dtype=torch.float32, grad_dtype=None):
        return self.deferred

    def project_p_ef(self, grads, momentums, qs, P, nonzero, transposed, ef_P, ef_R, alpha):
        for b, M in enumerate(momentums):
            if ef_P[b] is not None:
                # the eager update's arithmetic in the state dtype (ef_apply below)
                Pb, Rb = ef_P[b].to(M.dtype), ef_R[b].to(M.dtype)
                upd = (Rb @ Pb.mT) if transposed else (Pb @ Rb.mT)
                M.add_(upd * alpha)
        self.project_p(grads, momentums, qs, P, nonzero, transposed)

    def project_p(self, grads, momentums, qs, P, nonzero, transposed):
        for b, M in enumerate(momentums):
            if grads is not None:
                M.add_(grads[b].to(M.dtype))
            X = M.mT if transposed else M
            P[b] = X @ qs[b].to(X.dtype)          # bf16 state: a bf16 matmul (runtime.py:1607-1616)
            nonzero[b] = int(bool((M != 0).any()))

    def orthonormalize(self, P, m, n, transposed, seed, oversample=1.25, sketch=None, state_dtype=torch.float32,
                       fix_nonzero=None, p_split=None):
        for b in range(P.shape[0]):
            S = sketch
            if S is None and self.sketch_lookup is not None:
                S = self.sketch_lookup(P[b:b + 1])
            gen = torch.Generator().manual_seed(int(seed) & ((1 << 63) - 1))
            out = O.orthogonalize(P[b:b + 1], oversample, sketch=S, generator=gen)
            P[b:b + 1] = out.to(state_dtype)      # ortho.py:123 casts back to P's dtype
            if fix_nonzero is not None:           # the fused fix-up (kernels.py:185-188)
                P[b] = torch.zeros_like(P[b]) if int(fix_nonzero[b]) == 0 else P[b].nan_to_num()

    # distributed RCQR pieces (dion/ortho.py:682-834): the reference's arithmetic, with the
    # triangular solves as products with the explicit inverses the codec interface passes on
    def dortho_sketch(self, P, m, n, transposed, seed, row_offset, oversample, SP, sketch=None):
        if sketch is None:
            raise RuntimeError("[ORACLE_CODEC] the distributed sketch needs an explicit slice on CPU")
        SP.copy_(sketch.to(torch.float32) @ P)

    def dortho_qr_inv(self, SP, R1inv):
        R1 = torch.linalg.qr(SP.to(torch.float32), mode="r")[1]
        eye = torch.eye(R1.shape[-1], dtype=torch.float32).expand_as(R1)
        R1inv.copy_(torch.linalg.solve_triangular(R1, eye, upper=True))

    def dortho_apply(self, P_in, Uinv, P_out, m, n, transposed):
        P_out.copy_(P_in @ Uinv)

    def dortho_gram(self, P, gram, m, n, transposed):
        gram.copy_(P.mT @ P)

    def dortho_chol_inv(self, gram, R2inv):
        R2 = torch.linalg.cholesky_ex(gram.to(torch.float32), upper=True)[0]
        eye = torch.eye(R2.shape[-1], dtype=torch.float32).expand_as(R2)
        R2inv.copy_(torch.linalg.solve_triangular(R2, eye, upper=True))

    def round_bf16(self, X):
        X.copy_(X.to(torch.bfloat16).float())

    def project_r(self, momentums, P, R, transposed, nonzero=None, p_split=None):
        for b, M in enumerate(momentums):
            X = M.mT if transposed else M
            R[b] = X.mT @ P[b].to(X.dtype)

    def project_r_fixup(self, momentums, P, R, qs, nonzero, eps, transposed, p_split=None):
        self.project_r(momentums, P, R, transposed, nonzero=nonzero)
        m, n = momentums[0].shape[-2:]
        self.fixup_colnorm(None, R, qs, nonzero, eps, m, n, transposed)

    def fixup_colnorm(self, P, R, qs, nonzero, eps, m, n, transposed):
        B = len(qs)
        Q = torch.stack(qs, 0)
        zero = (nonzero[:B] == 0).view(B, 1, 1)
        if P is not None:  # None: fixed by orthonormalize(fix_nonzero=...)
            P[:B] = torch.where(zero, torch.zeros_like(P[:B]), P[:B].nan_to_num())
        R[:B] = torch.where(zero, Q.nan_to_num(), R[:B].nan_to_num())
        Qn = O.column_normalize(R[:B], eps)
        for b in range(B):
            qs[b].copy_(Qn[b])

    def fixup_colsum(self, P, R, qs, nonzero, colsum, m, n, transposed):
        B = len(qs)
        Q = torch.stack(qs, 0)
        zero = (nonzero[:B] == 0).view(B, 1, 1)
        P[:B] = torch.where(zero, torch.zeros_like(P[:B]), P[:B].nan_to_num())
        R[:B] = torch.where(zero, Q.nan_to_num().to(R.dtype), R[:B].nan_to_num())
        colsum[:B] = R[:B].to(torch.float32).square().sum(dim=-2)

    def colnorm_apply(self, R, qs, colsum, eps, m, n, transposed):
        for b in range(len(qs)):
            qn = R[b].to(torch.float32) / (colsum[b].sqrt() + eps)
            qs[b].copy_(qn.to(qs[b].dtype))

    def ef_apply(self, momentums, params, P, R, qs, nonzero, mu, lr, wd, scaled_lr, transposed):
        dt = qs[0].dtype  # the state dtype: factors carry it (kernels.py:54-83, 229-276)
        for b in range(len(qs)):
            Pb, Rb = P[b].to(dt), R[b].to(dt)
            if momentums is not None:
                upd = (Rb @ Pb.mT) if transposed else (Pb @ Rb.mT)
                momentums[b].add_(upd * (-(1.0 - mu)))
            if params is not None:
                W = params[b]
                if wd > 0:
                    W.mul_(1 - lr * wd)
                delta = (qs[b] @ Pb.mT) if transposed else (Pb @ qs[b].mT)
                W.add_(delta.to(W.dtype), alpha=-scaled_lr)

    def grad_sum_sq(self, grads, out):
        out += O.grad_sum_sq_fp64(grads).to(out.device)

    def elementwise_adamw(self, params, grads, first_moments, second_moments, **kw):
        O.elementwise_adamw(params, grads, first_moments, second_moments, **kw)

    def elementwise_lion(self, params, grads, first_moments, **kw):
        O.elementwise_lion(params, grads, first_moments, **kw)

