"""Dev check (numpy, CPU): the RCQR with fp32 substitution solves against the explicit-inverse
GEMM solves (fp16x3 products with per-row / per-column power-of-two scales; the inverse in fp64
or by fp32 back substitution as tri_inv_kernel does), final P against an fp64 run of the same
algorithm, over 0 / 3 / 6 decades of column scales.  Output: profiles/r05/solve_precision_numpy.txt
"""
import numpy as np, scipy.linalg as sl
rng = np.random.default_rng(0)
def h3(x, axis=None):
    a = np.abs(x).max(axis=axis, keepdims=True) if axis is not None else np.abs(x).max()
    a = np.where(a > 0, a, 1.0)
    e = np.frexp(a)[1]; s = 2.0**(15-e)
    xs = (x*s).astype(np.float32)
    hi = xs.astype(np.float16).astype(np.float32)
    lo = (xs-hi).astype(np.float16).astype(np.float32)
    return hi, lo, s
def h3mm(A, B):
    ah, al, sa = h3(A, axis=1); bh, bl, sb = h3(B, axis=0)
    out = (ah.astype(np.float64)@bh + ah.astype(np.float64)@bl + al.astype(np.float64)@bh)
    return (out/(sa*sb)).astype(np.float32)
def inv32(R):
    # column-parallel back substitution in fp32 with the reciprocal diagonal (tri_inv_kernel order)
    r = R.shape[0]; R = R.astype(np.float32); d = (np.float32(1.0)/np.diag(R)).astype(np.float32)
    X = np.zeros((r, r), np.float32)
    for i in range(r-1, -1, -1):
        acc = (np.arange(r) == i).astype(np.float32)
        for k in range(i+1, r):
            acc = (acc - R[i, k]*X[k]).astype(np.float32)
        X[i] = np.where(np.arange(r) >= i, acc*d[i], 0).astype(np.float32)
    return X
def trsm32(P, R):
    X = P.astype(np.float32).copy(); r = R.shape[0]
    for k in range(r):
        X[:, k] = X[:, k] * np.float32(1.0/R[k, k])
        X[:, k+1:] -= np.outer(X[:, k], R[k, k+1:]).astype(np.float32)
    return X
for d in (0, 3, 6):
    m, r, k = 2048, 64, 128
    U = np.linalg.qr(rng.standard_normal((m, r)))[0]; V = np.linalg.qr(rng.standard_normal((r, r)))[0]
    s = np.logspace(0, -d, r)
    P = ((U*s)@V.T).astype(np.float32)
    S = (rng.choice([-1.0, 1.0], size=(k, m))/np.sqrt(k)).astype(np.float32)
    SP = S.astype(np.float64)@P.astype(np.float64)
    R1 = np.linalg.qr(SP, mode='r'); P1 = sl.solve_triangular(R1.T, P.astype(np.float64).T, lower=True).T
    R2 = np.linalg.cholesky(P1.T@P1).T; Pref = sl.solve_triangular(R2.T, P1.T, lower=True).T
    out = {}
    for mode in ('trsm32', 'h3inv64', 'h3inv32'):
        R1f = np.linalg.qr((S@P).astype(np.float64), mode='r').astype(np.float32)
        if mode == 'trsm32':
            P1f = trsm32(P, R1f)
        else:
            T1 = np.linalg.inv(R1f.astype(np.float64)).astype(np.float32) if mode == 'h3inv64' else inv32(R1f)
            P1f = h3mm(P, T1)
        G = (P1f.T@P1f).astype(np.float32)
        R2f = np.linalg.cholesky(G.astype(np.float64)).T.astype(np.float32)
        if mode == 'trsm32':
            Pf = trsm32(P1f, R2f)
        else:
            T2 = np.linalg.inv(R2f.astype(np.float64)).astype(np.float32) if mode == 'h3inv64' else inv32(R2f)
            Pf = h3mm(P1f, T2)
        sg = np.sign((Pf*Pref).sum(0)); Pf = Pf*sg
        err = np.abs(Pf-Pref).max()/np.abs(Pref).max()
        orth = np.abs(Pf.T.astype(np.float64)@Pf - np.eye(r)).max()
        out[mode] = f"err {err:.2e} orth {orth:.2e}"
    print(f"decades {d}: " + " | ".join(f"{k}: {v}" for k, v in out.items()))
