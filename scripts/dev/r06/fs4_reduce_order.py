"""Which summation order does the reference's FS = 4 bf16 reduce-scatter use?  Recompute every
rank's partial P_k = X_k Q_k (bf16) of step 0 from the captures (M0 + G, Q0) and compare the
owner's captured orthogonalize input (the reduced P) with candidate orders:
  fp32:   the fp32 sum of the four terms rounded to bf16 once (this build's scheme)
  seq:    ((p0 + p1) + p2) + p3, rounding after each add (rank order)
  ring:   the ring reduce-scatter order for the chunk rank r keeps: p_{r+1}, +p_{r+2}, +p_{r+3}, +p_r
  pair:   (p0 + p1) + (p2 + p3)
Prints, per case and candidate, the elements that differ and the largest difference in bf16 ulps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
from tests._golden import FsCase  # noqa: E402


def ulps(a, b):
    """|a - b| in units of bf16 ulp of max(|a|, |b|)."""
    m = torch.maximum(a.abs(), b.abs()).float()
    e = torch.floor(torch.log2(m.clamp_min(1e-30)))
    ulp = torch.pow(2.0, e - 7)
    return ((a.float() - b.float()).abs() / ulp)


def bf(x):
    return x.to(torch.bfloat16)


def main(names):
    for name in names:
        case = FsCase(name)
        W = case.world
        step = 0
        gshape = {n: (m, k) for n, m, k in case.mats}
        stats = {}
        for b in case.batches(0, step):
            members, real = b["members"], int(b["real"])
            parts = []
            for k in range(W):
                # the reference's batched product (runtime.py:1602-1616: stack, then one bmm) over
                # the whole batch, padded entries zero: a per-matrix mm rounds differently
                Xs, Qs = [], []
                for i, n in enumerate(members):
                    src = members[0] if i >= real else n
                    M = (case.t(k, step, f"{src}_M0").to(torch.bfloat16) + case.t(k, step, f"{src}_G").to(torch.bfloat16))
                    Q = case.t(k, step, f"{src}_Q0").to(torch.bfloat16)
                    if i >= real:
                        M, Q = torch.zeros_like(M), torch.zeros_like(Q)
                    Xs.append(M.mT if case.fs_dim(src) == 0 else M)
                    Qs.append(Q)
                parts.append(list(torch.stack(Xs) @ torch.stack(Qs)))
            idx = b["fs_indices"]
            for k in range(W):  # rank k owns entry idx[k]
                e = idx[k]
                if e >= real:
                    continue
                p = [parts[j][e] for j in range(W)]
                cand = {
                    "fp32": bf(sum(x.float() for x in p)),
                    "seq": bf(bf(bf(p[0] + p[1]) + p[2]) + p[3]) if W == 4 else None,
                    "ring": None,
                    "pair": bf(bf(p[0] + p[1]) + bf(p[2] + p[3])) if W == 4 else None,
                }
                acc = p[(k + 1) % W]
                for j in range(2, W + 1):
                    acc = bf(acc + p[(k + j) % W])
                cand["ring"] = acc
                calls = case.ortho_calls(k, step)
                got = min((c["p_in"] for c in calls if c["p_in"].shape[-2:] == p[0].shape),
                          key=lambda t: (t[0].float() - cand["fp32"].float()).abs().max().item())[0]
                for c, v in cand.items():
                    if v is None:
                        continue
                    d = ulps(v.float(), got.float())
                    s = stats.setdefault(c, [0, 0, 0.0])
                    s[0] += int((d > 0).sum())
                    s[1] += d.numel()
                    s[2] = max(s[2], float(d.max()))
        for c, (nd, nt, mx) in stats.items():
            print(f"{name}: {c:5s} {nd}/{nt} elements differ, max {mx:.2f} bf16 ulp")


if __name__ == "__main__":
    main(sys.argv[1:] or ["f6_fs4_bf16_cols", "f7_fs4_bf16_mixed"])


def rotations(names):
    """Per element: which cyclic orders p_s, +p_{s+1}, +p_{s+2}, +p_{s+3} (s = 0..3, both ring
    directions) reproduce the reference's reduced value exactly."""
    for name in names:
        case = FsCase(name)
        W = case.world
        total = anymatch = 0
        hist = {}
        for step in range(case.steps if False else 1):
            for b in case.batches(0, step):
                members, real = b["members"], int(b["real"])
                parts = []
                for k in range(W):
                    Xs, Qs = [], []
                    for i, n in enumerate(members):
                        src = members[0] if i >= real else n
                        M = case.t(k, step, f"{src}_M0").to(torch.bfloat16) + case.t(k, step, f"{src}_G").to(torch.bfloat16)
                        Q = case.t(k, step, f"{src}_Q0").to(torch.bfloat16)
                        if i >= real:
                            M, Q = torch.zeros_like(M), torch.zeros_like(Q)
                        Xs.append(M.mT if case.fs_dim(src) == 0 else M)
                        Qs.append(Q)
                    parts.append(list(torch.stack(Xs) @ torch.stack(Qs)))
                flat_off = 0
                for k in range(W):
                    e = b["fs_indices"][k]
                    p = [parts[j][e] for j in range(W)]
                    if e >= real:
                        continue
                    fp = bf(sum(x.float() for x in p))
                    got = min((c["p_in"] for c in case.ortho_calls(k, step) if c["p_in"].shape[-2:] == p[0].shape),
                              key=lambda t: (t[0].float() - fp.float()).abs().max().item())[0]
                    ok = torch.zeros_like(got, dtype=torch.int64)
                    for d in (1, -1):
                        for s in range(W):
                            acc = p[s]
                            for j in range(1, W):
                                acc = bf(acc + p[(s + d * j) % W])
                            ok |= ((acc.float() == got.float()).to(torch.int64) << (s + (0 if d == 1 else W)))
                    total += got.numel()
                    anymatch += int((ok != 0).sum())
                    for v in ok.flatten().tolist():
                        hist[v] = hist.get(v, 0) + 1
        print(f"{name}: {anymatch}/{total} elements match some cyclic order; order-mask histogram (top 8):",
              sorted(hist.items(), key=lambda kv: -kv[1])[:8])


if __name__ == "__main__" and os.environ.get("ROT"):
    rotations(["f6_fs4_bf16_cols", "f7_fs4_bf16_mixed"])


def layout(name):
    """Unique matching cyclic order per element vs its flat position in P_batch."""
    case = FsCase(name)
    W = case.world
    step = 0
    for bi, b in enumerate(case.batches(0, step)):
        members, real = b["members"], int(b["real"])
        parts = []
        for k in range(W):
            Xs, Qs = [], []
            for i, n in enumerate(members):
                src = members[0] if i >= real else n
                M = case.t(k, step, f"{src}_M0").to(torch.bfloat16) + case.t(k, step, f"{src}_G").to(torch.bfloat16)
                Q = case.t(k, step, f"{src}_Q0").to(torch.bfloat16)
                if i >= real:
                    M, Q = torch.zeros_like(M), torch.zeros_like(Q)
                Xs.append(M.mT if case.fs_dim(src) == 0 else M)
                Qs.append(Q)
            parts.append(list(torch.stack(Xs) @ torch.stack(Qs)))
        per = parts[0][0].numel()
        print(f"batch {bi}: members {members} real {real} per-entry {per} total {per * W}")
        for k in range(W):
            e = b["fs_indices"][k]
            if e >= real:
                continue
            p = [parts[j][e] for j in range(W)]
            fp = bf(sum(x.float() for x in p))
            got = min((c["p_in"] for c in case.ortho_calls(k, step) if c["p_in"].shape[-2:] == p[0].shape),
                      key=lambda t: (t[0].float() - fp.float()).abs().max().item())[0].flatten()
            uniq = []
            for i in range(got.numel()):
                ms = []
                for d in (1, -1):
                    for s in range(W):
                        acc = p[s].flatten()[i]
                        for j in range(1, W):
                            acc = bf(acc + p[(s + d * j) % W].flatten()[i])
                        if float(acc) == float(got[i]):
                            ms.append((s, d))
                if len(ms) <= 2:
                    uniq.append((e * per + i, ms))
            # compress runs
            runs, last = [], None
            for pos, ms in uniq:
                key = tuple(ms)
                if last is None or last[1] != key:
                    runs.append([pos, pos, key])
                    last = (pos, key)
                else:
                    runs[-1][1] = pos
            print(f"  rank {k} entry {e}: {len(uniq)} determined elements; runs:", runs[:12])


if __name__ == "__main__" and os.environ.get("LAYOUT"):
    layout(os.environ["LAYOUT"])


def ring_check(names):
    """The order the layout found: rank k's chunk is p_{k-1} + p_{k-2} + ... + p_k (a ring
    reduce-scatter, bf16 rounding after every hop).  Count the elements it reproduces, all steps
    (step s > 0 from the captured M0 of that step)."""
    for name in names:
        case = FsCase(name)
        W = case.world
        tot = same = 0
        for step in range(case.steps):
            for b in case.batches(0, step):
                members, real = b["members"], int(b["real"])
                parts = []
                for k in range(W):
                    Xs, Qs = [], []
                    for i, n in enumerate(members):
                        src = members[0] if i >= real else n
                        M = case.t(k, step, f"{src}_M0").to(torch.bfloat16) + case.t(k, step, f"{src}_G").to(torch.bfloat16)
                        Q = case.t(k, step, f"{src}_Q0").to(torch.bfloat16)
                        if i >= real:
                            M, Q = torch.zeros_like(M), torch.zeros_like(Q)
                        Xs.append(M.mT if case.fs_dim(src) == 0 else M)
                        Qs.append(Q)
                    parts.append(list(torch.stack(Xs) @ torch.stack(Qs)))
                for k in range(W):
                    e = b["fs_indices"][k]
                    if e >= real:
                        continue
                    p = [parts[j][e] for j in range(W)]
                    acc = p[(k - 1) % W]
                    for j in range(2, W + 1):
                        acc = bf(acc + p[(k - j) % W])
                    got = min((c["p_in"] for c in case.ortho_calls(k, step) if c["p_in"].shape[-2:] == p[0].shape),
                              key=lambda t: (t[0].float() - acc.float()).abs().max().item())[0]
                    tot += got.numel()
                    same += int((got.float() == acc.float()).sum())
        print(f"{name}: ring order (k-1, k-2, ..., k) reproduces {same}/{tot} elements of the reduced P")


if __name__ == "__main__" and os.environ.get("RING"):
    ring_check(["f6_fs4_bf16_cols", "f7_fs4_bf16_mixed"])
