import torch
a, b = torch.load("gpurun_out/diag_default.pt"), torch.load("gpurun_out/diag_kr1.pt")
for i, (x, y) in enumerate(zip(a["M"], b["M"])):
    d = (x - y).abs()
    rows = (d.amax(dim=1) > 1e-9).nonzero().flatten().tolist()
    print("M", i, "max", d.max().item(), "bad rows", len(rows), rows[:40])
d = (a["P"] - b["P"]).abs()
print("P max", d.max().item(), "bad rows", (d.amax(dim=2) > 1e-6 * a["P"].abs().max()).nonzero()[:20].tolist())
print("nz", a["nz"].tolist(), b["nz"].tolist())
