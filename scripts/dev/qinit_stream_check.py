"""Dev: does one device draw of the full Q equal the per-row offset draws the reference
makes (dion/state.py:97-108)?  Prints the max difference per shape."""
import time
import torch

dev = torch.device("cuda", 0)
for rows, cols in ((64, 16), (4096, 64), (14336, 64), (4095, 63), (1000, 30)):
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234)
    t0 = time.perf_counter()
    per_row = torch.empty(rows, cols, device=dev)
    for r in range(rows):
        start = r * cols
        aligned = (start // 4) * 4
        prefix = start - aligned
        gen.set_offset(aligned)
        v = torch.empty(prefix + cols, device=dev)
        v.normal_(0.0, 1.0, generator=gen)
        per_row[r].copy_(v[prefix:])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gen2 = torch.Generator(device="cuda")
    gen2.manual_seed(1234)
    full = torch.randn(rows, cols, device=dev, generator=gen2)
    gen3 = torch.Generator(device="cuda")
    gen3.manual_seed(1234)
    gen3.set_offset(0)
    full3 = torch.empty(rows, cols, device=dev).normal_(0.0, 1.0, generator=gen3)
    print(f"{rows}x{cols}: per-row {1e3*(t1-t0):.1f} ms; randn==per_row {torch.equal(full, per_row)} "
          f"normal_==per_row {torch.equal(full3, per_row)} maxdiff {(full3-per_row).abs().max().item():.3e}", flush=True)
