#!/usr/bin/env python3
"""Speed-of-light reference for the conv kernel's GEMMs: torch._int_mm (hipBLASLt int8 GEMM,
int32 out) on the dense GEMM of an R50 conv with the three activation limbs stacked as rows
(M = 3 * pixels, K = kh*kw*cin, N = cout), i.e. the same int8 MACs as the conv's limb passes with
the im2col already materialised and no epilogue. Diagnostics only.

    python tools/probe_int_mm.py"""
import json

import torch

SHAPES = [  # name, pixels (B=256), K, N
    ("c2_256_256_14 (3x3)", 256 * 14 * 14, 2304, 256),
    ("c2_128_128_28 (3x3)", 256 * 28 * 28, 1152, 128),
    ("c2_512_512_7 (3x3)", 256 * 7 * 7, 4608, 512),
    ("c1_1024_256_14", 256 * 14 * 14, 1024, 256),
    ("c3_256_1024_14", 256 * 14 * 14, 256, 1024),
    ("c3_64_256_56", 256 * 56 * 56, 64, 256),
]
dev = torch.device("cuda")
res = []
for name, px, k, n in SHAPES:
    a = torch.randint(-128, 128, (3 * px, k), dtype=torch.int8, device=dev)
    b = torch.randint(-128, 128, (n, k), dtype=torch.int8, device=dev).t()  # column-major B
    for _ in range(3):
        torch._int_mm(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch._int_mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e-3
    macs = 3 * px * k * n
    res.append({"shape": name, "M": 3 * px, "K": k, "N": n, "us": round(t * 1e6, 1),
                "TMAC_s": round(macs / t / 1e12, 1), "frac_of_2339": round(macs / t / 2339e12, 3)})
    print(json.dumps(res[-1]), flush=True)
