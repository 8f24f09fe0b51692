"""Vendor-library calibration on MI355X: hipBLASLt/rocBLAS through torch on the layer-11 shapes."""
import json
import time

import torch


def t(fn, it=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


out = {}
for (M, N, K) in [(8192, 11264, 2048), (8192, 2048, 5632), (8192, 8192, 8192), (546, 2816, 2048)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(N, K, device="cuda", dtype=torch.float16)
    ms = t(lambda: torch.matmul(a, b.t()))
    out[f"fp16 {M}x{N}x{K}"] = round(2 * M * N * K / ms / 1e9, 1)
    try:
        ai = torch.randint(-127, 127, (M, K), device="cuda", dtype=torch.int8)
        bi = torch.randint(-127, 127, (K, N), device="cuda", dtype=torch.int8)
        ms = t(lambda: torch._int_mm(ai, bi))
        out[f"int8 {M}x{N}x{K}"] = round(2 * M * N * K / ms / 1e9, 1)
    except Exception as e:  # noqa: BLE001
        out[f"int8 {M}x{N}x{K}"] = f"unavailable: {type(e).__name__}: {str(e)[:80]}"
print(json.dumps(out, indent=1))
