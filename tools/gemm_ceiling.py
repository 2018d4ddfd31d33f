"""Practical bf16 MFMA ceiling on this box: the vendor GEMM (torch.matmul ->
hipBLASLt) on the block-key pass's shape -- 8192 queries x 768 dims against
corpus chunks of 262144 rows -- and on a square 8192^3 GEMM (bf16 in, bf16
out, random normal data), timed
with HIP events over back-to-back launches after a 2 s warm-up.  Prints one
JSON line: TFLOP/s and the fraction of the 2.5 PF dense bf16 peak, for
comparison with k_qs_blockkey's rate on the same box (tools/qs_probe.py)."""
import json
import time

import torch

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(7)
B, D, N = 8192, 768, 262144
Q = torch.randn((B, D), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
X = torch.randn((N, D), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
out = torch.empty((B, N), device=dev, dtype=torch.bfloat16)
S = 8192  # the library's best case: a square 8192^3 bf16 GEMM
A = torch.randn((S, S), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
Bm = torch.randn((S, S), generator=g, device=dev, dtype=torch.float32).to(torch.bfloat16)
C = torch.empty((S, S), device=dev, dtype=torch.bfloat16)
res = {}
cases = (("Q @ X^T (bf16 out)", lambda: torch.matmul(Q, X.t(), out=out), 2.0 * B * N * D),
         ("8192^3 square (bf16 out)", lambda: torch.matmul(A, Bm, out=C), 2.0 * S * S * S))
for name, fn, fl in cases:
    t0 = time.perf_counter()  # warm-up: library kernel choice + clock settling
    while time.perf_counter() - t0 < 2.0:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 40
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = fl / (ms * 1e-3) / 1e12
    res[name] = dict(ms=ms, tflops=tf, frac_of_2500=tf / 2500.0)
print(json.dumps(dict(shape=dict(M=B, N=N, K=D), data="randn bf16", results=res)), flush=True)
