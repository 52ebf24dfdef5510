"""Micro-benchmark and check of the matrix-core hidden layer
(csrc/f110_ddpg.hip k_linear_relu) against torch._addmm_activation on the
learner's shapes: time per call (HIP events, 200 reps) and max |diff| /
max |ref|."""
import json
import sys

import torch

sys.path.insert(0, ".")
from f110_gymnasium_ros2_jazzy_amd.ddpg_heads import linear_relu  # noqa: E402


def timeit(f, reps=200):
    for _ in range(10):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


out = []
for M, K, N in [(4096, 1088, 128), (8192, 1088, 128), (4096, 128, 128), (8192, 128, 128), (333, 1088, 128)]:
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.rand(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * (2.0 / K) ** 0.5
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    ref = torch._addmm_activation(b, x, W.t())
    got = linear_relu(x, W, b)
    err = float((got - ref).abs().max() / ref.abs().max())
    t_blas = timeit(lambda: torch._addmm_activation(b, x, W.t()))
    t_mfma = timeit(lambda: linear_relu(x, W, b))
    out.append({"M": M, "K": K, "N": N, "rel_err": err, "blas_us": round(t_blas, 2), "mfma_us": round(t_mfma, 2),
                "mfma_GBps": round((M * K + N * K + M * N) * 4 / t_mfma / 1e3, 1)})
    print(json.dumps(out[-1]), flush=True)
