"""Microbenchmark of the learner GEMMs at C5's shapes (batch 4096, obs 1088,
hidden 128): csrc/f110_gemm.hip against torch (hipBLASLt, with the shipped
TunableOp file when F110_TUNABLEOP != 0).  Event-timed loops of 200 calls
(launch-bound calls show their launch cost too); one JSON line.  Run under
rocprofv3 --kernel-trace --stats for per-kernel times.

    python scripts/learner_gemm_mb.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd import learner_gemm as lg  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.ddpg import TunedGemms, enable_tuned_gemms  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps  # us per call


def main():
    dev = torch.device("cuda:0")
    tuned = enable_tuned_gemms(dev)
    M, D, H = int(os.environ.get("MB_M", 4096)), 1088, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    S, S2, W1, W2, W3, b = r(M, D), r(M, D), r(H, D), r(H, D), r(H, D), r(H)
    Z, act, Ws2, G, Y = r(M, H), r(M, 2), r(H, H + 2), r(M, H), r(M, H)
    out = {"M": M, "tuned_torch": tuned, "us": {}}
    us = out["us"]
    y1, y2, y3 = (torch.empty(M, H, device="cuda") for _ in range(3))
    with TunedGemms(tuned):
        us["torch_fwd_1088"] = timed(lambda: torch._addmm_activation(b, S, W1.t()))
        us["ours_fwd_1088"] = timed(lambda: lg.gemm([lg.op(S, W1, y1, H, D, D, D, H, bias=b, relu=True)], M, dev))
        us["ours_fwd_1088_x2"] = timed(lambda: lg.gemm([lg.op(S, W1, y1, H, D, D, D, H, bias=b, relu=True),
                                                       lg.op(S, W2, y2, H, D, D, D, H, bias=b, relu=True)], M, dev))
        us["ours_fwd_1088_x3"] = timed(lambda: lg.gemm([lg.op(S2, W1, y1, H, D, D, D, H, bias=b, relu=True),
                                                       lg.op(S2, W2, y2, H, D, D, D, H, bias=b, relu=True),
                                                       lg.op(S, W3, y3, H, D, D, D, H, bias=b, relu=True)], M, dev))
        zc = torch.cat([Z, act], 1)
        us["torch_fwd_130"] = timed(lambda: torch._addmm_activation(b, zc, Ws2.t()))
        us["ours_fwd_128_plus_action"] = timed(lambda: lg.gemm([lg.op(Z, Ws2, y1, H, H, H, H + 2, H, bias=b, x2=act,
                                                                      w2=(Ws2, H), nx2=2, ldx2=2, ldw2=H + 2,
                                                                      relu=True)], M, dev))
        us["torch_dgrad_128"] = timed(lambda: G.mm(Ws2))
        us["ours_dgrad_128_masked"] = timed(lambda: lg.gemm([lg.op(G, Ws2, y1, H, H, H, H + 2, H, omask=Z,
                                                                   nn=True)], M, dev))
        us["torch_wgrad_1088"] = timed(lambda: G.t().mm(S))
        dW = torch.empty(H, D, device="cuda")
        db = torch.empty(H, device="cuda")
        us["ours_wgrad_1088"] = timed(lambda: lg.wgrad([lg.wop(G, S, dW, H, D, H, D, D, db=db)], M, dev))
        us["torch_wgrad_128"] = timed(lambda: G.t().mm(Z))
        dW2 = torch.empty(H, H + 2, device="cuda")
        us["ours_wgrad_128_130_1088"] = timed(lambda: lg.wgrad([lg.wop(G, Z, dW2, H, H, H, H, H + 2, db=db),
                                                               lg.wop(G, act, (dW2, H), H, 2, H, 2, H + 2),
                                                               lg.wop(Y, S, dW, H, D, H, D, D, db=db)], M, dev))
    flops = 2.0 * M * D * H
    out["tflops"] = {k: flops * n / (us[k] * 1e-6) / 1e12 for k, n in
                     (("ours_fwd_1088", 1), ("ours_fwd_1088_x2", 2), ("ours_fwd_1088_x3", 3), ("torch_fwd_1088", 1),
                      ("ours_wgrad_1088", 1), ("torch_wgrad_1088", 1))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
