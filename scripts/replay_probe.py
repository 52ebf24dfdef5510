"""Replay-buffer kernels at the C5 bench's shape (GPU box): a 2^20-row
prioritized buffer of 1088-float observations filled to RP_FILL rows, then
RP_STEPS rounds of the learner's pattern -- add 4096 rows, sample 4096
(keys, radix select, weights, row gather), update their priorities from
random TD errors -- on one stream.  Prints one JSON line with the ms per
round (events) and a digest of the last sample (idx, weights) so that two
builds can be checked for identical draws; run it under rocprofv3
--kernel-trace --stats for the per-kernel split.

    RP_FILL=524288 RP_STEPS=200 python scripts/replay_probe.py
"""
import json
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.replay import DeviceReplayBuffer  # noqa: E402


def main():
    fill = int(os.environ.get("RP_FILL", 1 << 19))
    steps = int(os.environ.get("RP_STEPS", 200))
    B, D, N = 4096, 1088, 4096
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    rb = DeviceReplayBuffer(1 << 20, B, obs_dim=D, device=dev, max_add=1 << 16)
    s = torch.rand(N, D, device=dev, generator=g)
    ns = torch.rand(N, D, device=dev, generator=g)
    a = torch.rand(N, 2, device=dev, generator=g)
    r = torch.rand(N, device=dev, generator=g)
    d = torch.zeros(N, device=dev)
    while rb._added < fill:
        rb.add(s, a, r, ns, d)
    td = torch.randn(steps + 20, B, device=dev, generator=g)

    def round_(k):
        rb.add(s, a, r, ns, d)
        idx, _, w = rb.sample(0.4)
        rb.update_priorities(idx, td[k], td_errors=True, add_eps=1e-6)
        return idx, w

    for k in range(20):
        round_(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(steps):
        idx, w = round_(20 + k)
    e1.record()
    torch.cuda.synchronize()
    dig = zlib.crc32(idx.cpu().numpy().tobytes() + w.cpu().numpy().tobytes())
    print(json.dumps({"fill": fill, "steps": steps, "ms_per_round": e0.elapsed_time(e1) / steps,
                      "length": len(rb), "digest": dig}), flush=True)
    rb.close()


if __name__ == "__main__":
    main()
