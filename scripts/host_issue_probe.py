"""Host issue rate vs GPU time at small shards (GPU box): env-steps/s of one
BatchSim context stepped (a) one f110_step call per step from Python, (b) by
f110_step_n over the same resident action block (no host work between steps),
and of the bench's stream sub-shards (one f110_step per sub-shard per step),
plus the host's own time per f110_step call with the GPU kept busy.  If (b) is
well above (a) the host's per-call issue cost bounds the small shards.

    HP_ENVS=8192,4096 python scripts/host_issue_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    tm = load_map("Spielberg_map")
    tm.ensure_edt()
    sp = centerline_spawns("Spielberg", 1)
    K, W = 300, 30
    out = {}
    for E in [int(x) for x in os.environ.get("HP_ENVS", "8192,4096").split(",")]:
        p0 = sp[np.random.default_rng(1).integers(0, sp.shape[0], E)]
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        acts = torch.rand(W + K, E, 1, 2, device=dev, generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        kw = dict(n_agents=1, device=dev, noise_std=0.01, autoreset=True, spawn_poses=sp)
        one = BatchSim(tm, n_envs=E, **kw)
        sh = StreamShards(tm, n_envs=E, n_streams=bench.auto_streams(E, 1), **kw)
        res = {}
        for rnd in range(3):
            for name, r in (("one_per_call", one), ("one_step_n", one), ("shards_per_call", sh)):
                r.reset(p0)
                t_end = time.perf_counter() + 0.5
                while time.perf_counter() < t_end:
                    for k in range(W):
                        r.step(acts[k], minimal_outputs=True)
                    torch.cuda.synchronize()
                r.reset(p0)
                for k in range(W):
                    r.step(acts[k], minimal_outputs=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if name == "one_step_n":
                    r.step_n(acts[W:], minimal_outputs=True)
                    host = time.perf_counter() - t0
                else:
                    for k in range(W, W + K):
                        r.step(acts[k], minimal_outputs=True)
                    host = time.perf_counter() - t0
                    if hasattr(r, "join"):
                        r.join()
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
                res.setdefault(name, []).append((E * K / t, host / K * 1e6))
        out[str(E)] = {n: {"env_steps_per_s": float(np.median([v[0] for v in vs])),
                           "host_us_per_step_call": float(np.median([v[1] for v in vs]))} for n, vs in res.items()}
        one.close()
        sh.close()
        print(json.dumps({"E": E, **out[str(E)]}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
