"""k_post_multi probe: k_post per launch (f110_profile events) at two-agent
env counts (C4 / C5 shapes), one context, autoreset.  One JSON line.

    python scripts/post_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402


def main():
    out = {"note": "ms per launch (f110_profile events), 200 profiled steps after 50; 2 agents", "runs": []}
    track = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 2)
    for E in (4096, 8192):
        sim = BatchSim(track, n_envs=E, n_agents=2, autoreset=True, spawn_poses=sp)
        rng = np.random.default_rng(0)
        sim.reset(sp[rng.integers(0, sp.shape[0], E)])
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand(250, E, 2, 2, device="cuda", generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        for k in range(50):
            sim.step(acts[k], minimal_outputs=True)
        sim.profile_begin(200)
        for k in range(50, 250):
            sim.step(acts[k], minimal_outputs=True)
        pk = sim.profile_end()
        out["runs"].append({"envs": E, **{k: pk[k] for k in ("k_agents_ms", "k_rays_ms", "k_post_ms")}})
        print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
        sim.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
