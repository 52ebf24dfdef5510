"""k_post_multi's agent ray_cast work per step (GPU box, a counting build via
F110_LIB: counters 12 / 13 / 14 = beams enumerated from the window ranges,
beams inside the box's window, beams the pass shortened), two-agent envs at
the C4 / C5 shapes, post_probe.py's inputs.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402


def main():
    out = {"runs": []}
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
        torch.cuda.synchronize()
        c0 = [sim.read_counter(i) for i in (12, 13, 14)]
        for k in range(50, 250):
            sim.step(acts[k], minimal_outputs=True)
        torch.cuda.synchronize()
        c1 = [sim.read_counter(i) for i in (12, 13, 14)]
        n = 200 * E
        out["runs"].append({"envs": E, "enumerated_per_env": (c1[0] - c0[0]) / n,
                            "in_window_per_env": (c1[1] - c0[1]) / n, "shortened_per_env": (c1[2] - c0[2]) / n})
        sim.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
