"""k_post_multi's per-block phase times (GPU box, a timing build via F110_LIB
(hipcc ... -DF110_POST_PHASES, the _build.py flags and sources):
counters 8-12 = summed wall_clock64 ticks (100 MHz) of prologue, GJK + pair
geometry, agent ray_cast, outputs + epilogue, and the block count), two-agent
envs at the C4 / C5 shapes, post_probe.py's inputs.  One JSON line (us per
block, averaged)."""
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
        c0 = [sim.read_counter(i) for i in range(8, 13)]
        for k in range(50, 250):
            sim.step(acts[k], minimal_outputs=True)
        torch.cuda.synchronize()
        c1 = [sim.read_counter(i) for i in range(8, 13)]
        nb = c1[4] - c0[4]
        us = [(c1[i] - c0[i]) / nb / 100.0 for i in range(4)]  # 100 MHz ticks -> us
        out["runs"].append({"envs": E, "blocks": nb, "us_per_block": dict(zip(
            ("prologue", "gjk_and_geometry", "agent_ray_cast", "outputs_epilogue"), us))})
        sim.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
