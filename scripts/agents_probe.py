"""k_agents latency probe: the per-launch time of k_agents (HIP events of
f110_profile_*) at several car counts, RK4 vs Euler integrator, one agent,
autoreset on, centerline spawns, uniform random actions.  One JSON line.

    python scripts/agents_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd import _lib  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402


def main():
    out = {"note": "k_agents ms per launch (f110_profile events), 200 profiled steps after 50", "runs": []}
    track = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)
    for integ, name in ((_lib.INTEGRATOR_RK4, "rk4"), (_lib.INTEGRATOR_EULER, "euler")):
        for E in (256, 4096, 65536):
            sim = BatchSim(track, n_envs=E, n_agents=1, integrator=integ, autoreset=True, spawn_poses=sp)
            rng = np.random.default_rng(0)
            sim.reset(sp[rng.integers(0, sp.shape[0], E)])
            g = torch.Generator(device="cuda").manual_seed(0)
            acts = torch.rand(250, E, 1, 2, device="cuda", generator=g)
            acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
            acts[..., 1] *= 20
            for k in range(50):
                sim.step(acts[k], minimal_outputs=True)
            sim.profile_begin(200)
            for k in range(50, 250):
                sim.step(acts[k], minimal_outputs=True)
            pk = sim.profile_end()
            out["runs"].append({"integrator": name, "envs": E, **{k: pk[k] for k in ("k_agents_ms", "k_rays_ms",
                                                                                     "k_post_ms")}})
            sim.close()
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
