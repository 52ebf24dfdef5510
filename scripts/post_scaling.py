"""k_post_multi time vs env count (GPU box): a flat curve means one long
env (a tail) sets the kernel time, a linear one means throughput.  Two-agent
envs, uniform random actions (train_ddpg warm-up), 100 timed steps."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 2)
res = {}
for E in (64, 1024, 8192):
    rng = np.random.default_rng(0)
    sim = BatchSim(tm, n_envs=E, n_agents=2, noise_std=0.01, autoreset=True, spawn_poses=sp)
    sim.reset(sp[rng.integers(0, sp.shape[0], E)])
    acts = torch.rand(130, E, 2, 2, device="cuda")
    acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
    acts[..., 1] *= 20
    for k in range(30):
        sim.step(acts[k], minimal_outputs=True)
    sim.profile_begin(100)
    for k in range(100):
        sim.step(acts[30 + k], minimal_outputs=True)
    torch.cuda.synchronize()
    p = sim.profile_end()
    res[E] = {"k_agents_us": round(p["k_agents_ms"] * 1e3, 1), "k_rays_us": round(p["k_rays_ms"] * 1e3, 1),
              "k_post_us": round(p["k_post_ms"] * 1e3, 1)}
    sim.close()
print(json.dumps(res))
