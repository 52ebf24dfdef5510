"""k_gap_follow time vs scan count (GPU box), on the scans of a two-agent
sim after 100 random-action steps.  Prints one JSON line (us per call)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.opponent import gap_follow
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

E = 8192
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 2)
rng = np.random.default_rng(0)
sim = BatchSim(tm, n_envs=E, n_agents=2, noise_std=0.01, autoreset=True, spawn_poses=sp)
sim.reset(sp[rng.integers(0, sp.shape[0], E)])
acts = torch.rand(100, E, 2, 2, device="cuda")
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
for k in range(100):
    out = sim.step(acts[k])
scans = out.scans[:, 1].contiguous()
res = {}
for M in (64, 1024, 8192):
    s = scans[:M]
    for _ in range(5):
        gap_follow(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        gap_follow(s)
    e1.record()
    torch.cuda.synchronize()
    res[M] = round(e0.elapsed_time(e1) / 50 * 1000, 1)
print(json.dumps(res))
