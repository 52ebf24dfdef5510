"""C4 (8192 envs x 2 agents) on one context for rocprofv3 --kernel-trace
(GPU box): C4_STEPS steps after a 1 s clock ramp; prints ms per step.

    rocprofv3 --kernel-trace -d out -- python scripts/c4_trace.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402

E = int(os.environ.get("C4_ENVS", 8192))
A = int(os.environ.get("C4_AGENTS", 2))
K = int(os.environ.get("C4_STEPS", 100))
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", A, gap=25)
p0 = sp[np.random.default_rng(1).integers(0, sp.shape[0], E)]
g = torch.Generator(device="cuda")
g.manual_seed(0)
acts = torch.rand(K + 20, E, A, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
r = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=7)
r.reset(p0)
t_end = time.perf_counter() + 1.0
k = 0
while time.perf_counter() < t_end:
    r.step(acts[k % 20], minimal_outputs=True)
    k += 1
    if k % 16 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in range(K):
    r.step(acts[s], minimal_outputs=True)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"envs": E, "agents": A, "steps": K, "ms_per_step": el / K * 1e3, "env_steps_per_s": E * K / el,
                  "ray_refill": r.ray_refill}))
r.close()
