"""Study (GPU box): how much of a ray wave's lanes idle on the longest ray,
and how much of that a per-car beam permutation sorted by the PREVIOUS
step's per-ray lookup counts would recover.  Prints one JSON line:
wave-iterations per car (sum over its 17 waves of the wave's max lookups)
for consecutive beams (today), beams sorted by this step's counts (ideal)
and by the previous step's counts (realisable)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

E = 8192
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 1)
rng = np.random.default_rng(12345)
p0 = sp[rng.integers(0, sp.shape[0], E)]
sim = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp)
g = torch.Generator(device="cuda").manual_seed(0)
acts = torch.rand(200, E, 1, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
sim.reset(p0)


def counts():
    st = sim.agent_states()[:, 0]
    pose = torch.stack([st[:, 0], st[:, 1], st[:, 4]], 1)
    _, look, _ = sim.scan_batch(pose, probe=True)
    L = torch.zeros(E, 17 * 64, dtype=torch.int32, device="cuda")
    L[:, :look.shape[1]] = look
    return L


def waveit(L):
    return L.view(E, 17, 64).max(-1).values.sum(-1).double().mean().item()


res = {}
prev = counts()
for t in range(120):
    sim.step(acts[t], minimal_outputs=True)
    cur = counts()
    if t in (1, 30, 100, 119):
        own = torch.sort(cur, 1, descending=True).values
        perm = torch.argsort(prev, 1, descending=True)
        pv = torch.gather(cur, 1, perm)
        # 2-byte buckets: a counting sort on min(count, 63) (what a cheap device sort would do)
        perm63 = torch.sort(prev.clamp(max=63), dim=1, descending=True, stable=True).indices
        pv63 = torch.gather(cur, 1, perm63)
        res[f"t{t}"] = {"lookups_per_car_over_64": round(cur.sum(1).double().mean().item() / 64, 2),
                        "consecutive": round(waveit(cur), 2), "sorted_own": round(waveit(own), 2),
                        "sorted_prev": round(waveit(pv), 2), "sorted_prev_clamp63": round(waveit(pv63), 2)}
    prev = cur
print(json.dumps(res))
