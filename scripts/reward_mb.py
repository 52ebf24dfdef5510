"""Micro-benchmark of k_reward (GPU box): the train_ddpg configuration at
8192 two-agent envs on real observations, and the same with the wall term
(grace_steps_wall = 1e9) or the projection (no progress track) switched
off, to attribute its time.  Prints one JSON line (us per call)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import MAP_DIR, centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.reward import BatchedCenterlineReward, CenterlineTrack
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
from f110_gymnasium_ros2_jazzy_amd.train import REWARD_KW

E, A = 8192, 2
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", A)
rng = np.random.default_rng(1)
sim = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp)
sim.reset(sp[rng.integers(0, sp.shape[0], E)])
acts = np.stack([rng.uniform(-0.2, 0.2, (E, A)), rng.uniform(2, 8, (E, A))], -1).astype(np.float32)
for _ in range(30):
    out = sim.step(acts)
obs = out.obs.clone()
cl = np.load(os.path.join(MAP_DIR, "Spielberg_centerline.npz"))
track = CenterlineTrack(cl["xy"], cl["w_right"], cl["w_left"], device=0)


def time_reward(**over):
    kw = dict(REWARD_KW)
    kw.update(over)
    prog = kw.pop("progress", track)
    rf = BatchedCenterlineReward(E, dt=0.01, progress=prog, device="cuda:0", **kw)
    for _ in range(30):  # past the grace steps
        rf(obs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        rf(obs)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / 50 * 1000, 1)


res = {"full_us": time_reward(), "no_wall_us": time_reward(grace_steps_wall=10 ** 9),
       "no_progress_us": time_reward(progress=None), "full_again_us": time_reward()}
print(json.dumps(res))

# how far the observed cars are from the centerline (the grid search falls
# back to a full scan when the 5th nearest midpoint is beyond the 3x3 block)
B = 1080
o = obs.reshape(E, -1).double().cpu().numpy()
pts = np.concatenate([o[:, B:B + 2], o[:, B + 4:B + 6]])
mid = 0.5 * (cl["xy"][1:] + cl["xy"][:-1])
d = np.sqrt(((pts[:, None, :] - mid[None, :, :]) ** 2).sum(-1))
d5 = np.sort(d, 1)[:, 4]
gx0 = mid[:, 0].min() - 4.0
gy0 = mid[:, 1].min() - 4.0
fx = (pts[:, 0] - gx0) / 4.0 - np.floor((pts[:, 0] - gx0) / 4.0)
fy = (pts[:, 1] - gy0) / 4.0 - np.floor((pts[:, 1] - gy0) / 4.0)
lb = 4.0 + 4.0 * np.minimum(np.minimum(fx, 1 - fx), np.minimum(fy, 1 - fy))
print(json.dumps({"d5_quantiles": np.quantile(d5, [0.5, 0.9, 0.99, 1.0]).round(2).tolist(),
                  "fallback_frac": float(np.mean(d5 >= lb)), "n": int(len(d5))}))
