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

E, A = int(os.environ.get("RMB_E", 8192)), 2
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", A)
rng = np.random.default_rng(1)
sim = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp)
sim.reset(sp[rng.integers(0, sp.shape[0], E)])
MODE = os.environ.get("RMB_ACTIONS", "gentle")  # "train": uniform over the action box, as train_ddpg's warm-up
for t in range(int(os.environ.get("RMB_STEPS", 30))):
    if MODE == "train":
        acts = np.stack([rng.uniform(-0.4189, 0.4189, (E, A)), rng.uniform(0, 20, (E, A))], -1).astype(np.float32)
    else:
        acts = np.stack([rng.uniform(-0.2, 0.2, (E, A)), rng.uniform(2, 8, (E, A))], -1).astype(np.float32)
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


if os.environ.get("RMB_ONLY_FULL"):  # profiler runs: the full reward only
    res = {"full_us": time_reward()}
else:
    res = {"full_us": time_reward(), "no_wall_us": time_reward(grace_steps_wall=10 ** 9),
           "no_progress_us": time_reward(progress=None), "full_again_us": time_reward()}
print(json.dumps(res))

# which search each projected point takes (the kernel's grid logic, restated:
# cells of 16 median segment lengths, (2r+1)^2 blocks for r = 1, 2, 4, full
# scan otherwise)
B = 1080
o = obs.reshape(E, -1).double().cpu().numpy()
pts = np.concatenate([o[:, B:B + 2], o[:, B + 4:B + 6]])
xy = cl["xy"]
mid = 0.5 * (xy[1:] + xy[:-1])
seg = np.hypot(*(xy[1:] - xy[:-1]).T)
h = 16.0 * np.sort(seg)[len(seg) // 2]
gx0, gy0 = mid[:, 0].min() - h, mid[:, 1].min() - h
gnx = int((mid[:, 0].max() - gx0) / h) + 2
gny = int((mid[:, 1].max() - gy0) / h) + 2
d = np.sqrt(((pts[:, None, :] - mid[None, :, :]) ** 2).sum(-1))
d5 = np.sort(d, 1)[:, 4]
fx, fy = (pts[:, 0] - gx0) / h, (pts[:, 1] - gy0) / h
ci, cj = np.clip(np.floor(fx), 0, gnx - 1), np.clip(np.floor(fy), 0, gny - 1)  # off-grid: from the edge cell
path = np.full(len(pts), -1)
for r in (1, 2, 4):
    lb = np.full(len(pts), np.inf)
    m = ci - r >= 0
    lb[m] = np.minimum(lb[m], (pts[m, 0] - (gx0 + (ci[m] - r) * h)))
    m = ci + r < gnx
    lb[m] = np.minimum(lb[m], gx0 + (ci[m] + r + 1) * h - pts[m, 0])
    m = cj - r >= 0
    lb[m] = np.minimum(lb[m], (pts[m, 1] - (gy0 + (cj[m] - r) * h)))
    m = cj + r < gny
    lb[m] = np.minimum(lb[m], gy0 + (cj[m] + r + 1) * h - pts[m, 1])
    ok = (path < 0) & (d5 < lb)
    path[ok] = r
print(json.dumps({"h": round(float(h), 3), "d5_quantiles": np.quantile(d5, [0.5, 0.9, 0.99, 1.0]).round(2).tolist(),
                  "r1": int((path == 1).sum()), "r2": int((path == 2).sum()), "r4": int((path == 4).sum()),
                  "full_scan": int((path < 0).sum()), "n": int(len(d5)),
                  "full_scan_examples": pts[path < 0][:5].round(2).tolist()}))
