"""The small-shard floor: the ray kernel for cars whose longest ray is known
(offline, oracle tables), alone and in growing batches, per dependent step.
Poses: 8192 centerline spawns (seed 0, yaw jitter 0.3 rad) as in DESIGN 3.9;
the car with the longest ray is replicated n times (the same lines, cache-warm
after the first step) or the first n poses are used (distinct cars)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np, torch
import oracle as O
from f110_gymnasium_ros2_jazzy_amd.maps import load_map, centerline_spawns
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

tm = load_map("Spielberg_map")
sc = O.OracleScanner(tm.free_mask, tm.resolution, tm.origin)
sp = centerline_spawns("Spielberg", 1)
rng = np.random.default_rng(0)
poses = sp.reshape(sp.shape[0], -1)[rng.integers(0, sp.shape[0], 8192)][:, :3].copy()
poses[:, 2] += rng.uniform(-0.3, 0.3, len(poses))
_, look, _ = sc.scan(poses, with_probe=True, threads=8)
cm = look.max(1)
worst = int(np.argmax(cm))
res = {"longest_ray": int(cm.max()), "per_car_longest_mean": float(cm.mean())}


def run(p, steps=50):
    E = p.shape[0]
    sim = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.0, autoreset=False, seed=1)
    sim.reset(p[:, None, :].copy())
    zero = torch.zeros(E, 1, 2, device="cuda")
    for _ in range(10):
        sim.step(zero, minimal_outputs=True)
    torch.cuda.synchronize()
    sim.reset_counters()
    sim.profile_begin(steps)
    for _ in range(steps):
        sim.step(zero, minimal_outputs=True)
    pk = sim.profile_end()
    lk, rays = sim.read_counters()
    rk, rf = sim.ray_kernel, sim.ray_refill
    sim.close()
    return {"k_rays_ms": pk["k_rays_ms"], "k_agents_ms": pk["k_agents_ms"], "k_post_ms": pk["k_post_ms"],
            "mean_lookups": lk / max(rays, 1), "ray_kernel": rk, "ray_refill": rf}


for n in (1, 64, 1024, 8192):
    r = run(np.repeat(poses[worst:worst + 1], n, 0))
    r["us_per_step_of_longest"] = r["k_rays_ms"] * 1e3 / cm.max()
    res[f"worst_car_x{n}"] = r
for n in (64, 1024, 4096, 8192):
    r = run(poses[:n])
    r["longest_in_batch"] = int(cm[:n].max())
    r["us_per_step_of_longest"] = r["k_rays_ms"] * 1e3 / cm[:n].max()
    res[f"first_{n}"] = r
print(json.dumps(res))
