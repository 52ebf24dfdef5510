"""Kernel micro-benchmarks (times via HIP events on the launch stream)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
from f110_gymnasium_ros2_jazzy_amd.maps import load_map, centerline_spawns

def timeit(fn, n=20, warm=3):
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n

E = int(os.environ.get("MB_ENVS", 8192))
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 1)
rng = np.random.default_rng(0)
poses = sp[rng.integers(0, sp.shape[0], E), 0]
poses = poses + np.stack([rng.normal(0, .2, E), rng.normal(0, .2, E), rng.normal(0, .2, E)], 1)
sims = {}
variants = {"rowmajor": {"F110_RAY_KERNEL": "0"}, "tiled": {"F110_RAY_KERNEL": "1"}}
for K, envs in variants.items():
    os.environ.update(envs)
    sims[K] = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp, keep_f64_scans=True)
sim = sims["rowmajor"]
pt = torch.as_tensor(poses, device="cuda")
scans = torch.empty(E, 1080, dtype=torch.float64, device="cuda")
res = {}
t_end = time.time() + 2.0            # DVFS ramp: the idle GPU sits at ~450 MHz
while time.time() < t_end:
    sim.scan_batch(pt); torch.cuda.synchronize()
sim.reset_counters()
res["scan_batch_ms"] = timeit(lambda: sim.scan_batch(pt))
lk, rays = sim.read_counters(); res["lookups_per_ray"] = lk / rays
res["scan_probe_ms"] = timeit(lambda: sim.scan_batch(pt, probe=True))
os.environ["F110_SCAN_VARIANT"] = "1"
res["scan_batch_div_ms"] = timeit(lambda: sim.scan_batch(pt))
os.environ["F110_SCAN_VARIANT"] = "0"
res["scan_batch_ms_again"] = timeit(lambda: sim.scan_batch(pt))
acts = torch.rand(E, 1, 2, device="cuda"); acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189; acts[..., 1] *= 20
p0 = sp[rng.integers(0, sp.shape[0], E)]
for rnd in range(3):  # interleaved rounds (A/B in one process)
    for K, sm in sims.items():
        sm.reset(p0)
        for _ in range(30): sm.step(acts, minimal_outputs=True)
        sm.profile_begin(100)
        t = timeit(lambda: sm.step(acts, minimal_outputs=True), n=100, warm=0)
        pk = sm.profile_end()
        res.setdefault(f"step_ms_{K}", []).append(round(t, 4))
        res.setdefault(f"rays_ms_{K}", []).append(round(pk["k_rays_ms"], 4))
# parity of the variants: same inputs -> identical scans
outs = {}
for K, sm in sims.items():
    sm.reset(p0); o = sm.step(acts)
    outs[K] = o.scans_f64.clone()
res["variants_identical"] = all(bool(torch.equal(outs["rowmajor"], v)) for v in outs.values())
res["agents_ms"] = round(pk["k_agents_ms"], 4); res["post_ms"] = round(pk["k_post_ms"], 4)
print(json.dumps(res))
