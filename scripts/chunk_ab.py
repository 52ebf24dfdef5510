"""A/B of the ray-kernel dispatch orders in one process (GPU box):
flat ray order (F110_RAY_KERNEL=1) vs chunked centre-out (=2) vs chunked in
the order of measured per-chunk cost.  Also per-chunk lookup statistics of the
bench poses (mean lookups, mean wave max) and a bit-identity check of the
variants' outputs.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

E = int(os.environ.get("AB_ENVS", 8192))
A = int(os.environ.get("AB_AGENTS", 1))
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", A)
rng = np.random.default_rng(12345)
p0 = sp[rng.integers(0, sp.shape[0], E)]

# per-chunk cost of the bench poses (probe lookups per ray)
os.environ["F110_RAY_KERNEL"] = "1"
probe = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp)
poses = torch.as_tensor(p0[:, 0], device="cuda")
look = None
res = {}
try:
    out = probe.scan_batch(poses, probe=True)
    look = out[1] if isinstance(out, tuple) else None
except Exception as exc:  # probe API differences: record and continue
    res["probe_error"] = repr(exc)
if look is not None:
    L = look.reshape(E, -1).cpu().numpy().astype(np.float64)
    B = L.shape[1]
    nch = (B + 63) // 64
    mean_c, wmax_c = [], []
    for k in range(nch):
        blk = L[:, k * 64:(k + 1) * 64]
        mean_c.append(float(blk.mean()))
        wmax_c.append(float(blk.max(1).mean()))
    res["chunk_mean_lookups"] = [round(x, 2) for x in mean_c]
    res["chunk_mean_wave_max"] = [round(x, 2) for x in wmax_c]
    order = list(np.argsort(-np.asarray(wmax_c), kind="stable"))
    res["measured_order"] = [int(k) for k in order]
    os.environ["F110_CHUNK_ORDER"] = ",".join(str(int(k)) for k in order)
probe.close()

DESC = ",".join(str(k) for k in range(16, -1, -1))
variants = {"flat": {"F110_RAY_KERNEL": "1"},
            "chunk_desc": {"F110_RAY_KERNEL": "2", "F110_CHUNK_ORDER": DESC, "F110_HEAVY_T": "0"},
            "chunk_asc": {"F110_RAY_KERNEL": "2", "F110_CHUNK_ORDER": ",".join(str(k) for k in range(17)),
                          "F110_HEAVY_T": "0"},
            "heavy12": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "12"},
            "heavy16": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "16"},
            "heavy20": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "20"},
            "heavy24": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24"},
            "heavy24_wpb4": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24", "F110_RAY_WPB": "4"},
            "heavy24_div12": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24", "F110_HEAVY_DIV": "12"},
            "heavy24_div16": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24", "F110_HEAVY_DIV": "16"},
            "heavy20_div8": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "20"},
            "heavy16_div6": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "16", "F110_HEAVY_DIV": "6"},
            "heavy20_div6": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "20", "F110_HEAVY_DIV": "6"},
            "heavy16_div4": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "16", "F110_HEAVY_DIV": "4"},
            "heavy24_asc": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24",
                            "F110_CHUNK_ORDER": ",".join(str(k) for k in range(17))},
            "heavy24_centre": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "24",
                               "F110_CHUNK_ORDER": "8,9,7,10,6,11,5,12,4,13,3,14,2,15,1,16,0"},
            "heavy32": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "32"},
            "heavy40": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "40"},
            "heavy64": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "64"},
            "heavy40_asc": {"F110_RAY_KERNEL": "2", "F110_HEAVY_T": "40",
                            "F110_CHUNK_ORDER": ",".join(str(k) for k in range(17))}}
if os.environ.get("AB_ONLY"):
    variants = {k: v for k, v in variants.items() if k in os.environ["AB_ONLY"].split(",")}
sims = {}
for name, env in variants.items():
    for k in ("F110_RAY_KERNEL", "F110_CHUNK_ORDER", "F110_HEAVY_T", "F110_RAY_WPB", "F110_HEAVY_DIV"):
        os.environ.pop(k, None)
    os.environ.update(env)
    sims[name] = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp,
                          keep_f64_scans=True)

g = torch.Generator(device="cuda").manual_seed(0)
acts = torch.rand(200, E, A, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
for sm in sims.values():  # DVFS ramp + warm
    sm.reset(p0)
    for k in range(100):
        sm.step(acts[k], minimal_outputs=True)
torch.cuda.synchronize()
for rnd in range(3):
    for name, sm in sims.items():
        sm.reset(p0)
        for k in range(30):
            sm.step(acts[k], minimal_outputs=True)
        sm.profile_begin(150)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(150):
            sm.step(acts[30 + k], minimal_outputs=True)
        e1.record()
        torch.cuda.synchronize()
        pk = sm.profile_end()
        res.setdefault(f"step_ms_{name}", []).append(round(e0.elapsed_time(e1) / 150, 4))
        res.setdefault(f"rays_ms_{name}", []).append(round(pk["k_rays_ms"], 4))
# bit identity of the variants after the same 40 steps
outs = {}
for name, sm in sims.items():
    sm.reset(p0)
    for k in range(40):
        o = sm.step(acts[k])
    torch.cuda.synchronize()
    outs[name] = (o.scans_f64.clone(), o.obs.clone(), sm.agent_states().clone())
ref = next(iter(outs.values()))
res["variants_identical"] = all(all(torch.equal(a, b) for a, b in zip(ref, v)) for v in outs.values())
print(json.dumps(res))
