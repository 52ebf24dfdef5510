"""A/B of ray-kernel variants in one process (GPU box): per-kernel times
(HIP events on each kernel's own dispatch, interleaved rounds) and a
bit-identity check of every variant's outputs against the first one (obs, f64
scans, states, collisions after the same steps, noise + autoreset on, a masked
reset in the middle).  Prints one JSON line.

A variant is `name:KEY=V,KEY=V`; keys: F110_RAY_KERNEL / F110_FX_PAD (env at
create; F110_FXS_SG: k_rays_fxs's scalar gathers), LANES (f110_debug_set_ray_lanes), REFILL (f110_debug_set_ray_refill), HEAVY=0
(f110_debug_disable_heavy_first), NOISE.

    AB_ENVS=8192,65536 AB_VARIANTS='fxn:REFILL=0,LANES=2;fxs:REFILL=1,LANES=2' python scripts/ray_ab.py
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

ENV_KNOBS = ("F110_RAY_KERNEL", "F110_FX_PAD", "F110_FXS_SG", "F110_FX_SG")


def parse_variants(spec):
    out = {}
    for item in spec.split(";"):
        if not item.strip():
            continue
        name, _, kv = item.partition(":")
        env = {}
        for pair in kv.split(","):
            if "=" in pair:
                k, v = pair.split("=", 1)
                env[k.strip()] = v.strip()
        out[name.strip()] = env
    return out


def make(tm, sp, E, A, spec, **kw):
    for k in ENV_KNOBS:
        os.environ.pop(k, None)
    os.environ.update({k: v for k, v in spec.items() if k in ENV_KNOBS})
    noise = float(spec.get("NOISE", os.environ.get("AB_NOISE", "0.01")))
    sm = BatchSim(tm, n_envs=E, n_agents=A, noise_std=noise, autoreset=True, spawn_poses=sp, seed=7,
                  keep_f64_scans=True, **kw)
    for k in ENV_KNOBS:
        os.environ.pop(k, None)
    if "LANES" in spec:
        sm.set_ray_lanes(int(spec["LANES"]))
    if "REFILL" in spec:
        sm.set_ray_refill(int(spec["REFILL"]))
    if spec.get("HEAVY") == "0":
        sm.disable_heavy_first()
    return sm


def snapshot(sm):
    torch.cuda.synchronize()
    return {"obs": sm.out.obs.clone(), "scans_f64": sm.out.scans_f64.clone(), "state": sm.agent_states().clone(),
            "col": sm.out.collisions.clone(), "term": sm.out.terminated.clone()}


def main():
    envs = [int(x) for x in os.environ.get("AB_ENVS", "8192").split(",")]
    A = int(os.environ.get("AB_AGENTS", 1))
    variants = parse_variants(os.environ.get("AB_VARIANTS", "k2:F110_RAY_KERNEL=2;k3:F110_RAY_KERNEL=3"))
    steps = int(os.environ.get("AB_STEPS", 100))
    rounds = int(os.environ.get("AB_ROUNDS", 3))
    simt = os.environ.get("AB_SIMT") == "1"
    tm = load_map(os.environ.get("AB_MAP", "Spielberg_map"))
    sp = centerline_spawns(os.environ.get("AB_MAP", "Spielberg_map").replace("_map", ""), A)
    res = {"agents": A, "variants": variants, "by_envs": {}}
    for E in envs:
        rng = np.random.default_rng(12345)
        p0 = sp[rng.integers(0, sp.shape[0], E)]
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        acts = torch.rand(40 + steps, E, A, 2, device="cuda", generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        sims = {n: make(tm, sp, E, A, spec) for n, spec in variants.items()}
        kernels = {n: {"ray_kernel": sm.ray_kernel, "lanes": sm.ray_lanes, "refill": sm.ray_refill}
                   for n, sm in sims.items()}
        # bit identity: 40 steps with every output, plus a masked reset in the middle
        ref = None
        ident = {}
        mask = torch.zeros(E, dtype=torch.uint8, device="cuda")
        mask[::3] = 1
        for n, sm in sims.items():
            sm.reset(p0)
            for k in range(40):
                if k == 20:
                    sm.reset(p0, env_mask=mask)
                sm.step(acts[k])
            snap = snapshot(sm)
            if ref is None:
                ref = snap
                ident[n] = True
            else:
                ident[n] = all(bool(torch.equal(snap[f], ref[f])) for f in snap)
                if not ident[n]:
                    ident[n + "_diff"] = {f: int((snap[f] != ref[f]).sum()) for f in snap}
        # timing: interleaved rounds, minimal outputs (the bench's timed mode)
        times = {n: [] for n in sims}
        look = {}
        diag = {}
        for _ in range(rounds):
            for n, sm in sims.items():
                sm.reset(p0)
                for k in range(30):
                    sm.step(acts[k], minimal_outputs=True)
                torch.cuda.synchronize()
                sm.reset_counters()
                sm.profile_begin(steps)
                for k in range(steps):
                    sm.step(acts[40 + k], minimal_outputs=True)
                pk = sm.profile_end()
                lk, rays = sm.read_counters()
                look[n] = lk / max(rays, 1)
                times[n].append(pk)
        if simt:  # counters in a separate pass (their atomics are not part of the timed launches)
            for n, sm in sims.items():
                sm.reset(p0)
                sm.set_simt(True)
                sm.reset_counters()
                for k in range(steps):
                    sm.step(acts[40 + k], minimal_outputs=True)
                lk, rays = sm.read_counters()
                slots = sm.read_counter(2)
                cars = E * A * steps
                sg = sm.read_counter(4)  # lookups gathered by scalar loads (k_rays_fxs, SG > 0)
                diag[n] = {"simt": (lk - rays - sg) / max(slots, 1), "slot_gathers_per_car": slots / 64 / cars,
                           "other_loads_per_car": sm.read_counter(3) / cars, "scalar_gathers_per_car": sg / cars,
                           "closed_slot_trips_per_car": sm.read_counter(5) / cars}
                sm.set_simt(False)
        line = {"kernels": kernels, "identical": ident, "mean_lookups": look, "diag": diag}
        for n, ts in times.items():
            line[n] = {key: float(np.median([t[key] for t in ts])) for key in ts[0]}
        res["by_envs"][str(E)] = line
        for sm in sims.values():
            sm.close()
        del sims
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
