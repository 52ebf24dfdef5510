"""A/B of two libf110 builds in one process (GPU box): the current build and
an alternate one (AB_LIB, e.g. ab_libs/head.so from scripts/build_ab_lib.sh: an earlier
commit), each loaded once (ctypes, local symbols), their contexts stepped in
interleaved rounds on the same poses and actions.  Per build and size: the
per-kernel times of the one-context runner (HIP events on each kernel's own
dispatch, median over rounds), the wall time per step of the one-context and
the bench's stream sub-shard runner (bench.auto_streams), and whether the two
builds' outputs are bit-identical (obs, f64 scans, states after 40 steps with
noise, autoreset and a masked reset).  Prints one JSON line.

    AB_LIB=ab_libs/head.so AB_ENVS=65536,8192 python scripts/lib_ab.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd import _build, _lib  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards  # noqa: E402


def load_lib(path):
    _lib._lib = None
    if path == _build.LIB:
        os.environ.pop("F110_LIB", None)
    else:
        os.environ["F110_LIB"] = path
    L = _lib.load(build_if_missing=False)
    _lib._lib = None
    os.environ.pop("F110_LIB", None)
    return L


def with_lib(L, fn):
    _lib._lib = L
    try:
        return fn()
    finally:
        _lib._lib = None


def main():
    envs = [int(x) for x in os.environ.get("AB_ENVS", "65536,8192").split(",")]
    A = int(os.environ.get("AB_AGENTS", 1))
    steps = int(os.environ.get("AB_STEPS", 100))
    rounds = int(os.environ.get("AB_ROUNDS", 3))
    libs = {"new": _build.LIB, "alt": os.path.join(REPO, os.environ.get("AB_LIB", "ab_libs/head.so"))}
    Ls = {n: load_lib(p) for n, p in libs.items()}
    tm = load_map("Spielberg_map")
    tm.ensure_edt()
    sp = centerline_spawns("Spielberg", A)
    dev = torch.device("cuda:0")
    kw = dict(n_agents=A, device=dev, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=7, keep_f64_scans=True)
    res = {"agents": A, "libs": libs, "by_envs": {}}
    for E in envs:
        rng = np.random.default_rng(12345)
        p0 = sp[rng.integers(0, sp.shape[0], E)]
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        acts = torch.rand(40 + steps, E, A, 2, device=dev, generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        one = {n: with_lib(L, lambda: BatchSim(tm, n_envs=E, **kw)) for n, L in Ls.items()}
        S = bench.auto_streams(E, A)
        shards = {n: with_lib(L, lambda: StreamShards(tm, n_envs=E, n_streams=S, **kw)) for n, L in Ls.items()}
        mask = torch.zeros(E, dtype=torch.uint8, device=dev)
        mask[::3] = 1
        snaps = {}
        for n, sm in one.items():
            sm.reset(p0)
            for k in range(40):
                if k == 20:
                    sm.reset(p0, env_mask=mask)
                sm.step(acts[k])
            torch.cuda.synchronize()
            snaps[n] = [sm.out.obs.clone(), sm.out.scans_f64.clone(), sm.agent_states().clone(), sm.out.collisions.clone()]
        ident = all(torch.equal(a, b) for a, b in zip(snaps["new"], snaps["alt"]))
        kt = {n: [] for n in Ls}
        wall_one = {n: [] for n in Ls}
        wall_sh = {n: [] for n in Ls}
        for _ in range(rounds):
            for n in Ls:
                sm = one[n]
                sm.reset(p0)
                for k in range(30):
                    sm.step(acts[k], minimal_outputs=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(steps):
                    sm.step(acts[40 + k], minimal_outputs=True)
                torch.cuda.synchronize()
                wall_one[n].append((time.perf_counter() - t0) / steps * 1e3)
                sm.profile_begin(steps)
                for k in range(steps):
                    sm.step(acts[40 + k], minimal_outputs=True)
                kt[n].append(sm.profile_end())
                sh = shards[n]
                sh.reset(p0)
                for k in range(30):
                    sh.step(acts[k], minimal_outputs=True)
                sh.join()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(steps):
                    sh.step(acts[40 + k], minimal_outputs=True)
                sh.join()
                torch.cuda.synchronize()
                wall_sh[n].append((time.perf_counter() - t0) / steps * 1e3)
        line = {"identical": ident, "streams": S}
        for n in Ls:
            line[n] = {key: float(np.median([t[key] for t in kt[n]])) for key in ("k_agents_ms", "k_rays_ms", "k_post_ms")}
            line[n]["one_context_step_ms"] = float(np.median(wall_one[n]))
            line[n]["shards_step_ms"] = float(np.median(wall_sh[n]))
            line[n]["shards_env_steps_per_s"] = E / (line[n]["shards_step_ms"] * 1e-3)
        res["by_envs"][str(E)] = line
        for x in list(one.values()) + list(shards.values()):
            x.close()
        torch.cuda.empty_cache()
        print(json.dumps({"E": E, **line}), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
