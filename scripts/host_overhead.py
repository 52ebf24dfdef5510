"""Probe (GPU box): is the small-shard step bound by the host's submission
loop?  For each (envs, sub-shards) it times K steps twice: the submission
loop alone (perf_counter around the Python calls, no sync inside) and the
wall time to the final synchronize.  Host time close to the wall time means
the GPU waits on Python.  Prints one JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards

K = int(os.environ.get("K", "400"))
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 1)
cases = [(int(e), int(s)) for e, s in (c.split("x") for c in os.environ.get("CASES", "8192x1,8192x4,65536x2").split(","))]
for E, S in cases:
    rng = np.random.default_rng(12345)
    p0 = torch.as_tensor(sp[rng.integers(0, sp.shape[0], E)], device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(K, E, 1, 2, device="cuda", generator=g, dtype=torch.float64)
    acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
    acts[..., 1] *= 20
    kw = dict(n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp)
    if S == 1:
        sim = BatchSim(tm, n_envs=E, **kw)
        step = lambda a: sim.step(a, minimal_outputs=True)
        reset = sim.reset
    else:
        sim = StreamShards(tm, E, n_streams=S, heavy_first=os.environ.get("HF", "0") == "1", **kw)
        step = lambda a: sim.step(a, minimal_outputs=True)
        reset = sim.reset
    reset(p0)
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:  # clock ramp
        for k in range(50):
            step(acts[k])
        torch.cuda.synchronize()
    res = {"envs": E, "streams": S}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            step(acts[k])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[f"host_us_{rep}"] = (t1 - t0) / K * 1e6
        res[f"wall_us_{rep}"] = (t2 - t0) / K * 1e6
    # the C call alone (no Python around it): one context, f110_step through ctypes
    if S == 1:
        import ctypes
        from f110_gymnasium_ros2_jazzy_amd import _lib
        a = acts[0].contiguous()
        outs = sim._outs_min
        st = sim._stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            sim.L.f110_step(sim.ctx, ctypes.c_void_p(a.data_ptr()), _lib.F64, ctypes.byref(outs), st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res["raw_ctypes_host_us"] = (t1 - t0) / K * 1e6
        res["raw_ctypes_wall_us"] = (time.perf_counter() - t0) / K * 1e6
    print(json.dumps(res), flush=True)
    if S > 1:
        sim.close()
    del sim
    torch.cuda.synchronize()
