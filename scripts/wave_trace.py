"""Wave timeline of one ray launch (diagnostic; GPU box).

For each chunk order in WT_ORDERS (';'-separated, '' = library default),
records one traced f110_step of the 8192-env bench workload
(f110_debug_wave_trace) and prints per-order statistics: launch span, the
times by which 50/90/99/100 % of the waves had finished, per-XCD spans,
occupancy (resident waves per CU) over time, and per-chunk wave durations."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from f110_gymnasium_ros2_jazzy_amd import _lib
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

E = int(os.environ.get("WT_ENVS", 8192))
A = int(os.environ.get("WT_AGENTS", 1))
orders = os.environ.get("WT_ORDERS", ";0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16").split(";")
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", A)
rng = np.random.default_rng(12345)
p0 = sp[rng.integers(0, sp.shape[0], E)]
g = torch.Generator(device="cuda").manual_seed(0)
acts = torch.rand(120, E, A, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
res = {}
for order in orders:
    if order:
        os.environ["F110_CHUNK_ORDER"] = order
    else:
        os.environ.pop("F110_CHUNK_ORDER", None)
    sim = BatchSim(tm, n_envs=E, n_agents=A, noise_std=0.01, autoreset=True, spawn_poses=sp)
    L = sim.L
    nw = ctypes.c_int64()
    s = sim._stream()
    sim.reset(p0)
    for k in range(100):
        sim.step(acts[k], minimal_outputs=True)
    traces = []
    for rep in range(3):
        _lib.check(L.f110_debug_wave_trace(sim.ctx, 1, None, 0, ctypes.byref(nw), s), "trace arm")
        sim.step(acts[100 + rep], minimal_outputs=True)
        buf = np.zeros((nw.value, 4), np.uint64)
        _lib.check(L.f110_debug_wave_trace(sim.ctx, 0, buf.ctypes.data, nw.value, ctypes.byref(nw), s), "trace read")
        traces.append(buf)
    sim.close()
    out = []
    for buf in traces:
        live = buf[:, 1] > 0
        missing = int(np.sum(~live))
        t0 = buf[live, 0].astype(np.int64)
        t1 = buf[live, 1].astype(np.int64)
        base = t0.min()
        t0 = (t0 - base) * 10e-3  # us (100 MHz ticks)
        t1 = (t1 - base) * 10e-3
        hw = buf[live, 2]
        xcc = (hw >> np.uint64(32)).astype(np.int64)
        slot = (buf[live, 3] >> np.uint64(32)).astype(np.int64)
        dur = t1 - t0
        span = float(t1.max())
        fin = np.sort(t1)
        n = fin.size
        o = {"span_us": round(span, 2), "waves": int(n), "missing": missing,
             "t_done_50_90_99_100": [round(float(fin[int(q * (n - 1))]), 2) for q in (0.5, 0.9, 0.99, 1.0)],
             "last_start_us": round(float(t0.max()), 2),
             "mean_wave_us": round(float(dur.mean()), 3), "max_wave_us": round(float(dur.max()), 2),
             "xcc_end_us": [round(float(t1[xcc == x].max()), 1) if np.any(xcc == x) else None for x in range(8)],
             "xcc_wave_us_sum": [round(float(dur[xcc == x].sum()), 0) for x in range(8)]}
        bins = np.arange(0.0, span + 10, 10.0)  # resident waves per CU over time (10 us bins)
        o["resident_waves_per_cu_10us"] = [round(float(np.sum((t0 < b0 + 10) & (t1 > b0))) / 256, 2)
                                           for b0 in bins[:-1]]
        slots = np.unique(slot)
        o["slot_mean_wave_us"] = [round(float(dur[slot == q].mean()), 2) for q in slots]
        o["slot_end_us"] = [round(float(t1[slot == q].max()), 1) for q in slots]
        o["slot_start_us"] = [round(float(t0[slot == q].min()), 1) for q in slots]
        out.append(o)
    res[order or "default"] = out
print(json.dumps(res))
