"""Wave timeline of the ray launch of one step (diagnostic; GPU box).

For each size in WT_ENVS, the bench workload (Spielberg, random actions,
noise, autoreset) runs 100 warm-up steps, then one traced step
(f110_debug_wave_trace: per wave start / end s_memrealtime stamps, 100 MHz, on
one clock for every context of the device).  Modes (WT_MODE):
  one     one BatchSim context (the ray kernel f110_create picks for the size)
  shards  streams.StreamShards as bench.py runs it (auto_streams sub-shards,
          their ray launches traced in the same step, on one common clock)
Per launch it prints: span, the times by which 50 / 90 / 99 / 100 % of the
waves had ended, the in-flight wave count over time (40 bins), and the split
into ramp (until >= 90 % of the peak in-flight waves run), steady state and
tail (after in-flight drops below 90 % of the peak for good).  One JSON line.

    WT_ENVS=8192,65536 WT_MODE=one python scripts/wave_trace.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd import _lib  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def read_trace(sm, arm):
    nw = ctypes.c_int64()
    s = sm._stream()
    if arm:
        _lib.check(sm.L.f110_debug_wave_trace(sm.ctx, 1, None, 0, ctypes.byref(nw), s), "trace arm")
        return None
    _lib.check(sm.L.f110_debug_wave_trace(sm.ctx, 0, None, 0, ctypes.byref(nw), s), "trace size")
    buf = np.zeros((nw.value, 4), np.uint64)
    _lib.check(sm.L.f110_debug_wave_trace(sm.ctx, 0, buf.ctypes.data, nw.value, ctypes.byref(nw), s), "trace read")
    return buf[buf[:, 1] > 0]


def summarize(t0, t1, bins=40):
    base = t0.min()
    s = (t0 - base).astype(np.float64) * TICK_US
    e = (t1 - base).astype(np.float64) * TICK_US
    span = float(e.max())
    grid = np.linspace(0.0, span, 400)
    inflight = np.array([np.sum((s <= t) & (e > t)) for t in grid])
    peak = int(inflight.max())
    hi = np.flatnonzero(inflight >= 0.9 * peak)
    ramp_end = float(grid[hi[0]]) if hi.size else 0.0
    tail_start = float(grid[hi[-1]]) if hi.size else span
    dur = e - s
    edges = np.linspace(0.0, span, bins + 1)
    hist = [int(np.sum((s <= (a + b) / 2) & (e > (a + b) / 2))) for a, b in zip(edges[:-1], edges[1:])]
    return {"waves": int(s.size), "span_us": span,
            "end_quantiles_us": {q: float(np.quantile(e, f)) for q, f in (("p50", .5), ("p90", .9), ("p99", .99),
                                                                            ("max", 1.0))},
            "wave_us": {"mean": float(dur.mean()), "p50": float(np.median(dur)), "p99": float(np.quantile(dur, .99)),
                        "max": float(dur.max())},
            "peak_inflight": peak, "ramp_us": ramp_end, "steady_us": tail_start - ramp_end,
            "tail_us": span - tail_start, "inflight_bins": hist}


def main():
    envs = [int(x) for x in os.environ.get("WT_ENVS", "8192").split(",")]
    mode = os.environ.get("WT_MODE", "one")
    reps = int(os.environ.get("WT_REPS", 3))
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)
    res = {"mode": mode, "by_envs": {}}
    for E in envs:
        rng = np.random.default_rng(12345)
        p0 = sp[rng.integers(0, sp.shape[0], E)]
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        acts = torch.rand(100 + reps, E, 1, 2, device="cuda", generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        kw = dict(n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=7)
        if mode == "shards":
            import bench
            from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
            S = bench.auto_streams(E, 1)
            runner = StreamShards(tm, n_envs=E, n_streams=S, **kw)
            sims = runner.sims
        else:
            runner = BatchSim(tm, n_envs=E, **kw)
            sims = [runner]
        runner.reset(p0)
        for k in range(100):
            runner.step(acts[k], minimal_outputs=True)
        torch.cuda.synchronize()
        out = []
        for rep in range(reps):
            for sm in sims:
                read_trace(sm, True)
            runner.step(acts[100 + rep], minimal_outputs=True)
            torch.cuda.synchronize()
            bufs = [read_trace(sm, False) for sm in sims]
            allw = np.concatenate(bufs)
            line = summarize(allw[:, 0], allw[:, 1])
            if len(bufs) > 1:
                line["per_shard_span_us"] = [float((b[:, 1].max() - b[:, 0].min()) * TICK_US) for b in bufs]
            out.append(line)
        kinds = {"ray_kernel": sims[0].ray_kernel, "lanes": sims[0].ray_lanes, "refill": sims[0].ray_refill,
                 "contexts": len(sims)}
        res["by_envs"][str(E)] = {"kernel": kinds, "reps": out}
        runner.close()
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
