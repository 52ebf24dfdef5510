"""Stream-split study: one GPU's env shard stepped as S independent sub-shards,
each BatchSim context on its own HIP stream.

Envs are independent, so sub-shard s may start step t+1 while
sub-shard s' is still in step t: the latency-bound k_agents / k_post launches
(one thread per car, 128 waves at 8192 cars) and the ray kernel's tail then
overlap another sub-shard's ray pass.  Same work per step (E envs), same RNG
keying (global env id = sub-shard offset + local id), so outputs are the ones
of the single-context run.

    python scripts/stream_split.py --envs 8192 --splits 1 2 4 --steps 1000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def run(E, S, K, W, seed, track, spawn, dev, join=False, fast=False, gate=False, cumask=False):
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    rng = np.random.default_rng(seed)
    gidx = rng.integers(0, spawn.shape[0], size=E)
    poses0 = spawn[gidx]
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    acts = torch.rand(W + K, E, 1, 2, device=dev, generator=gen, dtype=torch.float32)
    acts[..., 0] = acts[..., 0] * (2 * 0.4189) - 0.4189
    acts[..., 1] = acts[..., 1] * 20.0
    Es = E // S
    sims, streams = [], []
    for s in range(S):
        sims.append(BatchSim(track, n_envs=Es, n_agents=1, device=dev, seed=seed, noise_std=0.01,
                             autoreset=True, spawn_poses=spawn, env_offset=s * Es))
        if S > 1 and cumask:   # a full-CU-mask stream gets a HW queue of its own (not shared round-robin)
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            words = (ncu + 31) // 32
            mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
            h = ctypes.c_void_p()
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
            assert rc == 0, rc
            streams.append(torch.cuda.ExternalStream(h.value, device=dev))
        else:
            streams.append(torch.cuda.Stream(dev) if S > 1 else torch.cuda.current_stream(dev))
    sl = [slice(s * Es, (s + 1) * Es) for s in range(S)]
    evs = []
    if gate:   # ring of events: sub-shard s's ray pass waits for s-1's (f110_debug_set_ray_gate)
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        for s in range(S):
            e = ctypes.c_void_p()
            assert hip.hipEventCreateWithFlags(ctypes.byref(e), 0x2) == 0   # hipEventDisableTiming
            evs.append(e)
        for s in range(S):
            assert sims[s].L.f110_debug_set_ray_gate(sims[s].ctx, evs[(s - 1) % S], evs[s]) == 0
    torch.cuda.synchronize(dev)
    for s in range(S):
        with torch.cuda.stream(streams[s]):
            sims[s].reset(poses0[sl[s]])
    for w in range(W):
        for s in range(S):
            with torch.cuda.stream(streams[s]):
                sims[s].step(acts[w, sl[s]], minimal_outputs=True)
    torch.cuda.synchronize(dev)
    main = torch.cuda.current_stream(dev)
    t0 = time.perf_counter()
    if fast:   # direct C-ABI calls, pointers and stream handles prepared up front
        import ctypes
        from f110_gymnasium_ros2_jazzy_amd import _lib
        step = sims[0].L.f110_step
        ctx = [sm.ctx for sm in sims]
        outs = [ctypes.byref(sm._outs_min) for sm in sims]
        hs = [ctypes.c_void_p(st.cuda_stream) for st in streams]
        base = acts.data_ptr()
        per_step = E * 2 * 4
        ptrs = [[ctypes.c_void_p(base + (W + k) * per_step + s * Es * 8) for s in range(S)] for k in range(K)]
        t0 = time.perf_counter()
        for k in range(K):
            pk = ptrs[k]
            for s in range(S):
                rc = step(ctx[s], pk[s], _lib.F32, outs[s], hs[s])
                if rc != 0:
                    raise RuntimeError(f"f110_step {rc}")
        K_loop = 0
    else:
        K_loop = K
    for k in range(K_loop):
        if join:   # fork from / join back into the caller's stream every step
            ev = main.record_event()
            for s in range(S):
                streams[s].wait_event(ev)
        for s in range(S):
            with torch.cuda.stream(streams[s]):
                sims[s].step(acts[W + k, sl[s]], minimal_outputs=True)
        if join:
            for s in range(S):
                main.wait_event(streams[s].record_event())
    t_sub = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    run.host_ms = t_sub / K * 1e3
    for s in range(S):
        if gate:
            sims[s].L.f110_debug_set_ray_gate(sims[s].ctx, None, None)
    obs = torch.cat([sims[s].out.obs for s in range(S)], 0).cpu()
    return E * K / dt, dt / K * 1e3, obs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--join", type=int, nargs="+", default=[0])
    ap.add_argument("--fast", type=int, nargs="+", default=[0])
    ap.add_argument("--gate", type=int, nargs="+", default=[0])
    ap.add_argument("--cumask", type=int, nargs="+", default=[0])
    args = ap.parse_args()
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
    dev = torch.device("cuda:0")
    track = load_map("Spielberg_map")
    track.ensure_edt()
    spawn = centerline_spawns("Spielberg", 1)
    res, ref = [], None
    for S, join, fast, gate, cm, rep in [(S, j, f, g, c, r) for S in args.splits for j in args.join
                                         for f in args.fast for g in args.gate for c in args.cumask
                                         for r in range(args.reps)]:
        if not (join and fast):
            v, ms, obs = run(args.envs, S, args.steps, args.warmup, args.seed, track, spawn, dev,
                             bool(join), bool(fast), bool(gate), bool(cm))
            if ref is None:
                ref = obs
            same = bool(torch.equal(obs, ref))
            line = {"splits": S, "join": join, "fast": fast, "gate": gate, "cumask": cm, "rep": rep, "host_submit_ms": run.host_ms, "env_steps_per_s": v, "ms_per_step": ms,
                    "obs_equal_to_S1": same}
            print(json.dumps(line), flush=True)
            res.append(line)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
