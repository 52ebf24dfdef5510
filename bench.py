#!/usr/bin/env python
"""bench.py — env-steps/s of the batched F1TENTH step on MI355X.

Metric (BASELINE.json): env-steps/sec at 65536 parallel envs, 1080-beam
lidar; scan L2 vs CPU ref.  Weak scaling: every GPU steps the same shard of
--envs-per-gpu single-agent envs (8192 -> 65536 envs at 8 GPUs, the
metric's configuration).  One "step" = one f110_step launch: ST dynamics
(RK4) + 1080-beam EDT sphere-trace + TTC/GJK/ray_cast + obs pack for every
env of the shard, with scan noise and device-side autoreset on.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0.  See DESIGN.md §Measurement for the
roofline accounting; the cpu_baseline leg (rank 0, N=1) times the C oracle
(oracle/) on the host cores for a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env-steps/sec at 65536 parallel envs, 1080-beam lidar; scan L2 vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs-per-gpu", type=int, default=8192)
    ap.add_argument("--agents", type=int, default=1)
    ap.add_argument("--map", default="Spielberg_map")
    ap.add_argument("--no-noise", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=512)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--streams", type=int, default=2,
                    help="sub-shards of the GPU's envs on concurrent dedicated-queue streams "
                         "(streams.StreamShards); 1 = one context on the current stream")
    ap.add_argument("--workload", choices=["step", "ddpg"], default="step",
                    help="step: the env step (headline); ddpg: config 5, the batched train_ddpg loop")
    ap.add_argument("--ddpg-batch", type=int, default=4096)
    ap.add_argument("--ddpg-memory", type=int, default=1 << 20)
    return ap.parse_args()


def bench_ddpg(args):
    """Config 5 (BASELINE.json): the batched train_ddpg loop, --envs-per-gpu
    two-agent envs per GPU (gap-follow opponent, device reward, replay add,
    one learner update of --ddpg-batch rows per vector step with the actor /
    critic gradients all-reduced over the ranks by RCCL)."""
    import torch
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
    rank, world, local = D.init()
    dev_index = D.local_device_index(local)
    torch.cuda.set_device(dev_index)
    shard = D.shard_range(args.envs_per_gpu * world, world, rank)
    K, W = args.steps, args.warmup
    # learner updates start once the memory holds a batch: ceil(batch / envs) steps
    fill = -(-args.ddpg_batch // max(shard.count, 1)) + 1
    tr = VectorTrainer(shard.count, batch_size=args.ddpg_batch, memory_size=args.ddpg_memory,
                       warmup_steps=min(fill, W), seed=args.seed, env_offset=shard.offset, rank_seed=rank)
    for _ in range(W):
        tr.step()
    assert tr.last is not None, "warm-up too short: no learner update ran"
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.max_over_ranks(t1 - t0)
    total = D.sum_over_ranks(shard.count * K)
    # phase split (separate pass, events on the current stream; not part of `value`)
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    KP = min(K, 100)
    ph = {"env_step_reward_ms": 0.0, "replay_add_ms": 0.0, "learner_update_ms": 0.0}
    for _ in range(KP):
        act = tr.agent.choose_action(tr.obs, training=True)
        ev[0].record(stream)
        nxt, rew, term, _, info = tr.env.step(act)
        ev[1].record(stream)
        tr.agent.remember(tr.obs, act, rew.to(torch.float32), nxt, term, mask=~info["reset"])
        ev[2].record(stream)
        tr.last = tr.agent.replay()
        ev[3].record(stream)
        tr.obs = nxt
        torch.cuda.synchronize()
        ph["env_step_reward_ms"] += ev[0].elapsed_time(ev[1]) / KP
        ph["replay_add_ms"] += ev[1].elapsed_time(ev[2]) / KP
        ph["learner_update_ms"] += ev[2].elapsed_time(ev[3]) / KP
    # data-parallel consistency: every rank must hold the same weights
    wsum = float(sum(float(p.double().sum()) for p in tr.agent.actor.parameters()))
    in_sync = D.max_over_ranks(wsum) == -D.max_over_ranks(-wsum)
    result = {
        "metric": "env-steps/sec, end-to-end DDPG (BASELINE config 5)", "value": total / elapsed,
        "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W, "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64 env / f32 learner",
        "data": "synthetic: Spielberg map, centerline spawns, actor + Gaussian noise actions",
        "config": {"workload": f"{shard.count} two-agent envs per GPU (gap-follow opponent), device reward, "
                               f"PER replay, 1 learner update of {args.ddpg_batch} rows per vector step",
                   "envs_per_gpu": args.envs_per_gpu, "global_envs": args.envs_per_gpu * world,
                   "batch_per_rank": args.ddpg_batch, "memory_per_rank": args.ddpg_memory,
                   "parallelism": f"env-shard x{world}, DDPG data-parallel (RCCL all-reduce of grads)"},
        "phases_ms": ph,
        "learner": {"critic_loss": float(tr.last["critic_loss"]), "actor_loss": float(tr.last["actor_loss"]),
                    "updates": tr.agent.global_step, "ranks_in_sync": in_sync},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    tr.close()
    D.shutdown()


def algorithmic_bytes_per_env_step(B: int, A: int, mean_lookups: float) -> float:
    """B x (4 L + 4) + 120 per agent-step: each EDT lookup
    credited at 4 B (the exact uint32 k cell), 4 B of f32 output per ray,
    2 x 56 B state read/write + 8 B action per agent."""
    return A * (B * (4.0 * mean_lookups + 4.0) + 120.0)


def load_pmc_traffic(E: int, A: int):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("envs")) == E and int(d.get("agents")) == A:
            return float(d["bytes_per_launch"]), d
    except Exception:
        pass
    return None, None


def cpu_baseline(track, spawn_poses, actions_np, args, gpu_sim):
    """Oracle (C restatement, OpenMP) on the host cores; bounded sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure: the checker, never the product)
    O.build()
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or threads))
    sc = O.OracleScanner(track.free_mask, track.resolution, track.origin)
    E = min(args.cpu_envs, spawn_poses.shape[0])
    A = args.agents
    sim = O.OracleSim(sc, E, A)
    sim.reset(spawn_poses[:E])
    t0 = time.perf_counter()
    sim.step(actions_np[0, :E], threads=threads)
    t1 = time.perf_counter()
    per = max(t1 - t0, 1e-4)
    steps = int(max(2, min(2000, args.cpu_seconds / per)))
    sim.reset(spawn_poses[:E])
    t0 = time.perf_counter()
    for k in range(steps):
        sim.step(actions_np[k % actions_np.shape[0], :E], threads=threads)
    dt = time.perf_counter() - t0
    # scan parity at the GPU's current poses (the metric's "scan L2 vs CPU ref")
    import torch
    st = gpu_sim.agent_states()[:64].reshape(-1, 7).cpu().numpy()
    poses = np.stack([st[:, 0], st[:, 1], st[:, 4]], 1)
    g = gpu_sim.scan_batch(poses).cpu().numpy()
    ref = sc.scan(poses, threads=threads)
    diff = g - ref
    return {
        "value": E * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
        "sample": f"{E} envs x {steps} steps ({args.agents} agent, {args.map}, RK4, noise-free), "
                  f"C oracle oracle/f110_oracle.c, OpenMP over envs, {dt:.1f} s",
        "scan_l2_vs_cpu": float(np.sqrt(np.sum(diff * diff))),
        "scan_max_abs_vs_cpu": float(np.max(np.abs(diff))),
        "scan_rays_compared": int(diff.size),
    }


def main():
    args = parse()
    if args.workload == "ddpg":
        return bench_ddpg(args)
    import numpy as np
    import torch
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim

    rank, world, local = D.init()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev_index = D.local_device_index(local)
    torch.cuda.set_device(dev_index)
    dev = torch.device(f"cuda:{dev_index}")
    E, A = args.envs_per_gpu, args.agents
    shard = D.shard_range(E * world, world, rank)

    track = load_map(args.map)
    track.ensure_edt()
    spawn = centerline_spawns(args.map.replace("_map", ""), A)
    # initial spawn per GLOBAL env id (independent of GPU count)
    rng = np.random.default_rng(args.seed)
    gidx = rng.integers(0, spawn.shape[0], size=E * world)[shard.offset:shard.offset + shard.count]
    poses0 = spawn[gidx]
    sim = BatchSim(track, n_envs=shard.count, n_agents=A, device=dev, seed=args.seed,
                   noise_std=0.0 if args.no_noise else 0.01, autoreset=True, spawn_poses=spawn,
                   env_offset=shard.offset)

    K, W = args.steps, args.warmup
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000003 * 0 + shard.offset)
    acts = torch.rand(W + K, shard.count, A, 2, device=dev, generator=gen, dtype=torch.float32)
    acts[..., 0] = acts[..., 0] * (2 * 0.4189) - 0.4189   # steer in [-0.4189, 0.4189]
    acts[..., 1] = acts[..., 1] * 20.0                   # speed in [0, 20] (ddpg_config.yaml:19-20)
    stream = torch.cuda.current_stream(dev)
    S = max(1, args.streams)
    runner = sim
    if S > 1:
        from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards
        runner = StreamShards(track, n_envs=shard.count, n_streams=S, env_offset=shard.offset, n_agents=A,
                              device=dev, seed=args.seed, noise_std=0.0 if args.no_noise else 0.01,
                              autoreset=True, spawn_poses=spawn)

    def timed(r):
        """W untimed steps, then K steps between barrier + synchronize (max over ranks)."""
        r.reset(poses0)
        for w in range(W):
            r.step(acts[w], minimal_outputs=True)
        torch.cuda.synchronize(dev)
        r.reset_counters()
        D.barrier()
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(K):
            r.step(acts[W + k], minimal_outputs=True)
        if r is not sim:
            r.join()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        D.barrier()
        return D.max_over_ranks(t1 - t0), ev0.elapsed_time(ev1) / K, r.read_counters()

    elapsed, kernel_ms, (lookups, rays) = timed(runner)
    mean_look = lookups / max(rays, 1)
    total_env_steps = D.sum_over_ranks(shard.count * K)
    single = None
    if runner is not sim:
        # the same workload on one context / one stream, for comparison (not `value`)
        el1, _, _ = timed(sim)
        single = {"value": total_env_steps / el1, "ms_per_step": el1 / K * 1e3}
        runner.close()

    # second, separate pass: per-kernel HIP-event timing (not part of `value`)
    KP = min(K, 300)
    sim.profile_begin(KP)
    for k in range(KP):
        sim.step(acts[W + (k % K)], minimal_outputs=True)
    per_kernel = sim.profile_end()

    B = sim.B
    # k_rays (the dominant kernel): per ray 4 B per EDT lookup (exact uint32 k
    # cell) + 4 B of f32 range out; the 120 B/agent of state I/O
    # belong to k_agents.
    rays_bytes_launch = shard.count * A * B * (4.0 * mean_look + 4.0)
    achieved = rays_bytes_launch / (per_kernel["k_rays_ms"] * 1e-3) / 1e9
    bytes_launch = shard.count * algorithmic_bytes_per_env_step(B, A, mean_look)
    traffic, _ = load_pmc_traffic(shard.count, A)
    result = {
        "metric": METRIC,
        "value": total_env_steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: i.i.d. uniform random actions, centerline spawn poses, Spielberg map",
        "config": {
            "workload": f"{E} single-agent envs per GPU ({E * world} total); C3 shard at 8 GPUs = 65536 envs"
            if A == 1 else f"{E} {A}-agent envs per GPU",
            "envs_per_gpu": E, "global_envs": E * world, "agents": A, "beams": B, "map": args.map,
            "integrator": "RK4", "scan_noise": not args.no_noise, "autoreset": True,
            "parallelism": f"env-shard x{world} (no collectives)",
            "streams_per_gpu": S,
        },
        "roofline": {
            "kernel": "k_rays", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel_ms": per_kernel["k_rays_ms"], "algorithmic_bytes_per_launch": rays_bytes_launch,
            "mean_lookups_per_ray": mean_look,
            "step_kernels_ms": {"k_agents": per_kernel["k_agents_ms"], "k_rays": per_kernel["k_rays_ms"],
                                "k_post": per_kernel["k_post_ms"], "stream_per_step": kernel_ms},
            "step_algorithmic_bytes_per_env": bytes_launch / max(shard.count, 1),
        },
    }
    if single is not None:
        result["single_stream"] = single
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(track, poses0, acts[:64].cpu().numpy(), args, sim)
        except Exception as exc:  # report, never hide
            result["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    sim.close()
    D.shutdown()


if __name__ == "__main__":
    main()
