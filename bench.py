#!/usr/bin/env python
"""bench.py — env-steps/s of the batched F1TENTH step on MI355X.

Metric (BASELINE.json): env-steps/sec at 65536 parallel envs, 1080-beam
lidar; scan L2 vs CPU ref.  The job steps --global-envs (65536) single-agent
envs split over the ranks (strong scaling: 65536 on one MI355X, 8192 per GPU
at 8).  One "step" = one f110_step launch: ST dynamics (RK4) + 1080-beam EDT
sphere-trace + TTC/GJK/ray_cast + obs pack for every env of the shard, with
scan noise and device-side autoreset on.  At N=1 the line also carries the
8192-env C3 shard and the 4096-env C2 workload (`secondary`), the one-stream
runner a policy loop uses (`single_stream`), the scan check of the timed
kernel against the CPU oracle (`scan_check`), the roofline and the CPU
baseline.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N > 1` without a launcher (no WORLD_SIZE in the environment) starts
its own N ranks: the parent decides from argv / env alone, before anything
touches the GPU (no torch import), runs torch.distributed.run over 127.0.0.1
with the same arguments and exits with its return code.  Under a launcher,
WORLD_SIZE must equal --gpus (else exit 2).

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
GLOBAL_ENVS = 65536
DIGEST_ENVS = 64  # trajectory_digest: obs rows of global envs 0, G/64, 2G/64, ...


def metric_name(global_envs: int, agents: int) -> str:
    """BASELINE.json's metric for the run's own workload (the headline is
    65536 single-agent envs; other --global-envs / --agents runs name theirs)."""
    if global_envs == GLOBAL_ENVS and agents == 1:
        return METRIC
    who = "parallel envs" if agents == 1 else f"parallel {agents}-agent envs"
    return f"env-steps/sec at {global_envs} {who}, 1080-beam lidar; scan L2 vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# texture-address cycles per wave-level 8-byte load whatever its lanes do: MEASURED (rocprofv3
# TA_BUSY / SQ_INSTS_VMEM_RD), not a datasheet figure.  The roofline takes it from the
# committed PMC pass of the same configuration (profiles/pmc_busy_E<E>_A<A>.json, its
# ta_cycles_per_vmem_rd); this is the fallback when no such file exists (round 3's 65536-car value)
TA_CYCLES_PER_LOAD = 20.1
N_CU, CLOCK_GHZ = 256, 2.4  # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--global-envs", type=int, default=GLOBAL_ENVS,
                    help="envs of the whole job, split over the ranks (the metric's 65536; strong scaling)")
    ap.add_argument("--envs-per-gpu", type=int, default=None,
                    help="fixed envs per rank instead (weak scaling); --workload ddpg defaults to 4096")
    ap.add_argument("--agents", type=int, default=1)
    ap.add_argument("--map", default="Spielberg_map")
    ap.add_argument("--no-noise", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-outputs", action="store_true",
                    help="skip the every-output one-context pass (rocprofv3 runs: its launches write more and "
                         "would mix into the ray kernel's average)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C3-shard (8192) / C2 (4096) secondary lines at N=1")
    ap.add_argument("--cpu-envs", type=int, default=GLOBAL_ENVS,
                    help="envs of the CPU baseline (default: the metric's 65536, all on the host)")
    ap.add_argument("--cpu-steps", type=int, default=30,
                    help="timed CPU steps (30 x 65536 envs: ~13 s on 16 threads)")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--ramp-s", type=float, default=1.0,
                    help="untimed steps for at least this long before the W warm-up steps (the idle GPU "
                         "clocks down; DVFS ramp), reported as config.ramp")
    ap.add_argument("--streams", type=int, default=0,
                    help="sub-shards of the GPU's envs on concurrent dedicated-queue streams "
                         "(streams.StreamShards); 1 = one context on the current stream; 0 (default) = "
                         "auto_streams(envs per GPU)")
    ap.add_argument("--runner", choices=["auto", "streams", "one"], default="auto",
                    help="the timed runner: streams = StreamShards sub-shards of the three-launch step; one = one "
                         "context, three launches per step (the policy-loop path); auto = streams")
    ap.add_argument("--workload", choices=["step", "ddpg"], default="step",
                    help="step: the env step (headline); ddpg: config 5, the batched train_ddpg loop")
    ap.add_argument("--ddpg-batch", type=int, default=4096)
    ap.add_argument("--ddpg-memory", type=int, default=1 << 20)
    return ap.parse_args()


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for the self-launched ranks' rendezvous."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launcher_cmd(argv: list, n: int, port: int) -> list:
    """The command the parent runs for --gpus n without an outer launcher:
    torch.distributed.run, one node, n ranks, rendezvous on 127.0.0.1, this
    file with the caller's own arguments (--gpus n among them)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def self_launch(args, argv: list) -> int:
    """--gpus N > 1 with no WORLD_SIZE: run the N ranks as children and return
    their launcher's exit code (non-zero when any rank failed).  Called before
    any torch import, so this process never initialises HIP."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL's IPC on this host (dmabuf only)
    env.setdefault("OMP_NUM_THREADS", "1")  # torch.distributed.run would warn and set it anyway
    return subprocess.call(launcher_cmd(argv, args.gpus, free_port()), env=env)


def check_world(args) -> None:
    """Under a launcher, its WORLD_SIZE must be --gpus: a mismatch exits 2
    instead of printing an N-GPU line for a different rank count."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a mismatched run",
              file=sys.stderr)
        sys.exit(2)


def learner_roofline(M: int, obs: int, update_ms: float) -> dict:
    """The learner update against the fp32 MFMA peak (its GEMMs run on
    v_mfma_f32_32x32x2_f32, csrc/f110_gemm.hip): GEMM FLOPs per update / the
    update's measured time (phases_ms.learner_update_ms, events around
    replay(): sampling, heads, Adam and the all-reduces included)."""
    fl = learner_flops_per_update(M, obs)
    tf = fl / (update_ms * 1e-3) / 1e12 if update_ms > 0 else None
    return {"bound": "mfma", "flops_per_update": fl, "update_ms": update_ms, "achieved": tf,
            "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP32_MFMA_PEAK_TFLOPS if tf else None,
            "note": "GEMM FLOPs of the update (bench.learner_flops_per_update) / the whole update's time"}


def bench_ddpg(args):
    """Config 5 (BASELINE.json): the batched train_ddpg loop, --envs-per-gpu
    two-agent envs per GPU (gap-follow opponent, device reward, replay add,
    one learner update of --ddpg-batch rows per vector step with the actor /
    critic gradients all-reduced over the ranks by RCCL)."""
    import torch
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    rank, world, local = D.init()
    dev_index = D.local_device_index(local)
    torch.cuda.set_device(dev_index)
    result = run_ddpg(args, args.envs_per_gpu or 4096, args.steps, args.warmup)  # C5: 32768 envs over 8 GPUs
    if rank == 0:
        print(json.dumps(result), flush=True)
    D.shutdown()


def run_ddpg(args, per_gpu: int, K: int, W: int) -> dict:
    """The C5 loop on this rank's share of per_gpu x world envs: W untimed
    vector steps, K timed ones (barrier + synchronize, max over ranks), then a
    phase split and the data-parallel consistency check.  Returns the line."""
    import torch
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    from f110_gymnasium_ros2_jazzy_amd.train import VectorTrainer
    rank, world, _ = D.env_rank_world()
    shard = D.shard_range(per_gpu * world, world, rank)
    # learner updates start once the memory holds a batch: ceil(batch / envs) steps
    fill = -(-args.ddpg_batch // max(shard.count, 1)) + 1
    tr = VectorTrainer(shard.count, batch_size=args.ddpg_batch, memory_size=args.ddpg_memory,
                       warmup_steps=min(fill, W), seed=args.seed, env_offset=shard.offset, rank_seed=rank)
    # untimed steps for >= ramp_s seconds first (the idle GPU clocks down; DVFS ramp), in blocks of 25
    # whose end every rank agrees on (the learner's all-reduces need the same step count on each rank)
    t_end = time.perf_counter() + args.ramp_s
    ramp = 0
    while args.ramp_s > 0:
        for _ in range(25):
            tr.step()
        ramp += 25
        torch.cuda.synchronize()
        if D.max_over_ranks(float(time.perf_counter() >= t_end)) > 0:
            break
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
    # phase split (separate pass of 100 steps, events on the current stream; not part of `value`):
    # the steps are submitted back to back as in the timed loop (no synchronize between them, which
    # would start every phase on an idle GPU) and the events read once at the end
    stream = torch.cuda.current_stream()
    KP = 100
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(KP)]
    ph = {"env_step_reward_ms": 0.0, "replay_add_ms": 0.0, "learner_update_ms": 0.0}
    # the gradient-bucket all-reduces inside the update (several ranks): events around each
    # GradBucket.reduce on the current stream (RCCL enqueues there; gloo blocks the host meanwhile)
    ar_pairs = []
    if world > 1:
        ph["learner_allreduce_ms"] = 0.0
        for bucket in (tr.agent.critic_grads, tr.agent.actor_grads):
            def timed_reduce(f=bucket.reduce):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                f()
                e1.record(stream)
                ar_pairs.append((e0, e1))
            bucket.reduce = timed_reduce
    for ev in evs:
        act = tr.agent.choose_action(tr.obs, training=True, out=tr.env.agent_actions())  # as VectorTrainer.step
        ev[0].record(stream)
        nxt, rew, term, was_reset = tr.env.step_transition(act)
        ev[1].record(stream)
        tr.agent.remember_env(tr.obs, act, rew, nxt, term, was_reset)
        ev[2].record(stream)
        tr.last = tr.agent.replay()
        ev[3].record(stream)
        tr.obs = nxt
    torch.cuda.synchronize()
    for ev in evs:
        ph["env_step_reward_ms"] += ev[0].elapsed_time(ev[1]) / KP
        ph["replay_add_ms"] += ev[1].elapsed_time(ev[2]) / KP
        ph["learner_update_ms"] += ev[2].elapsed_time(ev[3]) / KP
    if ar_pairs:
        ph["learner_allreduce_ms"] = sum(e0.elapsed_time(e1) for e0, e1 in ar_pairs) / KP
    # data-parallel consistency: every rank must hold the same weights
    wsum = float(sum(float(p.detach().double().sum()) for p in tr.agent.actor.parameters()))
    in_sync = D.max_over_ranks(wsum) == -D.max_over_ranks(-wsum)
    result = {
        "metric": "env-steps/sec, end-to-end DDPG (BASELINE config 5)", "value": total / elapsed,
        "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W, "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64 env / f32 learner",
        "data": "synthetic: Spielberg map, centerline spawns, actor + Gaussian noise actions",
        "config": {"workload": f"{shard.count} two-agent envs per GPU (gap-follow opponent), device reward, "
                               f"PER replay, 1 learner update of {args.ddpg_batch} rows per vector step",
                   "envs_per_gpu": per_gpu, "global_envs": per_gpu * world,
                   "batch_per_rank": args.ddpg_batch, "memory_per_rank": args.ddpg_memory,
                   "ramp": {"seconds": args.ramp_s, "steps": ramp},
                   "parallelism": (f"env-shard x{world}, DDPG data-parallel ({D.describe()['backend']} all-reduce of grads; nccl = RCCL)"
                                   if world > 1 else "one GPU, one learner (no all-reduce)"),
                   "dist": D.describe()},
        "phases_ms": ph,
        "learner_roofline": learner_roofline(args.ddpg_batch, tr.agent.obs_dim, ph["learner_update_ms"]),
        "learner": {"critic_loss": float(tr.last["critic_loss"]), "actor_loss": float(tr.last["actor_loss"]),
                    "updates": tr.agent.global_step, "ranks_in_sync": in_sync},
    }
    tr.close()
    return result


FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (exact f32), dense


def learner_flops_per_update(M: int, obs: int, act: int = 2, hid: int = 128) -> float:
    """GEMM FLOPs of one DDPG learner update (agent.py:302-331) on M rows, as
    the explicit learner runs it (learner_fused.py): critic phase = actor_target
    and critic_target forward on next_states, critic forward on states, critic
    backward (q, fcs2 weight + input gradients, fcs1 weight gradient; no
    gradient into obs); actor phase = actor forward, the updated critic forward
    on (states, actions), backward through q / fcs2 to the action columns, then
    the actor's weight and input gradients (fc3, fc2; fc1 weight only).  2 M K N
    per [M x K] x [K x N] product; the heads' N = 1-2 GEMVs included."""
    def mm(k, n):
        return 2.0 * M * k * n
    actor_fwd = mm(obs, hid) + mm(hid, hid) + mm(hid, act)
    critic_fwd = mm(obs, hid) + mm(hid + act, hid) + mm(hid, 1)
    critic_bwd = (mm(1, hid) + mm(hid, 1)          # q: dh, dW
                  + mm(hid + act, hid) + mm(hid, hid)  # fcs2: dW, dX (the fcs1 columns)
                  + mm(obs, hid))                  # fcs1: dW
    actor_bwd = (mm(1, hid) + mm(hid, act)          # critic q dh, fcs2 dX (action columns)
                 + mm(hid, act) + mm(act, hid)      # fc3: dW, dX
                 + mm(hid, hid) + mm(hid, hid)      # fc2: dW, dX
                 + mm(obs, hid))                    # fc1: dW
    critic_phase = actor_fwd + critic_fwd + critic_fwd + critic_bwd  # targets on next_states, critic on states
    actor_phase = actor_fwd + critic_fwd + actor_bwd
    return critic_phase + actor_phase


def algorithmic_bytes_per_env_step(B: int, A: int, mean_lookups: float) -> float:
    """B x (4 L + 4) + 120 per agent-step: each EDT lookup
    credited at 4 B (the exact uint32 k cell), 4 B of f32 output per ray,
    2 x 56 B state read/write + 8 B action per agent."""
    return A * (B * (4.0 * mean_lookups + 4.0) + 120.0)


def load_profile(kind: str, E: int, A: int):
    """A profiles/ summary recorded at this exact configuration (or None):
    pmc_traffic (FETCH/WRITE bytes per k_rays launch, scripts/profile_round.py)
    or pmc_busy (VALU busy / wave occupancy, scripts/profile_round.py)."""
    for name in (f"{kind}_E{E}_A{A}.json", f"{kind}.json"):
        path = os.path.join(REPO, "profiles", name)
        try:
            with open(path) as f:
                d = json.load(f)
            if int(d.get("envs")) == E and int(d.get("agents")) == A:
                d["file"] = "profiles/" + name
                return d
        except Exception:
            pass
    return None


def affinity_cpus() -> int:
    """CPUs this process may run on (os.cpu_count() counts the whole machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_threads() -> int:
    """OMP_NUM_THREADS when the host sets it (the GPU box sets 16: one GPU's
    share of a 256-thread machine), else every CPU of the affinity set."""
    n = affinity_cpus()
    t = int(os.environ.get("OMP_NUM_THREADS") or 0) or n
    return max(1, min(t, n))


def oracle_module():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure: the checker, never the product)
    O.build()
    return O


def auto_streams(envs, agents=1):
    """Stream sub-shards per GPU (measured 300-step bench lines):
    8192 envs 40.4 / 46.6 / 49.2 M env-steps/s at S = 1 / 2 / 4; 16384 55.2 /
    48.4 at S = 2 / 4; 32768 61.8 / 46.2; 65536 62.4 / 52.7.  Small shards
    leave CUs idle in k_agents / k_post and the grid tail, which more
    concurrent sub-shards fill; large ones fill the GPU themselves.  Counted
    in cars (envs x agents).  Round 2, end (k_rays_fxn / k_rays_fxr): 16384 envs
    61.3 / 63.1 M at S = 2 / 4 (fxn), 65.3 M at S = 4 with k_rays_fxr
    (profiles/r02_refill_small/): S = 4 up to 16384 cars.  Round 3 (k_rays_fxs): 32768 envs 76.7 M at
    S = 2, 78.7 / 75.8 M at S = 4 on two boxes (profiles/r03_ab/e32768_*.json): no change.  Round 6
    (profiles/r06/shard_rules_streams_large_sizes.jsonl, S = 1 / 2 / 4): 65536 90.4 / 101.9 / 99.0 M,
    32768 80.2 / 100.0 / 98.3 M, 16384 66.2 / 82.0 / 85.7 M: the rule stands."""
    return 4 if envs * agents <= 16384 else 2


def cpu_baseline(O, scanner, poses, acts_np, args):
    """The C oracle (oracle/f110_oracle.c, OpenMP over envs) on the host cores:
    BASELINE.md §3's plan -- cpu_envs envs (default the metric's 65536, the
    GPU run's own spawn poses and actions), cpu_warmup + cpu_steps steps, scan
    noise on (a host draw).  The sample is bounded by steps, not envs: every
    env of the configuration is stepped."""
    threads = cpu_threads()
    E = min(args.cpu_envs, poses.shape[0])
    A = args.agents
    sim = O.OracleSim(scanner, E, A)
    sim.set_noise(0.0 if args.no_noise else 0.01, args.seed)
    sim.reset(poses[:E])
    T = acts_np.shape[0]
    for k in range(args.cpu_warmup):
        sim.step(acts_np[k % T, :E], threads=threads)
    t0 = time.perf_counter()
    for k in range(args.cpu_steps):
        sim.step(acts_np[(args.cpu_warmup + k) % T, :E], threads=threads)
    dt = time.perf_counter() - t0
    omp = os.environ.get("OMP_NUM_THREADS")
    return {
        "value": E * args.cpu_steps / dt, "unit": "env-steps/s", "cores": threads,
        "affinity_cpus": affinity_cpus(), "nproc": os.cpu_count(), "omp_num_threads": omp,
        "cores_note": ("OMP_NUM_THREADS caps the threads: the GPU host sets it to its per-GPU CPU share "
                       "(the machine's CPUs are shared by its GPUs' jobs)" if omp and int(omp) < affinity_cpus()
                       else "every CPU of the process's affinity set"),
        "kind": "port",
        "threads": threads, "envs": E, "steps": args.cpu_steps,
        "sample": f"{E} envs x {args.cpu_steps} steps after {args.cpu_warmup} warm-up ({A} agent, {args.map}, RK4, "
                  f"noise {'off' if args.no_noise else 'on'}, the GPU run's spawn poses and actions), C oracle "
                  f"oracle/f110_oracle.c, OpenMP over envs on {threads} threads, {dt:.1f} s timed",
    }


def scan_check(O, scanner, runner, act, threads):
    """Scan L2 of the TIMED kernel against the CPU oracle: one more step of the
    timed runner (k_rays_tiled, same dispatch) with its f64 scan output on and
    the noise zeroed through the caller-noise input (range + 0.0 is exact),
    compared with oracle scans at the cars' post-step poses (the scan pose:
    lidar_dist = 0).  Cars whose TTC fired are skipped: the collision response
    zeroed their yaw after the scan (base_classes.py:246-249)."""
    import numpy as np
    import torch
    sims = getattr(runner, "sims", [runner])
    if sims[0].A != 1:
        return scan_check_multi(O, scanner, runner, act, threads)
    for sm in sims:
        sm.set_scan_noise(torch.zeros(sm.E, sm.B, dtype=torch.float64, device=sm.device))
    runner.step(act, minimal_outputs=False)
    if hasattr(runner, "join"):
        runner.join()
    torch.cuda.synchronize()
    g, poses, skipped = [], [], 0
    for sm in sims:
        st = sm.agent_states().reshape(-1, 7).cpu().numpy()
        col = sm.out.collisions.reshape(-1).cpu().numpy().astype(bool)
        sc = sm.out.scans_f64.reshape(-1, sm.B).cpu().numpy()
        sm.set_scan_noise(None)
        skipped += int(col.sum())
        g.append(sc[~col])
        poses.append(np.stack([st[~col, 0], st[~col, 1], st[~col, 4]], 1))
    g = np.concatenate(g)
    poses = np.concatenate(poses)
    ref = scanner.scan(poses, threads=threads)
    diff = g - ref
    return {"kernel": f"{ray_kernel_name(sims[0], shared=len(sims) > 1)} (the timed runner, one extra step)", "cars": int(poses.shape[0]),
            "cars_skipped_ttc": skipped, "rays": int(diff.size),
            "l2": float(np.sqrt(np.sum(diff * diff))), "max_abs": float(np.max(np.abs(diff))),
            "bit_exact_fraction": float(np.mean(diff == 0.0))}


def ray_kernel_name(sm, shared=False):
    """The ray kernel launch_env_step picks for this context's unmasked steps (shared: a stream
    sub-shard, f110_set_device_share with several contexts: single-agent k_rays_fxs then takes the
    theta table in LDS, 8 waves per block)."""
    names = {1: "k_rays_tiled (flat)", 2: "k_rays_tiled (chunked)", 3: "k_rays_fx"}
    if sm.ray_kernel == 3 and sm.ray_refill > 0:
        lds = ", theta table in LDS" if shared and sm.A == 1 else ""
        return (f"k_rays_fxs ({sm.ray_refill} wave(s) per car, 2 software-pipelined chunk slots with refill, "
                f"padded EDT{lds})")
    if sm.ray_kernel == 3 and sm.ray_lanes > 1:
        return f"k_rays_fxn ({sm.ray_lanes} rays per lane)"
    return names.get(sm.ray_kernel, str(sm.ray_kernel))


def scan_check_multi(O, scanner, runner, act, threads, S=256):
    """Multi-agent scan check of the timed kernel: the agent ray_cast edits
    the traced scans, so the oracle steps a sample of S envs in lock-step
    instead (Simulator.step, base_classes.py:566-625): the oracle takes the
    device's pre-step state (state, steer buffer and count) and the same
    actions, noise zeroed on both sides; envs the step autoreset are skipped.
    Ray_cast beams may differ in the last ulps (ocml vs glibc trig); the
    count of non-bit-exact beams is reported."""
    import numpy as np
    import torch
    sm = runner.sims[0] if hasattr(runner, "sims") else runner
    A, B = sm.A, sm.B
    S = min(S, sm.E)
    st, sb, sc = sm.get_state()
    ref = O.OracleSim(scanner, S, A)
    ref.state[:] = st[:, :S * A].t().cpu().numpy()
    ref.buf[:] = sb[:, :S * A].t().cpu().numpy()
    ref.cnt[:] = sc[:S * A].cpu().numpy()
    sims = getattr(runner, "sims", [runner])
    for m in sims:
        m.set_scan_noise(torch.zeros(m.E, m.B, dtype=torch.float64, device=m.device))
    runner.step(act, minimal_outputs=False)
    if hasattr(runner, "join"):
        runner.join()
    torch.cuda.synchronize()
    a = act[:S] if act.shape[0] >= S else act
    rs, _ = ref.step(a.double().cpu().numpy().reshape(S, A, 2), threads=threads)
    g = sm.out.scans_f64[:S].cpu().numpy()
    keep = sm.out.was_reset[:S].cpu().numpy() == 0
    for m in sims:
        m.set_scan_noise(None)
    diff = (g - rs)[keep]
    return {"kernel": f"{ray_kernel_name(sm)} + k_post_multi (the timed runner, one extra step), oracle in lock-step",
            "envs": int(keep.sum()), "agents": A, "rays": int(diff.size),
            "l2": float(np.sqrt(np.sum(diff * diff))), "max_abs": float(np.max(np.abs(diff))) if diff.size else 0.0,
            "bit_exact_fraction": float(np.mean(diff == 0.0)) if diff.size else 1.0,
            "non_bit_exact_beams": int(np.sum(diff != 0.0))}


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, sys.argv[1:]))
    check_world(args)
    if os.environ.get("F110_BENCH_ECHO_RANKS") == "1":  # launcher test hook (tests/test_bench_launch.py): no GPU
        line = json.dumps({"rank": int(os.environ.get("RANK", 0)), "world": int(os.environ.get("WORLD_SIZE", 1)),
                           "local_rank": int(os.environ.get("LOCAL_RANK", 0)),
                           "master_addr": os.environ.get("MASTER_ADDR"), "gpus": args.gpus,
                           "argv": sys.argv[1:]}) + "\n"
        sys.stdout.flush()
        os.write(1, line.encode())  # one write: the ranks share the launcher's stdout pipe
        return
    if args.workload == "ddpg":
        return bench_ddpg(args)
    import numpy as np
    import torch
    from f110_gymnasium_ros2_jazzy_amd import distributed as D
    from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
    from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
    from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards

    rank, world, local = D.init()
    dev_index = D.local_device_index(local)
    torch.cuda.set_device(dev_index)
    dev = torch.device(f"cuda:{dev_index}")
    A = args.agents
    weak = args.envs_per_gpu is not None
    G = args.envs_per_gpu * world if weak else args.global_envs
    shard = D.shard_range(G, world, rank)
    E = shard.count
    K, W = args.steps, args.warmup
    noise = 0.0 if args.no_noise else 0.01

    track = load_map(args.map)
    track.ensure_edt()
    spawn = centerline_spawns(args.map.replace("_map", ""), A)
    # initial spawn per GLOBAL env id (independent of GPU count)
    rng = np.random.default_rng(args.seed)
    gidx = rng.integers(0, spawn.shape[0], size=G)[shard.offset:shard.offset + E]
    poses0 = spawn[gidx]

    def actions(n_steps, n_envs, offset, n_global, A_=A):
        """Uniform random actions keyed by GLOBAL env id: the job's [T, n_global]
        draw (one seed, one shape on every rank), then this rank's columns, so
        an env steps the same actions whatever the GPU count."""
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed)
        a = torch.rand(n_steps, n_global, A_, 2, device=dev, generator=gen, dtype=torch.float32)
        a = a[:, offset:offset + n_envs].contiguous()
        a[..., 0] = a[..., 0] * (2 * 0.4189) - 0.4189   # steer in [-0.4189, 0.4189]
        a[..., 1] = a[..., 1] * 20.0                   # speed in [0, 20] (ddpg_config.yaml:19-20)
        return a

    acts = actions(W + K + 1, E, shard.offset, G)
    stream = torch.cuda.current_stream(dev)

    kind = args.runner
    if kind == "auto":
        kind = "streams"
    policy_kind = "one"  # what a policy loop steps: one call per step, one context

    def make(n_envs, offset, kind_, A_=A, spawn_=spawn):
        kw = dict(n_agents=A_, device=dev, seed=args.seed, noise_std=noise, autoreset=True, spawn_poses=spawn_,
                  keep_f64_scans=True)
        if kind_ == "streams":
            s = args.streams if args.streams > 0 else auto_streams(n_envs, A_)
            if s > 1 and n_envs % s == 0:
                r = StreamShards(track, n_envs=n_envs, n_streams=s, env_offset=offset, **kw)
                r.kind = "streams"
                return r
        r = BatchSim(track, n_envs=n_envs, env_offset=offset, **kw)
        r.kind = "one"
        return r

    def steps(r, a, k0, n, minimal):
        """Steps k0 .. k0 + n - 1 of the action block a, one call per step."""
        for k in range(k0, k0 + n):
            r.step(a[k], minimal_outputs=minimal)

    ramp = {"seconds": args.ramp_s, "steps": 0}

    def timed(r, p0, a, minimal=True):
        """W untimed steps, then K steps between barrier + synchronize (max over ranks).
        Before them, untimed steps for >= ramp_s seconds bring the clocks up
        (the timed region is unchanged: exactly K full steps)."""
        r.reset(p0)
        t_end = time.perf_counter() + args.ramp_s
        n = 0
        while time.perf_counter() < t_end:
            steps(r, a, 0, max(W, 1), minimal)
            n += max(W, 1)
            torch.cuda.synchronize(dev)
        ramp["steps"] = max(ramp["steps"], n)
        if n:
            torch.cuda.synchronize(dev)
            r.reset(p0)
        steps(r, a, 0, W, minimal)
        torch.cuda.synchronize(dev)
        r.reset_counters()
        D.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        steps(r, a, W, K, minimal)
        if hasattr(r, "join"):
            r.join()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        D.barrier()
        return D.max_over_ranks(t1 - t0)

    def count_replay(r, p0, a):
        """(lookups, rays) of the timed steps: the default ray kernel counts only in its counting build
        (f110_debug_set_simt), so the timed region runs uncounted and this replays it counted -- reset,
        the W warm-up steps, then the same K steps: trajectories are deterministic after a reset (the
        digest's premise), so the counts are the timed steps' own."""
        r.reset(p0)
        steps(r, a, 0, W, True)
        torch.cuda.synchronize(dev)
        r.set_simt(True)
        r.reset_counters()
        steps(r, a, W, K, True)
        if hasattr(r, "join"):
            r.join()
        torch.cuda.synchronize(dev)
        out = r.read_counters()
        r.set_simt(False)
        return out

    def digest(r):
        """trajectory_digest: sha256 over the obs rows (f32 bytes) of global envs
        0, G/64, 2G/64, ... after the timed steps, gathered in global-id order
        (each row hashed by its owning rank): equal for N = 1 and N > 1 runs of
        the same K / W / seed."""
        import hashlib
        stride = max(1, G // DIGEST_ENVS)
        ids = list(range(0, G, stride))[:DIGEST_ENVS]
        obs = r.obs if hasattr(r, "sims") else r.out.obs
        h = torch.zeros(len(ids), dtype=torch.int64)
        for j, gid in enumerate(ids):
            if shard.offset <= gid < shard.offset + E:
                row = obs[gid - shard.offset].cpu().numpy().tobytes()
                h[j] = int.from_bytes(hashlib.sha256(row).digest()[:7], "little") + 1
        h = D.sum_tensor_over_ranks(h)
        return {"sha256": hashlib.sha256(h.numpy().tobytes()).hexdigest()[:32], "envs": len(ids), "stride": stride}

    def secondary_c4(n):
        """BASELINE config 4 on this GPU: n two-agent envs (ego + opponent, inter-car GJK and agent
        ray_cast), the same runners and K / W as the headline, the scan check in lock-step with the
        oracle (its non-bit-exact ray_cast beams counted)."""
        sp2 = centerline_spawns(args.map.replace("_map", ""), 2)
        p2 = sp2[np.random.default_rng(args.seed + 4).integers(0, sp2.shape[0], size=n)]
        a2 = actions(W + K + 1, n, 0, n, A_=2)
        r2 = make(n, 0, kind, A_=2, spawn_=sp2)
        el2 = timed(r2, p2, a2)
        line = {"envs": n, "agents": 2, "value": n * K / el2, "ms_per_step": el2 / K * 1e3, "runner_kind": r2.kind,
                "streams": r2.S if not isinstance(r2, BatchSim) else 1}
        line["scan_check"] = scan_check_multi(O, scanner, r2, a2[W + K], cpu_threads())
        r2.close()
        if kind != policy_kind:
            r1 = make(n, 0, policy_kind, A_=2, spawn_=sp2)
            el1 = timed(r1, p2, a2)
            line["single_stream"] = {"value": n * K / el1, "ms_per_step": el1 / K * 1e3, "runner_kind": r1.kind}
            r1.close()
        return line

    runner = make(E, shard.offset, kind)
    elapsed = timed(runner, poses0, acts)
    traj = digest(runner)
    lookups, rays = count_replay(runner, poses0, acts)
    mean_look = lookups / max(rays, 1)
    total_env_steps = D.sum_over_ranks(E * K)
    RUNNER_TEXT = {
        "streams": "StreamShards: unjoined stream sub-shards of the three-launch step, actions resident in HBM",
        "one": "one BatchSim context, three launches per step (k_agents, ray kernel, k_post)"}
    sim = runner if getattr(runner, "kind", "") == policy_kind else make(E, shard.offset, policy_kind)
    prof = runner if isinstance(runner, BatchSim) else sim  # the per-kernel pass: the headline's own kernel

    # The one-context pass (what a policy loop steps) and the per-kernel profile of its kernels, in
    # alternating chunks of PC steps: an unprofiled chunk timed by the host clock between two
    # synchronizes, then a chunk whose kernels carry HIP events on their own dispatches
    # (hipExtLaunchKernel: each kernel's begin / end timestamps, as rocprofv3 records them).  Both
    # halves see the same clock and thermal state (measured one after the other, the later pass ran
    # on a hotter, slower GPU: BENCH r02 / r03 kernel_le_step), so the kernel time is checked against
    # the step that contains it.  >= 100 profiled steps whatever --steps is; not part of `value`.
    PC = 50
    KP = max(100, min(K, 300))
    prof.reset(poses0)
    t_end = time.perf_counter() + args.ramp_s
    while time.perf_counter() < t_end:
        steps(prof, acts, 0, max(W, 1), True)
        torch.cuda.synchronize(dev)
    steps(prof, acts, 0, W, True)
    torch.cuda.synchronize(dev)
    plain_s, plain_n, prof_s, prof_n = 0.0, 0, 0.0, 0
    acc = {"k_agents_ms": 0.0, "k_rays_ms": 0.0, "k_post_ms": 0.0}
    launches = 0
    koff = 0

    def chunk_rows(n):
        """First action row of a chunk of n <= K steps inside the timed block [W, W + K)."""
        nonlocal koff
        k = W + koff % (K - n + 1)
        koff += n
        return k

    while plain_n < K or prof_n < KP:
        if plain_n < K:
            n = min(PC, K - plain_n)
            k0 = chunk_rows(n)
            D.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            steps(prof, acts, k0, n, True)
            torch.cuda.synchronize(dev)
            plain_s += D.max_over_ranks(time.perf_counter() - t0)
            plain_n += n
        if prof_n < KP:
            n = min(PC, KP - prof_n, K)
            k0 = chunk_rows(n)
            t0 = time.perf_counter()
            prof.profile_begin(n)
            steps(prof, acts, k0, n, True)
            pk = prof.profile_end()  # per-launch means over this chunk
            torch.cuda.synchronize(dev)
            prof_s += time.perf_counter() - t0
            nl = pk["steps"]  # one launch of each kernel per step
            for key in acc:
                acc[key] += pk[key] * nl
            launches += nl
            prof_n += n
    per_kernel = {key: acc[key] / max(launches, 1) for key in acc}
    per_kernel["steps"] = launches

    def runner_ray_time(r, n_steps):
        """The timed runner's own ray time (StreamShards: its sub-shards' ray launches run concurrently on
        their streams): every launch's begin / end (HIP events on the kernels' own dispatches, against one
        reference event), the union of those intervals over chunks of PC steps, per step; and each
        launch's mean duration (what rocprofv3 averages per kernel).  Not part of `value`."""
        union = 0.0
        durs = []
        done = 0
        wall = 0.0
        while done < n_steps:
            n = min(PC, n_steps - done, K)
            k0 = chunk_rows(n)
            ref = torch.cuda.Event(enable_timing=True)
            ref.record(torch.cuda.current_stream(dev))
            for sm in r.sims:
                sm.profile_begin(n)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            steps(r, acts, k0, n, True)
            r.join()
            torch.cuda.synchronize(dev)
            wall += time.perf_counter() - t0
            iv = []
            for sm in r.sims:
                st = sm.profile_stamps(ref, n)
                sm.profile_end()
                iv += [(float(a), float(b)) for a, b in st[:, 2:4]]
                durs += list(st[:, 3] - st[:, 2])
            iv.sort()
            cur_a, cur_b = iv[0]
            for a_, b_ in iv[1:]:
                if a_ > cur_b:
                    union += cur_b - cur_a
                    cur_a, cur_b = a_, b_
                else:
                    cur_b = max(cur_b, b_)
            union += cur_b - cur_a
            done += n
        return {"ray_union_ms_per_step": union / n_steps, "launch_ms_mean": float(sum(durs) / len(durs)),
                "launches_per_step": len(r.sims), "steps": n_steps, "pass_wall_ms_per_step": wall / n_steps * 1e3}

    timed_rays = runner_ray_time(runner, KP) if not isinstance(runner, BatchSim) else None
    prof_step_ms = prof_s / max(prof_n, 1) * 1e3  # wall time per profiled step (events included)
    plain_step_ms = plain_s / max(plain_n, 1) * 1e3
    single = None
    if prof is not runner:
        single = {"value": total_env_steps / (plain_s * K / max(plain_n, 1)), "ms_per_step": plain_step_ms,
                  "runner": RUNNER_TEXT[policy_kind] + ", minimal outputs",
                  "timing": f"{plain_n} steps in chunks of {PC} between synchronizes, alternating with the "
                            f"per-kernel profiled chunks (roofline.kernel_ms)"}
    # SIMT efficiency of the ray loop: its lane-slot counter costs ~2 % of k_rays, so it runs on 50 more
    # steps after the timed passes, not inside them
    prof.set_simt(True)
    prof.reset_counters()
    simt_steps = min(K, 50)
    steps(prof, acts, W, simt_steps, True)
    loop_lookups, lane_slots = prof.read_simt()
    other_loads = prof.read_counter(3)  # the loop's other wave-level vector loads (tables, re-gathers)
    scalar_looks = prof.read_counter(4)  # k_rays_fxs: lookups of one-ray slots gathered by scalar loads
    closed_trips = prof.read_counter(5)  # k_rays_fxs: slot-trips of a closed slot (no gather issued)
    prof.set_simt(False)
    full_outputs = None
    if not args.no_full_outputs:
        el_full = timed(sim, poses0, acts, minimal=False)
        full_outputs = {"value": total_env_steps / el_full, "ms_per_step": el_full / K * 1e3,
                        "runner": RUNNER_TEXT[policy_kind] + ", every output (f32 + f64 scans, laps, sim_time, "
                                                             "was_reset)"}

    O = scanner = None
    checks = None
    if rank == 0:
        O = oracle_module()
        scanner = O.OracleScanner(track.free_mask, track.resolution, track.origin)
        checks = scan_check(O, scanner, runner, acts[W + K], cpu_threads())

    B = prof.B
    # the dominant kernel: k_rays.  Per ray 4 B per EDT lookup (exact uint32 k
    # cell) + 4 B of f32 range out; the 120 B/agent of state I/O
    # go with the step (k_agents).
    kernel_bytes = E * A * B * (4.0 * mean_look + 4.0)
    one_ms = per_kernel["k_rays_ms"]  # the one-context runner's ray launch, per step
    # the roofline of the timed runner's own ray launches: with stream sub-shards, the union of their
    # (concurrent) launch intervals per step; with one context, its launch
    k_ms = timed_rays["ray_union_ms_per_step"] if timed_rays else one_ms
    achieved = kernel_bytes / (k_ms * 1e-3) / 1e9
    pmc = load_profile("pmc_traffic", E, A)
    busy = load_profile("pmc_busy", E, A)
    traffic = pmc.get("bytes_per_launch") if pmc else None
    roof = {
        "kernel": "k_rays",
        "timed_runner": (
            {"ray_kernel": ray_kernel_name(runner.sims[0], shared=runner.S > 1) +
                           f", {runner.S} concurrent sub-shard launches per step",
             "kernel_ms_is": "the union of the sub-shards' ray-launch intervals per step (HIP events on the "
                             "kernels' own dispatches)", **timed_rays}
            if timed_rays else {"ray_kernel": ray_kernel_name(runner), "kernel_ms_is": "the one launch per step"}),
        "one_context": {"ray_kernel": ray_kernel_name(prof), "kernel_ms": one_ms,
                        "achieved": kernel_bytes / (one_ms * 1e-3) / 1e9,
                        "frac": kernel_bytes / (one_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "profiled_launches": per_kernel["steps"]},
        "profiled_steps": KP,
        "profiled_launches": per_kernel["steps"],
        "bound": ("the texture-address path, per wave-level vector load (gather_roofline.ta_cycles_per_load TA cycles "
                  "each whatever its lanes do; HBM is not the limit: see hbm_traffic_frac; DESIGN.md 3.9)" if prof.ray_kernel == 3 and prof.ray_refill > 0
                  else "latency of the dependent EDT gather chain (HBM is not the limit: see hbm_traffic_frac; capping "
                  "occupancy at 6/4/2 waves per SIMD costs 1.31x/1.62x/2.9x, DESIGN.md 3.2)"),
        "ray_kernel": (ray_kernel_name(runner.sims[0], shared=runner.S > 1) if timed_rays else ray_kernel_name(runner)),
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic, "kernel_ms": k_ms, "algorithmic_bytes_per_launch": kernel_bytes,
        "kernel_ms_note": "per step: the timed runner's ray time (timed_runner.kernel_ms_is); bytes: all of the "
                          "step's cars (every sub-shard launch), lookups from a counting replay of the timed steps",
        "mean_lookups_per_ray": mean_look,
        "step_kernels_ms_one_context": {"k_agents": per_kernel["k_agents_ms"], "k_rays": one_ms,
                                        "k_post": per_kernel["k_post_ms"]},
        "step_algorithmic_bytes_per_env": algorithmic_bytes_per_env_step(B, A, mean_look),
        # vector-gathered lookups of the loop / (64 x the wave-level vector gathers it issued, the ended
        # lanes' zero-cell reads included), from the kernel's own counters; lookups a k_rays_fxs slot
        # gathered by scalar loads (one ray left) are counted apart
        "simt_efficiency": (loop_lookups - scalar_looks) / lane_slots if lane_slots else None,
        "scalar_gathered_lookups_per_launch": scalar_looks / max(1, simt_steps),
        "closed_slot_trips_per_launch": closed_trips / max(1, simt_steps),
    }
    # the gather bound, per instruction, the form the counters show: the texture-address
    # unit spends ~20.1 cycles (measured) on every wave-level load whatever its lanes do, so the
    # kernel's vector loads need at least loads x 20.1 / 256 CUs / 2.4 GHz.  Loads per launch from the
    # kernel's own counters: the loop's gathers (lane slots / 64) + its table loads and guard-band
    # re-gathers (counter 3); compare with SQ_INSTS_VMEM_RD in profiles/
    look_launch = E * A * B * (mean_look - 1.0)  # the kernel's own lookups (the first is k_agents')
    ta_cyc = TA_CYCLES_PER_LOAD
    ta_src = "fallback constant (round 3, 65536 cars)"
    if busy and busy.get("ta_cycles_per_vmem_rd"):
        ta_cyc = float(busy["ta_cycles_per_vmem_rd"])
        ta_src = busy["file"]
    roof["gather_roofline"] = {"bound": "texture-address cycles per wave-level vector load (measured)",
                               "lookups_per_launch": look_launch, "ta_cycles_per_load": ta_cyc,
                               "ta_cycles_source": ta_src}
    if lane_slots:
        gathers = lane_slots / 64.0 / max(1, simt_steps)  # per launch
        loads = gathers + other_loads / max(1, simt_steps)
        min_ms = loads * ta_cyc / N_CU / (CLOCK_GHZ * 1e9) * 1e3
        # the counts and the TA cycles per load are the one-context kernel's (its SIMT pass, its PMC file)
        roof["gather_roofline"].update({"slot_gathers_per_launch": gathers, "vmem_loads_per_launch": loads,
                                        "ta_min_ms": min_ms, "ta_frac_one_context": min_ms / one_ms})
    # consistency: each kernel runs inside the step it is timed in (the timed runner's ray time against its
    # ms_per_step; the one-context launch against that runner's own wall time per step, measured in the
    # chunks interleaved with the profiled ones)
    pass_ms = timed_rays["pass_wall_ms_per_step"] if timed_rays else plain_step_ms
    roof["kernel_le_step"] = {"ok": bool(k_ms <= pass_ms and one_ms <= plain_step_ms), "kernel_ms": k_ms,
                              "kernel_pass_ms_per_step": pass_ms, "timed_ms_per_step": elapsed / K * 1e3,
                              "one_context_kernel_ms": one_ms,
                              "one_context_step_ms": plain_step_ms, "profiled_pass_step_ms": prof_step_ms,
                              "one_context_kernels_sum_ms": sum(per_kernel[k] for k in ("k_agents_ms", "k_rays_ms",
                                                                                          "k_post_ms"))}
    if pmc and traffic:
        roof["hbm_traffic_gbs"] = traffic / (k_ms * 1e-3) / 1e9
        roof["hbm_traffic_frac"] = roof["hbm_traffic_gbs"] / HBM_PEAK_GBS
        if pmc.get("write_bytes"):
            roof["write_ratio"] = pmc["write_bytes"] / (E * A * B * 4.0)
        roof["l2_hit_rate"] = pmc.get("l2_hit_rate")
        roof["traffic_source"] = pmc["file"]
    if busy:
        for k in ("valu_busy", "waves_per_simd"):
            if k in busy:
                roof[k] = busy[k]
        roof["busy_source"] = busy["file"]

    result = {
        "metric": metric_name(G, A),
        "value": total_env_steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: i.i.d. uniform random actions, centerline spawn poses, Spielberg map",
        "config": {
            "workload": f"{G} {'single' if A == 1 else f'{A}'}-agent envs"
                        + (f" ({E} per GPU x {world})" if world > 1 else " on one GPU"),
            "global_envs": G, "envs_per_gpu": E, "agents": A, "beams": B, "map": args.map,
            "integrator": "RK4", "scan_noise": not args.no_noise, "autoreset": True,
            "parallelism": f"env-shard x{world} (no collectives)",
            "dist": D.describe(),
            "streams_per_gpu": runner.S if not isinstance(runner, BatchSim) else 1,
            "ramp": ramp,
            "runner": RUNNER_TEXT[runner.kind] + "; minimal outputs (obs, collisions, terminated): no f32 "
                      "info['scans'] copy, lap_times/counts, sim_time, was_reset",
            "runner_kind": runner.kind,
        },
        "trajectory_digest": traj,
        "single_stream": single,
        "single_stream_full_outputs": full_outputs,
        "scan_l2_vs_cpu": checks["l2"] if checks and "l2" in checks else None,
        "scan_check": checks,
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_secondary:
        sec = {}
        for label, n in (("C3_shard_8192", 8192), ("C2_4096", 4096)):
            if n >= E:
                continue
            p2 = spawn[rng.integers(0, spawn.shape[0], size=n)]
            a2 = actions(W + K, n, 0, n)
            r2 = make(n, 0, kind)
            el2 = timed(r2, p2, a2)
            line = {"envs": n, "value": n * K / el2, "ms_per_step": el2 / K * 1e3, "runner_kind": r2.kind,
                    "streams": r2.S if not isinstance(r2, BatchSim) else 1}
            r2.close()
            if kind != policy_kind:
                r1 = make(n, 0, policy_kind)
                el1 = timed(r1, p2, a2)
                line["single_stream"] = {"value": n * K / el1, "ms_per_step": el1 / K * 1e3, "runner_kind": r1.kind}
                r1.close()
            sec[label] = line
        if A == 1:
            sec["C4_8192x2"] = secondary_c4(8192)
        result["secondary"] = sec
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            T = args.cpu_warmup + args.cpu_steps
            a_cpu = acts if acts.shape[0] >= T else actions(T, E, shard.offset, G)
            n = min(args.cpu_envs, E)
            result["cpu_baseline"] = cpu_baseline(O, scanner, poses0[:n], a_cpu[:T, :n].cpu().numpy(), args)
        except Exception as exc:  # report, never hide
            result["cpu_baseline"] = {"error": repr(exc)}
    if sim is not runner:
        sim.close()
    runner.close()
    if rank == 0 and world == 1 and not args.no_secondary and A == 1:
        # BASELINE config 5's per-GPU share (4096 two-agent envs, the batched train_ddpg loop)
        c5 = run_ddpg(args, 4096, K, max(W, 2))
        result["secondary"]["C5_ddpg_4096"] = {k: c5[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup",
                                                                 "phases_ms", "learner_roofline", "learner")}
        result["secondary"]["C5_ddpg_4096"]["workload"] = c5["config"]["workload"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
