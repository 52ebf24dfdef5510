"""Per-GPU shard rules (GPU box): env-steps/s of one GPU's E envs stepped as S
stream sub-shards (streams.StreamShards) for each ray-kernel choice, in one
process, interleaved rounds (the bench's timing: clock ramp, W warm-up, K
timed steps between synchronizes).  The choices are (rays per lane, waves per
car of k_rays_fxs): (1, 0) k_rays_fx, (2, 0) k_rays_fxn<2>, (2, w) k_rays_fxs
with w waves per car; (0, w): the bench's own sub-shards (f110_set_device_share:
single-agent k_rays_fxs with the LDS theta table) with their waves per car set
to w afterwards (0: the size rule's).  Bit-identity of the obs rows against the
first choice is checked after the timed steps.  Prints one JSON line per (E, S).

    SR_ENVS=8192,4096 SR_STREAMS=1,2,4 SR_CHOICES=1:0,2:1 python scripts/shard_rules.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.streams import StreamShards  # noqa: E402


def main():
    envs = [int(x) for x in os.environ.get("SR_ENVS", "8192").split(",")]
    streams = [int(x) for x in os.environ.get("SR_STREAMS", "4").split(",")]
    choices = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("SR_CHOICES", "1:0,2:1").split(",")]
    K = int(os.environ.get("SR_STEPS", 300))
    W = int(os.environ.get("SR_WARMUP", 30))
    rounds = int(os.environ.get("SR_ROUNDS", 3))
    A = int(os.environ.get("SR_AGENTS", 1))
    dev = torch.device("cuda:0")
    track = load_map("Spielberg_map")
    track.ensure_edt()
    spawn = centerline_spawns("Spielberg", A)
    for E in envs:
        rng = np.random.default_rng(12345)
        p0 = spawn[rng.integers(0, spawn.shape[0], E)]
        g = torch.Generator(device=dev)
        g.manual_seed(12345)
        acts = torch.rand(W + K, E, A, 2, device=dev, generator=g)
        acts[..., 0] = acts[..., 0] * (2 * 0.4189) - 0.4189
        acts[..., 1] *= 20.0
        for S in streams:
            if E % S:
                continue
            kw = dict(n_agents=A, device=dev, seed=12345, noise_std=0.01, autoreset=True, spawn_poses=spawn)
            if os.environ.get("SR_INTEGRATOR"):  # 1: RK4, 2: Euler (probe of k_agents' share of a small shard's step)
                kw["integrator"] = int(os.environ["SR_INTEGRATOR"])
            runs = {}
            for lanes, refill in choices:
                name = f"lanes{lanes}_refill{refill}" if lanes else f"shared_refill{refill}"
                if lanes == 0:  # the bench's runner (device share), then its waves per car
                    r = (StreamShards(track, n_envs=E, n_streams=S, **kw) if S > 1
                         else BatchSim(track, n_envs=E, **kw))
                    if refill:
                        for sm in getattr(r, "sims", [r]):
                            sm.set_ray_refill(refill)
                elif S == 1:
                    r = BatchSim(track, n_envs=E, **kw)
                    r.set_ray_lanes(lanes)
                    r.set_ray_refill(refill)
                else:
                    r = StreamShards(track, n_envs=E, n_streams=S, ray_lanes=lanes, refill=refill, **kw)
                runs[name] = r
            times = {n: [] for n in runs}
            last = {}
            for _ in range(rounds):
                for n, r in runs.items():
                    r.reset(p0)
                    t_end = time.perf_counter() + 0.5
                    while time.perf_counter() < t_end:  # clock ramp
                        for k in range(W):
                            r.step(acts[k], minimal_outputs=True)
                        torch.cuda.synchronize()
                    r.reset(p0)
                    for k in range(W):
                        r.step(acts[k], minimal_outputs=True)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in range(W, W + K):
                        r.step(acts[k], minimal_outputs=True)
                    if hasattr(r, "join"):
                        r.join()
                    torch.cuda.synchronize()
                    times[n].append(time.perf_counter() - t0)
                    last[n] = (r.obs if hasattr(r, "sims") else r.out.obs).clone()
            ref = next(iter(last.values()))
            line = {"envs": E, "agents": A, "streams": S, "steps": K, "rounds": rounds}
            for n in runs:
                t = float(np.median(times[n]))
                line[n] = {"value": E * K / t, "ms_per_step": t / K * 1e3,
                           "identical": bool(torch.equal(last[n], ref))}
            print(json.dumps(line), flush=True)
            for r in runs.values():
                r.close()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
