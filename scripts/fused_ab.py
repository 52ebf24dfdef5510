"""Wall time per step of the single-agent step runners (GPU box): the
three-launch step on one context, k_step1 one launch per step (f110_set_fused),
k_step1 over n steps per launch (f110_step_n), and StreamShards sub-shards;
after a 1 s clock ramp, K timed steps between synchronizes, best of R rounds.
Prints one JSON line.

    FA_ENVS=65536,8192,4096 FA_STEPS=200 FA_CHUNK=50 python scripts/fused_ab.py
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
    envs = [int(x) for x in os.environ.get("FA_ENVS", "65536,8192,4096").split(",")]
    K = int(os.environ.get("FA_STEPS", 200))
    chunk = int(os.environ.get("FA_CHUNK", 50))
    rounds = int(os.environ.get("FA_ROUNDS", 3))
    modes = os.environ.get("FA_MODES", "three,fused,fused_n,streams").split(",")
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)
    out = {"steps": K, "chunk": chunk, "by_envs": {}}
    for E in envs:
        rng = np.random.default_rng(12345)
        p0 = sp[rng.integers(0, sp.shape[0], E)]
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        acts = torch.rand(K + 20, E, 1, 2, device="cuda", generator=g)
        acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
        acts[..., 1] *= 20
        line = {}
        for mode in modes:
            kw = dict(n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=7)
            if mode == "streams":
                S = 4 if E <= 16384 else 2
                r = StreamShards(tm, n_envs=E, n_streams=S, **kw)
            else:
                r = BatchSim(tm, n_envs=E, **kw)
                r.set_fused(mode != "three")
            best = None
            for _ in range(rounds):
                r.reset(p0)
                t_end = time.perf_counter() + 1.0
                k = 0
                while time.perf_counter() < t_end:  # clock ramp
                    r.step(acts[k % 20], minimal_outputs=True)
                    k += 1
                    if k % 16 == 0:
                        torch.cuda.synchronize()
                r.reset(p0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode == "fused_n":
                    for s in range(0, K, chunk):
                        r.step_n(acts[s:min(K, s + chunk)], minimal_outputs=True)
                else:
                    for s in range(K):
                        r.step(acts[s], minimal_outputs=True)
                if hasattr(r, "join"):
                    r.join()
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                best = el if best is None else min(best, el)
            line[mode] = {"ms_per_step": best / K * 1e3, "env_steps_per_s": E * K / best}
            r.close()
        out["by_envs"][str(E)] = line
        print(json.dumps({E: line}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
