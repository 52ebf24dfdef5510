"""k_agents' per-wave phase times (GPU box, a timing build via F110_LIB: hipcc ...
-DF110_AGENTS_PHASES with the _build.py flags and sources, e.g. ab_libs/agents_phases.so):
counters 8-11 = summed s_memrealtime ticks (100 MHz) per wave of prologue + reset, update_pose
(RK4), scan pose + first EDT lookup, beam runs; 13 = waves.  Single-agent envs, autoreset,
random actions, RK4 and Euler.  The phase edges are scheduling barriers, not memory fences: a
load issued in one phase may be waited for in the next.  One JSON line (us per wave).

    F110_LIB=ab_libs/agents_phases.so python scripts/agents_phases.py
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


def main():
    out = {"runs": []}
    track = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)
    for integ, name in ((_lib.INTEGRATOR_RK4, "rk4"), (_lib.INTEGRATOR_EULER, "euler")):
        for E in (2048, 8192, 65536):
            sim = BatchSim(track, n_envs=E, n_agents=1, integrator=integ, autoreset=True, spawn_poses=sp)
            rng = np.random.default_rng(0)
            sim.reset(sp[rng.integers(0, sp.shape[0], E)])
            g = torch.Generator(device="cuda").manual_seed(0)
            acts = torch.rand(250, E, 1, 2, device="cuda", generator=g)
            acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
            acts[..., 1] *= 20
            for k in range(50):
                sim.step(acts[k], minimal_outputs=True)
            torch.cuda.synchronize()
            c0 = [sim.read_counter(i) for i in range(8, 14)]
            sim.profile_begin(200)
            for k in range(50, 250):
                sim.step(acts[k], minimal_outputs=True)
            pk = sim.profile_end()
            c1 = [sim.read_counter(i) for i in range(8, 14)]
            nw = c1[5] - c0[5]
            us = [(c1[i] - c0[i]) / nw / 100.0 for i in range(4)]
            out["runs"].append({"integrator": name, "envs": E, "waves": nw, "k_agents_ms": pk["k_agents_ms"],
                                "us_per_wave": dict(zip(("prologue_reset", "update_pose", "scan_pose_first_lookup",
                                                         "beam_runs"), us))})
            sim.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
