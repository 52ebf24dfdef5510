"""Counter-collection target: 100 f110_step launches at MB_ENVS envs (bench
workload), nothing else on the GPU.  Used with rocprofv3 --pmc.  Heavy-first
dispatch is off unless MB_HEAVY=1, as in the bench's timed runner
(streams.StreamShards turns it off)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
from f110_gymnasium_ros2_jazzy_amd.maps import load_map, centerline_spawns
E = int(os.environ.get("MB_ENVS", 8192))
A = int(os.environ.get("MB_AGENTS", 1))
sp = centerline_spawns("Spielberg", A)
sim = BatchSim(load_map("Spielberg_map"), n_envs=E, n_agents=A, autoreset=True, spawn_poses=sp)
if os.environ.get("MB_HEAVY", "0") != "1":
    from f110_gymnasium_ros2_jazzy_amd import _lib
    _lib.check(sim.L.f110_debug_disable_heavy_first(sim.ctx), "f110_debug_disable_heavy_first")
if os.environ.get("MB_REFILL"):  # a forced ray kernel: k_rays_fxs (waves per car) or, with 0, k_rays_fx(n)
    sim.set_ray_lanes(int(os.environ.get("MB_LANES", 2)))
    sim.set_ray_refill(int(os.environ["MB_REFILL"]))
sim.reset(sp[np.random.default_rng(0).integers(0, sp.shape[0], E)])
g = torch.Generator(device="cuda"); g.manual_seed(0)
acts = torch.rand(100, E, A, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189; acts[..., 1] *= 20
# RAY_PMC_COUNTS=<path>: the same launches also keep the kernel's own load counters (lane slots of
# the loop's gathers, counter 3 = its other wave-level loads; returnless lane-0 atomics, no reads),
# written to <path> beside the PMC pass that counts SQ_INSTS_VMEM_RD on them
counts = os.environ.get("RAY_PMC_COUNTS")
p0 = sp[np.random.default_rng(0).integers(0, sp.shape[0], E)]
for k in range(100):
    sim.step(acts[k], minimal_outputs=True)
torch.cuda.synchronize()
if counts:  # k_rays_fxs counts in its COUNT build (another kernel name, left out of the PMC averages):
    # the same 100 steps again from the same reset, counted
    sim.reset(p0)
    sim.set_simt(True)
    sim.reset_counters()
    for k in range(100):
        sim.step(acts[k], minimal_outputs=True)
    torch.cuda.synchronize()
    import json
    _, slots = sim.read_simt()
    other = sim.read_counter(3)
    with open(counts, "w") as f:
        json.dump({"envs": E, "agents": A, "launches": 100, "ray_kernel": sim.ray_kernel, "lanes": sim.ray_lanes,
               "refill": sim.ray_refill, "scalar_gathers_per_launch": sim.read_counter(4) / 100.0,
               "closed_slot_trips_per_launch": sim.read_counter(5) / 100.0,
               "slot_gathers_per_launch": slots / 64.0 / 100,
                   "other_loads_per_launch": other / 100.0, "vmem_loads_per_launch": (slots / 64.0 + other) / 100},
                  f)
print("done")
