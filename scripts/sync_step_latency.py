"""Per-step latency with a host sync (and a short host gap) between steps, per
ray-dispatch variant: the F110Env facade's usage pattern.  Prints JSON."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
tm = load_map("Spielberg_map")
res = {}
for E in (1, 8192):
    sp = centerline_spawns("Spielberg", 1)
    p0 = sp[np.random.default_rng(0).integers(0, sp.shape[0], E)]
    for name, env in (("flat", {"F110_RAY_KERNEL": "1"}), ("chunk_desc", {"F110_RAY_KERNEL": "2"}),
                      ("chunk_asc", {"F110_RAY_KERNEL": "2", "F110_CHUNK_ORDER": ",".join(map(str, range(17)))})):
        os.environ.pop("F110_CHUNK_ORDER", None)
        os.environ.update(env)
        sim = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp)
        sim.reset(p0)
        a = torch.rand(E, 1, 2, device="cuda"); a[..., 1] *= 5
        for _ in range(20):
            sim.step(a, minimal_outputs=True)
        torch.cuda.synchronize()
        ts = []
        for k in range(30):
            time.sleep(0.02 if k % 3 == 0 else 0.0)
            t0 = time.perf_counter()
            sim.step(a, minimal_outputs=True)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res[f"{name}_E{E}_ms"] = [round(float(np.median(ts)), 3), round(float(np.max(ts)), 3)]
        sim.close()
print(json.dumps(res))
