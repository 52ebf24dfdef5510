"""A short run of the single-agent step on one context, three-launch then
fused (k_step1), for rocprofv3 counter passes (GPU box):

    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ... -- python scripts/fused_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402

E = int(os.environ.get("FP_ENVS", 65536))
K = int(os.environ.get("FP_STEPS", 10))
tm = load_map("Spielberg_map")
sp = centerline_spawns("Spielberg", 1)
p0 = sp[np.random.default_rng(1).integers(0, sp.shape[0], E)]
g = torch.Generator(device="cuda")
g.manual_seed(0)
acts = torch.rand(K, E, 1, 2, device="cuda", generator=g)
acts[..., 0] = acts[..., 0] * 0.8378 - 0.4189
acts[..., 1] *= 20
MODES = os.environ.get("FP_MODES", "three,fused").split(",")
for fused in [m == "fused" for m in MODES]:
    r = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=sp, seed=7)
    r.set_fused(fused)
    r.reset(p0)
    for s in range(K):
        r.step(acts[s], minimal_outputs=True)
    torch.cuda.synchronize()
    r.close()
print("done")
