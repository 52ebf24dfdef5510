"""SIMT efficiency of the one-ray-per-lane sphere trace (run on the GPU box).

Per-ray EDT lookup counts come from f110_scan_batch's probe output at
bench-like poses (centerline spawns + jitter).  Reports:
  * SIMT efficiency = mean lookups / mean over waves of the wave's longest ray
  * the share of wave-iterations spent in waves whose longest ray is > 40
  * what two alternative schedules would save, in wave-iterations:
    - "evict": a wave hands its last <= T active rays to a tail pass once it
      has run >= Kmin iterations; the tail pass traces them 64 per wave
    - "split": rays predicted long (> K lookups at the previous pose) traced
      in a separate compacted pass
  * the ideal (perfect lane refill) = sum(lookups) / 64
Writes one JSON line (profiles/<tag>_simt.json when --out is given).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim  # noqa: E402


def waves(x):
    n = -(-x.size // 64)
    return np.concatenate([x, np.zeros(n * 64 - x.size, x.dtype)]).reshape(-1, 64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=8192)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    N = args.poses
    rng = np.random.default_rng(0)
    sp = centerline_spawns("Spielberg", 1)
    p1 = sp[rng.integers(0, sp.shape[0], N), 0]
    p1 = p1 + np.stack([rng.normal(0, .2, N), rng.normal(0, .2, N), rng.normal(0, .2, N)], 1)
    v = rng.uniform(0, 0.2, N)   # one step later: <= 0.2 m along the heading
    p2 = p1.copy()
    p2[:, 0] += v * np.cos(p1[:, 2])
    p2[:, 1] += v * np.sin(p1[:, 2])
    p2[:, 2] += rng.normal(0, 0.01, N)
    sim = BatchSim(load_map("Spielberg_map"), n_envs=1, n_agents=1)
    L1 = sim.scan_batch(torch.as_tensor(p1), probe=True)[1].cpu().numpy().reshape(-1).astype(np.int64)
    L2 = sim.scan_batch(torch.as_tensor(p2), probe=True)[1].cpu().numpy().reshape(-1).astype(np.int64)
    W = waves(L2)
    wmax = W.max(1)
    base = wmax.sum()
    res = {"poses": N, "mean_lookups": float(L2.mean()), "max_lookups": int(L2.max()),
           "mean_wave_max": float(wmax.mean()), "simt_efficiency": float(L2.mean() / wmax.mean()),
           "wave_iter_share_in_waves_max_gt_40": float(wmax[wmax > 40].sum() / base),
           "waves_max_gt_40": float((wmax > 40).mean()),
           "ideal_refill_vs_now": float(L2.sum() / 64 / base)}
    ev = {}
    for T, Kmin in ((4, 16), (8, 16), (16, 8)):
        ph1, tail = 0, []
        for w in W:
            m = w.max()
            stop = next((i for i in range(Kmin, m + 1) if (w > i).sum() <= T), None)
            if stop is None or stop >= m:
                ph1 += m
                continue
            ph1 += stop
            tail += list(w[w > stop] - stop)
        tail = np.asarray(tail, np.int64)
        ph2 = waves(tail).max(1).sum() if tail.size else 0
        ev[f"T{T}_K{Kmin}"] = float((ph1 + ph2) / base)
    res["evict_vs_now"] = ev
    sp_ = {}
    for K in (24, 32, 48):
        pred = L1 > K
        s_it = waves(np.where(pred, 0, L2)).max(1).sum()
        l_it = waves(L2[pred]).max(1).sum() if pred.any() else 0
        sp_[f"K{K}"] = float((s_it + l_it) / base)
    res["split_prev_step_vs_now"] = sp_
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    sim.close()


if __name__ == "__main__":
    main()
