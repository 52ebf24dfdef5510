"""Offline model: k_rays_fxr's two chunk slots over beams ordered by the
previous step's per-beam lookup counts (temporal coherence), against the
natural (descending-chunk) order.  Counts from the C oracle's probe at two
consecutive steps of a random-action rollout (CPU; oracle = test
infrastructure, lookup counts only).

    python scripts/sorted_chunk_model.py -> one JSON line
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402
from lane_refill_model import sim_chunk  # noqa: E402


def two_step_counts(n_envs=1024, steps=50, seed=0):
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)[:, 0]
    sc = O.OracleScanner(tm.free_mask, tm.resolution, tm.origin)
    sim = O.OracleSim(sc, n_envs, 1)
    rng = np.random.default_rng(seed)
    sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
    Ls = []
    for t in range(1, steps + 3):
        a = np.stack([rng.uniform(-0.4189, 0.4189, n_envs), rng.uniform(0, 20, n_envs)], 1)
        _, col = sim.step(a[:, None, :], threads=8)
        if t >= steps + 1:
            p = np.stack([sim.state[:, 0], sim.state[:, 1], sim.state[:, 4]], 1)
            _, L, _ = sc.scan(p, with_probe=True, threads=8)
            Ls.append(L.astype(np.int32))
        elif col[:, 0].any():
            hit = np.flatnonzero(col[:, 0] > 0)
            st = sim.state.copy()
            sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
            keep = np.ones(n_envs, bool)
            keep[hit] = False
            sim.state[keep] = st[keep]
    return Ls[0], Ls[1]


def main():
    L0, L1 = two_step_counts()
    n, B = L1.shape
    nch = -(-B // 64)
    nat, _ = sim_chunk(L1)
    # sorted: beams by the previous step's count, most expensive first; sim_chunk
    # traces chunks in descending index order, so put the heaviest beams last
    order = np.argsort(L0, axis=1, kind="stable")  # ascending: heaviest at the end
    Ls = np.take_along_axis(L1, order, 1)
    srt, _ = sim_chunk(Ls)
    oracle_order = np.argsort(L1, axis=1, kind="stable")
    best, _ = sim_chunk(np.take_along_axis(L1, oracle_order, 1))
    lane = (L1 - 1).sum(1)
    res = {"cars": int(n), "beams": int(B),
           "natural": {"wave_iters_per_car": float(nat.mean()), "simt": float(lane.sum() / (nat.sum() * 128))},
           "prev_step_sorted": {"wave_iters_per_car": float(srt.mean()), "simt": float(lane.sum() / (srt.sum() * 128))},
           "this_step_sorted": {"wave_iters_per_car": float(best.mean()), "simt": float(lane.sum() / (best.sum() * 128))},
           "count_change": {"mean_abs": float(np.abs(L1 - L0).mean()), "corr": float(np.corrcoef(L0.ravel(), L1.ravel())[0, 1])}}
    print(json.dumps(res))


if __name__ == "__main__" and not os.environ.get("SC_CHUNK"):
    main()


def chunk_order_model():
    """Chunk-level orders for the two slots (whole 64-beam chunks, as
    k_rays_fxr traces them): descending index (today) against the previous
    step's per-chunk max lookups, longest first (LPT)."""
    L0, L1 = two_step_counts()
    n, B = L1.shape
    nch = -(-B // 64)
    pad0 = np.ones((n, nch * 64), np.int64)
    pad1 = np.ones((n, nch * 64), np.int64)
    pad0[:, :B] = L0
    pad1[:, :B] = L1
    c0 = pad0.reshape(n, nch, 64).max(2)
    res = {}
    for name, order in (("descending", np.tile(np.arange(nch)[::-1], (n, 1))),
                        ("prev_lpt", np.argsort(-c0, axis=1, kind="stable")),
                        ("this_lpt", np.argsort(-pad1.reshape(n, nch, 64).max(2), axis=1, kind="stable"))):
        # sim_chunk traces chunks in descending index order: hand it the chunks
        # already permuted and reversed
        ch = pad1.reshape(n, nch, 64)
        perm = np.take_along_axis(ch, order[:, :, None], 1)[:, ::-1].reshape(n, nch * 64)
        it, ev = sim_chunk(perm[:, :nch * 64])
        res[name] = {"wave_iters_per_car": float(it.mean()), "simt": float((L1 - 1).sum() / (it.sum() * 128))}
    print(json.dumps(res))


if __name__ == "__main__" and os.environ.get("SC_CHUNK"):
    chunk_order_model()
