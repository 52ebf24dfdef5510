"""Offline model of ray-to-lane schedules for the sphere trace (CPU, oracle
lookup counts).  Per-ray EDT lookup counts come from the C oracle's probe at
bench-like poses (centerline spawns + jitter); a schedule's cost is counted in
wave-iterations (one loop-body issue of a 64-lane wave) and re-arm events
(one divergent set-up/epilogue pass of a wave).

  chunk     today: one wave per 64 consecutive beams of a car, no refill
  refill_T  one wave per car, the car's beams pulled in order by idle lanes,
            a re-arm pass whenever >= T lanes are idle (or the wave would
            otherwise stall), beams taken in descending-chunk order
Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402  (test infrastructure: lookup counts only)
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402


def chunk_cost(L):
    n, B = L.shape
    nch = -(-B // 64)
    pad = np.zeros((n, nch * 64), L.dtype)
    pad[:, :B] = L
    return int(pad.reshape(n, nch, 64).max(2).sum()), n * nch


def refill_cost(L, T, order):
    """Simulate one wave per car: returns (wave_iters, rearm_events)."""
    iters = 0
    events = 0
    for row in L:
        q = row[order]
        nxt = 0
        rem = np.zeros(64, np.int64)  # lookups left per lane (0 = idle)
        B = q.size
        while True:
            idle = np.flatnonzero(rem == 0)
            if nxt < B and (idle.size >= T or idle.size == 64 or (rem > 0).sum() == 0):
                k = min(idle.size, B - nxt)
                rem[idle[:k]] = q[nxt:nxt + k]
                nxt += k
                events += 1
            act = rem > 0
            if not act.any():
                break
            # advance to the next time the idle count reaches T (or all done)
            live = np.sort(rem[act])
            need = T - (64 - live.size)  # more lanes that must finish before the next re-arm
            if nxt >= B:
                step = int(live[-1])
            elif need <= 0:
                step = 1
            else:
                step = int(live[min(need, live.size) - 1])
            rem[act] -= step
            rem[rem < 0] = 0
            iters += step
    return iters, events


def main():
    N = int(os.environ.get("RS_CARS", 512))
    rng = np.random.default_rng(0)
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)
    p = sp[rng.integers(0, sp.shape[0], N), 0]
    p = p + np.stack([rng.normal(0, .2, N), rng.normal(0, .2, N), rng.normal(0, .2, N)], 1)
    sc = O.OracleScanner(tm.free_mask, tm.resolution, tm.origin)
    _, L, _ = sc.scan(p, with_probe=True, threads=8)
    L = L.astype(np.int64)
    B = L.shape[1]
    base, waves = chunk_cost(L)
    res = {"cars": N, "mean_lookups": float(L.mean()), "chunk_wave_iters_per_car": base / N,
           "ideal_wave_iters_per_car": float(L.sum() / 64 / N), "chunk_waves_per_car": waves / N}
    nch = -(-B // 64)
    desc = np.concatenate([np.arange(k * 64, min(B, k * 64 + 64)) for k in range(nch - 1, -1, -1)])
    for T in (1, 8, 16, 24, 32, 48):
        it, ev = refill_cost(L, T, desc)
        res[f"refill_T{T}"] = {"wave_iters_per_car": it / N, "rearm_events_per_car": ev / N,
                               "vs_chunk": it / base}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
