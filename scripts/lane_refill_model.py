"""Offline model of one-wave-per-car ray schedules (CPU, oracle lookup counts).

Per-ray EDT lookup counts come from the C oracle's probe at bench-like car
states: a random-action rollout (steer U(+-0.4189), speed U(0, 20), the
bench's distribution) of OracleSim with crashed cars respawned on the
centerline, sampled every 10 steps.  A schedule is simulated iteration by
iteration for every car at once and costed in

  iters   wave-iterations (one pass of the loop body over all NS slots)
  events  refill passes (a divergent finish + re-arm section of the wave)
  served  rays finished per refill pass

Schedules:
  chunk   k_rays_fxr today: NS 64-beam chunk slots, a slot re-armed with the
          car's next chunk when all 64 of its rays have ended
  lane    NS ray slots per lane, the car's beams pulled from one queue by
          idle slots; a refill pass whenever >= T slots have ended (or no
          slot is still tracing)

    python scripts/lane_refill_model.py  -> one JSON line per schedule
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402  (test infrastructure: lookup counts only)
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402


def rollout_counts(n_envs=2048, steps=100, every=10, seed=0):
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)[:, 0]
    sc = O.OracleScanner(tm.free_mask, tm.resolution, tm.origin)
    sim = O.OracleSim(sc, n_envs, 1)
    rng = np.random.default_rng(seed)
    sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
    out = []
    for t in range(1, steps + 1):
        a = np.stack([rng.uniform(-0.4189, 0.4189, n_envs), rng.uniform(0, 20, n_envs)], 1)
        _, col = sim.step(a[:, None, :], threads=8)
        if t % every == 0:
            p = np.stack([sim.state[:, 0], sim.state[:, 1], sim.state[:, 4]], 1)
            _, L, _ = sc.scan(p, with_probe=True, threads=8)
            out.append(L.astype(np.int32))
        hit = np.flatnonzero(col[:, 0] > 0)
        if hit.size:  # autoreset: respawn crashed cars
            st = sim.state.copy()
            sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
            keep = np.ones(n_envs, bool)
            keep[hit] = False
            sim.state[keep] = st[keep]
    return np.concatenate(out)


def sim_chunk(L, NS=2):
    n, B = L.shape
    nch = -(-B // 64)
    pad = np.zeros((n, nch * 64), np.int64)
    pad[:, :B] = L - 1
    ch = pad.reshape(n, nch, 64)[:, ::-1]  # descending chunks
    tot = np.zeros(n, np.int64)
    ev = np.zeros(n, np.int64)
    for i in range(n):
        slots = [None] * NS
        q = 0
        it = 0
        while True:
            for r in range(NS):
                if slots[r] is None or not (slots[r] > 0).any():
                    if slots[r] is not None:
                        ev[i] += 1
                        slots[r] = None
                    if q < nch:
                        slots[r] = ch[i, q].copy()
                        q += 1
            live = [s for s in slots if s is not None and (s > 0).any()]
            if not live and q >= nch and all(s is None for s in slots):
                break
            if not live:
                continue
            # advance to the next slot end
            k = min(int(s[s > 0].max()) for s in live)
            for s in live:
                s -= np.minimum(s, k)
            it += k
        tot[i] = it
    return tot, ev


def sim_lane(L, NS=2, T=32, order="desc", pair=False):
    """All cars at once, one wave-iteration per loop pass."""
    n, B = L.shape
    nch = -(-B // 64)
    need = (L - 1).astype(np.int64)
    if order == "desc":
        seq = np.concatenate([np.arange(k * 64, min(B, k * 64 + 64)) for k in range(nch - 1, -1, -1)])
    else:
        seq = np.arange(B)
    if pair:  # a unit = beams (b, b + 64) of a 128-beam block, traced one after the other in one slot
        units = []
        for blk in range((B + 127) // 128 - 1, -1, -1):
            for l in range(64):
                b = blk * 128 + l
                if b < B:
                    units.append((b, b + 64 if b + 64 < B else -1))
        U = len(units)
        first = np.array([u[0] for u in units])
        second = np.array([u[1] for u in units])
        q_first = need[:, first]
        q_second = np.where(second[None] >= 0, need[:, np.maximum(second, 0)], -1)
    else:
        U = B
        q_first = need[:, seq]
        q_second = np.full((n, U), -1, np.int64)
    rem = np.full((n, 64, NS), -1, np.int64)   # -1 empty, 0 ended, >0 tracing
    sec = np.full((n, 64, NS), -1, np.int64)    # the slot's pending second ray (pair units)
    nxt = np.zeros(n, np.int64)
    iters = np.zeros(n, np.int64)
    events = np.zeros(n, np.int64)
    served = np.zeros(n, np.int64)
    lane_iters = np.zeros(n, np.int64)
    ar = np.arange(n)
    while True:
        # first arm of every slot (rem starts empty)
        start = (rem == -1).reshape(n, -1).all(1) & (nxt == 0)
        for c in np.flatnonzero(start):
            k = min(64 * NS, U)
            flat = rem[c].reshape(-1)
            flat[:k] = q_first[c, :k]
            sec[c].reshape(-1)[:k] = q_second[c, :k]
            nxt[c] = k
            rem[c] = flat.reshape(64, NS)
        ended = rem == 0
        n_end = ended.reshape(n, -1).sum(1)
        tracing = (rem > 0).reshape(n, -1).any(1)
        more = (nxt < U) | (sec >= 0).reshape(n, -1).any(1)
        ev = (n_end > 0) & ((n_end >= T) | ~tracing)
        if not ev.any() and not tracing.any():
            break
        if ev.any():
            events += ev
            served += np.where(ev, n_end, 0)
            for c in np.flatnonzero(ev):
                e_idx = np.flatnonzero(ended[c].reshape(-1))
                # slots holding a pair's second ray continue with it
                s2 = sec[c].reshape(-1)[e_idx]
                has2 = s2 >= 0
                flat = rem[c].reshape(-1)
                flat[e_idx[has2]] = s2[has2]
                sec[c].reshape(-1)[e_idx[has2]] = -1
                free = e_idx[~has2]
                k = min(free.size, U - nxt[c])
                if k > 0:
                    flat[free[:k]] = q_first[c, nxt[c]:nxt[c] + k]
                    sec[c].reshape(-1)[free[:k]] = q_second[c, nxt[c]:nxt[c] + k]
                    nxt[c] += k
                flat[free[k:]] = -1
                rem[c] = flat.reshape(64, NS)
        act = rem > 0
        car_act = act.reshape(n, -1).any(1)
        if not car_act.any():
            if not ((rem == 0).any() or (nxt < U).any()):
                break
            continue
        iters += car_act
        lane_iters += act.reshape(n, -1).sum(1)
        rem[act] -= 1
    return iters, events, served, lane_iters


def sim_queue(Q, NS=2, T=32):
    """Lane refill over per-wave queues Q [n_waves, U] of ray iteration counts
    (-1 = padding at the end).  Returns per-wave (iters, events, lane_iters)."""
    n, U = Q.shape
    qlen = (Q >= 0).sum(1)
    rem = np.full((n, 64 * NS), -1, np.int64)
    k0 = np.minimum(64 * NS, qlen)
    for c in range(n):
        rem[c, :k0[c]] = Q[c, :k0[c]]
    nxt = k0.copy()
    iters = np.zeros(n, np.int64)
    events = np.zeros(n, np.int64)
    lane_iters = np.zeros(n, np.int64)
    while True:
        ended = rem == 0
        n_end = ended.sum(1)
        tracing = (rem > 0).any(1)
        ev = (n_end > 0) & ((n_end >= T) | ~tracing)
        if not ev.any() and not tracing.any():
            break
        for c in np.flatnonzero(ev):
            free = np.flatnonzero(ended[c])
            events[c] += len(np.unique(free // 64))  # slot arrays (r = j // 64) the pass touches
            k = min(free.size, qlen[c] - nxt[c])
            if k > 0:
                rem[c, free[:k]] = Q[c, nxt[c]:nxt[c] + k]
                nxt[c] += k
            rem[c, free[k:]] = -1
        act = rem > 0
        wa = act.any(1)
        iters += wa
        lane_iters += act.sum(1)
        rem[act] -= 1
    return iters, events, lane_iters


def pooled_queues(need, C, order, pred=None):
    """Queues of C consecutive cars per wave.  order: 'chunk' (descending chunk
    index, the C cars' chunk k together), 'lpt' (rays sorted by their own
    cost: an oracle bound), 'pred' (64-beam chunks sorted by the predicted
    per-chunk max from `pred`, the previous step's counts)."""
    n, B = need.shape
    nch = -(-B // 64)
    W = n // C
    out = []
    for w in range(W):
        cars = need[w * C:(w + 1) * C]
        if order == "lpt":
            q = np.sort(cars.ravel())[::-1]
        else:
            pad = np.full((C, nch * 64), -1, np.int64)
            pad[:, :B] = cars
            ch = pad.reshape(C, nch, 64)
            if order == "chunk":
                q = ch[:, ::-1].transpose(1, 0, 2).reshape(-1)
            else:
                pp = np.zeros((C, nch * 64), np.int64)
                pp[:, :B] = pred[w * C:(w + 1) * C]
                cost = pp.reshape(C, nch, 64).max(2).ravel()
                o = np.argsort(-cost, kind="stable")
                q = ch.reshape(C * nch, 64)[o].reshape(-1)
            q = q[q >= 0] if False else q
        out.append(q)
    Q = np.stack(out)
    # move padding (-1) to the end, keep order
    res = np.full_like(Q, -1)
    for i in range(Q.shape[0]):
        v = Q[i][Q[i] >= 0]
        res[i, :v.size] = v
    return res


def consecutive_counts(n_envs=1024, steps=60, seed=1):
    """Pairs of consecutive steps' counts (t-1, t) of a random-action rollout."""
    tm = load_map("Spielberg_map")
    sp = centerline_spawns("Spielberg", 1)[:, 0]
    sc = O.OracleScanner(tm.free_mask, tm.resolution, tm.origin)
    sim = O.OracleSim(sc, n_envs, 1)
    rng = np.random.default_rng(seed)
    sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
    prev = None
    pairs = []
    for t in range(1, steps + 1):
        a = np.stack([rng.uniform(-0.4189, 0.4189, n_envs), rng.uniform(0, 20, n_envs)], 1)
        _, col = sim.step(a[:, None, :], threads=8)
        if t >= steps - 1:
            p = np.stack([sim.state[:, 0], sim.state[:, 1], sim.state[:, 4]], 1)
            _, L, _ = sc.scan(p, with_probe=True, threads=8)
            if prev is not None:
                pairs.append((prev, L.astype(np.int64)))
            prev = L.astype(np.int64)
        hit = np.flatnonzero(col[:, 0] > 0)
        if hit.size:
            st = sim.state.copy()
            sim.reset(sp[rng.integers(0, sp.shape[0], n_envs)])
            keep = np.ones(n_envs, bool)
            keep[hit] = False
            sim.state[keep] = st[keep]
    return pairs[-1]


def main_pool():
    prev, cur = consecutive_counts(int(os.environ.get("LR_ENVS", 1024)))
    need, pneed = cur - 1, prev - 1
    n = need.shape[0]
    w = need.sum()
    for C in (1, 2, 3, 4):
        for NS in (2,):
            for order in ("chunk", "pred"):
                for T in (32, 48, 64, 80, 96, 112):
                    Q = pooled_queues(need, C, order, pneed)
                    it, ev, li = sim_queue(Q, NS, T)
                    print(json.dumps({"C": C, "NS": NS, "order": order, "T": T,
                                      "iters_per_car": float(it.sum() / n), "events_per_car": float(ev.sum() / n),
                                      "cost_per_car(40/it,70/ev)": float((40 * it.sum() + 70 * ev.sum()) / n),
                                      "served_per_event": float(1080 * n / max(ev.sum(), 1)),
                                      "simt": float(w / (it.sum() * 64 * NS)),
                                      "wave_iters_p50_p90_max": [float(np.percentile(it, 50)), float(np.percentile(it, 90)), int(it.max())]}),
                          flush=True)


def main():
    N = int(os.environ.get("LR_ENVS", 1024))
    L = rollout_counts(n_envs=N)
    n, B = L.shape
    work = (L - 1).sum(1)
    res = {"cars": int(n), "mean_lookups": float(L.mean()),
           "max_ray_iters_per_car_mean": float((L - 1).max(1).mean()),
           "max_ray_iters_per_car_p90": float(np.percentile((L - 1).max(1), 90)),
           "ray_iters_per_car": float(work.mean())}
    print(json.dumps(res), flush=True)
    sub = L[: min(n, 2048)]
    w = (sub - 1).sum(1)
    it, ev = sim_chunk(sub, 2)
    print(json.dumps({"schedule": "chunk", "NS": 2, "iters": float(it.mean()), "events": float(ev.mean()),
                      "simt": float(w.sum() / (it.sum() * 128))}), flush=True)
    for NS in (2, 3, 4):
        for T in (16, 32, 48, 64, 96):
            if T > 64 * NS:
                continue
            for pair in (False, True):
                it, ev, sv, li = sim_lane(sub, NS, T, pair=pair)
                print(json.dumps({"schedule": "lane", "NS": NS, "T": T, "pair_units": pair,
                                  "iters": float(it.mean()), "events": float(ev.mean()),
                                  "served_per_event": float(sv.sum() / max(ev.sum(), 1)),
                                  "simt": float(li.sum() / (it.sum() * 64 * NS))}), flush=True)


if __name__ == "__main__":
    if os.environ.get("LR_POOL"):
        main_pool()
    else:
        main()
