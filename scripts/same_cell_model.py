"""Host-only model: how often does a ray's next EDT lookup land in the cell it just read?  (A wave
whose active lanes all stay in their previous cell could skip that trip's gather: the value is
the one it already holds.)  Rays of 96 spawn poses traced on the Spielberg EDT as in
gather_lines_model.py; per 64-beam chunk and trip, whether every active lane's cell is unchanged;
per ray, its same-cell steps; and the same for the longest 1 % of rays (the launch's critical
chains).

    python scripts/same_cell_model.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from f110_gymnasium_ros2_jazzy_amd.maps import centerline_spawns, load_map  # noqa: E402

t = load_map("Spielberg_map")
k = t.ensure_edt()
dt = t.resolution * np.sqrt(k.astype(np.float64))
H, W = dt.shape
res = t.resolution
ox, oy = t.origin[0], t.origin[1]
sp = centerline_spawns("Spielberg", 1)
rng = np.random.default_rng(0)
cars = sp[rng.integers(0, sp.shape[0], int(os.environ.get("SC_CARS", 96)))]
B, fov, mr = 1080, 4.7, 30.0
ang = -fov / 2 + np.arange(B) * (fov / (B - 1))
trips = skip_trips = 0
steps_all = same_all = 0
per_ray = []  # (steps, same-cell steps)
chunk_trips = []  # (trips, skippable trips) per chunk
for (x0, y0, th0) in cars.reshape(cars.shape[0], -1)[:, :3]:
    th = th0 + ang
    c, s = np.cos(th), np.sin(th)
    x = np.full(B, x0)
    y = np.full(B, y0)

    def cell(x, y):
        cc = np.clip(np.floor((x - ox) / res).astype(np.int64), 0, W - 1)
        rr = np.clip(np.floor((y - oy) / res).astype(np.int64), 0, H - 1)
        return rr, cc

    rr, cc = cell(x, y)
    d = dt[rr, cc]
    tot = d.copy()
    active = (d > 0) & (tot <= mr)
    nsteps = np.zeros(B, np.int64)
    nsame = np.zeros(B, np.int64)
    ct = np.zeros((B + 63) // 64, np.int64)
    cs = np.zeros_like(ct)
    for it in range(2000):
        if not active.any():
            break
        x = np.where(active, x + d * c, x)
        y = np.where(active, y + d * s, y)
        r2, c2 = cell(x, y)
        same = (r2 == rr) & (c2 == cc)
        nsteps += active
        nsame += active & same
        for ch in range(0, B, 64):
            a = active[ch:ch + 64]
            if not a.any():
                continue
            ct[ch // 64] += 1
            if np.all(same[ch:ch + 64][a]):
                cs[ch // 64] += 1
        rr, cc = r2, c2
        d = np.where(active, dt[rr, cc], d)
        tot = np.where(active, tot + d, tot)
        active = active & (d > 0) & (tot <= mr)
    per_ray.append(np.stack([nsteps, nsame], 1))
    chunk_trips.append(np.stack([ct, cs], 1))
pr = np.concatenate(per_ray)
ch = np.concatenate(chunk_trips)
long_cut = np.quantile(pr[:, 0], 0.99)
lg = pr[pr[:, 0] >= long_cut]
top = pr[np.argsort(pr[:, 0])[-20:]]
out = {"cars": int(cars.shape[0]), "rays": int(pr.shape[0]),
       "mean_steps": float(pr[:, 0].mean()), "same_cell_step_frac": float(pr[:, 1].sum() / pr[:, 0].sum()),
       "chunk_trips": int(ch[:, 0].sum()), "skippable_trip_frac": float(ch[:, 1].sum() / ch[:, 0].sum()),
       "longest_1pct": {"min_steps": float(long_cut), "mean_steps": float(lg[:, 0].mean()),
                        "same_cell_step_frac": float(lg[:, 1].sum() / lg[:, 0].sum())},
       "longest_20_rays": [[int(a), int(b)] for a, b in top],
       "longest_chunks_trips_skippable": [[int(a), int(b)] for a, b in ch[np.argsort(ch[:, 0])[-10:]]]}
print(json.dumps(out))
