"""Host-only model of the ray kernel's gathers: rays of 96 spawn poses traced on
the Spielberg EDT (the reference's march: x += d cos, y += d sin until d == 0 or the range is
exceeded), each 64-beam chunk's trip as one gather; distinct 128-B lines per gather and the
per-quad line count (the 8-byte gather's address cost) for the row-major padded table and tiled
layouts.

    python scripts/gather_lines_model.py
"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from f110_gymnasium_ros2_jazzy_amd.maps import load_map, centerline_spawns
t = load_map('Spielberg_map'); k = t.ensure_edt(); dt = t.resolution * np.sqrt(k.astype(np.float64))
H, W = dt.shape; res = t.resolution; ox, oy = t.origin[0], t.origin[1]
print('map', H, W, 'max k', int(k.max()), 'frac k<65536', float((k < 65536).mean()))
sp = centerline_spawns('Spielberg', 1)
rng = np.random.default_rng(0)
cars = sp[rng.integers(0, sp.shape[0], 96)]
B = 1080; fov = 4.7; mr = 30.0
ang = -fov / 2 + np.arange(B) * (fov / (B - 1))
P = 200; Wp = ((W + 2 * P + 1 + 511) // 512) * 512 - 1
layouts = {}
def rowmajor(r, c, lb):  # line index for byte line size lb
    return ((r + P) * Wp + (c + P)) * 8 // lb
def tiled(tw, th):
    def f(r, c, lb):
        rr, cc = r + P, c + P
        tiles_x = (Wp + tw - 1) // tw
        tile = (rr // th) * tiles_x + cc // tw
        within = (rr % th) * tw + cc % tw
        return (tile * tw * th + within) * 8 // lb
    return f
lays = {'rowmajor': rowmajor, 'tile4x4': tiled(4, 4), 'tile8x2': tiled(8, 2), 'tile2x8': tiled(2, 8), 'tile8x8': tiled(8, 8)}
stats = {(n, lb): [] for n in lays for lb in (64, 128)}
qstats = {n: [] for n in lays}
ZERO = 1 << 40
for (x0, y0, th0) in cars.reshape(cars.shape[0], -1)[:, :3]:
    th = th0 + ang
    c, s = np.cos(th), np.sin(th)
    x = np.full(B, x0); y = np.full(B, y0)
    def cell(x, y):
        cc = np.clip(((x - ox) / res).astype(np.int64), 0, W - 1); rr = np.clip(((y - oy) / res).astype(np.int64), 0, H - 1)
        return rr, cc
    rr, cc = cell(x, y); d = dt[rr, cc]; tot = d.copy()
    active = (d > 0) & (tot <= mr)
    for it in range(400):
        if not active.any(): break
        x = np.where(active, x + d * c, x); y = np.where(active, y + d * s, y)
        rr, cc = cell(x, y)
        for ch in range(0, B, 64):
            a = active[ch:ch + 64]
            if not a.any(): continue
            r_, c_ = rr[ch:ch + 64][a], cc[ch:ch + 64][a]
            for n, f in lays.items():
                for lb in (64, 128):
                    stats[(n, lb)].append(len(np.unique(f(r_, c_, lb))))
                ln = np.where(a, f(rr[ch:ch + 64], cc[ch:ch + 64], 128), ZERO)
                ln = np.concatenate([ln, np.full(64 - ln.size, ZERO)]).reshape(16, 4)
                qs = np.sort(ln, axis=1); qstats[n].append(int(1 * 16 + (qs[:, 1:] != qs[:, :-1]).sum()))
        d = np.where(active, dt[rr, cc], d); tot = np.where(active, tot + d, tot)
        active = active & (d > 0) & (tot <= mr)
for key, v in qstats.items():
    v = np.array(v); print('quad-model cycles', key, round(v.mean(), 2))
for key, v in stats.items():
    v = np.array(v); print(key, 'gathers', v.size, 'mean distinct lines', round(v.mean(), 2), 'p50', np.median(v), 'p90', np.percentile(v, 90))
