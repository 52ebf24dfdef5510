"""CPU restatement of the training reward — TEST INFRASTRUCTURE ONLY.

Only tests/ use this module, as the checker of libf110's f110_reward; the
product path never imports it.  It restates
  rl_training/utils/track_progress.py:CenterlineProgress (:5-110) and
  rl_training/utils/rewards.py:CenterlineSafetyProgressReward (:185-355),
  parse_flat_obs (:11-41), _Prog (:86-183), _ProgFallback (:72-84)
with NumPy/Python floats in the reference's evaluation order; the kd-tree
query (scipy cKDTree, k=5) is replaced by an exact selection of the 5
midpoints of smallest squared distance (ties: lower index).  Pinned against
tests/golden/reward.npz (rewards produced by the reference classes).
"""
from __future__ import annotations

import math

import numpy as np


class TrackOracle:
    """CenterlineProgress's derived arrays and project_xy (track_progress.py:29-97)."""

    def __init__(self, xy, w_right=None, w_left=None, closed=True):
        self.xy = np.asarray(xy, dtype=float)
        self.n = len(self.xy)
        seg = np.diff(self.xy, axis=0)
        seg_len = np.linalg.norm(seg, axis=1)
        self.s = np.concatenate([[0.0], np.cumsum(seg_len)])
        self.L = self.s[-1]
        self.closed = bool(closed)
        self.tan = seg / np.maximum(seg_len[:, None], 1e-12)
        self.nrm = np.stack([-self.tan[:, 1], self.tan[:, 0]], axis=1)
        self.mid = (self.xy[:-1] + self.xy[1:]) * 0.5
        self.wR = None if w_right is None else np.asarray(w_right, dtype=float)
        self.wL = None if w_left is None else np.asarray(w_left, dtype=float)

    def nearest5(self, p):
        d = self.mid - p
        d2 = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]
        order = np.lexsort((np.arange(d2.size), d2))
        return order[:min(5, d2.size)]

    def project_xy(self, x, y):
        p = np.array([x, y], dtype=float)
        best = None
        for idx in self.nearest5(p):
            a = self.xy[idx]
            ab = self.xy[idx + 1] - a
            L2 = np.dot(ab, ab)
            if L2 <= 1e-12:
                continue
            ap = p - a
            t_par = np.clip(np.dot(ap, ab) / L2, 0.0, 1.0)
            proj = a + t_par * ab
            s_proj = self.s[idx] + t_par * np.linalg.norm(ab)
            t_signed = np.dot(p - proj, self.nrm[idx])
            cand = (np.linalg.norm(p - proj), s_proj, t_signed)
            if best is None or cand[0] < best[0]:
                best = cand
        if best is None:
            j = np.argmin(np.linalg.norm(self.xy - p, axis=1))
            return float(self.s[j]), 0.0
        return float(best[1]), float(best[2])

    def delta_s(self, cur, prev):
        ds = cur - prev
        if self.closed:
            if ds > 0.5 * self.L:
                ds -= self.L
            if ds < -0.5 * self.L:
                ds += self.L
        return ds

    def seg_at(self, s):
        idx = int(np.searchsorted(self.s, s, side="right") - 1)
        return max(0, min(idx, self.n - 2))


def _wrap(a):
    return ((a + np.pi) % (2 * np.pi)) - np.pi


class RewardOracle:
    """One env's CenterlineSafetyProgressReward (progress=None: _ProgFallback)."""

    def __init__(self, track: TrackOracle | None, dt=0.01, w_prog=1.2, forward_sign=1.0, alive_bonus=0.02,
                 w_rel_lead=0.0, lead_clip=5.0, w_lat=0.35, lat_cap=4.0, default_half_width=1.5, lidar_max=1.0,
                 near_wall_dist=0.35 / 30.0, w_wall=1.0, wall_quantile=0.05, opp_safe_dist=0.7, w_opp=0.8,
                 ego_crash_penalty=50.0, opp_crash_bonus=50.0, grace_steps_wall=25, grace_steps_opp=25):
        self.T = track
        self.k = dict(w_prog=float(w_prog), forward_sign=float(forward_sign), alive_bonus=float(alive_bonus),
                      w_rel_lead=float(w_rel_lead), lead_clip=float(lead_clip), w_lat=float(w_lat),
                      lat_cap=float(lat_cap), half=float(default_half_width), lidar_max=float(lidar_max),
                      near=float(near_wall_dist), w_wall=float(w_wall), q=float(wall_quantile),
                      safe=float(opp_safe_dist), w_opp=float(w_opp), crash=float(ego_crash_penalty),
                      bonus=float(opp_crash_bonus), gw=int(grace_steps_wall), go=int(grace_steps_opp))
        self.reset()

    def reset(self):
        self.steps = 0
        self.s_prev = [None, None]
        self.p_prev = [None, None]
        self.cum = [0.0, 0.0]
        self.ema = 0.0
        self.flip = 1.0
        self.auto = []

    def _progress(self, poses):
        T = self.T
        out = []
        if T is None:  # _ProgFallback.update
            for w, (x, y) in enumerate(poses):
                if self.p_prev[w] is None:
                    self.p_prev[w] = (x, y)
                    out.append(0.0)
                    continue
                px, py = self.p_prev[w]
                dx, dy = x - px, y - py
                self.p_prev[w] = (x, y)
                out.append((dx * dx + dy * dy) ** 0.5)
            self.cum[0] += out[0]
            self.cum[1] += out[1]
            self.ema = 0.8 * self.ema + (1 - 0.8) * out[0]
            return out[0], out[1], None
        pj = [T.project_xy(x, y) for x, y in poses]
        for w in range(2):
            if self.s_prev[w] is None:
                self.s_prev[w] = pj[w][0]
        for w, (x, y) in enumerate(poses):
            ds_geom = T.delta_s(pj[w][0], self.s_prev[w])
            if self.p_prev[w] is None:
                self.p_prev[w] = (x, y)
                out.append(0.0)
                continue
            dx, dy = x - self.p_prev[w][0], y - self.p_prev[w][1]
            self.p_prev[w] = (x, y)
            tx, ty = T.tan[T.seg_at(pj[w][0])]
            ds_sign = dx * tx + dy * ty
            out.append(math.copysign(abs(ds_geom), ds_sign if abs(ds_sign) > 1e-6 else ds_geom))
        self.s_prev = [pj[0][0], pj[1][0]]
        de, do = out
        if len(self.auto) < 20:
            self.auto.append(de)
            if len(self.auto) == 20 and sum(self.auto) / max(1, len(self.auto)) < 0.0:
                self.flip = -1.0
        de *= self.flip
        do *= self.flip
        self.cum[0] += de
        self.cum[1] += do
        self.ema = 0.8 * self.ema + (1.0 - 0.8) * abs(de)
        return de, do, pj[0]

    def __call__(self, obs):
        k = self.k
        o = np.asarray(obs, dtype=np.float32)
        B = o.shape[0] - 8
        lidar = o[:B]
        ego = [float(o[B]), float(o[B + 1]), _wrap(float(o[B + 2]))]
        ego_col = bool(o[B + 3])
        opp = [float(o[B + 4]), float(o[B + 5]), _wrap(float(o[B + 6]))]
        opp_col = bool(o[B + 7])
        self.steps += 1
        if ego_col:
            return -k["crash"]
        if opp_col and k["bonus"] > 0.0:
            return +k["bonus"]
        de, _, pe = self._progress([(ego[0], ego[1]), (opp[0], opp[1])])
        if self.steps < 10:
            de = max(0.0, de)
        r_prog = k["w_prog"] * k["forward_sign"] * de
        r_lead = 0.0
        if k["w_rel_lead"] != 0.0 and self.T is not None:
            lead = np.clip(self.cum[0] - self.cum[1], -k["lead_clip"], k["lead_clip"])
            r_lead = k["w_rel_lead"] * (lead / k["lead_clip"])
        r_lat = 0.0
        if self.T is not None:
            s_ego, t_ego = pe
            if self.T.wR is None:
                wR = wL = k["half"]
            else:
                i = self.T.seg_at(s_ego)
                wR, wL = float(self.T.wR[i]), float(self.T.wL[i])
            w_eff = max(0.2, float(wL if t_ego >= 0.0 else wR))
            lat = abs(t_ego) / w_eff
            r_lat = -k["w_lat"] * min(lat * lat, k["lat_cap"])
        r_wall = 0.0
        if len(lidar) and self.steps >= k["gw"]:
            r = np.where((lidar <= 0.0) | ~np.isfinite(lidar), k["lidar_max"], lidar)
            r = np.clip(r, 0.0, k["lidar_max"])
            dmin = float(np.quantile(r, k["q"]))
            if dmin < k["near"]:
                x = (k["near"] - dmin) / max(1e-6, k["near"])
                r_wall = -k["w_wall"] * (x ** 2)
        r_opp = 0.0
        if self.steps >= k["go"]:
            rho = math.hypot(ego[0] - opp[0], ego[1] - opp[1])
            if rho < k["safe"]:
                y = (k["safe"] - rho) / max(1e-6, k["safe"])
                r_opp = -k["w_opp"] * (y ** 2)
        r_flank = 0.0
        dx, dy = ego[0] - opp[0], ego[1] - opp[1]
        c, s = math.cos(-opp[2]), math.sin(-opp[2])
        x_rel, y_rel = c * dx - s * dy, s * dx + c * dy
        if 0.2 <= x_rel <= 1.8 and 0.25 <= abs(y_rel) <= 0.8:
            y_band = max(0.0, 0.8 - abs(abs(y_rel) - 0.525))
            r_flank = 0.1 * (x_rel / 1.8) * (y_band / 0.8)
        return float(r_prog + k["alive_bonus"] + r_lead + r_lat + r_wall + r_opp + r_flank)
