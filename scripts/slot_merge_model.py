"""Offline model: k_rays_fxs's two pipelined chunk slots, with and without
slot merging (CPU, oracle lookup counts; the oracle is test infrastructure and
only supplies per-ray lookup counts here).

Per car (one wave, two 64-lane slots, chunks armed in descending order):

  fxs    today: each slot is re-armed with the car's next chunk when all of
         its rays have ended; both slots gather every trip (a closed slot on
         the zero cell) until both are closed.
  merge  as fxs, and when both slots hold active rays whose count fits one
         wave (cnt0 + cnt1 <= 64), the ended rays of both slots are finished,
         slot 1's active rays move into slot 0's free lanes, and slot 1 is
         re-armed with the next chunk (or closed: a closed slot skips its
         gather).  `min_gain` skips merges that would save fewer lanes.

Counted per car: trips, slot gathers (wave-level loads of the trace), finish
passes (full = a whole chunk, partial = the ended lanes of a slot at a merge),
arms, merges.

    python scripts/slot_merge_model.py -> JSON lines
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))
import numpy as np  # noqa: E402

from lane_refill_model import rollout_counts  # noqa: E402


def chunks_desc(need, B):
    nch = -(-B // 64)
    pad = np.full(nch * 64, -1, np.int64)  # -1: no beam in this lane
    pad[:B] = need
    return [pad[k * 64:(k + 1) * 64].copy() for k in range(nch - 1, -1, -1)]


def sim_car(need, B, merge, closed_skip=None, cap=64):
    """One car.  rem per slot lane: >0 tracing, 0 ended (not finished), -1 empty."""
    ch = chunks_desc(need, B)
    q = 0
    slots = [None, None]
    for r in range(2):
        if q < len(ch):
            slots[r] = ch[q].copy()
            q += 1
    c = dict(trips=0, gathers=0, full=0, partial=0, arms=2, merges=0, lane_lookups=int(need.sum()))
    skip = merge if closed_skip is None else closed_skip
    while True:
        for r in range(2):
            s = slots[r]
            if s is not None and not (s > 0).any():
                c["full"] += 1  # finish the chunk's (or the merged slot's) rays
                if q < len(ch):
                    slots[r] = ch[q].copy()
                    q += 1
                    c["arms"] += 1
                else:
                    slots[r] = None
        if merge and slots[0] is not None and slots[1] is not None:
            a0, a1 = int((slots[0] > 0).sum()), int((slots[1] > 0).sum())
            if a0 and a1 and a0 + a1 <= cap:
                c["merges"] += 1
                c["partial"] += int((slots[0] == 0).any()) + int((slots[1] == 0).any())
                moved = slots[1][slots[1] > 0]
                s0 = slots[0].copy()
                s0[s0 == 0] = -1  # finished
                free = np.flatnonzero(s0 <= 0)
                s0[free[:moved.size]] = moved
                slots[0] = s0
                if q < len(ch):
                    slots[1] = ch[q].copy()
                    q += 1
                    c["arms"] += 1
                else:
                    slots[1] = None
        openn = sum(s is not None for s in slots)
        if openn == 0:
            break
        c["trips"] += 1
        c["gathers"] += openn if skip else 2
        for s in slots:
            if s is not None:
                s[s > 0] -= 1
    return c


def run(L, merge, **kw):
    n, B = L.shape
    acc = {}
    for i in range(n):
        c = sim_car((L[i] - 1).astype(np.int64), B, merge, **kw)
        for k, v in c.items():
            acc[k] = acc.get(k, 0) + v
    out = {k: v / n for k, v in acc.items()}
    out["simt_issued"] = acc["lane_lookups"] / (acc["gathers"] * 64)
    return out


def main():
    N = int(os.environ.get("SM_ENVS", 512))
    L = rollout_counts(n_envs=N, steps=40, every=20)
    print(json.dumps({"cars": int(L.shape[0]), "mean_lookups": float(L.mean())}), flush=True)
    for name, kw in (("fxs", dict(merge=False)), ("fxs_closed_skip", dict(merge=False, closed_skip=True)),
                     ("merge", dict(merge=True)), ("merge_cap48", dict(merge=True, cap=48))):
        print(json.dumps({"schedule": name, **{k: round(v, 3) for k, v in run(L, **kw).items()}}), flush=True)


if __name__ == "__main__":
    main()
