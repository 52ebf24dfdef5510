"""Per-kernel average durations from rocprofv3 rocpd databases (run_results.db), side by side,
plus one late dispatch sequence starting at a named kernel: the A/B summaries that
scripts/gpu_rpab.sh's traces are read with.

    python scripts/rocpd_kernels.py DIR_A DIR_B ... [--seq k_keys] [--min-calls 100]
"""
import argparse
import glob
import json
import os
import sqlite3
import sys


def load(d):
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    return [(n.split("(")[0].replace("f110::", "").replace("(anonymous namespace)::", ""), s, e) for n, s, e in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--seq", default="k_keys")
    ap.add_argument("--min-calls", type=int, default=100)
    a = ap.parse_args()
    runs = {os.path.basename(d.rstrip("/")): load(d) for d in a.dirs}
    stats = {}
    for k, rows in runs.items():
        acc = {}
        for n, s, e in rows:
            c, t = acc.get(n, (0, 0.0))
            acc[n] = (c + 1, t + (e - s) / 1000.0)
        stats[k] = {n: (c, t / c) for n, (c, t) in acc.items()}
    first = next(iter(stats))
    names = sorted(stats[first], key=lambda n: -stats[first][n][0] * stats[first][n][1])
    out = {"avg_us": {}, "seq": {}}
    for n in names:
        if stats[first][n][0] < a.min_calls:
            continue
        out["avg_us"][n] = {k: round(stats[k].get(n, (0, 0.0))[1], 2) for k in stats}
    for k, rows in runs.items():
        idx = [i for i, r in enumerate(rows) if r[0].endswith(a.seq)]
        if len(idx) < 5:
            continue
        i0 = idx[-5]
        t0 = rows[i0][1]
        out["seq"][k] = [[n, round((s - t0) / 1000, 2), round((e - s) / 1000, 2)] for n, s, e in rows[i0:i0 + 10]]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
