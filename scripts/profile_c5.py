"""Config-5 (end-to-end DDPG) evidence on the GPU box: the bench line at C5's
per-GPU share (4096 two-agent envs, batch 4096) and a rocprofv3 kernel trace of
the same command, summarised per step by stage: env step, opponent, reward,
replay, learner GEMMs (hipBLASLt), learner heads / ReLU backward (libf110),
Adam, other torch kernels.  The parent never touches the GPU.

    python scripts/profile_c5.py r02      # -> gpurun_out/prof_c5_r02/{bench.json, summary.json, kernel_stats.csv}
"""
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
OUT = os.path.join(REPO, "gpurun_out", f"prof_c5_{tag}")
os.makedirs(OUT, exist_ok=True)
env = dict(os.environ, TMPDIR="/tmp")
STEPS, WARM = 200, 20
BENCH = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", "ddpg", "--steps", str(STEPS),
         "--warmup", str(WARM)]

SUMMARIZE_ONLY = "--summarize" in sys.argv  # re-summarise a merged kernel_stats.csv (no GPU)
d = os.path.join(OUT, "trace")
if not SUMMARIZE_ONLY:
    with open(os.path.join(OUT, "bench.json"), "w") as f:
        subprocess.run(["timeout", "-k", "10", "300"] + BENCH, cwd=REPO, env=env, stdout=f, check=True)
    with open(os.path.join(OUT, "trace.log"), "w") as log:
        subprocess.run(["timeout", "-k", "10", "400", "rocprofv3", "--kernel-trace", "--stats", "--output-format",
                        "csv", "-d", d, "-o", "run", "--"] + BENCH, cwd="/tmp", env=env, stdout=log,
                       stderr=subprocess.STDOUT, check=True)
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
else:
    stats = os.path.join(OUT, "kernel_stats.csv")


REPLAY = ("k_add_copy", "k_add_scan", "k_count", "k_finish", "k_gather", "k_hist", "k_keys", "k_place",
          "k_prio_max", "k_sample_replace", "k_select", "k_update")
HEADS = ("k_colsum_finish", "k_head_bwd_rows", "k_head_fwd", "k_head_wgrad", "k_loss_finish",
         "k_relu_bwd", "k_wgrad_finish")


def stage(name):
    n = name
    if "f110::" in n:
        k = n.split("(f110::")[0].split("(float")[0].split("(int")[0].split("<")[0].split("::")[-1]
        if k.startswith("k_rays") or k in ("k_agents", "k_post_multi", "k_post_single"):
            return "env_step"
        if k.startswith("k_gap_follow"):
            return "opponent_gap_follow"
        if k == "k_reward":
            return "reward"
        if k in REPLAY:
            return "replay"
        if k == "k_adam":
            return "learner_adam"
        if k in HEADS:
            return "learner_heads"
        if k in ("k_lgemm", "k_lwgrad", "k_lwgrad_finish"):  # csrc/f110_gemm.hip
            return "learner_gemm"
    if n.startswith("Cijk") or "gemm" in n.lower() or "hipblaslt" in n.lower():
        return "learner_gemm"
    return "other_torch"


rows, total = [], 0.0
with open(stats) as f:
    for r in csv.DictReader(f):
        t = float(r["TotalDurationNs"])
        rows.append({"name": r["Name"][:120], "calls": int(r["Calls"]), "total_ms": t / 1e6,
                     "avg_us": float(r["AverageNs"]) / 1e3, "stage": stage(r["Name"])})
        total += t
# the traced command runs WARM + STEPS timed steps plus the phase-split pass (min(STEPS, 100) more)
steps = WARM + STEPS + min(STEPS, 100)
by_stage = {}
for r in rows:
    by_stage[r["stage"]] = by_stage.get(r["stage"], 0.0) + r["total_ms"]
summary = {
    "command": " ".join(os.path.basename(a) if a.endswith(".py") else a for a in BENCH[1:]),
    "steps_traced": steps,
    "kernel_ms_per_step_by_stage": {k: v / steps for k, v in sorted(by_stage.items(), key=lambda kv: -kv[1])},
    "kernel_ms_per_step_total": total / 1e6 / steps,
    "top_kernels": sorted(rows, key=lambda r: -r["total_ms"])[:25],
    "note": "per-step = total kernel time / traced steps (warm-up + timed + phase-split pass); learner GEMMs "
            "are libf110's k_lgemm / k_lwgrad (hipBLASLt Cijk* on the autograd path), heads / Adam are libf110 "
            "kernels",
}
import shutil  # noqa: E402
if not SUMMARIZE_ONLY:
    shutil.copy(stats, os.path.join(OUT, "kernel_stats.csv"))
json.dump(summary, open(os.path.join(OUT, "summary.json"), "w"), indent=1)
print(json.dumps(summary["kernel_ms_per_step_by_stage"]))
