"""bench.py's launcher (CPU): `--gpus N` without an outer launcher starts its
own N ranks through torch.distributed.run before anything touches the GPU,
and a WORLD_SIZE that disagrees with --gpus exits non-zero (the
driver's scaling runs must record N-rank lines or fail, never a mislabelled
1-rank line).  F110_BENCH_ECHO_RANKS=1 makes each rank report its
environment and return before importing torch."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
sys.path.insert(0, REPO)


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_command_line():
    import bench
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "20"], 4, 29611)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29611"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "20"] and cmd[-5] == os.path.abspath(BENCH)


def test_self_launch_starts_n_ranks_without_touching_the_gpu():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       env=_env(F110_BENCH_ECHO_RANKS="1"), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    for x in lines:
        assert x["world"] == 2 and x["gpus"] == 2 and x["local_rank"] == x["rank"]
        assert x["master_addr"] == "127.0.0.1"
        assert x["argv"] == ["--gpus", "2", "--steps", "3", "--warmup", "1"]


def test_parent_never_imports_torch():
    """The self-launching parent decides from argv / env alone: a probe that
    stubs subprocess.call shows it returns the children's code with torch
    never imported (no HIP initialisation in the parent)."""
    probe = (
        "import sys, subprocess; sys.argv = ['bench.py', '--gpus', '8', '--workload', 'ddpg']\n"
        "calls = []\n"
        "subprocess.call = lambda cmd, env=None: calls.append((cmd, env)) or 3\n"
        f"sys.path.insert(0, {REPO!r})\n"
        "import bench\n"
        "try:\n"
        "    bench.main()\n"
        "except SystemExit as e:\n"
        "    rc = e.code\n"
        "cmd, env = calls[0]\n"
        "assert '--nproc-per-node=8' in cmd and cmd[-4:] == ['--gpus', '8', '--workload', 'ddpg'], cmd\n"
        "assert env['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'\n"
        "print(rc, 'torch' in sys.modules)\n")
    r = subprocess.run([sys.executable, "-c", probe], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["3", "False"]


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0",
                                                                         F110_BENCH_ECHO_RANKS="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE 3" in r.stderr
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
                                                                         F110_BENCH_ECHO_RANKS="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
