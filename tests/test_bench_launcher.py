"""CPU checks of bench.py's rank launcher: `python bench.py --gpus N` (the driver's command shape) must run N ranks,
one per GPU, through torch.distributed.run on 127.0.0.1 -- not one process that prints n_gpus 1 -- and must fail
loudly when the node has fewer GPUs than asked for (this container has none)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=240)


def test_dry_run_launch_plumbs_arguments_and_env():
    r = run(["--gpus", "8", "--steps", "7", "--warmup", "2", "--workload", "c3", "--dry-run-launch"])
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = d["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2", "--workload", "c3"]
    assert d["nproc"] == 8
    assert d["env"] == {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "MASTER_ADDR": "127.0.0.1"}


def test_more_gpus_than_the_node_has_fails_loudly():
    r = run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_launcher_world_size_mismatch_fails():
    r = run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
