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


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args(mod, argv):
    import argparse
    ns = argparse.Namespace(gpus=None, rehearse_gloo=False, dry_run_launch=False)
    for i, a in enumerate(argv):
        if a == "--gpus":
            ns.gpus = int(argv[i + 1])
        elif a == "--rehearse-gloo":
            ns.rehearse_gloo = True
    return ns


def _node(root, idx, gfx):
    d = root / str(idx)
    d.mkdir()
    (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\ngfx_target_version {gfx}\nmax_waves 8\n")


def test_visible_gpus_counts_kfd_gpu_nodes(tmp_path, monkeypatch):
    mod = _bench_module()
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert mod.visible_gpus(str(tmp_path)) is None  # no topology: unknown, not zero
    _node(tmp_path, 0, 0)  # the CPU agent
    for i in range(1, 9):
        _node(tmp_path, i, 90500)  # gfx950
    assert mod.visible_gpus(str(tmp_path)) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert mod.visible_gpus(str(tmp_path)) == 2


def test_launcher_makes_no_hip_call(monkeypatch):
    """the parent counts GPUs without torch.cuda (whose device_count can fall back to
    hipGetDeviceCount) and starts the ranks as children."""
    import subprocess as sp
    import torch
    mod = _bench_module()

    def boom(*a, **k):
        raise AssertionError("the launcher touched torch.cuda")
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    monkeypatch.setattr(mod, "visible_gpus", lambda *a, **k: 8)
    calls = []
    monkeypatch.setattr(sp, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    argv = ["--gpus", "8", "--steps", "3"]
    assert mod.launch_ranks(_args(mod, argv), argv) == 0
    (cmd, env), = calls
    assert "--nproc-per-node=8" in cmd and env["MASTER_ADDR"] == "127.0.0.1"


def test_more_gpus_than_the_node_has_fails_loudly(monkeypatch, capsys):
    import subprocess as sp
    mod = _bench_module()
    monkeypatch.setattr(mod, "visible_gpus", lambda *a, **k: 1)
    monkeypatch.setattr(sp, "call", lambda *a, **k: (_ for _ in ()).throw(AssertionError("ranks started")))
    argv = ["--gpus", "2", "--steps", "1"]
    assert mod.launch_ranks(_args(mod, argv), argv) == 2
    assert "needs 2 visible GPUs" in capsys.readouterr().err


def test_combine_with_gloo_rehearsal_is_rejected():
    r = run(["--gpus", "2", "--combine", "--rehearse-gloo", "--dry-run-launch"])
    assert r.returncode != 0
    assert "--combine with --rehearse-gloo" in r.stderr


def test_launcher_world_size_mismatch_fails():
    r = run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
