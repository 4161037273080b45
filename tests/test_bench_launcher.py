"""bench.py --gpus N run directly (the driver's BENCH form) must start N ranks, or fail loudly.

A direct `python bench.py --gpus N` (no WORLD_SIZE) starts `torch.distributed.run` as a child
before anything touches the GPU and forwards rank 0's JSON line; with fewer than N GPUs it exits
non-zero instead of printing a one-GPU line. CPU only: this container has no GPU, so the
refusal path runs for real.
"""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_n_builds_the_launcher_command():
    b = _bench()
    argv = ["--gpus", "2", "--steps", "3", "--warmup", "1"]
    cmd = b.launcher_cmd(argv, 2, 29533)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29533"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    script = os.path.abspath(os.path.join(ROOT, "bench.py"))
    assert cmd[-len(argv) - 1:] == [script, *argv]


def test_free_port_is_bindable():
    import socket

    b = _bench()
    p = b.free_port()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", p))


def test_gpus_2_without_two_gpus_exits_nonzero():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode != 0
    assert r.stdout.strip() == "", "no JSON line may be printed for a world the machine cannot run"
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr


def test_share_runs_are_labelled_as_configs2_shares():
    """a 1,250-replicate run is configs[2]'s per-GPU share, not configs[1]."""
    assert _bench().workload_label(False, None, 10000, 1, 10000).startswith("configs[1]:")
    assert _bench().workload_label(False, None, 1250, 1, 1250).startswith("configs[2]'s per-GPU share at 8 GPUs")
    assert _bench().workload_label(True, None, 10000, 8, 1250).startswith("configs[2]:")
    assert "not a BASELINE config" in _bench().workload_label(False, None, 3000, 1, 3000)
