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


def test_launch_ranks_refuses_fewer_gpus(monkeypatch, capsys):
    """The refusal itself, with the GPU count stubbed: exit 3, nothing on stdout, whatever the box."""
    b = _bench()
    monkeypatch.setattr(b, "probe_gpu_count", lambda: 1)
    assert b.launch_ranks(["--gpus", "2"], 2) == 3
    out = capsys.readouterr()
    assert out.out == "" and "--gpus 2 needs 2 visible GPUs" in out.err


def test_gpus_2_without_two_gpus_exits_nonzero():
    """End to end through a real child process; only meaningful where fewer than 2 GPUs exist (on a
    box with two or more, --gpus 2 would launch a real two-rank bench)."""
    import pytest

    if _bench().probe_gpu_count() >= 2:
        pytest.skip("this machine has >= 2 GPUs: the refusal path does not apply")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode != 0
    assert r.stdout.strip() == "", "no JSON line may be printed for a world the machine cannot run"
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr


def test_share_runs_are_labelled_as_configs2_shares():
    """a 1,250-replicate run is configs[2]'s per-GPU share, not configs[1]; a weak
    run on several GPUs is never labelled configs[1]."""
    b = _bench()
    assert b.workload_label("single", None, 10000, 1, 10000).startswith("configs[1]:")
    assert b.workload_label("single", None, 1250, 1, 1250).startswith("configs[2]'s per-GPU share at 8 GPUs")
    assert b.workload_label("strong", None, 10000, 8, 1250).startswith("configs[2]:")
    assert "not a BASELINE config" in b.workload_label("single", None, 3000, 1, 3000)
    for n in (2, 4, 8):
        lab = b.workload_label("weak", None, 10000 * n, n, 10000)
        assert lab.startswith("configs[1]'s panel, 10,000 replicates per GPU, weak"), lab
        assert not lab.startswith("configs[1]:")


def test_default_multi_gpu_run_is_configs2_strong():
    """the driver's `bench.py --gpus N` (N > 1, no other flags) measures configs[2] --
    10,000 replicates per step in total, sharded -- and `--gpus 1` keeps the configs[1] line."""
    b = _bench()
    args = b.parse_args(["--gpus", "8"])  # the driver's argv, with its --steps/--warmup or without
    assert (args.gpus, args.reps, args.weak, args.strong) == (8, 10000, False, False)
    assert b.replicate_plan(args.reps, 8, args.strong, args.weak) == ("strong", 10000, 1250)
    args = b.parse_args(["--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert b.replicate_plan(args.reps, 8, args.strong, args.weak) == ("strong", 10000, 1250)
    assert b.replicate_plan(10000, 1) == ("single", 10000, 10000)
    assert b.replicate_plan(1250, 1) == ("single", 1250, 1250)
    assert b.workload_label("single", None, 10000, 1, 10000).startswith("configs[1]:")
    for n, per in ((2, 5000), (4, 2500), (8, 1250)):
        mode, total, per_rank = b.replicate_plan(10000, n)
        assert (mode, total, per_rank) == ("strong", 10000, per), n
        assert b.workload_label(mode, None, total, n, per_rank).startswith("configs[2]:")
    assert b.replicate_plan(10000, 8, weak=True) == ("weak", 80000, 10000)
    assert b.replicate_plan(10000, 8, strong=True) == ("strong", 10000, 1250)


def test_one_gpu_line_is_labelled_single():
    """one GPU is neither weak nor strong scaling; the N = 1 line says "single", also
    with --weak or --strong given."""
    b = _bench()
    for kw in ({}, {"weak": True}, {"strong": True}):
        assert b.replicate_plan(10000, 1, **kw)[0] == "single", kw
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert src.count('"weak" if world > 1 else "single"') == 2  # the --mm and --heckman lines

