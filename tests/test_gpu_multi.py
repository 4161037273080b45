"""Multi-GPU path and the resample counts themselves, on the MI355X.

* OBRS-3 counts (builder.rs:822-827, polars sample_n_literal): the level-1 tile counts and the
  per-row count images the Gram kernel consumes (ob_debug_counts) must equal the oracle's
  restatement bit for bit -- np.bincount of oracle.resample_indices -- not only through rows.
* The engine's RCCL path (ob_ctx_create_rank + ob_boot_run_sharded[_device], ob_boot_run_multi,
  ob_prepared_boot_sharded) at world 1 on the box's single GPU: rows and ok bitwise equal to the
  plain ob_boot_run. A communicator cannot hold two ranks on one GPU, so world > 1 runs on the
  driver's 8-GPU node (bench.py); the sharding arithmetic itself is covered on CPU with gloo.
* torch.distributed with backend nccl at world 1: gather_rows' on-device branch and
  fit_sharded (both gathers) equal the single-process run bitwise.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x0B5EED


def _panel(ob, O, na, nb, p=1, weighted=False, seed=0):
    rng = np.random.default_rng(na + nb + seed)
    xa = rng.normal(size=(na, p))
    xb = rng.normal(size=(nb, p)) + 0.1
    ya = 1.0 + xa @ np.full(p, 0.5) + rng.normal(size=na)
    yb = 0.8 + xb @ np.full(p, 0.4) + rng.normal(size=nb)
    wa = rng.uniform(0.5, 2.0, na) if weighted else None
    wb = rng.uniform(0.5, 2.0, nb) if weighted else None
    return ob.Panel(xa, ya, xb, yb, wa, wb)


@pytest.mark.parametrize("na,nb", [(65536, 256), (65537, 300), (131372, 1000), (200000, 70000), (257, 65535),
                                   (1, 5), (777, 64)])
def test_counts_bitwise_match_oracle(ob, O, na, nb):
    """Level-1 tile counts and per-row counts == the oracle's index stream, for both groups, at the
    level-1 tree's shape edges (one tile, 256 / 257 tiles, partial tails, rejection rounds)."""
    panel = _panel(ob, O, na, nb)
    try:
        for g, n in ((0, na), (1, nb)):
            first, reps = 3, 70  # two 64-replicate batches, the second partial
            l1, rc = panel.debug_counts(SEED, first, reps, g)
            for r in range(reps):
                idx = O.resample_indices(SEED, first + r, g, n)
                want = np.bincount(idx, minlength=n)
                assert want.max() < 256
                assert np.array_equal(rc[r], want.astype(np.uint8)), f"group {g} replicate {first + r}"
                assert np.array_equal(l1[r], O.level1_counts(SEED, first + r, g, n)), f"level 1, rep {first + r}"
                assert int(l1[r].sum()) == n and int(rc[r].sum(dtype=np.int64)) == n
    finally:
        panel.close()


def test_counts_bitwise_500k_group(ob, O):
    """configs[1]'s group size (500,000 rows, 1954 tiles, D = 11) over replicate ids far apart."""
    n = 500_000
    panel = _panel(ob, O, n, 4096)
    try:
        for first in (0, 9_999, 123_456, 2**31 + 17):
            l1, rc = panel.debug_counts(SEED, first, 3, 0)
            for r in range(3):
                idx = O.resample_indices(SEED, first + r, 0, n)
                assert np.array_equal(rc[r], np.bincount(idx, minlength=n).astype(np.uint8))
                assert np.array_equal(l1[r], O.level1_counts(SEED, first + r, 0, n))
    finally:
        panel.close()


@pytest.mark.parametrize("n", [40961 * 256 + 77, 24_000_001])
def test_counts_bitwise_subtree_level1(ob, O, n):
    """Groups past 40,960 tiles run level 1 as subtrees under the top levels:
    tile counts and per-row counts must still equal the oracle's single-tree stream bitwise."""
    panel = _panel(ob, O, n, 4096)
    try:
        l1, rc = panel.debug_counts(SEED, 7, 2, 0)
        for r in range(2):
            want_l1 = O.level1_counts(SEED, 7 + r, 0, n)
            assert np.array_equal(l1[r], want_l1), f"level 1, rep {7 + r}"
            idx = O.resample_indices(SEED, 7 + r, 0, n)
            assert np.array_equal(rc[r], np.bincount(idx, minlength=n).astype(np.uint8)), f"rows, rep {7 + r}"
    finally:
        panel.close()


def test_rank_context_world1_sharded_equals_boot(ob, O, N):
    """ob_ctx_create_rank(world 1) + ob_boot_run_sharded: the RCCL all-gather runs and returns
    exactly ob_boot_run's rows (one outcome and three outcomes, odd replicate counts)."""
    uid = N.unique_id()
    ctx = N.rank_context(0, 0, 1, uid)
    r_ = ctypes_int_pair(N, ctx)
    assert r_ == (0, 1)
    d = O.synthetic_panel(6000, 5, True, seed=5)
    plain = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], device=0)
    ranked = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], ctx=ctx)
    for first, n in ((0, 1), (5, 97), (1000, 640)):
        for ref in (0, 2):
            a_rows, a_ok = plain.boot(SEED, first, n, ref)
            b_rows, b_ok = ranked.boot_sharded(SEED, first, n, ref)
            assert np.array_equal(a_ok, b_ok) and np.array_equal(a_rows, b_rows)
    assert ranked.timing()["gather_ms"] > 0.0
    ya3 = np.column_stack([d["ya"], ob.rif(d["ya"], 0.1), ob.rif(d["ya"], 0.9)])
    yb3 = np.column_stack([d["yb"], ob.rif(d["yb"], 0.1), ob.rif(d["yb"], 0.9)])
    p3 = ob.Panel(d["xa"], ya3, d["xb"], yb3, d["wa"], d["wb"], device=0)
    r3 = ob.Panel(d["xa"], ya3, d["xb"], yb3, d["wa"], d["wb"], ctx=ctx)
    a_rows, a_ok = p3.boot(SEED, 7, 101, 0)
    b_rows, b_ok = r3.boot_sharded(SEED, 7, 101, 0)
    assert np.array_equal(a_ok, b_ok) and np.array_equal(a_rows, b_rows)


def ctypes_int_pair(N, ctx):
    import ctypes as C

    r, w = C.c_int(-1), C.c_int(-1)
    N.check(N.lib().ob_ctx_rank(ctx, C.byref(r), C.byref(w)))
    return r.value, w.value


def test_sharded_device_into_torch_tensors(ob, O, N):
    """ob_boot_run_sharded_device writes the gathered rows into device buffers on the caller's
    stream (the bench's timed path)."""
    import torch

    ctx = N.rank_context(0, 0, 1, N.unique_id())
    d = O.synthetic_panel(5000, 4, False, seed=9)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], ctx=ctx)
    rows = torch.empty((300, panel.row_len), dtype=torch.float64, device="cuda:0")
    ok = torch.empty(300, dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.current_stream(0).cuda_stream
    panel.boot_sharded_device(SEED, 40, 300, rows.data_ptr(), ok.data_ptr(), 1, stream=stream)
    panel.sync()
    a_rows, a_ok = panel.boot(SEED, 40, 300, 1)
    assert np.array_equal(rows.cpu().numpy(), a_rows) and np.array_equal(ok.cpu().numpy(), a_ok)


def test_boot_multi_one_device(ob, O, N):
    """ob_boot_run_multi over a one-device RCCL clique == ob_boot_run; two panels on one device
    are refused (a clique needs distinct GPUs)."""
    d = O.synthetic_panel(4000, 3, True, seed=2)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], device=0)
    rows, ok = ob.boot_multi([panel], SEED, 11, 257, 3)
    a_rows, a_ok = panel.boot(SEED, 11, 257, 3)
    assert np.array_equal(rows, a_rows) and np.array_equal(ok, a_ok)
    other = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], device=0)
    with pytest.raises(N.OaxacaError) as e:
        ob.boot_multi([panel, other], SEED, 0, 10, 0)
    assert e.value.code == N.OB_E_INVALID


@pytest.mark.parametrize("n_y", [1, 3])
def test_shard_sim_world_gt1_bitwise(ob, O, n_y):
    """ob_shard.cpp's world > 1 arithmetic (ob_shard_layout.h: short and empty tail shards, padded
    per-rank blocks, outcome-major n_y blocks sent at t * per and received at t * W * per) run on
    one GPU with the all-gather's placement simulated: every rank's delivered rows equal
    ob_boot_run bit for bit, for W in {2, 3, 8}, n % W != 0 and n < W."""
    d = O.synthetic_panel(5000, 4, True, seed=21)
    ya, yb = d["ya"], d["yb"]
    if n_y == 3:
        ya = np.column_stack([ya, ob.rif(ya, 0.1), ob.rif(ya, 0.9)])
        yb = np.column_stack([yb, ob.rif(yb, 0.1), ob.rif(yb, 0.9)])
    panel = ob.Panel(d["xa"], ya, d["xb"], yb, d["wa"], d["wb"], device=0)
    try:
        for world, first, n in ((2, 3, 37), (3, 0, 10), (8, 11, 5), (8, 0, 1001), (3, 7, 2)):
            a_rows, a_ok = panel.boot(SEED, first, n, 2)
            for me in sorted({0, world - 1, world // 2}):
                rows, ok = panel.debug_shard_sim(world, me, SEED, first, n, 2)
                assert np.array_equal(ok, a_ok) and np.array_equal(rows, a_rows), (world, n, me)
    finally:
        panel.close()


def test_shard_sim_component_gather(ob, O):
    """With the gather narrowed to the aggregation's columns (48 of 153 at K = 21 in the bench):
    those columns equal ob_boot_run for every replicate; the others hold this rank's own
    replicates and NaN for the rest; aggregation over the delivered rows is unchanged."""
    d = O.synthetic_panel(6000, 6, True, seed=22)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], device=0)
    try:
        cols = panel.component_columns()
        assert len(cols) == 6 + 2 * 7
        n, world = 203, 4
        a_rows, a_ok = panel.boot(SEED, 0, n, 0)
        panel.set_gather_columns(cols)
        per = -(-n // world)
        for me in (0, 3):
            rows, ok = panel.debug_shard_sim(world, me, SEED, 0, n, 0)
            assert np.array_equal(ok, a_ok) and np.array_equal(rows[:, cols], a_rows[:, cols])
            rest = [c for c in range(panel.row_len) if c not in cols]
            mine = np.zeros(n, bool)
            mine[me * per: min(n, (me + 1) * per)] = True
            assert np.array_equal(rows[mine][:, rest], a_rows[mine][:, rest])
            assert np.isnan(rows[~mine][:, rest]).all()
            c32 = np.asarray(cols, dtype=np.int32)
            assert np.array_equal(ob.aggregate(rows, ok, c32), ob.aggregate(a_rows, a_ok, c32))
        panel.set_gather_columns(None)
        rows, ok = panel.debug_shard_sim(world, 1, SEED, 0, n, 0)
        assert np.array_equal(rows, a_rows)
    finally:
        panel.close()


def test_boot_device_returns_before_the_work_finishes(ob, O):
    """ob_boot_run_device only enqueues (no host synchronization once the panel's chunk table and
    digit images exist): right after the call the caller's stream still has the work pending."""
    import time

    import torch

    d = O.synthetic_panel(1_000_000, 20, True)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"], device=0)
    try:
        n = 10_000
        rows = torch.empty((n, panel.row_len), dtype=torch.float64, device="cuda:0")
        ok = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        stream = torch.cuda.Stream(device=0)  # a real stream (the default stream's handle, 0, means the engine's own)
        panel.boot_device(SEED, 0, n, rows.data_ptr(), ok.data_ptr(), 0, stream=stream.cuda_stream)
        panel.sync()  # first call: builds the digit images
        t0 = time.perf_counter()
        panel.boot_device(SEED, n, n, rows.data_ptr(), ok.data_ptr(), 0, stream=stream.cuda_stream)
        t_call = time.perf_counter() - t0
        pending = not stream.query()
        panel.sync()
        t_all = time.perf_counter() - t0
        assert pending and t_call < 0.5 * t_all, (t_call, t_all)
        r_host, ok_host = panel.boot(SEED, n, 64, 0)
        assert np.array_equal(rows[:64].cpu().numpy(), r_host)
    finally:
        panel.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torch_nccl_world1_gather_and_fit_sharded(ob, tmp_path):
    """backend nccl, world 1: gather_rows takes its on-GPU branch (boot_device into torch tensors
    + all_gather_into_tensor on device) and fit_sharded with either gather equals run()."""
    script = tmp_path / "w.py"
    script.write_text(f"""
import importlib, json, os, sys
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
import numpy as np, torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
ob = importlib.import_module("oaxaca-blinder-rs_amd")
D = importlib.import_module("oaxaca-blinder-rs_amd.distributed")
from test_gpu_parity import synthetic_frame
f = synthetic_frame(4000)
def builder():
    return (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
            .categorical_predictors(["sector"]).weights("w").bootstrap_reps(333).reference_coefficients(2).seed(7))
prep = builder().prepare()
rows, ok = D.gather_rows(prep, 333)
r0, o0 = prep.boot(0, 333)
out = {{"gather_equal": bool(np.array_equal(rows, r0) and np.array_equal(ok, o0))}}
prep.close()
ref = builder().run()
for eng in (False, True):
    r = D.fit_sharded(builder(), engine=eng)
    out[f"fit_equal_{{eng}}"] = ([c.std_err for c in r.two_fold.aggregate] == [c.std_err for c in ref.two_fold.aggregate]
                               and [c.ci_lower for c in r.two_fold.detailed_explained]
                               == [c.ci_lower for c in ref.two_fold.detailed_explained])
json.dump(out, open({str(tmp_path / 'out.json')!r}, "w"))
dist.destroy_process_group()
""")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    subprocess.run([sys.executable, str(script)], check=True, env=env, timeout=300)
    got = json.load(open(tmp_path / "out.json"))
    assert got == {"gather_equal": True, "fit_equal_False": True, "fit_equal_True": True}
