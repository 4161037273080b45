#!/usr/bin/env python3
"""Bootstrap replicates/s of the Oaxaca-Blinder bootstrap driver on MI355X.

Workload = BASELINE.json configs[1]: a 1,000,000-row two-group panel (500k/500k) with 20 numeric
predictors, two-fold WLS decomposition (builder default reference coefficients GroupA), 10,000
bootstrap replicates per step. One step = one full bootstrap run with the panel already
resident in HBM: OBRS-3 resampling + Gram + solves + OB terms for every replicate (HIP), the
RCCL all-gather of the per-replicate component columns over xGMI (N > 1), and the SE/p/CI aggregation of
every reported component on rank 0 (builder.rs:841-930). On N > 1 GPUs the default is configs[2]:
the 10,000 replicates of a step are sharded over the ranks (strong scaling); --weak gives each rank
its own 10,000 replicate ids per step.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line (contract in the task brief); see DESIGN.md §5 for the roofline.
"""
from __future__ import annotations

import argparse
import contextlib
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

F64_MFMA_PEAK_TFLOPS = 78.6  # MI355X dense FP64 matrix peak (v_mfma_f64_16x16x4_f64, 2.4 GHz)
F64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (spec): 32 FLOP/clk/SIMD, the same rate as the f64 MFMA
I8_MFMA_PEAK_TOPS = 5000.0  # dense I8 MFMA: 2x the ~2.5 PF dense BF16 rate per clock (MI355X_MICROARCH.md, Matrix cores)
OZ_SLICES = 7  # ob_gram_i8.hip: balanced 8-bit digits per pair product (54-bit fixed point)
OZ_PAIRS_PER_TILE = 32
HBM_PEAK_GBPS = 8000.0


def synthetic(rows, preds, weighted, seed=20260424):
    """SURVEY.md §8d wage panel (same recipe as oracle.synthetic_panel, regenerated on-box)."""
    rng = np.random.default_rng(seed)
    na = rows // 2
    nb = rows - na
    beta_b = np.concatenate([[5.0, 0.08, 0.03, -0.04], 0.1 * np.ones(max(preds - 3, 0))])[: preds + 1]
    out = {}
    for g, ng in (("a", na), ("b", nb)):
        x = np.empty((ng, preds), order="F")
        x[:, 0] = np.clip(np.round(rng.normal(13.0, 2.5, ng)), 8, 20)
        x[:, 1] = rng.uniform(0.0, 40.0, ng)
        x[:, 2] = x[:, 1] ** 2 / 100.0
        x[:, 3:] = rng.normal(0.2 if g == "a" else 0.0, 1.0, (ng, preds - 3))
        beta = beta_b + (0.05 if g == "a" else 0.0)
        out["x" + g] = x
        out["y" + g] = beta[0] + x @ beta[1:] + rng.normal(0.0, 0.5, ng)
        out["w" + g] = rng.uniform(0.5, 2.0, ng) if weighted else None
    return out


@contextlib.contextmanager
def stdout_to_stderr():
    """RCCL prints a version banner on stdout when a communicator starts; the bench's stdout must
    carry only its one JSON line, so fd 1 points at stderr while communicators are created."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def cgroup_cpu_quota():
    """CPUs this process's cgroup may use (cpu.max / cfs quota), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            return None if q == "max" else max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else max(1, -(-q // per))
    except (OSError, ValueError):
        return None


def host_cores():
    """Threads the CPU baselines use: every core this process may run on, as the reference's Rayon
    global pool does (builder.rs:816-817) -- the affinity set, capped by the
    cgroup's CPU quota (a box may show 256 CPUs and grant 16: more threads than that only queue)."""
    cores = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    return min(cores, quota) if quota else cores


def omp_share():
    """The box's per-GPU CPU share (OMP_NUM_THREADS as the GPU box sets it), reported beside."""
    try:
        return int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    except ValueError:
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_info(threads):
    return {"cores": threads, "cpu_model": cpu_model(), "host_cpus_visible": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": cgroup_cpu_quota(), "omp_num_threads_share": omp_share()}


def cpu_baseline(d, preds, weighted, ref, target_s, threads):
    """The oracle's reference-algorithm bootstrap (gather every column, full X^T W X, Cholesky,
    solve, residuals, sigma^2, inverse -- builder.rs:816-839 + ols.rs:44-144) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    cfg = O.PassConfig(preds + 1, preds, O.REF_FROM_ENUM[ref], weighted)
    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    args = (cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"], 0x0B5EED)
    t0 = time.perf_counter()
    O.boot_ref(*args, 0, threads, threads=threads, full=True)  # one replicate per thread: calibrate
    dt = time.perf_counter() - t0
    n = min(max(threads, int(target_s / max(dt, 1e-6)) * threads), 100000)
    t0 = time.perf_counter()
    _, ok = O.boot_ref(*args, 1000, n, threads=threads, full=True)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "replicates/s", **host_info(threads), "kind": "port",
            "sample": f"{n} replicates of the same {d['ya'].size + d['yb'].size}-row x {preds}-predictor "
                      f"{'WLS' if weighted else 'OLS'} panel, oracle/ob_oracle.c orc_boot_ref (full=1), "
                      f"{threads} threads, {dt:.1f} s"}


def cpu_baseline_mm(d, sims, target_s, threads, min_fits=8):
    """The oracle's QR (HiGHS exact LP, one group's full design) timed on host cores, at least
    min_fits fits spread over a thread pool; an MM replicate is 2 x sims such fits
    (quantile_decomposition.rs:221-229), so replicates/s = fits/s / (2 sims). The reference's own
    solver (Clarabel IPM) is not runnable here."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    x = O.with_intercept(d["xa"])
    c = np.ones(len(d["ya"]), dtype=np.int64)
    taus = [0.1 + 0.8 * ((i * 0.618) % 1.0) for i in range(max(min_fits, threads))]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(lambda t: O.qr_exact(x, d["ya"], c, t), taus))
    dt = time.perf_counter() - t0
    n = len(taus)
    return {"value": n / dt / (2 * sims), "unit": "replicates/s", **host_info(threads), "kind": "port",
            "sample": f"{n} HiGHS QR fits of group A ({len(d['ya'])} rows x {x.shape[1]} columns) on {threads} "
                      f"threads, {dt:.1f} s ({dt / n * threads:.1f} s per fit per thread); "
                      f"replicates/s = fits/s / {2 * sims}"}


def bench_mm(args, world, rank, local, dist):
    """configs[4]: Machado-Mata, R bootstrap replicates per GPU per step (no point pass)."""
    import torch

    ob = importlib.import_module("oaxaca-blinder-rs_amd")
    d = synthetic(args.rows, args.preds, False)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], device=local)
    qs = [0.1, 0.25, 0.5, 0.75, 0.9]
    R, seed = args.reps, 0x0B5EED
    dev = torch.device("cuda", local)

    def step(i):
        rows, ok = panel.mm(seed, args.sims, qs, (i * world + rank) * R, R, with_point=False)
        t = panel.timing()
        if dist:
            g = torch.from_numpy(rows).to(dev)
            out = torch.empty((world * R, rows.shape[1]), dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(out, g)
            rows = out.cpu().numpy()
        return rows, ok, t

    for i in range(args.warmup):
        step(i)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    asm_ms, fit_rows, iters, last = 0.0, 0.0, 0, None
    for i in range(args.steps):
        ts = time.perf_counter()
        rows, ok, t = step(args.warmup + i)
        print(f"mm step {i}: {time.perf_counter() - ts:.3f} s, assemble {t['mm_assemble_ms']:.1f} ms, "
              f"{t['mm_iterations']} iterations", file=sys.stderr, flush=True)
        asm_ms += t["mm_assemble_ms"]
        fit_rows += t["mm_fit_rows"]
        iters = max(iters, t["mm_iterations"])
        last = (rows, ok)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt[0])
    if rank != 0:
        return
    k = args.preds + 1
    bytes_row = 48.0  # mm_assemble per live (fit, row): x, z, w read, x, z, w written (direction replayed)
    pmc = load_mm_pmc(args.rows, args.preds, args.sims, R)
    flops_row = 2.0 * (k * (k + 1) / 2 + 4 * k)  # X'QX pairs, X'Q r, x.bprev, x.dba, x.db
    gbps = fit_rows * bytes_row / (asm_ms * 1e-3) / 1e9
    value = world * R * args.steps / elapsed
    out = {
        "metric": "Machado-Mata bootstrap replicates/sec (configs[4]: 1000 QR draws per group per replicate)",
        "value": value, "unit": "replicates/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak" if world > 1 else "single", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (SURVEY.md §8d wage panel, numpy seed 20260424; OBRS-3/MM-1 seed 0x0B5EED)",
        "config": {"workload": "configs[4]: Machado-Mata, 1000 simulations, quantiles 0.1/0.25/0.5/0.75/0.9",
                   "rows": args.rows, "predictors": args.preds, "simulations": args.sims,
                   "replicates_per_gpu_per_step": R, "parallelism": f"replicates sharded x{world}, RCCL all-gather"},
        "roofline": {"bound": "hbm", "achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": gbps / HBM_PEAK_GBPS,
                     "traffic": pmc["bytes_per_live_fit_row"] * fit_rows / args.steps if pmc else None,
                     "traffic_unit": "HBM bytes per step over the step's mm_assemble launches (PMC bytes per live "
                                     "fit-row x this run's live fit-rows)",
                     "traffic_source": "profiles/pmc_mm.json (FETCH_SIZE + WRITE_SIZE, 8-B loads calibrated on "
                                       "the affine pass)" if pmc else None,
                     "kernel": "mm_assemble_mfma_kernel<16, true>",
                     "assemble_ms": asm_ms, "live_fit_rows": fit_rows, "bytes_per_fit_row": bytes_row,
                     "tflops": fit_rows * flops_row / (asm_ms * 1e-3) / 1e12, "max_ipm_iterations": iters},
    }
    out["cpu_baseline"] = cpu_baseline_mm(d, args.sims, args.cpu_seconds, args.cpu_threads) \
        if world == 1 and args.cpu_seconds > 0 else None
    rows, ok = last
    out["check"] = {"ok_replicates": int(ok.sum()), "q50_gap_mean": float(np.nanmean(rows[:, 6]))}
    print(json.dumps(out), flush=True)


def heckman_frame(rows, preds, seed=20260425):
    """configs[1]'s wage panel plus a selection equation (builder .heckman_selection): s = 1[0.3 +
    0.5 z1 - 0.4 z2 + 0.2 x4 + u > 0], outcomes kept on unselected rows (tests/test_gpu_heckman.py's
    design at scale). Returns (frame, predictor names, selection predictor names)."""
    d = synthetic(rows, preds, False)
    rng = np.random.default_rng(seed)
    x = np.vstack([d["xa"], d["xb"]])
    n = x.shape[0]
    z1, z2 = rng.normal(size=n), rng.normal(size=n)
    s = (0.3 + 0.5 * z1 - 0.4 * z2 + 0.2 * x[:, 3] + rng.normal(size=n) > 0).astype(np.float64)
    names = [f"x{j + 1}" for j in range(preds)]
    frame = {"y": np.concatenate([d["ya"], d["yb"]]),
             "g": np.array(["M"] * len(d["ya"]) + ["F"] * len(d["yb"]), dtype=object), "s": s, "z1": z1, "z2": z2}
    frame.update({nm: np.ascontiguousarray(x[:, j]) for j, nm in enumerate(names)})
    return frame, names, ["z1", "z2", "x4"]


def bench_heckman(args, world, rank, local, dist):
    """Heckman two-step bootstrap (estimation.rs:114-260) on configs[1]'s panel: per replicate the
    probit of s on [1, z1, z2, x4] by Fisher scoring, the IMR sums and the IMR-augmented solve."""
    import torch

    ob = importlib.import_module("oaxaca-blinder-rs_amd")
    frame, names, zs = heckman_frame(args.rows, args.preds)
    b = (ob.OaxacaBuilder(frame, "y", "g", "F").predictors(names).heckman_selection("s", zs)
         .bootstrap_reps(args.reps).seed(0x0B5EED).device(local))
    pr = b.prepare()
    B, dev = args.reps, torch.device("cuda", local)
    rows = torch.empty((B, pr.row_len), dtype=torch.float64, device=dev)
    ok = torch.empty(B, dtype=torch.uint8, device=dev)

    def step(i):
        stream = torch.cuda.current_stream(dev).cuda_stream
        pr.boot_device((i * world + rank) * B, B, rows.data_ptr(), ok.data_ptr(), stream)
        if dist:
            g = torch.empty((world * B, pr.row_len), dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(g, rows)
        pr.sync()
        return pr.timing()

    for i in range(args.warmup):
        step(i)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tm_sum = {"gram_ms": 0.0, "heckman_ms": 0.0, "probit_ms": 0.0, "heck_sums_ms": 0.0, "level1_ms": 0.0,
              "counts_ms": 0.0}
    iters, launches = 0, 0
    for i in range(args.steps):
        tm = step(args.warmup + i)
        for k_ in tm_sum:
            tm_sum[k_] += tm[k_]
        iters = max(iters, tm["probit_iterations"])
        launches += tm["probit_launches"]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt[0])
    if rank != 0:
        pr.close()
        return
    ks = 1 + len(zs)
    probit_ms = tm_sum["probit_ms"] / max(1, launches)  # per ob_probit_kernel launch, HIP events
    pmc = load_probit_pmc(args.rows, args.preds, B, ks)
    flops_launch = pmc.get("f64_flops_per_dispatch") if pmc else None
    achieved = flops_launch / (probit_ms * 1e-3) / 1e12 if flops_launch else None
    okh = ok.cpu().numpy()
    out = {
        "metric": "Heckman two-step bootstrap replicates/sec (configs[1] panel + selection equation)",
        "value": world * B * args.steps / elapsed, "unit": "replicates/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak" if world > 1 else "single", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md §8d wage panel + s = 1[0.3 + 0.5 z1 - 0.4 z2 + 0.2 x4 + u > 0])",
        "config": {"workload": "heckman_selection(s, [z1, z2, x4]), GroupA reference coefficients",
                   "rows": args.rows, "predictors": args.preds, "selection_predictors": len(zs),
                   "replicates_per_gpu_per_step": B, "parallelism": f"replicates sharded x{world}"},
        # the dominant kernel: one Fisher-scoring pass of the probit (erfc, exp, reciprocals and the
        # Hessian/score FMAs per (replicate, row) with a nonzero count), bound by the f64 VALU
        "roofline": {"bound": "valu-f64", "achieved": achieved, "peak": F64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / F64_VALU_PEAK_TFLOPS if achieved else None, "traffic": None,
                     "kernel": f"ob_probit_kernel<{ks}>", "avg_launch_ms": probit_ms, "launches": launches,
                     "f64_flops_per_launch": flops_launch,
                     "flops_source": "rocprofv3 SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64 lanes "
                                     "(profiles/pmc_probit.json, tools/pmc_f64.py)",
                     "share_of_step": tm_sum["probit_ms"] / (elapsed * 1e3)},
        "breakdown_ms_per_step": {k_: v / args.steps for k_, v in tm_sum.items()},
        "gram_path": "i8 MFMA (exact slices)" if tm["gram_path"] == 2 else "f64 MFMA",
        "max_probit_iterations": iters,
        "cpu_baseline": None,
        "check": {"ok_replicates": int(okh.sum()), "explained_mean": float(rows[:, 0].mean().item())},
    }
    if world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline_heckman(frame, names, zs, args.cpu_seconds, args.cpu_threads)
    pr.close()
    print(json.dumps(out), flush=True)


def cpu_baseline_heckman(frame, names, zs, target_s, threads):
    """The oracle's heckman_single_pass (probit.rs / heckman.rs restated in numpy) on whole
    resampled replicates of the same panel, one replicate per task over a thread pool (numpy
    releases the GIL in its array kernels), as many rounds as fit in target_s."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    ia = np.flatnonzero(frame["g"] == "M")
    ib = np.flatnonzero(frame["g"] == "F")
    groups = []
    for rows in (ia, ib):
        x = np.column_stack([np.ones(len(rows))] + [frame[nm][rows] for nm in names])
        z = np.column_stack([np.ones(len(rows))] + [frame[nm][rows] for nm in zs])
        groups.append(dict(x=x, y=frame["y"][rows], w=None, zsel=z, s=frame["s"][rows]))

    def one(rep):
        take = []
        for gi, g in enumerate(groups):
            idx = O.resample_indices(0x0B5EED, 100000 + rep, gi, len(g["y"]))
            take.append({k_: (None if v is None else v[idx]) for k_, v in g.items()})
        O.heckman_single_pass(take[0], take[1], 0, False)

    n, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        while n == 0 or time.perf_counter() - t0 < target_s:
            list(ex.map(one, range(n, n + threads)))
            n += threads
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "replicates/s", **host_info(threads), "kind": "port",
            "sample": f"{n} replicates of the same panel through oracle.heckman_single_pass (numpy), "
                      f"{threads} threads, {dt:.1f} s"}


def load_mm_pmc(rows, preds, sims, reps):
    """mm_assemble's measured HBM bytes per live (fit, row) from the committed PMC summary
    (tools/gpu_r5_mm.sh -> profiles/pmc_mm.json), when it was taken at this shape."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_mm.json")) as f:
            j = json.load(f)
        if (j.get("rows"), j.get("predictors"), j.get("simulations"), j.get("replicates")) == (rows, preds, sims, reps):
            return j["kernels"]["mm_assemble_mfma_kernel<16, true>"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def load_probit_pmc(rows, preds, reps, ks):
    """f64 FLOPs per ob_probit_kernel launch from the committed PMC summary (tools/pmc_f64.py)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_probit.json")) as f:
            j = json.load(f)
        # the counts belong to one build of the kernel: the normal pdf/cdf path must match
        # (ob_heckman.hip: npdf_ncdf unless option hk_erfc = 0, which only a tuning build reads
        # from OB_HK_ERFC)
        ob = importlib.import_module("oaxaca-blinder-rs_amd")
        tuning = ob._native.lib().ob_tuning_build() == 1
        variant = "library_erfc" if tuning and os.environ.get("OB_HK_ERFC", "").strip() == "0" else "npdf_ncdf"
        if ((j.get("rows"), j.get("preds"), j.get("reps"), j.get("ks")) == (rows, preds, reps, ks)
                and j.get("erfc", "library_erfc") == variant):
            return j
    except (OSError, ValueError):
        pass
    return None


def load_traffic(rows, preds, reps, gram_path=1, kernel=None):
    """HBM bytes per Gram launch (ob_gram_kernel, or the i8 path's oz_gram_w_kernel / oz_gram_kernel)
    from the committed rocprofv3 PMC summary of that kernel at that size, else None."""
    path = os.path.join(ROOT, "profiles", "pmc_gram.json" if gram_path == 1 else "pmc_gram_i8.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if kernel and j.get("kernel") != kernel:
            return None
        if j.get("rows") == rows and j.get("preds") == preds and j.get("reps") == reps:
            return j.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def end_to_end(ob, ctx, d, ya, yb, n, ref, stat_cols, dev):
    """One configs[1] run() from a fresh panel, as the reference's published figures are whole runs
    (README.md:316-317): host -> HBM upload and the Gram panel (ob_panel_create), the point
    estimate on the unresampled panel (ob_point_estimate, builder.rs:810-811), the digit images
    and exception rows (prep, first boot of the panel), n replicates, and the aggregation of every
    reported component on the host. Host clock around all of it; prep_ms by HIP events."""
    import torch

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    panel = ob.Panel(d["xa"], ya, d["xb"], yb, d["wa"], d["wb"], ctx=ctx)
    t_create = time.perf_counter() - t0
    panel.set_gather_columns(list(range(len(stat_cols))))
    t1 = time.perf_counter()
    point = panel.point_estimate(ref)  # run_single_pass on the unresampled panel (builder.rs:810-811)
    t_point = time.perf_counter() - t1
    rows = torch.empty((n, panel.row_len), dtype=torch.float64, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    t2 = time.perf_counter()
    panel.boot_sharded_device(0x0B5EED, 0, n, rows.data_ptr(), ok.data_ptr(), ref,
                              stream=torch.cuda.current_stream(dev).cuda_stream)
    t_enqueue = time.perf_counter() - t2
    panel.sync()
    t_boot = time.perf_counter() - t2
    tm = panel.timing()
    t3 = time.perf_counter()
    hr = rows[:, : len(stat_cols)].cpu().numpy()
    ob.aggregate(np.ascontiguousarray(hr), ok.cpu().numpy(), stat_cols)
    t_agg = time.perf_counter() - t3
    total_s = time.perf_counter() - t0
    assert np.isfinite(point[: len(stat_cols)]).all(), "point estimate"

    panel.close()
    return {"replicates": n, "ms": total_s * 1e3, "replicates_per_s": n / total_s,
            "panel_create_ms": t_create * 1e3, "point_estimate_ms": t_point * 1e3, "prep_ms": tm["prep_ms"],
            "boot_enqueue_ms": t_enqueue * 1e3, "boot_wall_ms": t_boot * 1e3, "aggregate_ms": t_agg * 1e3,
            "boot_ms": tm["level1_ms"] + tm["counts_ms"] + tm["gram_ms"] + tm["reduce_ms"] + tm["solve_ms"],
            "oz_exceptions": tm["oz_exceptions"], "oz_bits": tm["oz_bits"],
            "what": "run() as builder.rs:787-983 runs it: fresh ob_panel_create (H2D + Gram panel) + the point "
                    "estimate (ob_point_estimate, builder.rs:810-811) + digit images/exception rows + one boot of n "
                    "replicates + host aggregation, host clock"}


def replicate_plan(reps, world, strong=False, weak=False):
    """(scaling, replicates per step in total, replicates per GPU per step). One GPU: configs[1],
    reps per step. Several GPUs: configs[2] by default -- reps per step in total, sharded over the
    ranks (strong scaling: the reference runs a fixed replicate count as independent Rayon tasks,
    builder.rs:816-839); --weak gives every rank its own reps per step instead."""
    if weak and strong:
        raise SystemExit("bench.py: --weak and --strong exclude each other")
    if world > 1 and not weak:
        strong = True
    total = reps if strong else reps * world
    if world == 1:  # one GPU is neither weak nor strong scaling
        return "single", total, total
    return ("strong" if strong else "weak"), total, -(-total // world)


def workload_label(mode, taus, total, world, per_rank):
    """config.workload of the default bench line, named for what it runs: configs[1] is one GPU at
    10,000 replicates per step; configs[2] is 10,000 per step in total sharded over the GPUs; a weak
    run on several GPUs is configs[1]'s panel at a per-GPU replicate count, never configs[1]; a
    one-GPU run at 1,250 is configs[2]'s per-GPU share at 8 GPUs."""
    if taus:
        return f"configs[3]: RIF decomposition at tau={taus}, two-fold WLS, GroupA"
    if mode == "strong" and world > 1:
        if total == 10000:
            return f"configs[2]: 10,000 replicates per step in total, sharded over {world} GPUs (strong)"
        return f"configs[1]'s panel, {total:,} replicates per step in total, sharded over {world} GPUs (strong)"
    if world > 1:
        return f"configs[1]'s panel, {per_rank:,} replicates per GPU, weak ({world} GPUs)"
    if per_rank == 10000:
        return "configs[1]: two-fold WLS bootstrap, GroupA reference coefficients"
    if 10000 % per_rank == 0 and 10000 // per_rank > 1:
        return (f"configs[2]'s per-GPU share at {10000 // per_rank} GPUs: configs[1]'s panel at {per_rank} "
                "replicates per GPU per step")
    return f"configs[1]'s panel at {per_rank} replicates per GPU per step (not a BASELINE config)"


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The torch.distributed.run command that runs this bench as n ranks on one node (one process
    per GPU, rendezvous on 127.0.0.1), with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def probe_gpu_count():
    """GPUs visible to a fresh process, counted in a child so that this process never touches the
    GPU before it starts the launcher (a process that initialised HIP must not exec or fork ranks)."""
    import subprocess

    code = "import torch; print(torch.cuda.device_count())"
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        return int(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError):
        return 0


def launch_ranks(argv, n):
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N ranks under torch.distributed.run
    as a child, forward rank 0's JSON line to stdout (everything else to stderr) and return the
    launcher's exit code. Fails loudly, before starting anything, when fewer than N GPUs exist."""
    import subprocess

    have = probe_gpu_count()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, this machine has {have}; "
              f"refusing to print a {have}-GPU line for an {n}-GPU run", file=sys.stderr, flush=True)
        return 3
    cmd = launcher_cmd(argv, n, free_port())
    print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            print(s, flush=True)
        else:
            sys.stderr.write(line)
    return proc.wait()


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10000,
                    help="replicates per step: in total, sharded over the GPUs (configs[2], the default for "
                         "N > 1), or per GPU with --weak")
    ap.add_argument("--strong", action="store_true",
                    help="--reps replicates per step in total, sharded over the GPUs (already the default)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: every GPU runs its own --reps replicates per step")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--preds", type=int, default=20)
    ap.add_argument("--ref", type=int, default=0, help="ReferenceCoefficients (0 = GroupA)")
    ap.add_argument("--unweighted", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="0 disables the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may use (host_cores())")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end configs[1] run from a fresh panel")
    ap.add_argument("--taus", type=str, default="",
                    help="configs[3]: comma-separated RIF quantiles sharing one bootstrap (e.g. 0.1,0.5,0.9); "
                         "reports replicate-quantiles/s instead of the headline metric")
    ap.add_argument("--mm", action="store_true",
                    help="configs[4]: Machado-Mata (defaults 500k rows x 15 predictors, 1000 simulations, "
                         "12 replicates per GPU per step, one batch; configs[4] is 125 per GPU); reports MM "
                         "replicates/s")
    ap.add_argument("--sims", type=int, default=1000, help="--mm: quantile regressions per group per replicate")
    ap.add_argument("--heckman", action="store_true",
                    help="Heckman two-step bootstrap on configs[1]'s panel plus a selection equation "
                         "(2000 replicates per GPU per step); reports Heckman replicates/s")
    args = ap.parse_args(argv)
    explicit = set(x.split("=")[0] for x in argv)
    if args.heckman and "--reps" not in explicit:
        args.reps = 2000
    if args.mm:
        if "--rows" not in explicit:
            args.rows = 500_000
        if "--preds" not in explicit:
            args.preds = 15
        if "--reps" not in explicit:
            args.reps = 12
    return args


def main():
    args = parse_args(sys.argv[1:])
    taus = [float(t) for t in args.taus.split(",") if t.strip()]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; the line reports the launched world "
              f"({world} ranks)", file=sys.stderr, flush=True)
    args.cpu_threads_explicit = args.cpu_threads > 0
    if args.cpu_threads <= 0:
        args.cpu_threads = host_cores()
    import torch

    torch.cuda.set_device(local)
    dist = None
    if "RANK" in os.environ or world > 1:  # launched by torch.distributed.run (world 1 included)
        import torch.distributed as dist

        with stdout_to_stderr():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.mm or args.heckman:
        (bench_mm if args.mm else bench_heckman)(args, world, rank, local, dist)
        if dist:
            dist.destroy_process_group()
        return
    ob = importlib.import_module("oaxaca-blinder-rs_amd")
    N = ob._native
    weighted = not args.unweighted
    d = synthetic(args.rows, args.preds, weighted)
    ya, yb = d["ya"], d["yb"]
    if taus:  # builder.rs:711-757: each group's outcome replaced by its RIF, one column per tau
        ya = np.column_stack([ob.rif(d["ya"], t) for t in taus])
        yb = np.column_stack([ob.rif(d["yb"], t) for t in taus])
    # the engine's own RCCL communicator (ob_ctx_create_rank): every step's rows are all-gathered
    # by ob_boot_run_sharded_device inside the timed loop, at N = 1 too
    with stdout_to_stderr():
        uid = [N.unique_id() if rank == 0 else None]
        if dist is not None and world > 1:
            dist.broadcast_object_list(uid, src=0)
        ctx = N.rank_context(local, rank, world, uid[0])
    rccl_rank, rccl_world = N.ctx_rank(ctx)
    if (rccl_rank, rccl_world) != (rank, world):
        raise RuntimeError(f"engine RCCL communicator is rank {rccl_rank} of {rccl_world}, expected {rank} of {world}")
    panel = ob.Panel(d["xa"], ya, d["xb"], yb, d["wa"], d["wb"], ctx=ctx)
    # strong (configs[2], the default at N > 1): --reps per step in total; --weak: --reps per rank
    mode, total, per_rank = replicate_plan(args.reps, world, args.strong, args.weak)
    rl, ny = panel.row_len, panel.n_y
    dev = torch.device("cuda", local)
    kd = panel.k + panel.n_base
    ns = 6 + 2 * kd  # every reported component (+ total_gap): the only columns the aggregation reads
    stat_cols = np.arange(ns, dtype=np.int32)
    panel.set_gather_columns(list(range(ns)))  # the RCCL all-gather moves only these 48 of 153 f64 (K = 21)
    seed = 0x0B5EED
    # Two row buffers: step i's replicates run on the GPU while rank 0 aggregates step i - 1's on
    # the host (builder.rs:841-930 after the loop of :816-839); the component columns come back
    # on a copy stream, overlapping the next step's kernels.
    rows = [torch.empty((ny * total, rl), dtype=torch.float64, device=dev) for _ in range(2)]
    ok = [torch.empty(ny * total, dtype=torch.uint8, device=dev) for _ in range(2)]
    h_rows = [torch.empty((ny * total, ns), dtype=torch.float64, pin_memory=True) for _ in range(2)]
    h_ok = [torch.empty(ny * total, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    copy_stream = torch.cuda.Stream(dev)
    booted = [torch.cuda.Event() for _ in range(2)]
    copied = [torch.cuda.Event() for _ in range(2)]
    pending = []  # buffers whose rows await aggregation on rank 0

    def aggregate(b):  # per outcome: bootstrap_stats over that outcome's block, in replicate order
        copied[b].synchronize()
        hr = h_rows[b].numpy().reshape(ny, total, ns)
        hk = h_ok[b].numpy().reshape(ny, total)
        return [ob.aggregate(np.ascontiguousarray(hr[t]), np.ascontiguousarray(hk[t]), stat_cols) for t in range(ny)][0]

    def step(i):
        b = i % 2
        cur = torch.cuda.current_stream(dev)
        cur.wait_event(copied[b])  # step i - 2's copy out of this buffer is done
        panel.boot_sharded_device(seed, i * total, total, rows[b].data_ptr(), ok[b].data_ptr(), args.ref,
                                  stream=cur.cuda_stream)
        stats = None
        if rank == 0:
            booted[b].record(cur)
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_event(booted[b])
                h_rows[b].copy_(rows[b][:, :ns], non_blocking=True)
                h_ok[b].copy_(ok[b], non_blocking=True)
                copied[b].record(copy_stream)
            if pending:
                stats = aggregate(pending.pop())
            pending.append(b)
        # no host synchronization per step: step i + 1 is enqueued while step i runs; the engine
        # sums the HIP-event kernel times of every call until panel.sync() (ob_panel_sync)
        return stats

    def drain():
        return aggregate(pending.pop()) if pending else None

    for i in range(args.warmup):
        step(i)
    drain()
    panel.sync()  # collects (and clears) the warmup's timings and overflow flag
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = None
    for i in range(args.steps):
        s_ = step(args.warmup + i)
        stats = s_ if s_ is not None else stats
    stats = drain() if rank == 0 else None  # the last step's aggregation, inside the timed region
    panel.sync()  # every timed call's kernel times (HIP events), the overflow checks
    tm = panel.timing()
    sums = {k_: tm[k_] for k_ in ("gram_ms", "level1_ms", "counts_ms", "reduce_ms", "solve_ms", "gather_ms")}
    launches = tm["gram_launches"]
    gram_path = tm["gram_path"]
    tiles6 = (tm["oz_tiles6"], tm["oz_tiles"])
    gram_kernel = "oz_gram_w_kernel" if tm["oz_wide"] else "oz_gram_kernel"
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, sums["gram_ms"] / max(launches, 1)], dtype=torch.float64, device=dev)
    if dist and world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, gram_launch_ms = float(t[0]), float(t[1])

    e2e = None
    if not args.no_e2e and not taus and world == 1:
        e2e = end_to_end(ob, ctx, d, ya, yb, total, args.ref, stat_cols, dev)

    if rank == 0:
        value = total * args.steps / elapsed
        k = args.preds + 1
        flops_rep = 2.0 * args.rows * (k * (k + 1) / 2 + ny * k)  # SURVEY.md §8d (X^T W X + one X^T W y per outcome)
        bytes_rep = args.rows * (args.preds + (2 if weighted else 1)) * 8.0
        reps_per_launch = min(per_rank, 16384) if launches else 0
        achieved = flops_rep * reps_per_launch / (gram_launch_ms * 1e-3) / 1e12 if gram_launch_ms else 0.0
        traffic = load_traffic(args.rows, args.preds, per_rank, gram_path,
                               gram_kernel if gram_path == 2 else "ob_gram_kernel") if not taus else None
        if gram_path == 2:
            # exact integer-sliced Gram (ob_gram_i8.hip): the algorithmic work is one i8 multiply-add per
            # (replicate, row, live pair, 8-bit digit slice run): 7 slices, 6 on the (chunk, column tile)
            # blocks of narrow magnitude range (oz_tiles6 of oz_tiles); the MFMA work pads pairs to
            # 32-wide column tiles
            pairs = (k + ny) * (k + ny + 1) // 2
            slices = OZ_SLICES - (tiles6[0] / tiles6[1] if tiles6[1] else 0.0)
            ops_rep = 2.0 * args.rows * pairs * slices
            ops_issued = 2.0 * args.rows * (-(-pairs // OZ_PAIRS_PER_TILE) * OZ_PAIRS_PER_TILE) * slices
            i8_tops = ops_rep * reps_per_launch / (gram_launch_ms * 1e-3) / 1e12 if gram_launch_ms else 0.0
            roof = {"bound": "mfma", "achieved": i8_tops, "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS (i8)",
                    "frac": i8_tops / I8_MFMA_PEAK_TOPS, "traffic": traffic,
                    "traffic_source": "profiles/pmc_gram_i8.json (PMC 2 x FETCH_SIZE + WRITE_SIZE of this kernel at this size, round 6)",
                    "kernel": gram_kernel,
                    "avg_launch_ms": gram_launch_ms, "i8_ops_per_replicate": ops_rep,
                    "i8_ops_issued_per_replicate": ops_issued, "digit_slices_mean": slices,
                    "tiles_on_6_slices": list(tiles6),
                    "f64_equivalent_tflops": achieved, "f64_flops_per_replicate": flops_rep,
                    "f64_equivalent_x_of_f64_mfma_peak": achieved / F64_MFMA_PEAK_TFLOPS}
        else:
            roof = {"bound": "mfma", "achieved": achieved, "peak": F64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / F64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                    "kernel": "ob_gram_kernel", "avg_launch_ms": gram_launch_ms,
                    "flops_per_replicate": flops_rep}
        out = {
            "metric": "bootstrap replicates/sec on 1M-row×20-pred panel at 1/2/4/8 MI355X" if not taus else
                      "RIF bootstrap replicate-quantiles/sec (configs[3], quantiles share each resample)",
            "value": value * ny,
            "unit": "replicates/s" if not taus else "replicate-quantiles/s",
            "n_gpus": world,
            "rccl_world": rccl_world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": mode,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8d wage panel, numpy seed 20260424; OBRS-3 bootstrap seed 0x0B5EED)",
            "config": {"workload": workload_label(mode, taus, total, world, per_rank),
                       "rows": args.rows, "predictors": args.preds, "weighted": weighted,
                       "replicates_per_step": total, "replicates_per_gpu_per_step": per_rank,
                       "parallelism": f"replicates sharded x{world}, engine RCCL all-gather (ob_boot_run_sharded_device)"},
            "roofline": roof,
            "gram_path": ("i8 MFMA (v_mfma_i32_16x16x64_i8), 7 balanced 8-bit digit slices of a 54-bit fixed point, "
                          "the last dropped on narrow-range tiles (DESIGN.md §5.0)") if gram_path == 2 else "f64 MFMA",
            # what a per-replicate row gather would have to stream: a rate, not a
            # roofline fraction -- the Gram reads each panel byte once per 256-replicate tile instead
            "gather_equivalent": {"algorithmic_bytes_per_replicate": bytes_rep,
                                  "GBps": bytes_rep * value / world / 1e9,
                                  "x_of_hbm_peak": bytes_rep * value / world / 1e9 / HBM_PEAK_GBPS},
            "breakdown_ms_per_step_rank0": {k_: v / args.steps for k_, v in sums.items()},
            "end_to_end": e2e,
        }
        if world == 1 and args.cpu_seconds > 0 and not taus:
            # every usable core (the reference's Rayon pool); when the box's per-GPU share
            # (OMP_NUM_THREADS) is smaller, that share too, and the faster of the two is the value
            runs = [cpu_baseline(d, args.preds, weighted, args.ref, args.cpu_seconds, args.cpu_threads)]
            share = omp_share()
            if not args.cpu_threads_explicit and share and share < args.cpu_threads:
                runs.append(cpu_baseline(d, args.preds, weighted, args.ref, args.cpu_seconds, share))
            best = max(runs, key=lambda r: r["value"])
            best["other_thread_counts"] = [{"cores": r["cores"], "value": r["value"]} for r in runs if r is not best]
            out["cpu_baseline"] = best
        else:
            out["cpu_baseline"] = None
        out["check"] = {"explained_se": float(stats[0][0]), "unexplained_se": float(stats[1][0]),
                        "ok_replicates": int(ok[(args.warmup + args.steps - 1) % 2].sum().item()),
                        "quantiles": taus or None}
        print(json.dumps(out), flush=True)
    panel.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
