"""Design aid for the Machado-Mata row reduction (Portnoy & Koenker 1997, "the Gaussian hare and
the Laplacian tortoise"): solve each QR on a subsample, keep the rows whose residual lies in a
band around the fit's quantile, fix the others at their bound (x_i = c_i above the hyperplane, 0
below), solve the reduced LP and verify the fixed rows' signs. Measures, at the configs[4] group
size, the kept fraction and the misclassified rows for several band rules.
usage: python tools/qr_pk_proto.py
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 2)[0])
import bench  # noqa: E402
from qr_ipm_proto import qr_ipm  # noqa: E402


def band(X, y, c, beta, tau, delta, ns=4096):
    """(lo, hi): the count-weighted tau -/+ delta quantiles of ns residuals at a fixed stride."""
    act = np.flatnonzero(c)
    pick = act[(np.arange(ns) * len(act)) // ns]
    r = y[pick] - X[pick] @ beta
    o = np.argsort(r)
    cw = np.cumsum(c[pick][o]).astype(float)
    W = cw[-1]
    lo = r[o][min(np.searchsorted(cw, max(tau - delta, 0.0) * W), ns - 1)] if tau - delta > 0 else -np.inf
    hi = r[o][min(np.searchsorted(cw, min(tau + delta, 1.0) * W), ns - 1)] if tau + delta < 1 else np.inf
    return lo, hi


def main():
    d = bench.synthetic(500000, 15, False)
    n = 250000
    X = np.column_stack([np.ones(n), d["xa"]])
    y = d["ya"]
    c = np.random.default_rng(3).multinomial(n, np.ones(n) / n)
    K = X.shape[1]
    sub = np.zeros(n, dtype=np.int64)
    sub[::8] = c[::8]  # phase 1: every 8th row
    m = int((sub > 0).sum())
    print(f"n={n} active={int((c > 0).sum())} K={K} subsample m={m}")
    for tau in (0.02, 0.1, 0.25, 0.5, 0.75, 0.9, 0.98):
        t0 = time.time()
        bstar, it, ok = qr_ipm(X, y, c, tau)
        t1 = time.time()
        bhat, it1, ok1 = qr_ipm(X, y, sub, tau, tol=1e-6)
        rstar = y - X @ bstar
        rhat = y - X @ bhat
        line = f"tau={tau:.2f} full its={it} ({t1 - t0:.1f}s) phase1 its={it1}"
        for kappa in (2.0, 3.0, 4.0):
            delta = kappa * np.sqrt(tau * (1 - tau) * K / m) + 0.01
            lo, hi = band(X, y, c, bhat, tau, delta)
            keep = (rhat >= lo) & (rhat <= hi) & (c > 0)
            above = (rhat > hi) & (c > 0)
            below = (rhat < lo) & (c > 0)
            bad = int((above & (rstar < -1e-9)).sum() + (below & (rstar > 1e-9)).sum())
            line += f" | k={kappa}: keep {keep.sum() / (c > 0).sum():.3f} bad {bad}"
        print(line, flush=True)


if __name__ == "__main__" and "--block" not in sys.argv and "--lev" not in sys.argv:
    main()


def qr_ipm_b(X, y, c, tau, b, beta0, tol=1e-12, max_iter=200, eta=0.99995, start="plain", dscale=0.01, dlt=None):
    """qr_ipm with a general right-hand side X'x = b (infeasible start x = (1 - tau) c) and a
    given starting beta: phase 2 of the row reduction."""
    act = c > 0
    X, y, c = X[act], y[act], c[act].astype(float)
    n, K = X.shape
    x = (1.0 - tau) * c
    beta = beta0.copy()
    r = y - X @ beta
    if dlt is None:
        dlt = dscale * (1.0 + np.sqrt((c * r * r).sum() / c.sum()))
    z = np.maximum(-r, 0.0) + dlt
    w = np.maximum(r, 0.0) + dlt
    if start == "centered":  # x z = (c - x) w: x = c w / (z + w)
        x = c * w / (z + w)
    for it in range(1, max_iter + 1):
        s = c - x
        gap = x @ z + s @ w
        obj = y @ x
        rp = b - X.T @ x
        if gap < tol * (1.0 + abs(obj)) and np.abs(rp).max() < 1e-9 * (1 + np.abs(b).max()):
            return beta, it - 1, True
        mu = gap / (2 * n)
        rd = y - X @ beta - w + z
        q = 1.0 / (z / x + w / s)
        M = (X.T * q) @ X
        L = np.linalg.cholesky(M)
        sol = lambda v: np.linalg.solve(L.T, np.linalg.solve(L, v))
        rho_a = rd + w - z
        dba = sol(X.T @ (q * rho_a) - rp)
        dxa = q * (rho_a - X @ dba)
        dza = -z - z * dxa / x
        dwa = -w + w * dxa / s

        def maxstep(v, dv, cap=1.0):
            m = dv < 0
            return min(cap, (-v[m] / dv[m]).min()) if m.any() else cap
        ap = min(maxstep(x, dxa), maxstep(s, -dxa))
        ad = min(maxstep(z, dza), maxstep(w, dwa))
        mu_a = ((x + ap * dxa) @ (z + ad * dza) + (s - ap * dxa) @ (w + ad * dwa)) / (2 * n)
        sig = (mu_a / mu) ** 3
        rho0 = rho_a - dxa * (dwa / s + dza / x)
        rho1 = 1.0 / x - 1.0 / s
        db = sol(X.T @ (q * rho0) + sig * mu * (X.T @ (q * rho1)) - rp)
        rho_c = rho0 + sig * mu * rho1
        dx = q * (rho_c - X @ db)
        rxz = sig * mu - x * z - dxa * dza
        rsw = sig * mu - s * w + dxa * dwa
        dz = (rxz - z * dx) / x
        dw = (rsw + w * dx) / s
        ap = min(1.0, eta * min(maxstep(x, dx, 1e300), maxstep(s, -dx, 1e300)))
        ad = min(1.0, eta * min(maxstep(z, dz, 1e300), maxstep(w, dw, 1e300)))
        x = x + ap * dx
        beta = beta + ad * db
        z = z + ad * dz
        w = w + ad * dw
    return beta, max_iter, False


def block_study(kappa=4.0, nfit=64, center=0.5):
    d = bench.synthetic(500000, 15, False)
    n = 250000
    X = np.column_stack([np.ones(n), d["xa"]])
    y = d["ya"]
    c = np.random.default_rng(3).multinomial(n, np.ones(n) / n)
    K = X.shape[1]
    sub = np.zeros(n, dtype=np.int64)
    sub[::8] = c[::8]
    m = int((sub > 0).sum())
    taus = np.sort(np.random.default_rng(5).uniform(size=1000))
    j0 = int(np.searchsorted(taus, center))
    j0 = min(max(j0 - nfit // 2, 0), 1000 - nfit)
    blk = taus[j0:j0 + nfit]
    fits = []
    union = np.zeros(n, dtype=bool)
    for tau in blk:
        bhat, it1, _ = qr_ipm(X, y, sub, tau, tol=1e-6)
        rhat = y - X @ bhat
        delta = kappa * np.sqrt(tau * (1 - tau) * K / m) + 0.01
        lo, hi = band(X, y, c, bhat, tau, delta)
        keep = (rhat >= lo) & (rhat <= hi) & (c > 0)
        union |= keep
        fits.append((tau, bhat, rhat, lo, hi, it1))
    act = c > 0
    print(f"block tau [{blk[0]:.3f}, {blk[-1]:.3f}]: union keeps {union.sum() / act.sum():.3f} of active rows")
    for tau, bhat, rhat, lo, hi, it1 in fits[:: max(1, nfit // 6)]:
        cr = np.where(union, c, 0)
        above = act & ~union & (rhat > hi)
        b = (1.0 - tau) * (X.T @ c) - X[above].T @ c[above]
        b2, it2, ok2 = qr_ipm_b(X, y, cr, tau, b, bhat)
        rf = rhat[act]
        dfull = 0.01 * (1.0 + np.sqrt((c[act] * rf * rf).sum() / c[act].sum()))
        its = [qr_ipm_b(X, y, cr, tau, b, bhat, start="centered", dscale=ds)[1] for ds in (0.01, 0.03, 0.1)]
        its.append(qr_ipm_b(X, y, cr, tau, b, bhat, start="centered", dlt=dfull)[1])
        bstar, it, _ = qr_ipm(X, y, c, tau)
        rs = y - X @ b2
        below = act & ~union & (rhat < lo)
        bad = int((above & (rs < -1e-9)).sum() + (below & (rs > 1e-9)).sum())
        err = np.abs(b2 - bstar).max() / (1 + np.abs(bstar).max())
        print(f"  tau={tau:.3f} phase1 its={it1} phase2 its={it2} centered {its} ok={ok2} full its={it} bad={bad} rel.err={err:.1e}",
              flush=True)


if __name__ == "__main__" and "--block" in sys.argv:
    for ctr in [float(a) for a in sys.argv[2:]] or (0.5, 0.1, 0.03):
        block_study(center=ctr)


def leverage_study(nfit=100, kappa=4.0):
    """Misclassified rows against their leverage lev_i = sqrt(n x_i' G^-1 x_i) (G = X'CX of the
    phase-1 subsample), and the kept fraction of leverage-scaled bands."""
    d = bench.synthetic(500000, 15, False)
    n = 250000
    X = np.column_stack([np.ones(n), d["xa"]])
    y = d["ya"]
    c = np.random.default_rng(3).multinomial(n, np.ones(n) / n)
    K = X.shape[1]
    sub = np.zeros(n, dtype=np.int64)
    sub[::8] = c[::8]
    m = int((sub > 0).sum())
    act = c > 0
    G = (X[sub > 0].T * sub[sub > 0]) @ X[sub > 0]
    L = np.linalg.cholesky(G)
    v = np.linalg.solve(L, X.T).T
    lev = np.sqrt(sub.sum() * (v * v).sum(1))
    print(f"lev: mean {lev[act].mean():.2f} sqrtK {np.sqrt(K):.2f} p99 {np.percentile(lev[act], 99):.2f} max {lev[act].max():.2f}")
    rules = {"plain": lambda lo, hi, s: (lo, hi),
             "mult": lambda lo, hi, s: (lo * np.maximum(1, lev / np.sqrt(K)), hi * np.maximum(1, lev / np.sqrt(K))),
             "add": lambda lo, hi, s: (lo - s * np.maximum(lev - np.sqrt(K), 0), hi + s * np.maximum(lev - np.sqrt(K), 0))}
    stats = {k: [0, 0.0] for k in rules}
    for tau in np.linspace(0.02, 0.98, nfit):
        bstar, _, _ = qr_ipm(X, y, c, tau)
        bhat, _, _ = qr_ipm(X, y, sub, tau, tol=1e-6)
        rhat = y - X @ bhat
        rs = y - X @ bstar
        delta = kappa * np.sqrt(tau * (1 - tau) * K / m) + 0.01
        lo, hi = band(X, y, c, bhat, tau, delta)
        se = kappa * np.sqrt(tau * (1 - tau) / m) * ((hi - lo) / (2 * delta) if np.isfinite(hi - lo) else 0.0)
        for k, rule in rules.items():
            l2, h2 = rule(lo, hi, se)
            keep = act & (rhat >= l2) & (rhat <= h2)
            bad = (act & ~keep & (rhat > h2) & (rs < -1e-9)) | (act & ~keep & (rhat < l2) & (rs > 1e-9))
            stats[k][0] += bool(bad.any())
            stats[k][1] += keep.sum() / act.sum()
            if k == "plain" and bad.any():
                print(f"  tau {tau:.3f}: {bad.sum()} bad rows, lev {np.round(lev[bad], 2)}", flush=True)
    for k, (nb, kf) in stats.items():
        print(f"{k}: fits with a misclassified row {nb}/{nfit}, mean kept fraction {kf / nfit:.3f}")


if __name__ == "__main__" and "--lev" in sys.argv:
    leverage_study()
