"""Numpy prototype of the GPU quantile-regression solver (ob_mm.hip): Mehrotra predictor-corrector
on the bounded dual LP  max y'x  s.t.  X'x = (1 - tau) X'c,  0 <= x <= c  (c = resample counts),
whose equality multipliers are the QR coefficients. Pass structure mirrors the kernels:
  assemble (M = X'QX, X'q r), affine step + corrector right-hand sides, final step lengths.
Design aid only (compared here with scipy HiGHS); the oracle does not use it.
usage: python tools/qr_ipm_proto.py [--start]   (--start: iteration counts of the OLS start vs the
shifted start of mm_shift_kernel at n = 250k, the configs[4] group size)
"""
import sys

import numpy as np
from scipy.optimize import linprog

NO_RP = True  # the kernels assume A x = b (feasible start, A dx = 0 steps)


def qr_ipm(X, y, c, tau, tol=1e-12, max_iter=100, eta=0.99995, shift=True):
    act = c > 0
    X, y, c = X[act], y[act], c[act].astype(float)
    n, K = X.shape
    b = (1.0 - tau) * (X.T @ c)
    # start: x interior and feasible, beta = weighted OLS, z - w = X beta - y (dual feasible)
    x = (1.0 - tau) * c
    G = (X.T * c) @ X
    beta = np.linalg.solve(G, X.T @ (c * y))
    r = y - X @ beta
    if shift:  # mm_shift_kernel: intercept to the tau-quantile of the OLS residuals (count-weighted)
        o = np.argsort(r)
        cw = np.cumsum(c[o])
        beta[0] += r[o][np.searchsorted(cw, tau * cw[-1])]
        r = y - X @ beta
        dlt = 0.01 * (1.0 + np.sqrt((c * r * r).sum() / c.sum()))
    else:  # the plain OLS start
        dlt = 0.1 * (1.0 + np.sqrt((c * r * r).sum() / c.sum()))
    z = np.maximum(-r, 0.0) + dlt
    w = np.maximum(r, 0.0) + dlt
    for it in range(1, max_iter + 1):
        s = c - x
        gap = x @ z + s @ w
        obj = y @ x
        rp = (b - X.T @ x) * (0.0 if NO_RP else 1.0)
        if gap < tol * (1.0 + abs(obj)):
            return beta, it - 1, True
        mu = gap / (2 * n)
        rd = y - X @ beta - w + z
        q = 1.0 / (z / x + w / s)
        M = (X.T * q) @ X
        L = np.linalg.cholesky(M)
        sol = lambda v: np.linalg.solve(L.T, np.linalg.solve(L, v))
        # affine (sigma = 0): rho = rd + w - z
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


def qr_highs(X, y, c, tau):
    act = c > 0
    X, y, c = X[act], y[act], c[act].astype(float)
    res = linprog(-y, A_eq=X.T, b_eq=(1 - tau) * (X.T @ c), bounds=list(zip(np.zeros(len(c)), c)), method="highs")
    assert res.status == 0
    return -res.eqlin.marginals


def main():
    rng = np.random.default_rng(1)
    worst, its = 0.0, []
    for trial in range(40):
        n = int(rng.integers(50, 3000))
        K = int(rng.integers(2, 9))
        X = np.column_stack([np.ones(n), rng.normal(size=(n, K - 1))])
        if trial % 4 == 0:
            X[:, 1] = np.round(rng.uniform(8, 20, n))  # integer covariate
        y = X @ rng.normal(size=K) + rng.standard_t(3, size=n)
        c = rng.multinomial(n, np.ones(n) / n) if trial % 2 else np.ones(n, dtype=int)
        tau = float(rng.uniform(0.01, 0.99))
        b1, it, ok = qr_ipm(X, y, c, tau)
        b2 = qr_highs(X, y, c, tau)
        err = np.abs(b1 - b2).max() / (1 + np.abs(b2).max())
        worst = max(worst, err)
        its.append(it)
        print(f"n={n:5d} K={K} tau={tau:.3f} boot={trial % 2} its={it:3d} ok={ok} rel.err={err:.2e}")
    print("worst", worst, "iterations median", np.median(its), "max", max(its))


def start_study():
    sys.path.insert(0, __file__.rsplit("/", 2)[0])
    import bench

    d = bench.synthetic(500000, 15, False)
    X = np.column_stack([np.ones(250000), d["xa"]])
    c = np.random.default_rng(3).multinomial(250000, np.ones(250000) / 250000)
    for tau in (0.01, 0.05, 0.2, 0.5, 0.8, 0.95, 0.99):
        its = [qr_ipm(X, d["ya"], c, tau, max_iter=300, shift=sh)[1] for sh in (False, True)]
        print(f"tau={tau:.2f} iterations: OLS start {its[0]}, shifted start {its[1]}", flush=True)


if __name__ == "__main__":
    start_study() if "--start" in sys.argv else main()
