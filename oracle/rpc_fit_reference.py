"""CPU restatement of the RPC lens-model fits.

TEST INFRASTRUCTURE (oracle/): only tests/ may call this.

    genUndistDistPairs   rpc_distortion.cc:519-557
    DistortCentered      camera_params.cc:260-314 (vectorised)
    compute_rpc          rpc_distortion.cc:116-160
    init_as_identity / increment_degree   :303-318, :336-356
    fitRpcDist / fitRpcUndist             :622-656, :658-721
    fitCurrDegRPC        :559-609: Ceres LM (numpy, dense exact steps, the
                         control flow of oracle/lm_reference.py)
    evalRpcDistUndist    :723-737

The fit itself is pinned by convergence: the parity test compares the fitted
models' outputs on the samples, not LM trajectories.
"""
from __future__ import annotations

import numpy as np


def rpc_degree(n: int) -> int:
    return int(round(np.sqrt(2.0 * n + 5.0) / 2.0 - 1.5))


def _monomials(x, y, d):
    """[N, nl] monomials x^(deg-i) y^i, deg = 0..d, i = 0..deg (reference order)."""
    cols = []
    for dg in range(d + 1):
        for i in range(dg + 1):
            cols.append(x ** (dg - i) * y ** i)
    return np.stack(cols, axis=1)


def compute_rpc(p, c):
    """p [N, 2], c: 2 (d+1)(d+2) - 2 coefficients."""
    d = rpc_degree(len(c))
    nl = (d + 1) * (d + 2) // 2
    m = 2 * nl - 1
    M = _monomials(p[:, 0], p[:, 1], d)
    out = np.empty_like(p)
    for h in range(2):
        cn = c[h * m:h * m + nl]
        cd = c[h * m + nl:(h + 1) * m]
        out[:, h] = (M @ cn) / (1.0 + M[:, 1:] @ cd)
    return out


def distort_centered(u, cam):
    f = cam["focal"]
    c = np.asarray(cam["center"], dtype=np.float64)
    h = np.asarray(cam["image_size"], dtype=np.float64) / 2.0
    k = np.asarray(cam["dist"], dtype=np.float64)
    K = k.size
    if K == 0:
        return u + c - h
    if K == 1:
        n = u / f
        ru = np.linalg.norm(n, axis=1)
        rd = np.arctan(ru * (2 * np.tan(k[0] / 2))) * (1 / k[0])
        conv = np.where(ru > 1e-5, rd / np.where(ru > 0, ru, 1.0), 1.0)
        return (c - h) + conv[:, None] * n * f
    if K in (4, 5):
        k1, k2, p1, p2 = k[:4]
        k3 = k[4] if K == 5 else 0.0
        n = u / f
        r2 = (n * n).sum(axis=1)
        rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
        o = rad[:, None] * n
        o[:, 0] += 2 * p1 * n[:, 0] * n[:, 1] + p2 * (r2 + 2 * n[:, 0] ** 2)
        o[:, 1] += p1 * (r2 + 2 * n[:, 1] ** 2) + 2 * p2 * n[:, 0] * n[:, 1]
        return o * f + (c - h)
    return compute_rpc(u, k[:K // 2])


def pairs(cam, num_samples):
    """genUndistDistPairs: (undist_c, dist_c) of the samples inside the crop box."""
    S = num_samples
    uw, uh = cam["undist_size"]
    ix, iy = np.meshgrid(np.arange(S), np.arange(S), indexing="ij")
    x = (uw - 1.0) * ix.reshape(-1) / (S - 1.0)
    y = (uh - 1.0) * iy.reshape(-1) / (S - 1.0)
    uh2 = np.array([uw / 2.0, uh / 2.0])
    dh = np.asarray(cam["image_size"], dtype=np.float64) / 2.0
    u = np.stack([x, y], axis=1) - uh2
    dpix = distort_centered(u, cam) + dh
    W, H = cam["image_size"]
    cw, ch = cam["crop_size"]
    keep = ~((np.abs(dpix[:, 0] - W / 2.0) > cw / 2.0) | (np.abs(dpix[:, 1] - H / 2.0) > ch / 2.0))
    return u[keep], (dpix - dh)[keep]


def _fit_degree(inp, tgt, c, max_iter, ptol):
    d = rpc_degree(len(c))
    nl = (d + 1) * (d + 2) // 2
    m = 2 * nl - 1
    M = _monomials(inp[:, 0], inp[:, 1], d)

    def evaluate(x, jac):
        r = np.empty((len(inp), 2))
        J = np.zeros((2 * len(inp), 2 * m)) if jac else None
        for h in range(2):
            cn, cd = x[h * m:h * m + nl], x[h * m + nl:(h + 1) * m]
            N = M @ cn
            D = 1.0 + M[:, 1:] @ cd
            r[:, h] = N / D - tgt[:, h]
            if jac:
                J[h::2, h * m:h * m + nl] = M / D[:, None]
                J[h::2, h * m + nl:(h + 1) * m] = -M[:, 1:] * (N / D ** 2)[:, None]
        return r.reshape(-1), J

    x = c.copy()
    r, J = evaluate(x, True)
    cost = 0.5 * r @ r
    g = J.T @ r
    H = J.T @ J
    s = 1.0 / (1.0 + np.sqrt(np.diag(H)))
    if np.abs(g).max() <= 1e-16:
        return x
    radius, decrease, invalid = 1e4, 2.0, 0
    for _ in range(max_iter):
        A = s[:, None] * H * s[None, :]
        A[np.diag_indices_from(A)] += np.clip(np.diag(A), 1e-6, 1e32) / radius
        try:
            delta = s * np.linalg.solve(A, -s * g)
        except np.linalg.LinAlgError:
            delta = None
        model = -(g @ delta + 0.5 * delta @ H @ delta) if delta is not None else -1.0
        if delta is None or not np.isfinite(model) or model <= 0:
            invalid += 1
            if invalid > 5:
                return x
            radius /= decrease
            decrease *= 2
            continue
        invalid = 0
        xn = x + delta
        rn, _ = evaluate(xn, False)
        cn = 0.5 * rn @ rn
        if np.linalg.norm(delta) <= ptol * (np.linalg.norm(x) + ptol):
            return x
        if abs(cost - cn) <= 1e-16 * cost:
            return x
        rho = (cost - cn) / model
        if np.isfinite(cn) and rho > 1e-3:
            x = xn
            r, J = evaluate(x, True)
            cost = 0.5 * r @ r
            g = J.T @ r
            H = J.T @ J
            radius = min(1e16, radius / max(1 / 3, 1 - (2 * rho - 1) ** 3))
            decrease = 2.0
            if np.abs(g).max() <= 1e-16:
                return x
        else:
            radius /= decrease
            decrease *= 2
            if radius < 1e-32:
                return x
    return x


def identity(d=1):
    nl = (d + 1) * (d + 2) // 2
    m = 2 * nl - 1
    c = np.zeros(2 * m)
    c[1] = 1.0
    c[m + 2] = 1.0
    return c


def increment_degree(c):
    d = rpc_degree(len(c))
    nl = (d + 1) * (d + 2) // 2
    m = 2 * nl - 1
    add = np.zeros(d + 2)
    out = []
    for h in range(2):
        out += [c[h * m:h * m + nl], add, c[h * m + nl:(h + 1) * m], add]
    return np.concatenate(out)


def fit(inp, tgt, degree, num_iterations, parameter_tolerance):
    c = identity(1)
    for dg in range(1, degree + 1):
        if dg >= 2:
            c = increment_degree(c)
        c = _fit_degree(inp, tgt, c, num_iterations, parameter_tolerance)
    return c


def fit_rpc_dist(cam, degree, num_samples, num_iterations=100, parameter_tolerance=1e-12):
    u, dc = pairs(cam, num_samples)
    return fit(u, dc, degree, num_iterations, parameter_tolerance), u


def fit_rpc_undist(cam, dist_coeffs, num_samples, num_iterations=100, parameter_tolerance=1e-12):
    u, _ = pairs(cam, num_samples)
    dc = compute_rpc(u, dist_coeffs)
    c = fit(dc, u, rpc_degree(len(dist_coeffs)), num_iterations, parameter_tolerance)
    err = np.linalg.norm(u - compute_rpc(compute_rpc(u, dist_coeffs), c), axis=1).max()
    return c, u, dc, err
