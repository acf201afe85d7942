"""CPU reference of the solver path — TEST INFRASTRUCTURE ONLY.

Levenberg-Marquardt with the control flow of Ceres 1.14's TrustRegionMinimizer +
LevenbergMarquardtStrategy [ext, not vendored] (the solver rig_calibrator.cc:1910-1919
configures), with EXACT linear solves (dense LU of J'J + D; sparse LU above
SPARSE_COLUMNS free columns) in place of
ITERATIVE_SCHUR's truncated CG, on the Jacobian of oracle.cpp (the restatement of
BracketedCamError, rig_calibrator.cc:419-514). Used by tests to check that
mvba_solve converges to the same parameters. Parity unpinned (Ceres is absent from
this image: no reference solver run is available to compare trajectories with).
"""
from __future__ import annotations

import dataclasses

import numpy as np

from . import oracle_py

FIXED = (7, 7, 7, 3, 1, 1, 2)


def _columns(P):
    """Free parameter columns: non-constant blocks referenced by residuals, in
    block-id order (points included)."""
    K_of = P.camera_dist_size[P.residual_camera]
    used = np.zeros(len(P.block_size), dtype=bool)
    for b in range(7):
        used[P.residual_blocks[:, b]] = True
    used[P.residual_blocks[K_of > 0, 7]] = True
    if P.num_depth_residuals:
        db = P.depth_blocks.reshape(-1)
        used[db[db >= 0]] = True  # -1: the mesh point of a BracketedDepthMeshError block
    if P.num_xyz_residuals:
        used[P.xyz_block] = True
    free = np.nonzero(used & (P.block_constant == 0))[0]
    col = np.full(len(P.block_size), -1, dtype=np.int64)
    pos = 0
    idx = []
    for b in free:
        col[b] = pos
        o, n = int(P.block_offset[b]), int(P.block_size[b])
        idx.extend(range(o, o + n))
        pos += n
    return col, np.array(idx, dtype=np.int64)


# Above this many free columns the Jacobian is kept sparse (CSR) and the damped
# normal equations are solved by sparse LU (scipy.sparse.linalg.splu): the same
# exact step, without a dense 2N x n matrix (BASELINE c1: 10k rows x 3.4k
# columns). Smaller problems keep the dense path.
SPARSE_COLUMNS = 2000


class _Triplets:
    """COO accumulation with np.add.at's semantics (duplicates summed)."""

    def __init__(self, nrows, ncols):
        self.shape = (nrows, ncols)
        self.r, self.c, self.v = [], [], []

    def add(self, rows, cols, vals):
        self.r.append(np.asarray(rows, dtype=np.int64).reshape(-1))
        self.c.append(np.broadcast_to(np.asarray(cols, dtype=np.int64), np.shape(rows)).reshape(-1))
        self.v.append(np.asarray(vals, dtype=np.float64).reshape(-1))

    def csr(self):
        import scipy.sparse as sp

        cat = (lambda a, t: np.concatenate(a) if a else np.zeros(0, t))
        return sp.coo_matrix((cat(self.v, np.float64), (cat(self.r, np.int64), cat(self.c, np.int64))),
                             shape=self.shape).tocsr()


def _jacobian_sparse(P, params, col, ncols, use_loss, thr):
    """_jacobian as a CSR matrix (same entries; reprojection, depth and XYZ rows)."""
    from multiview_amd._lib import JAC_BASE
    Q = dataclasses.replace(P, params=params)
    cost, r, J = oracle_py.evaluate(Q, oracle_py.ANALYTIC, apply_loss=use_loss, robust_threshold=thr)
    N = P.num_residuals
    nrows = 2 * N + 3 * P.num_depth_residuals + 3 * P.num_xyz_residuals
    T = _Triplets(nrows, ncols)
    K_of = P.camera_dist_size[P.residual_camera]
    rows = np.arange(N)
    for b in range(8):
        for K in (np.unique(K_of) if b == 7 else [None]):
            sel = rows if b < 7 else rows[K_of == K]
            n = FIXED[b] if b < 7 else int(K)
            if n == 0 or sel.size == 0:
                continue
            c0 = col[P.residual_blocks[sel, b]]
            ok = c0 >= 0
            Jb = J[sel, JAC_BASE[b]:JAC_BASE[b] + 2 * n].reshape(-1, 2, n)
            for k in range(n):
                for comp in range(2):
                    T.add(2 * sel[ok] + comp, c0[ok] + k, Jb[ok, comp, k])
    r = r.reshape(-1)
    row0 = 2 * N
    if P.num_depth_residuals:
        cd, rd, Jd = oracle_py.evaluate_depth(Q, oracle_py.ANALYTIC, apply_loss=use_loss, robust_threshold=thr)
        for j in range(P.num_depth_residuals):
            for b in range(7):
                bid = int(P.depth_blocks[j, b])
                if bid < 0 or col[bid] < 0:
                    continue
                size = int(P.block_size[bid])
                base = oracle_py.DJAC_BASE[b]
                blk = Jd[j, base:base + 3 * size].reshape(3, size)
                rr, cc = np.meshgrid(np.arange(3), np.arange(size), indexing="ij")
                T.add(row0 + 3 * j + rr, col[bid] + cc, blk)
        cost += cd
        r = np.concatenate([r, rd.reshape(-1)])
        row0 += 3 * P.num_depth_residuals
    if P.num_xyz_residuals:
        cx, rx, Jx = oracle_py.evaluate_xyz(Q, apply_loss=use_loss)
        for j in range(P.num_xyz_residuals):
            c0 = col[int(P.xyz_block[j])]
            if c0 >= 0:
                rr, cc = np.meshgrid(np.arange(3), np.arange(3), indexing="ij")
                T.add(row0 + 3 * j + rr, c0 + cc, Jx[j].reshape(3, 3))
        cost += cx
        r = np.concatenate([r, rx.reshape(-1)])
    return cost, r, T.csr()


def _jacobian(P, params, col, ncols, use_loss, thr):
    if ncols > SPARSE_COLUMNS:
        return _jacobian_sparse(P, params, col, ncols, use_loss, thr)
    from multiview_amd._lib import JAC_BASE
    Q = dataclasses.replace(P, params=params)
    cost, r, J = oracle_py.evaluate(Q, oracle_py.ANALYTIC, apply_loss=use_loss, robust_threshold=thr)
    N = P.num_residuals
    D = np.zeros((2 * N, ncols))
    K_of = P.camera_dist_size[P.residual_camera]
    rows = np.arange(N)
    for b in range(8):
        size = FIXED[b] if b < 7 else None
        for K in (np.unique(K_of) if b == 7 else [None]):
            sel = rows if b < 7 else rows[K_of == K]
            n = size if b < 7 else int(K)
            if n == 0 or sel.size == 0:
                continue
            c0 = col[P.residual_blocks[sel, b]]
            ok = c0 >= 0
            Jb = J[sel, JAC_BASE[b]:JAC_BASE[b] + 2 * n].reshape(-1, 2, n)
            for k in range(n):
                for comp in range(2):
                    np.add.at(D, (2 * sel[ok] + comp, c0[ok] + k), Jb[ok, comp, k])
    r = r.reshape(-1)
    if P.num_depth_residuals:
        # BracketedDepthError rows (rig_calibrator.cc:547-583), 3 per block
        cd, rd, Jd = oracle_py.evaluate_depth(Q, oracle_py.ANALYTIC, apply_loss=use_loss, robust_threshold=thr)
        nd = P.num_depth_residuals
        Dd = np.zeros((3 * nd, ncols))
        for j in range(nd):
            for b in range(7):
                bid = int(P.depth_blocks[j, b])
                if bid < 0:
                    continue
                c0 = col[bid]
                if c0 < 0:
                    continue
                size = int(P.block_size[bid])
                base = oracle_py.DJAC_BASE[b]
                Dd[3 * j:3 * j + 3, c0:c0 + size] += Jd[j, base:base + 3 * size].reshape(3, size)
        cost += cd
        r = np.concatenate([r, rd.reshape(-1)])
        D = np.vstack([D, Dd])
    if P.num_xyz_residuals:
        cx, rx, Jx = oracle_py.evaluate_xyz(Q, apply_loss=use_loss)
        nx = P.num_xyz_residuals
        Dx = np.zeros((3 * nx, ncols))
        for j in range(nx):
            c0 = col[int(P.xyz_block[j])]
            if c0 >= 0:
                Dx[3 * j:3 * j + 3, c0:c0 + 3] = Jx[j].reshape(3, 3)
        cost += cx
        r = np.concatenate([r, rx.reshape(-1)])
        D = np.vstack([D, Dx])
    return cost, r, D


def _cost(P, params, use_loss, thr):
    Q = dataclasses.replace(P, params=params)
    c, _, _ = oracle_py.evaluate(Q, oracle_py.ANALYTIC, apply_loss=use_loss, robust_threshold=thr)
    if P.num_depth_residuals:
        c += oracle_py.evaluate_depth(Q, oracle_py.RESIDUAL, apply_loss=use_loss, robust_threshold=thr)[0]
    if P.num_xyz_residuals:
        c += oracle_py.evaluate_xyz(Q, apply_loss=use_loss)[0]
    return c


def solve(P, max_num_iterations=50, function_tolerance=1e-6, gradient_tolerance=1e-10,
          parameter_tolerance=1e-8, use_loss=False, robust_threshold=3.0, lower_bounds=None,
          upper_bounds=None, initial_trust_region_radius=1e4, jacobi_scaling=True):
    """Returns (packed params, summary dict). Bounds: packed arrays (projection only,
    no line search: used by tests on problems where the bounds are inactive)."""
    col, idx = _columns(P)
    n = idx.size
    params = P.params.copy()
    lo = lower_bounds[idx] if lower_bounds is not None else None
    hi = upper_bounds[idx] if upper_bounds is not None else None

    def plus(x, d):
        v = x + d
        if lo is not None:
            v = np.maximum(v, lo)
        if hi is not None:
            v = np.minimum(v, hi)
        return v

    def with_x(x):
        p = params.copy()
        p[idx] = x
        return p

    sparse = n > SPARSE_COLUMNS

    def colsq(J):
        return np.asarray(J.multiply(J).sum(axis=0)).reshape(-1) if sparse else np.einsum("ij,ij->j", J, J)

    def damped_step(J, s, c, g, radius):
        if not sparse:
            Js = J * s
            As = Js.T @ Js + np.diag(np.clip(s * s * c, 1e-6, 1e32) / radius)
            return -s * np.linalg.solve(As, s * g)
        import scipy.sparse as sp
        from scipy.sparse.linalg import splu

        Js = J @ sp.diags(s)
        As = (Js.T @ Js + sp.diags(np.clip(s * s * c, 1e-6, 1e32) / radius)).tocsc()
        return -s * splu(As).solve(s * g)

    x = params[idx].copy()
    cost, r, J = _jacobian(P, with_x(x), col, n, use_loss, robust_threshold)
    g = J.T @ r
    c = colsq(J)
    s = 1.0 / (1.0 + np.sqrt(c)) if jacobi_scaling else np.ones(n)
    gmax = np.abs(x - plus(x, -g)).max() if n else 0.0
    radius, decrease = initial_trust_region_radius, 2.0
    it, successful = 0, True
    summary = dict(initial_cost=cost, iterations=0, successful=1, unsuccessful=0, message="")
    while True:
        if it >= max_num_iterations:
            summary["message"] = "max iterations"
            break
        if successful and gmax <= gradient_tolerance:
            summary["message"] = "gradient tolerance"
            break
        if radius <= 1e-32:
            summary["message"] = "min radius"
            break
        it += 1
        # Ceres solves the damped system on the Jacobi-scaled Jacobian J S
        # (TrustRegionMinimizer + LevenbergMarquardtStrategy [ext]); the same step
        # as (J'J + D)^-1 g in exact arithmetic, but far better conditioned when
        # column norms span many decades (RPC degree >= 5: cond 1e46 unscaled).
        delta = damped_step(J, s, c, g, radius)
        Jd = J @ delta
        mcc = -(g @ delta + 0.5 * Jd @ Jd)
        if not (mcc > 0):
            radius /= decrease
            decrease *= 2
            successful = False
            summary["unsuccessful"] += 1
            continue
        xn = plus(x, delta)
        cand = _cost(P, with_x(xn), use_loss, robust_threshold)
        xnorm = np.linalg.norm(x)
        if np.linalg.norm(xn - x) <= parameter_tolerance * (xnorm + parameter_tolerance):
            summary["message"] = "parameter tolerance"
            break
        change = cost - cand
        if abs(change) <= function_tolerance * cost:
            summary["message"] = "function tolerance"
            break
        ratio = change / mcc
        if ratio > 1e-3:
            x = xn
            cost, r, J = _jacobian(P, with_x(x), col, n, use_loss, robust_threshold)
            g = J.T @ r
            c = colsq(J)
            gmax = np.abs(x - plus(x, -g)).max()
            radius = min(1e16, radius / max(1.0 / 3.0, 1.0 - (2.0 * ratio - 1.0) ** 3))
            decrease = 2.0
            successful = True
            summary["successful"] += 1
        else:
            radius /= decrease
            decrease *= 2
            successful = False
            summary["unsuccessful"] += 1
    summary.update(final_cost=cost, iterations=it)
    return with_x(x), summary


def first_step_system(P, use_loss=False, robust_threshold=3.0, initial_trust_region_radius=1e4):
    """The damped, Jacobi-scaled normal equations of the first LM iteration,
    A y = b with A = (J S)'(J S) + diag(clip(S^2 c, 1e-6, 1e32) / radius),
    b = -S g and the step delta = S y (the system damped_step solves in
    solve()), plus the spectrum bounds that turn a residual into an error bound:
    ||y - y*|| / ||y*|| <= kappa ||A y - b|| / ||b|| for the SPD A.
    Returns dict(A (scipy CSC), b, s, idx (packed parameter indices of the free
    columns), x0, lam_max, lam_min, kappa, y_exact)."""
    import scipy.sparse as sp
    from scipy.sparse.linalg import eigsh, splu

    col, idx = _columns(P)
    n = idx.size
    x0 = P.params[idx].copy()
    _, r, J = _jacobian(P, P.params.copy(), col, n, use_loss, robust_threshold)
    J = sp.csr_matrix(J)
    g = J.T @ r
    c = np.asarray(J.multiply(J).sum(axis=0)).reshape(-1)
    s = 1.0 / (1.0 + np.sqrt(c))
    Js = J @ sp.diags(s)
    A = (Js.T @ Js + sp.diags(np.clip(s * s * c, 1e-6, 1e32) / initial_trust_region_radius)).tocsc()
    b = -s * g
    lu = splu(A)
    y = lu.solve(b)
    lam_max = float(eigsh(A, k=1, which="LA", return_eigenvectors=False, tol=1e-6)[0])
    lam_min = float(eigsh(A, k=1, sigma=0.0, which="LM", return_eigenvectors=False, tol=1e-6)[0])
    return dict(A=A, b=b, s=s, idx=idx, x0=x0, lam_max=lam_max, lam_min=lam_min, kappa=lam_max / lam_min,
                y_exact=y)
