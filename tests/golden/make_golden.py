"""Generate golden vectors for the BracketedCamError residual path.

An INDEPENDENT restatement of the reference formulas in mpmath at 50 digits
(not the C++ oracle, not the HIP kernels):
  array_to_rigid_transform  dense_map_utils.cc:171-178
  linearInterp / slerp      dense_map_utils.cc:315-329 (Eigen 3.4 [ext])
  calc_world_to_cam_trans   rig_calibrator.cc:322-390
  BracketedCamError         rig_calibrator.cc:447-482
  DistortCentered           camera_params.cc:260-314, compute_rpc rpc_distortion.cc:116-160
Jacobians by mpmath.diff (high-precision numerical differentiation), a method
independent of both the dual numbers of oracle/oracle.cpp and the analytic chain
rule of the GPU kernels.

The reference ships no tests/fixtures and cannot be built here,
so these vectors pin the oracle restatement, not the reference binary
("parity unpinned" — DESIGN.md "Oracle").

Run (container only, ~1 min):  python tests/golden/make_golden.py
Writes tests/golden/cam_error_golden.json.
"""
from __future__ import annotations

import json
import os
import sys

import mpmath as mp
import numpy as np

mp.mp.dps = 50
EPS = 2.0 ** -52

HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------- formulas
def quat_to_rot(x, y, z, w):
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return [[1 - (tyy + tzz), txy - twz, txz + twy],
            [txy + twz, 1 - (txx + tzz), tyz - twx],
            [txz - twy, tyz + twx, 1 - (txx + tyy)]]


def rot_to_quat(m):
    t = m[0][0] + m[1][1] + m[2][2]
    q = [None] * 4
    if t > 0:
        t = mp.sqrt(t + 1)
        q[3] = t / 2
        t = mp.mpf(1) / (2 * t)
        q[0] = (m[2][1] - m[1][2]) * t
        q[1] = (m[0][2] - m[2][0]) * t
        q[2] = (m[1][0] - m[0][1]) * t
    else:
        i = 0
        if m[1][1] > m[0][0]:
            i = 1
        if m[2][2] > m[i][i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = mp.sqrt(m[i][i] - m[j][j] - m[k][k] + 1)
        q[i] = t / 2
        t = mp.mpf(1) / (2 * t)
        q[3] = (m[k][j] - m[j][k]) * t
        q[j] = (m[j][i] + m[i][j]) * t
        q[k] = (m[k][i] + m[i][k]) * t
    return q


def rigid(p):
    x, y, z, w = p[3], p[4], p[5], p[6]
    n = mp.sqrt(x * x + y * y + z * z + w * w)
    return quat_to_rot(x / n, y / n, z / n, w / n), [p[0], p[1], p[2]]


def matmul(A, B):
    return [[sum(A[r][k] * B[k][c] for k in range(3)) for c in range(3)] for r in range(3)]


def matvec(A, v):
    return [sum(A[r][k] * v[k] for k in range(3)) for r in range(3)]


def world_to_cam(p0, p1, p2, off, sb, se, sc):
    if sb == se:
        return rigid(p0)
    R0, t0 = rigid(p0)
    R1, t1 = rigid(p1)
    R2, t2 = rigid(p2)
    alpha = ((mp.mpf(sc) - mp.mpf(sb)) - off) / (mp.mpf(se) - mp.mpf(sb))
    if alpha < 0 or alpha > 1:
        raise ValueError("Out of bounds in interpolation.")
    q0, q1 = rot_to_quat(R0), rot_to_quat(R1)
    ti = [(1 - alpha) * t0[k] + alpha * t1[k] for k in range(3)]
    d = sum(q0[k] * q1[k] for k in range(4))
    ad = abs(d)
    if ad >= 1 - mp.mpf(EPS):
        s0, s1 = 1 - alpha, alpha
    else:
        th = mp.acos(ad)
        st = mp.sin(th)
        s0 = mp.sin((1 - alpha) * th) / st
        s1 = mp.sin(alpha * th) / st
    if d < 0:
        s1 = -s1
    qi = [s0 * q0[k] + s1 * q1[k] for k in range(4)]
    Ri = quat_to_rot(*qi)
    return matmul(R2, Ri), [a + b for a, b in zip(matvec(R2, ti), t2)]


def rpc(x, y, coeffs):
    n = len(coeffs)
    deg = int(round((np.sqrt(2.0 * n + 5.0) / 2.0 - 1.5)))
    vals = [mp.mpf(0), mp.mpf(1), mp.mpf(0), mp.mpf(1)]
    ci = 0
    for cnt in range(4):
        start = 1 if cnt in (1, 3) else 0
        for dg in range(start, deg + 1):
            for i in range(dg + 1):
                vals[cnt] += coeffs[ci] * x ** (dg - i) * y ** i
                ci += 1
    return vals[0] / vals[1], vals[2] / vals[3]


def distort(u0, u1, f, c, k, h):
    K = len(k)
    if K == 0:
        d = (u0 + c[0] - h[0], u1 + c[1] - h[1])
    elif K == 1:
        pc1 = 1 / k[0]
        pc2 = 2 * mp.tan(k[0] / 2)
        n0, n1 = u0 / f, u1 / f
        ru = mp.sqrt(n0 * n0 + n1 * n1)
        rd = mp.atan(ru * pc2) * pc1
        conv = rd / ru if ru > 1e-5 else mp.mpf(1)
        d = (c[0] - h[0] + conv * n0 * f, c[1] - h[1] + conv * n1 * f)
    elif K in (4, 5):
        k1, k2, p1, p2 = k[:4]
        k3 = k[4] if K == 5 else 0
        n0, n1 = u0 / f, u1 / f
        r2 = n0 * n0 + n1 * n1
        rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
        e0 = rad * n0 + 2 * p1 * n0 * n1 + p2 * (r2 + 2 * n0 * n0)
        e1 = rad * n1 + p1 * (r2 + 2 * n1 * n1) + 2 * p2 * n0 * n1
        d = (e0 * f + c[0] - h[0], e1 * f + c[1] - h[1])
    else:
        d = rpc(u0, u1, k[:K // 2])
    return d[0] + h[0], d[1] + h[1]


def residual(blocks, h, meas, sb, se, sc):
    p0, p1, p2, X, off, f, c, k = blocks
    R, t = world_to_cam(p0, p1, p2, off[0], sb, se, sc)
    Xc = [a + b for a, b in zip(matvec(R, X), t)]
    u0 = f[0] * (Xc[0] / Xc[2])
    u1 = f[0] * (Xc[1] / Xc[2])
    d = distort(u0, u1, f[0], c, k, h)
    return [d[0] - meas[0], d[1] - meas[1]]


# ----------------------------------------------------------------- cases
def qaxis(axis, deg):
    a = np.asarray(axis, dtype=float)
    a = a / np.linalg.norm(a)
    th = np.deg2rad(deg)
    return list(a * np.sin(th / 2)) + [float(np.cos(th / 2))]


def make_cases():
    rng = np.random.default_rng(20240515)
    cases = []
    models = {
        "none": [], "fov": [0.9], "radtan5": [-0.25, 0.07, 1e-3, -5e-4, 0.01],
        "radtan4": [-0.2, 0.05, 2e-3, 1e-3],
    }
    for deg in (1, 2, 3):
        n = 2 * (deg + 1) * (deg + 2) - 2
        nl = (deg + 1) * (deg + 2) // 2
        half = np.zeros(n)
        half[1] = 1.0
        half[2 * nl - 1 + 2] = 1.0
        half += rng.normal(0, 1e-5, size=n) * np.array(
            [512.0 ** -max(0, int(np.floor(np.sqrt(2 * (j % nl) + 0.25) - 0.5))) for j in range(n)])
        models[f"rpc{deg}"] = list(np.concatenate([half, half + rng.normal(0, 1e-6, n)]))

    def base_pose(j):
        phi = np.deg2rad(10.0 * j)
        C = np.array([8 * np.cos(phi), 0.2, 8 * np.sin(phi)])
        fwd = -C / np.linalg.norm(C)
        xc = np.cross([0, 1, 0], fwd); xc /= np.linalg.norm(xc)
        yc = np.cross(fwd, xc)
        Rw = np.stack([xc, yc, fwd], axis=0)  # world_to_cam rotation (rows)
        t = -Rw @ C
        # quaternion of Rw (any sign), unnormalised on purpose
        w = np.sqrt(max(1e-12, 1 + np.trace(Rw))) / 2
        if w > 0.1:
            q = [(Rw[2, 1] - Rw[1, 2]) / (4 * w), (Rw[0, 2] - Rw[2, 0]) / (4 * w), (Rw[1, 0] - Rw[0, 1]) / (4 * w), w]
        else:
            i = int(np.argmax(np.diag(Rw))); jx, k = (i + 1) % 3, (i + 2) % 3
            s = np.sqrt(1 + Rw[i, i] - Rw[jx, jx] - Rw[k, k]) * 2
            q = [0, 0, 0, 0]
            q[i] = s / 4; q[3] = (Rw[k, jx] - Rw[jx, k]) / s
            q[jx] = (Rw[jx, i] + Rw[i, jx]) / s; q[k] = (Rw[k, i] + Rw[i, k]) / s
        q = np.array(q) * (1.0 + 0.01 * rng.normal())
        return list(t) + list(q)

    r2c = list(np.array([0.1, -0.02, 0.03])) + list(np.array(qaxis([0.1, 1, 0.05], 15.0)) * 0.98)
    ident = [0, 0, 0, 0, 0, 0, 1]
    sb, se = 1.6e9 + 12.5, 1.6e9 + 13.0
    kinds = ["ref", "interp", "interp_alpha0", "interp_alpha1", "no_rig", "slerp_lin", "slerp_neg", "axis"]
    for mname, k in models.items():
        for kind in kinds:
            p0 = base_pose(rng.integers(0, 36))
            p1 = base_pose(rng.integers(0, 36))
            X = list(rng.normal(0, 1.5, 3))
            off = [0.01]
            sc = sb + 0.25 + off[0]
            f = [600.0 * (1 + 0.01 * rng.normal())]
            c = [515.0 + rng.normal(), 382.0 + rng.normal()]
            h = [512.0, 384.0]
            s_b, s_e, s_c = sb, se, sc
            e1, rr = p1, r2c
            if kind in ("ref", "no_rig"):
                s_b = s_e = s_c = sb
                e1 = ident
            elif kind == "interp_alpha0":
                off = [0.0]
                s_c = sb  # alpha == 0 exactly
            elif kind == "interp_alpha1":
                off = [0.0]
                s_c = se  # alpha == 1 exactly
            elif kind == "slerp_lin":
                e1 = list(p0)
            elif kind == "slerp_neg":
                p0 = [0.3, -0.1, 8.0] + qaxis([1, 0, 0], 100.0)
                e1 = [0.35, -0.12, 8.1] + qaxis([1, 0, 0], -100.0)
                X = [0.2, 0.1, 2.0]
                rr = ident
            elif kind == "axis":
                # optical-axis point (FOV ru < 1e-5 branch)
                p0 = [0.0, 0.0, 5.0, 0.0, 0.0, 0.0, 1.0]
                s_b = s_e = s_c = sb
                e1 = ident
                X = [0.0, 0.0, 1.0]
            # measurement near the projection
            blocks_f = [p0, e1, rr, X, list(off), f, c, k]
            mblocks = [[mp.mpf(v) for v in b] for b in blocks_f]
            try:
                r_exact = residual(mblocks, h, [0, 0], s_b, s_e, s_c)
            except ValueError:
                continue
            meas = [float(np.float32(float(r_exact[0]) + rng.normal(0, 0.7))),
                    float(np.float32(float(r_exact[1]) + rng.normal(0, 0.7)))]
            cases.append(dict(model=mname, kind=kind, blocks=[list(map(float, b)) for b in blocks_f],
                              half=h, meas=meas, stamps=[s_b, s_e, s_c]))
    return cases


def jacobian(case):
    blocks = [[mp.mpf(v) for v in b] for b in case["blocks"]]
    h, meas = case["half"], case["meas"]
    sb, se, sc = case["stamps"]
    r = residual(blocks, h, meas, sb, se, sc)
    J = []
    for b, blk in enumerate(blocks):
        cols = []
        for j in range(len(blk)):
            def fr(t, i, b=b, j=j):
                bb = [list(x) for x in blocks]
                bb[b][j] = bb[b][j] + t
                return residual(bb, h, meas, sb, se, sc)[i]
            col = None
            # alpha exactly 0 or 1: the offset derivative exists one-sided only
            for direction in (0, -1, 1):
                try:
                    col = [float(mp.diff(lambda t: fr(t, 0), 0, direction=direction)),
                           float(mp.diff(lambda t: fr(t, 1), 0, direction=direction))]
                    break
                except ValueError:
                    continue
            cols.append(col)
        # row-major 2 x size (Ceres)
        J.append([cc[0] for cc in cols] + [cc[1] for cc in cols])
    return [float(r[0]), float(r[1])], J


def main():
    cases = make_cases()
    out = []
    for i, cs in enumerate(cases):
        r, J = jacobian(cs)
        cs["residual"] = r
        cs["jacobian"] = J
        out.append(cs)
        print(f"{i + 1}/{len(cases)} {cs['model']} {cs['kind']}", file=sys.stderr)
    with open(os.path.join(HERE, "cam_error_golden.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden.py", "mp_dps": 50, "cases": out}, fh, indent=0)


if __name__ == "__main__":
    main()
