"""Generate golden vectors for BracketedDepthError (rig_calibrator.cc:547-583).

An independent 50-digit mpmath restatement (shares only the pose formulas of
make_golden.py, themselves independent of the C++ oracle and the kernels):
  T_wc      = calc_world_to_cam_trans(beg, end, ref_to_cam, stamps, offset)
  D         = array_to_rigid_transform(p3) or array_to_affine_transform(p3)
              (dense_map_utils.cc:171-178, :195-208), linear part *= scale (p4)
  M         = T_wc^-1 (D meas)            (generic affine inverse)
  r         = weight (X - M)              (3 residuals)
Jacobians by mpmath.diff, row-major 3 x size per block (Ceres layout).

Run (container only, ~1 min):  python tests/golden/make_golden_depth.py
Writes tests/golden/depth_error_golden.json.
"""
from __future__ import annotations

import json
import os
import sys

import mpmath as mp
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import matvec, qaxis, rigid, world_to_cam  # noqa: E402

mp.mp.dps = 50
HERE = os.path.dirname(os.path.abspath(__file__))


def inv3(R):
    mi = mp.matrix(R) ** -1
    return [[mi[r, c] for c in range(3)] for r in range(3)]


def depth_residual(blocks, weight, meas, sb, se, sc):
    p0, p1, p2, dti, scale, X, off = blocks
    R, t = world_to_cam(p0, p1, p2, off[0], sb, se, sc)
    if len(dti) == 12:
        L = [[dti[4 * r + c] for c in range(3)] for r in range(3)]
        td = [dti[4 * r + 3] for r in range(3)]
    else:
        L, td = rigid(dti)
    L = [[L[r][c] * scale[0] for c in range(3)] for r in range(3)]
    Md = [a + b for a, b in zip(matvec(L, meas), td)]
    Ri = inv3(R)
    M = matvec(Ri, [Md[k] - t[k] for k in range(3)])  # T^-1 y = R^-1 (y - t)
    return [weight * (X[k] - M[k]) for k in range(3)]


def make_cases():
    rng = np.random.default_rng(20240601)
    sb, se = 1.6e9 + 12.5, 1.6e9 + 13.0
    r2c = [0.1, -0.02, 0.03] + list(np.array(qaxis([0.1, 1, 0.05], 15.0)) * 0.98)
    ident = [0, 0, 0, 0, 0, 0, 1]
    cases = []
    for affine in (False, True):
        for kind in ("ref", "interp", "no_rig", "scale"):
            phi = rng.uniform(0, 2 * np.pi)
            p0 = [8 * np.cos(phi), 0.2, 8 * np.sin(phi)] + list(np.array(qaxis(rng.normal(size=3), 40.0)) * 1.01)
            p1 = [8 * np.cos(phi + 0.01), 0.21, 8 * np.sin(phi + 0.01)] + list(
                np.array(qaxis(rng.normal(size=3), 41.0)) * 0.99)
            if affine:
                A = np.eye(3) + rng.normal(0, 0.02, (3, 3))
                dti = list(np.concatenate([A, rng.normal(0, 0.05, (3, 1))], axis=1).reshape(-1))
            else:
                dti = [0.05, -0.02, 0.01] + list(np.array(qaxis(rng.normal(size=3), 2.0)) * 1.02)
            scale = [1.0 + (0.03 if kind == "scale" else 0.0)]
            X = list(rng.normal(0, 1.5, 3))
            off = [0.01]
            s_b, s_e, s_c, e1, rr = sb, se, sb + 0.25 + 0.01, p1, r2c
            if kind in ("ref", "no_rig"):
                s_b = s_e = s_c = sb
                e1 = ident
            meas = list(np.float32(rng.normal(0, 2.0, 3)).astype(np.float64))
            weight = 10.0
            cases.append(dict(affine=affine, kind=kind, blocks=[p0, e1, rr, dti, scale, X, off], weight=weight,
                              meas=meas, stamps=[s_b, s_e, s_c]))
    return cases


def jacobian(case):
    blocks = [[mp.mpf(v) for v in b] for b in case["blocks"]]
    meas = [mp.mpf(v) for v in case["meas"]]
    w = mp.mpf(case["weight"])
    sb, se, sc = case["stamps"]
    r = depth_residual(blocks, w, meas, sb, se, sc)
    J = []
    for b, blk in enumerate(blocks):
        cols = []
        for j in range(len(blk)):
            def fr(t, i, b=b, j=j):
                bb = [list(x) for x in blocks]
                bb[b][j] = bb[b][j] + t
                return depth_residual(bb, w, meas, sb, se, sc)[i]
            cols.append([float(mp.diff(lambda t: fr(t, i), 0)) for i in range(3)])
        J.append([cc[i] for i in range(3) for cc in cols])  # row-major 3 x size
    return [float(v) for v in r], J


def main():
    out = []
    for i, cs in enumerate(make_cases()):
        r, J = jacobian(cs)
        cs["blocks"] = [list(map(float, b)) for b in cs["blocks"]]
        cs["residual"] = r
        cs["jacobian"] = J
        out.append(cs)
        print(f"{i + 1} {cs['affine']} {cs['kind']}", file=sys.stderr)
    with open(os.path.join(HERE, "depth_error_golden.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden_depth.py", "mp_dps": 50, "cases": out}, fh, indent=0)


if __name__ == "__main__":
    main()
