"""Generate golden vectors for BracketedDepthMeshError (rig_calibrator.cc:641-673).

50-digit mpmath restatement (pose formulas shared with make_golden.py, the
depth-cloud transform with make_golden_depth.py; independent of the C++ oracle
and the kernels):
  T_wc = calc_world_to_cam_trans(beg, end, ref_to_cam, stamps, offset)
  M    = T_wc^-1 ((scale * D.linear) meas + D.translation)
  r    = weight (mesh_xyz - M)        (3 residuals; mesh_xyz is data)
Blocks [beg, end, ref_to_cam, depth_to_image (7 | 12), scale, offset];
Jacobians by mpmath.diff, row-major 3 x size per block (Ceres layout).

Run (container only, ~1 min):  python tests/golden/make_golden_depth_mesh.py
Writes tests/golden/depth_mesh_error_golden.json.
"""
from __future__ import annotations

import json
import os
import sys

import mpmath as mp
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import qaxis  # noqa: E402
from make_golden_depth import depth_residual  # noqa: E402

mp.mp.dps = 50
HERE = os.path.dirname(os.path.abspath(__file__))


def mesh_residual(blocks, weight, meas, mesh, sb, se, sc):
    # weight (mesh - M) = depth_residual with the landmark replaced by the mesh point
    p0, p1, p2, dti, scale, off = blocks
    return depth_residual([p0, p1, p2, dti, scale, mesh, off], weight, meas, sb, se, sc)


def make_cases():
    rng = np.random.default_rng(20241016)
    sb, se = 1.6e9 + 40.0, 1.6e9 + 40.5
    r2c = [-0.1, 0.02, 0.05] + list(np.array(qaxis([0.2, 1, -0.1], 12.0)) * 1.01)
    ident = [0, 0, 0, 0, 0, 0, 1]
    cases = []
    for affine in (False, True):
        for kind in ("ref", "interp", "scale"):
            phi = rng.uniform(0, 2 * np.pi)
            p0 = [8 * np.cos(phi), -0.1, 8 * np.sin(phi)] + list(np.array(qaxis(rng.normal(size=3), 35.0)) * 0.97)
            p1 = [8 * np.cos(phi + 0.01), -0.09, 8 * np.sin(phi + 0.01)] + list(
                np.array(qaxis(rng.normal(size=3), 36.0)) * 1.02)
            if affine:
                A = np.eye(3) + rng.normal(0, 0.02, (3, 3))
                dti = list(np.concatenate([A, rng.normal(0, 0.05, (3, 1))], axis=1).reshape(-1))
            else:
                dti = [0.04, 0.01, -0.02] + list(np.array(qaxis(rng.normal(size=3), 3.0)) * 0.99)
            scale = [1.0 + (0.02 if kind == "scale" else 0.0)]
            off = [-0.02]
            s_b, s_e, s_c, e1 = sb, se, sb + 0.3 - 0.02, p1
            if kind == "ref":
                s_b = s_e = s_c = sb
                e1 = ident
            meas = list(np.float32(rng.normal(0, 2.0, 3)).astype(np.float64))
            mesh = list(4.0 * rng.normal(size=3) / 1.7)
            cases.append(dict(affine=affine, kind=kind, blocks=[p0, e1, r2c, dti, scale, off], weight=5.0,
                              meas=meas, mesh=mesh, stamps=[s_b, s_e, s_c]))
    return cases


def jacobian(case):
    blocks = [[mp.mpf(v) for v in b] for b in case["blocks"]]
    meas = [mp.mpf(v) for v in case["meas"]]
    mesh = [mp.mpf(v) for v in case["mesh"]]
    w = mp.mpf(case["weight"])
    sb, se, sc = case["stamps"]
    r = mesh_residual(blocks, w, meas, mesh, sb, se, sc)
    J = []
    for b, blk in enumerate(blocks):
        cols = []
        for j in range(len(blk)):
            def fr(t, i, b=b, j=j):
                bb = [list(x) for x in blocks]
                bb[b][j] = bb[b][j] + t
                return mesh_residual(bb, w, meas, mesh, sb, se, sc)[i]
            cols.append([float(mp.diff(lambda t: fr(t, i), 0)) for i in range(3)])
        J.append([cc[i] for i in range(3) for cc in cols])
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
    with open(os.path.join(HERE, "depth_mesh_error_golden.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_golden_depth_mesh.py", "mp_dps": 50, "cases": out}, fh, indent=0)


if __name__ == "__main__":
    main()
