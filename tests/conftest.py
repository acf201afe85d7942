import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "cam_error_golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libmvba.so)")


def golden_cases():
    with open(GOLDEN) as fh:
        return json.load(fh)["cases"]


def case_problem(case, constant=None):
    """One golden case as a single-residual CamProblem (8 blocks)."""
    from multiview_amd.problem import ProblemBuilder

    pb = ProblemBuilder()
    ids = []
    for b, vals in enumerate(case["blocks"]):
        if b == 7 and len(vals) == 0:
            ids.append(pb.add_parameter_block([0.0]))  # distortion_placeholder
        else:
            ids.append(pb.add_parameter_block(vals))
    if constant:
        for b in constant:
            pb.set_parameter_block_constant(ids[b])
    if len(case["blocks"][7]) == 0:
        pb.set_parameter_block_constant(ids[7])
    h = case["half"]
    cam = pb.add_camera(len(case["blocks"][7]), (2 * h[0], 2 * h[1]))
    s = case["stamps"]
    pb.add_residual_block(case["meas"], s[0], s[1], s[2], ids, cam)
    return pb.build()


def golden_jacobian_row(case, stride):
    """Golden Jacobian in the Ceres layout (MVBA_JAC_BASE_*)."""
    from multiview_amd._lib import JAC_BASE

    J = np.zeros(stride)
    for b, blk in enumerate(case["jacobian"]):
        J[JAC_BASE[b]:JAC_BASE[b] + len(blk)] = blk
    return J


def fd_bound(problem, J_ref, pix_scale):
    """Rounding bound of the reference's central differences per column
    (Ceres 1.14 numeric_diff.h [ext]): |err| <~ eps*|pixel|/delta_j, with
    delta_j = max(sqrt(eps), 1e-6*|x_j|); plus truncation (1e-6 relative)."""
    from multiview_amd._lib import JAC_BASE

    eps = np.finfo(float).eps
    n, stride = J_ref.shape
    bound = np.zeros((n, stride))
    half = problem.camera_half_size
    for i in range(n):
        blks = problem.residual_blocks[i]
        cam = problem.residual_camera[i]
        K = int(problem.camera_dist_size[cam])
        for b in range(8):
            vals = problem.block_values(blks[b])
            size = (7, 7, 7, 3, 1, 1, 2)[b] if b < 7 else K
            for j in range(size):
                delta = max(np.sqrt(eps), 1e-6 * abs(vals[j]))
                tb = 64 * eps * max(pix_scale[i], 1.0) / delta
                for row in range(2):
                    bound[i, JAC_BASE[b] + row * size + j] = tb
        if K >= 20:
            # RPC denominator coefficient b with monomial m: f = N/D(b), so
            # f''' = -6 q (m/D)^3 with q = N/D and m/D = -J/q: truncation of the
            # central difference delta^2 |f'''| / 6 = delta^2 |J|^3 / q^2 (x2 for
            # the higher-order terms; it exceeds |J| where FD is meaningless).
            nh = K // 2
            deg = int(round(np.sqrt(2.0 * nh + 5.0) / 2.0 - 1.5))
            nl = (deg + 1) * (deg + 2) // 2
            vals = problem.block_values(blks[7])
            meas = problem.residual_meas[i]
            for row, lo in ((0, nl), (1, 3 * nl - 1)):
                r = J_ref[i]  # exact Jacobian row block
                for j in range(lo, lo + nl - 1):
                    col = JAC_BASE[7] + row * K + j
                    delta = max(np.sqrt(eps), 1e-6 * abs(vals[j]))
                    q = max(abs(meas[row] - half[cam][row]), 1.0)
                    x = delta * abs(r[col]) / q  # relative change of D over one step
                    if x > 0.02:
                        bound[i, col] = np.inf  # FD series diverges: the reference's FD column is not a derivative
                    else:
                        bound[i, col] += 3.0 * delta ** 2 * abs(r[col]) ** 3 / q ** 2
    return bound + 1e-6 * np.abs(J_ref).max(axis=0, keepdims=True)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_py

    oracle_py.load()
    return oracle_py


def have_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
