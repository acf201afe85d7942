import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "cam_error_golden.json")


def pytest_sessionstart(session):
    # Bring up torch's HIP runtime before any test spawns worker processes: a
    # parent that used the GPU only through libmvba could not initialise torch's
    # runtime after mp.spawn children had run (seen on the MI355X box).
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # noqa: BLE001 - CPU container: nothing to do
        pass


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


def fd_bound(problem, J_ref, r_ref):
    """Error bound of the reference's central differences per Jacobian entry
    (Ceres 1.14 numeric_diff.h [ext]) with delta_j = max(sqrt(eps), 1e-6*|x_j|):
      * rounding: 64 eps |pixel| / delta_j;
      * RPC denominator coefficient b (monomial m): the residual is EXACTLY
        N / (D0 + b m) in b, whose central difference equals the derivative
        times 1 / (1 - x^2), x = delta m / D = delta |J| / |q|, q = N/D. So the
        FD error is |J| x^2 / (1 - x^2); for x >= 0.5 the FD column is not a
        derivative and the entry is not compared (bound = inf);
      * 1e-6 of the column maximum for everything else (truncation)."""
    from multiview_amd._lib import JAC_BASE

    eps = np.finfo(float).eps
    n, stride = J_ref.shape
    bound = np.zeros((n, stride))
    half = problem.camera_half_size
    pix = np.maximum(np.abs(problem.residual_meas + r_ref).max(axis=1), 1.0)
    for i in range(n):
        blks = problem.residual_blocks[i]
        cam = problem.residual_camera[i]
        K = int(problem.camera_dist_size[cam])
        for b in range(8):
            vals = problem.block_values(blks[b])
            size = (7, 7, 7, 3, 1, 1, 2)[b] if b < 7 else K
            for j in range(size):
                delta = max(np.sqrt(eps), 1e-6 * abs(vals[j]))
                tb = 64 * eps * pix[i] / delta
                for row in range(2):
                    bound[i, JAC_BASE[b] + row * size + j] = tb
        if K >= 20:
            nh = K // 2
            deg = int(round(np.sqrt(2.0 * nh + 5.0) / 2.0 - 1.5))
            nl = (deg + 1) * (deg + 2) // 2
            vals = problem.block_values(blks[7])
            for row, lo in ((0, nl), (1, 3 * nl - 1)):
                q = abs(r_ref[i, row] + problem.residual_meas[i, row] - half[cam][row])
                for j in range(lo, lo + nl - 1):
                    col = JAC_BASE[7] + row * K + j
                    delta = max(np.sqrt(eps), 1e-6 * abs(vals[j]))
                    x = delta * abs(J_ref[i, col]) / max(q, 1e-300)
                    if x >= 0.5:
                        bound[i, col] = np.inf
                    else:
                        bound[i, col] += 1.01 * abs(J_ref[i, col]) * x * x / (1.0 - x * x)
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
