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
    for i in range(n):
        blks = problem.residual_blocks[i]
        for b in range(8):
            vals = problem.block_values(blks[b])
            size = len(vals) if b == 7 else (7, 7, 7, 3, 1, 1, 2)[b]
            if b == 7:
                size = int(problem.camera_dist_size[problem.residual_camera[i]])
            for j in range(size):
                delta = max(np.sqrt(eps), 1e-6 * abs(vals[j]))
                tb = 64 * eps * max(pix_scale[i], 1.0) / delta
                for row in range(2):
                    bound[i, JAC_BASE[b] + row * size + j] = tb
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
