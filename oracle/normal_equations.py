"""Numpy normal equations of Ceres-layout residuals and Jacobians — TEST
INFRASTRUCTURE ONLY (importable from tests/ as the checker of
mvba_linearize_device; never from the product package).

Gradient J^T r and block-diagonal J_b^T J_b per parameter block, in the
camera-side (mvba_cam_block_map) and packed point-side layouts. Follows the
accumulation Ceres' BlockSparseMatrix / implicit Schur code performs for the
residual blocks of rig_calibrator.cc:1695-1699 [ext]."""
from __future__ import annotations

import numpy as np


def normal_equations_reference(problem, r: np.ndarray, J: np.ndarray, layout: dict):
    """Gradient J^T r and block-diagonal J_b^T J_b from Ceres-layout residuals
    and Jacobians (numpy; test reference for mvba_linearize_device)."""
    from multiview_amd._lib import JAC_BASE

    cam_g = np.zeros(layout["cam_grad_size"])
    cam_h = np.zeros(layout["cam_hess_size"])
    npts = layout["num_points"]
    pt_g = np.zeros((npts, 3))
    pt_h = np.zeros((npts, 6))
    cam_pos = {int(b): k for k, b in enumerate(layout["cam_block_ids"])}
    pt_pos = {int(b): k for k, b in enumerate(layout["point_block_ids"])}
    K_of = problem.camera_dist_size[problem.residual_camera]
    for b in range(8):
        for K in np.unique(K_of):
            sel = np.nonzero(K_of == K)[0]
            size = (7, 7, 7, 3, 1, 1, 2)[b] if b < 7 else int(K)
            if size == 0 or sel.size == 0:
                continue
            Jb = J[sel, JAC_BASE[b]:JAC_BASE[b] + 2 * size].reshape(-1, 2, size)
            gi = np.einsum("nrc,nr->nc", Jb, r[sel])
            Hi = np.einsum("nrc,nrd->ncd", Jb, Jb)
            bids = problem.residual_blocks[sel, b]
            if b == 3:
                idx = np.array([pt_pos.get(int(x), -1) for x in bids])
                ok = idx >= 0
                np.add.at(pt_g, idx[ok], gi[ok])
                packed = Hi[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
                np.add.at(pt_h, idx[ok], packed[ok])
                continue
            for n, bid in enumerate(bids):
                k = cam_pos.get(int(bid))
                if k is None:
                    continue
                go, ho = layout["cam_goff"][k], layout["cam_hoff"][k]
                cam_g[go:go + size] += gi[n]
                cam_h[ho:ho + size * size] += Hi[n].reshape(-1)
    return cam_g, cam_h, pt_g.reshape(-1), pt_h.reshape(-1)
