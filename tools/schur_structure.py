#!/usr/bin/env python3
"""Structure of the reduced camera system S = F'F - F'E (E'E)^-1 E'F of a
BASELINE config (DESIGN.md §5 "Why the reduced camera system is not formed",
row X1), from the problem topology alone (no GPU):

* D: camera-side unknowns (free non-point blocks referenced by residuals);
* per point, m_p = the camera-side columns its observations touch; forming S
  scatters m_p^2 / 2 entry updates (symmetric half) and costs 2 * 3 * m_p^2
  flop for G_p^T G_p with G_p = L_p^-1 E_p^T F_p (3 x m_p, sparse columns);
* S's pattern: with the shared blocks (ref_to_cam, offsets, intrinsics:
  coupled to every pose) ordered last, the pose part is banded (a point's
  observers lie within +-window reference frames); a band + dense border
  Cholesky costs about sum_i w_i^2 (w_i = envelope width of row i) plus the
  border's n * B^2 + B^3 / 3, against D^3 / 3 dense.

    python3 tools/schur_structure.py [config] [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multiview_amd import rig  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    R = rig.make_rig(**rig.CONFIGS[cfg])
    P = rig.build_problem(R, rig.FloatFlags(**rig.CONFIG_FLAGS.get(cfg, {})))
    rb = P.residual_blocks
    free = P.block_constant == 0
    size = P.block_size.astype(np.int64)
    cam_cols = [0, 1, 2, 4, 5, 6, 7]  # beg, end, ref_to_cam, offset, focal, center, distortion
    used = np.zeros(len(size), dtype=bool)
    for c in cam_cols:
        used[rb[:, c]] = True
    cam = used & free
    cam[rb[:, 3]] = False
    D = int(size[cam].sum())
    # pose blocks (world_to_ref, one per reference frame) vs shared blocks
    pose_ids = np.unique(np.concatenate([rb[:, 0], rb[:, 1]]))
    pose_ids = pose_ids[cam[pose_ids]]
    is_pose = np.zeros(len(size), dtype=bool)
    is_pose[pose_ids] = True
    border = cam & ~is_pose
    B = int(size[border].sum())
    # per point: camera columns touched (unique free blocks of its observations)
    pid = rb[:, 3]
    order = np.argsort(pid, kind="stable")
    pid_s = pid[order]
    starts = np.flatnonzero(np.r_[True, pid_s[1:] != pid_s[:-1]])
    ends = np.r_[starts[1:], pid_s.size]
    m = np.zeros(starts.size, dtype=np.int64)
    pose_rank = np.full(len(size), -1, dtype=np.int64)
    pose_rank[pose_ids] = np.arange(pose_ids.size)
    lo_r = np.zeros(starts.size, dtype=np.int64)
    hi_r = np.zeros(starts.size, dtype=np.int64)
    blocks = rb[order][:, cam_cols]
    for k, (a, b) in enumerate(zip(starts, ends)):
        u = np.unique(blocks[a:b])
        u = u[cam[u]]
        m[k] = size[u].sum()
        pr = pose_rank[u]
        pr = pr[pr >= 0]
        lo_r[k], hi_r[k] = (pr.min(), pr.max()) if pr.size else (0, 0)
    scatter = float((m * (m + 1) // 2).sum())
    syrk = float((6 * m * m).sum())
    # envelope of the pose part in reference-frame units: row r's first partner
    npose = pose_ids.size
    first = np.arange(npose)
    np.minimum.at(first, hi_r, lo_r)
    first = np.minimum.accumulate(first[::-1])[::-1]  # an envelope is monotone
    w_ref = np.arange(npose) - first                  # partners below, in frames
    # scalar envelope widths (7 scalars per pose block)
    ps = size[pose_ids]
    w_scalar = np.repeat(w_ref * 7, ps) + np.tile(np.arange(7), npose)[: int(ps.sum())]
    band_flops = float((w_scalar.astype(np.float64) ** 2).sum())
    n_pose = int(ps.sum())
    border_flops = 2.0 * n_pose * B * B + (w_scalar.astype(np.float64) * B * 2).sum() + B ** 3 / 3.0
    res = {
        "config": cfg, "num_points": int(starts.size), "num_observations": int(pid.size),
        "camera_side_unknowns_D": D, "pose_unknowns": n_pose, "shared_unknowns_border": B,
        "dense_S_bytes": 8.0 * D * D, "dense_cholesky_flop": D ** 3 / 3.0,
        "columns_per_point": {"mean": float(m.mean()), "max": int(m.max()), "p50": float(np.median(m))},
        "form_S_entry_updates": scatter, "form_S_flop_sparse_Gp": syrk,
        "pose_band_halfwidth_frames": {"max": int(w_ref.max()), "mean": float(w_ref.mean())},
        "S_nonzeros_band_plus_border": float(2 * w_scalar.sum() + n_pose + 2 * n_pose * B + B * B),
        "band_plus_border_cholesky_flop": band_flops + border_flops,
        "note": "shared blocks (ref_to_cam, offsets, focal, centre, distortion) ordered last; the pose part's "
                "envelope from each point's first and last observing reference frame",
    }
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
