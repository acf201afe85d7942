"""Write a synthetic rig (multiview_amd.rig.make_rig) as rig_calibrator input files.

    out_dir/rig_config.txt        readRigConfig format (dense_map_utils.cc:940-1057)
    out_dir/cameras.nvm          NVM_V3 (interest_point.cc:1248-1331): every image
                                 with its world_to_cam, the tracks with their
                                 keypoints relative to the optical center
    out_dir/<sensor>/<t>.jpg      image names only (the calibrator never reads the
                                 pixels); <t> = repr(timestamp) so atof() of the
                                 file name returns the exact double
    out_dir/<sensor>/<t>.pc       depth clouds of ``depth_sensors`` images
                                 (readXyzImage: int32 rows, cols, channels; float32)

Inputs are the rig's perturbed initial values (``rig.init``): reference images
carry init world_to_ref, the other images init world_to_cam; the configuration
carries init intrinsics, ref_to_cam, timestamp offsets and depth_to_image.
"""
from __future__ import annotations

import os

import numpy as np

from .rig import IMAGE_SIZE, Rig, mat_to_quat, quat_to_mat


def _r(x) -> str:
    return repr(float(x))


def _aff_str(R, t) -> str:
    v = list(np.asarray(R, dtype=np.float64).reshape(-1)) + list(np.asarray(t, dtype=np.float64).reshape(-1))
    return " ".join(repr(float(x)) for x in v)


def _dist_type(k: int) -> str:
    if k == 0:
        return "no_distortion"
    if k == 1:
        return "fisheye"
    if k in (4, 5):
        return "radtan"
    return "rpc"


def image_name(out_dir: str, sensor: str, stamp: float) -> str:
    return os.path.join(out_dir, sensor, repr(float(stamp)) + ".jpg")


def write_rig_config(rig: Rig, path: str, depth_to_image=None) -> None:
    init = rig.init
    lines = [f"ref_sensor_name: {rig.sensor_names[0]}"]
    for s in range(rig.num_sensors):
        r2c = init["ref_to_cam"][s]
        dti = np.eye(4) if depth_to_image is None else depth_to_image[s]
        d = np.asarray(init["dist"][s], dtype=np.float64)
        lines += ["", f"sensor_name: {rig.sensor_names[s]}",
                  f"focal_length: {float(init['focal'][s])!r}",
                  f"optical_center: {float(init['center'][s][0])!r} {float(init['center'][s][1])!r}",
                  "distortion_coeffs: " + " ".join(repr(float(x)) for x in d),
                  f"distortion_type: {_dist_type(d.size)}",
                  f"image_size: {IMAGE_SIZE[0]} {IMAGE_SIZE[1]}",
                  f"distorted_crop_size: {IMAGE_SIZE[0]} {IMAGE_SIZE[1]}",
                  f"undistorted_image_size: {IMAGE_SIZE[0]} {IMAGE_SIZE[1]}",
                  "ref_to_sensor_transform: " + _aff_str(quat_to_mat(r2c[3:][None])[0], r2c[:3]),
                  "depth_to_image_transform: " + _aff_str(dti[:3, :3], dti[:3, 3]),
                  f"ref_to_sensor_timestamp_offset: {float(init['offsets'][s])!r}"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def init_world_to_cam(rig: Rig) -> np.ndarray:
    """[N_img, 4, 4] input poses: init world_to_ref for reference images, init
    world_to_cam for the others."""
    out = np.zeros((len(rig.cam_type), 4, 4))
    out[:, 3, 3] = 1
    for k in range(len(rig.cam_type)):
        a = rig.init["world_to_ref"][rig.cam_beg[k]] if rig.cam_type[k] == 0 else rig.init["world_to_cam"][k]
        out[k, :3, :3] = quat_to_mat(a[3:][None])[0]
        out[k, :3, 3] = a[:3]
    return out


def write_nvm(rig: Rig, path: str, names: list, w2c: np.ndarray) -> None:
    center = np.asarray(rig.init["center"], dtype=np.float64)
    focal = np.asarray(rig.init["focal"], dtype=np.float64)
    nimg = len(names)
    # keypoints per image, fid in track order
    kp = [[] for _ in range(nimg)]
    tracks = []
    pids, starts = np.unique(rig.obs_pid, return_index=True)
    ends = np.r_[starts[1:], rig.obs_pid.size]
    for p, a, b in zip(pids, starts, ends):
        if b - a < 2:
            continue
        t = []
        for o in range(a, b):
            c = int(rig.obs_cid[o])
            s = int(rig.cam_type[c])
            t.append((c, len(kp[c])))
            kp[c].append(rig.obs_pix[o] - center[s])
        tracks.append((int(p), t))
    lines = ["NVM_V3", str(nimg)]
    for k in range(nimg):
        R, t = w2c[k, :3, :3], w2c[k, :3, 3]
        # Eigen Quaterniond(R) (Shepperd), camera center -R^T t
        q = mat_to_quat(R[None])[0]  # x y z w
        C = -R.T @ t
        lines.append(f"{names[k]} {_r(focal[rig.cam_type[k]])} {_r(q[3])} {_r(q[0])} {_r(q[1])} {_r(q[2])} "
                     f"{_r(C[0])} {_r(C[1])} {_r(C[2])} 0 0")
    lines.append(str(len(tracks)))
    X = rig.init["xyz"]
    for p, t in tracks:
        meas = " ".join(f"{c} {fid} {_r(kp[c][fid][0])} {_r(kp[c][fid][1])}" for c, fid in t)
        lines.append(f"{_r(X[p][0])} {_r(X[p][1])} {_r(X[p][2])} 0 0 0 {len(t)} {meas}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_depth_clouds(rig: Rig, names: list, depth_to_image=None) -> int:
    """One float32 cloud per image of a depth sensor: at round(keypoint) the
    observed landmark in depth coordinates (depth_to_image^-1 of the camera-frame
    point, true poses, float32), zero elsewhere. Returns the number of clouds."""
    if rig.depth_obs is None or rig.depth_obs.size == 0:
        return 0
    W, H = IMAGE_SIZE
    clouds = {}
    for j, o in enumerate(rig.depth_obs):
        c = int(rig.obs_cid[o])
        if c not in clouds:
            clouds[c] = np.zeros((H, W, 3), dtype=np.float32)
        col, row = (int(np.round(v)) for v in rig.obs_pix[o])
        if 0 <= col < W and 0 <= row < H:
            clouds[c][row, col] = rig.depth_meas[j].astype(np.float32)
    for c, cloud in clouds.items():
        base = os.path.splitext(names[c])[0]
        with open(base + ".pc", "wb") as f:
            np.array([H, W, 3], dtype=np.int32).tofile(f)
            cloud.tofile(f)
    return len(clouds)


def write_dataset(rig: Rig, out_dir: str, depth_to_image=None) -> dict:
    """All inputs of one calibration run; returns the paths and image names.
    ``depth_to_image``: [N_sensor, 4, 4] written to the configuration (identity
    by default)."""
    os.makedirs(out_dir, exist_ok=True)
    for n in rig.sensor_names:
        os.makedirs(os.path.join(out_dir, n), exist_ok=True)
    names = [image_name(out_dir, rig.sensor_names[int(s)], st) for s, st in zip(rig.cam_type, rig.cam_stamp)]
    cfg = os.path.join(out_dir, "rig_config.txt")
    nvm = os.path.join(out_dir, "cameras.nvm")
    write_rig_config(rig, cfg, depth_to_image)
    write_nvm(rig, nvm, names, init_world_to_cam(rig))
    nclouds = write_depth_clouds(rig, names, depth_to_image)
    return {"rig_config": cfg, "nvm": nvm, "images": names, "num_clouds": nclouds}


def write_ply(path: str, vertices, faces, binary: bool = True) -> None:
    """A triangle mesh as PLY (what --mesh reads, mve::geom::load_ply_mesh):
    float x y z per vertex, "list uchar int vertex_indices" per face."""
    V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    F = np.ascontiguousarray(faces, dtype=np.int64).reshape(-1, 3)
    head = ("ply\nformat {} 1.0\nelement vertex {}\nproperty float x\nproperty float y\nproperty float z\n"
            "element face {}\nproperty list uchar int vertex_indices\nend_header\n").format(
                "binary_little_endian" if binary else "ascii", V.shape[0], F.shape[0])
    with open(path, "wb") as f:
        f.write(head.encode())
        if binary:
            f.write(V.astype("<f4").tobytes())
            rec = np.zeros(F.shape[0], dtype=[("n", "u1"), ("v", "<i4", 3)])
            rec["n"] = 3
            rec["v"] = F
            f.write(rec.tobytes())
        else:
            for v in V:
                f.write(("%.9g %.9g %.9g\n" % tuple(v)).encode())
            for q in F:
                f.write(("3 %d %d %d\n" % tuple(q)).encode())
