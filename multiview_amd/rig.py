"""Deterministic synthetic rigs and the rig_calibrator problem
assembly over them (rig_calibrator.cc:1614-1752).

A rig has N_s sensors; sensor 0 is the reference sensor. Reference poses follow a
circle of radius 8 m looking at the origin (0.5 deg per frame, 1 deg jitter);
reference timestamps are 1.6e9 + 0.5 j s. A non-reference sensor s has clock
offset 0.01 s, an extrinsic yaw and a lateral offset, and one image per
reference interval at its own time t_j + 0.25 + offset_s, bracketed by
reference frames j and j+1 (dense_map_utils.cc:1441-1658 would select exactly
these brackets). Landmarks are uniform in a 4 m ball; each is observed by images
near an anchor time, so that a frame's points are spatially coherent as in a real
sequence. Pixels are projected with the true parameters, perturbed by N(0, 0.5^2)
px and rounded to float32 (keypoints are std::pair<float, float>,
rig_calibrator.cc:1672). Initial values are the truth perturbed by 1 cm / 0.1 deg
(poses), 2 cm (points) and 0.5 % (focal length).

The synthetic data stand in for the NVM/rig_config inputs of a real run (no
dataset is available offline); see DESIGN.md "Workloads".
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .problem import CamProblem, rpc_num_dist_params

IMAGE_SIZE = (1024, 768)
FOCAL = 600.0
CENTER = (515.0, 382.0)
RADTAN = (-0.25, 0.07, 1e-3, -5e-4, 0.0)
FOV_W = 0.9


# ------------------------------------------------------------------ rotations
def rot_axis(axis: str, ang: np.ndarray) -> np.ndarray:
    ang = np.asarray(ang, dtype=np.float64)
    c, s = np.cos(ang), np.sin(ang)
    o, z = np.ones_like(ang), np.zeros_like(ang)
    if axis == "x":
        m = [[o, z, z], [z, c, -s], [z, s, c]]
    elif axis == "y":
        m = [[c, z, s], [z, o, z], [-s, z, c]]
    else:
        m = [[c, -s, z], [s, c, z], [z, z, o]]
    return np.moveaxis(np.array(m), (0, 1), (-2, -1))


def small_rot(rng, n: int, sigma_rad: float) -> np.ndarray:
    v = rng.normal(0.0, sigma_rad, size=(n, 3))
    th = np.linalg.norm(v, axis=1)
    k = v / np.maximum(th, 1e-300)[:, None]
    K = np.zeros((n, 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -k[:, 2], k[:, 1]
    K[:, 1, 0], K[:, 1, 2] = k[:, 2], -k[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -k[:, 1], k[:, 0]
    s, c = np.sin(th)[:, None, None], np.cos(th)[:, None, None]
    return np.eye(3)[None] + s * K + (1 - c) * (K @ K)


def mat_to_quat(R: np.ndarray) -> np.ndarray:
    """Rotation matrices [n,3,3] -> quaternions [n,4] as (x, y, z, w), w >= 0."""
    R = np.asarray(R)
    n = R.shape[0]
    q = np.zeros((n, 4))
    tr = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]
    for i in range(n):
        m = R[i]
        if tr[i] > 0:
            t = np.sqrt(tr[i] + 1.0)
            w = 0.5 * t
            t = 0.5 / t
            q[i] = [(m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w]
        else:
            a = int(np.argmax([m[0, 0], m[1, 1], m[2, 2]]))
            b, c = (a + 1) % 3, (a + 2) % 3
            t = np.sqrt(m[a, a] - m[b, b] - m[c, c] + 1.0)
            v = np.zeros(4)
            v[a] = 0.5 * t
            t = 0.5 / t
            v[3] = (m[c, b] - m[b, c]) * t
            v[b] = (m[b, a] + m[a, b]) * t
            v[c] = (m[c, a] + m[a, c]) * t
            q[i] = v
    q *= np.where(q[:, 3:4] < 0, -1.0, 1.0)
    return q


def quat_to_mat(q: np.ndarray) -> np.ndarray:
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = 1 - 2 * (y * y + z * z)
    R[..., 0, 1] = 2 * (x * y - z * w)
    R[..., 0, 2] = 2 * (x * z + y * w)
    R[..., 1, 0] = 2 * (x * y + z * w)
    R[..., 1, 1] = 1 - 2 * (x * x + z * z)
    R[..., 1, 2] = 2 * (y * z - x * w)
    R[..., 2, 0] = 2 * (x * z - y * w)
    R[..., 2, 1] = 2 * (y * z + x * w)
    R[..., 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def slerp(q0: np.ndarray, q1: np.ndarray, a: np.ndarray) -> np.ndarray:
    d = np.sum(q0 * q1, axis=-1)
    s = np.where(d < 0, -1.0, 1.0)
    ad = np.abs(d)
    th = np.arccos(np.clip(ad, -1, 1))
    st = np.sin(th)
    lin = ad >= 1 - np.finfo(float).eps
    w0 = np.where(lin, 1 - a, np.sin((1 - a) * th) / np.where(lin, 1, st))
    w1 = np.where(lin, a, np.sin(a * th) / np.where(lin, 1, st)) * s
    return w0[..., None] * q0 + w1[..., None] * q1


# ------------------------------------------------------------------ distortion
def distort(model: str, k: np.ndarray, u: np.ndarray, f: float, c, h) -> np.ndarray:
    """Vectorised DistortCentered + half size (camera_params.cc:260-314) used only
    to SYNTHESISE measurements; the evaluator parity is checked by the oracle."""
    c = np.asarray(c, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    if model == "none":
        return u + c
    if model == "fov":
        w = k[0]
        m = u / f
        ru = np.linalg.norm(m, axis=1)
        rd = np.arctan(ru * 2 * np.tan(w / 2)) / w
        conv = np.where(ru > 1e-5, rd / np.maximum(ru, 1e-300), 1.0)
        return c + conv[:, None] * m * f
    if model == "radtan":
        k1, k2, p1, p2 = k[:4]
        k3 = k[4] if len(k) > 4 else 0.0
        m = u / f
        r2 = np.sum(m * m, axis=1)
        rad = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
        e = rad[:, None] * m
        e[:, 0] += 2 * p1 * m[:, 0] * m[:, 1] + p2 * (r2 + 2 * m[:, 0] ** 2)
        e[:, 1] += p1 * (r2 + 2 * m[:, 1] ** 2) + 2 * p2 * m[:, 0] * m[:, 1]
        return e * f + c
    if model.startswith("rpc"):
        deg = int(model[3:])
        n = len(k) // 2
        coef = k[:n]
        nl = (deg + 1) * (deg + 2) // 2
        x, y = u[:, 0], u[:, 1]
        mono = [x ** (dg - i) * y ** i for dg in range(deg + 1) for i in range(dg + 1)]
        ci = 0
        vals = []
        for cnt in range(4):
            start = cnt & 1
            acc = np.full(x.shape, 1.0 if start else 0.0)
            for j, mo in enumerate(mono):
                if start and j == 0:
                    continue
                acc = acc + coef[ci] * mo
                ci += 1
            vals.append(acc)
        assert ci == n and nl
        return np.stack([vals[0] / vals[1], vals[2] / vals[3]], axis=1) + h
    raise ValueError(model)


def model_dist_size(model: str) -> int:
    if model == "none":
        return 0
    if model == "fov":
        return 1
    if model == "radtan":
        return 5
    if model == "radtan4":
        return 4
    if model.startswith("rpc"):
        return 2 * rpc_num_dist_params(int(model[3:]))
    raise ValueError(model)


def default_coeffs(model: str, rng) -> np.ndarray:
    if model == "none":
        return np.zeros(0)
    if model == "fov":
        return np.array([FOV_W])
    if model == "radtan":
        return np.array(RADTAN)
    if model == "radtan4":
        return np.array(RADTAN[:4])
    if model.startswith("rpc"):
        deg = int(model[3:])
        n = rpc_num_dist_params(deg)
        nl = (deg + 1) * (deg + 2) // 2
        # Identity (rpc_distortion.cc:303-318) perturbed: numerator coefficient of a
        # degree-d monomial sigma 1e-3 * 512^(1-d), denominator 1e-4 * 512^-d.
        degs = [dg for dg in range(deg + 1) for _ in range(dg + 1)]
        half = []
        for cnt in range(4):
            start = cnt & 1
            for j, dg in enumerate(degs):
                if start and j == 0:
                    continue
                if start:
                    half.append(rng.normal(0, 1e-4 * 512.0 ** (-dg)))
                else:
                    half.append(rng.normal(0, 1e-3 * 512.0 ** (1 - dg)))
        half = np.array(half)
        # identity: num_x[1] (x) = 1, num_y[2] (y) = 1
        half[1] += 1.0
        half[nl + (nl - 1) + 2] += 1.0
        assert half.size == n
        return np.concatenate([half, half])  # undistortion half = distortion half
    raise ValueError(model)


# ------------------------------------------------------------------ the rig
@dataclass
class Rig:
    sensor_models: list
    ref_stamps: np.ndarray            # [N_ref]
    offsets: np.ndarray               # [N_s] ref_to_cam timestamp offsets
    world_to_ref: np.ndarray          # [N_ref, 7] true
    ref_to_cam: np.ndarray            # [N_s, 7] true
    focal: np.ndarray                 # [N_s]
    center: np.ndarray                # [N_s, 2]
    dist: list                        # [N_s] arrays
    cam_type: np.ndarray              # [N_img]
    cam_beg: np.ndarray               # [N_img]
    cam_end: np.ndarray               # [N_img]
    cam_stamp: np.ndarray             # [N_img]
    world_to_cam: np.ndarray          # [N_img, 7] true (for --no_rig)
    xyz: np.ndarray                   # [N_pts, 3] true
    obs_pid: np.ndarray               # [N_obs] sorted by (pid, cid)
    obs_cid: np.ndarray
    obs_pix: np.ndarray               # [N_obs, 2] float32-rounded measurements
    init: dict = field(default_factory=dict)  # perturbed initial values
    sensor_names: list = field(default_factory=list)
    # depth clouds (config c5): per observation of a depth sensor, the cloud point
    depth_obs: np.ndarray = None      # [N_d] indices into obs_* (observations with depth)
    depth_meas: np.ndarray = None     # [N_d, 3] float32-rounded depth-cloud points
    depth_to_image: np.ndarray = None  # [N_s, 7 | 12] true depth_to_image per sensor

    @property
    def num_sensors(self):
        return len(self.sensor_models)


def _pose_arrays(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    return np.concatenate([t, mat_to_quat(R)], axis=1)


def _sensor_yaw_deg(s: int, n_s: int) -> float:
    if n_s <= 3:
        return 15.0 * s
    # more sensors: alternate around the reference direction so all see the scene
    return 10.0 * ((s + 1) // 2) * (1.0 if s % 2 else -1.0)


def make_rig(num_sensors=3, num_ref=50, num_points=1000, obs_per_point=5.0, models=None,
             seed=1001, point_range=None, window=20, noise_px=0.5, depth_sensors=(),
             depth_noise=0.01, affine_depth=False, surface=None, alpha_shift=0.0) -> Rig:
    """Build a synthetic rig. ``point_range=(lo, hi)`` generates only points
    [lo, hi) of a larger problem (landmark-range sharding): the
    cameras are identical on every shard, points use a per-shard stream.
    ``depth_sensors``: sensors that also carry a depth cloud (config c5); every
    observation of such a sensor gets the cloud point of its landmark,
    depth_to_image^-1 (X_cam) + N(0, depth_noise^2), rounded to float32 (clouds
    are float32, dense_map_utils.cc:1382). ``surface="sphere"``: landmarks on the
    sphere of radius SPHERE_RADIUS (the surface ``sphere_mesh`` triangulates, for
    the --mesh constraints), observed only by cameras on their outer side.
    ``alpha_shift``: the bracketed images' true poses are interpolated at
    alpha + alpha_shift (extrapolated past the bracket when the sum leaves
    [0, 1]) while their timestamps stay put, so the offset that explains the
    data lies outside the bracket (a test rig for the interpolation range check,
    rig_calibrator.cc:346)."""
    models = list(models or ["radtan"] * num_sensors)
    assert len(models) == num_sensors
    rng = np.random.default_rng(seed)
    ns, nr = num_sensors, num_ref
    ref_stamps = 1.6e9 + 0.5 * np.arange(nr)
    offsets = np.array([0.0] + [0.01 * s for s in range(1, ns)])

    # reference trajectory
    phi = np.deg2rad(0.5) * np.arange(nr)
    C = np.stack([8 * np.cos(phi), 0.3 * np.sin(3 * phi), 8 * np.sin(phi)], axis=1)
    fwd = -C / np.linalg.norm(C, axis=1, keepdims=True)
    up = np.array([0.0, 1.0, 0.0])
    xc = np.cross(up, fwd)
    xc /= np.linalg.norm(xc, axis=1, keepdims=True)
    yc = np.cross(fwd, xc)
    Rc2w = np.stack([xc, yc, fwd], axis=2)
    Rc2w = Rc2w @ small_rot(rng, nr, np.deg2rad(1.0))
    Rw2r = np.transpose(Rc2w, (0, 2, 1))
    tw2r = -np.einsum("nij,nj->ni", Rw2r, C)
    world_to_ref = _pose_arrays(Rw2r, tw2r)

    Rr2c = np.stack([rot_axis("y", np.deg2rad(_sensor_yaw_deg(s, ns))) for s in range(ns)])
    tr2c = np.array([[0.1 * s, 0.0, 0.0] for s in range(ns)])
    ref_to_cam = _pose_arrays(Rr2c, tr2c)
    ref_to_cam[0] = [0, 0, 0, 0, 0, 0, 1]

    focal = np.full(ns, FOCAL)
    center = np.tile(np.array(CENTER), (ns, 1))
    dist = [default_coeffs(m, rng) for m in models]

    # images (lookupImagesAndBrackets order: by ref index, then sensor)
    cam_type, cam_beg, cam_end, cam_stamp = [], [], [], []
    for j in range(nr):
        for s in range(ns):
            if s == 0:
                cam_type.append(0); cam_beg.append(j); cam_end.append(j); cam_stamp.append(ref_stamps[j])
            elif j + 1 < nr:
                cam_type.append(s); cam_beg.append(j); cam_end.append(j + 1)
                cam_stamp.append(ref_stamps[j] + 0.25 + offsets[s])
    cam_type = np.array(cam_type, dtype=np.int32)
    cam_beg = np.array(cam_beg, dtype=np.int32)
    cam_end = np.array(cam_end, dtype=np.int32)
    cam_stamp = np.array(cam_stamp)
    nimg = len(cam_type)

    # true world_to_cam per image (interpolation + extrinsics)
    alpha = np.where(cam_beg == cam_end, 0.0,
                     ((cam_stamp - ref_stamps[cam_beg]) - offsets[cam_type]) /
                     np.where(cam_beg == cam_end, 1.0, ref_stamps[cam_end] - ref_stamps[cam_beg]))
    alpha = np.where(cam_beg == cam_end, alpha, alpha + alpha_shift)
    q0, q1 = world_to_ref[cam_beg, 3:], world_to_ref[cam_end, 3:]
    qi = slerp(q0, q1, alpha)
    Ri = quat_to_mat(qi)
    ti = (1 - alpha)[:, None] * world_to_ref[cam_beg, :3] + alpha[:, None] * world_to_ref[cam_end, :3]
    Rc = np.einsum("nij,njk->nik", Rr2c[cam_type], Ri)
    tc = np.einsum("nij,nj->ni", Rr2c[cam_type], ti) + tr2c[cam_type]
    ref_img = cam_type == 0
    Rc[ref_img] = quat_to_mat(world_to_ref[cam_beg[ref_img], 3:])
    tc[ref_img] = world_to_ref[cam_beg[ref_img], :3]
    world_to_cam = _pose_arrays(Rc, tc)

    # landmarks
    lo, hi = (0, num_points) if point_range is None else point_range
    prng = np.random.default_rng([seed, lo, hi])
    npts = hi - lo
    v = prng.normal(size=(npts, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    if surface == "sphere":
        xyz = SPHERE_RADIUS * v
    elif surface is None:
        xyz = 4.0 * v * prng.random(npts)[:, None] ** (1 / 3)
    else:
        raise ValueError(surface)

    # observations: candidates near an anchor reference index
    cid_of = -np.ones((nr, ns), dtype=np.int64)
    cid_of[cam_beg, cam_type] = np.arange(nimg)
    n_target = int(round(obs_per_point))
    frac = obs_per_point - int(obs_per_point)
    ncand = max(2 * n_target + 4, 8)
    anchor = prng.integers(0, nr, size=npts)
    dj = prng.integers(-window, window + 1, size=(npts, ncand))
    js = np.clip(anchor[:, None] + dj, 0, nr - 1)
    ss = prng.integers(0, ns, size=(npts, ncand))
    cand = cid_of[js, ss]
    # project candidates with the true model
    P = np.repeat(np.arange(npts), ncand)
    Cf = cand.reshape(-1)
    ok = Cf >= 0
    Cs = np.where(ok, Cf, 0)
    Xc = np.einsum("nij,nj->ni", Rc[Cs], xyz[P]) + tc[Cs]
    z = Xc[:, 2]
    pix = np.zeros((P.size, 2))
    ok &= z > 0.5
    if surface == "sphere":
        # visible side only, away from the silhouette: the viewing ray meets the
        # surface normal at less than ~72 degrees
        Cw = -np.einsum("nji,nj->ni", Rc[Cs], tc[Cs])
        ray = Cw - xyz[P]
        ok &= np.einsum("ni,ni->n", ray, xyz[P]) > 0.3 * SPHERE_RADIUS * np.linalg.norm(ray, axis=1)
    for s in range(ns):
        sel = ok & (cam_type[Cs] == s)
        if not sel.any():
            continue
        u = FOCAL * (Xc[sel, :2] / Xc[sel, 2:3])
        h = np.array(IMAGE_SIZE, dtype=np.float64) / 2.0
        pix[sel] = distort(models[s] if models[s] != "radtan4" else "radtan", dist[s], u,
                           focal[s], center[s] if not models[s].startswith("rpc") else h, h)
    ok &= (pix[:, 0] >= 1) & (pix[:, 0] < IMAGE_SIZE[0] - 1) & (pix[:, 1] >= 1) & (pix[:, 1] < IMAGE_SIZE[1] - 1)
    ok = ok.reshape(npts, ncand)
    # unique images per point, first n_target valid (vectorised dedupe)
    candv = np.where(ok, cand, -1)
    srt = np.sort(candv, axis=1)
    dup = np.zeros_like(ok)
    dup[:, 1:] = srt[:, 1:] == srt[:, :-1]
    valid = (srt >= 0) & ~dup
    keep_n = np.full(npts, n_target) + (prng.random(npts) < frac)
    # keep a random subset: shuffle valid columns by random key
    key = np.where(valid, prng.random(valid.shape), 2.0)
    order = np.argsort(key, axis=1)
    rank = np.empty_like(order)
    np.put_along_axis(rank, order, np.arange(ncand)[None, :].repeat(npts, 0), axis=1)
    take = valid & (rank < keep_n[:, None])
    # need >= 2 observations per track (appendMatchesFromNvm keeps tracks with >= 2)
    good = take.sum(axis=1) >= 2
    take &= good[:, None]
    pidx, col = np.nonzero(take)
    obs_pid = pidx.astype(np.int64)
    obs_cid = srt[pidx, col]
    # order by (pid, cid): std::map<int,int> iteration order of pid_to_cid_fid
    o = np.lexsort((obs_cid, obs_pid))
    obs_pid, obs_cid = obs_pid[o], obs_cid[o]
    # measured pixels: recompute for kept observations + noise, float32 rounding
    Xo = np.einsum("nij,nj->ni", Rc[obs_cid], xyz[obs_pid]) + tc[obs_cid]
    pix_o = np.zeros((obs_pid.size, 2))
    h = np.array(IMAGE_SIZE, dtype=np.float64) / 2.0
    for s in range(ns):
        sel = cam_type[obs_cid] == s
        if not sel.any():
            continue
        u = FOCAL * (Xo[sel, :2] / Xo[sel, 2:3])
        m = models[s] if models[s] != "radtan4" else "radtan"
        pix_o[sel] = distort(m, dist[s], u, focal[s], center[s] if not m.startswith("rpc") else h, h)
    pix_o += prng.normal(0, noise_px, size=pix_o.shape)
    obs_pix = pix_o.astype(np.float32).astype(np.float64)

    # perturbed initial values
    irng = np.random.default_rng([seed, 7])
    init = {}
    dR = small_rot(irng, nr, np.deg2rad(0.1))
    init["world_to_ref"] = _pose_arrays(np.einsum("nij,njk->nik", dR, Rw2r),
                                        tw2r + irng.normal(0, 0.01, size=(nr, 3)))
    dRc = small_rot(irng, ns, np.deg2rad(0.1))
    init["ref_to_cam"] = _pose_arrays(np.einsum("nij,njk->nik", dRc, Rr2c),
                                      tr2c + irng.normal(0, 0.01, size=(ns, 3)))
    init["ref_to_cam"][0] = [0, 0, 0, 0, 0, 0, 1]
    dRw = small_rot(irng, nimg, np.deg2rad(0.1))
    init["world_to_cam"] = _pose_arrays(np.einsum("nij,njk->nik", dRw, Rc),
                                        tc + irng.normal(0, 0.01, size=(nimg, 3)))
    xrng = np.random.default_rng([seed, 11, lo, hi])
    init["xyz"] = xyz + xrng.normal(0, 0.02, size=xyz.shape)
    init["focal"] = focal * (1 + irng.normal(0, 0.005, size=ns))
    init["center"] = center.copy()
    init["dist"] = [d.copy() for d in dist]
    init["offsets"] = offsets.copy()

    # depth clouds: true depth_to_image per sensor (small rotation + offset), scale 1
    drng = np.random.default_rng([seed, 13])
    nd_par = 12 if affine_depth else 7
    dti_true = np.zeros((ns, nd_par))
    dti_init = np.zeros((ns, nd_par))
    Rd = small_rot(drng, ns, np.deg2rad(2.0))
    td = np.array([0.05, -0.02, 0.01]) + drng.normal(0, 0.01, size=(ns, 3))
    dRd = small_rot(irng, ns, np.deg2rad(0.1))
    tdi = td + irng.normal(0, 0.01, size=(ns, 3))
    for s_ in range(ns):
        if affine_depth:
            dti_true[s_] = np.concatenate([Rd[s_], td[s_][:, None]], axis=1).reshape(-1)
            dti_init[s_] = np.concatenate([dRd[s_] @ Rd[s_], tdi[s_][:, None]], axis=1).reshape(-1)
        else:
            dti_true[s_] = np.r_[td[s_], mat_to_quat(Rd[s_][None])[0]]
            dti_init[s_] = np.r_[tdi[s_], mat_to_quat((dRd[s_] @ Rd[s_])[None])[0]]
    init["depth_to_image"] = dti_init
    init["depth_scale"] = np.ones(ns)
    dsel = np.nonzero(np.isin(cam_type[obs_cid], np.asarray(depth_sensors, dtype=np.int64)))[0]
    dt = cam_type[obs_cid[dsel]]
    Xc_d = Xo[dsel]
    # meas = dti^-1 (X_cam) = R_d^T (X_cam - t_d)
    dmeas = np.einsum("nji,nj->ni", Rd[dt], Xc_d - td[dt])
    dmeas += np.random.default_rng([seed, 17, lo, hi]).normal(0, depth_noise, size=dmeas.shape)
    dmeas = dmeas.astype(np.float32).astype(np.float64)

    names = ["ref_cam"] + [f"cam{s}" for s in range(1, ns)]
    return Rig(sensor_models=models, ref_stamps=ref_stamps, offsets=offsets,
               world_to_ref=world_to_ref, ref_to_cam=ref_to_cam, focal=focal, center=center,
               dist=dist, cam_type=cam_type, cam_beg=cam_beg, cam_end=cam_end,
               cam_stamp=cam_stamp, world_to_cam=world_to_cam, xyz=xyz, obs_pid=obs_pid,
               obs_cid=obs_cid, obs_pix=obs_pix, init=init, sensor_names=names,
               depth_obs=dsel, depth_meas=dmeas, depth_to_image=dti_true)


SPHERE_RADIUS = 4.0


def shard_points(R: Rig, rank: int, world: int) -> Rig:
    """Rank's landmark-range shard of ``R`` in capture order:
    landmarks ordered by the capture time of their first observation (then by
    id), cut into ``world`` contiguous ranges of equal observation count. A
    shard keeps every camera and the observations of its landmarks, relabelled
    0..k-1 in id order (pid-major order is kept). Contiguous ranges of the
    user's ids would give every shard observations in every image; ranges in
    capture order give each shard the images of one stretch of the trajectory
    (plus the tracks' reach), so its per-image work shrinks with the split too."""
    import dataclasses

    npts = len(R.xyz)
    first = np.full(npts, np.inf)
    np.minimum.at(first, R.obs_pid, R.cam_stamp[R.obs_cid])
    order = np.lexsort((np.arange(npts), first))
    cum = np.cumsum(np.bincount(R.obs_pid, minlength=npts)[order])
    tot = int(cum[-1]) if npts else 0
    cuts = [0] + [int(np.searchsorted(cum, tot * r // world, side="right")) for r in range(1, world)] + [npts]
    sel = np.sort(order[cuts[rank]:cuts[rank + 1]])
    newid = -np.ones(npts, dtype=np.int64)
    newid[sel] = np.arange(sel.size)
    keep = newid[R.obs_pid] >= 0
    init = dict(R.init)
    init["xyz"] = R.init["xyz"][sel]
    depth_obs, depth_meas = R.depth_obs, R.depth_meas
    if depth_obs is not None:
        obs_new = np.cumsum(keep) - 1
        dk = keep[depth_obs]
        depth_obs, depth_meas = obs_new[depth_obs[dk]], depth_meas[dk]
    return dataclasses.replace(R, xyz=R.xyz[sel], obs_pid=newid[R.obs_pid[keep]], obs_cid=R.obs_cid[keep],
                               obs_pix=R.obs_pix[keep], init=init, depth_obs=depth_obs, depth_meas=depth_meas)


def sphere_mesh(subdiv: int = 5, radius: float = SPHERE_RADIUS):
    """Icosphere (float32 vertices on the sphere, uint32 faces, outward winding):
    the synthetic stand-in for the --mesh PLY of a scene with surface="sphere"."""
    t = (1.0 + 5.0 ** 0.5) / 2.0
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    verts = [np.array(v, dtype=np.float64) / np.linalg.norm(v) for v in V]
    for _ in range(subdiv):
        mid = {}
        nf = []

        def m(a, b):
            k = (min(a, b), max(a, b))
            if k not in mid:
                x = verts[a] + verts[b]
                verts.append(x / np.linalg.norm(x))
                mid[k] = len(verts) - 1
            return mid[k]
        for a, b, c in F:
            ab, bc, ca = m(a, b), m(b, c), m(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        F = nf
    return (radius * np.array(verts)).astype(np.float32), np.array(F, dtype=np.uint32)


# ------------------------------------------------------------ problem assembly
@dataclass
class FloatFlags:
    """The hot-path flags of rig_calibrator.cc:135-316 that shape the problem."""
    camera_poses_to_float: tuple = ("ref_cam",)
    rig_transforms_to_float: tuple = ("*",)      # "*" = every non-reference sensor
    intrinsics_to_float: tuple = ("focal_length", "optical_center", "distortion")
    float_timestamp_offsets: bool = True
    no_rig: bool = False
    # depth (rig_calibrator.cc:1755-1791)
    depth_tri_weight: float = 0.0
    depth_to_image_transforms_to_float: tuple = ()
    float_scale: bool = False
    affine_depth_to_image: bool = False
    # XYZError prior on every point (rig_calibrator.cc:1889-1898)
    tri_weight: float = 0.0
    tri_robust_threshold: float = 0.0
    # --mesh constraints (rig_calibrator.cc:1796-1877): BracketedDepthMeshError
    # per depth observation with a mesh hit, XYZError to the track's mean hit
    depth_mesh_weight: float = 0.0
    mesh_tri_weight: float = 0.0
    robust_threshold: float = 3.0


def build_problem(rig: Rig, flags: FloatFlags | None = None, use_init: bool = True, mesh_xyz=None) -> CamProblem:
    """Assemble the BracketedCamError problem exactly as rig_calibrator.cc:1614-1752.
    ``mesh_xyz = (feature_xyz [N_obs, 3], point_xyz [N_pts, 3])`` from
    meshTriangulations (1e100 = no hit) enables the --mesh constraints.

    Packed parameter vector (DESIGN.md "Workloads"): world_to_ref | identity |
    ref_to_cam | xyz | offsets | focal | center | distortion | placeholder,
    (no_rig: world_to_cam replaces world_to_ref)."""
    flags = flags or FloatFlags()
    src = rig.init if use_init else {
        "world_to_ref": rig.world_to_ref, "ref_to_cam": rig.ref_to_cam, "xyz": rig.xyz,
        "focal": rig.focal, "center": rig.center, "dist": rig.dist, "offsets": rig.offsets,
        "world_to_cam": rig.world_to_cam}
    ns = rig.num_sensors
    nr = len(rig.ref_stamps)
    nimg = len(rig.cam_type)
    npts = rig.xyz.shape[0]
    names = rig.sensor_names
    poses = src["world_to_cam"] if flags.no_rig else src["world_to_ref"]
    npose = nimg if flags.no_rig else nr

    sizes, values, const = [], [], []

    def add(vals, c):
        vals = np.asarray(vals, dtype=np.float64).reshape(-1)
        sizes.append(vals.size)
        values.append(vals)
        const.append(1 if c else 0)
        return len(sizes) - 1

    ref_float = names[0] in flags.camera_poses_to_float
    pose_b0 = len(sizes)
    for k in range(npose):
        if flags.no_rig:
            c = names[rig.cam_type[k]] not in flags.camera_poses_to_float
        else:
            c = not ref_float
        add(poses[k], c)
    ident_b = add([0, 0, 0, 0, 0, 0, 1], True)
    r2c_b0 = len(sizes)
    for s in range(ns):
        fl = ("*" in flags.rig_transforms_to_float or names[s] in flags.rig_transforms_to_float)
        add(src["ref_to_cam"][s], (not fl) or s == 0 or flags.no_rig)
    xyz_b0 = len(sizes)
    # points are plain arrays: add in bulk
    for p in range(npts):
        sizes.append(3)
        const.append(0)
    values.append(np.asarray(src["xyz"], dtype=np.float64).reshape(-1))
    off_b0 = len(sizes)
    for s in range(ns):
        add([src["offsets"][s]], (not flags.float_timestamp_offsets) or s == 0 or flags.no_rig)
    foc_b0 = len(sizes)
    for s in range(ns):
        add([src["focal"][s]], "focal_length" not in flags.intrinsics_to_float)
    ctr_b0 = len(sizes)
    for s in range(ns):
        add(src["center"][s], "optical_center" not in flags.intrinsics_to_float)
    dist_b = []
    for s in range(ns):
        K = len(src["dist"][s])
        if K > 0:
            dist_b.append(add(src["dist"][s], "distortion" not in flags.intrinsics_to_float))
        else:
            dist_b.append(-1)
    ph_b = add([0.0], True)  # distortion_placeholder (rig_calibrator.cc:1608)
    dist_b = [b if b >= 0 else ph_b for b in dist_b]
    has_depth = rig.depth_obs is not None and rig.depth_obs.size > 0
    bad = 1.0e+100
    mesh_dep = np.zeros(0, dtype=np.int64)
    if mesh_xyz is not None and flags.depth_mesh_weight > 0 and has_depth:
        mesh_dep = rig.depth_obs[mesh_xyz[0][rig.depth_obs, 0] != bad]
    use_depth = (flags.depth_tri_weight > 0 and has_depth) or mesh_dep.size > 0
    if use_depth:
        dti_src = src.get("depth_to_image", rig.depth_to_image) if use_init else rig.depth_to_image
        want = 12 if flags.affine_depth_to_image else 7
        if dti_src.shape[1] != want:
            raise ValueError("rig depth_to_image kind does not match affine_depth_to_image")
        dti_b0 = len(sizes)
        for s in range(ns):
            add(dti_src[s], names[s] not in flags.depth_to_image_transforms_to_float)
        scl_b0 = len(sizes)
        for s in range(ns):
            add([src.get("depth_scale", np.ones(ns))[s] if use_init else 1.0],
                (not flags.float_scale) or flags.affine_depth_to_image)

    sizes = np.array(sizes, dtype=np.int32)
    offs = np.zeros(len(sizes), dtype=np.int64)
    offs[1:] = np.cumsum(sizes[:-1])
    params = np.concatenate(values)
    const = np.array(const, dtype=np.uint8)

    # residual blocks (one per observation, pid-major then cid, :1614-1699)
    cid = rig.obs_cid
    ct = rig.cam_type[cid]
    n = cid.size
    blocks = np.empty((n, 8), dtype=np.int32)
    stamps = np.empty((n, 3))
    if flags.no_rig:
        blocks[:, 0] = pose_b0 + cid
        blocks[:, 1] = ident_b
        stamps[:, 0] = rig.cam_stamp[cid]
        stamps[:, 1] = rig.cam_stamp[cid]
    else:
        beg, end = rig.cam_beg[cid], rig.cam_end[cid]
        blocks[:, 0] = pose_b0 + beg
        blocks[:, 1] = np.where((ct == 0) | (beg == end), ident_b, pose_b0 + end)
        stamps[:, 0] = rig.ref_stamps[beg]
        stamps[:, 1] = rig.ref_stamps[end]
    stamps[:, 2] = rig.cam_stamp[cid]
    blocks[:, 2] = r2c_b0 + ct
    blocks[:, 3] = xyz_b0 + rig.obs_pid
    blocks[:, 4] = off_b0 + ct
    blocks[:, 5] = foc_b0 + ct
    blocks[:, 6] = ctr_b0 + ct
    blocks[:, 7] = np.array(dist_b, dtype=np.int32)[ct]

    dsize = np.array([len(d) for d in src["dist"]], dtype=np.int32)
    half = np.tile(np.array(IMAGE_SIZE, dtype=np.float64) / 2.0, (ns, 1))
    P = CamProblem(block_size=sizes, block_offset=offs, block_constant=const, params=params,
                   camera_dist_size=dsize, camera_half_size=half, residual_blocks=blocks,
                   residual_camera=ct.astype(np.int32), residual_meas=rig.obs_pix.copy(),
                   residual_stamps=stamps,
                   residual_names=None if n > 100000 else [names[t] for t in ct])
    if use_depth:
        # after the observation's BracketedCamError: its BracketedDepthError
        # (rig_calibrator.cc:1755-1791), then its BracketedDepthMeshError
        # (:1796-1834), with the same beg/end/ref_to_cam/offset/stamps
        d_obs = rig.depth_obs if flags.depth_tri_weight > 0 else np.zeros(0, dtype=np.int64)
        meas_of = {int(o): q for q, o in enumerate(rig.depth_obs)}
        k = np.concatenate([d_obs, mesh_dep])
        kind = np.concatenate([np.zeros(d_obs.size, dtype=np.int8), np.ones(mesh_dep.size, dtype=np.int8)])
        o = np.lexsort((kind, k))
        k, kind = k[o], kind[o]
        dct = ct[k]
        db = np.empty((k.size, 7), dtype=np.int32)
        db[:, 0] = blocks[k, 0]
        db[:, 1] = blocks[k, 1]
        db[:, 2] = blocks[k, 2]
        db[:, 3] = dti_b0 + dct
        db[:, 4] = scl_b0 + dct
        db[:, 5] = np.where(kind == 1, -1, blocks[k, 3])
        db[:, 6] = blocks[k, 4]
        P.depth_blocks = db
        P.depth_meas = rig.depth_meas[[meas_of[int(x)] for x in k]].reshape(-1, 3).copy()
        P.depth_weight = np.where(kind == 1, float(flags.depth_mesh_weight), float(flags.depth_tri_weight))
        P.depth_stamps = stamps[k].copy()
        P.depth_after = k.astype(np.int64)
        if mesh_dep.size:
            P.depth_mesh_xyz = np.where(kind[:, None] == 1, mesh_xyz[0][k], 0.0)
    # per point: the mesh_tri prior (:1857-1877), then the tri prior (:1880-1898)
    xb, xr, xw, xt, xk = [], [], [], [], []
    if mesh_xyz is not None and flags.mesh_tri_weight > 0:
        good = np.nonzero(mesh_xyz[1][:, 0] != bad)[0]
        xb.append(xyz_b0 + good)
        xr.append(np.asarray(mesh_xyz[1])[good])
        xw.append(np.full(good.size, float(flags.mesh_tri_weight)))
        xt.append(np.full(good.size, float(flags.robust_threshold)))
        xk.append(np.ones(good.size, dtype=np.uint8))
    if flags.tri_weight > 0:
        # --tri_weight: keep points near their values before the optimisation
        # (xyz_vec_orig, :1571-1578), Cauchy(--tri_robust_threshold)
        if not flags.tri_robust_threshold > 0:
            raise ValueError("a positive --tri_robust_threshold is needed with --tri_weight")
        xb.append(xyz_b0 + np.arange(npts))
        xr.append(np.asarray(src["xyz"], dtype=np.float64).reshape(-1, 3).copy())
        xw.append(np.full(npts, float(flags.tri_weight)))
        xt.append(np.full(npts, float(flags.tri_robust_threshold)))
        xk.append(np.zeros(npts, dtype=np.uint8))
    if xb:
        b = np.concatenate(xb)
        o = np.argsort(b, kind="stable")  # point-major, mesh_tri before tri
        P.xyz_block = b[o].astype(np.int32)
        P.xyz_ref = np.concatenate(xr)[o]
        P.xyz_weight = np.concatenate(xw)[o]
        P.xyz_threshold = np.concatenate(xt)[o]
        P.xyz_kind = np.concatenate(xk)[o]
    return P


# Workload presets. c5 runs with CONFIG_FLAGS["c5"].
CONFIGS = {
    "c1": dict(num_sensors=3, num_ref=50, num_points=1000, obs_per_point=5.0, models=["none"] * 3, seed=1001),
    "c2": dict(num_sensors=3, num_ref=1000, num_points=100000, obs_per_point=10.0, models=["radtan"] * 3, seed=1002),
    "c3": dict(num_sensors=3, num_ref=3000, num_points=1000000, obs_per_point=10.0, models=["rpc2"] * 3, seed=1003),
    "c4": dict(num_sensors=8, num_ref=2500, num_points=5000000, obs_per_point=10.0, models=["radtan"] * 8, seed=1004),
    # 3 image sensors + 1 image+depth sensor: ~1M reprojection + ~250k depth blocks
    "c5": dict(num_sensors=4, num_ref=1000, num_points=100000, obs_per_point=10.0, models=["radtan"] * 4, seed=1005,
               depth_sensors=(3,)),
}


def offset_bounds(rig: Rig, problem: CamProblem, flags: FloatFlags | None = None, max_change: float = 1.0):
    """Lower/upper bounds (packed vector, +-inf elsewhere) of the floated timestamp
    offsets: the range keeping every bracketed image inside its bracket, clamped to
    offset +- timestamp_offsets_max_change and tightened by 1e-5
    (dense_map_utils.cc:1603-1656, applied at rig_calibrator.cc:1741-1745)."""
    flags = flags or FloatFlags()
    lower = np.full(problem.params.size, -np.inf)
    upper = np.full(problem.params.size, np.inf)
    if flags.no_rig or not flags.float_timestamp_offsets:
        return lower, upper
    ns = rig.num_sensors
    lo = np.full(ns, -1.0e100)
    hi = np.full(ns, 1.0e100)
    for k in range(len(rig.cam_type)):
        t = rig.cam_type[k]
        if t == 0:
            continue
        lo[t] = max(lo[t], rig.cam_stamp[k] - rig.ref_stamps[rig.cam_end[k]])
        hi[t] = min(hi[t], rig.cam_stamp[k] - rig.ref_stamps[rig.cam_beg[k]])
    # offsets block of sensor s: residual_blocks[:, 4] for that camera
    for s in range(1, ns):
        sel = np.nonzero(problem.residual_camera == s)[0]
        if sel.size == 0:
            continue
        b = int(problem.residual_blocks[sel[0], 4])
        o = int(problem.block_offset[b])
        cur = problem.params[o]
        lower[o] = max(lo[s], cur - max_change) + 1.0e-5
        upper[o] = min(hi[s], cur + max_change) - 1.0e-5
    return lower, upper


# FloatFlags of the presets beyond the default "everything floats"
CONFIG_FLAGS = {
    "c5": dict(depth_tri_weight=10.0, depth_to_image_transforms_to_float=("cam3",), float_scale=True),
}
