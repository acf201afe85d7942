"""Tracks: per-pass triangulation and outlier flagging.

Host-side mirror of rig_calibrator's track state: ``pid_to_cid_fid`` (features
of each landmark, images in increasing order, as the std::map iterates),
``keypoint_vec`` (distorted pixels) and ``pid_cid_fid_inlier`` (0/1 per
feature), flattened to CSR arrays. The computation runs in libmvba
(``mvba_triangulate`` = multiViewTriangulation, interest_point.cc:649-722;
``mvba_flag_outliers`` = flagOutliersByTriAngleAndReprojErr,
rig_calibrator.cc:1045-1154); there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib


@dataclass
class Tracks:
    world_to_cam: np.ndarray        # [N_img, 12] R row-major + t
    image_camera: np.ndarray        # [N_img] camera model
    focal: np.ndarray               # [N_cam]
    center: np.ndarray              # [N_cam, 2]
    dist: list                      # [N_cam] distortion vectors (RPC: [dist | undist])
    dist_half: np.ndarray           # [N_cam, 2]
    undist_half: np.ndarray         # [N_cam, 2]
    track_begin: np.ndarray         # [N_pts + 1]
    track_image: np.ndarray         # [N_obs]
    track_pix: np.ndarray           # [N_obs, 2]
    _keep: list = field(default_factory=list, repr=False)

    @property
    def num_obs(self) -> int:
        return int(self.track_begin[-1])

    @property
    def num_points(self) -> int:
        return int(self.track_begin.size - 1)

    def desc(self) -> _lib.TracksDesc:
        sizes = np.array([len(d) for d in self.dist], dtype=np.int32)
        offs = np.zeros(len(sizes), dtype=np.int64)
        if len(sizes):
            offs[1:] = np.cumsum(sizes[:-1])
        dist = np.concatenate([np.asarray(d, dtype=np.float64) for d in self.dist]) if sizes.sum() else np.zeros(1)
        arrs = [np.ascontiguousarray(self.world_to_cam, dtype=np.float64).reshape(-1),
                np.ascontiguousarray(self.image_camera, dtype=np.int32),
                np.ascontiguousarray(self.focal, dtype=np.float64),
                np.ascontiguousarray(self.center, dtype=np.float64).reshape(-1),
                sizes, offs, np.ascontiguousarray(dist),
                np.ascontiguousarray(self.dist_half, dtype=np.float64).reshape(-1),
                np.ascontiguousarray(self.undist_half, dtype=np.float64).reshape(-1),
                np.ascontiguousarray(self.track_begin, dtype=np.int64),
                np.ascontiguousarray(self.track_image, dtype=np.int32),
                np.ascontiguousarray(self.track_pix, dtype=np.float64).reshape(-1)]
        self._keep = arrs
        d = _lib.TracksDesc()
        d.num_images = len(arrs[1])
        d.world_to_cam, d.image_camera = arrs[0].ctypes.data, arrs[1].ctypes.data
        d.num_cameras = len(sizes)
        d.focal, d.center = arrs[2].ctypes.data, arrs[3].ctypes.data
        d.dist_size, d.dist_offset, d.dist = arrs[4].ctypes.data, arrs[5].ctypes.data, arrs[6].ctypes.data
        d.dist_half, d.undist_half = arrs[7].ctypes.data, arrs[8].ctypes.data
        d.num_points = self.num_points
        d.track_begin, d.track_image, d.track_pix = arrs[9].ctypes.data, arrs[10].ctypes.data, arrs[11].ctypes.data
        return d


def _check(st):
    if st != _lib.MVBA_OK:
        raise _lib.MvbaError(st, _lib.load().mvba_tracks_error().decode())


def triangulate(tracks: Tracks, inlier=None, device: int = 0):
    """Returns (inlier [N_obs] uint8, xyz [N_pts, 3])."""
    lib = _lib.load()
    inl = np.ones(tracks.num_obs, dtype=np.uint8) if inlier is None else np.array(inlier, dtype=np.uint8)
    xyz = np.zeros((tracks.num_points, 3))
    d = tracks.desc()
    _check(lib.mvba_triangulate(C.byref(d), int(device), inl.ctypes.data, xyz.ctypes.data))
    return inl, xyz


def flag_outliers(tracks: Tracks, xyz, residuals, min_triangulation_angle, max_reprojection_error, inlier,
                  device: int = 0):
    """Returns (inlier, counts[4]) — counts: outliers by angle, features in the
    angle pass, outliers by reprojection error, features in the reprojection pass
    (the numbers rig_calibrator prints, :1111-1114 and :1149-1151)."""
    lib = _lib.load()
    inl = np.array(inlier, dtype=np.uint8)
    x = np.ascontiguousarray(xyz, dtype=np.float64)
    r = np.ascontiguousarray(residuals, dtype=np.float64)
    counts = np.zeros(4, dtype=np.int64)
    d = tracks.desc()
    _check(lib.mvba_flag_outliers(C.byref(d), int(device), x.ctypes.data, r.ctypes.data,
                                  float(min_triangulation_angle), float(max_reprojection_error),
                                  inl.ctypes.data, counts.ctypes.data))
    return inl, counts


def from_rig(rig, world_to_cam, use_init: bool = True) -> Tracks:
    """Tracks of a synthetic rig (multiview_amd.rig): features = observations
    (already (pid, cid)-ordered), keypoints = measured pixels, cameras = sensors
    with the rig's intrinsics (undistorted size = distorted size)."""
    from .rig import IMAGE_SIZE

    src = rig.init if use_init else {"focal": rig.focal, "center": rig.center, "dist": rig.dist}
    ns = rig.num_sensors
    half = np.tile(np.array(IMAGE_SIZE, dtype=np.float64) / 2.0, (ns, 1))
    dist = []
    for s in range(ns):
        k = np.asarray(src["dist"][s], dtype=np.float64)
        dist.append(k)
    tb = np.zeros(rig.xyz.shape[0] + 1, dtype=np.int64)
    np.add.at(tb, rig.obs_pid + 1, 1)
    tb = np.cumsum(tb)
    return Tracks(world_to_cam=np.asarray(world_to_cam).reshape(-1, 12), image_camera=rig.cam_type.astype(np.int32),
                  focal=np.asarray(src["focal"], dtype=np.float64), center=np.asarray(src["center"], dtype=np.float64),
                  dist=dist, dist_half=half, undist_half=half.copy(), track_begin=tb,
                  track_image=rig.obs_cid.astype(np.int32), track_pix=rig.obs_pix.copy())


# ---------------------------------------------------------------- mesh (--mesh)
class Mesh:
    """A triangle mesh on the GPU with its BVH (mvba_mesh_create; the reference's
    loadMeshBuildTree, texture_processing.cc:264-285). ``vertices`` [V, 3]
    float32, ``faces`` [F, 3] vertex indices."""

    def __init__(self, vertices, faces, device: int = 0):
        self.lib = _lib.load()
        self.vertices = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        self.faces = np.ascontiguousarray(faces, dtype=np.uint32).reshape(-1, 3)
        d = _lib.MeshDesc()
        d.num_vertices = self.vertices.shape[0]
        d.vertices = self.vertices.ctypes.data
        d.num_faces = self.faces.shape[0]
        d.faces = self.faces.ctypes.data
        self.h = C.c_void_p()
        st = self.lib.mvba_mesh_create(C.byref(d), int(device), C.byref(self.h))
        if st != _lib.MVBA_OK:
            raise _lib.MvbaError(st, self.lib.mvba_mesh_error().decode())

    def info(self) -> dict:
        n, dp = C.c_int64(), C.c_int32()
        self.lib.mvba_mesh_info(self.h, C.byref(n), C.byref(dp))
        return {"num_nodes": n.value, "depth": dp.value}

    def intersect_device(self, orig, dirs, tmin, tmax, t_out, face_out, stream=None):
        """Closest hits of device rays (torch float32 [n, 3] tensors), rayint's Ray
        semantics; t_out (float32, -1 = miss) and face_out (int32) [n]."""
        n = int(orig.shape[0])
        st = self.lib.mvba_mesh_intersect_device(self.h, n, C.c_void_p(orig.data_ptr()), C.c_void_p(dirs.data_ptr()),
                                                 float(tmin), float(tmax), C.c_void_p(t_out.data_ptr()),
                                                 C.c_void_p(face_out.data_ptr()), C.c_void_p(stream or 0))
        if st != _lib.MVBA_OK:
            raise _lib.MvbaError(st, self.lib.mvba_mesh_error().decode())

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.mvba_mesh_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def mesh_triangulate(tracks: Tracks, mesh: Mesh, inlier, min_ray_dist: float = 0.0, max_ray_dist: float = 100.0):
    """meshTriangulations (texture_processing.cc:1566-1625). Returns
    (feature_xyz [N_obs, 3], point_xyz [N_pts, 3]); 1e100 marks no hit."""
    lib = _lib.load()
    inl = np.ascontiguousarray(inlier, dtype=np.uint8)
    fx = np.zeros((tracks.num_obs, 3))
    px = np.zeros((tracks.num_points, 3))
    d = tracks.desc()
    _check(lib.mvba_mesh_triangulate(C.byref(d), mesh.h, inl.ctypes.data, float(min_ray_dist), float(max_ray_dist),
                                     fx.ctypes.data, px.ctypes.data))
    return fx, px
