"""ctypes loader of the CPU oracle (liboracle_mvba.so).

TEST INFRASTRUCTURE ONLY — importable from tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. PARITY UNPINNED against the
reference binary (see oracle.cpp header and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_mvba.so")

RESIDUAL, NUMDIFF, ANALYTIC = 0, 1, 2
# evaluate_mt only: mode 1 numbers with the reference's per-call copies and checks
# (CameraParameters deep copy, SetDistortion, compute_rpc vectors, Ceres 1.14
# DynamicNumericDiffCostFunction / ResidualBlock::Evaluate bookkeeping)
NUMDIFF_FAITHFUL = 3
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.oracle_triangulate.restype = C.c_int
    lib.oracle_triangulate.argtypes = [C.c_int64] + [C.c_void_p] * 14
    lib.oracle_flag_outliers.restype = None
    lib.oracle_flag_outliers.argtypes = [C.c_int64] + [C.c_void_p] * 5 + [C.c_double, C.c_double] + \
        [C.c_void_p] * 2
    lib.oracle_evaluate.restype = C.c_int
    lib.oracle_evaluate.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_double,
                                    C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.oracle_evaluate_mt.restype = C.c_int
    lib.oracle_evaluate_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_double,
                                       C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p]
    lib.oracle_validate.restype = C.c_int
    lib.oracle_validate.argtypes = [C.c_void_p]
    lib.oracle_last_error.restype = C.c_char_p
    lib.oracle_jacobian_stride.restype = C.c_int
    lib.oracle_jacobian_stride.argtypes = [C.c_void_p]
    lib.oracle_world_to_cam.restype = C.c_int
    lib.oracle_world_to_cam.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                        C.c_double, C.c_double, C.c_void_p]
    lib.oracle_distort.restype = C.c_int
    lib.oracle_distort.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                   C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_void_p]
    lib.oracle_depth_mesh_error.restype = C.c_int
    lib.oracle_depth_mesh_error.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_double, C.c_void_p, C.c_void_p,
                                            C.c_double, C.c_double, C.c_double, C.c_int, C.c_void_p, C.c_void_p]
    lib.oracle_ray_mesh.restype = None
    lib.oracle_ray_mesh.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_int64,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.oracle_mesh_triangulate.restype = C.c_int
    lib.oracle_mesh_triangulate.argtypes = [C.c_int64] + [C.c_void_p] * 13 + [C.c_double, C.c_double, C.c_int64] + \
        [C.c_void_p] * 4
    lib.oracle_depth_error.restype = C.c_int
    lib.oracle_depth_error.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_double, C.c_void_p,
                                       C.c_double, C.c_double, C.c_double, C.c_int, C.c_void_p,
                                       C.c_void_p]
    lib.oracle_residual_stats.restype = None
    lib.oracle_residual_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p,
                                          C.c_void_p]
    _lib = lib
    return lib


class OracleError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"oracle status {status}: {msg}")
        self.status = status


def evaluate(problem, mode=ANALYTIC, apply_loss=False, robust_threshold=3.0, begin=0, end=-1):
    """Evaluate a CamProblem on the CPU. Returns (cost, r [n,2], J [n,stride] or None)."""
    lib = load()
    desc = problem.desc()
    n = problem.num_residuals if end < 0 else end - begin
    stride = lib.oracle_jacobian_stride(C.byref(desc))
    r = np.empty((n, 2))
    J = np.zeros((n, stride)) if mode != RESIDUAL else None
    cost = C.c_double()
    flags = 0x4 if apply_loss else 0
    st = lib.oracle_evaluate(C.byref(desc), problem.params.ctypes.data, mode, flags,
                             float(robust_threshold), int(begin), int(end), C.byref(cost),
                             r.ctypes.data, J.ctypes.data if J is not None else None)
    if st != 0:
        raise OracleError(st, lib.oracle_last_error().decode())
    return cost.value, r, J


def evaluate_mt(problem, mode=NUMDIFF, begin=0, end=-1, threads=1, want_jac=True):
    """Multi-threaded (OpenMP over residual blocks, like Ceres num_threads) timing
    path for the cpu_baseline: writes residuals and Jacobian rows."""
    lib = load()
    desc = problem.desc()
    n = problem.num_residuals if end < 0 else end - begin
    stride = lib.oracle_jacobian_stride(C.byref(desc))
    r = np.empty((n, 2))
    J = np.zeros((n, stride)) if want_jac else None
    st = lib.oracle_evaluate_mt(C.byref(desc), problem.params.ctypes.data, mode, 0, 3.0,
                                int(begin), int(end), int(threads), r.ctypes.data,
                                J.ctypes.data if J is not None else None)
    if st != 0:
        raise OracleError(st, lib.oracle_last_error().decode())
    return r, J


def validate(problem):
    lib = load()
    desc = problem.desc()
    st = lib.oracle_validate(C.byref(desc))
    return st, lib.oracle_last_error().decode()


def world_to_cam(beg, end, r2c, sb, se, off, sc):
    lib = load()
    out = np.empty(12)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (beg, end, r2c)]
    st = lib.oracle_world_to_cam(arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data,
                                 sb, se, off, sc, out.ctypes.data)
    if st != 0:
        raise OracleError(st, "Out of bounds in interpolation.")
    return out[:9].reshape(3, 3), out[9:]


def distort(u, f, c, k, half):
    lib = load()
    k = np.ascontiguousarray(k, dtype=np.float64)
    out = np.empty(2)
    st = lib.oracle_distort(float(u[0]), float(u[1]), float(f), float(c[0]), float(c[1]),
                            k.ctypes.data if k.size else None, int(k.size), float(half[0]),
                            float(half[1]), out.ctypes.data)
    if st != 0:
        raise OracleError(st, "Recieved irregular distortion vector size.")
    return out


def depth_error(blocks, constant, weight, meas, sb, se, sc, mode=ANALYTIC):
    """BracketedDepthError (rig_calibrator.cc:547-583). blocks: 7 arrays."""
    lib = load()
    arrs = [np.ascontiguousarray(b, dtype=np.float64) for b in blocks]
    ptrs = (C.c_void_p * 7)(*[a.ctypes.data for a in arrs])
    const = np.ascontiguousarray(constant, dtype=np.uint8)
    m = np.ascontiguousarray(meas, dtype=np.float64)
    r = np.empty(3)
    nj = 3 * sum(a.size for a in arrs)
    J = np.zeros(nj)
    st = lib.oracle_depth_error(ptrs, arrs[3].size, const.ctypes.data, float(weight), m.ctypes.data,
                                sb, se, sc, mode, r.ctypes.data, J.ctypes.data)
    if st < 0:
        raise OracleError(-st, "depth error")
    return r, J


def depth_mesh_error(blocks, constant, weight, meas, mesh, sb, se, sc, mode=ANALYTIC):
    """BracketedDepthMeshError (rig_calibrator.cc:641-673). blocks: 6 arrays (beg,
    end, ref_to_cam, depth_to_image, scale, offset); J rows 3 x size_b per block."""
    lib = load()
    arrs = [np.ascontiguousarray(b, dtype=np.float64) for b in blocks]
    ptrs = (C.c_void_p * 6)(*[a.ctypes.data for a in arrs])
    const = np.ascontiguousarray(constant, dtype=np.uint8)
    m = np.ascontiguousarray(meas, dtype=np.float64)
    x = np.ascontiguousarray(mesh, dtype=np.float64)
    r = np.empty(3)
    J = np.zeros(3 * sum(a.size for a in arrs))
    st = lib.oracle_depth_mesh_error(ptrs, arrs[3].size, const.ctypes.data, float(weight), m.ctypes.data,
                                     x.ctypes.data, sb, se, sc, mode, r.ctypes.data, J.ctypes.data)
    if st < 0:
        raise OracleError(-st, "depth mesh error")
    return r, J


def residual_stats(residuals, name_ids, num_names):
    lib = load()
    r = np.ascontiguousarray(residuals, dtype=np.float64)
    ids = np.ascontiguousarray(name_ids, dtype=np.int32)
    out = np.empty(4 * num_names)
    cnt = np.empty(num_names, dtype=np.int64)
    lib.oracle_residual_stats(r.ctypes.data, ids.ctypes.data, r.size, num_names, out.ctypes.data,
                              cnt.ctypes.data)
    return out.reshape(num_names, 4), cnt


DJAC_BASE = (0, 21, 42, 63, 99, 102, 111)
DJAC_ROWS = 114


def evaluate_depth(problem, mode=ANALYTIC, apply_loss=False, robust_threshold=3.0):
    """All BracketedDepthError blocks of a CamProblem (rig_calibrator.cc:547-583),
    depth insertion order. Returns (cost, r [n,3], J [n,DJAC_ROWS] or None) with
    Ceres' Cauchy corrector applied when apply_loss (as Problem::Evaluate)."""
    n = problem.num_depth_residuals
    r = np.zeros((n, 3))
    J = np.zeros((n, DJAC_ROWS)) if mode != RESIDUAL else None
    b = robust_threshold * robust_threshold
    cost = 0.0
    mesh_xyz = getattr(problem, "depth_mesh_xyz", np.zeros((0, 3)))
    for j in range(n):
        blk = problem.depth_blocks[j]
        if blk[5] == -1:
            # BracketedDepthMeshError: blocks without xyz; the xyz rows stay zero
            ids = [int(blk[q]) for q in (0, 1, 2, 3, 4, 6)]
            six = [problem.block_values(x) for x in ids]
            rj, J6 = depth_mesh_error(six, problem.block_constant[ids], problem.depth_weight[j],
                                      problem.depth_meas[j], mesh_xyz[j], *problem.depth_stamps[j], mode=mode)
            blocks = six[:5] + [np.zeros(3)] + six[5:]
            Jj = np.concatenate([J6[:3 * (21 + six[3].size + 1)], np.zeros(9), J6[3 * (21 + six[3].size + 1):]])
        else:
            blocks = [problem.block_values(int(x)) for x in blk]
            const = problem.block_constant[blk]
            rj, Jj = depth_error(blocks, const, problem.depth_weight[j], problem.depth_meas[j],
                                 *problem.depth_stamps[j], mode=mode)
        s2 = float(rj @ rj)
        sr = 1.0
        if apply_loss:
            cost += 0.5 * (b * np.log(1.0 + s2 / b))
            sr = np.sqrt(max(np.finfo(float).tiny, 1.0 / (1.0 + s2 / b)))
        else:
            cost += 0.5 * s2
        r[j] = rj * sr
        if J is not None:
            off = 0
            for bb in range(7):
                size = blocks[bb].size
                J[j, DJAC_BASE[bb]:DJAC_BASE[bb] + 3 * size] = Jj[off:off + 3 * size] * sr
                off += 3 * size
    return cost, r, J


def evaluate_xyz(problem, apply_loss=False):
    """XYZError (rig_calibrator.cc:720-724): r = weight (xyz - ref), Jacobian
    weight * I (3x3 row-major, zero for constant points), each block with its
    own Cauchy threshold. Returns (cost, r [n,3], J [n,9])."""
    n = problem.num_xyz_residuals
    r = np.zeros((n, 3))
    J = np.zeros((n, 9))
    cost = 0.0
    for j in range(n):
        b = int(problem.xyz_block[j])
        x = problem.block_values(b)
        w = problem.xyz_weight[j]
        rj = w * (x - problem.xyz_ref[j])
        s2 = float(rj @ rj)
        sr = 1.0
        if apply_loss:
            bb = problem.xyz_threshold[j] ** 2
            cost += 0.5 * (bb * np.log(1.0 + s2 / bb))
            sr = np.sqrt(max(np.finfo(float).tiny, 1.0 / (1.0 + s2 / bb)))
        else:
            cost += 0.5 * s2
        r[j] = rj * sr
        if not problem.block_constant[b]:
            J[j] = (w * sr * np.eye(3)).reshape(-1)
    return cost, r, J


def triangulate(tracks, inlier=None):
    """multiViewTriangulation restated (oracle.cpp). tracks: multiview_amd.tracks.Tracks."""
    lib = load()
    d = tracks.desc()
    ar = tracks._keep
    inl = np.ones(tracks.num_obs, dtype=np.uint8) if inlier is None else np.array(inlier, dtype=np.uint8)
    xyz = np.zeros((tracks.num_points, 3))
    st = lib.oracle_triangulate(C.c_int64(tracks.num_points), ar[9].ctypes.data, ar[10].ctypes.data,
                                ar[1].ctypes.data, ar[0].ctypes.data, ar[2].ctypes.data, ar[3].ctypes.data,
                                ar[4].ctypes.data, ar[5].ctypes.data, ar[6].ctypes.data, ar[7].ctypes.data,
                                ar[8].ctypes.data, ar[11].ctypes.data, inl.ctypes.data, xyz.ctypes.data)
    if st != 0:
        raise OracleError(st, "triangulate")
    del d
    return inl, xyz


def flag_outliers(tracks, xyz, residuals, min_angle, max_err, inlier):
    """flagOutliersByTriAngleAndReprojErr restated (oracle.cpp)."""
    lib = load()
    d = tracks.desc()
    ar = tracks._keep
    inl = np.array(inlier, dtype=np.uint8)
    x = np.ascontiguousarray(xyz, dtype=np.float64)
    r = np.ascontiguousarray(residuals, dtype=np.float64)
    counts = np.zeros(4, dtype=np.int64)
    lib.oracle_flag_outliers(C.c_int64(tracks.num_points), ar[9].ctypes.data, ar[10].ctypes.data, ar[0].ctypes.data,
                             x.ctypes.data, r.ctypes.data, C.c_double(min_angle), C.c_double(max_err),
                             inl.ctypes.data, counts.ctypes.data)
    del d
    return inl, counts


def ray_mesh(orig, dir, tmin, tmax, verts, faces):
    """Closest hit of each ray, brute force over every face (rayint's test restated,
    float). Returns (t [n] float32, -1 = miss; face [n] int32, -1 = miss)."""
    lib = load()
    o = np.ascontiguousarray(orig, dtype=np.float32).reshape(-1)
    d = np.ascontiguousarray(dir, dtype=np.float32).reshape(-1)
    v = np.ascontiguousarray(verts, dtype=np.float32).reshape(-1)
    f = np.ascontiguousarray(faces, dtype=np.uint32).reshape(-1)
    n = o.size // 3
    t = np.empty(n, dtype=np.float32)
    face = np.empty(n, dtype=np.int32)
    lib.oracle_ray_mesh(C.c_int64(n), o.ctypes.data, d.ctypes.data, C.c_float(tmin), C.c_float(tmax),
                        C.c_int64(f.size // 3), v.ctypes.data, f.ctypes.data, t.ctypes.data, face.ctypes.data)
    return t, face


def mesh_triangulate(tracks, inlier, min_ray_dist, max_ray_dist, verts, faces):
    """meshTriangulations restated (oracle.cpp). Returns (feature_xyz [n_obs,3],
    point_xyz [n_pts,3]) with bad = 1e100."""
    lib = load()
    d = tracks.desc()
    ar = tracks._keep
    inl = np.ascontiguousarray(inlier, dtype=np.uint8)
    v = np.ascontiguousarray(verts, dtype=np.float32).reshape(-1)
    f = np.ascontiguousarray(faces, dtype=np.uint32).reshape(-1)
    fx = np.zeros((tracks.num_obs, 3))
    px = np.zeros((tracks.num_points, 3))
    st = lib.oracle_mesh_triangulate(C.c_int64(tracks.num_points), ar[9].ctypes.data, ar[10].ctypes.data,
                                     ar[1].ctypes.data, ar[0].ctypes.data, ar[2].ctypes.data, ar[3].ctypes.data,
                                     ar[4].ctypes.data, ar[5].ctypes.data, ar[6].ctypes.data, ar[7].ctypes.data,
                                     ar[8].ctypes.data, ar[11].ctypes.data, inl.ctypes.data,
                                     C.c_double(min_ray_dist), C.c_double(max_ray_dist), C.c_int64(f.size // 3),
                                     v.ctypes.data, f.ctypes.data, fx.ctypes.data, px.ctypes.data)
    if st != 0:
        raise OracleError(st, "mesh_triangulate")
    del d
    return fx, px
