"""RPC lens-model fitting through the C ABI (mvba_rpc_fit).

    fit_rpc_undistortion(camera, dist_coeffs)  = updateRpcUndistortion /
                                                 fitRpcUndist (camera_params.cc:214-253)
    fit_rpc_distortion(camera, degree)         = fitRpcDist (rpc_distortion.cc:622-656)

``camera``: dict(focal, center, dist, image_size, crop_size, undist_size) — the
fields of camera::CameraParameters the fits read.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


def _camera(cam: dict, keep: list) -> _lib.RpcCamera:
    d = np.ascontiguousarray(cam.get("dist", np.zeros(0)), dtype=np.float64)
    keep.append(d)
    rc = _lib.RpcCamera()
    rc.focal = float(cam["focal"])
    rc.center[0], rc.center[1] = (float(v) for v in cam["center"])
    rc.dist_size = int(d.size)
    rc.dist = d.ctypes.data if d.size else None
    for name in ("image_size", "crop_size", "undist_size"):
        arr = getattr(rc, name)
        v = cam.get(name, cam["image_size"])
        arr[0], arr[1] = int(v[0]), int(v[1])
    return rc


def _report(r: _lib.RpcFitReport, degree: int) -> dict:
    return dict(num_samples_used=int(r.num_samples_used), undist_box=list(r.undist_box), dist_box=list(r.dist_box),
                initial_cost=list(r.initial_cost)[:degree], final_cost=list(r.final_cost)[:degree],
                iterations=list(r.iterations)[:degree], termination=list(r.termination)[:degree],
                max_dist_undist_error=float(r.max_dist_undist_error))


def _fit(cam, mode, degree, dist_coeffs, num_samples, num_iterations, parameter_tolerance, device):
    lib = _lib.load()
    keep = []
    rc = _camera(cam, keep)
    n = 2 * (degree + 1) * (degree + 2) - 2
    out = np.empty(n)
    rep = _lib.RpcFitReport()
    dc = None
    if dist_coeffs is not None:
        dc = np.ascontiguousarray(dist_coeffs, dtype=np.float64)
    st = lib.mvba_rpc_fit(C.byref(rc), mode, degree, dc.ctypes.data if dc is not None else None, num_samples,
                          num_iterations, parameter_tolerance, device, out.ctypes.data, C.byref(rep))
    if st != 0:
        raise _lib.MvbaError(st, (lib.mvba_rpc_error() or b"").decode())
    return out, _report(rep, degree)


def fit_rpc_undistortion(cam: dict, dist_coeffs, num_samples=400, num_iterations=100, parameter_tolerance=1e-12,
                         device=0):
    d = int(round(np.sqrt(2.0 * len(dist_coeffs) + 5.0) / 2.0 - 1.5))
    return _fit(cam, _lib.RPC_FIT_UNDISTORTION, d, dist_coeffs, num_samples, num_iterations, parameter_tolerance,
                device)


def fit_rpc_distortion(cam: dict, degree: int, num_samples=400, num_iterations=100, parameter_tolerance=1e-12,
                       device=0):
    return _fit(cam, _lib.RPC_FIT_DISTORTION, degree, None, num_samples, num_iterations, parameter_tolerance, device)
