"""Python handle over the C ABI (one ``mvba_handle``).

This is a thin convenience layer used by tests and bench.py; the boundary a
maintainer binds is include/mvba/mvba.h. Every computing
call goes to libmvba.so on the GPU — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .problem import CamProblem


class PinnedBuffer:
    """Pinned host doubles from mvba_host_alloc (a DMA target for the host
    evaluations); ``array`` is a numpy view, valid until ``free()``."""

    def __init__(self, n: int):
        self.lib = _lib.load()
        self.n = int(n)
        self.ptr = self.lib.mvba_host_alloc(max(self.n, 1) * 8)
        if not self.ptr:
            raise MemoryError("mvba_host_alloc failed")
        self.array = np.ctypeslib.as_array((C.c_double * max(self.n, 1)).from_address(self.ptr))[:self.n]

    def free(self):
        if self.ptr:
            self.array = None
            self.lib.mvba_host_free(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()


class Evaluator:
    """GPU evaluator for a CamProblem (BracketedCamError residual blocks)."""

    def __init__(self, problem: CamProblem, device: int = 0):
        self.lib = _lib.load()
        self.problem = problem
        self._desc = problem.desc()
        opts = _lib.Options(device=device, reserved0=0, reserved1=0.0)
        h = C.c_void_p()
        st = self.lib.mvba_create(C.byref(self._desc), C.byref(opts), C.byref(h))
        _lib.check(st, create=True)
        self.h = h
        self.stride = int(self.lib.mvba_jacobian_stride(self.h))
        self.num_residuals = int(self.lib.mvba_num_residuals(self.h))
        self.num_slots = int(self.lib.mvba_num_slots(self.h))
        self.ld = ((self.num_slots + 63) // 64) * 64
        self.num_frames = int(self.lib.mvba_num_frames(self.h))
        self.num_points = int(self.lib.mvba_num_points(self.h))
        self.num_depth = int(self.lib.mvba_num_depth_residuals(self.h))
        self.num_depth_slots = int(self.lib.mvba_num_depth_slots(self.h))

    # ---------------------------------------------------------------- params
    def set_params(self, params: np.ndarray | None = None):
        p = self.problem.params if params is None else params
        p = np.ascontiguousarray(p, dtype=np.float64)
        if p.size != self.problem.params.size:
            raise ValueError("packed parameter vector has the wrong size")
        _lib.check(self.lib.mvba_set_params(self.h, p.ctypes.data), self.h)

    def set_params_device(self, tensor, stream=None):
        """tensor: torch float64 CUDA tensor with the packed parameters."""
        _lib.check(self.lib.mvba_set_params_device(self.h, C.c_void_p(tensor.data_ptr()),
                                                   C.c_void_p(stream or 0)), self.h)

    # ------------------------------------------------------------ evaluation
    def evaluate(self, jacobian: bool = True, apply_loss: bool = False,
                 robust_threshold: float = 3.0):
        """Host evaluation in AddResidualBlock order.

        Returns (cost, residuals [N, 2], jacobian [N, stride] or None), the
        Jacobian in the Ceres layout (MVBA_JAC_BASE_*), constant blocks zero."""
        n = self.num_residuals
        r = np.empty((n, 2), dtype=np.float64)
        J = np.empty((n, self.stride), dtype=np.float64) if jacobian else None
        cost = C.c_double(0.0)
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | \
            (_lib.EVAL_APPLY_LOSS if apply_loss else 0)
        st = self.lib.mvba_evaluate(self.h, flags, float(robust_threshold), C.byref(cost),
                                    r.ctypes.data, J.ctypes.data if J is not None else None)
        _lib.check(st, self.h)
        return cost.value, r, J

    def set_transfer_blocks(self, transfer=None) -> np.ndarray:
        """Select the parameter blocks whose Jacobian columns evaluate_packed
        transfers (bool per block; None = every non-constant block). Returns the
        per-residual row offsets [N + 1]."""
        off = np.empty(self.num_residuals + 1, dtype=np.int64)
        tp = None
        if transfer is not None:
            t = np.ascontiguousarray(transfer, dtype=np.uint8)
            if t.size != len(self.problem.block_size):
                raise ValueError("transfer needs one entry per parameter block")
            tp = t.ctypes.data
        _lib.check(self.lib.mvba_set_transfer_blocks(self.h, tp, off.ctypes.data), self.h)
        return off

    def evaluate_packed(self, jacobian: bool = True, apply_loss: bool = False, robust_threshold: float = 3.0,
                        out=None, res_out=None, want_cost: bool = True):
        """Host evaluation with the packed Jacobian layout (set_transfer_blocks).
        out / res_out: optional float64 arrays of mvba_packed_size() / 2N entries
        (e.g. views of pinned memory from PinnedBuffer). Returns (cost or None,
        residuals [N, 2], packed)."""
        n = self.num_residuals
        size = int(self.lib.mvba_packed_size(self.h))
        if size < 0:
            self.set_transfer_blocks(None)
            size = int(self.lib.mvba_packed_size(self.h))
        r = np.empty((n, 2), dtype=np.float64) if res_out is None else res_out.reshape(n, 2)
        J = None
        if jacobian:
            J = np.empty(size, dtype=np.float64) if out is None else out
            if J.size < size or J.dtype != np.float64 or not J.flags.c_contiguous:
                raise ValueError("out must be a contiguous float64 array of mvba_packed_size() entries")
        cost = C.c_double(0.0)
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | \
            (_lib.EVAL_APPLY_LOSS if apply_loss else 0)
        st = self.lib.mvba_evaluate_packed(self.h, flags, float(robust_threshold),
                                           C.byref(cost) if want_cost else None, r.ctypes.data,
                                           J.ctypes.data if J is not None else None)
        _lib.check(st, self.h)
        return (cost.value if want_cost else None), r, J

    def evaluate_depth(self, jacobian: bool = True, apply_loss: bool = False, robust_threshold: float = 3.0):
        """BracketedDepthError blocks, host, depth insertion order: (cost,
        residuals [N_d, 3], Jacobian [N_d, DJAC_ROWS] or None)."""
        n = self.num_depth
        r = np.empty((n, 3), dtype=np.float64)
        J = np.empty((n, _lib.DJAC_ROWS), dtype=np.float64) if jacobian else None
        cost = C.c_double(0.0)
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | \
            (_lib.EVAL_APPLY_LOSS if apply_loss else 0)
        st = self.lib.mvba_evaluate_depth(self.h, flags, float(robust_threshold), C.byref(cost), r.ctypes.data,
                                          J.ctypes.data if J is not None else None)
        _lib.check(st, self.h)
        return cost.value, r, J

    def evaluate_xyz(self, jacobian: bool = True, apply_loss: bool = False):
        """XYZError priors, insertion order: (cost, residuals [n, 3], Jacobian [n, 9])."""
        n = self.problem.num_xyz_residuals
        r = np.empty((n, 3))
        J = np.empty((n, 9)) if jacobian else None
        cost = C.c_double(0.0)
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | \
            (_lib.EVAL_APPLY_LOSS if apply_loss else 0)
        st = self.lib.mvba_evaluate_xyz(self.h, flags, C.byref(cost), r.ctypes.data,
                                        J.ctypes.data if J is not None else None)
        _lib.check(st, self.h)
        return cost.value, r, J

    def evaluate_device(self, jacobian: bool = True, apply_loss: bool = False,
                        robust_threshold: float = 3.0, residuals=None, jac=None, ld: int = 0,
                        stream=None, phase: int = 0):
        """Asynchronous device evaluation. residuals/jac: optional torch float64
        CUDA tensors of shape [2, ld] / [stride, ld] (caller-owned outputs);
        float32 tensors select the fp32-output evaluation."""
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | \
            (_lib.EVAL_APPLY_LOSS if apply_loss else 0) | phase
        rp = C.c_void_p(residuals.data_ptr()) if residuals is not None else None
        jp = C.c_void_p(jac.data_ptr()) if jac is not None else None
        f32 = residuals is not None and str(residuals.dtype) == "torch.float32"
        fn = self.lib.mvba_evaluate_device_f32 if f32 else self.lib.mvba_evaluate_device
        st = fn(self.h, flags, float(robust_threshold), rp, jp, int(ld), C.c_void_p(stream or 0))
        _lib.check(st, self.h)

    def sync(self, stream=None):
        _lib.check(self.lib.mvba_sync_status(self.h, C.c_void_p(stream or 0)), self.h)

    def device_view(self) -> _lib.DeviceView:
        v = _lib.DeviceView()
        _lib.check(self.lib.mvba_device_buffers(self.h, C.byref(v)), self.h)
        return v

    def order(self) -> np.ndarray:
        """device slot -> AddResidualBlock index (-1 = padding slot)."""
        out = np.empty(self.num_slots, dtype=np.int64)
        _lib.check(self.lib.mvba_residual_order(self.h, out.ctypes.data), self.h)
        return out

    def depth_order(self) -> np.ndarray:
        """device depth slot -> depth insertion index (-1 = padding slot)."""
        out = np.empty(self.num_depth_slots, dtype=np.int64)
        _lib.check(self.lib.mvba_depth_order(self.h, out.ctypes.data), self.h)
        return out

    def evaluate_depth_device(self, jacobian: bool = True, residuals=None, jac=None, ld: int = 0,
                              stream=None, phase: int = 0):
        """Asynchronous device evaluation of the depth blocks into caller-owned
        torch planes [3, ld] / [DJAC_ROWS, ld] (float64 or float32)."""
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0) | phase
        f32 = str(residuals.dtype) == "torch.float32"
        fn = self.lib.mvba_evaluate_depth_device_f32 if f32 else self.lib.mvba_evaluate_depth_device
        st = fn(self.h, flags, 0.0, C.c_void_p(residuals.data_ptr()),
                C.c_void_p(jac.data_ptr()) if jac is not None else None, int(ld), C.c_void_p(stream or 0))
        _lib.check(st, self.h)

    def eval_bytes(self, jacobian: bool = True) -> float:
        flags = _lib.EVAL_RESIDUALS | (_lib.EVAL_JACOBIAN if jacobian else 0)
        return float(self.lib.mvba_eval_bytes(self.h, flags))

    def eval_bytes_prep(self) -> float:
        """Algorithmic bytes of the prep (landmark gather + K0 frame records)."""
        return float(self.lib.mvba_eval_bytes(self.h, _lib.EVAL_PREP_ONLY))

    def eval_form(self) -> int:
        """Launch form of a full evaluation (_lib.FORM_SPLIT / FORM_FUSED / FORM_LOCAL)."""
        return int(self.lib.mvba_eval_form(self.h))

    # ------------------------------------------------------- normal equations
    def lin_layout(self) -> dict:
        L = _lib.LinLayout()
        _lib.check(self.lib.mvba_lin_layout_info(self.h, C.byref(L)), self.h)
        nb = L.num_cam_blocks
        ids = np.empty(nb, dtype=np.int32)
        goff = np.empty(nb, dtype=np.int64)
        hoff = np.empty(nb, dtype=np.int64)
        _lib.check(self.lib.mvba_cam_block_map(self.h, ids.ctypes.data, goff.ctypes.data,
                                               hoff.ctypes.data), self.h)
        pids = np.empty(L.num_points, dtype=np.int32)
        _lib.check(self.lib.mvba_point_block_map(self.h, pids.ctypes.data), self.h)
        return dict(cam_grad_size=L.cam_grad_size, cam_hess_size=L.cam_hess_size,
                    num_points=L.num_points, supported=bool(L.supported), cam_block_ids=ids,
                    cam_goff=goff, cam_hoff=hoff, point_block_ids=pids)

    def linearize_device(self, cam_grad, cam_hess, pt_grad, pt_hess, cost=None,
                         apply_loss: bool = False, robust_threshold: float = 3.0, stream=None,
                         skip_prep: bool = False, side: str = "both", deterministic: bool = False):
        """Gradient and block-diagonal Hessian into caller-owned torch float64
        CUDA tensors (layouts: include/mvba/mvba.h, mvba_linearize_device).
        side: "both", "camera" (MVBA_LIN_CAMERA_ONLY) or "points" (timing);
        deterministic: MVBA_LIN_DETERMINISTIC (fixed-order camera-side sums)."""
        flags = (_lib.EVAL_APPLY_LOSS if apply_loss else 0) | (_lib.EVAL_SKIP_PREP if skip_prep else 0) | \
            {"both": 0, "camera": _lib.LIN_CAMERA_ONLY, "points": _lib.LIN_POINTS_ONLY}[side] | \
            (_lib.LIN_DETERMINISTIC if deterministic else 0)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        st = self.lib.mvba_linearize_device(self.h, flags, float(robust_threshold), ptr(cam_grad),
                                            ptr(cam_hess), ptr(pt_grad), ptr(pt_hess), ptr(cost),
                                            C.c_void_p(stream or 0))
        _lib.check(st, self.h)

    # ------------------------------------------------------- residual stats
    def residual_stats(self, sensor_names=None) -> list:
        """evalResiduals + calc_residuals_stats (rig_calibrator.cc:1157-1180,
        :753-789) on the GPU. Returns [(name, p25, p50, p75, p100, count)] in the
        reference's print order (std::map: names sorted), only names that have
        residual blocks."""
        ncam = len(self.problem.camera_dist_size)
        names = list(sensor_names or [f"cam{c}" for c in range(ncam)])
        ng = 2 * ncam + 12
        out = np.empty(4 * ng)
        counts = np.empty(ng, dtype=np.int64)
        _lib.check(self.lib.mvba_residual_stats(self.h, out.ctypes.data, counts.ctypes.data, None), self.h)
        labels = stats_labels(names)
        rows = [(labels[g], *out[4 * g:4 * g + 4], int(counts[g])) for g in range(ng) if counts[g] > 0]
        return sorted(rows, key=lambda r: r[0])

    @staticmethod
    def format_residual_stats(rows, tag: str) -> str:
        """The reference's stdout block (calc_residuals_stats, setprecision(5))."""
        lines = [f"The 25, 50, 75, and 100th percentile residual stats {tag}"]
        for name, a, b, c, d, n in rows:
            lines.append(f"{name}: {a:.5g} {b:.5g} {c:.5g} {d:.5g} ({n} residuals)")
        return "\n".join(lines)

    # ---------------------------------------------------------------- solver
    def get_params(self) -> np.ndarray:
        out = np.empty(self.problem.params.size, dtype=np.float64)
        _lib.check(self.lib.mvba_get_params(self.h, out.ctypes.data), self.h)
        return out

    def solve(self, options: "_lib.SolverOptions | None" = None, stream=None, **kw) -> dict:
        """Levenberg-Marquardt on the GPU from the current parameters
        (mvba_solve; ceres::Solve replacement). Keyword arguments override
        fields of mvba_solver_default_options. Returns the summary as a dict;
        the solution stays in the handle (get_params)."""
        if options is None:
            n = self.problem.params.size
            for k in ("lower_bounds", "upper_bounds"):
                v = kw.get(k)
                if v is not None and np.asarray(v).size != n:
                    # the library reads num_param_doubles values from each bound array
                    raise ValueError(f"{k} has {np.asarray(v).size} values, the packed parameter vector {n}")
        o = options or default_solver_options(**kw)
        s = _lib.SolverSummary()
        st = self.lib.mvba_solve(self.h, C.byref(o), C.byref(s), C.c_void_p(stream or 0))
        cb_errors = getattr(o, "_callback_errors", None)
        if st != _lib.MVBA_OK and cb_errors:
            # the library only sees a non-zero return from the all-reduce
            # callback: name the Python exception that caused it
            msg = self.lib.mvba_last_error(self.h).decode()
            first = cb_errors[0]
            raise _lib.MvbaError(st, f"{msg} ({type(first).__name__}: {first})") from first
        _lib.check(st, self.h)
        return summary_dict(s)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.mvba_destroy(self.h)
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


def stats_labels(sensor_names) -> list:
    """Residual names of the mvba_residual_stats groups (rig_calibrator.cc:1690-1691,
    :1769-1771, :1818-1820, :1873-1875, :1893-1895)."""
    return [f"{n}_pix_{xy}" for n in sensor_names for xy in "xy"] + \
        [f"{kind}_{a}_m" for kind in ("depth_tri", "tri", "depth_mesh", "mesh_tri") for a in "xyz"]


def _hip_sync(stream) -> int:
    """hipStreamSynchronize on a raw stream handle (libamdhip64, loaded by torch)."""
    from .dist import _hip

    return _hip().hipStreamSynchronize(stream or None)


def default_solver_options(**kw) -> _lib.SolverOptions:
    """mvba_solver_default_options, then overrides (lower_bounds/upper_bounds as
    numpy arrays over the packed parameter vector; allreduce as a Python callable
    ``f(device_ptr, count, op[, hip_stream]) -> None`` honouring the
    stream-ordered contract of mvba_allreduce_fn; comm as a dist.Comm)."""
    lib = _lib.load()
    o = _lib.SolverOptions()
    lib.mvba_solver_default_options(C.byref(o))
    keep = []
    cb_errors = []
    for k, v in kw.items():
        if k in ("lower_bounds", "upper_bounds"):
            if v is None:
                continue
            arr = np.ascontiguousarray(v, dtype=np.float64)
            keep.append(arr)
            setattr(o, k, arr.ctypes.data)
        elif k == "comm":
            # library-native communicator (dist.Comm): the C all-reduce itself
            if v is None:
                continue
            addr = C.cast(lib.mvba_comm_allreduce, C.c_void_p).value
            o.allreduce = _lib.AllreduceFn(addr)
            o.allreduce_user = v.h
            keep.append(v)
        elif k == "allreduce":
            if v is None:
                continue
            import inspect

            nargs = len(inspect.signature(v).parameters)

            def _cb(ptr, count, op, stream, user, _f=v, _n=nargs, _errs=cb_errors):
                try:
                    if _n >= 4:
                        _f(ptr, count, op, stream or 0)
                    else:
                        # a 3-argument callback predates the stream-ordered
                        # contract: it reads and writes the buffer on the host
                        # side, so the solver's stream must have drained first
                        if _hip_sync(stream) != 0:
                            raise RuntimeError("hipStreamSynchronize failed")
                        _f(ptr, count, op)
                    return 0
                except Exception as e:  # noqa: BLE001 - reported as a failed status
                    print(f"allreduce callback failed: {e!r}")
                    _errs.append(e)
                    return 1
            fn = _lib.AllreduceFn(_cb)
            keep.append(fn)
            o.allreduce = fn
        else:
            if not hasattr(o, k):
                raise AttributeError(f"unknown solver option {k}")
            setattr(o, k, v)
    o._keep = keep  # keep arrays / callback alive for the call
    o._callback_errors = cb_errors  # exceptions the all-reduce callback swallowed
    return o


def summary_dict(s: _lib.SolverSummary) -> dict:
    return dict(initial_cost=s.initial_cost, final_cost=s.final_cost, num_iterations=s.num_iterations,
                num_successful_steps=s.num_successful_steps, num_unsuccessful_steps=s.num_unsuccessful_steps,
                num_linear_iterations=s.num_linear_iterations, termination_type=s.termination_type,
                cg_graph_launches=s.cg_graph_launches,
                total_time_s=s.total_time_s, linearize_time_s=s.linearize_time_s,
                linear_solver_time_s=s.linear_solver_time_s, eval_time_s=s.eval_time_s,
                message=s.message.decode(errors="replace"))
