"""ctypes binding of the C ABI in include/mvba/mvba.h (libmvba.so).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``python -m multiview_amd.build``). There is no CPU fallback: if the library or
a GPU is missing, every computing call raises ``MvbaError``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MVBA_LIB: another build of the same ABI (A/B measurements on one box)
LIB_PATH = os.environ.get("MVBA_LIB") or os.path.join(_HERE, "libmvba.so")

# Status codes (mvba_status).
MVBA_OK = 0
MVBA_E_ALPHA_RANGE = 1
MVBA_E_BLOCK_SIZES = 2
MVBA_E_BAD_DISTORTION = 3
MVBA_E_HIP = 4
MVBA_E_INVALID = 5
MVBA_E_NO_DEVICE = 6
MVBA_E_DEPTH_BLOCK_SIZES = 7
MVBA_E_XYZ_BLOCK_SIZES = 8
MVBA_E_DEVICE_WAIT = 9

STATUS_NAMES = {
    0: "MVBA_OK", 1: "MVBA_E_ALPHA_RANGE", 2: "MVBA_E_BLOCK_SIZES",
    3: "MVBA_E_BAD_DISTORTION", 4: "MVBA_E_HIP", 5: "MVBA_E_INVALID",
    6: "MVBA_E_NO_DEVICE", 7: "MVBA_E_DEPTH_BLOCK_SIZES", 8: "MVBA_E_XYZ_BLOCK_SIZES",
    9: "MVBA_E_DEVICE_WAIT",
}

EVAL_RESIDUALS = 0x1
EVAL_JACOBIAN = 0x2
EVAL_APPLY_LOSS = 0x4
EVAL_PREP_ONLY = 0x8
EVAL_SKIP_PREP = 0x10
EVAL_DEPTH = 0x100

# mvba_eval_form: the launch form of a full evaluation
FORM_SPLIT, FORM_FUSED, FORM_LOCAL = 0, 1, 2
FORM_NAMES = {FORM_SPLIT: "split", FORM_FUSED: "k_eval", FORM_LOCAL: "k_eval_local"}

# Jacobian row bases (MVBA_JAC_BASE_*), block order of rig_calibrator.cc:1695-1699.
JAC_BASE = (0, 14, 28, 42, 48, 50, 52, 56)
FIXED_BLOCK_SIZES = (7, 7, 7, 3, 1, 1, 2)


class MvbaError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status
        self.message = message


class ProblemDesc(C.Structure):
    _fields_ = [
        ("num_blocks", C.c_int32),
        ("block_size", C.c_void_p),
        ("block_offset", C.c_void_p),
        ("block_constant", C.c_void_p),
        ("num_param_doubles", C.c_int64),
        ("num_cameras", C.c_int32),
        ("camera_dist_size", C.c_void_p),
        ("camera_half_size", C.c_void_p),
        ("num_residuals", C.c_int64),
        ("residual_blocks", C.c_void_p),
        ("residual_camera", C.c_void_p),
        ("residual_meas", C.c_void_p),
        ("residual_stamps", C.c_void_p),
        ("num_depth_residuals", C.c_int64),
        ("depth_blocks", C.c_void_p),
        ("depth_meas", C.c_void_p),
        ("depth_weight", C.c_void_p),
        ("depth_stamps", C.c_void_p),
        ("num_xyz_residuals", C.c_int64),
        ("xyz_block", C.c_void_p),
        ("xyz_ref", C.c_void_p),
        ("xyz_weight", C.c_void_p),
        ("xyz_threshold", C.c_void_p),
        ("depth_mesh_xyz", C.c_void_p),   # ABI 5: BracketedDepthMeshError targets (depth xyz block -1)
        ("xyz_kind", C.c_void_p),         # ABI 5: 0 tri prior, 1 mesh_tri prior (statistics groups)
    ]


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("reserved0", C.c_int32), ("reserved1", C.c_double)]


class DeviceView(C.Structure):
    _fields_ = [
        ("num_residuals", C.c_int64),
        ("num_slots", C.c_int64),
        ("ld", C.c_int64),
        ("jac_rows", C.c_int32),
        ("max_dist_size", C.c_int32),
        ("residuals", C.c_void_p),
        ("jacobian", C.c_void_p),
        ("order", C.c_void_p),
        ("row_written", C.c_void_p),
    ]


class LinLayout(C.Structure):
    _fields_ = [
        ("cam_grad_size", C.c_int64),
        ("cam_hess_size", C.c_int64),
        ("num_points", C.c_int64),
        ("num_cam_blocks", C.c_int32),
        ("supported", C.c_int32),
    ]


# BracketedDepthError Jacobian layout (MVBA_DJAC_BASE_*): rows per block,
# depth_to_image given 12 columns of room.
DJAC_BASE = (0, 21, 42, 63, 99, 102, 111)
DJAC_ROWS = 114

REDUCE_SUM, REDUCE_MAX = 0, 1
LIN_CAMERA_ONLY, LIN_POINTS_ONLY, LIN_DETERMINISTIC = 0x20, 0x40, 0x80
CONVERGENCE, NO_CONVERGENCE, FAILURE = 0, 1, 2

# int32_t (*)(double* device_buf, int64_t count, int32_t op, void* stream, void* user)
AllreduceFn = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p)


class SolverOptions(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32),
        ("function_tolerance", C.c_double),
        ("gradient_tolerance", C.c_double),
        ("parameter_tolerance", C.c_double),
        ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double),
        ("min_trust_region_radius", C.c_double),
        ("min_lm_diagonal", C.c_double),
        ("max_lm_diagonal", C.c_double),
        ("min_relative_decrease", C.c_double),
        ("eta", C.c_double),
        ("min_linear_solver_iterations", C.c_int32),
        ("max_linear_solver_iterations", C.c_int32),
        ("max_num_consecutive_invalid_steps", C.c_int32),
        ("jacobi_scaling", C.c_int32),
        ("use_loss", C.c_int32),
        ("robust_threshold", C.c_double),
        ("lower_bounds", C.c_void_p),
        ("upper_bounds", C.c_void_p),
        ("progress_to_stdout", C.c_int32),
        ("allreduce", AllreduceFn),
        ("allreduce_user", C.c_void_p),
        ("deterministic", C.c_int32),
    ]


class SolverSummary(C.Structure):
    _fields_ = [
        ("initial_cost", C.c_double),
        ("final_cost", C.c_double),
        ("num_iterations", C.c_int32),
        ("num_successful_steps", C.c_int32),
        ("num_unsuccessful_steps", C.c_int32),
        ("num_linear_iterations", C.c_int32),
        ("termination_type", C.c_int32),
        ("cg_graph_launches", C.c_int32),
        ("total_time_s", C.c_double),
        ("linearize_time_s", C.c_double),
        ("linear_solver_time_s", C.c_double),
        ("eval_time_s", C.c_double),
        ("message", C.c_char * 256),
    ]


class TracksDesc(C.Structure):
    _fields_ = [
        ("num_images", C.c_int32),
        ("world_to_cam", C.c_void_p),
        ("image_camera", C.c_void_p),
        ("num_cameras", C.c_int32),
        ("focal", C.c_void_p),
        ("center", C.c_void_p),
        ("dist_size", C.c_void_p),
        ("dist_offset", C.c_void_p),
        ("dist", C.c_void_p),
        ("dist_half", C.c_void_p),
        ("undist_half", C.c_void_p),
        ("num_points", C.c_int64),
        ("track_begin", C.c_void_p),
        ("track_image", C.c_void_p),
        ("track_pix", C.c_void_p),
    ]


class MeshDesc(C.Structure):
    _fields_ = [
        ("num_vertices", C.c_int64),
        ("vertices", C.c_void_p),
        ("num_faces", C.c_int64),
        ("faces", C.c_void_p),
    ]


RPC_FIT_DISTORTION = 0
RPC_FIT_UNDISTORTION = 1


class RpcCamera(C.Structure):
    _fields_ = [
        ("focal", C.c_double),
        ("center", C.c_double * 2),
        ("dist_size", C.c_int32),
        ("dist", C.c_void_p),
        ("image_size", C.c_int32 * 2),
        ("crop_size", C.c_int32 * 2),
        ("undist_size", C.c_int32 * 2),
    ]


class RpcFitReport(C.Structure):
    _fields_ = [
        ("num_samples_used", C.c_int64),
        ("undist_box", C.c_double * 4),
        ("dist_box", C.c_double * 4),
        ("initial_cost", C.c_double * 6),
        ("final_cost", C.c_double * 6),
        ("iterations", C.c_int32 * 6),
        ("termination", C.c_int32 * 6),
        ("max_dist_undist_error", C.c_double),
    ]


# Every symbol include/mvba/mvba.h declares, with (restype, argtypes).
SIGNATURES = {
    "mvba_abi_version": (C.c_int, []),
    "mvba_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "mvba_create": (C.c_int, [C.POINTER(ProblemDesc), C.POINTER(Options), C.POINTER(C.c_void_p)]),
    "mvba_destroy": (None, [C.c_void_p]),
    "mvba_last_error": (C.c_char_p, [C.c_void_p]),
    "mvba_create_error": (C.c_char_p, []),
    "mvba_set_params": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_set_params_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_evaluate": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_jacobian_stride": (C.c_int32, [C.c_void_p]),
    "mvba_host_alloc": (C.c_void_p, [C.c_size_t]),
    "mvba_host_free": (None, [C.c_void_p]),
    "mvba_set_transfer_blocks": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_packed_size": (C.c_int64, [C.c_void_p]),
    "mvba_evaluate_packed": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_evaluate_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.c_void_p]),
    "mvba_evaluate_device_f32": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                                           C.c_int64, C.c_void_p]),
    "mvba_device_buffers": (C.c_int, [C.c_void_p, C.POINTER(DeviceView)]),
    "mvba_sync_status": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_residual_order": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_num_residuals": (C.c_int64, [C.c_void_p]),
    "mvba_num_slots": (C.c_int64, [C.c_void_p]),
    "mvba_num_frames": (C.c_int64, [C.c_void_p]),
    "mvba_num_points": (C.c_int64, [C.c_void_p]),
    "mvba_eval_bytes": (C.c_double, [C.c_void_p, C.c_int32]),
    "mvba_eval_form": (C.c_int32, [C.c_void_p]),
    "mvba_lin_layout_info": (C.c_int, [C.c_void_p, C.POINTER(LinLayout)]),
    "mvba_cam_block_map": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_point_block_map": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_linearize_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_num_depth_residuals": (C.c_int64, [C.c_void_p]),
    "mvba_num_depth_slots": (C.c_int64, [C.c_void_p]),
    "mvba_depth_order": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_evaluate_depth": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_evaluate_depth_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                                             C.c_int64, C.c_void_p]),
    "mvba_evaluate_depth_device_f32": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p, C.c_void_p,
                                                 C.c_int64, C.c_void_p]),
    "mvba_residual_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_num_xyz_residuals": (C.c_int64, [C.c_void_p]),
    "mvba_triangulate": (C.c_int, [C.POINTER(TracksDesc), C.c_int32, C.c_void_p, C.c_void_p]),
    "mvba_flag_outliers": (C.c_int, [C.POINTER(TracksDesc), C.c_int32, C.c_void_p, C.c_void_p, C.c_double,
                                     C.c_double, C.c_void_p, C.c_void_p]),
    "mvba_frame_poses": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_tracks_error": (C.c_char_p, []),
    "mvba_mesh_create": (C.c_int, [C.POINTER(MeshDesc), C.c_int32, C.POINTER(C.c_void_p)]),
    "mvba_mesh_destroy": (None, [C.c_void_p]),
    "mvba_mesh_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "mvba_mesh_intersect_device": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_float, C.c_float,
                                             C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_mesh_triangulate": (C.c_int, [C.POINTER(TracksDesc), C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                        C.c_void_p, C.c_void_p]),
    "mvba_mesh_error": (C.c_char_p, []),
    "mvba_rpc_fit": (C.c_int, [C.POINTER(RpcCamera), C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                               C.c_double, C.c_int32, C.c_void_p, C.POINTER(RpcFitReport)]),
    "mvba_rpc_error": (C.c_char_p, []),
    "mvba_evaluate_xyz": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mvba_solver_default_options": (None, [C.POINTER(SolverOptions)]),
    "mvba_solve": (C.c_int, [C.c_void_p, C.POINTER(SolverOptions), C.POINTER(SolverSummary), C.c_void_p]),
    "mvba_get_params": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mvba_lin_mfma_flops": (C.c_double, [C.c_void_p]),
    "mvba_comm_unique_id": (C.c_int, [C.c_void_p]),
    "mvba_comm_init_rccl": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "mvba_comm_init_rccl_deadline": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                               C.POINTER(C.c_void_p)]),
    "mvba_comm_init_local": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p]),
    "mvba_comm_abort": (C.c_int, [C.c_void_p]),
    "mvba_comm_destroy": (None, [C.c_void_p]),
    "mvba_comm_rank": (C.c_int32, [C.c_void_p]),
    "mvba_comm_size": (C.c_int32, [C.c_void_p]),
    "mvba_comm_error": (C.c_char_p, []),
    "mvba_comm_allreduce": (C.c_int32, [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p]),
}

COMM_ID_BYTES = 128

_lib = None


def load(path: str = LIB_PATH):
    """Load libmvba.so and bind every ABI symbol. Raises if the library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MvbaError(MVBA_E_NO_DEVICE,
                        f"{path} not built — run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = missing export: fail loudly
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, handle=None, create: bool = False):
    if status == MVBA_OK:
        return
    lib = load()
    if create:
        msg = lib.mvba_create_error().decode()
    elif handle is not None:
        msg = lib.mvba_last_error(handle).decode()
    else:
        msg = ""
    raise MvbaError(status, msg)
