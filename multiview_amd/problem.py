"""Host-side mirror of the reference's problem-assembly interface for the
BracketedCamError path.

The reference builds one ``ceres::CostFunction`` per observation with
``BracketedCamError::Create(meas, left_stamp, right_stamp, cam_stamp,
block_sizes, cam_params)`` (rig_calibrator.cc:485-505) and registers it with
``problem.AddResidualBlock(cost, CauchyLoss(robust_threshold), beg, end,
ref_to_cam, xyz, offset, focal, center, dist)`` (:1695-1699), then marks blocks
constant with ``SetParameterBlockConstant`` (:1702-1752).

``CamProblem`` keeps the same vocabulary (parameter blocks, residual blocks,
constant blocks, camera parameters) but stores it as flat arrays so that a
million-observation problem can be described without a Python object per
observation. It produces the ``mvba_problem_desc`` of include/mvba/mvba.h.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib

FIXED_BLOCK_SIZES = _lib.FIXED_BLOCK_SIZES


def rpc_degree(num_dist_params: int) -> int:
    """rpc_distortion.cc:43-45."""
    return int(round(np.sqrt(2.0 * num_dist_params + 5.0) / 2.0 - 1.5))


def rpc_num_dist_params(deg: int) -> int:
    """rpc_distortion.cc:47-49."""
    return 2 * (deg + 1) * (deg + 2) - 2


def distortion_size_valid(K: int) -> bool:
    """Sizes camera::CameraParameters::SetDistortion accepts (camera_params.cc:181-207)."""
    if K in (0, 1, 4, 5):
        return True
    if K % 2:
        return False
    n = K // 2
    d = rpc_degree(n)
    return d > 0 and rpc_num_dist_params(d) == n


@dataclass
class CamProblem:
    """A problem made of BracketedCamError residual blocks (flat-array form)."""

    # parameter blocks
    block_size: np.ndarray            # int32 [B]
    block_offset: np.ndarray          # int64 [B]
    block_constant: np.ndarray        # uint8 [B]
    params: np.ndarray                # float64 [num_param_doubles] (packed values)
    # camera models (CameraParameters captured by Create)
    camera_dist_size: np.ndarray      # int32 [C]
    camera_half_size: np.ndarray      # float64 [C, 2]
    # residual blocks in AddResidualBlock order
    residual_blocks: np.ndarray       # int32 [N, 8]
    residual_camera: np.ndarray       # int32 [N]
    residual_meas: np.ndarray         # float64 [N, 2]
    residual_stamps: np.ndarray       # float64 [N, 3]
    residual_names: list = field(default_factory=list)  # per residual block: sensor name
    # BracketedDepthError blocks (optional): 7 block ids each (MVBA_DBLK_* order)
    depth_blocks: np.ndarray = field(default_factory=lambda: np.zeros((0, 7), dtype=np.int32))
    depth_meas: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    depth_weight: np.ndarray = field(default_factory=lambda: np.zeros(0))
    depth_stamps: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    depth_after: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.int64))  # preceding cam block
    # BracketedDepthMeshError blocks share the depth list: xyz block id -1 and the
    # fixed mesh point in depth_mesh_xyz (rows of other blocks ignored); empty = none
    depth_mesh_xyz: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    # XYZError priors (optional): point block, reference xyz, weight, Cauchy threshold
    xyz_block: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.int32))
    xyz_ref: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    xyz_weight: np.ndarray = field(default_factory=lambda: np.zeros(0))
    xyz_threshold: np.ndarray = field(default_factory=lambda: np.zeros(0))
    xyz_kind: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.uint8))  # 1 = mesh_tri prior
    _keep: list = field(default_factory=list, repr=False)

    @property
    def num_residuals(self) -> int:
        return int(self.residual_blocks.shape[0])

    @property
    def num_depth_residuals(self) -> int:
        return int(self.depth_blocks.shape[0])

    @property
    def num_xyz_residuals(self) -> int:
        return int(self.xyz_block.shape[0])

    def jacobian_stride(self) -> int:
        kmax = int(self.camera_dist_size.max()) if len(self.camera_dist_size) else 0
        return 56 + 2 * kmax

    def desc(self) -> _lib.ProblemDesc:
        """Build the C description. Arrays are kept alive on this object."""
        arrs = [
            np.ascontiguousarray(self.block_size, dtype=np.int32),
            np.ascontiguousarray(self.block_offset, dtype=np.int64),
            np.ascontiguousarray(self.block_constant, dtype=np.uint8),
            np.ascontiguousarray(self.camera_dist_size, dtype=np.int32),
            np.ascontiguousarray(self.camera_half_size, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.residual_blocks, dtype=np.int32).reshape(-1),
            np.ascontiguousarray(self.residual_camera, dtype=np.int32),
            np.ascontiguousarray(self.residual_meas, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.residual_stamps, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.depth_blocks, dtype=np.int32).reshape(-1),
            np.ascontiguousarray(self.depth_meas, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.depth_weight, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.depth_stamps, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.xyz_block, dtype=np.int32).reshape(-1),
            np.ascontiguousarray(self.xyz_ref, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.xyz_weight, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.xyz_threshold, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.depth_mesh_xyz, dtype=np.float64).reshape(-1),
            np.ascontiguousarray(self.xyz_kind, dtype=np.uint8).reshape(-1),
        ]
        if arrs[17].size not in (0, 3 * self.num_depth_residuals):
            raise ValueError("depth_mesh_xyz needs 3 values per depth residual block")
        if arrs[18].size not in (0, self.num_xyz_residuals):
            raise ValueError("xyz_kind needs one value per XYZ prior")
        self._keep = arrs
        d = _lib.ProblemDesc()
        d.num_blocks = len(arrs[0])
        d.block_size = arrs[0].ctypes.data
        d.block_offset = arrs[1].ctypes.data
        d.block_constant = arrs[2].ctypes.data
        d.num_param_doubles = int(self.params.size)
        d.num_cameras = len(arrs[3])
        d.camera_dist_size = arrs[3].ctypes.data
        d.camera_half_size = arrs[4].ctypes.data
        d.num_residuals = self.num_residuals
        d.residual_blocks = arrs[5].ctypes.data
        d.residual_camera = arrs[6].ctypes.data
        d.residual_meas = arrs[7].ctypes.data
        d.residual_stamps = arrs[8].ctypes.data
        d.num_depth_residuals = self.num_depth_residuals
        d.depth_blocks = arrs[9].ctypes.data
        d.depth_meas = arrs[10].ctypes.data
        d.depth_weight = arrs[11].ctypes.data
        d.depth_stamps = arrs[12].ctypes.data
        d.num_xyz_residuals = self.num_xyz_residuals
        d.xyz_block = arrs[13].ctypes.data
        d.xyz_ref = arrs[14].ctypes.data
        d.xyz_weight = arrs[15].ctypes.data
        d.xyz_threshold = arrs[16].ctypes.data
        d.depth_mesh_xyz = arrs[17].ctypes.data if arrs[17].size else None
        d.xyz_kind = arrs[18].ctypes.data if arrs[18].size else None
        return d

    def subset(self, idx: np.ndarray) -> "CamProblem":
        """Problem made of the residual blocks ``idx`` (same parameter blocks, no
        depth blocks)."""
        idx = np.asarray(idx)
        return CamProblem(
            block_size=self.block_size, block_offset=self.block_offset,
            block_constant=self.block_constant, params=self.params,
            camera_dist_size=self.camera_dist_size, camera_half_size=self.camera_half_size,
            residual_blocks=self.residual_blocks[idx], residual_camera=self.residual_camera[idx],
            residual_meas=self.residual_meas[idx], residual_stamps=self.residual_stamps[idx],
            residual_names=[self.residual_names[i] for i in idx] if self.residual_names else [],
        )

    def block_values(self, b: int) -> np.ndarray:
        o = int(self.block_offset[b])
        return self.params[o:o + int(self.block_size[b])]


class ProblemBuilder:
    """Incremental builder with the reference's call vocabulary (small problems,
    tests). ``add_parameter_block`` returns a block id; ``add_residual_block``
    takes the 8 block ids in the AddResidualBlock order of rig_calibrator.cc:1695-1699."""

    def __init__(self):
        self._values = []
        self._const = []
        self._cams = []
        self._res = []

    def add_parameter_block(self, values) -> int:
        self._values.append(np.array(values, dtype=np.float64).reshape(-1))
        self._const.append(0)
        return len(self._values) - 1

    def set_parameter_block_constant(self, b: int):
        self._const[b] = 1

    def set_parameter_block_variable(self, b: int):
        self._const[b] = 0

    def add_camera(self, dist_size: int, image_size) -> int:
        """camera::CameraParameters with distortion length K and image size (w, h);
        half size = image_size / 2 (camera_params.cc:107-110)."""
        self._cams.append((int(dist_size), float(image_size[0]) / 2.0, float(image_size[1]) / 2.0))
        return len(self._cams) - 1

    def add_residual_block(self, meas, left_stamp, right_stamp, cam_stamp, blocks, camera,
                           name: str = ""):
        if len(blocks) != 8:
            raise ValueError("BracketedCamError takes 8 parameter blocks")
        self._res.append((tuple(float(m) for m in meas), float(left_stamp), float(right_stamp),
                          float(cam_stamp), tuple(int(b) for b in blocks), int(camera), name))
        return len(self._res) - 1

    def build(self) -> CamProblem:
        sizes = np.array([v.size for v in self._values], dtype=np.int32)
        offs = np.zeros(len(sizes), dtype=np.int64)
        if len(sizes):
            offs[1:] = np.cumsum(sizes[:-1])
        params = np.concatenate(self._values) if self._values else np.zeros(0)
        n = len(self._res)
        return CamProblem(
            block_size=sizes, block_offset=offs,
            block_constant=np.array(self._const, dtype=np.uint8), params=params,
            camera_dist_size=np.array([c[0] for c in self._cams], dtype=np.int32),
            camera_half_size=np.array([[c[1], c[2]] for c in self._cams], dtype=np.float64).reshape(-1, 2),
            residual_blocks=np.array([r[4] for r in self._res], dtype=np.int32).reshape(n, 8),
            residual_camera=np.array([r[5] for r in self._res], dtype=np.int32),
            residual_meas=np.array([r[0] for r in self._res], dtype=np.float64).reshape(n, 2),
            residual_stamps=np.array([[r[1], r[2], r[3]] for r in self._res], dtype=np.float64).reshape(n, 3),
            residual_names=[r[6] for r in self._res],
        )

