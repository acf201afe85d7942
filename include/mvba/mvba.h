/*
 * mvba.h — C ABI of the MI355X-native bundle-adjustment evaluator for
 * MultiView's rig_calibrator hot path.
 *
 * What this replaces (reference, oleg-alexandrov/MultiView):
 *   - dense_map::BracketedCamError::operator() / ::Create
 *       rig_calibrator/bin/rig_calibrator.cc:419-514
 *     wrapped in ceres::DynamicNumericDiffCostFunction<..., CENTRAL>
 *       (Ceres 1.14 [ext]; rig_calibrator.cc:489-505)
 *   - the per-observation pose math it calls:
 *       calc_world_to_cam_trans      rig_calibrator.cc:362-390
 *       calc_interp_world_to_ref     rig_calibrator.cc:322-353
 *       array_to_rigid_transform     rig_calibrator/src/dense_map_utils.cc:171-178
 *       linearInterp (slerp)         rig_calibrator/src/dense_map_utils.cc:315-329
 *   - the camera model it calls:
 *       CameraParameters::Convert<UNDISTORTED_C,DISTORTED>  camera_model/camera_params.cc:412-415
 *       CameraParameters::DistortCentered                    camera_model/camera_params.cc:260-314
 *       RPCLensDistortion::distort_centered / compute_rpc    camera_model/rpc_distortion.cc:116-160, 358-360
 *   - the Ceres Evaluate path over all residual blocks
 *       evalResiduals → Problem::Evaluate                    rig_calibrator.cc:1157-1180
 *   - the Cauchy loss applied by Ceres (GetLossFunction)      rig_calibrator.cc:394-411
 *
 * The reference evaluates one heap-allocated functor per observation and
 * obtains the Jacobian by central differences (1 + 2*n_free functor calls per
 * observation). This library evaluates ALL residual blocks of a problem in one
 * pass on the GPU, with the analytic Jacobian, writing results to HBM.
 *
 * Rules of the boundary
 *   - extern "C", plain pointers and sizes, no exceptions cross it.
 *   - Host memory is caller-owned; the library copies what it needs.
 *   - Device buffers are library-owned unless passed in by the caller
 *     (mvba_evaluate_into).
 *   - A handle is NOT re-entrant: one evaluation at a time per handle
 *     (ceres::EvaluationCallback guarantees this).
 *   - Every entry point returns an mvba_status; on error the message is
 *     available from mvba_last_error(handle) and mirrors the reference's
 *     LOG(FATAL) text for the same condition.
 */
#ifndef MVBA_MVBA_H_
#define MVBA_MVBA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVBA_ABI_VERSION 6

/* Status codes. Non-zero codes mirror the reference's fatal checks. */
typedef enum mvba_status {
  MVBA_OK = 0,
  /* "Out of bounds in interpolation." rig_calibrator.cc:346 */
  MVBA_E_ALPHA_RANGE = 1,
  /* "BracketedCamError: The block sizes were not set up properly." rig_calibrator.cc:433-440 */
  MVBA_E_BLOCK_SIZES = 2,
  /* "Recieved irregular distortion vector size." camera_params.cc:199-206 */
  MVBA_E_BAD_DISTORTION = 3,
  /* HIP runtime failure (allocation, launch, copy). */
  MVBA_E_HIP = 4,
  /* Invalid argument (null pointer, out-of-range index, ...). */
  MVBA_E_INVALID = 5,
  /* No usable GPU (the product path has no CPU fallback). */
  MVBA_E_NO_DEVICE = 6,
  /* "BracketedDepthError: The block sizes were not set up properly." rig_calibrator.cc:534-543
   * (or "BracketedDepthMeshError: ..." rig_calibrator.cc:630-638 for a mesh block) */
  MVBA_E_DEPTH_BLOCK_SIZES = 7,
  /* "XYZError: The block sizes were not set up properly." rig_calibrator.cc:714-715 */
  MVBA_E_XYZ_BLOCK_SIZES = 8,
  /* Device-side bounded wait given up (the one-launch evaluation's frame-record
   * hand-off, k_eval): the evaluation's outputs are not valid. No reference
   * counterpart (the reference has no device). */
  MVBA_E_DEVICE_WAIT = 9
} mvba_status;

/* Parameter-block order of one BracketedCamError residual block, exactly the
 * AddResidualBlock argument order of rig_calibrator.cc:1695-1699. */
enum {
  MVBA_BLK_BEG = 0,        /* beg world_to_ref (7: tx ty tz qx qy qz qw) */
  MVBA_BLK_END = 1,        /* end world_to_ref (7) */
  MVBA_BLK_REF_TO_CAM = 2, /* ref_to_cam (7) */
  MVBA_BLK_XYZ = 3,        /* triangulated point (3) */
  MVBA_BLK_OFFSET = 4,     /* ref_to_cam timestamp offset (1) */
  MVBA_BLK_FOCAL = 5,      /* focal length (1) */
  MVBA_BLK_CENTER = 6,     /* optical center (2) */
  MVBA_BLK_DIST = 7,       /* distortion (K = GetDistortion().size()) */
  MVBA_NUM_CAM_BLOCKS = 8
};

/* Jacobian row layout of one residual block (2 residual rows), identical in
 * the host Ceres layout and in the device column-plane layout:
 * block b occupies rows [mvba_jac_row_base(b), +2*size_b), row-major 2 x size_b
 * (Ceres convention: jacobians[b][r * size_b + c]). */
#define MVBA_JAC_BASE_BEG 0
#define MVBA_JAC_BASE_END 14
#define MVBA_JAC_BASE_REF_TO_CAM 28
#define MVBA_JAC_BASE_XYZ 42
#define MVBA_JAC_BASE_OFFSET 48
#define MVBA_JAC_BASE_FOCAL 50
#define MVBA_JAC_BASE_CENTER 52
#define MVBA_JAC_BASE_DIST 56 /* 2*K rows follow */

/* Description of a problem made of BracketedCamError residual blocks.
 * All arrays are caller-owned and only read during mvba_create(). */
typedef struct mvba_problem_desc {
  /* Parameter blocks, packed into one vector of doubles. */
  int32_t num_blocks;
  const int32_t* block_size;     /* [num_blocks] */
  const int64_t* block_offset;   /* [num_blocks] offset into the packed vector */
  const uint8_t* block_constant; /* [num_blocks] 1 = Problem::SetParameterBlockConstant */
  int64_t num_param_doubles;

  /* Camera models: the camera::CameraParameters copies captured by
   * BracketedCamError::Create (rig_calibrator.cc:512). Only the distorted
   * half size and the distortion length are used on the residual path. */
  int32_t num_cameras;
  const int32_t* camera_dist_size; /* [num_cameras] K = GetDistortion().size() */
  const double* camera_half_size;  /* [2*num_cameras] GetDistortedHalfSize() */

  /* Residual blocks, in AddResidualBlock order (= Problem::Evaluate order). */
  int64_t num_residuals;
  const int32_t* residual_blocks; /* [8*num_residuals] block ids, MVBA_BLK_* order */
  const int32_t* residual_camera; /* [num_residuals] camera model index */
  const double* residual_meas;    /* [2*num_residuals] meas_dist_pix */
  const double* residual_stamps;  /* [3*num_residuals] left_ref, right_ref, cam stamp */

  /* Optional BracketedDepthError residual blocks (rig_calibrator.cc:522-609),
   * added by rig_calibrator.cc:1755-1791 when --depth_tri_weight > 0. Each must
   * share (beg, end, ref_to_cam, offset, stamps) with at least one
   * BracketedCamError block (the image the depth cloud belongs to). Zero-fill
   * these fields when there are none. */
  int64_t num_depth_residuals;
  const int32_t* depth_blocks;   /* [7*n] beg, end, ref_to_cam, depth_to_image (7 rigid | 12 affine),
                                    scale (1), xyz (3), offset (1): MVBA_DBLK_* order.
                                    xyz = -1 marks a BracketedDepthMeshError block
                                    (rig_calibrator.cc:615-705, added by :1796-1834 with
                                    --mesh and --depth_mesh_weight): r = weight *
                                    (mesh_xyz - M), mesh_xyz from depth_mesh_xyz. Both
                                    kinds share this list in AddResidualBlock order. */
  const double* depth_meas;      /* [3*n] meas_depth_xyz (depth-cloud point) */
  const double* depth_weight;    /* [n] weight (FLAGS_depth_tri_weight) */
  const double* depth_stamps;    /* [3*n] left_ref, right_ref, cam stamp */

  /* Optional XYZError residual blocks (rig_calibrator.cc:709-751): r = weight *
   * (xyz - ref_xyz) on one point block, with their own Cauchy threshold:
   * --tri_weight / --tri_robust_threshold (:1889-1898) or --mesh_tri_weight /
   * --robust_threshold (:1866-1877). Zero-fill when there are none. */
  int64_t num_xyz_residuals;
  const int32_t* xyz_block;      /* [n] point block id (size 3) */
  const double* xyz_ref;         /* [3*n] reference xyz */
  const double* xyz_weight;      /* [n] weight */
  const double* xyz_threshold;   /* [n] Cauchy threshold used with MVBA_EVAL_APPLY_LOSS (> 0) */

  /* ABI 5. [3*num_depth_residuals], nullable when no depth block has xyz = -1:
   * the fixed mesh point of each BracketedDepthMeshError block (rows of other
   * blocks are ignored). */
  const double* depth_mesh_xyz;
  /* ABI 5. [num_xyz_residuals], nullable (all 0): 0 = "tri" prior (--tri_weight,
   * :1880-1898), 1 = "mesh_tri" prior (--mesh_tri_weight, :1857-1877). Only the
   * residual statistics' grouping reads it. */
  const uint8_t* xyz_kind;
} mvba_problem_desc;

/* Depth block order (BracketedDepthError) and its Jacobian layout: rows
 * MVBA_DJAC_BASE_b + i*size_b + j = entry (residual row i, column j) of block b,
 * i.e. Ceres' row-major 3 x size_b block concatenated, with depth_to_image always
 * given 12 columns of room (a rigid 7-parameter block uses the first 21 rows). */
enum {
  MVBA_DBLK_BEG = 0,
  MVBA_DBLK_END = 1,
  MVBA_DBLK_REF_TO_CAM = 2,
  MVBA_DBLK_DEPTH_TO_IMAGE = 3,
  MVBA_DBLK_SCALE = 4,
  MVBA_DBLK_XYZ = 5,
  MVBA_DBLK_OFFSET = 6
};
#define MVBA_DJAC_BASE_BEG 0
#define MVBA_DJAC_BASE_END 21
#define MVBA_DJAC_BASE_REF_TO_CAM 42
#define MVBA_DJAC_BASE_DEPTH_TO_IMAGE 63
#define MVBA_DJAC_BASE_SCALE 99
#define MVBA_DJAC_BASE_XYZ 102
#define MVBA_DJAC_BASE_OFFSET 111
#define MVBA_DJAC_ROWS 114

typedef struct mvba_options {
  int32_t device;        /* HIP device ordinal */
  int32_t reserved0;
  double reserved1;
} mvba_options;

/* Evaluation flags. */
#define MVBA_EVAL_RESIDUALS 0x1
#define MVBA_EVAL_JACOBIAN 0x2
/* Apply the Cauchy loss through the Ceres corrector (r*sqrt(rho'), J*sqrt(rho')).
 * Without it residuals/Jacobians are raw, as a ceres::CostFunction returns them. */
#define MVBA_EVAL_APPLY_LOSS 0x4
/* Phase control of mvba_evaluate_device (for timing the kernels separately):
 * PREP_ONLY runs only the point gather and the per-frame kernel (K0);
 * SKIP_PREP runs only the per-observation kernels (K1), reusing the frame
 * records of the previous evaluation (parameters must be unchanged since). */
#define MVBA_EVAL_PREP_ONLY 0x8
#define MVBA_EVAL_SKIP_PREP 0x10

/* Device view of the last evaluation (device order = grouped by camera model,
 * then by image frame; see DESIGN.md "HBM layout"). */
typedef struct mvba_device_view {
  int64_t num_residuals;
  int64_t num_slots;       /* device slots (residuals + line-alignment padding) */
  int64_t ld;              /* leading dimension (elements) of residual/Jacobian planes */
  int32_t jac_rows;        /* 56 + 2*K_max rows per residual */
  int32_t max_dist_size;   /* K_max */
  double* residuals;       /* [2][ld]  plane 0 = x residual, plane 1 = y residual */
  double* jacobian;        /* [jac_rows][ld] column planes */
  const int64_t* order;    /* [num_slots] device slot -> AddResidualBlock index, -1 = padding */
  const uint8_t* row_written; /* [num_slots] bit b set = block b written (non-constant) */
} mvba_device_view;

/* Library / device queries. */
int mvba_abi_version(void);
mvba_status mvba_device_count(int32_t* count);

/* Create a handle: validates block sizes and distortion sizes (the reference's
 * constructor checks), groups residual blocks into image frames and uploads
 * the static topology to HBM. */
mvba_status mvba_create(const mvba_problem_desc* desc, const mvba_options* opts,
                        struct mvba_handle** out);
void mvba_destroy(struct mvba_handle* h);
const char* mvba_last_error(const struct mvba_handle* h);
/* Error text of the last failed mvba_create (thread-local). */
const char* mvba_create_error(void);

/* Upload the packed parameter vector (num_param_doubles doubles, host). */
mvba_status mvba_set_params(struct mvba_handle* h, const double* packed_params);
/* Same, from device memory (e.g. a GPU-resident solver's state), on stream. */
mvba_status mvba_set_params_device(struct mvba_handle* h, const double* d_packed_params,
                                   void* hip_stream);

/* Evaluate all residual blocks. Host outputs in AddResidualBlock order.
 *   cost      : nullable; 0.5*sum(r^2), or sum 0.5*rho(|r|^2) with APPLY_LOSS
 *   residuals : nullable; [2*num_residuals]
 *   jacobian  : nullable; [num_residuals * jac_stride] Ceres layout
 *               (MVBA_JAC_BASE_*), constant blocks zero-filled,
 *               jac_stride = mvba_jacobian_stride(h).
 * Blocks until the results are on the host. */
mvba_status mvba_evaluate(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                          double* cost, double* residuals, double* jacobian);
int32_t mvba_jacobian_stride(const struct mvba_handle* h);

/* ---- Host hand-over (the ceres::CostFunction surface) --------------------
 * mvba_evaluate / mvba_evaluate_packed / mvba_evaluate_depth rewrite the
 * device's column planes into AddResidualBlock-order rows ON THE DEVICE and
 * move them with one device-to-host copy (rig_calibrator.cc:1695-1699 is the
 * layout Ceres consumes). Outputs in pinned memory (mvba_host_alloc, or a
 * caller's hipHostRegister) are DMA targets; pageable outputs go through the
 * library's pinned double buffer. */
void* mvba_host_alloc(size_t bytes);  /* pinned host memory, NULL on failure */
void mvba_host_free(void* p);
/* Packed Jacobian: only the columns of the parameter blocks with transfer[b]
 * != 0 (num_blocks bytes; NULL = every non-constant block). Residual block i's
 * entries start at offsets[i] (num_residuals + 1 int64, nullable; rows are
 * stored in the device's frame order, so offsets are not increasing in i;
 * offsets[num_residuals] = the total) and hold, in block-position order
 * (MVBA_BLK_*), the row-major 2 x size_b Jacobian of each transferred block it
 * references (zero if that block is constant).
 * Replaces CostFunction::Evaluate's per-block jacobians[b] (NULL for the blocks
 * Ceres holds constant), so blocks nobody asks for never cross PCIe. */
mvba_status mvba_set_transfer_blocks(struct mvba_handle* h, const uint8_t* transfer, int64_t* offsets);
int64_t mvba_packed_size(const struct mvba_handle* h); /* doubles; -1 before mvba_set_transfer_blocks */
/* Like mvba_evaluate with the packed Jacobian layout (mvba_packed_size doubles). */
mvba_status mvba_evaluate_packed(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                 double* cost, double* residuals, double* packed_jacobian);

/* Device-resident evaluation (no host transfer). Outputs go to the library's
 * buffers (see mvba_device_buffers) or, if d_residuals/d_jacobian are non-null,
 * into caller-owned device memory with leading dimension ld (>= mvba_num_slots(),
 * multiple of 16; base pointers 128-byte aligned).
 * Asynchronous on hip_stream (NULL = default stream). Errors raised by the
 * kernels (interpolation alpha out of range) are reported by mvba_sync_status(). */
mvba_status mvba_evaluate_device(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                 double* d_residuals, double* d_jacobian, int64_t ld,
                                 void* hip_stream);
mvba_status mvba_device_buffers(struct mvba_handle* h, mvba_device_view* view);
/* fp32 output of the same evaluation ("fp32 eval, fp64
 * solve"): identical fp64 arithmetic, each residual/Jacobian value rounded once
 * to float at the store, half the output bytes. Caller-owned float planes with
 * the same layout and ld rules as mvba_evaluate_device. */
mvba_status mvba_evaluate_device_f32(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                     float* d_residuals, float* d_jacobian, int64_t ld, void* hip_stream);
/* Host copy of the device order: out[p] = AddResidualBlock index of device
 * slot p, -1 for padding (mvba_num_slots() int64). */
mvba_status mvba_residual_order(const struct mvba_handle* h, int64_t* out);
/* Wait for the stream and convert any device-side error word into a status. */
mvba_status mvba_sync_status(struct mvba_handle* h, void* hip_stream);

/* ---- Normal equations (K2): gradient and block-diagonal Hessian ----------
 * For the solver (Ceres' Jacobi preconditioner of ITERATIVE_SCHUR, and the
 * RCCL all-reduce of per-pose blocks when observations are sharded by landmark).
 * With J the Jacobian of the (optionally Cauchy-corrected) residuals r:
 *   gradient g = J^T r, Hessian blocks H_bb = J_b^T J_b per parameter block b,
 * in two compact layouts:
 *   camera side: every non-constant, non-point block in block-id order;
 *     g at goff[b] (size_b doubles), H_bb row-major at hoff[b] (size_b^2);
 *   point side : point index p (mvba_point_block_map), g at 3p, H packed
 *     (xx xy xz yy yz zz) at 6p.
 * cost (nullable) = sum over residual blocks of 0.5*|r|^2 (or 0.5*rho). */
typedef struct mvba_lin_layout {
  int64_t cam_grad_size;   /* doubles */
  int64_t cam_hess_size;   /* doubles */
  int64_t num_points;
  int32_t num_cam_blocks;
  int32_t supported;       /* 0 if a camera model is outside the linearization (RPC degree > 6) */
} mvba_lin_layout;

mvba_status mvba_lin_layout_info(const struct mvba_handle* h, mvba_lin_layout* out);
/* [num_cam_blocks] each, nullable */
mvba_status mvba_cam_block_map(const struct mvba_handle* h, int32_t* block_ids, int64_t* goff,
                               int64_t* hoff);
/* [num_points]: parameter block id of point index p; -1 for the fixed point of
 * a BracketedDepthMeshError block (constant: zero gradient and Hessian) */
mvba_status mvba_point_block_map(const struct mvba_handle* h, int32_t* block_ids);
/* flags: MVBA_EVAL_APPLY_LOSS, MVBA_EVAL_SKIP_PREP, and for timing the two
 * sides separately MVBA_LIN_CAMERA_ONLY (camera-side gradient, block Hessians
 * and cost only; point outputs untouched, nullable) or MVBA_LIN_POINTS_ONLY.
 * The point side runs on a library stream beside the camera side and is
 * joined to hip_stream before the call's work on hip_stream completes.
 * Asynchronous on hip_stream. */
#define MVBA_LIN_CAMERA_ONLY 0x20
#define MVBA_LIN_POINTS_ONLY 0x40
/* Camera side summed in a fixed order (no fp64 atomics): bit-reproducible. */
#define MVBA_LIN_DETERMINISTIC 0x80
mvba_status mvba_linearize_device(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                  double* d_cam_grad, double* d_cam_hess, double* d_pt_grad,
                                  double* d_pt_hess, double* d_cost, void* hip_stream);
/* fp64 MFMA flops the camera-side Gram kernel issues per linearization
 * (v_mfma_f64_16x16x4: 2048 flops each, zero-padded tile columns included). */
double mvba_lin_mfma_flops(const struct mvba_handle* h);

/* ---- Depth residuals (BracketedDepthError) -------------------------------
 * Host: residuals [3n] and Jacobian [n * MVBA_DJAC_ROWS] (nullable) in depth
 * insertion order, Cauchy corrector applied with MVBA_EVAL_APPLY_LOSS, cost =
 * sum of 0.5*rho over depth blocks. Device: column planes res[3][ld],
 * J[MVBA_DJAC_ROWS][ld] in device order (mvba_depth_order), ld >=
 * mvba_num_depth_slots(), multiple of 16 (of 32 for fp32 outputs to keep every
 * plane on 128-B lines). mvba_evaluate / mvba_linearize_device
 * / mvba_solve include the depth blocks' cost and normal equations. */
int64_t mvba_num_depth_residuals(const struct mvba_handle* h);
int64_t mvba_num_depth_slots(const struct mvba_handle* h);
mvba_status mvba_depth_order(const struct mvba_handle* h, int64_t* out /* [num_depth_slots] */);
mvba_status mvba_evaluate_depth(struct mvba_handle* h, int32_t flags, double cauchy_threshold, double* cost,
                                double* residuals, double* jacobian);
mvba_status mvba_evaluate_depth_device(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                       double* d_res, double* d_J, int64_t ld, void* hip_stream);
/* fp32 output of the depth evaluation (same rules as mvba_evaluate_device_f32). */
mvba_status mvba_evaluate_depth_device_f32(struct mvba_handle* h, int32_t flags, double cauchy_threshold,
                                           float* d_res, float* d_J, int64_t ld, void* hip_stream);

/* ---- XYZ priors (XYZError) ---------------------------------------------
 * Host, insertion order: residuals [3n], Jacobian [9n] (row-major 3x3, nullable),
 * cost = sum 0.5*rho (each block's own threshold with MVBA_EVAL_APPLY_LOSS).
 * mvba_linearize_device and mvba_solve include them (point blocks only). */
int64_t mvba_num_xyz_residuals(const struct mvba_handle* h);
mvba_status mvba_evaluate_xyz(struct mvba_handle* h, int32_t flags, double* cost, double* residuals,
                              double* jacobian);

/* ---- Tracks: triangulation and outlier flagging --------
 * Per optimisation pass rig_calibrator re-triangulates every track from the
 * current cameras (multiViewTriangulation, interest_point.cc:649-722:
 * undistort each inlier keypoint with Convert<DISTORTED, UNDISTORTED_C>, then
 * openMVG::Triangulation::compute(3), triangulation_nview.cc:87-150, with
 * P = diag(f, f, 1) [R | t]) and afterwards flags outliers by triangulation
 * angle and reprojection error (flagOutliersByTriAngleAndReprojErr,
 * rig_calibrator.cc:1045-1154). Both are one GPU thread per track. */
typedef struct mvba_tracks_desc {
  int32_t num_images;
  const double* world_to_cam;    /* [12*num_images]: R row-major (9), then t (3) */
  const int32_t* image_camera;   /* [num_images] camera model index */
  int32_t num_cameras;
  const double* focal;           /* [num_cameras] */
  const double* center;          /* [2*num_cameras] optical offset */
  const int32_t* dist_size;      /* [num_cameras] K (RPC: [dist | undist], 2x the coefficients) */
  const int64_t* dist_offset;    /* [num_cameras] into dist */
  const double* dist;            /* packed distortion vectors */
  const double* dist_half;       /* [2*num_cameras] distorted half size */
  const double* undist_half;     /* [2*num_cameras] undistorted half size */
  int64_t num_points;
  const int64_t* track_begin;    /* [num_points+1] */
  const int32_t* track_image;    /* [num_obs] image of each feature (increasing within a track) */
  const double* track_pix;       /* [2*num_obs] keypoint (distorted pixel) */
} mvba_tracks_desc;

/* inlier [num_obs] in/out (0/1); xyz [3*num_points] out. Tracks with < 2 inlier
 * rays, or a non-finite solution, get all their features flagged outliers; their
 * xyz is left as in the reference (0 for < 2 rays, the non-finite value otherwise). */
mvba_status mvba_triangulate(const mvba_tracks_desc* d, int32_t device, uint8_t* inlier, double* xyz);
/* residuals [2*num_obs]: the pixel residual of each feature (evalResiduals after
 * the solve; only read for inliers). counts[4] out: outliers by angle, features
 * seen by the angle pass, outliers by reprojection error, features seen by the
 * reprojection pass. */
mvba_status mvba_flag_outliers(const mvba_tracks_desc* d, int32_t device, const double* xyz,
                               const double* residuals, double min_triangulation_angle,
                               double max_reprojection_error, uint8_t* inlier, int64_t* counts);
/* world_to_cam of every frame (image) at the handle's current parameters, from
 * the K0 frame records: out [12*num_frames] (R row-major, t); frame_of_residual
 * [num_residuals] (nullable): the frame of each BracketedCamError block in
 * AddResidualBlock order. Synchronous. */
mvba_status mvba_frame_poses(struct mvba_handle* h, double* out, int32_t* frame_of_residual);
/* Message of the last failed mvba_triangulate / mvba_flag_outliers on this thread. */
const char* mvba_tracks_error(void);

/* ---- Mesh constraints (--mesh) ----------------------
 * The reference loads a PLY mesh and builds rayint's BVH over it
 * (loadMeshBuildTree, texture_processing.cc:264-285), then per pass intersects
 * every inlier feature's ray with it (meshTriangulations,
 * texture_processing.cc:1566-1625 -> ray_mesh_intersect, :1436-1479): the ray
 * leaves the camera centre through the undistorted pixel, in float (rayint's
 * Ray: origin, unit dir, tmin = --min_ray_dist, tmax = --max_ray_dist), and the
 * closest hit t gives intersection = cam_ctr + t * world_ray (double). Each
 * track's mesh point is the mean of its features' hits; features that are
 * outliers or miss keep `bad` = (1e100, 1e100, 1e100) (:1546), as do tracks
 * without any hit. Those feed BracketedDepthMeshError blocks and "mesh_tri"
 * XYZError priors.
 * Here the BVH is built on the host once per mesh (median splits, leaves of <= 4
 * triangles, depth <= 31) and traversed on the GPU, one lane per ray. */
typedef struct mvba_mesh_desc {
  int64_t num_vertices;
  const float* vertices;   /* [3*num_vertices] x y z (mve's Vec3f) */
  int64_t num_faces;
  const uint32_t* faces;   /* [3*num_faces] vertex indices */
} mvba_mesh_desc;
struct mvba_mesh;
mvba_status mvba_mesh_create(const mvba_mesh_desc* d, int32_t device, struct mvba_mesh** out);
void mvba_mesh_destroy(struct mvba_mesh* m);
/* BVH size (nodes) and depth, for reporting. */
mvba_status mvba_mesh_info(const struct mvba_mesh* m, int64_t* num_nodes, int32_t* depth);
/* Closest hit of n rays (device buffers, float, rayint's Ray): orig/dir [3n]
 * (dir unit length), hit parameter t_out [n] (-1 = no hit in [tmin, tmax]) and
 * face_out [n] (-1 = none; ties in t go to the lower face index). Asynchronous
 * on hip_stream. */
mvba_status mvba_mesh_intersect_device(struct mvba_mesh* m, int64_t n, const float* d_orig, const float* d_dir,
                                       float tmin, float tmax, float* d_t, int32_t* d_face, void* hip_stream);
/* meshTriangulations over a tracks description (same rules as mvba_triangulate):
 * inlier [num_obs] in; feature_xyz [3*num_obs] out (nullable); point_xyz
 * [3*num_points] out. Synchronous. */
mvba_status mvba_mesh_triangulate(const mvba_tracks_desc* d, struct mvba_mesh* m, const uint8_t* inlier,
                                  double min_ray_dist, double max_ray_dist, double* feature_xyz,
                                  double* point_xyz);
/* Message of the last failed mvba_mesh_* call on this thread. */
const char* mvba_mesh_error(void);

/* ---- Residual statistics (evalResiduals + calc_residuals_stats,
 * rig_calibrator.cc:1157-1180, :753-789) ------------------------------------
 * Raw residuals (no loss) divided by their scale (1 for pixels, the depth weight
 * for depth blocks), |r| grouped by residual name, and per group the values at
 * sorted positions int(0.25 len), int(0.5 len), int(0.75 len), len-1.
 * Groups (num_cameras*2 + 12): 2c + k = camera c, pixel component k
 * ("<sensor>_pix_x", "<sensor>_pix_y"); 2*num_cameras + k = depth component k
 * ("depth_tri_{x,y,z}_m"); 2*num_cameras + 3 + k = XYZ prior component k
 * ("tri_{x,y,z}_m", scale = its weight); 2*num_cameras + 6 + k = mesh depth
 * block component k ("depth_mesh_{x,y,z}_m"); 2*num_cameras + 9 + k =
 * mesh_tri prior component k ("mesh_tri_{x,y,z}_m"). out [4*groups] (NaN for
 * empty groups), counts [groups].
 * Synchronous. */
mvba_status mvba_residual_stats(struct mvba_handle* h, double* out, int64_t* counts, void* hip_stream);

/* mvba_eval_bytes(h, MVBA_EVAL_DEPTH): algorithmic bytes of one materialised
 * depth evaluation (per block 32 meas+weight, 24 landmark, 24 residual, 24 per
 * written Jacobian column). */
#define MVBA_EVAL_DEPTH 0x100

/* Counts for reporting. */
int64_t mvba_num_residuals(const struct mvba_handle* h);
/* Device slots = residuals + padding that line-aligns every frame's range (32
 * slots); device output planes need ld >= mvba_num_slots(), ld a multiple of 16
 * (of 32 for fp32 outputs to keep every plane on 128-B lines). Padding slots
 * that share a 128-B line with a frame's last residual receive a copy of it
 * (whole-line stores); no entry point reads them back. */
int64_t mvba_num_slots(const struct mvba_handle* h);
int64_t mvba_num_frames(const struct mvba_handle* h);
int64_t mvba_num_points(const struct mvba_handle* h);
/* Algorithmic HBM bytes of one materialised evaluation (residual+Jacobian),
 * per DESIGN.md: per residual 16 (meas) + 4 (point index) + 24 (point) +
 * 16 (residual) + 16 * (written Jacobian columns). With MVBA_EVAL_PREP_ONLY:
 * the prep's bytes (per landmark 65: parameters, offset, free flag, record
 * store; per frame 1,456: descriptor, pose parameters, 144-double record). */
double mvba_eval_bytes(const struct mvba_handle* h, int32_t flags);

/* The launch form a full mvba_evaluate_device takes on this handle (ABI 6):
 * MVBA_FORM_SPLIT = prep launch + one K1 launch per model group (several
 * camera models, or one model past 24 segments of 64 observations per image,
 * where recomputing the frame record in every wave costs more than the prep
 * launch); MVBA_FORM_FUSED = one k_eval launch (K0 blocks hand the frame
 * records to the K1 waves of the same grid; MVBA_EVAL_MODE=fused);
 * MVBA_FORM_LOCAL = one k_eval_local launch (each K1 wave computes its frame's
 * record; the default for one camera model up to that density). */
enum { MVBA_FORM_SPLIT = 0, MVBA_FORM_FUSED = 1, MVBA_FORM_LOCAL = 2 };
int32_t mvba_eval_form(const struct mvba_handle* h);

/* ---- Solver: GPU-resident Levenberg-Marquardt ----------------------------
 * Replaces ceres::Solve(options, &problem, &summary) of rig_calibrator.cc:1910-1919
 * (linear_solver_type = ITERATIVE_SCHUR, gradient/function tolerance 1e-16,
 * parameter_tolerance = FLAGS_parameter_tolerance, max_num_iterations =
 * FLAGS_num_iterations) for a problem made of BracketedCamError blocks.
 * Trust-region LM with Ceres 1.14's step control, Jacobi column scaling and
 * stopping rules [ext]; the reduced camera system is solved matrix-free by
 * preconditioned CG on the implicit Schur complement (points eliminated).
 * The solution is left in the handle's parameters (mvba_get_params).
 *
 * Sharded solves: each rank's handle holds all camera-side
 * blocks and the observations of its landmark range; `allreduce` (non-null)
 * is called with an in-place device buffer to sum (op MVBA_REDUCE_SUM) or max
 * (MVBA_REDUCE_MAX) across ranks. The call is STREAM-ORDERED: the library
 * does not synchronise before it, and the reduction must be enqueued on
 * hip_stream so that work enqueued after the call sees the result (e.g.
 * ncclAllReduce on that stream: mvba_comm_allreduce below). A callback that
 * works on the host must synchronise hip_stream itself before reading the
 * buffer and leave the result there before returning. Every rank must obtain
 * bit-identical results (the camera-side CG state is replicated and its
 * device-side stopping decisions must agree, or the collectives fall out of
 * step). It is called once per linearization (camera gradient + block
 * Hessians + cost), once per CG iteration (the reduced-system product, also
 * for iterations the device has gated off past the CG stop) and for a few
 * scalars per LM step. */
enum { MVBA_REDUCE_SUM = 0, MVBA_REDUCE_MAX = 1 };
typedef int32_t (*mvba_allreduce_fn)(double* device_buf, int64_t count, int32_t op, void* hip_stream,
                                     void* user);

/* Communicators for sharded solves (mvba_comm.hip). Pass
 * `allreduce = mvba_comm_allreduce, allreduce_user = comm` in the solver
 * options.
 *   RCCL, one process per GPU: rank 0 calls mvba_comm_unique_id and the caller
 *   broadcasts the MVBA_COMM_ID_BYTES bytes (e.g. torch.distributed); every
 *   rank then calls mvba_comm_init_rccl (collective: returns once all joined).
 *   The RCCL communicator is non-blocking (ncclConfig_t.blocking = 0): its init
 *   and every collective enqueue are polled against a deadline
 *   (mvba_comm_init_rccl_deadline; mvba_comm_init_rccl uses MVBA_COMM_TIMEOUT_S,
 *   else 300 s), and past it the communicator is aborted and the call fails
 *   (mvba_comm_error says why) instead of hanging the rank.
 *   Local, several shards in one process (one host thread and one HIP stream
 *   per shard; shards may share a device): mvba_comm_init_local fills
 *   comms[nranks]; the all-reduce meets the other shards' threads at enqueue
 *   time only and sums the shards' buffers on the device in rank order.
 * mvba_comm_abort releases every rank of a failed solve (RCCL: ncclCommAbort;
 * local: the waiting threads return failure); it may be called from another
 * thread while the owner waits on the solver's stream (a watchdog). */
#define MVBA_COMM_ID_BYTES 128
typedef struct mvba_comm mvba_comm;
mvba_status mvba_comm_unique_id(uint8_t* id /* [MVBA_COMM_ID_BYTES] */);
mvba_status mvba_comm_init_rccl(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, mvba_comm** out);
mvba_status mvba_comm_init_rccl_deadline(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                                         double timeout_s /* <= 0: the default */, mvba_comm** out);
mvba_status mvba_comm_init_local(int32_t nranks, const int32_t* devices, mvba_comm** comms /* [nranks] */);
mvba_status mvba_comm_abort(mvba_comm* comm);
void mvba_comm_destroy(mvba_comm* comm);
int32_t mvba_comm_rank(const mvba_comm* comm);
int32_t mvba_comm_size(const mvba_comm* comm);
const char* mvba_comm_error(void);
int32_t mvba_comm_allreduce(double* device_buf, int64_t count, int32_t op, void* hip_stream, void* comm);

enum { MVBA_CONVERGENCE = 0, MVBA_NO_CONVERGENCE = 1, MVBA_FAILURE = 2 };

typedef struct mvba_solver_options {
  int32_t max_num_iterations;          /* Solver::Options default 50; rig_calibrator passes its flag */
  double function_tolerance;           /* 1e-16 in rig_calibrator (:1916) */
  double gradient_tolerance;           /* 1e-16 (:1915) */
  double parameter_tolerance;          /* FLAGS_parameter_tolerance (:1917) */
  double initial_trust_region_radius;  /* 1e4 */
  double max_trust_region_radius;      /* 1e16 */
  double min_trust_region_radius;      /* 1e-32 */
  double min_lm_diagonal;              /* 1e-6 */
  double max_lm_diagonal;              /* 1e32 */
  double min_relative_decrease;        /* 1e-3 */
  double eta;                          /* 0.1: CG q-criterion tolerance */
  int32_t min_linear_solver_iterations; /* 0 */
  int32_t max_linear_solver_iterations; /* 500 */
  int32_t max_num_consecutive_invalid_steps; /* 5 */
  int32_t jacobi_scaling;              /* 1 */
  int32_t use_loss;                    /* Cauchy loss on every residual block */
  double robust_threshold;             /* CauchyLoss(robust_threshold) (rig_calibrator.cc:394-411) */
  const double* lower_bounds;          /* host, [num_param_doubles] or NULL (-inf) */
  const double* upper_bounds;          /* host, [num_param_doubles] or NULL (+inf) */
  int32_t progress_to_stdout;          /* minimizer_progress_to_stdout (:1914) */
  mvba_allreduce_fn allreduce;         /* NULL: single rank */
  void* allreduce_user;
  int32_t deterministic;               /* 1: no fp64 atomics in the normal equations and the
                                          Schur products (fixed-order slab gathers): two runs
                                          give bit-identical CG counts and parameters, at some
                                          cost per CG iteration. Default 0. */
} mvba_solver_options;

typedef struct mvba_solver_summary {
  double initial_cost;
  double final_cost;
  int32_t num_iterations;              /* LM iterations after iteration 0 */
  int32_t num_successful_steps;
  int32_t num_unsuccessful_steps;
  int32_t num_linear_iterations;       /* total CG iterations */
  int32_t termination_type;            /* MVBA_CONVERGENCE / NO_CONVERGENCE / FAILURE */
  int32_t cg_graph_launches;           /* captured CG runs replayed (hipGraphLaunch); 0: every CG kernel
                                          launched eagerly (was padding: same layout) */
  double total_time_s;
  double linearize_time_s;             /* Jacobian / normal equations (incl. exchange) */
  double linear_solver_time_s;         /* CG + back-substitution */
  double eval_time_s;                  /* candidate-point cost evaluations */
  char message[256];
} mvba_solver_summary;

void mvba_solver_default_options(mvba_solver_options* o);
/* Runs LM from the handle's current parameters (mvba_set_params first).
 * Host-synchronous: returns when the solve is done. hip_stream: the stream the
 * solve runs on. NULL with a single-rank solve (allreduce NULL): the library
 * waits for all earlier device work (hipDeviceSynchronize) and runs on its own
 * per-device stream, whose CG iterations it can capture and replay as graphs
 * (the null stream cannot be captured); likewise a solve sharded over an
 * RCCL communicator (mvba_comm_init_rccl: one process per device). NULL with
 * any other sharded solve: the null stream itself. */
mvba_status mvba_solve(struct mvba_handle* h, const mvba_solver_options* o, mvba_solver_summary* summary,
                       void* hip_stream);
/* Copy the handle's current packed parameter vector to host memory. */
mvba_status mvba_get_params(struct mvba_handle* h, double* packed);

/* ---- RPC lens-model fitting -----------------------
 * fitRpcUndist (rpc_distortion.cc:658-721), as run by
 * CameraParameters::updateRpcUndistortion (camera_params.cc:214-253) after a
 * pass that floated RPC distortion (rig_calibrator.cc:1946-1948), and
 * fitRpcDist (:622-656, the fit_rpc tool). Samples the undistorted image on a
 * num_samples^2 grid (genUndistDistPairs, :519-557; samples whose distorted
 * pixel leaves the distorted crop box are dropped), then fits RPC coefficients
 * of degree 1, 2, ..., rpc_degree, each degree starting from the previous fit
 * (identity at degree 1), by Levenberg-Marquardt with Ceres 1.14's step
 * control, gradient/function tolerance 1e-16, the given parameter tolerance and
 * iteration cap per degree.
 *   MVBA_RPC_FIT_UNDISTORTION: fits undist with undist(rpc(u, dist)) ~ u, where
 *     dist = rpc_dist_coeffs (2 (d+1)(d+2) - 2 values, degree rpc_degree);
 *   MVBA_RPC_FIT_DISTORTION: fits rpc(u) ~ the camera's distorted pixel
 *     (any distortion model of the camera).
 * coeffs_out: 2 (d+1)(d+2) - 2 values (RPCLensDistortion layout). Synchronous. */
enum { MVBA_RPC_FIT_DISTORTION = 0, MVBA_RPC_FIT_UNDISTORTION = 1 };
typedef struct mvba_rpc_camera {
  double focal;
  double center[2];            /* optical offset */
  int32_t dist_size;           /* GetDistortion().size() (RPC: [dist | undist]) */
  const double* dist;
  int32_t image_size[2];       /* distorted size */
  int32_t crop_size[2];        /* distorted crop size */
  int32_t undist_size[2];      /* undistorted size */
} mvba_rpc_camera;
typedef struct mvba_rpc_fit_report {
  int64_t num_samples_used;
  double undist_box[4];        /* centred undistorted pixels: min x, min y, max x, max y */
  double dist_box[4];          /* centred distorted pixels */
  double initial_cost[6];      /* per degree 1..6 */
  double final_cost[6];
  int32_t iterations[6];
  int32_t termination[6];      /* MVBA_CONVERGENCE / NO_CONVERGENCE / FAILURE */
  double max_dist_undist_error; /* evalRpcDistUndist (:723-737), UNDISTORTION mode; -1 otherwise */
} mvba_rpc_fit_report;
mvba_status mvba_rpc_fit(const mvba_rpc_camera* cam, int32_t mode, int32_t rpc_degree,
                         const double* rpc_dist_coeffs, int32_t num_samples, int32_t num_iterations,
                         double parameter_tolerance, int32_t device, double* coeffs_out,
                         mvba_rpc_fit_report* report);
/* Message of the last failed mvba_rpc_fit on this thread. */
const char* mvba_rpc_error(void);

#ifdef __cplusplus
}
#endif

#endif /* MVBA_MVBA_H_ */
