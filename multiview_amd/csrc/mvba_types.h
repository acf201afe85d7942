// mvba_types.h — host/device shared records of the MI355X evaluator.
// See DESIGN.md "HBM layout" for how these are laid out in device memory.
#ifndef MVBA_TYPES_H_
#define MVBA_TYPES_H_

#include <stdint.h>

namespace mvba {

// Per image frame (one unique set of pose blocks, intrinsics blocks and stamps;
// calc_world_to_cam_trans depends only on these, rig_calibrator.cc:362-390,
// called per image at :1633-1651). 128 bytes, read with scalar loads.
struct FrameDesc {
  int64_t off[8];      // offsets of the 8 parameter blocks in the packed vector (off[3] unused)
  double sb, se, sc;   // left_ref_stamp, right_ref_stamp, cam_stamp
  double h0, h1;       // distorted half size (camera_params.cc:107-110)
  int32_t cam;         // camera model index
  int32_t K;           // distortion length
  int32_t free_mask;   // bit b: block b is not constant (b != 3)
  int32_t pad;
};

// K0 output per frame, in doubles:
//   [0..8]   R_wc row-major      [9..11]  t_wc
//   [12 + 6k .. 12 + 6k + 5] for pose column k (22 columns:
//        beg tx ty tz qx qy qz qw | end (7) | ref_to_cam (7) | offset (1)):
//        omega_k (3), v_k (3), with d(Xc)/dp_k = omega_k x Xc + v_k.
constexpr int kFrameRecDoubles = 144;

// Per-frame projection record for the solver's point-order pass (built once per
// linear solve, the parameters being fixed during CG), so one observation needs
// two independent loads (this record and the frame's CG direction) instead of
// the frame descriptor -> parameter vector chain:
//   [0..11] R_wc, t_wc | 12 f | 13, 14 optical centre | 15, 16 half size |
//   17 K (as double) | 18.. live distortion coefficients (<= kProjDist)
constexpr int kProjDoubles = 128;
constexpr int kProjDist = kProjDoubles - 18;
constexpr int kPoseCols = 22;

// A segment = up to 64 consecutive device-order residuals of ONE frame,
// processed by one wavefront (frame data is wave-uniform -> scalar loads).
struct Segment {
  int32_t begin;
  int32_t count;
  int32_t frame;
  int32_t pad;
};

// Distortion model kinds (camera_params.cc:181-207 dispatch by size).
enum ModelKind : int32_t {
  kModelNone = 0,    // K = 0
  kModelFov = 1,     // K = 1
  kModelRadtan = 2,  // K = 4 or 5
  kModelRpc = 3      // K = 2 * (2 (d+1)(d+2) - 2)
};

constexpr int kMaxRpcDegree = 6;
constexpr int kMaxLinRpcDegree = 6;
constexpr int kChunkSegs = 8;       // segments per solver chunk (one wave; 4 -> 8: c3 pass B 210 -> 197 us,
                                     // c2 23.1 -> 22.4 us, profiles/r04/r04o/)
#ifndef MVBA_PART_SEGS
#define MVBA_PART_SEGS 16
#endif
constexpr int kPartSegs = MVBA_PART_SEGS;  // segments per K2 frame part (one block)
constexpr int kDepthReplicas = 32;  // replicas the depth Gram adds into (frame-segment mod 32)

// Deterministic accumulation (mvba_solver_options.deterministic,
// MVBA_LIN_DETERMINISTIC): a producer (K2 frame part, solver chunk, depth
// segment) stores each of its contributions to a shared camera-side entry in
// its own slab row instead of adding it into a replica with an fp64 atomic;
// a gather kernel then sums every entry over its producers in a fixed order,
// so the result no longer depends on the order atomics arrive in.
struct Slab {
  double* val;        // [units x width]; null: replica atomics (default mode)
  int32_t* dst;       // record pass only: destination entry of every slab position
  int64_t width;      // doubles per unit
  int64_t unit_base;  // slab row of this launch's first unit
};
// Slab row layout of one K2 producer (frame part or depth segment): pose
// blocks beg / end / ref_to_cam at 56 b (7 gradient + 49 Hessian entries),
// offset at 168 (2), focal at 170 (2), centre at 172 (6), distortion at 178
// (K + K^2), cost in the last position; depth: depth_to_image gradient at 170
// (12), Hessian at 182 (144), scale at 326 (2).
constexpr int kSlabFocal = 170, kSlabCenter = 172, kSlabDist = 178;
constexpr int kSlabDti = 170, kSlabDtiHess = 182, kSlabScale = 326;
inline int64_t lin_slab_width(int kmax) {
  const int64_t w = kSlabDist + (int64_t)kmax + (int64_t)kmax * kmax + 1;
  return w > kSlabScale + 3 ? w : kSlabScale + 3;
}
// Solver pass B producers (chunk or depth segment): one position per lane of
// the final scatter: 22 pose columns, then focal, centre (2), distortion (K);
// depth segments: depth_to_image (12) at 22, scale at 34.
// Gather tiers by producer count (slab_gather): <= kSlabLight one thread,
// <= kSlabMedium one wave, more one block.
constexpr int kSlabLight = 16;
constexpr int kSlabMedium = 512;
struct SlabTiers {
  const int64_t* heavy;
  const int64_t* medium;
  const int64_t* light;
  int64_t nheavy, nmedium, nlight;
};
inline int64_t vec_slab_width(int kmax) { return 25 + kmax > 35 ? 25 + kmax : 35; }

// Per-frame record of the linearization (K2 expand); mirrors mvba::FrameLin in
// mvba_kernels.hip (checked with mvba_frame_lin_size()).
struct FrameLinHost {
  int64_t slab_off;
  int32_t chunk_count;
  int32_t width, w16;
  int32_t first_chunk;
  int64_t goff[8];
  int64_t hoff[8];
};

// Per BracketedDepthError residual (device order: sorted by frame), 64 bytes.
// The frame is the image whose pose blocks and stamps it shares (its world_to_cam
// and generators are the frame's K0 record).
struct DepthDesc {
  int64_t dti_off, scale_off;    // packed offsets of depth_to_image and scale
  int64_t goff_dti, goff_scale;  // camera-side gradient offsets (-1: constant)
  int64_t hoff_dti, hoff_scale;  // camera-side Hessian offsets
  int32_t frame, pid;            // frame record, point index
  int32_t dti_n;                 // 7 (rigid) or 12 (affine)
  int32_t free_mask;             // bits MVBA_DBLK_*: block is free (Jacobian written)
};

// Point-ordered views of the point-side residual blocks beyond BracketedCamError,
// passed by value to the point-order kernels:
//  * depth blocks: CSR point -> depth slots (begin == nullptr: none);
//  * XYZError priors: CSR point -> prior entries (xbegin == nullptr: none), entry
//    = (ref xyz, weight) + Cauchy c = 1/threshold^2.
struct PointExtra {
  const int64_t* begin;    // [num_points + 1]
  const int32_t* slot;     // [num_depth] depth slot of each entry
  const DepthDesc* dd;     // [depth slots]
  const void* meas;        // double4 [depth slots] (x, y, z, weight)
  const int64_t* xbegin;   // [num_points + 1]
  const void* xref;        // double4 [num_xyz] (x, y, z, weight), point order
  const double* xcc;       // [num_xyz] Cauchy c of each prior
};

// Device-resident control of one preconditioned-CG solve (single-rank solves):
// the scalar steps of conjugate_gradients_solver.cc [ext] run in the
// finalising block of the reductions, so the host enqueues iterations in
// batches without reading scalars back; `done` gates every kernel of the
// iterations enqueued past the stopping point.
struct CgCtl {
  int32_t done;     // 1: stopped (later iterations are no-ops)
  int32_t status;   // 0 converged, 1 no convergence (x usable), 2 failure
  int32_t iters;    // CgResult::iters
  int32_t first;    // next direction update is p = z
  double rho;       // r.z of the current iteration
  double beta;      // next direction update p = z + beta p
  double alpha;     // step of the current iteration
  double Q0;        // q-criterion state
  double eta;
  int32_t min_iter;
  int32_t max_iter;
  double rho_step;  // sharded solves: rho of the current step, snapshot by the replica reduction
  double bb;        // b.b of the linear solve (|b| = 0: converged at iteration 0, x = 0)
  int32_t it;       // next CG iteration number (the update kernel's finalisation counts on the device,
                    // so a captured iteration's launch arguments do not depend on its number)
  uint32_t mseq;    // mirror writes of this linear solve (CgMirror::seq)
};

// The CG state a batch of iterations ends in, written by the batch's last
// update launch straight into host-coherent pinned memory (no copy launch, no
// event): seq last, with a system-scope release, so the host that sees the seq
// it waits for sees the fields written before it.
struct CgMirror {
  int32_t done;
  int32_t status;
  int32_t iters;
  uint32_t seq;
};
constexpr int32_t kIterFromCtl = -2;  // k_cg_update iter argument: take it from CgCtl::it

// Camera-side entry of the reduced system as the CG update reads it: its
// block's first entry, the block size and the offset of the entry's row of
// the block-Jacobi inverse (one load per entry instead of a block-id chain).
struct CgEntry {
  int32_t o;
  int32_t nb;
  int64_t moff;
};

// The CG search direction formed where it is first read (k_frame_dir):
// p_new = z (first) or z + beta p_old, with first/beta from ctl when set.
struct LazyDir {
  const double* z;
  const double* p_old;
  double* p_new;
  int64_t n;
  const CgCtl* ctl;
  int32_t first;
  double beta;
};

// The frame direction records the CG passes read (dir[frame * kDirStride]: the
// frame's 6 pose sums w x | intrinsic entries). Outside CG iterations d = dz.
// Inside them d = W p_new with p_new = z (first) or z + beta p_old, formed as
// d = dz + beta dp from dz = W z (the CG update kernel's frame blocks) and
// dp = W p_old (the previous product's records, stored by pass A into dp_out),
// so no separate direction kernel runs between the update and pass A.
// With z set, only the 6 pose sums come from dz / dp: the intrinsic entries of
// d are the camera-side entries of p_new themselves, formed from the global
// vectors z and p_old (fl: the frame's block offsets), as the reduction that
// stores p_new forms them (the update's frame blocks then skip them: at RPC
// degree 2 they were 47 block-row products per frame, most of the update).
struct DirPair {
  const double* dz;
  const double* dp;  // null: d = dz
  double* dp_out;    // pass A: d stored here by one wave per frame (null: not stored)
  const CgCtl* ctl;  // first / beta
  const double* z = nullptr;      // intrinsic entries from z / p_old (null: from dz / dp)
  const double* p_old = nullptr;
  const void* fl = nullptr;       // FrameLin
  // set (with dz null): the pose sums W_f z are formed here from z and the
  // frame records (w_k per pose column) instead of read from dz, so the CG
  // update needs no frame blocks
  const double* frec = nullptr;
};

// The fused CG step (k_upd_pass_a: the update of iteration i-1 and pass A of
// iteration i in one launch). Pass A cannot know beta (the update's grid
// reduction finishes inside the same launch), so it forms both products
// c_z = J_pt^T J_cam d_z and c_p = J_pt^T J_cam d_p (d_z: the frame record of
// z = M^-1 r_new, recomputed by each wave from r, q and alpha; d_p: the
// previous direction's record) and the next launch combines them with beta:
// k_point_w sums c_z + beta c_p (cbuf: c_z | c_p.x, cbuf2: c_p.y, c_p.z) and its
// frame blocks store d = d_z + beta d_p for pass B and the next step.
struct FusedStep {
  const double* dz = nullptr;    // [frames * dir stride] z records (the fused pass A's writers)
  const double* dp = nullptr;    // previous direction records
  double* dp_out = nullptr;      // this iteration's direction records
  const FrameDesc* fd = nullptr;
  const void* fl = nullptr;      // FrameLin
  const CgCtl* ctl = nullptr;    // beta
  const double* cbuf2 = nullptr;  // [2 per slot] c_p.y, c_p.z
  int32_t nframes = 0;
  int32_t point_blocks = 0;      // k_point_w: blocks from here on are frame blocks
};

// Frame blocks of the CG update kernel: dz = W z for every frame, z = M^-1 r_new
// recomputed from the same inputs as the entry blocks (owner_blocks of them);
// the 6 pose sums only (pass A forms the intrinsic entries, DirPair::z).
struct FrameDirZ {
  const void* fl;  // FrameLin
  const FrameDesc* fd;
  const double* frec;
  double* dz;
  int32_t nframes;
  int32_t owner_blocks;
};

}  // namespace mvba

#endif  // MVBA_TYPES_H_
