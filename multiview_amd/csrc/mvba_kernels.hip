// mvba_kernels.hip — gfx950 kernels of the rig_calibrator evaluator.
//
//   k_prep    one launch of
//     K0 (frames): per image frame, world_to_cam (R_wc, t_wc) and the analytic
//               derivative generators of the 22 pose columns, 16 lanes per frame.
//               Restates calc_world_to_cam_trans / calc_interp_world_to_ref /
//               array_to_rigid_transform / linearInterp (rig_calibrator.cc:322-390,
//               dense_map_utils.cc:171-178, :315-329; Eigen 3.4 slerp [ext]);
//     point gather: xyz blocks of the packed parameter vector into 32-byte
//               records (x, y, z, free) — two 16 B loads per observation later.
//   k_obs<M>  (K1): per observation residual + analytic Jacobian, one lane per
//               observation, one wavefront per frame segment. Restates
//               BracketedCamError::operator() (rig_calibrator.cc:447-482) and
//               DistortCentered (camera_params.cc:260-314) / compute_rpc
//               (rpc_distortion.cc:116-160). Output: column planes in HBM.
//
// Derivation of the Jacobian (DESIGN.md "Analytic Jacobian"): every pose
// parameter p_k moves the camera by a left perturbation
//     dR_wc/dp_k = [w_k]x R_wc,   d(Xc)/dp_k = w_k x Xc + v_k,
// so per observation the 22 pose columns are  J_ik = (Xc x G_i).w_k + G_i.v_k
// with G = d(pixel)/d(Xc) (2x3). w_k, v_k depend only on the frame (K0).
#include "mvba_depth.h"

namespace mvba {

// ------------------------------------------------------------ prep (K0 + point gather)
// One launch: blocks [0, frame_blocks) run K0 with kThreadsPerFrame lanes per
// frame (each lane recomputes the frame's common part and emits a subset of the
// 22 pose columns); the remaining blocks gather the points.
constexpr int kThreadsPerFrame = 16;
#ifndef MVBA_K0_SHARE
#define MVBA_K0_SHARE 1  // k_eval_local: one K0 per frame and block (obs_body)
#endif
#ifndef MVBA_K0_LANES
#define MVBA_K0_LANES 32  // lanes of a k_eval_local wave running its frame's K0 (22 pose columns: one pass)
#endif
constexpr int kPrepBlock = 256;
#ifndef MVBA_PREP_POINTS
#define MVBA_PREP_POINTS 4
#endif
constexpr int kPrepPoints = MVBA_PREP_POINTS;  // landmarks gathered per thread

// WT: every store of the record write-through (agent-scope relaxed atomic
// store, `global_store ... sc1`): the fused evaluation hands the record to K1
// waves of the same launch (k_eval; MI355X_MICROARCH.md visibility, valid forms).
template <bool WT>
__device__ __forceinline__ void wr(double* p, double v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool WT>
__device__ __forceinline__ void put_col_wt(double* rec, int k, const double* om, const double* dt, const double* t) {
  double c[3];
  cross(om, t, c);
  double* o = rec + 12 + 6 * k;
  wr<WT>(o + 0, om[0]); wr<WT>(o + 1, om[1]); wr<WT>(o + 2, om[2]);
  wr<WT>(o + 3, dt[0] - c[0]); wr<WT>(o + 4, dt[1] - c[1]); wr<WT>(o + 5, dt[2] - c[2]);
}

// K0's common part split over the frame's lanes (MVBA_K0_SPLIT, default on):
// lane sub % 3 of the group builds the rigid transform (and quaternion) of the
// beg / end / ref_to_cam block and the sine and cosine of one of the three
// slerp angles, and the group takes each from its lane: one dependent chain
// instead of three, and (readlane) the common part's values in SGPRs:
// k_eval_local 148 -> 95 VGPRs, 3 -> 5 waves per SIMD. The same operations on
// the same values; the compiler's fp64 contractions around them differ, so the
// record moves by roundoff against the unsplit build (tools/k0_split_check.py)
// while every form, all built on frame_columns, still agrees bit for bit.
// BC: 0 every lane computes everything, 1 ds_bpermute within NT-lane groups
// (k_prep: 16 lanes per frame), 2 readlane (k_eval_local: one frame per wave,
// its lanes from lane 0). (profiles/r06/r06y: the c2 evaluation 121 -> 115 us
// with the Jacobian, 45 -> 37 us without; 32 K0 lanes: 114 / 35 us.)
#ifndef MVBA_K0_SPLIT
#define MVBA_K0_SPLIT 1
#endif
template <int BC, int NT>
__device__ __forceinline__ double from_lane(double v, int src) {
  if constexpr (BC == 2) return readlane_f64(v, src);
  else return __shfl(v, src, NT);
}

// NT: the lanes sharing the frame (lane sub takes columns sub, sub + NT, ...);
// BC: the common part's broadcast (above); stamp (probe builds): where lane 0
// records the end of the common part
template <bool WT, int NT = kThreadsPerFrame, int BC = (MVBA_K0_SPLIT ? 1 : 0)>
__device__ __forceinline__ void frame_columns(const FrameDesc& F, const double* __restrict__ params, double* rec,
                              int sub, int gen, int* err, unsigned long long* stamp = nullptr) {
  static_assert(BC == 0 || NT >= 3, "the split common part takes three lanes");
  const double* p0 = params + F.off[MVBA_BLK_BEG];
  const double t0[3] = {p0[0], p0[1], p0[2]};

  if (F.sb == F.se) {
    double R0[9], qh0[4], in0;
    rigid(p0, R0, qh0, &in0);
    // rig_calibrator.cc:371-374 — reference camera or --no_rig: T = rigid(p0).
    if (sub == 0) {
      for (int k = 0; k < 9; k++) wr<WT>(rec + k, R0[k]);
      wr<WT>(rec + 9, t0[0]); wr<WT>(rec + 10, t0[1]); wr<WT>(rec + 11, t0[2]);
    }
    for (int k = sub; k < kPoseCols; k += NT) {
      double om[3] = {0.0, 0.0, 0.0};
      // unit translation column by value (a dynamic index into dt would put the
      // array in scratch memory)
      double dt[3] = {k == 0 ? 1.0 : 0.0, k == 1 ? 1.0 : 0.0, k == 2 ? 1.0 : 0.0};
      if (k < 3) {
      } else if (k < 7) {
        quat_generator(qh0, 2.0 * in0, k - 3, om);
      }
      put_col_wt<WT>(rec, k, om, dt, t0);
    }
    return;
  }

  const double* p1 = params + F.off[MVBA_BLK_END];
  const double* p2 = params + F.off[MVBA_BLK_REF_TO_CAM];
  const double off = params[F.off[MVBA_BLK_OFFSET]];
  const double t1[3] = {p1[0], p1[1], p1[2]};
  const double t2[3] = {p2[0], p2[1], p2[2]};
  // linearInterp's quaternions of the beg / end rotations (Eigen slerp [ext])
  double qh0[4], in0, q0[4], qh1[4], in1, q1[4], R2[9], qh2[4], in2;
  if constexpr (BC == 0) {
    double R0[9], R1[9];
    rigid(p0, R0, qh0, &in0);
    rigid(p1, R1, qh1, &in1);
    rigid(p2, R2, qh2, &in2);
    rot_to_quat(R0, q0);
    rot_to_quat(R1, q1);
  } else {
    const int b = sub % 3;
    const double* pb = b == 0 ? p0 : b == 1 ? p1 : p2;
    double Rb[9], qhb[4], inb, qb[4];
    rigid(pb, Rb, qhb, &inb);
    rot_to_quat(Rb, qb);  // (ref_to_cam's lane: unused)
#pragma unroll
    for (int m = 0; m < 4; m++) {
      qh0[m] = from_lane<BC, NT>(qhb[m], 0);
      q0[m] = from_lane<BC, NT>(qb[m], 0);
      qh1[m] = from_lane<BC, NT>(qhb[m], 1);
      q1[m] = from_lane<BC, NT>(qb[m], 1);
      qh2[m] = from_lane<BC, NT>(qhb[m], 2);
    }
#pragma unroll
    for (int m = 0; m < 9; m++) R2[m] = from_lane<BC, NT>(Rb[m], 2);
    in0 = from_lane<BC, NT>(inb, 0);
    in1 = from_lane<BC, NT>(inb, 1);
    in2 = from_lane<BC, NT>(inb, 2);
  }

  // rig_calibrator.cc:343-346 (big stamps subtracted first).
  const double alpha = ((F.sc - F.sb) - off) / (F.se - F.sb);
  if (sub == 0 && (alpha < 0.0 || alpha > 1.0)) atomicMax(err, gen);

  // linearInterp with Eigen slerp [ext] (dense_map_utils.cc:315-329).
  const double sig0 = (q0[0] * qh0[0] + q0[1] * qh0[1] + q0[2] * qh0[2] + q0[3] * qh0[3]) >= 0.0 ? 1.0 : -1.0;
  const double sig1 = (q1[0] * qh1[0] + q1[1] * qh1[1] + q1[2] * qh1[2] + q1[3] * qh1[3]) >= 0.0 ? 1.0 : -1.0;
  const double d = q0[0] * q1[0] + q0[1] * q1[1] + q0[2] * q1[2] + q0[3] * q1[3];
  const double absD = fabs(d);
  double w0, w1, dw0_dth = 0.0, dw1_dth = 0.0, dw0_da, dw1_da, dth_dD = 0.0;
  if (absD >= 1.0 - DBL_EPSILON) {
    w0 = 1.0 - alpha;
    w1 = alpha;
    dw0_da = -1.0;
    dw1_da = 1.0;
  } else {
    const double th = acos(absD);
    double S, C, s0, c0, s1, c1;
    double iS;
    if constexpr (BC != 0) {
      // the three angles' sines and cosines on lanes 0 / 1 / 2 of the group
      const int b = sub % 3;
      const double x = b == 0 ? th : b == 1 ? (1.0 - alpha) * th : alpha * th;
      double sx, cx;
      if (MVBA_K0_FAST) {
        sincos(x, &sx, &cx);
      } else {
        sx = sin(x);
        cx = cos(x);
      }
      S = from_lane<BC, NT>(sx, 0);
      C = from_lane<BC, NT>(cx, 0);
      s0 = from_lane<BC, NT>(sx, 1);
      c0 = from_lane<BC, NT>(cx, 1);
      s1 = from_lane<BC, NT>(sx, 2);
      c1 = from_lane<BC, NT>(cx, 2);
      iS = 1.0 / S;
      w0 = MVBA_K0_FAST ? s0 * iS : s0 / S;
      w1 = MVBA_K0_FAST ? s1 * iS : s1 / S;
    } else if (MVBA_K0_FAST) {
      // one range reduction per angle (sincos), the weights through the
      // derivative terms' reciprocal: within an ulp of Eigen's divisions
      sincos(th, &S, &C);
      sincos((1.0 - alpha) * th, &s0, &c0);
      sincos(alpha * th, &s1, &c1);
      iS = 1.0 / S;
      w0 = s0 * iS;
      w1 = s1 * iS;
    } else {
      S = sin(th);
      C = cos(th);
      s0 = sin((1.0 - alpha) * th);
      c0 = cos((1.0 - alpha) * th);
      s1 = sin(alpha * th);
      c1 = cos(alpha * th);
      w0 = s0 / S;  // Eigen's slerp weights, divided as Eigen does
      w1 = s1 / S;
      iS = 1.0 / S;  // derivative terms: one reciprocal
    }
    dw0_dth = ((1.0 - alpha) * c0 * S - s0 * C) * (iS * iS);
    dw1_dth = (alpha * c1 * S - s1 * C) * (iS * iS);
    dw0_da = -th * c0 * iS;
    dw1_da = th * c1 * iS;
    dth_dD = -iS;
  }
  const double sgn = (d < 0.0) ? -1.0 : 1.0;
  if (d < 0.0) {
    w1 = -w1;
    dw1_dth = -dw1_dth;
    dw1_da = -dw1_da;
  }
  double qi[4];
  for (int k = 0; k < 4; k++) qi[k] = w0 * q0[k] + w1 * q1[k];
  double Ri[9];
  quat_to_rot(qi[0], qi[1], qi[2], qi[3], Ri);
  double ti[3];
  for (int k = 0; k < 3; k++) ti[k] = (1.0 - alpha) * t0[k] + alpha * t1[k];

  // world_to_cam = ref_to_cam * interp (rig_calibrator.cc:386), Affine product [ext].
  double Rw[9], tw[3];
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++)
      Rw[3 * r + c] = R2[3 * r + 0] * Ri[c] + R2[3 * r + 1] * Ri[3 + c] + R2[3 * r + 2] * Ri[6 + c];
    tw[r] = R2[3 * r + 0] * ti[0] + R2[3 * r + 1] * ti[1] + R2[3 * r + 2] * ti[2] + t2[r];
  }
  if (sub == 0) {
    for (int k = 0; k < 9; k++) wr<WT>(rec + k, Rw[k]);
    wr<WT>(rec + 9, tw[0]); wr<WT>(rec + 10, tw[1]); wr<WT>(rec + 11, tw[2]);
  }

#ifdef MVBA_EVAL_STAMPS
  if (stamp && sub == 0) *stamp = __builtin_amdgcn_s_memrealtime();
#else
  (void)stamp;
#endif
  for (int k = sub; k < kPoseCols; k += NT) {
    // Every per-column choice below is made by value (selects), never by a
    // dynamic index into a register array or a pointer to one of two arrays:
    // either would move the arrays to scratch memory (80 B per lane before).
    double om[3] = {0.0, 0.0, 0.0}, dt[3] = {0.0, 0.0, 0.0};
    if (k < 3 || (k >= 7 && k < 10) || (k >= 14 && k < 17)) {
      // translation columns of beg / end / ref_to_cam
      const int j = (k < 3) ? k : (k < 10) ? k - 7 : k - 14;
      const double scale = (k < 3) ? (1.0 - alpha) : (k < 10) ? alpha : 0.0;
      if (k >= 14) {
        dt[0] = j == 0 ? 1.0 : 0.0;
        dt[1] = j == 1 ? 1.0 : 0.0;
        dt[2] = j == 2 ? 1.0 : 0.0;
      } else {
        const double c0 = j == 0 ? R2[0] : j == 1 ? R2[1] : R2[2];
        const double c1 = j == 0 ? R2[3] : j == 1 ? R2[4] : R2[5];
        const double c2 = j == 0 ? R2[6] : j == 1 ? R2[7] : R2[8];
        dt[0] = scale * c0; dt[1] = scale * c1; dt[2] = scale * c2;
      }
    } else if (k < 14) {
      // quaternion columns of beg (3..6) and end (10..13) through slerp
      const bool side = (k >= 10);
      const int kk = side ? k - 10 : k - 3;
      const double sc = side ? sig1 * in1 : sig0 * in0;
      double qh[4], qo[4];
#pragma unroll
      for (int m = 0; m < 4; m++) {
        qh[m] = side ? qh1[m] : qh0[m];
        qo[m] = side ? q0[m] : q1[m];
      }
      const double qk = kk == 0 ? qh[0] : kk == 1 ? qh[1] : kk == 2 ? qh[2] : qh[3];
      double dq[4];
#pragma unroll
      for (int m = 0; m < 4; m++) dq[m] = sc * ((m == kk ? 1.0 : 0.0) - qh[m] * qk);
      const double dD = sgn * (qo[0] * dq[0] + qo[1] * dq[1] + qo[2] * dq[2] + qo[3] * dq[3]);
      const double dth = dth_dD * dD;
      const double ws = side ? w1 : w0;
      double dqi[4];
      for (int m = 0; m < 4; m++) dqi[m] = ws * dq[m] + dw0_dth * dth * q0[m] + dw1_dth * dth * q1[m];
      double omi[3];
      tangent_generator(dqi, qi, omi);
      matvec(R2, omi, om);
    } else if (k < 21) {
      // ref_to_cam quaternion: dR_wc = [w]x R_wc, dt_wc = w x (t_wc - t2)
      quat_generator(qh2, 2.0 * in2, k - 17, om);
      const double tt[3] = {tw[0] - t2[0], tw[1] - t2[1], tw[2] - t2[2]};
      cross(om, tt, dt);
    } else {
      // timestamp offset: d alpha / d offset = -1 / (se - sb)
      const double da = -1.0 / (F.se - F.sb);
      double dqi[4];
      for (int m = 0; m < 4; m++) dqi[m] = (dw0_da * q0[m] + dw1_da * q1[m]) * da;
      double omi[3];
      tangent_generator(dqi, qi, omi);
      matvec(R2, omi, om);
      const double dti[3] = {(t1[0] - t0[0]) * da, (t1[1] - t0[1]) * da, (t1[2] - t0[2]) * da};
      matvec(R2, dti, dt);
    }
    put_col_wt<WT>(rec, k, om, dt, tw);
  }
}

__global__ void __launch_bounds__(kPrepBlock) k_prep(const FrameDesc* __restrict__ fd, int64_t nframes,
                                                     int32_t frame_blocks, const double* __restrict__ params,
                                                     double* __restrict__ frec, const int64_t* __restrict__ pt_off,
                                                     const uint8_t* __restrict__ pt_free, int64_t npts,
                                                     double4* __restrict__ pts, int gen, int* __restrict__ err) {
  const int bid = (int)blockIdx.x;
  if (bid < frame_blocks) {
    const int64_t t = (int64_t)bid * kPrepBlock + threadIdx.x;
    const int64_t f = t / kThreadsPerFrame;
    if (f >= nframes) return;
    const FrameDesc F = fd[f];
    frame_columns<false>(F, params, frec + f * kFrameRecDoubles, (int)(t % kThreadsPerFrame), gen, err);
  } else {
    // kPrepPoints landmarks per thread, all loads in flight before the stores
    const int64_t p0 = (int64_t)(bid - frame_blocks) * kPrepBlock * kPrepPoints + threadIdx.x;
    int64_t o[kPrepPoints];
#pragma unroll
    for (int j = 0; j < kPrepPoints; j++) {
      const int64_t p = p0 + (int64_t)j * kPrepBlock;
      o[j] = p < npts ? pt_off[p] : -1;
    }
    double v[kPrepPoints][3];
    bool fr[kPrepPoints];
#pragma unroll
    for (int j = 0; j < kPrepPoints; j++) {
      const int64_t p = p0 + (int64_t)j * kPrepBlock;
      if (o[j] >= 0) {
        v[j][0] = params[o[j]];
        v[j][1] = params[o[j] + 1];
        v[j][2] = params[o[j] + 2];
        fr[j] = pt_free[p] != 0;
      }
    }
#pragma unroll
    for (int j = 0; j < kPrepPoints; j++)
      if (o[j] >= 0) pts[p0 + (int64_t)j * kPrepBlock] = make_double4(v[j][0], v[j][1], v[j][2], fr[j] ? 1.0 : 0.0);
  }
}

// ------------------------------------------------------------ K1: observations
// OT = double (fp64 output) or float (fp32 output: the same fp64 arithmetic,
// each value rounded once at the store; half the output bytes).
template <class OT>
__device__ __forceinline__ void stj(OT* J, int64_t ld, int row, int64_t i, double v) {
  __builtin_nontemporal_store((OT)v, J + (int64_t)row * ld + i);
}

// The fused evaluation's hand-off from its K0 blocks to its K1 waves.
struct FusedIn {
  const int64_t* pt_off;   // landmark offsets in the parameter vector
  const uint8_t* pt_free;  // landmark floats
  const unsigned* ready;   // one word per K0 block: = epoch once its 16 frame records are stored
  unsigned epoch;
  int64_t k1_block0;       // first K1 block of the grid (a multiple of 8: XCD order kept)
  int* err;                // error words: [0] alpha range (K0), [1] ready-word wait given up (k_eval)
  unsigned poll_limit;     // k_eval: polls of the ready word before a wave gives up (0: every wave fails at once, tests)
};

// How a K1 wave gets its frame record: kRecGlobal reads the prep kernel's
// record; kRecFused waits for the K0 blocks of the same launch (k_eval);
// kRecLocal computes it itself into its LDS area (k_eval_local: thin shards,
// about one segment per frame, where a hand-off costs more than the K0 work).
enum { kRecGlobal = 0, kRecFused = 1, kRecLocal = 2 };

// -DMVBA_EVAL_STAMPS builds (timing probes, tools/eval_stamps.py): lane 0 of
// each k_eval_local wave records the real-time counter (100 MHz) at its phase
// boundaries; mvba_debug_eval_stamps reads them back.
#ifdef MVBA_EVAL_STAMPS
constexpr int kStampWaves = 16384, kStamps = 8;
__device__ unsigned long long g_eval_stamps[kStampWaves * kStamps];
#define MVBA_STAMP(k)                                                                          \
  do {                                                                                         \
    if (RECM == kRecLocal && lane == 0 && wave < kStampWaves)                                  \
      g_eval_stamps[wave * kStamps + (k)] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#else
#define MVBA_STAMP(k) \
  do {                \
  } while (0)
#endif

template <int MODEL, int DEG, class OT, bool JAC, int RECM = kRecGlobal>
__device__ __forceinline__ void obs_body(
    const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
    const double2* __restrict__ obs_meas, OT* __restrict__ res, OT* __restrict__ J,
    int64_t ld, int32_t flags, double cauchy_c, const FusedIn& fu = FusedIn{}) {
  constexpr bool FUSED = (RECM == kRecFused);
  // 4 segments per block, XCD-contiguous
  const int64_t blk = xcd_block_of((int64_t)blockIdx.x - (RECM != kRecGlobal ? fu.k1_block0 : 0), (nseg + 3) / 4);
  if (blk < 0) return;
  const int wave = (int)((blk * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= nseg) return;
  MVBA_STAMP(0);
  const Segment sg = segs[wave];
  const int begin = __builtin_amdgcn_readfirstlane(sg.begin);
  const int count = __builtin_amdgcn_readfirstlane(sg.count);
  const int frame = __builtin_amdgcn_readfirstlane(sg.frame);
  MVBA_STAMP(5);  // (probes) the segment record arrived
  // Lanes past the frame's last observation up to the next 128-B line (16
  // fp64 / 32 fp32 slots; segments start on 16- or 32-slot boundaries) recompute the
  // last observation and store it into their padding slots, inside the same
  // store instructions: every line of every plane is then written whole (a
  // partly written line costs HBM a read-modify-write: 110 -> 98 us at c2).
  // No reader looks at padding slots.
  // sg.pad bounds the padding at the next frame's first slot (slot alignment 16:
  // fp32 outputs then write the frame's last half line).
  constexpr int kLine = 128 / (int)sizeof(OT);
  const bool active = lane < min((count + kLine - 1) & ~(kLine - 1), __builtin_amdgcn_readfirstlane(sg.pad));
  // (local records: every lane takes part in storing the record first)
  if (RECM == kRecGlobal && !active) return;
  const int64_t i = (int64_t)begin + lane;
  const int64_t isrc = (int64_t)begin + min(lane, count - 1);

  const FrameDesc& F = fd[frame];
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  const double* __restrict__ kd = params + F.off[MVBA_BLK_DIST];
  const int free_mask = F.free_mask;
  const int K = F.K;
#ifdef MVBA_EVAL_STAMPS
  asm volatile("" ::"v"(f));  // (probes) the frame descriptor and a parameter through it arrived
  MVBA_STAMP(6);
#endif

  double4 P;
  const double* rec;
  if constexpr (FUSED) {
    // landmark straight from the parameter vector (this launch's gather blocks
    // fill pts for later launches only), issued before the wait
    const int32_t pid = obs_pid[isrc];
    const int64_t po = fu.pt_off[pid];
    P = make_double4(params[po], params[po + 1], params[po + 2], fu.pt_free[pid] ? 1.0 : 0.0);
    // Wait for the frame's K0 block, then read its record: one lane polls the
    // ready word (relaxed agent load, sc1), every record load is an sc1 load to
    // registers (the record was stored write-through), staged in this wave's
    // LDS area (MI355X_MICROARCH.md, visibility: valid forms, first row).
    __shared__ double srec[4][kFrameRecDoubles];
    double* sr = srec[threadIdx.x >> 6];
    // HIP promises no dispatch order: the launch puts every K0 block in front of
    // the K1 blocks, and on gfx950 blocks start in index order, so the wait
    // ends within the K0 work. The wait is bounded all the same; a wave that
    // gives up raises error word [1] to this launch's epoch, so
    // mvba_sync_status fails (MVBA_E_DEVICE_WAIT) instead of returning
    // residuals built from a record that may be stale.
    // poll_limit 0 (tests) fails every wave before its first poll, whatever the
    // dispatch timing, so the error path is exercised deterministically.
    if (lane == 0 && fu.poll_limit == 0) {
      atomicMax(fu.err + 1, (int)fu.epoch);
    } else if (lane == 0) {
      const unsigned* w = fu.ready + (frame >> 4);  // 16 frames per K0 block
      for (unsigned n = 0; __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != fu.epoch; n++) {
        if (n >= fu.poll_limit) {
          atomicMax(fu.err + 1, (int)fu.epoch);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the record loads below the poll
    const double* g = frec + (int64_t)frame * kFrameRecDoubles;
    for (int m = lane; m < kFrameRecDoubles; m += 64)
      sr[m] = __hip_atomic_load(const_cast<double*>(g + m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (!active) return;
    rec = sr;
  } else if constexpr (RECM == kRecLocal) {
    // lanes 0..MVBA_K0_LANES-1 (present whatever the segment's count) run K0 for this wave's frame
    // into the wave's LDS area; then the landmark straight from the parameter
    // vector (no prep launch; loaded after K0 so the two register sets are
    // never live together: 3 waves per SIMD without spills)
    // (loading the landmark's offset and free flag before K0 measured no gain:
    // 20.0 vs 18.4-20.6 us on the 8-way shard, profiles/r03/ab_eval_local/)
    // MVBA_K0_SHARE (default on): a wave whose block predecessors hold the same
    // frame skips K0 and reads the record of the block's first wave of that
    // frame (a frame spans ~5 segment waves at c2 and its shards): K0 runs once
    // per frame and block instead of once per wave, the waves meet at one block
    // barrier. (Waves past nseg returned above: a finished wave leaves the
    // barrier's count.)
    __shared__ double srec[4][kFrameRecDoubles];
    const int wb = (int)(threadIdx.x >> 6);
    int lead = wb;
    if (MVBA_K0_SHARE)
      while (lead > 0 && __builtin_amdgcn_readfirstlane(segs[wave - (wb - lead) - 1].frame) == frame) lead--;
    double* sr = srec[lead];
#ifdef MVBA_EVAL_STAMPS
    unsigned long long* k0stamp = wave < kStampWaves ? g_eval_stamps + wave * kStamps + 7 : nullptr;
#else
    unsigned long long* k0stamp = nullptr;
#endif
    if (lead == wb && lane < MVBA_K0_LANES)
      frame_columns<false, MVBA_K0_LANES, (MVBA_K0_SPLIT ? 2 : 0)>(F, params, sr, lane, (int)fu.epoch, fu.err,
                                                                  k0stamp);
    const int32_t pid = obs_pid[isrc];
    const int64_t po = fu.pt_off[pid];
    P = make_double4(params[po], params[po + 1], params[po + 2], fu.pt_free[pid] ? 1.0 : 0.0);
    if (MVBA_K0_SHARE) {
      __syncthreads();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    rec = sr;
    MVBA_STAMP(1);
    // the wave of the frame's first segment stores the record for later
    // launches (solver, SKIP_PREP evaluations): in a one-group problem every
    // frame has a segment (frames are the reprojection residuals' images)
    if (wave == 0 || segs[wave - 1].frame != frame) {
      double* g = const_cast<double*>(frec) + (int64_t)frame * kFrameRecDoubles;  // k_eval_local owns frec
      for (int m = lane; m < kFrameRecDoubles; m += 64) g[m] = sr[m];  // all 64 lanes: the whole record
    }
    if (!active) return;
  } else {
    P = pts[obs_pid[isrc]];
    rec = frec + (int64_t)frame * kFrameRecDoubles;
  }
  const double2 meas = obs_meas[isrc];
  Proj o;
  project<MODEL, DEG>(rec, P.x, P.y, P.z, f, c0, c1, kd, K, F.h0, F.h1, o);
  MVBA_STAMP(2);

  double r0 = o.d0 - meas.x;  // rig_calibrator.cc:478-479
  double r1 = o.d1 - meas.y;
  double half_rho;
  const double sr = loss_scale(r0, r1, flags, cauchy_c, &half_rho);
  r0 *= sr;
  r1 *= sr;
  if (res) {
    __builtin_nontemporal_store((OT)r0, res + i);
    __builtin_nontemporal_store((OT)r1, res + ld + i);
  }
  if (!JAC) return;

  // G = A * du/dXc, du/dXc = (f/z) [[1, 0, -nx], [0, 1, -ny]]; scaled by the loss.
  const double fz = f / o.Xc[2] * sr;
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
  double a0[3], a1[3];
  cross(o.Xc, G0, a0);
  cross(o.Xc, G1, a1);

  // Pose columns: blocks beg (0), end (1), ref_to_cam (2), offset (4).
#pragma unroll
  for (int blk = 0; blk < 4; blk++) {
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    if (!(free_mask & (1 << b))) continue;
    const int ncol = (blk == 3) ? 1 : 7;
    const int k0 = blk * 7;
    const int base = (blk == 3) ? MVBA_JAC_BASE_OFFSET : 14 * blk;
#pragma unroll
    for (int c = 0; c < ncol; c++) {
      const double* w = rec + 12 + 6 * (k0 + c);
      const double j0 = a0[0] * w[0] + a0[1] * w[1] + a0[2] * w[2] + G0[0] * w[3] + G0[1] * w[4] + G0[2] * w[5];
      const double j1 = a1[0] * w[0] + a1[1] * w[1] + a1[2] * w[2] + G1[0] * w[3] + G1[1] * w[4] + G1[2] * w[5];
      stj(J, ld, base + c, i, j0);
      stj(J, ld, base + ncol + c, i, j1);
    }
  }
  // Point columns: dXc/dX = R_wc.
  if (P.w != 0.0) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const double j0 = G0[0] * rec[c] + G0[1] * rec[3 + c] + G0[2] * rec[6 + c];
      const double j1 = G1[0] * rec[c] + G1[1] * rec[3 + c] + G1[2] * rec[6 + c];
      stj(J, ld, MVBA_JAC_BASE_XYZ + c, i, j0);
      stj(J, ld, MVBA_JAC_BASE_XYZ + 3 + c, i, j1);
    }
  }
  if (free_mask & (1 << MVBA_BLK_FOCAL)) {
    stj(J, ld, MVBA_JAC_BASE_FOCAL, i, o.df0 * sr);
    stj(J, ld, MVBA_JAC_BASE_FOCAL + 1, i, o.df1 * sr);
  }
  if (free_mask & (1 << MVBA_BLK_CENTER)) {
    const double cc = (MODEL == kModelRpc) ? 0.0 : sr;  // RPC ignores the optical centre
    stj(J, ld, MVBA_JAC_BASE_CENTER + 0, i, cc);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 1, i, 0.0);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 2, i, 0.0);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 3, i, cc);
  }
  if (!(free_mask & (1 << MVBA_BLK_DIST))) return;
  dist_columns<MODEL, DEG>(o, f, K, sr, [&](int c, double v0, double v1) {
    stj(J, ld, MVBA_JAC_BASE_DIST + c, i, v0);
    stj(J, ld, MVBA_JAC_BASE_DIST + K + c, i, v1);
  });
  if constexpr (MODEL == kModelRpc) {
    // Undistortion half: structurally zero.
    for (int c = live_dist_cols<MODEL, DEG>(K); c < K; c++) {
      stj(J, ld, MVBA_JAC_BASE_DIST + c, i, 0.0);
      stj(J, ld, MVBA_JAC_BASE_DIST + K + c, i, 0.0);
    }
  }
}

// ------------------------------------------------------------ K2a: camera side, one launch
// Normal equations, camera side. For a frame f, every pose column is
// J_k = Z w_k with Z_i = [Xc x G_i | G_i] (per observation, 6 numbers per row)
// and w_k = [omega_k; v_k] (per frame), so the frame's whole camera-camera block
// follows from the Gram matrix of B = [Z | J_focal | J_center | J_dist | r]
// (2 rows per observation): B^T B holds Z^T Z, Z^T J_intr, J_intr^T J_intr and
// the gradients Z^T r, J_intr^T r; the expansion applies w.
//
// K1 with the Jacobian planes, and the residual-only evaluation under its own
// name (k_obs_res) so kernel statistics never mix the two.
template <int MODEL, int DEG, class OT>
__global__ void __launch_bounds__(256) k_obs(
    const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
    const double2* __restrict__ obs_meas, OT* __restrict__ res, OT* __restrict__ J,
    int64_t ld, int32_t flags, double cauchy_c) {
  obs_body<MODEL, DEG, OT, true>(segs, nseg, fd, frec, params, pts, obs_pid, obs_meas, res, J, ld, flags, cauchy_c);
}
template <int MODEL, int DEG, class OT>
__global__ void __launch_bounds__(256) k_obs_res(
    const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
    const double2* __restrict__ obs_meas, OT* __restrict__ res, OT* __restrict__ J,
    int64_t ld, int32_t flags, double cauchy_c) {
  obs_body<MODEL, DEG, OT, false>(segs, nseg, fd, frec, params, pts, obs_pid, obs_meas, res, J, ld, flags, cauchy_c);
}

// Fused evaluation (one model group): prep and K1 in one launch. Blocks
// [0, fb) run K0 for 16 frames each, storing the records write-through, and
// publish ready[block] = epoch behind every storing wave's vmcnt(0) wait and a
// block barrier; blocks [fb, fb + pb) gather the landmarks into pts (for later
// launches: the solver, SKIP_PREP evaluations); blocks from fu.k1_block0 run K1,
// whose waves issue their landmark loads, then wait for their frame's ready
// word. K0 blocks never wait and precede every K1 block in dispatch order, so
// every wait ends; the frame arithmetic overlaps the K1 waves' loads instead of
// a kernel boundary.
template <int MODEL, int DEG, class OT, bool JAC>
__global__ void __launch_bounds__(256) k_eval(
    const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd, int64_t nframes,
    int32_t fb, int32_t pb, double* __restrict__ frec, const double* __restrict__ params, int64_t npts,
    double4* __restrict__ pts, const int32_t* __restrict__ obs_pid, const double2* __restrict__ obs_meas,
    OT* __restrict__ res, OT* __restrict__ J, int64_t ld, int32_t flags, double cauchy_c, int gen,
    int* __restrict__ err, unsigned* __restrict__ ready, FusedIn fu) {
  const int bid = (int)blockIdx.x;
  if (bid < fb) {
    const int64_t t = (int64_t)bid * kPrepBlock + threadIdx.x;
    const int64_t f = t / kThreadsPerFrame;
    if (f < nframes) frame_columns<true>(fd[f], params, frec + f * kFrameRecDoubles, (int)(t % kThreadsPerFrame),
                                         gen, err);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's record stores have completed
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(ready + bid, fu.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if ((int64_t)bid < fu.k1_block0) {
    const int64_t p = (int64_t)(bid - fb) * kPrepBlock + threadIdx.x;
    if (bid - fb < pb && p < npts) {
      const int64_t o = fu.pt_off[p];
      pts[p] = make_double4(params[o], params[o + 1], params[o + 2], fu.pt_free[p] ? 1.0 : 0.0);
    }
    return;
  }
  obs_body<MODEL, DEG, OT, JAC, kRecFused>(segs, nseg, fd, frec, params, pts, obs_pid, obs_meas, res, J, ld, flags,
                                           cauchy_c, fu);
}

// Thin-shard evaluation in one launch (k_eval_local): landmark-gather blocks
// (for later launches: the solver, SKIP_PREP evaluations) come first, rounded
// up to a multiple of 8 blocks; then the K1 blocks, whose waves run K0 for
// their own frame into LDS (no hand-off, no wait) and store the record from the
// frame's first segment. Used when a frame has about one segment, so the
// per-wave K0 is not repeated: the prep launch and its boundary disappear.
// 3 waves per SIMD (the K0 arithmetic's register file).
template <int MODEL, int DEG, class OT, bool JAC>
__global__ void __launch_bounds__(256, 3) k_eval_local(
    const Segment* __restrict__ segs, int32_t nseg, int32_t pb, const FrameDesc* __restrict__ fd,
    double* __restrict__ frec, const double* __restrict__ params, int64_t npts, double4* __restrict__ pts,
    const int32_t* __restrict__ obs_pid, const double2* __restrict__ obs_meas, OT* __restrict__ res,
    OT* __restrict__ J, int64_t ld, int32_t flags, double cauchy_c, FusedIn fu) {
  const int bid = (int)blockIdx.x;
  if ((int64_t)bid >= fu.k1_block0) {
    obs_body<MODEL, DEG, OT, JAC, kRecLocal>(segs, nseg, fd, frec, params, pts, obs_pid, obs_meas, res, J, ld,
                                             flags, cauchy_c, fu);
#ifdef MVBA_EVAL_STAMPS
    {
      constexpr int RECM = kRecLocal;
      const int64_t blk = xcd_block_of((int64_t)blockIdx.x - fu.k1_block0, (nseg + 3) / 4);
      const int wave = (int)((blk * blockDim.x + threadIdx.x) >> 6);
      const int lane = threadIdx.x & 63;
      if (blk >= 0 && wave < nseg) {
        MVBA_STAMP(3);  // every store issued
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        MVBA_STAMP(4);  // every store acknowledged
      }
    }
#endif
    return;
  }
  const int64_t p = (int64_t)bid * kPrepBlock + threadIdx.x;
  if (bid < pb && p < npts) {
    const int64_t o = fu.pt_off[p];
    pts[p] = make_double4(params[o], params[o + 1], params[o + 2], fu.pt_free[p] ? 1.0 : 0.0);
  }
}

// k_frame_lin: one block per frame part (<= kPartSegs segments of ONE frame),
// WAVES waves per block. Each wave builds the Gram of its segments' rows (a
// K = 128-deep GEMM per segment on fp64 MFMA v_mfma_f64_16x16x4, B staged in
// the wave's own LDS area as [column][row], row stride kGramLd doubles: no
// block barrier inside the loop, waves run their segments independently). The
// waves' accumulators are summed through LDS in wave order, and the block maps
// the frame's Gram through w and adds pose / intrinsic blocks into replica
// (frame mod kLinReplicas) of [grad | hess | cost]: a sensor's extrinsic and
// intrinsic blocks are shared by all its frames, so the replicas keep the
// atomic adds per address low; k_rep_reduce sums them (and re-zeroes).
// The Gram entries stay in the accumulator layout: pair p = (ti, tj), ti <= tj,
// lane l and register r hold G[16 ti + (l >> 4) + 4 r][16 tj + (l & 15)].
constexpr int kGramLd = 66;  // 64 rows + 2 pad doubles: bank-conflict-free reads
#ifndef MVBA_LIN_REPLICAS
#define MVBA_LIN_REPLICAS 8
#endif
constexpr int kLinReplicas = MVBA_LIN_REPLICAS;  // power of two
#ifndef MVBA_FLIN_WAVES
#define MVBA_FLIN_WAVES 2
#endif
#define MVBA_FLIN_WAVES_SMALL_T_OVERRIDE (kTiles <= 2 ? MVBA_FLIN_WAVES : kTiles <= 4 ? 2 : 1)

template <int MODEL, int DEG>
struct GramShape {
  static constexpr int kDist = (MODEL == kModelNone) ? 0 : (MODEL == kModelFov) ? 1
                             : (MODEL == kModelRadtan) ? 5 : 2 * ((DEG + 1) * (DEG + 2)) - 2;
  static constexpr int kWidth = 6 + 1 + 2 + kDist + 1;  // Z | focal | center | dist | r
  static constexpr int kTiles = (kWidth + 15) / 16;
  static constexpr int kPairs = kTiles * (kTiles + 1) / 2;
  static constexpr int kColR = kWidth - 1;              // residual column
  // waves per block: LDS staging is kTiles*16*kGramLd doubles per wave
  static constexpr int kWaves = MVBA_FLIN_WAVES_SMALL_T_OVERRIDE;
  // the staging area also holds the wave's accumulators (kPairs * 256 doubles)
  static constexpr int kStage = kTiles * 16 * kGramLd > kPairs * 256 ? kTiles * 16 * kGramLd : kPairs * 256;
  // rows straight into LDS (no register row arrays) from 3 tiles up
  static constexpr bool kDirect = kTiles >= 3;
  static constexpr size_t kLdsBytes = sizeof(double) * ((size_t)kWaves * kStage + 2 * 6 * kPoseCols + kWaves);
};

// Entry (a, b) of a Gram held in the accumulator layout (T tiles per side).
template <int T>
__device__ __forceinline__ double gram_at(const double* __restrict__ G, int a, int b) {
  if (a / 16 > b / 16) {
    const int t = a;
    a = b;
    b = t;
  }
  const int ti = a >> 4, tj = b >> 4, i = a & 15, j = b & 15;
  const int p = ti * T - ti * (ti - 1) / 2 + (tj - ti);
  return G[(p * 4 + (i >> 2)) * 64 + (i & 3) * 16 + j];
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS hand-off between the lanes of ONE wave: wait for the wave's LDS ops
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int MODEL, int DEG>
__device__ __forceinline__ void points_lin_body(
    int64_t t, const int64_t* __restrict__ pt_begin, int64_t npts, const int32_t* __restrict__ po_frame,
    const double2* __restrict__ po_meas, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, double* __restrict__ pgrad, double* __restrict__ phess,
    int32_t flags, double cauchy_c, const PointExtra& dc);

// The point side (K2b) as extra blocks of the same launch (single-model problems):
// blocks past the frame parts take kLanesPerPoint threads per point.
struct PointLinArgs {
  const int64_t* pt_begin;
  int64_t npts;
  const int32_t* po_frame;
  const double2* po_meas;
  double* pgrad;
  double* phess;
  PointExtra dc;
};

template <int MODEL, int DEG, bool POINTS>
__global__ void __launch_bounds__((64 * GramShape<MODEL, DEG>::kWaves)) k_frame_lin(
    const int4* __restrict__ parts, int32_t nparts, const Segment* __restrict__ segs,
    const FrameDesc* __restrict__ fd, const FrameLin* __restrict__ fl, const double* __restrict__ frec,
    const double* __restrict__ params, const double4* __restrict__ pts,
    const int32_t* __restrict__ obs_pid, const double2* __restrict__ obs_meas,
    double* __restrict__ rep, int64_t ng, int64_t nh, int32_t flags, double cauchy_c, PointLinArgs pa, Slab sl,
    int32_t part_base, double4* __restrict__ obsx_out) {
  using S = GramShape<MODEL, DEG>;
  constexpr int T = S::kTiles;
  constexpr int NP = S::kPairs;
  constexpr int WAVES = S::kWaves;
  constexpr int W16 = T * 16;
  extern __shared__ double lds[];  // [WAVES][kStage] | w [6 x 22] | Tm [6 x 22] | cost [WAVES]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // frame parts in the plain block order: the XCD-contiguous order of the CG
  // passes measured slower here (c2 51.0 -> 59.3 us without the point blocks,
  // c3 +25 us: profiles/r03/ab_xcd_solver/), then the point blocks
  if ((int)blockIdx.x >= nparts) {
    if constexpr (POINTS)
      points_lin_body<MODEL, DEG>((int64_t)(blockIdx.x - nparts) * blockDim.x + tid, pa.pt_begin, pa.npts,
                                  pa.po_frame, pa.po_meas, fd, frec, params, pts, pa.pgrad, pa.phess, flags,
                                  cauchy_c, pa.dc);
    return;
  }
  const int4 part = parts[blockIdx.x];  // seg_begin, seg_count, frame, -
  const int frame = __builtin_amdgcn_readfirstlane(part.z);
  const FrameDesc& F = fd[frame];
  const double* __restrict__ rec = frec + (int64_t)frame * kFrameRecDoubles;
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  const double* __restrict__ kd = params + F.off[MVBA_BLK_DIST];
  const int K = F.K;
  double* st = lds + wave * S::kStage;

  dbl4 acc[NP];
#pragma unroll
  for (int p = 0; p < NP; p++) acc[p] = dbl4{0.0, 0.0, 0.0, 0.0};
  double cost = 0.0;

  // zero the padding columns of this wave's staging area once (they stay zero)
  if (lane < 32)
    for (int col = S::kWidth; col < W16; col++) *(dbl2v*)&st[col * kGramLd + 2 * lane] = dbl2v{0.0, 0.0};

  // One observation's row pair [Z | focal | centre | dist | r] (Cauchy-corrected),
  // emitted column by column as put(q, v_row0, v_row1).
  auto rows = [&](int64_t i, auto&& put) {
    const double4 P = pts[obs_pid[i]];
    const double2 meas = obs_meas[i];
    Proj o;
    project<MODEL, DEG>(rec, P.x, P.y, P.z, f, c0, c1, kd, K, F.h0, F.h1, o);
    const double r0 = o.d0 - meas.x, r1 = o.d1 - meas.y;
    double half_rho;
    const double sr = loss_scale(r0, r1, flags, cauchy_c, &half_rho);
    cost += half_rho;
    if (obsx_out) obsx_out[i] = make_double4(P.x, P.y, P.z, sr);  // the CG passes' per-slot record
    const double fz = f / o.Xc[2] * sr;
    const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
    const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
    double a0[3], a1[3];
    cross(o.Xc, G0, a0);
    cross(o.Xc, G1, a1);
#pragma unroll
    for (int q = 0; q < 3; q++) {
      put(q, a0[q], a1[q]);
      put(3 + q, G0[q], G1[q]);
    }
    put(6, o.df0 * sr, o.df1 * sr);
    const double cc = (MODEL == kModelRpc) ? 0.0 : sr;
    put(7, cc, 0.0);
    put(8, 0.0, cc);
    dist_columns<MODEL, DEG>(o, f, K, sr, [&](int q, double v0, double v1) { put(9 + q, v0, v1); });
    put(S::kColR, r0 * sr, r1 * sr);
  };
  // MFMA over the 64 staged rows: acc[(ti, tj)] += B_ti^T B_tj
  auto gram64 = [&]() {
    const int col = lane & 15, rsub = lane >> 4;
#pragma unroll 4
    for (int stp = 0; stp < 16; stp++) {
      const int row = 4 * stp + rsub;
      double v[T];
#pragma unroll
      for (int t = 0; t < T; t++) v[t] = st[(t * 16 + col) * kGramLd + row];
      int p = 0;
#pragma unroll
      for (int ti = 0; ti < T; ti++)
#pragma unroll
        for (int tj = ti; tj < T; tj++) {
          acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[ti], v[tj], acc[p], 0, 0, 0);
          p++;
        }
    }
  };

  for (int sidx = wave; sidx < part.y; sidx += WAVES) {
    const Segment sg = segs[part.x + sidx];
    const int count = __builtin_amdgcn_readfirstlane(sg.count);
    const int64_t i = (int64_t)sg.begin + lane;
    if constexpr (!S::kDirect) {
      // rows in registers, then staged as [column][row] 64 rows at a time; the
      // halves past the segment's last observation are all zero rows
      double row0[S::kWidth], row1[S::kWidth];
#pragma unroll
      for (int q = 0; q < S::kWidth; q++) row0[q] = row1[q] = 0.0;
      if (lane < count)
        rows(i, [&](int q, double v0, double v1) {
          row0[q] = v0;
          row1[q] = v1;
        });
      for (int half = 0; half < 2 && 32 * half < count; half++) {
        if ((lane >> 5) == half) {
#pragma unroll
          for (int q = 0; q < S::kWidth; q++)
            *(dbl2v*)&st[q * kGramLd + 2 * (lane & 31)] = dbl2v{row0[q], row1[q]};
        }
        wave_lds_sync();
        gram64();
        wave_lds_sync();
      }
    } else {
      // wide Grams (RPC degree >= 2): the lanes of the active half write their
      // columns straight into the staging area as they are produced (no row
      // arrays in registers; the other half idles through the projection)
      for (int half = 0; half < 2 && 32 * half < count; half++) {
        if ((lane >> 5) == half) {
          const int slot = 2 * (lane & 31);
          if (lane < count)
            rows(i, [&](int q, double v0, double v1) { *(dbl2v*)&st[q * kGramLd + slot] = dbl2v{v0, v1}; });
          else
            for (int q = 0; q < S::kWidth; q++) *(dbl2v*)&st[q * kGramLd + slot] = dbl2v{0.0, 0.0};
        }
        wave_lds_sync();
        gram64();
        wave_lds_sync();
      }
    }
  }
  // ---- the block's Gram: waves' accumulators summed in wave order (in place
  // in wave 0's staging area, accumulator layout)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cost += __shfl_xor(cost, off, 64);
  double* wbuf = lds + WAVES * S::kStage;  // w [a * 22 + k]
  double* Tm = wbuf + 6 * kPoseCols;        // T = G_ZZ w [a * 22 + k]
  double* wcost = Tm + 6 * kPoseCols;
  __syncthreads();  // every wave is done with its staging area
#pragma unroll
  for (int p = 0; p < NP; p++)
#pragma unroll
    for (int r = 0; r < 4; r++) st[(p * 4 + r) * 64 + lane] = acc[p][r];
  if (lane == 0) wcost[wave] = cost;
  for (int e = tid; e < 6 * kPoseCols; e += 64 * WAVES) {
    const int k = e / 6, a = e % 6;
    wbuf[a * kPoseCols + k] = rec[12 + 6 * k + a];
  }
  __syncthreads();
  if (WAVES > 1)
    for (int e = tid; e < NP * 256; e += 64 * WAVES) {
      double v = lds[e];
#pragma unroll
      for (int w = 1; w < WAVES; w++) v += lds[w * S::kStage + e];
      lds[e] = v;
    }
  __syncthreads();
  const double* G = lds;
  auto g = [&](int a, int b) -> double { return gram_at<T>(G, a, b); };
  for (int e = tid; e < 6 * kPoseCols; e += 64 * WAVES) {
    const int a = e / kPoseCols, k = e % kPoseCols;
    double t = 0.0;
#pragma unroll
    for (int b = 0; b < 6; b++) t += g(a, b) * wbuf[b * kPoseCols + k];
    Tm[e] = t;
  }
  __syncthreads();
  const FrameLin& L = fl[frame];
  const int R = S::kColR;
  // replica (frame mod kLinReplicas) of [grad | hess | cost], or this part's slab row
  double* grad = rep + (int64_t)(frame & (kLinReplicas - 1)) * (ng + nh + 1);
  const int64_t unit = part_base + (int64_t)blockIdx.x;
  // pose blocks: beg(0) cols 0..6, end(1) 7..13, ref_to_cam(2) 14..20, offset(4) 21
#pragma unroll
  for (int blk = 0; blk < 4; blk++) {
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    const int64_t go = L.goff[b];
    if (go < 0) continue;
    const int ncol = (blk == 3) ? 1 : 7, k0 = blk * 7;
    const int64_t ho = L.hoff[b];
    for (int e = tid; e < ncol + ncol * ncol; e += 64 * WAVES) {
      double v = 0.0;
      if (e < ncol) {
#pragma unroll
        for (int a = 0; a < 6; a++) v += wbuf[a * kPoseCols + k0 + e] * g(a, R);
        accumulate(grad, go + e, v, sl, unit, 56 * blk + e);
      } else {
        const int h = e - ncol, kk = h / ncol, kc = h % ncol;
#pragma unroll
        for (int a = 0; a < 6; a++) v += wbuf[a * kPoseCols + k0 + kk] * Tm[a * kPoseCols + k0 + kc];
        accumulate(grad, ng + ho + h, v, sl, unit, 56 * blk + e);
      }
    }
  }
  // intrinsics: focal col 6, center cols 7..8, dist cols 9..
  constexpr int kDistLive = S::kWidth - 10;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const int b = q == 0 ? MVBA_BLK_FOCAL : q == 1 ? MVBA_BLK_CENTER : MVBA_BLK_DIST;
    const int64_t go = L.goff[b];
    if (go < 0) continue;
    const int cs = q == 0 ? 6 : q == 1 ? 7 : 9;
    const int nc = q == 0 ? 1 : q == 1 ? 2 : (kDistLive < K ? kDistLive : K);  // radtan K=4: 4 of 5 columns
    const int bs = q == 2 ? K : nc;  // Hessian row length (RPC: K incl. the zero half)
    const int64_t ho = L.hoff[b];
    const int sbase = q == 0 ? kSlabFocal : q == 1 ? kSlabCenter : kSlabDist;
    for (int e = tid; e < nc + nc * nc; e += 64 * WAVES) {
      if (e < nc) {
        accumulate(grad, go + e, g(cs + e, R), sl, unit, sbase + e);
      } else {
        const int h = e - nc, r = h / nc, cc = h % nc;
        accumulate(grad, ng + ho + r * bs + cc, g(cs + r, cs + cc), sl, unit, sbase + e);
      }
    }
  }
  if (tid == 0) {
    double cv = 0.0;
    for (int w = 0; w < WAVES; w++) cv += wcost[w];
    accumulate(grad, ng + nh, cv, sl, unit, (int)(sl.width - 1));
  }
}

// Deterministic mode: out[e] = sum of entry e's slab positions in slab order
// (CSR e -> positions, slab_gather: a block per heavy entry, a wave per light
// one), written to grad | hess | cost.
__global__ void __launch_bounds__(256) k_slab_lin(SlabTiers tiers, const int64_t* __restrict__ begin,
                                                  const int64_t* __restrict__ pos, const double* __restrict__ val,
                                                  int64_t ng, int64_t nh, double* __restrict__ grad,
                                                  double* __restrict__ hess, double* __restrict__ cost) {
  int64_t e;
  double acc;
  if (!slab_gather(tiers, begin, pos, val, &e, &acc)) return;
  if (e < ng) grad[e] = acc;
  else if (e < ng + nh) hess[e - ng] = acc;
  else if (cost) *cost = acc;
}

__global__ void __launch_bounds__(256) k_rep_reduce(double* __restrict__ rep, int32_t nrep, int64_t ng, int64_t nh,
                                                    double* __restrict__ grad, double* __restrict__ hess,
                                                    double* __restrict__ cost) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = ng + nh + 1;
  if (e >= stride) return;
  double v[8];
  double acc = 0.0;
  // loads of 8 replicas in flight before the adds and the zeroing stores
  for (int r0 = 0; r0 < nrep; r0 += 8) {
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = rep[(int64_t)(r0 + r) * stride + e];
#pragma unroll
    for (int r = 0; r < 8; r++) acc += v[r];
#pragma unroll
    for (int r = 0; r < 8; r++) rep[(int64_t)(r0 + r) * stride + e] = 0.0;
  }
  if (e < ng) grad[e] = acc;
  else if (e < ng + nh) hess[e - ng] = acc;
  else if (cost) *cost = acc;
}

// ------------------------------------------------------------ K2b: point side
// One lane per point: loop over its observations (point-ordered copy of the
// observation records), recompute the projection, accumulate V_p = J_p^T J_p
// (packed xx xy xz yy yz zz) and g_p = J_p^T r. No atomics.
template <int MODEL, int DEG>
__device__ __forceinline__ void point_obs(const FrameDesc& F, const double* __restrict__ rec,
                                          const double* __restrict__ params, double X0, double X1,
                                          double X2, double2 meas, int32_t flags, double cauchy_c,
                                          double* V, double* g) {
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  Proj o;
  project<MODEL, DEG>(rec, X0, X1, X2, f, c0, c1, params + F.off[MVBA_BLK_DIST], F.K, F.h0, F.h1, o);
  const double r0 = o.d0 - meas.x, r1 = o.d1 - meas.y;
  double half_rho;
  const double sr = loss_scale(r0, r1, flags, cauchy_c, &half_rho);
  const double fz = f / o.Xc[2] * sr;
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
  double J0[3], J1[3];
  for (int c = 0; c < 3; c++) {
    J0[c] = G0[0] * rec[c] + G0[1] * rec[3 + c] + G0[2] * rec[6 + c];
    J1[c] = G1[0] * rec[c] + G1[1] * rec[3 + c] + G1[2] * rec[6 + c];
  }
  const double rr0 = r0 * sr, rr1 = r1 * sr;
  V[0] += J0[0] * J0[0] + J1[0] * J1[0];
  V[1] += J0[0] * J0[1] + J1[0] * J1[1];
  V[2] += J0[0] * J0[2] + J1[0] * J1[2];
  V[3] += J0[1] * J0[1] + J1[1] * J1[1];
  V[4] += J0[1] * J0[2] + J1[1] * J1[2];
  V[5] += J0[2] * J0[2] + J1[2] * J1[2];
  for (int c = 0; c < 3; c++) g[c] += J0[c] * rr0 + J1[c] * rr1;
}

// kLanesPerPoint lanes per point (each takes every kLanesPerPoint-th observation),
// combined with two xor-shuffles. MODEL < 0: mixed camera models (runtime
// dispatch per observation); otherwise the single model of the problem.
constexpr int kLanesPerPoint = 4;

// t: thread index of the point role (kLanesPerPoint consecutive threads per point)
template <int MODEL, int DEG>
__device__ __forceinline__ void points_lin_body(
    int64_t t, const int64_t* __restrict__ pt_begin, int64_t npts, const int32_t* __restrict__ po_frame,
    const double2* __restrict__ po_meas, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, double* __restrict__ pgrad, double* __restrict__ phess,
    int32_t flags, double cauchy_c, const PointExtra& dc) {
  const int64_t p = t / kLanesPerPoint;
  const int sub = (int)(t % kLanesPerPoint);
  const bool valid = p < npts;
  double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
  const double4 X = valid ? pts[p] : make_double4(0, 0, 0, 0);
  if (valid && X.w != 0.0) {
    const int64_t jb = pt_begin[p], je = pt_begin[p + 1];
    for (int64_t j = jb + sub; j < je; j += kLanesPerPoint) {
      const int32_t fr = po_frame[j];
      const FrameDesc& F = fd[fr];
      const double* rec = frec + (int64_t)fr * kFrameRecDoubles;
      const double2 m = po_meas[j];
      if constexpr (MODEL >= 0) {
        point_obs<MODEL, DEG>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
      } else {
        const int K = F.K;
        if (K == 0) point_obs<kModelNone, 0>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 1) point_obs<kModelFov, 0>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 4 || K == 5) point_obs<kModelRadtan, 0>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 20) point_obs<kModelRpc, 1>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 44) point_obs<kModelRpc, 2>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 76) point_obs<kModelRpc, 3>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 116) point_obs<kModelRpc, 4>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 164) point_obs<kModelRpc, 5>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
        else if (K == 220) point_obs<kModelRpc, 6>(F, rec, params, X.x, X.y, X.z, m, flags, cauchy_c, V, g);
      }
    }
  }
  if (dc.begin && valid && X.w != 0.0) {
    // BracketedDepthError blocks of this point: J_pt = P I (P = weight * sr)
    const double4* dmeas = reinterpret_cast<const double4*>(dc.meas);
    for (int64_t j = dc.begin[p] + sub; j < dc.begin[p + 1]; j += kLanesPerPoint) {
      const int32_t sl = dc.slot[j];
      const DepthDesc d = dc.dd[sl];
      DepthRows o;
      depth_rows(d, frec + (int64_t)d.frame * kFrameRecDoubles, params, dmeas[sl], X.x, X.y, X.z, flags, cauchy_c,
                 o);
      const double P2 = o.P * o.P;
      V[0] += P2;
      V[3] += P2;
      V[5] += P2;
#pragma unroll
      for (int c = 0; c < 3; c++) g[c] += o.P * o.r[c];
    }
  }
  if (dc.xbegin && valid && X.w != 0.0) {
    // XYZError priors (rig_calibrator.cc:720-724): J_pt = weight * sr * I
    const double4* xref = reinterpret_cast<const double4*>(dc.xref);
    for (int64_t j = dc.xbegin[p] + sub; j < dc.xbegin[p + 1]; j += kLanesPerPoint) {
      const double4 R = xref[j];
      const double r0 = R.w * (X.x - R.x), r1 = R.w * (X.y - R.y), r2 = R.w * (X.z - R.z);
      double hr;
      const double sr = loss_scale3(r0, r1, r2, flags, dc.xcc[j], &hr);
      const double P = R.w * sr;
      V[0] += P * P;
      V[3] += P * P;
      V[5] += P * P;
      g[0] += P * r0 * sr;
      g[1] += P * r1 * sr;
      g[2] += P * r2 * sr;
    }
  }
#pragma unroll
  for (int c = 0; c < 6; c++) V[c] = group_sum_f64<kLanesPerPoint>(V[c]);
#pragma unroll
  for (int c = 0; c < 3; c++) g[c] = group_sum_f64<kLanesPerPoint>(g[c]);
  if (!valid) return;
  // lane `sub` writes entries sub, sub + 4, ... of the 9 outputs
  for (int c = sub; c < 9; c += kLanesPerPoint) {
    if (c < 3) pgrad[3 * p + c] = g[c];
    else phess[6 * p + (c - 3)] = V[c - 3];
  }
}

template <int MODEL, int DEG>
__global__ void __launch_bounds__(256) k_points_lin(
    const int64_t* __restrict__ pt_begin, int64_t npts, const int32_t* __restrict__ po_frame,
    const double2* __restrict__ po_meas, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, double* __restrict__ pgrad, double* __restrict__ phess,
    int32_t flags, double cauchy_c, PointExtra dc) {
  points_lin_body<MODEL, DEG>((int64_t)blockIdx.x * blockDim.x + threadIdx.x, pt_begin, npts, po_frame, po_meas, fd,
                              frec, params, pts, pgrad, phess, flags, cauchy_c, dc);
}

}  // namespace mvba

// ------------------------------------------------------------ launchers
extern "C" {

hipError_t mvba_launch_prep(const mvba::FrameDesc* fd, int64_t nframes, const double* params,
                            double* frec, const int64_t* pt_off, const uint8_t* pt_free, int64_t npts,
                            double4* pts, int gen, int* err, hipStream_t s) {
  const int64_t fb = (nframes * mvba::kThreadsPerFrame + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
  const int64_t pb = (npts + mvba::kPrepBlock * mvba::kPrepPoints - 1) / (mvba::kPrepBlock * mvba::kPrepPoints);
  if (fb + pb == 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_prep, dim3((unsigned)(fb + pb)), dim3(mvba::kPrepBlock), 0, s, fd, nframes,
                     (int32_t)fb, params, frec, pt_off, pt_free, npts, pts, gen, err);
  return hipGetLastError();
}

#define MVBA_SWITCH_MODEL(model, deg, CALL)                        \
  switch (model) {                                                 \
    case mvba::kModelNone: CALL(mvba::kModelNone, 0); break;       \
    case mvba::kModelFov: CALL(mvba::kModelFov, 0); break;         \
    case mvba::kModelRadtan: CALL(mvba::kModelRadtan, 0); break;   \
    case mvba::kModelRpc:                                          \
      switch (deg) {                                               \
        case 1: CALL(mvba::kModelRpc, 1); break;                   \
        case 2: CALL(mvba::kModelRpc, 2); break;                   \
        case 3: CALL(mvba::kModelRpc, 3); break;                   \
        case 4: CALL(mvba::kModelRpc, 4); break;                   \
        case 5: CALL(mvba::kModelRpc, 5); break;                   \
        case 6: CALL(mvba::kModelRpc, 6); break;                   \
        default: return hipErrorInvalidValue;                      \
      }                                                            \
      break;                                                       \
    default: return hipErrorInvalidValue;                          \
  }

// model: ModelKind; deg: RPC degree (1..kMaxRpcDegree) when model == kModelRpc.
hipError_t mvba_launch_obs(int model, int deg, const mvba::Segment* segs, int32_t nseg,
                           const mvba::FrameDesc* fd, const double* frec, const double* params,
                           const double4* pts, const int32_t* obs_pid, const double2* obs_meas,
                           void* res, void* J, int64_t ld, int32_t flags, double cauchy_c, int32_t out_f32,
                           hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  const unsigned blocks = mvba::xcd_grid((nseg + 3) / 4);
#define MVBA_OBS_K(KER, M, D, OT)                                                                            \
  hipLaunchKernelGGL((mvba::KER<M, D, OT>), dim3(blocks), dim3(256), 0, s, segs, nseg, fd, frec, params, pts, \
                     obs_pid, obs_meas, (OT*)res, (OT*)J, ld, flags, cauchy_c)
#define MVBA_OBS(M, D)                                                                                   \
  if (flags & MVBA_EVAL_JACOBIAN) {                                                                      \
    if (out_f32) MVBA_OBS_K(k_obs, M, D, float);                                                         \
    else MVBA_OBS_K(k_obs, M, D, double);                                                                \
  } else {                                                                                               \
    if (out_f32) MVBA_OBS_K(k_obs_res, M, D, float);                                                     \
    else MVBA_OBS_K(k_obs_res, M, D, double);                                                            \
  }
  MVBA_SWITCH_MODEL(model, deg, MVBA_OBS)
#undef MVBA_OBS
#undef MVBA_OBS_K
  return hipGetLastError();
}

// Prep + K1 in one launch (k_eval): K0 blocks, landmark-gather blocks (one
// landmark per thread), then the K1 blocks from a multiple of 8 on. ready:
// >= mvba_eval_ready_words(nframes) words, zero before the first launch; epoch:
// a value no earlier launch on these words used (the handle's generation).
int64_t mvba_eval_ready_words(int64_t nframes) {
  return (nframes * mvba::kThreadsPerFrame + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
}

hipError_t mvba_launch_eval_fused(int model, int deg, const mvba::Segment* segs, int32_t nseg,
                                  const mvba::FrameDesc* fd, int64_t nframes, double* frec, const double* params,
                                  const int64_t* pt_off, const uint8_t* pt_free, int64_t npts, double4* pts,
                                  const int32_t* obs_pid, const double2* obs_meas, void* res, void* J, int64_t ld,
                                  int32_t flags, double cauchy_c, int32_t out_f32, int gen, int* err,
                                  unsigned* ready, unsigned poll_limit, hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  const int64_t fb = mvba_eval_ready_words(nframes);
  const int64_t pb = (npts + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
  const int64_t k1 = (fb + pb + mvba::kXcds - 1) / mvba::kXcds * mvba::kXcds;
  const unsigned blocks = (unsigned)(k1 + mvba::xcd_grid((nseg + 3) / 4));
  const mvba::FusedIn fu{pt_off, pt_free, ready, (unsigned)gen, k1, err, poll_limit};
#define MVBA_EVF_K(M, D, OT, JC)                                                                              \
  hipLaunchKernelGGL((mvba::k_eval<M, D, OT, JC>), dim3(blocks), dim3(256), 0, s, segs, nseg, fd, nframes,      \
                     (int32_t)fb, (int32_t)pb, frec, params, npts, pts, obs_pid, obs_meas, (OT*)res, (OT*)J, ld, \
                     flags, cauchy_c, gen, err, ready, fu)
#define MVBA_EVF(M, D)                                                                                   \
  if (flags & MVBA_EVAL_JACOBIAN) {                                                                      \
    if (out_f32) MVBA_EVF_K(M, D, float, true);                                                          \
    else MVBA_EVF_K(M, D, double, true);                                                                 \
  } else {                                                                                               \
    if (out_f32) MVBA_EVF_K(M, D, float, false);                                                         \
    else MVBA_EVF_K(M, D, double, false);                                                                \
  }
  MVBA_SWITCH_MODEL(model, deg, MVBA_EVF)
#undef MVBA_EVF
#undef MVBA_EVF_K
  return hipGetLastError();
}

// Thin-shard evaluation in one launch (k_eval_local): landmark-gather blocks,
// then the K1 blocks from a multiple of 8 on, whose waves run K0 for their own
// frame. One model group only (every frame has a segment).
hipError_t mvba_launch_eval_local(int model, int deg, const mvba::Segment* segs, int32_t nseg,
                                  const mvba::FrameDesc* fd, double* frec, const double* params,
                                  const int64_t* pt_off, const uint8_t* pt_free, int64_t npts, double4* pts,
                                  const int32_t* obs_pid, const double2* obs_meas, void* res, void* J, int64_t ld,
                                  int32_t flags, double cauchy_c, int32_t out_f32, int gen, int* err,
                                  hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  const int64_t pb = (npts + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
  const int64_t k1 = (pb + mvba::kXcds - 1) / mvba::kXcds * mvba::kXcds;
  const unsigned blocks = (unsigned)(k1 + mvba::xcd_grid((nseg + 3) / 4));
  const mvba::FusedIn fu{pt_off, pt_free, nullptr, (unsigned)gen, k1, err, 0u};
#define MVBA_EVL_K(M, D, OT, JC)                                                                               \
  hipLaunchKernelGGL((mvba::k_eval_local<M, D, OT, JC>), dim3(blocks), dim3(256), 0, s, segs, nseg, (int32_t)pb, \
                     fd, frec, params, npts, pts, obs_pid, obs_meas, (OT*)res, (OT*)J, ld, flags, cauchy_c, fu)
#define MVBA_EVL(M, D)                                                                                   \
  if (flags & MVBA_EVAL_JACOBIAN) {                                                                      \
    if (out_f32) MVBA_EVL_K(M, D, float, true);                                                          \
    else MVBA_EVL_K(M, D, double, true);                                                                 \
  } else {                                                                                               \
    if (out_f32) MVBA_EVL_K(M, D, float, false);                                                         \
    else MVBA_EVL_K(M, D, double, false);                                                                \
  }
  MVBA_SWITCH_MODEL(model, deg, MVBA_EVL)
#undef MVBA_EVL
#undef MVBA_EVL_K
  return hipGetLastError();
}

// Gram width of a model (host side; -1: no fused linearization for it).
int mvba_gram_width(int model, int deg) {
  switch (model) {
    case mvba::kModelNone: return mvba::GramShape<mvba::kModelNone, 0>::kWidth;
    case mvba::kModelFov: return mvba::GramShape<mvba::kModelFov, 0>::kWidth;
    case mvba::kModelRadtan: return mvba::GramShape<mvba::kModelRadtan, 0>::kWidth;
    case mvba::kModelRpc:
      switch (deg) {
        case 1: return mvba::GramShape<mvba::kModelRpc, 1>::kWidth;
        case 2: return mvba::GramShape<mvba::kModelRpc, 2>::kWidth;
        case 3: return mvba::GramShape<mvba::kModelRpc, 3>::kWidth;
        case 4: return mvba::GramShape<mvba::kModelRpc, 4>::kWidth;
        case 5: return mvba::GramShape<mvba::kModelRpc, 5>::kWidth;
        case 6: return mvba::GramShape<mvba::kModelRpc, 6>::kWidth;
        default: return -1;  // the evaluator covers RPC degree <= kMaxRpcDegree
      }
    default: return -1;
  }
}

// Camera side of the linearization into the replicas (one launch per model
// group); with pt_begin non-null the same launch also runs the point side
// (single-model problems: the point blocks follow the frame-part blocks).
hipError_t mvba_launch_frame_lin(int model, int deg, const int4* parts, int32_t nparts, const mvba::Segment* segs,
                                 const mvba::FrameDesc* fd, const void* fl, const double* frec, const double* params,
                                 const double4* pts, const int32_t* obs_pid, const double2* obs_meas, double* rep,
                                 int64_t ng, int64_t nh, int32_t flags, double cauchy_c, const int64_t* pt_begin,
                                 int64_t npts, const int32_t* po_frame, const double2* po_meas, double* pgrad,
                                 double* phess, mvba::PointExtra dc, mvba::Slab sl, int32_t part_base,
                                 double4* obsx_out, hipStream_t s) {
  const bool with_pts = pt_begin != nullptr && npts > 0;
  if (nparts <= 0 && !with_pts) return hipSuccess;
  const mvba::PointLinArgs pa{pt_begin, npts, po_frame, po_meas, pgrad, phess, dc};
#define MVBA_FLIN(M, D)                                                                                    \
  {                                                                                                        \
    using GS = mvba::GramShape<M, D>;                                                                      \
    const int64_t threads = 64 * GS::kWaves;                                                               \
    const int64_t pblocks = with_pts ? (npts * mvba::kLanesPerPoint + threads - 1) / threads : 0;          \
    if (with_pts)                                                                                          \
      hipLaunchKernelGGL((mvba::k_frame_lin<M, D, true>), dim3((unsigned)(nparts + pblocks)),             \
                         dim3((unsigned)threads), GS::kLdsBytes, s, parts, nparts, segs, fd,               \
                         (const mvba::FrameLin*)fl, frec, params, pts, obs_pid, obs_meas, rep, ng, nh, flags, \
                         cauchy_c, pa, sl, part_base, obsx_out);                                           \
    else                                                                                                   \
      hipLaunchKernelGGL((mvba::k_frame_lin<M, D, false>), dim3((unsigned)nparts), dim3((unsigned)threads), \
                         GS::kLdsBytes, s, parts, nparts, segs, fd, (const mvba::FrameLin*)fl, frec, params, \
                         pts, obs_pid, obs_meas, rep, ng, nh, flags, cauchy_c, pa, sl, part_base, obsx_out); \
  }
  switch (model) {
    case mvba::kModelNone: MVBA_FLIN(mvba::kModelNone, 0); break;
    case mvba::kModelFov: MVBA_FLIN(mvba::kModelFov, 0); break;
    case mvba::kModelRadtan: MVBA_FLIN(mvba::kModelRadtan, 0); break;
    case mvba::kModelRpc:
      switch (deg) {
        case 1: MVBA_FLIN(mvba::kModelRpc, 1); break;
        case 2: MVBA_FLIN(mvba::kModelRpc, 2); break;
        case 3: MVBA_FLIN(mvba::kModelRpc, 3); break;
        case 4: MVBA_FLIN(mvba::kModelRpc, 4); break;
        case 5: MVBA_FLIN(mvba::kModelRpc, 5); break;
        case 6: MVBA_FLIN(mvba::kModelRpc, 6); break;
        default: return hipErrorInvalidValue;
      }
      break;
    default: return hipErrorInvalidValue;
  }
#undef MVBA_FLIN
  return hipGetLastError();
}

hipError_t mvba_launch_slab_lin(mvba::SlabTiers t, int64_t grid, const int64_t* begin, const int64_t* pos,
                                const double* val, int64_t ng, int64_t nh, double* grad, double* hess, double* cost,
                                hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_slab_lin, dim3((unsigned)grid), dim3(256), 0, s, t, begin, pos, val, ng, nh, grad, hess,
                     cost);
  return hipGetLastError();
}

hipError_t mvba_launch_rep_reduce(double* rep, int32_t nrep, int64_t ng, int64_t nh, double* grad, double* hess,
                                  double* cost, hipStream_t s) {
  const int64_t n = ng + nh + 1;
  if (nrep % 8 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mvba::k_rep_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rep, nrep, ng, nh,
                     grad, hess, cost);
  return hipGetLastError();
}

int mvba_num_replicas(void) { return mvba::kLinReplicas; }

// model < 0: mixed models (runtime dispatch).
hipError_t mvba_launch_points_lin(int model, int deg, const int64_t* pt_begin, int64_t npts,
                                  const int32_t* po_frame, const double2* po_meas,
                                  const mvba::FrameDesc* fd, const double* frec, const double* params,
                                  const double4* pts, double* pgrad, double* phess, int32_t flags,
                                  double cauchy_c, mvba::PointExtra dc, hipStream_t s) {
  if (npts <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((npts * mvba::kLanesPerPoint + 255) / 256);
#define MVBA_PTS(M, D)                                                                                \
  hipLaunchKernelGGL((mvba::k_points_lin<M, D>), dim3(blocks), dim3(256), 0, s, pt_begin, npts,      \
                     po_frame, po_meas, fd, frec, params, pts, pgrad, phess, flags, cauchy_c, dc)
  if (model < 0) {
    MVBA_PTS(-1, 0);
  } else {
    switch (model) {
      case mvba::kModelNone: MVBA_PTS(mvba::kModelNone, 0); break;
      case mvba::kModelFov: MVBA_PTS(mvba::kModelFov, 0); break;
      case mvba::kModelRadtan: MVBA_PTS(mvba::kModelRadtan, 0); break;
      case mvba::kModelRpc:
        switch (deg) {
          case 1: MVBA_PTS(mvba::kModelRpc, 1); break;
          case 2: MVBA_PTS(mvba::kModelRpc, 2); break;
          case 3: MVBA_PTS(mvba::kModelRpc, 3); break;
          case 4: MVBA_PTS(mvba::kModelRpc, 4); break;
          case 5: MVBA_PTS(mvba::kModelRpc, 5); break;
          case 6: MVBA_PTS(mvba::kModelRpc, 6); break;
          default: return hipErrorInvalidValue;
        }
        break;
      default: return hipErrorInvalidValue;
    }
  }
#undef MVBA_PTS
  return hipGetLastError();
}

size_t mvba_frame_lin_size(void) { return sizeof(mvba::FrameLin); }

}  // extern "C"

#ifdef MVBA_EVAL_STAMPS
extern "C" int mvba_debug_eval_stamps(unsigned long long* out, int n) {
  const int m = n < mvba::kStampWaves * mvba::kStamps ? n : mvba::kStampWaves * mvba::kStamps;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mvba::g_eval_stamps), (size_t)m * sizeof(unsigned long long));
}
#endif
