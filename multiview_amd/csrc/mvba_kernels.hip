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
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "mvba_types.h"
#include "../../include/mvba/mvba.h"

namespace mvba {

// ------------------------------------------------------------ small helpers
__device__ __forceinline__ void quat_to_rot(double x, double y, double z, double w, double* R) {
  // Eigen QuaternionBase::toRotationMatrix [ext], no normalisation.
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
  R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// Eigen Quaternion(Matrix3d) [ext]: Shepperd's method. q = (x, y, z, w).
// Written with constant indices only (no scratch memory).
__device__ __forceinline__ void rot_to_quat(const double* m, double* q) {
  double t = m[0] + m[4] + m[8];
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m[7] - m[5]) * t;
    q[1] = (m[2] - m[6]) * t;
    q[2] = (m[3] - m[1]) * t;
    return;
  }
  int i = 0;
  if (m[4] > m[0]) i = 1;
  if (m[8] > (i == 0 ? m[0] : m[4])) i = 2;
  if (i == 0) {  // j = 1, k = 2
    t = sqrt(m[0] - m[4] - m[8] + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[7] - m[5]) * t;
    q[1] = (m[3] + m[1]) * t;
    q[2] = (m[6] + m[2]) * t;
  } else if (i == 1) {  // j = 2, k = 0
    t = sqrt(m[4] - m[8] - m[0] + 1.0);
    q[1] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[2] - m[6]) * t;
    q[2] = (m[7] + m[5]) * t;
    q[0] = (m[1] + m[3]) * t;
  } else {  // i = 2, j = 0, k = 1
    t = sqrt(m[8] - m[0] - m[4] + 1.0);
    q[2] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[3] - m[1]) * t;
    q[0] = (m[2] + m[6]) * t;
    q[1] = (m[5] + m[7]) * t;
  }
}

// array_to_rigid_transform (dense_map_utils.cc:171-178): normalised quaternion,
// its rotation and 1/|q| (for the derivative through normalize()).
__device__ __forceinline__ void rigid(const double* p, double* R, double* qh, double* inv_norm) {
  double x = p[3], y = p[4], z = p[5], w = p[6];
  const double n2 = x * x + y * y + z * z + w * w;
  double in = 1.0;
  if (n2 > 0.0) {
    const double n = sqrt(n2);
    x /= n; y /= n; z /= n; w /= n;
    in = 1.0 / n;
  }
  qh[0] = x; qh[1] = y; qh[2] = z; qh[3] = w;
  *inv_norm = in;
  quat_to_rot(x, y, z, w, R);
}

// Left generator of d R(q/|q|) / d q_raw[k]:  omega = (2/|q|) vec(e_k (x) q^*).
__device__ __forceinline__ void quat_generator(const double* qh, double s, int k, double* om) {
  const double vx = qh[0], vy = qh[1], vz = qh[2], w = qh[3];
  switch (k) {
    case 0: om[0] = s * w;   om[1] = s * vz;  om[2] = -s * vy; break;
    case 1: om[0] = -s * vz; om[1] = s * w;   om[2] = s * vx;  break;
    case 2: om[0] = s * vy;  om[1] = -s * vx; om[2] = s * w;   break;
    default: om[0] = -s * vx; om[1] = -s * vy; om[2] = -s * vz; break;
  }
}

// omega for a tangent perturbation dq of the (unit) quaternion q:
// 2 vec(dq (x) q^*) = 2 (q_w dq_v - dq_w q_v - dq_v x q_v).
__device__ __forceinline__ void tangent_generator(const double* dq, const double* q, double* om) {
  const double cx = dq[1] * q[2] - dq[2] * q[1];
  const double cy = dq[2] * q[0] - dq[0] * q[2];
  const double cz = dq[0] * q[1] - dq[1] * q[0];
  om[0] = 2.0 * (q[3] * dq[0] - dq[3] * q[0] - cx);
  om[1] = 2.0 * (q[3] * dq[1] - dq[3] * q[1] - cy);
  om[2] = 2.0 * (q[3] * dq[2] - dq[3] * q[2] - cz);
}

__device__ __forceinline__ void matvec(const double* R, const double* a, double* b) {
  b[0] = R[0] * a[0] + R[1] * a[1] + R[2] * a[2];
  b[1] = R[3] * a[0] + R[4] * a[1] + R[5] * a[2];
  b[2] = R[6] * a[0] + R[7] * a[1] + R[8] * a[2];
}

__device__ __forceinline__ void cross(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// Write one pose column record: omega, v = dt - omega x t.
__device__ __forceinline__ void put_col(double* rec, int k, const double* om, const double* dt,
                                        const double* t) {
  double c[3];
  cross(om, t, c);
  double* o = rec + 12 + 6 * k;
  o[0] = om[0]; o[1] = om[1]; o[2] = om[2];
  o[3] = dt[0] - c[0]; o[4] = dt[1] - c[1]; o[5] = dt[2] - c[2];
}

// ------------------------------------------------------------ prep (K0 + point gather)
// One launch: blocks [0, frame_blocks) run K0 with kThreadsPerFrame lanes per
// frame (each lane recomputes the frame's common part and emits a subset of the
// 22 pose columns); the remaining blocks gather the points.
constexpr int kThreadsPerFrame = 16;
constexpr int kPrepBlock = 256;

__device__ void frame_columns(const FrameDesc& F, const double* __restrict__ params, double* rec,
                              int sub, int gen, int* err) {
  const double* p0 = params + F.off[MVBA_BLK_BEG];
  double R0[9], qh0[4], in0;
  rigid(p0, R0, qh0, &in0);
  const double t0[3] = {p0[0], p0[1], p0[2]};

  if (F.sb == F.se) {
    // rig_calibrator.cc:371-374 — reference camera or --no_rig: T = rigid(p0).
    if (sub == 0) {
      for (int k = 0; k < 9; k++) rec[k] = R0[k];
      rec[9] = t0[0]; rec[10] = t0[1]; rec[11] = t0[2];
    }
    for (int k = sub; k < kPoseCols; k += kThreadsPerFrame) {
      double om[3] = {0.0, 0.0, 0.0}, dt[3] = {0.0, 0.0, 0.0};
      if (k < 3) {
        dt[k] = 1.0;
      } else if (k < 7) {
        quat_generator(qh0, 2.0 * in0, k - 3, om);
      }
      put_col(rec, k, om, dt, t0);
    }
    return;
  }

  const double* p1 = params + F.off[MVBA_BLK_END];
  const double* p2 = params + F.off[MVBA_BLK_REF_TO_CAM];
  const double off = params[F.off[MVBA_BLK_OFFSET]];
  double R1[9], qh1[4], in1, R2[9], qh2[4], in2;
  rigid(p1, R1, qh1, &in1);
  rigid(p2, R2, qh2, &in2);
  const double t1[3] = {p1[0], p1[1], p1[2]};
  const double t2[3] = {p2[0], p2[1], p2[2]};

  // rig_calibrator.cc:343-346 (big stamps subtracted first).
  const double alpha = ((F.sc - F.sb) - off) / (F.se - F.sb);
  if (sub == 0 && (alpha < 0.0 || alpha > 1.0)) atomicMax(err, gen);

  // linearInterp with Eigen slerp [ext] (dense_map_utils.cc:315-329).
  double q0[4], q1[4];
  rot_to_quat(R0, q0);
  rot_to_quat(R1, q1);
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
    const double S = sin(th), C = cos(th);
    const double s0 = sin((1.0 - alpha) * th), c0 = cos((1.0 - alpha) * th);
    const double s1 = sin(alpha * th), c1 = cos(alpha * th);
    w0 = s0 / S;
    w1 = s1 / S;
    dw0_dth = ((1.0 - alpha) * c0 * S - s0 * C) / (S * S);
    dw1_dth = (alpha * c1 * S - s1 * C) / (S * S);
    dw0_da = -th * c0 / S;
    dw1_da = th * c1 / S;
    dth_dD = -1.0 / S;
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
    for (int k = 0; k < 9; k++) rec[k] = Rw[k];
    rec[9] = tw[0]; rec[10] = tw[1]; rec[11] = tw[2];
  }

  for (int k = sub; k < kPoseCols; k += kThreadsPerFrame) {
    double om[3] = {0.0, 0.0, 0.0}, dt[3] = {0.0, 0.0, 0.0};
    if (k < 3 || (k >= 7 && k < 10) || (k >= 14 && k < 17)) {
      // translation columns of beg / end / ref_to_cam
      const int j = (k < 3) ? k : (k < 10) ? k - 7 : k - 14;
      const double scale = (k < 3) ? (1.0 - alpha) : (k < 10) ? alpha : 0.0;
      if (k >= 14) {
        dt[j] = 1.0;
      } else {
        dt[0] = scale * R2[j]; dt[1] = scale * R2[3 + j]; dt[2] = scale * R2[6 + j];
      }
    } else if (k < 14) {
      // quaternion columns of beg (3..6) and end (10..13) through slerp
      const bool side = (k >= 10);
      const int kk = side ? k - 10 : k - 3;
      const double* qh = side ? qh1 : qh0;
      const double sc = side ? sig1 * in1 : sig0 * in0;
      const double* qo = side ? q0 : q1;
      double dq[4];
      for (int m = 0; m < 4; m++) dq[m] = sc * ((m == kk ? 1.0 : 0.0) - qh[m] * qh[kk]);
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
    put_col(rec, k, om, dt, tw);
  }
}

__global__ void __launch_bounds__(kPrepBlock) k_prep(const FrameDesc* __restrict__ fd, int64_t nframes,
                                                     int32_t frame_blocks, const double* __restrict__ params,
                                                     double* __restrict__ frec, const int64_t* __restrict__ pt_off,
                                                     const uint8_t* __restrict__ pt_free, int64_t npts,
                                                     double4* __restrict__ pts, int gen, int* __restrict__ err) {
  if ((int)blockIdx.x < frame_blocks) {
    const int64_t t = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x;
    const int64_t f = t / kThreadsPerFrame;
    if (f >= nframes) return;
    const FrameDesc F = fd[f];
    frame_columns(F, params, frec + f * kFrameRecDoubles, (int)(t % kThreadsPerFrame), gen, err);
  } else {
    const int64_t p = (int64_t)(blockIdx.x - frame_blocks) * kPrepBlock + threadIdx.x;
    if (p >= npts) return;
    const int64_t o = pt_off[p];
    pts[p] = make_double4(params[o], params[o + 1], params[o + 2], pt_free[p] ? 1.0 : 0.0);
  }
}

// ------------------------------------------------------------ K1: observations
template <int MODEL, int DEG>
struct Distortion;

// Common output of a distortion model at one observation.
//   d     : distorted pixel (with the half size added back)
//   A     : d(d)/d(u) (u = f * hnormalized(Xc))
//   df    : total d(d)/d(f)
// and writes its own distortion block columns.

__device__ __forceinline__ void stj(double* J, int64_t ld, int row, int64_t i, double v) {
  __builtin_nontemporal_store(v, J + (int64_t)row * ld + i);
}

template <int MODEL, int DEG>
__global__ void __launch_bounds__(256) k_obs(
    const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
    const double2* __restrict__ obs_meas, double* __restrict__ res, double* __restrict__ J,
    int64_t ld, int32_t flags, double cauchy_c) {
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= nseg) return;
  const Segment sg = segs[wave];
  const int begin = __builtin_amdgcn_readfirstlane(sg.begin);
  const int count = __builtin_amdgcn_readfirstlane(sg.count);
  const int frame = __builtin_amdgcn_readfirstlane(sg.frame);
  if (lane >= count) return;
  const int64_t i = (int64_t)begin + lane;

  const FrameDesc& F = fd[frame];
  const double* __restrict__ rec = frec + (int64_t)frame * kFrameRecDoubles;
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  const double* __restrict__ kd = params + F.off[MVBA_BLK_DIST];
  const double h0 = F.h0, h1 = F.h1;
  const int free_mask = F.free_mask;
  const bool want_jac = (flags & MVBA_EVAL_JACOBIAN) != 0;

  const int pid = obs_pid[i];
  const double4 P = pts[pid];
  const double2 meas = obs_meas[i];

  // X = world_to_cam * X (rig_calibrator.cc:470)
  double Xc[3];
  Xc[0] = rec[0] * P.x + rec[1] * P.y + rec[2] * P.z + rec[9];
  Xc[1] = rec[3] * P.x + rec[4] * P.y + rec[5] * P.z + rec[10];
  Xc[2] = rec[6] * P.x + rec[7] * P.y + rec[8] * P.z + rec[11];
  // u = f .* X.hnormalized() (:473)
  const double nx = Xc[0] / Xc[2];
  const double ny = Xc[1] / Xc[2];
  const double u0 = f * nx, u1 = f * ny;

  double d0, d1, A00, A01, A10, A11, df0, df1;
  // Model-specific intermediates kept for the distortion columns.
  double m0 = 0, m1 = 0, r2 = 0, aux0 = 0, aux1 = 0, aux2 = 0;
  if constexpr (MODEL == kModelNone) {
    // camera_params.cc:268 then + half size (:414)
    d0 = ((u0 + c0) - h0) + h0;
    d1 = ((u1 + c1) - h1) + h1;
    A00 = 1.0; A01 = 0.0; A10 = 0.0; A11 = 1.0;
    df0 = nx; df1 = ny;
  } else if constexpr (MODEL == kModelFov) {
    // camera_params.cc:269-281, precalcs :185-190
    const double w = kd[0];
    const double tw2 = tan(0.5 * w);
    const double pc1 = 1.0 / w, pc2 = 2.0 * tw2;
    m0 = u0 / f; m1 = u1 / f;
    const double ru = sqrt(m0 * m0 + m1 * m1);
    const double a = ru * pc2;
    const double at = atan(a);
    const double rd = at * pc1;
    double conv = 1.0, dconv_dru = 0.0, dconv_dw = 0.0;
    if (ru > 1e-5) {
      conv = rd / ru;
      const double den = 1.0 / (1.0 + a * a);
      dconv_dru = (pc1 * pc2 * den - conv) / ru;
      dconv_dw = (ru * pc1 * (1.0 + tw2 * tw2) * den - at / (w * w)) / ru;
    }
    d0 = ((c0 - h0) + conv * (m0 * f)) + h0;
    d1 = ((c1 - h1) + conv * (m1 * f)) + h1;
    const double g = (ru > 1e-5) ? dconv_dru / ru : 0.0;
    A00 = conv + g * m0 * m0; A01 = g * m0 * m1;
    A10 = g * m1 * m0;        A11 = conv + g * m1 * m1;
    df0 = conv * m0; df1 = conv * m1;
    aux0 = f * dconv_dw;
  } else if constexpr (MODEL == kModelRadtan) {
    // camera_params.cc:282-308 (Tsai)
    const double k1 = kd[0], k2 = kd[1], p1 = kd[2], p2 = kd[3];
    const double k3 = (F.K == 5) ? kd[4] : 0.0;
    m0 = u0 / f; m1 = u1 / f;
    r2 = m0 * m0 + m1 * m1;
    const double radial = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2;
    double e0 = radial * m0, e1 = radial * m1;
    e0 += 2.0 * p1 * m0 * m1 + p2 * (r2 + 2.0 * m0 * m0);
    e1 += p1 * (r2 + 2.0 * m1 * m1) + 2.0 * p2 * m0 * m1;
    d0 = (e0 * f + (c0 - h0)) + h0;
    d1 = (e1 * f + (c1 - h1)) + h1;
    const double drad = k1 + 2.0 * k2 * r2 + 3.0 * k3 * r2 * r2;
    const double cross_t = 2.0 * drad * m0 * m1 + 2.0 * p1 * m0 + 2.0 * p2 * m1;
    A00 = radial + 2.0 * drad * m0 * m0 + 2.0 * p1 * m1 + 6.0 * p2 * m0;
    A01 = cross_t;
    A10 = cross_t;
    A11 = radial + 2.0 * drad * m1 * m1 + 6.0 * p1 * m1 + 2.0 * p2 * m0;
    df0 = e0; df1 = e1;
  } else {
    // RPC of degree DEG (rpc_distortion.cc:116-160); coefficients
    // [num_x(nl) | den_x(nl-1) | num_y(nl) | den_y(nl-1)], nl = (D+1)(D+2)/2.
    constexpr int nl = (DEG + 1) * (DEG + 2) / 2;
    double px[DEG + 1], py[DEG + 1];
    double vx = 1.0, vy = 1.0;
#pragma unroll
    for (int k = 0; k <= DEG; k++) {
      px[k] = vx; vx *= u0;
      py[k] = vy; vy *= u1;
    }
    double N[4] = {0.0, 1.0, 0.0, 1.0};  // Nx, Dx, Ny, Dy
    double Nx_[4] = {0.0, 0.0, 0.0, 0.0}, Ny_[4] = {0.0, 0.0, 0.0, 0.0};  // d/dx, d/dy
    int ci = 0;
#pragma unroll
    for (int cnt = 0; cnt < 4; cnt++) {
      const int start = (cnt & 1);
#pragma unroll
      for (int dg = start; dg <= DEG; dg++) {
#pragma unroll
        for (int q = 0; q <= dg; q++) {
          const double a = kd[ci];
          N[cnt] += a * px[dg - q] * py[q];
          if (dg - q > 0) Nx_[cnt] += a * (double)(dg - q) * px[dg - q - 1] * py[q];
          if (q > 0) Ny_[cnt] += a * (double)q * px[dg - q] * py[q - 1];
          ci++;
        }
      }
    }
    (void)nl;
    d0 = N[0] / N[1] + h0;
    d1 = N[2] / N[3] + h1;
    const double iDx = 1.0 / N[1], iDy = 1.0 / N[3];
    const double qx = N[0] * iDx, qy = N[2] * iDy;
    A00 = (Nx_[0] - qx * Nx_[1]) * iDx; A01 = (Ny_[0] - qx * Ny_[1]) * iDx;
    A10 = (Nx_[2] - qy * Nx_[3]) * iDy; A11 = (Ny_[2] - qy * Ny_[3]) * iDy;
    df0 = A00 * nx + A01 * ny;
    df1 = A10 * nx + A11 * ny;
    aux0 = iDx; aux1 = iDy; aux2 = qx; m0 = qy; m1 = 0.0;
    r2 = 0.0;
    // keep powers for the coefficient columns below (recomputed, cheap)
  }

  double r0 = d0 - meas.x;  // rig_calibrator.cc:478-479
  double r1 = d1 - meas.y;
  double sr = 1.0;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    // Ceres 1.14 CauchyLoss + Corrector [ext]: scale by sqrt(rho').
    const double s = r0 * r0 + r1 * r1;
    const double inv = 1.0 / (1.0 + s * cauchy_c);
    sr = sqrt(fmax(DBL_MIN, inv));
    r0 *= sr;
    r1 *= sr;
  }
  if (res) {
    __builtin_nontemporal_store(r0, res + i);
    __builtin_nontemporal_store(r1, res + ld + i);
  }
  if (!want_jac) return;

  // G = A * du/dXc, du/dXc = (f/z) [[1, 0, -nx], [0, 1, -ny]]; scaled by the loss.
  const double fz = f / Xc[2] * sr;
  double G0[3] = {fz * A00, fz * A01, -fz * (A00 * nx + A01 * ny)};
  double G1[3] = {fz * A10, fz * A11, -fz * (A10 * nx + A11 * ny)};
  double a0[3], a1[3];
  cross(Xc, G0, a0);
  cross(Xc, G1, a1);

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
      const double* o = rec + 12 + 6 * (k0 + c);
      const double j0 = a0[0] * o[0] + a0[1] * o[1] + a0[2] * o[2] + G0[0] * o[3] + G0[1] * o[4] + G0[2] * o[5];
      const double j1 = a1[0] * o[0] + a1[1] * o[1] + a1[2] * o[2] + G1[0] * o[3] + G1[1] * o[4] + G1[2] * o[5];
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
    stj(J, ld, MVBA_JAC_BASE_FOCAL, i, df0 * sr);
    stj(J, ld, MVBA_JAC_BASE_FOCAL + 1, i, df1 * sr);
  }
  if (free_mask & (1 << MVBA_BLK_CENTER)) {
    const double cc = (MODEL == kModelRpc) ? 0.0 : sr;  // RPC ignores the optical centre
    stj(J, ld, MVBA_JAC_BASE_CENTER + 0, i, cc);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 1, i, 0.0);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 2, i, 0.0);
    stj(J, ld, MVBA_JAC_BASE_CENTER + 3, i, cc);
  }
  if (!(free_mask & (1 << MVBA_BLK_DIST))) return;
  if constexpr (MODEL == kModelFov) {
    stj(J, ld, MVBA_JAC_BASE_DIST + 0, i, m0 * aux0 * sr);
    stj(J, ld, MVBA_JAC_BASE_DIST + 1, i, m1 * aux0 * sr);
  } else if constexpr (MODEL == kModelRadtan) {
    const int K = F.K;
    const double fs = f * sr;
    const double r4 = r2 * r2;
    const double cols0[5] = {r2 * m0, r4 * m0, 2.0 * m0 * m1, r2 + 2.0 * m0 * m0, r4 * r2 * m0};
    const double cols1[5] = {r2 * m1, r4 * m1, r2 + 2.0 * m1 * m1, 2.0 * m0 * m1, r4 * r2 * m1};
    for (int c = 0; c < K; c++) {
      stj(J, ld, MVBA_JAC_BASE_DIST + c, i, fs * cols0[c]);
      stj(J, ld, MVBA_JAC_BASE_DIST + K + c, i, fs * cols1[c]);
    }
  } else if constexpr (MODEL == kModelRpc) {
    constexpr int nl = (DEG + 1) * (DEG + 2) / 2;
    constexpr int nhalf = 4 * nl - 2;  // distortion coefficients used
    constexpr int K = 2 * nhalf;
    double px[DEG + 1], py[DEG + 1];
    double vx = 1.0, vy = 1.0;
#pragma unroll
    for (int k = 0; k <= DEG; k++) {
      px[k] = vx; vx *= u0;
      py[k] = vy; vy *= u1;
    }
    const double iDx = aux0 * sr, iDy = aux1 * sr;
    const double mqx = -aux2 * iDx, mqy = -m0 * iDy;  // -(N/D)/D
    int ci = 0;
#pragma unroll
    for (int cnt = 0; cnt < 4; cnt++) {
      const int start = (cnt & 1);
      const double s = (cnt == 0) ? iDx : (cnt == 1) ? mqx : (cnt == 2) ? iDy : mqy;
      const int row = (cnt < 2) ? 0 : 1;
#pragma unroll
      for (int dg = start; dg <= DEG; dg++) {
#pragma unroll
        for (int q = 0; q <= dg; q++) {
          const double mono = px[dg - q] * py[q];
          stj(J, ld, MVBA_JAC_BASE_DIST + row * K + ci, i, s * mono);
          stj(J, ld, MVBA_JAC_BASE_DIST + (1 - row) * K + ci, i, 0.0);
          ci++;
        }
      }
    }
    // Undistortion half: structurally zero.
#pragma unroll 4
    for (int c = nhalf; c < K; c++) {
      stj(J, ld, MVBA_JAC_BASE_DIST + c, i, 0.0);
      stj(J, ld, MVBA_JAC_BASE_DIST + K + c, i, 0.0);
    }
  }
}

}  // namespace mvba

// ------------------------------------------------------------ launchers
extern "C" {

hipError_t mvba_launch_prep(const mvba::FrameDesc* fd, int64_t nframes, const double* params,
                            double* frec, const int64_t* pt_off, const uint8_t* pt_free, int64_t npts,
                            double4* pts, int gen, int* err, hipStream_t s) {
  const int64_t fb = (nframes * mvba::kThreadsPerFrame + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
  const int64_t pb = (npts + mvba::kPrepBlock - 1) / mvba::kPrepBlock;
  if (fb + pb == 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_prep, dim3((unsigned)(fb + pb)), dim3(mvba::kPrepBlock), 0, s, fd, nframes,
                     (int32_t)fb, params, frec, pt_off, pt_free, npts, pts, gen, err);
  return hipGetLastError();
}

// model: ModelKind; deg: RPC degree (1..kMaxRpcDegree) when model == kModelRpc.
hipError_t mvba_launch_obs(int model, int deg, const mvba::Segment* segs, int32_t nseg,
                           const mvba::FrameDesc* fd, const double* frec, const double* params,
                           const double4* pts, const int32_t* obs_pid, const double2* obs_meas,
                           double* res, double* J, int64_t ld, int32_t flags, double cauchy_c,
                           hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((nseg + 3) / 4);
#define MVBA_LAUNCH(M, D)                                                                      \
  hipLaunchKernelGGL((mvba::k_obs<M, D>), dim3(blocks), dim3(256), 0, s, segs, nseg, fd, frec, \
                     params, pts, obs_pid, obs_meas, res, J, ld, flags, cauchy_c)
  switch (model) {
    case mvba::kModelNone: MVBA_LAUNCH(mvba::kModelNone, 0); break;
    case mvba::kModelFov: MVBA_LAUNCH(mvba::kModelFov, 0); break;
    case mvba::kModelRadtan: MVBA_LAUNCH(mvba::kModelRadtan, 0); break;
    case mvba::kModelRpc:
      switch (deg) {
        case 1: MVBA_LAUNCH(mvba::kModelRpc, 1); break;
        case 2: MVBA_LAUNCH(mvba::kModelRpc, 2); break;
        case 3: MVBA_LAUNCH(mvba::kModelRpc, 3); break;
        case 4: MVBA_LAUNCH(mvba::kModelRpc, 4); break;
        case 5: MVBA_LAUNCH(mvba::kModelRpc, 5); break;
        case 6: MVBA_LAUNCH(mvba::kModelRpc, 6); break;
        default: return hipErrorInvalidValue;
      }
      break;
    default: return hipErrorInvalidValue;
  }
#undef MVBA_LAUNCH
  return hipGetLastError();
}

}  // extern "C"
