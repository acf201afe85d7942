// mvba_depth.h — BracketedDepthError row math shared by the depth kernels
// (mvba_depth.hip) and the point-order passes (k_points_lin, k_pass_a).
#ifndef MVBA_DEPTH_H_
#define MVBA_DEPTH_H_

#include "mvba_device.h"

namespace mvba {

// Eigen Matrix3d::inverse (cofactors / determinant) as restated in oracle.cpp's
// affine_inverse (Affine3d::inverse in Affine mode [ext]).
__device__ __forceinline__ void inverse3(const double* m, double* o) {
  const double c00 = m[4] * m[8] - m[5] * m[7];
  const double c10 = m[5] * m[6] - m[3] * m[8];
  const double c20 = m[3] * m[7] - m[4] * m[6];
  const double det = c00 * m[0] + c10 * m[1] + c20 * m[2];
  const double inv = 1.0 / det;
  o[0] = c00 * inv;
  o[1] = (m[2] * m[7] - m[1] * m[8]) * inv;
  o[2] = (m[1] * m[5] - m[2] * m[4]) * inv;
  o[3] = c10 * inv;
  o[4] = (m[0] * m[8] - m[2] * m[6]) * inv;
  o[5] = (m[2] * m[3] - m[0] * m[5]) * inv;
  o[6] = c20 * inv;
  o[7] = (m[1] * m[6] - m[0] * m[7]) * inv;
  o[8] = (m[0] * m[4] - m[1] * m[3]) * inv;
}

__device__ __forceinline__ double loss_scale3(double r0, double r1, double r2, int32_t flags, double cauchy_c,
                                              double* half_rho) {
  const double s = r0 * r0 + r1 * r1 + r2 * r2;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    const double sum = 1.0 + s * cauchy_c;
    *half_rho = 0.5 * (log(sum) / cauchy_c);
    return sqrt(fmax(DBL_MIN, 1.0 / sum));
  }
  *half_rho = 0.5 * s;
  return 1.0;
}

// Residual and Jacobian rows of one depth block, all multiplied by the loss
// scale sr (Ceres' corrector for Cauchy, alpha = 0).
struct DepthRows {
  double r[3];       // corrected residual
  double rr[3];      // raw residual (host corrector path)
  double Z[3][6];    // pose rows: J_pose(i, k) = Z[i] . w_k
  double D[3][12];   // depth_to_image rows (dti_n used)
  double S[3];       // scale column
  double P;          // xyz: P * identity
  double sr, half_rho;
};

__device__ __forceinline__ void depth_rows(const DepthDesc& d, const double* __restrict__ rec,
                                           const double* __restrict__ params, double4 m, double X0, double X1,
                                           double X2, int32_t flags, double cauchy_c, DepthRows& o) {
  const double* p = params + d.dti_off;
  // rigid (7) and affine (12) forms computed side by side and selected by value:
  // branch-local stores into the same arrays defeat SROA (scratch spills)
  const bool aff = (d.dti_n == 12);
  double Rr[9], qh[4], in;
  rigid(p, Rr, qh, &in);
  double A[9], b[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int c = 0; c < 3; c++) A[3 * r + c] = aff ? p[4 * r + c] : Rr[3 * r + c];
    b[r] = aff ? p[4 * r + 3] : p[r];
  }
  const double s = params[d.scale_off];
  const double w = m.w;
  double Am[3];
#pragma unroll
  for (int r = 0; r < 3; r++) Am[r] = A[3 * r] * m.x + A[3 * r + 1] * m.y + A[3 * r + 2] * m.z;
  // (linear * scale) * meas + translation, in Eigen's order: ((s A) m) + b
  double M[3];
#pragma unroll
  for (int r = 0; r < 3; r++) M[r] = (s * A[3 * r]) * m.x + (s * A[3 * r + 1]) * m.y + (s * A[3 * r + 2]) * m.z + b[r];
  double Ri[9];
  inverse3(rec, Ri);
  const double ti[3] = {-(Ri[0] * rec[9] + Ri[1] * rec[10] + Ri[2] * rec[11]),
                        -(Ri[3] * rec[9] + Ri[4] * rec[10] + Ri[5] * rec[11]),
                        -(Ri[6] * rec[9] + Ri[7] * rec[10] + Ri[8] * rec[11])};
  const double X[3] = {X0, X1, X2};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const double Mw = Ri[3 * i] * M[0] + Ri[3 * i + 1] * M[1] + Ri[3 * i + 2] * M[2] + ti[i];
    o.rr[i] = w * (X[i] - Mw);
  }
  const double sr = loss_scale3(o.rr[0], o.rr[1], o.rr[2], flags, cauchy_c, &o.half_rho);
  o.sr = sr;
  const double ws = w * sr;
  o.P = ws;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    o.r[i] = o.rr[i] * sr;
    const double ri[3] = {Ri[3 * i], Ri[3 * i + 1], Ri[3 * i + 2]};
    double mx[3];
    cross(M, ri, mx);
#pragma unroll
    for (int q = 0; q < 3; q++) {
      o.Z[i][q] = ws * mx[q];
      o.Z[i][3 + q] = ws * ri[q];
    }
    o.S[i] = -ws * (ri[0] * Am[0] + ri[1] * Am[1] + ri[2] * Am[2]);
    double aD[12], rD[12];
#pragma unroll
    for (int rr = 0; rr < 3; rr++) {
      const double g = -ws * ri[rr];
      aD[4 * rr] = g * s * m.x;
      aD[4 * rr + 1] = g * s * m.y;
      aD[4 * rr + 2] = g * s * m.z;
      aD[4 * rr + 3] = g;
    }
    // rigid: translation, then quaternion dM/dq_k = s (om_k x Am) -> -ws s om_k . (Am x ri)
#pragma unroll
    for (int j = 0; j < 3; j++) rD[j] = -ws * ri[j];
    double axr[3];
    cross(Am, ri, axr);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      double om[3];
      quat_generator(qh, 2.0 * in, k, om);
      rD[3 + k] = -ws * s * (om[0] * axr[0] + om[1] * axr[1] + om[2] * axr[2]);
    }
#pragma unroll
    for (int q = 7; q < 12; q++) rD[q] = 0.0;
#pragma unroll
    for (int q = 0; q < 12; q++) o.D[i][q] = aff ? aD[q] : rD[q];
  }
}

// Compact form for the solver products (no explicit Jacobian rows):
//   J_cam,d x  = P Rinv (w_u x M + v_u - dM),   dM = dM/dtheta x_theta (+ Am x_scale)
//   J_cam,d^T u: rho = Rinv^T u;  pose (6) = P [M x rho ; rho];
//                depth_to_image = -P rho . dM/dtheta;  scale = -P rho . Am
struct DepthCore {
  double M[3], Am[3], Ri[9];
  double qh[4], in, s, P;
  double r[3];  // corrected residual
  bool aff;
};

__device__ __forceinline__ void depth_core(const DepthDesc& d, const double* __restrict__ rec,
                                           const double* __restrict__ params, double4 m, double X0, double X1,
                                           double X2, int32_t flags, double cauchy_c, DepthCore& c) {
  const double* p = params + d.dti_off;
  c.aff = (d.dti_n == 12);
  double Rr[9];
  rigid(p, Rr, c.qh, &c.in);
  double A[9], b[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int k = 0; k < 3; k++) A[3 * r + k] = c.aff ? p[4 * r + k] : Rr[3 * r + k];
    b[r] = c.aff ? p[4 * r + 3] : p[r];
  }
  c.s = params[d.scale_off];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    c.Am[r] = A[3 * r] * m.x + A[3 * r + 1] * m.y + A[3 * r + 2] * m.z;
    c.M[r] = (c.s * A[3 * r]) * m.x + (c.s * A[3 * r + 1]) * m.y + (c.s * A[3 * r + 2]) * m.z + b[r];
  }
  inverse3(rec, c.Ri);
  const double X[3] = {X0, X1, X2};
  double rr[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const double ti = -(c.Ri[3 * i] * rec[9] + c.Ri[3 * i + 1] * rec[10] + c.Ri[3 * i + 2] * rec[11]);
    const double Mw = c.Ri[3 * i] * c.M[0] + c.Ri[3 * i + 1] * c.M[1] + c.Ri[3 * i + 2] * c.M[2] + ti;
    rr[i] = m.w * (X[i] - Mw);
  }
  double hr;
  const double sr = loss_scale3(rr[0], rr[1], rr[2], flags, cauchy_c, &hr);
  c.P = m.w * sr;
#pragma unroll
  for (int i = 0; i < 3; i++) c.r[i] = rr[i] * sr;
}

// dM = dM/dtheta . x_theta + Am x_scale for the camera-side step x (entries at goff)
__device__ __forceinline__ void depth_dM(const DepthDesc& d, const DepthCore& c, const double4& m,
                                         const double* __restrict__ x, double* dM) {
  dM[0] = dM[1] = dM[2] = 0.0;
  if (d.goff_dti >= 0) {
    const double* xd = x + d.goff_dti;
    if (c.aff) {
#pragma unroll
      for (int r = 0; r < 3; r++)
        dM[r] = c.s * (xd[4 * r] * m.x + xd[4 * r + 1] * m.y + xd[4 * r + 2] * m.z) + xd[4 * r + 3];
    } else {
      // translation + combined quaternion generator om = sum_k om_k x_{3+k}
      double om[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        double ok[3];
        quat_generator(c.qh, 2.0 * c.in, k, ok);
#pragma unroll
        for (int q = 0; q < 3; q++) om[q] += ok[q] * xd[3 + k];
      }
      double t[3];
      cross(om, c.Am, t);
#pragma unroll
      for (int r = 0; r < 3; r++) dM[r] = xd[r] + c.s * t[r];
    }
  }
  if (d.goff_scale >= 0) {
    const double xs = x[d.goff_scale];
#pragma unroll
    for (int r = 0; r < 3; r++) dM[r] += c.Am[r] * xs;
  }
}

// z = J_cam,d x given the frame's u = [w_u ; v_u] and the camera-side vector x
__device__ __forceinline__ void depth_jx(const DepthDesc& d, const DepthCore& c, const double4& m,
                                         const double* __restrict__ u, const double* __restrict__ x, double* z) {
  double dM[3];
  depth_dM(d, c, m, x, dM);
  double wm[3];
  cross(u, c.M, wm);
  const double v[3] = {wm[0] + u[3] - dM[0], wm[1] + u[4] - dM[1], wm[2] + u[5] - dM[2]};
#pragma unroll
  for (int i = 0; i < 3; i++) z[i] = c.P * (c.Ri[3 * i] * v[0] + c.Ri[3 * i + 1] * v[1] + c.Ri[3 * i + 2] * v[2]);
}

// J_cam,d^T u: pose (6, frame-local), depth_to_image (12, dti_n used), scale
__device__ __forceinline__ void depth_jtu(const DepthCore& c, const double4& m, const double* u, double* pose6,
                                          double* dti, double* scale) {
  double rho[3];
#pragma unroll
  for (int q = 0; q < 3; q++) rho[q] = c.Ri[q] * u[0] + c.Ri[3 + q] * u[1] + c.Ri[6 + q] * u[2];
  double mr[3];
  cross(c.M, rho, mr);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    pose6[q] = c.P * mr[q];
    pose6[3 + q] = c.P * rho[q];
  }
  double aD[12], rD[12];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const double g = -c.P * rho[r];
    aD[4 * r] = g * c.s * m.x;
    aD[4 * r + 1] = g * c.s * m.y;
    aD[4 * r + 2] = g * c.s * m.z;
    aD[4 * r + 3] = g;
    rD[r] = g;
  }
  double axr[3];
  cross(c.Am, rho, axr);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double ok[3];
    quat_generator(c.qh, 2.0 * c.in, k, ok);
    rD[3 + k] = -c.P * c.s * (ok[0] * axr[0] + ok[1] * axr[1] + ok[2] * axr[2]);
  }
#pragma unroll
  for (int q = 7; q < 12; q++) rD[q] = 0.0;
#pragma unroll
  for (int q = 0; q < 12; q++) dti[q] = c.aff ? aD[q] : rD[q];
  *scale = -c.P * (rho[0] * c.Am[0] + rho[1] * c.Am[1] + rho[2] * c.Am[2]);
}

// P = weight * sr of one depth block (the xyz Jacobian is P I): residual only.
__device__ __forceinline__ double depth_p(const DepthDesc& d, const double* __restrict__ rec,
                                          const double* __restrict__ params, double4 m, double X0, double X1,
                                          double X2, int32_t flags, double cauchy_c) {
  if (!(flags & MVBA_EVAL_APPLY_LOSS)) return m.w;
  DepthCore c;
  depth_core(d, rec, params, m, X0, X1, X2, flags, cauchy_c, c);
  return c.P;
}

}  // namespace mvba

#endif  // MVBA_DEPTH_H_
