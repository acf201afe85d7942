// mvba_device.h — device-side math shared by the evaluator kernels
// (mvba_kernels.hip) and the solver kernels (mvba_solver.hip).
#ifndef MVBA_DEVICE_H_
#define MVBA_DEVICE_H_

#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "mvba_types.h"
#include "../../include/mvba/mvba.h"

namespace mvba {

// ------------------------------------------------------------ XCD-aware block order
// Workgroups are dealt round-robin over the 8 XCDs (block b -> XCD b % 8), each
// XCD with its own L2. Frame-ordered kernels renumber their blocks so that XCD
// x runs the contiguous range [x per, (x + 1) per) of logical blocks: a frame's
// records (K0 output, projection and direction records) and the landmarks its
// window of frames observes are then fetched into one XCD's L2 instead of all
// eight. Launch xcd_grid(nb) blocks; xcd_block returns -1 for the few surplus
// blocks. MVBA_XCD_MAP=0 keeps the plain order (A/B builds).
#ifndef MVBA_XCD_MAP
#define MVBA_XCD_MAP 1
#endif
constexpr int kXcds = 8;
__host__ __device__ __forceinline__ unsigned xcd_grid(int64_t nb) {
  return MVBA_XCD_MAP ? (unsigned)(((nb + kXcds - 1) / kXcds) * kXcds) : (unsigned)nb;
}
__device__ __forceinline__ int64_t xcd_block_of(int64_t b, int64_t nb) {
  if (!MVBA_XCD_MAP) return b < nb ? b : -1;
  const int64_t per = (nb + kXcds - 1) / kXcds;
  const int64_t l = (b % kXcds) * per + b / kXcds;
  return l < nb ? l : -1;
}
__device__ __forceinline__ int64_t xcd_block(int64_t nb) { return xcd_block_of(blockIdx.x, nb); }
// The CG passes over frame-ordered chunks (pass A, pass B, the |u|^2 sweep)
// and over landmarks (k_point_w: landmarks are numbered by first use in frame
// order) take the same order, so the landmark-side data of a window of frames
// (w_p gathers, c_o records) is fetched into one XCD's L2. MVBA_XCD_SOLVER=0
// keeps the plain order (A/B builds).
#ifndef MVBA_XCD_SOLVER
#define MVBA_XCD_SOLVER 1
#endif
__host__ __device__ __forceinline__ unsigned xcd_grid_solver(int64_t nb) {
  return MVBA_XCD_SOLVER ? (unsigned)(((nb + kXcds - 1) / kXcds) * kXcds) : (unsigned)nb;
}
__device__ __forceinline__ int64_t xcd_block_solver(int64_t nb) {
  const int64_t b = blockIdx.x;
  if (!MVBA_XCD_SOLVER) return b < nb ? b : -1;
  const int64_t per = (nb + kXcds - 1) / kXcds;
  const int64_t l = (b % kXcds) * per + b / kXcds;
  return l < nb ? l : -1;
}

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
// (MVBA_K0_FAST: one reciprocal and four products instead of four divisions:
// the frame record is K0's dependent chain on thin shards, within an ulp of
// Eigen's q / |q|)
#ifndef MVBA_K0_FAST
#define MVBA_K0_FAST 1
#endif
__device__ __forceinline__ void rigid(const double* p, double* R, double* qh, double* inv_norm) {
  double x = p[3], y = p[4], z = p[5], w = p[6];
  const double n2 = x * x + y * y + z * z + w * w;
  double in = 1.0;
  if (n2 > 0.0) {
    const double n = sqrt(n2);
    in = 1.0 / n;
    if (MVBA_K0_FAST) {
      x *= in; y *= in; z *= in; w *= in;
    } else {
      x /= n; y /= n; z /= n; w /= n;
    }
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

// Sum of v over the 64 lanes of a wave, returned to every lane (all lanes
// active) as a wave-uniform value. DPP moves only (VALU, no LDS round trip):
// xor 1 and xor 2 by quad_perm, row_half_mirror and row_mirror give every lane
// its 16-lane row's sum, row_bcast:15 / row_bcast:31 carry the row sums up to
// lane 63, whose total v_readlane returns. The __shfl_xor butterfly it replaces
// costs 12 ds_bpermute_b32 and six dependent LDS round trips per value.
//
// Requirements (gfx9 wave64 only, which is the only target this library
// builds): row_bcast:15/31 exist on GFX9 and not on GFX10+, and the lane-63
// readlane takes the total only if every lane of the wave is active (EXEC all
// ones) at the call. Every caller reduces with the whole wave converged (the
// reductions sit after the per-lane branches, whose inactive lanes contribute
// 0.0). MVBA_DPP_REDUCE=0 builds the shuffle butterfly, which needs neither.
#ifndef MVBA_DPP_REDUCE
#define MVBA_DPP_REDUCE 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && MVBA_DPP_REDUCE
// GFX9 (CDNA) runs wave64 only, so __GFX9__ asserts both the DPP controls and
// the wave size (this clang defines no wavefront-size macro)
#if !defined(__GFX9__)
#error "wave_sum_f64's DPP row_bcast reduction needs a GFX9 wave64 target (gfx950); or set MVBA_DPP_REDUCE=0"
#endif
#endif
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#if MVBA_DPP_REDUCE
  v += dpp_f64<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_f64<0x140, 0xf>(v);  // row_mirror: every lane holds its row's sum
  v += dpp_f64<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v += dpp_f64<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3: lane 63 holds the total
  return readlane_f64(v, 63);
#else
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
#endif
}

// Sum of v over aligned groups of N lanes (N = 4, 8 or 16), returned to every
// lane of the group (all lanes active): the first steps of wave_sum_f64.
template <int N>
__device__ __forceinline__ double group_sum_f64(double v) {
  static_assert(N == 4 || N == 8 || N == 16, "group of 4, 8 or 16 lanes");
#if MVBA_DPP_REDUCE
  v += dpp_f64<0xB1, 0xf>(v);
  v += dpp_f64<0x4E, 0xf>(v);
  if constexpr (N >= 8) v += dpp_f64<0x141, 0xf>(v);
  if constexpr (N >= 16) v += dpp_f64<0x140, 0xf>(v);
#else
  for (int off = 1; off < N; off <<= 1) v += __shfl_xor(v, off, 64);
#endif
  return v;
}

// Sums of NV per-lane values over the wave, TRANSPOSED (all lanes active):
// with P = the power of two >= NV (<= 64) and m = log2 P, each of the first m
// steps pairs every lane with a partner that differs in one lane bit (5, 4, 3,
// 2, 1, 0 in turn) and halves the values a lane holds: the lane keeps the half
// its bit selects and adds the partner's copy of it (the partner sends that
// half). The remaining 6 - m steps add the last value over the lower lane bits.
// On return v[0] of lane l is the total of value l >> (6 - m). Pairings:
// v_permlane32_swap / v_permlane16_swap (gfx950) for bits 5 and 4 (the swap
// itself selects the halves), DPP row_mirror / row_half_mirror / quad_perm
// for bits 3..0. About 4 instructions per value against wave_sum_f64's ~20
// per value (pass B reduces its 14..47 accumulators once per chunk).
__device__ __forceinline__ void swap32_f64(double& x, double& y) {
  const long long bx = __builtin_bit_cast(long long, x), by = __builtin_bit_cast(long long, y);
  const auto lo = __builtin_amdgcn_permlane32_swap((int)bx, (int)by, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((int)(bx >> 32), (int)(by >> 32), false, false);
  x = __builtin_bit_cast(double, ((long long)hi[0] << 32) | (unsigned)lo[0]);
  y = __builtin_bit_cast(double, ((long long)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {
  const long long bx = __builtin_bit_cast(long long, x), by = __builtin_bit_cast(long long, y);
  const auto lo = __builtin_amdgcn_permlane16_swap((int)bx, (int)by, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((int)(bx >> 32), (int)(by >> 32), false, false);
  x = __builtin_bit_cast(double, ((long long)hi[0] << 32) | (unsigned)lo[0]);
  y = __builtin_bit_cast(double, ((long long)hi[1] << 32) | (unsigned)lo[1]);
}
// the partner's v over lane bit B (B = 3, 2, 1, 0), inside a 16-lane row
template <int B>
__device__ __forceinline__ double partner_f64(double v) {
  if constexpr (B == 3) return dpp_f64<0x140, 0xf>(v);  // row_mirror: l <-> 15 - l
  else if constexpr (B == 2) return dpp_f64<0x141, 0xf>(v);  // row_half_mirror: l <-> 7 - l
  else if constexpr (B == 1) return dpp_f64<0x4E, 0xf>(v);  // quad_perm [2,3,0,1]
  else return dpp_f64<0xB1, 0xf>(v);  // quad_perm [1,0,3,2]
}
template <int B, int L>
__device__ __forceinline__ void tsum_step(double* v, int lane) {
  constexpr int H = L / 2;
  if constexpr (B == 5) {
#pragma unroll
    for (int j = 0; j < H; j++) {
      double x = v[j], y = v[j + H];
      swap32_f64(x, y);
      v[j] = x + y;
    }
  } else if constexpr (B == 4) {
#pragma unroll
    for (int j = 0; j < H; j++) {
      double x = v[j], y = v[j + H];
      swap16_f64(x, y);
      v[j] = x + y;
    }
  } else {
    const bool hi = (lane >> B) & 1;
#pragma unroll
    for (int j = 0; j < H; j++) {
      const double keep = hi ? v[j + H] : v[j];
      const double send = hi ? v[j] : v[j + H];
      v[j] = keep + partner_f64<B>(send);
    }
  }
}
template <int B>
__device__ __forceinline__ double plain_step(double x) {
  if constexpr (B == 5) {
    double y = x;
    swap32_f64(x, y);
    return x + y;
  } else if constexpr (B == 4) {
    double y = x;
    swap16_f64(x, y);
    return x + y;
  } else {
    return x + partner_f64<B>(x);
  }
}
template <int NV>
struct TSum {
  static constexpr int P = NV <= 1 ? 1 : NV <= 2 ? 2 : NV <= 4 ? 4 : NV <= 8 ? 8 : NV <= 16 ? 16 : NV <= 32 ? 32 : 64;
  static constexpr int M = P == 1 ? 0 : P == 2 ? 1 : P == 4 ? 2 : P == 8 ? 3 : P == 16 ? 4 : P == 32 ? 5 : 6;
  static constexpr int kShift = 6 - M;  // lane l holds value l >> kShift
};
// w: TSum<NV>::P values (entries NV.. zero), reduced in place
template <int NV>
__device__ __forceinline__ double wave_sum_transpose(double* w, int lane) {
  static_assert(NV >= 1 && NV <= 64, "1..64 values");
  using T = TSum<NV>;
  constexpr int P = T::P, M = T::M;
  // selection steps on bits 5 .. 6 - M (L values -> L / 2)
  if constexpr (M >= 1) tsum_step<5, P>(w, lane);
  if constexpr (M >= 2) tsum_step<4, P / 2>(w, lane);
  if constexpr (M >= 3) tsum_step<3, P / 4>(w, lane);
  if constexpr (M >= 4) tsum_step<2, P / 8>(w, lane);
  if constexpr (M >= 5) tsum_step<1, P / 16>(w, lane);
  if constexpr (M >= 6) tsum_step<0, P / 32>(w, lane);
  // plain sums over the remaining lower bits
  double r = w[0];
  if constexpr (M <= 0) r = plain_step<5>(r);
  if constexpr (M <= 1) r = plain_step<4>(r);
  if constexpr (M <= 2) r = plain_step<3>(r);
  if constexpr (M <= 3) r = plain_step<2>(r);
  if constexpr (M <= 4) r = plain_step<1>(r);
  if constexpr (M <= 5) r = plain_step<0>(r);
  return r;
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

// ------------------------------------------------------------ observation model
// Projection + distortion of one observation (rig_calibrator.cc:470-479,
// camera_params.cc:260-314, rpc_distortion.cc:116-160) with the pieces of its
// analytic derivative that every consumer needs.
struct Proj {
  double Xc[3];
  double nx, ny;           // hnormalized(Xc)
  double u0, u1;           // f * (nx, ny): centred undistorted pixel
  double d0, d1;           // distorted pixel (half size added back)
  double A00, A01, A10, A11;  // d(d)/d(u)
  double df0, df1;         // total d(d)/d(f)
  double m0, m1, r2;       // FOV / RADTAN: u / f, |u/f|^2
  double aux0, aux1, aux2, aux3;  // FOV: f dconv/dw; RPC: 1/Dx, 1/Dy, Nx/Dx, Ny/Dy
  double iz;               // 1 / Xc[2] (FAST projections only)
};

// f / Xc[2] * s: the division as the reference writes it, or (FAST) by the
// reciprocal the FAST projection already took
template <bool FAST>
__device__ __forceinline__ double fz_of(double f, const Proj& o, double s) {
  if constexpr (FAST) return f * o.iz * s;
  else return f / o.Xc[2] * s;
}

// FAST (the CG passes only: their rows feed inner products, never a residual
// or Jacobian an API returns): one reciprocal instead of the reference's
// divisions, u / f taken as X.hnormalized() itself, RPC quotients by the
// denominators' reciprocals. Each fp64 division is a ~12-instruction sequence;
// pass B at c2 issued 6 per observation. Results differ by rounding only.
template <int MODEL, int DEG, bool FAST = false>
__device__ __forceinline__ void project(const double* __restrict__ rec, double X0, double X1, double X2,
                                        double f, double c0, double c1, const double* __restrict__ kd,
                                        int K, double h0, double h1, Proj& o) {
  // X = world_to_cam * X (rig_calibrator.cc:470)
  o.Xc[0] = rec[0] * X0 + rec[1] * X1 + rec[2] * X2 + rec[9];
  o.Xc[1] = rec[3] * X0 + rec[4] * X1 + rec[5] * X2 + rec[10];
  o.Xc[2] = rec[6] * X0 + rec[7] * X1 + rec[8] * X2 + rec[11];
  // u = f .* X.hnormalized() (:473)
  if constexpr (FAST) {
    o.iz = 1.0 / o.Xc[2];
    o.nx = o.Xc[0] * o.iz;
    o.ny = o.Xc[1] * o.iz;
  } else {
    o.nx = o.Xc[0] / o.Xc[2];
    o.ny = o.Xc[1] / o.Xc[2];
  }
  const double u0 = f * o.nx, u1 = f * o.ny;
  o.u0 = u0;
  o.u1 = u1;
  o.m0 = o.m1 = o.r2 = 0.0;
  o.aux0 = o.aux1 = o.aux2 = o.aux3 = 0.0;
  if constexpr (MODEL == kModelNone) {
    // camera_params.cc:268 then + half size (:414)
    o.d0 = ((u0 + c0) - h0) + h0;
    o.d1 = ((u1 + c1) - h1) + h1;
    o.A00 = 1.0; o.A01 = 0.0; o.A10 = 0.0; o.A11 = 1.0;
    o.df0 = o.nx; o.df1 = o.ny;
  } else if constexpr (MODEL == kModelFov) {
    // camera_params.cc:269-281, precalcs :185-190
    const double w = kd[0];
    const double tw2 = tan(0.5 * w);
    const double pc1 = 1.0 / w, pc2 = 2.0 * tw2;
    const double m0 = FAST ? o.nx : u0 / f, m1 = FAST ? o.ny : u1 / f;
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
    o.d0 = ((c0 - h0) + conv * (m0 * f)) + h0;
    o.d1 = ((c1 - h1) + conv * (m1 * f)) + h1;
    const double g = (ru > 1e-5) ? dconv_dru / ru : 0.0;
    o.A00 = conv + g * m0 * m0; o.A01 = g * m0 * m1;
    o.A10 = g * m1 * m0;        o.A11 = conv + g * m1 * m1;
    o.df0 = conv * m0; o.df1 = conv * m1;
    o.m0 = m0; o.m1 = m1;
    o.aux0 = f * dconv_dw;
  } else if constexpr (MODEL == kModelRadtan) {
    // camera_params.cc:282-308 (Tsai)
    const double k1 = kd[0], k2 = kd[1], p1 = kd[2], p2 = kd[3];
    const double k3 = (K == 5) ? kd[4] : 0.0;
    const double m0 = FAST ? o.nx : u0 / f, m1 = FAST ? o.ny : u1 / f;
    const double r2 = m0 * m0 + m1 * m1;
    const double radial = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2;
    double e0 = radial * m0, e1 = radial * m1;
    e0 += 2.0 * p1 * m0 * m1 + p2 * (r2 + 2.0 * m0 * m0);
    e1 += p1 * (r2 + 2.0 * m1 * m1) + 2.0 * p2 * m0 * m1;
    o.d0 = (e0 * f + (c0 - h0)) + h0;
    o.d1 = (e1 * f + (c1 - h1)) + h1;
    const double drad = k1 + 2.0 * k2 * r2 + 3.0 * k3 * r2 * r2;
    const double cross_t = 2.0 * drad * m0 * m1 + 2.0 * p1 * m0 + 2.0 * p2 * m1;
    o.A00 = radial + 2.0 * drad * m0 * m0 + 2.0 * p1 * m1 + 6.0 * p2 * m0;
    o.A01 = cross_t;
    o.A10 = cross_t;
    o.A11 = radial + 2.0 * drad * m1 * m1 + 6.0 * p1 * m1 + 2.0 * p2 * m0;
    o.df0 = e0; o.df1 = e1;
    o.m0 = m0; o.m1 = m1; o.r2 = r2;
  } else {
    // RPC of degree DEG (rpc_distortion.cc:116-160); coefficients
    // [num_x(nl) | den_x(nl-1) | num_y(nl) | den_y(nl-1)], nl = (D+1)(D+2)/2.
    double px[DEG + 1], py[DEG + 1];
    double vx = 1.0, vy = 1.0;
#pragma unroll
    for (int k = 0; k <= DEG; k++) {
      px[k] = vx; vx *= u0;
      py[k] = vy; vy *= u1;
    }
    double N[4] = {0.0, 1.0, 0.0, 1.0};  // Nx, Dx, Ny, Dy
    double Nx_[4] = {0.0, 0.0, 0.0, 0.0}, Ny_[4] = {0.0, 0.0, 0.0, 0.0};
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
    const double iDx = 1.0 / N[1], iDy = 1.0 / N[3];
    if constexpr (FAST) {
      o.d0 = N[0] * iDx + h0;
      o.d1 = N[2] * iDy + h1;
    } else {
      o.d0 = N[0] / N[1] + h0;
      o.d1 = N[2] / N[3] + h1;
    }
    const double qx = N[0] * iDx, qy = N[2] * iDy;
    o.A00 = (Nx_[0] - qx * Nx_[1]) * iDx; o.A01 = (Ny_[0] - qx * Ny_[1]) * iDx;
    o.A10 = (Nx_[2] - qy * Nx_[3]) * iDy; o.A11 = (Ny_[2] - qy * Ny_[3]) * iDy;
    o.df0 = o.A00 * o.nx + o.A01 * o.ny;
    o.df1 = o.A10 * o.nx + o.A11 * o.ny;
    o.aux0 = iDx; o.aux1 = iDy; o.aux2 = qx; o.aux3 = qy;
  }
}

// Number of distortion columns that can be non-zero (RPC: the undistortion
// half is structurally zero).
template <int MODEL, int DEG>
__host__ __device__ constexpr int live_dist_cols(int K) {
  return MODEL == kModelRpc ? 2 * ((DEG + 1) * (DEG + 2)) - 2 : (MODEL == kModelNone ? 0 : K);
}

// Distortion block columns of one observation, emitted as emit(c, v_row0, v_row1)
// for c < live_dist_cols (scaled by s = fs or the loss factor).
template <int MODEL, int DEG, class Emit>
__device__ __forceinline__ void dist_columns(const Proj& o, double f, int K, double s, Emit&& emit) {
  if constexpr (MODEL == kModelFov) {
    emit(0, o.m0 * o.aux0 * s, o.m1 * o.aux0 * s);
  } else if constexpr (MODEL == kModelRadtan) {
    const double fs = f * s;
    const double m0 = o.m0, m1 = o.m1, r2 = o.r2, r4 = r2 * r2;
    emit(0, fs * r2 * m0, fs * r2 * m1);
    emit(1, fs * r4 * m0, fs * r4 * m1);
    emit(2, fs * 2.0 * m0 * m1, fs * (r2 + 2.0 * m1 * m1));
    emit(3, fs * (r2 + 2.0 * m0 * m0), fs * 2.0 * m0 * m1);
    if (K == 5) emit(4, fs * r4 * r2 * m0, fs * r4 * r2 * m1);
  } else if constexpr (MODEL == kModelRpc) {
    double px[DEG + 1], py[DEG + 1];
    double vx = 1.0, vy = 1.0;
#pragma unroll
    for (int k = 0; k <= DEG; k++) {
      px[k] = vx; vx *= o.u0;
      py[k] = vy; vy *= o.u1;
    }
    const double iDx = o.aux0 * s, iDy = o.aux1 * s;
    const double mqx = -o.aux2 * iDx, mqy = -o.aux3 * iDy;  // -(N/D)/D
    int ci = 0;
#pragma unroll
    for (int cnt = 0; cnt < 4; cnt++) {
      const int start = (cnt & 1);
      const double sc = (cnt == 0) ? iDx : (cnt == 1) ? mqx : (cnt == 2) ? iDy : mqy;
#pragma unroll
      for (int dg = start; dg <= DEG; dg++) {
#pragma unroll
        for (int q = 0; q <= dg; q++) {
          const double v = sc * px[dg - q] * py[q];
          if (cnt < 2) emit(ci, v, 0.0);
          else emit(ci, 0.0, v);
          ci++;
        }
      }
    }
  }
  (void)f; (void)K; (void)o; (void)s;
}

__device__ __forceinline__ double loss_scale(double r0, double r1, int32_t flags, double cauchy_c,
                                             double* half_rho) {
  const double s = r0 * r0 + r1 * r1;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    // Ceres 1.14 CauchyLoss + Corrector [ext]: scale by sqrt(rho'), rho = b log(1 + s c).
    const double sum = 1.0 + s * cauchy_c;
    *half_rho = 0.5 * (log(sum) / cauchy_c);
    return sqrt(fmax(DBL_MIN, 1.0 / sum));
  }
  *half_rho = 0.5 * s;
  return 1.0;
}

// Per-frame record of the linearization (K2 expand), see mvba_kernels.hip.
struct FrameLin {
  int64_t slab_off;                  // reserved (0)
  int32_t chunk_count;               // solver chunks of this frame
  int32_t width, w16;                // Gram width and padded width
  int32_t first_chunk;               // global index of the frame's first chunk
  int64_t goff[8];                   // camera-side gradient offsets per block (-1: constant/none)
  int64_t hoff[8];                   // camera-side Hessian offsets per block
};

// Add v into camera-side entry dst: an fp64 atomic into the replica `rep`, or,
// in deterministic mode, a plain store into the producer's slab row (and, in
// the record pass, the destination of that slab position).
__device__ __forceinline__ void accumulate(double* rep, int64_t dst, double v, const Slab& s, int64_t unit,
                                           int local) {
  if (s.val) {
    const int64_t pos = (s.unit_base + unit) * s.width + local;
    s.val[pos] = v;
    if (s.dst) s.dst[pos] = (int32_t)dst;
  } else {
    atomicAdd(rep + dst, v);
  }
}

// Sum of val[pos[j]] for j in [b, e) over one wave, in a fixed order: lane l
// adds items l, l + 64, l + 128, ... in sequence, then a fixed butterfly. The
// loads of 8 consecutive items per lane are issued before their adds (a heavy
// entry, e.g. a sensor's intrinsics, has thousands of producers). Returns the
// total in every lane.
__device__ __forceinline__ double slab_entry_sum(int64_t b, int64_t e, const int64_t* __restrict__ pos,
                                                 const double* __restrict__ val) {
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  int64_t j = b + lane;
  for (; j + 7 * 64 < e; j += 8 * 64) {
    int64_t q[8];
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = pos[j + 64 * k];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = val[q[k]];
#pragma unroll
    for (int k = 0; k < 8; k++) acc += v[k];
  }
  for (; j < e; j += 64) acc += val[pos[j]];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  return acc;
}

// Last-block finalisation of a grid reduction: every block stores its partial,
// the last block to arrive sums them into out[0] and re-arms the counter.
// Sum of K values over the block (blockDim.x a multiple of 64, <= 1024):
// butterflies inside each wave, then the wave sums added in wave order, so the
// result is deterministic and every thread of the block gets it.
template <int K>
__device__ __forceinline__ void block_sum(double* v) {
  __shared__ double wsum[K][16];
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = wave_sum_f64(v[k]);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();  // wsum may still be read by a previous call
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; k++) wsum[k][w] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; k++) {
    double s = 0.0;
    for (int j = 0; j < nw; j++) s += wsum[k][j];
    v[k] = s;
  }
}

// Deterministic gather over a DetPlan (host: mvba_internal.h), three tiers by
// producer count so the grid stays small (its reduction counter is contended
// per arriving block): blocks [0, nheavy) take one heavy entry each (more than
// kSlabMedium producers: a sensor's extrinsics and intrinsics; 256 threads,
// lane-strided, fixed block reduction); the next nmed_blocks blocks take four
// medium entries, one wave each (slab_entry_sum); the rest take 256 light
// entries (at most kSlabLight producers, e.g. a reference pose), one thread
// each summing its producers in order. Returns true in the one thread holding
// entry *e's total in *acc. Control flow is block-uniform.
__device__ __forceinline__ bool slab_gather(const SlabTiers& t, const int64_t* __restrict__ begin,
                                            const int64_t* __restrict__ pos, const double* __restrict__ val,
                                            int64_t* e_out, double* acc_out) {
  const int64_t blk = blockIdx.x;
  if (blk < t.nheavy) {
    const int64_t e = t.heavy[blk];
    const int64_t b = begin[e], end = begin[e + 1];
    double acc = 0.0;
    int64_t j = b + threadIdx.x;
    for (; j + 3 * 256 < end; j += 4 * 256) {
      int64_t q[4];
      double v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = pos[j + 256 * k];
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = val[q[k]];
#pragma unroll
      for (int k = 0; k < 4; k++) acc += v[k];
    }
    for (; j < end; j += 256) acc += val[pos[j]];
    block_sum<1>(&acc);
    *e_out = e;
    *acc_out = acc;
    return threadIdx.x == 0;
  }
  const int64_t med_blocks = (t.nmedium + 3) / 4;
  if (blk < t.nheavy + med_blocks) {
    const int64_t k = (blk - t.nheavy) * 4 + (threadIdx.x >> 6);
    if (k >= t.nmedium) return false;
    const int64_t e = t.medium[k];
    *e_out = e;
    *acc_out = slab_entry_sum(begin[e], begin[e + 1], pos, val);
    return (threadIdx.x & 63) == 0;
  }
  const int64_t k = (blk - t.nheavy - med_blocks) * 256 + threadIdx.x;
  if (k >= t.nlight) return false;
  const int64_t e = t.light[k];
  const int64_t b = begin[e], n = begin[e + 1] - b;
  int64_t q[kSlabLight];
#pragma unroll
  for (int u = 0; u < kSlabLight; u++) q[u] = u < n ? pos[b + u] : -1;
  double acc = 0.0;
#pragma unroll
  for (int u = 0; u < kSlabLight; u++)
    if (u < n) acc += val[q[u]];
  *e_out = e;
  *acc_out = acc;
  return true;
}

// Cross-block hand-off of the reduction partials without __threadfence():
// on gfx950 an agent-scope fence is an L2 write-back plus an L2 invalidate
// (buffer_wbl2 sc1 / buffer_inv sc1) of the whole XCD, paid by every block.
// The partials are the only data handed over, so they are written and read as
// agent-scope relaxed atomics (sc1: at the coherence point), and the arrival
// on the counter waits for the partial store to complete (s_waitcnt) instead.
//
// ISA assumption (gfx950 only; this library is built for gfx950 alone): this is
// the first row of MI355X_MICROARCH.md's "hand-offs measured with sc1 loads in
// place of the acquire" table: ONE lane per workgroup stores its partials sc1,
// waits vmcnt(0) (stores are counted in vmcnt), then adds to ONE unsharded
// agent-scope counter; the workgroup whose add returned gridDim.x - 1 loads
// every partial with sc1 loads after a workgroup barrier. The C++ memory model
// gives no happens-before for relaxed atomics, so the waitcnt is an inline-asm
// statement with a memory clobber: a compiler barrier that keeps the partial
// store above it and the counter add below it (the builtin waitcnt is IntrNoMem
// and would not stop the compiler from reordering the two relaxed atomics).
__device__ __forceinline__ void partial_put(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double partial_get(double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// nb: the blocks that take part (the grid's first nb; 0 = the whole grid)
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned nb = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial stores above have completed
  const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // partial loads of the last block stay below the add
  return prev == (nb ? nb : gridDim.x) - 1;
}

__device__ __forceinline__ bool grid_sum_finalize(double v, double* __restrict__ partial,
                                                  unsigned* __restrict__ counter, double* __restrict__ out) {
  __shared__ bool last;
  block_sum<1>(&v);
  if (threadIdx.x == 0) {
    partial_put(&partial[blockIdx.x], v);
    last = arrive_last(counter);
  }
  __syncthreads();
  if (!last) return false;
  double acc = 0.0;
  for (unsigned e = threadIdx.x; e < gridDim.x; e += blockDim.x) acc += partial_get(&partial[e]);
  block_sum<1>(&acc);
  if (threadIdx.x == 0) {
    out[0] = acc;
    *counter = 0u;
  }
  return true;
}

// Three sums in one last-block finalisation (block partials interleaved as
// partial[3 b + k]); the last block also returns the sums in res[0..2].
// nb: blocks [0, nb) take part (0 = the whole grid); later blocks must not call it
__device__ __forceinline__ bool grid_sum3_finalize(double a, double b, double c, double* __restrict__ partial,
                                                   unsigned* __restrict__ counter, double* __restrict__ out,
                                                   double* res, unsigned nb = 0) {
  __shared__ bool last;
  double v[3] = {a, b, c};
  block_sum<3>(v);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; k++) partial_put(&partial[3 * blockIdx.x + k], v[k]);
    last = arrive_last(counter, nb);
  }
  __syncthreads();
  if (!last) return false;
  double acc[3] = {0.0, 0.0, 0.0};
  const unsigned nblk = nb ? nb : gridDim.x;
  for (unsigned e = threadIdx.x; e < nblk; e += blockDim.x)
    for (int k = 0; k < 3; k++) acc[k] += partial_get(&partial[3 * e + k]);
  block_sum<3>(acc);
  for (int k = 0; k < 3; k++) res[k] = acc[k];
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; k++) out[k] = acc[k];
    *counter = 0u;
  }
  return true;
}

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2v __attribute__((ext_vector_type(2)));

}  // namespace mvba

#endif  // MVBA_DEVICE_H_
