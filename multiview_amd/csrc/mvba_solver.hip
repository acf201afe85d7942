// mvba_solver.hip — gfx950 kernels of the GPU-resident Levenberg-Marquardt
// solver (replacing ceres::Solve with ITERATIVE_SCHUR, rig_calibrator.cc:1910-1919).
//
// The Schur complement S = U - W V^-1 W^T over the camera-side parameters is
// never formed: S x is applied matrix-free in two passes per CG iteration,
//   pass A (point order, 4 lanes/point): z_o = J_cam,o x  (via the frame's
//          generators: J_pose = Z w, so J_pose x = Z (w x)), t_p = sum J_pt^T z_o,
//          w_p = (V_p + D_p)^-1 t_p, u_o = z_o - J_pt w_p;
//   pass B (frame order, one wave per frame chunk): y_frame = sum Z^T u_o and
//          sum J_intr^T u_o, mapped through w to the pose columns in the same
//          kernel: S x = J_cam^T u (+ LM damping).
// Same two passes give the reduced right-hand side and the point back-substitution.
#include "mvba_depth.h"

namespace mvba {

// the CG passes' projection with reciprocals instead of the reference's
// divisions (project<..., FAST>, mvba_device.h); MVBA_FAST_PROJ=0 builds the
// divisions (A/B builds)
#ifndef MVBA_FAST_PROJ
#define MVBA_FAST_PROJ 1
#endif
constexpr bool kFastProj = MVBA_FAST_PROJ;

constexpr int kDirStride = 128;    // per-frame direction record: u (6) | x_intr (<= 122: RPC degree 6 has 113)
// pass-B vector replicas (chunk mod R): 32 since round 2 (8 contended then).
// Round 6 re-decided 16 vs 32 on timing alone, with the solver tests that once
// decided it re-grounded (each solve against the CPU LM; the 16-replica build
// passes the whole GPU suite, profiles/r06/r06i/pytest_gpu_r06i.log). Kernel
// traces, same box, two runs each (r06i/cg_iter_r06i.txt): c2 61.5 / 61.4 vs
// 62.3 / 61.8 us per CG iteration, c3 447.3 / 448.9 vs 450.9 / 445.5, the 1/8
// shard 27.7 / 28.8 vs 27.2 / 27.2 (its pass B 7.4-7.6 vs 6.8-6.9: 16 replicas
// contend on a thin shard's shared entries). 32 kept: the thin shard is the
// 8-GPU path. -DMVBA_VEC_REPLICAS=16 for A/B builds.
#ifndef MVBA_VEC_REPLICAS
#define MVBA_VEC_REPLICAS 32
#endif
constexpr int kVecReplicas = MVBA_VEC_REPLICAS;  // power of two

// Camera-side columns of one observation at a frame, as a row pair:
// Z (6), intrinsics (focal, center 2, live distortion nd), J_pt (3), corrected r.
template <int MODEL, int DEG>
// sr_given >= 0: the Cauchy weight K2 stored with the slot's landmark (the
// residual and the loss are not recomputed; r and half_rho are then not set).
__device__ __forceinline__ void obs_rows(const FrameDesc& F, const double* __restrict__ rec,
                                         const double* __restrict__ params, double X0, double X1,
                                         double X2, double2 meas, int32_t flags, double cauchy_c,
                                         double* Z0, double* Z1, double* I0, double* I1, double* P0,
                                         double* P1, double* r, double* half_rho, double sr_given = -1.0) {
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  Proj o;
  project<MODEL, DEG, kFastProj>(rec, X0, X1, X2, f, c0, c1, params + F.off[MVBA_BLK_DIST], F.K, F.h0, F.h1, o);
  double sr = sr_given;
  if (sr < 0.0) {
    const double r0 = o.d0 - meas.x, r1 = o.d1 - meas.y;
    sr = loss_scale(r0, r1, flags, cauchy_c, half_rho);
    r[0] = r0 * sr;
    r[1] = r1 * sr;
  }
  const double fz = fz_of<kFastProj>(f, o, sr);
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
  double a0[3], a1[3];
  cross(o.Xc, G0, a0);
  cross(o.Xc, G1, a1);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    Z0[q] = a0[q]; Z0[3 + q] = G0[q];
    Z1[q] = a1[q]; Z1[3 + q] = G1[q];
    P0[q] = G0[0] * rec[q] + G0[1] * rec[3 + q] + G0[2] * rec[6 + q];
    P1[q] = G1[0] * rec[q] + G1[1] * rec[3 + q] + G1[2] * rec[6 + q];
  }
  I0[0] = o.df0 * sr;
  I1[0] = o.df1 * sr;
  const double cc = (MODEL == kModelRpc) ? 0.0 : sr;
  I0[1] = cc; I0[2] = 0.0;
  I1[1] = 0.0; I1[2] = cc;
  dist_columns<MODEL, DEG>(o, f, F.K, sr, [&](int q, double v0, double v1) {
    I0[3 + q] = v0;
    I1[3 + q] = v1;
  });
}

// RPC monomials of the centred undistorted pixel in the coefficient order of
// compute_rpc (rpc_distortion.cc:116-160: degree dg, then q): m[k] = u0^(dg-q) u1^q.
// Every RPC distortion column is one of them times a per-row scale (the
// coefficients of num_x / den_x / num_y / den_y: iDx m_k, -(Nx/Dx)/Dx m_k, and
// the same for y, dist_columns), with the other row structurally zero: the CG
// passes fold the columns into dot products with the monomials instead of
// forming them (no multiply-adds of structural zeros).
template <int DEG>
struct RpcShape {
  static constexpr int kNl = (DEG + 1) * (DEG + 2) / 2;  // coefficients of a numerator
  // first distortion column of num_x, den_x (no constant), num_y, den_y
  static constexpr int kNx = 0, kDx = kNl, kNy = 2 * kNl - 1, kDy = 3 * kNl - 1;
};
template <int DEG>
__device__ __forceinline__ void rpc_monomials(double u0, double u1, double* m) {
  double px[DEG + 1], py[DEG + 1];
  double vx = 1.0, vy = 1.0;
#pragma unroll
  for (int k = 0; k <= DEG; k++) {
    px[k] = vx; vx *= u0;
    py[k] = vy; vy *= u1;
  }
  int k = 0;
#pragma unroll
  for (int dg = 0; dg <= DEG; dg++)
#pragma unroll
    for (int q = 0; q <= dg; q++) m[k++] = px[dg - q] * py[q];
}

template <int MODEL, int DEG>
struct RowShape {
  static constexpr int kDist = (MODEL == kModelNone) ? 0 : (MODEL == kModelFov) ? 1
                             : (MODEL == kModelRadtan) ? 5 : 2 * ((DEG + 1) * (DEG + 2)) - 2;
  static constexpr int kIntr = 3 + kDist;  // focal, center (2), live distortion
};

// ------------------------------------------------------------ per-frame direction
// dir_f = [ w_f x_pose (6) | x_focal | x_center (2) | x_dist (live) ]
// With lz.z set, x is the CG direction p_new = z (+ beta p_old) (LazyDir): the
// frame threads evaluate it where they read it and the trailing blocks
// (beyond the frame blocks) store it for the kernels that follow.
__device__ __forceinline__ double lazy_p(const LazyDir& lz, int32_t first, double beta, int64_t e) {
  return first ? lz.z[e] : __fma_rn(beta, lz.p_old[e], lz.z[e]);
}

// The first N entries of frame `frame`'s direction record into this wave's LDS
// area sd: d = dz, or inside CG iterations d = dz + beta dp (dp ignored on the
// first iteration, as lazy_p ignores p_old); the writer wave also stores d into
// dp_out for the next product. Wave-local: no block barrier.
template <int N>
__device__ __forceinline__ void stage_dir(const DirPair& D, int frame, double* sd, bool writer) {
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)frame * kDirStride;
  int32_t first = 1;
  double beta = 0.0;
  if (D.dp) {
    first = D.ctl->first;
    beta = D.ctl->beta;
  }
  const int nrec = D.z ? 6 : N;  // entries taken from the frame records
  if (D.frec) {
    // the 6 pose sums W_f z of the frame from z itself (frame_dir_body's
    // arithmetic): lane k < 22 takes pose column k, a butterfly over 32 lanes
    const FrameLin& L = ((const FrameLin*)D.fl)[frame];
    double u[6] = {0, 0, 0, 0, 0, 0};
    if (lane < kPoseCols) {
      const int blk = lane / 7;  // 0 beg, 1 end, 2 ref_to_cam, 3 offset (lane 21)
      const int64_t g = L.goff[(blk == 3) ? MVBA_BLK_OFFSET : blk];
      if (g >= 0) {
        const double zv = D.z[g + (lane - 7 * blk)];
        const double* wk = D.frec + (int64_t)frame * kFrameRecDoubles + 12 + 6 * lane;
#pragma unroll
        for (int a = 0; a < 6; a++) u[a] = wk[a] * zv;
      }
    }
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) u[a] += __shfl_xor(u[a], off, 64);
    if (lane < 6) {
      double v = u[0];
#pragma unroll
      for (int a = 1; a < 6; a++)
        if (lane == a) v = u[a];
      if (!first) v = __fma_rn(beta, D.dp[base + lane], v);
      sd[lane] = v;
      if (writer) D.dp_out[base + lane] = v;
    }
  } else {
    for (int m = lane; m < nrec; m += 64) {
      double v = D.dz[base + m];
      if (!first) v = __fma_rn(beta, D.dp[base + m], v);
      sd[m] = v;
      if (writer) D.dp_out[base + m] = v;
    }
  }
  if (D.z) {
    // intrinsic entries 0 focal, 1..2 centre, 3.. distortion: p_new's own
    // entries, lazy_p's arithmetic (zero for constant blocks and past K)
    const FrameLin& L = ((const FrameLin*)D.fl)[frame];
    const int nd = L.width - 10;  // live distortion entries
    for (int m = 6 + lane; m < N; m += 64) {
      const int q = m - 6;
      int64_t e = -1;
      if (q == 0) e = L.goff[MVBA_BLK_FOCAL];
      else if (q < 3) e = L.goff[MVBA_BLK_CENTER] >= 0 ? L.goff[MVBA_BLK_CENTER] + (q - 1) : -1;
      else if (q - 3 < nd) e = L.goff[MVBA_BLK_DIST] >= 0 ? L.goff[MVBA_BLK_DIST] + (q - 3) : -1;
      const double v = e < 0 ? 0.0 : first ? D.z[e] : __fma_rn(beta, D.p_old[e], D.z[e]);
      sd[m] = v;
      if (writer) D.dp_out[base + m] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One wave per frame: lane k < 22 takes pose column k (w_k x_k, butterfly-summed
// over the wave), lanes 22.. copy the intrinsic entries. X(b, j): entry j of the
// frame's camera block b (MVBA_BLK_*) of x; called only for floating blocks.
template <bool POSE_ONLY = false, class XF>
__device__ __forceinline__ void frame_dir_body(const FrameLin& L, int32_t K, const double* __restrict__ frec_f,
                                               int lane, XF X, double* __restrict__ d) {
  double u[6] = {0, 0, 0, 0, 0, 0};
  if (lane < kPoseCols) {
    const int blk = lane / 7;  // 0 beg, 1 end, 2 ref_to_cam, 3 offset (lane 21)
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    if (L.goff[b] >= 0) {
      const double xv = X(b, lane - 7 * blk);
      const double* wk = frec_f + 12 + 6 * lane;
#pragma unroll
      for (int a = 0; a < 6; a++) u[a] = wk[a] * xv;
    }
  }
#pragma unroll
  for (int a = 0; a < 6; a++)
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) u[a] += __shfl_xor(u[a], off, 64);  // lanes 0..31 hold all columns
  if (lane < 6) {
    double v = u[0];
#pragma unroll
    for (int a = 1; a < 6; a++)
      if (lane == a) v = u[a];
    d[lane] = v;
  }
  if constexpr (POSE_ONLY) return;
  // lanes 22.. copy the intrinsic entries: 0 focal, 1..2 centre, 3.. distortion
  const int nd = L.width - 10;
  for (int m = lane - kPoseCols; m >= 0 && m < 3 + nd; m += 64 - kPoseCols) {
    double v = 0.0;
    if (m == 0) {
      if (L.goff[MVBA_BLK_FOCAL] >= 0) v = X(MVBA_BLK_FOCAL, 0);
    } else if (m < 3) {
      if (L.goff[MVBA_BLK_CENTER] >= 0) v = X(MVBA_BLK_CENTER, m - 1);
    } else if (L.goff[MVBA_BLK_DIST] >= 0 && m - 3 < K) {
      v = X(MVBA_BLK_DIST, m - 3);
    }
    d[6 + m] = v;
  }
}

__global__ void __launch_bounds__(64) k_frame_dir(const FrameLin* __restrict__ fl, int32_t nframes,
                                                  const FrameDesc* __restrict__ fd,
                                                  const double* __restrict__ frec,
                                                  const double* __restrict__ x, double* __restrict__ dir,
                                                  const int32_t* __restrict__ gate, LazyDir lz) {
  if (gate && *gate) return;
  int32_t first = lz.first;
  double beta = lz.beta;
  if (lz.ctl) {
    first = lz.ctl->first;
    beta = lz.ctl->beta;
  }
  const int lane = threadIdx.x;
  if ((int32_t)blockIdx.x >= nframes) {
    const int64_t e = (int64_t)(blockIdx.x - nframes) * blockDim.x + lane;
    if (e < lz.n) lz.p_new[e] = lazy_p(lz, first, beta, e);
    return;
  }
  const int f = blockIdx.x;
  const FrameLin& L = fl[f];
  auto X = [&](int b, int j) {
    const int64_t e = L.goff[b] + j;
    return lz.z ? lazy_p(lz, first, beta, e) : x[e];
  };
  frame_dir_body(L, fd[f].K, frec + (int64_t)f * kFrameRecDoubles, lane, X, dir + (int64_t)f * kDirStride);
}

// ------------------------------------------------------------ pass A (point order)
// For each point: z_o = J_cam x (dir != null) for its observations, t = tinit +
// sum J_pt^T z_o, w = (V + diag(dp))^-1 t, u_o = z_o - J_pt w.
// store_u: write u_o (point order, 2 doubles); wout: w per point (3, nullable);
// sq_partial: per-block sum of |u_o|^2 (nullable); gdot_partial: per-block sum
// of g_p . w (nullable, with gp).
__device__ __forceinline__ void solve3(const double* V, const double* dp, const double* t, double* w) {
  // (V + diag(dp)) w = t, V packed xx xy xz yy yz zz; explicit inverse by cofactors
  const double a = V[0] + dp[0], b = V[1], c = V[2];
  const double d = V[3] + dp[1], e = V[4], f = V[5] + dp[2];
  const double A = d * f - e * e, B = c * e - b * f, C = b * e - c * d;
  const double det = a * A + b * B + c * C;
  if (!(fabs(det) > 0.0)) {
    w[0] = w[1] = w[2] = 0.0;
    return;
  }
  const double id = 1.0 / det;
  const double D = a * f - c * c, E = b * c - a * e, Fv = a * d - b * b;
  w[0] = (A * t[0] + B * t[1] + C * t[2]) * id;
  w[1] = (B * t[0] + D * t[1] + E * t[2]) * id;
  w[2] = (C * t[0] + E * t[1] + Fv * t[2]) * id;
}

// z_o = J_cam,o x and the point rows P = G R, with the camera-side columns
// folded into z as they are produced (never held as a row pair): the pose part
// (Xc x G_i).d + G_i.d' = G_i.(d x Xc + d'), then focal, centre and distortion
// columns times their direction entries. Keeps pass A's register footprint to
// the projection itself.
template <int MODEL, int DEG>
__device__ __forceinline__ void pass_a_obs(const double* __restrict__ rec, const double* dirf,
                                           double4 X, double2 m, int32_t flags, double cauchy_c,
                                           double* z, double* P0, double* P1, double sr_given = -1.0) {
  const double f = rec[12];
  const int K = (int)rec[17];
  Proj o;
  project<MODEL, DEG, kFastProj>(rec, X.x, X.y, X.z, f, rec[13], rec[14], rec + 18, K, rec[15], rec[16], o);
  double hr;
  const double sr = sr_given >= 0.0 ? sr_given : loss_scale(o.d0 - m.x, o.d1 - m.y, flags, cauchy_c, &hr);
  const double fz = fz_of<kFastProj>(f, o, sr);
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
#pragma unroll
  for (int q = 0; q < 3; q++) {
    P0[q] = G0[0] * rec[q] + G0[1] * rec[3 + q] + G0[2] * rec[6 + q];
    P1[q] = G1[0] * rec[q] + G1[1] * rec[3 + q] + G1[2] * rec[6 + q];
  }
  z[0] = z[1] = 0.0;
  if (!dirf) return;
  double v[3];
  cross(dirf, o.Xc, v);
#pragma unroll
  for (int q = 0; q < 3; q++) v[q] += dirf[3 + q];
  double z0 = G0[0] * v[0] + G0[1] * v[1] + G0[2] * v[2];
  double z1 = G1[0] * v[0] + G1[1] * v[1] + G1[2] * v[2];
  z0 += o.df0 * sr * dirf[6];
  z1 += o.df1 * sr * dirf[6];
  if constexpr (MODEL != kModelRpc) {  // centre columns (RPC: structurally zero)
    z0 += sr * dirf[7];
    z1 += sr * dirf[8];
  }
  // (the distortion columns one by one, structural zeros included: folding
  // them through the monomials as pass B does raised pass A from 74 to 100
  // VGPRs and its c3 time from 178 to 212 us, profiles/r04/r04o/)
  dist_columns<MODEL, DEG>(o, f, K, sr, [&](int q, double a0, double a1) {
    z0 += a0 * dirf[9 + q];
    z1 += a1 * dirf[9 + q];
  });
  z[0] = z0;
  z[1] = z1;
}

// pass_a_obs for two frame directions at once (the fused CG step: the z record
// and the previous direction's record), one projection: z1 = J_cam d1,
// z2 = J_cam d2 and the point rows.
template <int MODEL, int DEG>
__device__ __forceinline__ void pass_a_obs2(const double* __restrict__ rec, const double* d1, const double* d2,
                                            double4 X, double sr, double* z1, double* z2, double* P0, double* P1) {
  const double f = rec[12];
  const int K = (int)rec[17];
  Proj o;
  project<MODEL, DEG, kFastProj>(rec, X.x, X.y, X.z, f, rec[13], rec[14], rec + 18, K, rec[15], rec[16], o);
  const double fz = fz_of<kFastProj>(f, o, sr);
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
#pragma unroll
  for (int q = 0; q < 3; q++) {
    P0[q] = G0[0] * rec[q] + G0[1] * rec[3 + q] + G0[2] * rec[6 + q];
    P1[q] = G1[0] * rec[q] + G1[1] * rec[3 + q] + G1[2] * rec[6 + q];
  }
  double v[3], w[3];
  cross(d1, o.Xc, v);
  cross(d2, o.Xc, w);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    v[q] += d1[3 + q];
    w[q] += d2[3 + q];
  }
  double a0 = G0[0] * v[0] + G0[1] * v[1] + G0[2] * v[2];
  double a1 = G1[0] * v[0] + G1[1] * v[1] + G1[2] * v[2];
  double b0 = G0[0] * w[0] + G0[1] * w[1] + G0[2] * w[2];
  double b1 = G1[0] * w[0] + G1[1] * w[1] + G1[2] * w[2];
  const double fx = o.df0 * sr, fy = o.df1 * sr;
  a0 += fx * d1[6];
  a1 += fy * d1[6];
  b0 += fx * d2[6];
  b1 += fy * d2[6];
  if constexpr (MODEL != kModelRpc) {  // centre columns (RPC: structurally zero)
    a0 += sr * d1[7];
    a1 += sr * d1[8];
    b0 += sr * d2[7];
    b1 += sr * d2[8];
  }
  dist_columns<MODEL, DEG>(o, f, K, sr, [&](int q, double c0, double c1) {
    a0 += c0 * d1[9 + q];
    a1 += c1 * d1[9 + q];
    b0 += c0 * d2[9 + q];
    b1 += c1 * d2[9 + q];
  });
  z1[0] = a0;
  z1[1] = a1;
  z2[0] = b0;
  z2[1] = b1;
}

// kLanesA lanes per point; each lane keeps its first kCacheA observations' rows
// (z_o and the two J_pt rows: 8 doubles) in registers, later ones go through zbuf.
constexpr int kLanesA = 4;
constexpr int kCacheA = 3;

template <int MODEL, int DEG>
__device__ __forceinline__ void pass_a_dispatch(const double* __restrict__ rec, const double* dirf, double4 X,
                                                double2 m, int32_t flags, double cauchy_c, double* z, double* P0,
                                                double* P1) {
  if constexpr (MODEL >= 0) {
    pass_a_obs<MODEL, DEG>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
  } else {
    const int K = (int)rec[17];
    if (K == 0) pass_a_obs<kModelNone, 0>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 1) pass_a_obs<kModelFov, 0>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 4 || K == 5) pass_a_obs<kModelRadtan, 0>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 20) pass_a_obs<kModelRpc, 1>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 44) pass_a_obs<kModelRpc, 2>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 76) pass_a_obs<kModelRpc, 3>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 116) pass_a_obs<kModelRpc, 4>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else if (K == 164) pass_a_obs<kModelRpc, 5>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
    else pass_a_obs<kModelRpc, 6>(rec, dirf, X, m, flags, cauchy_c, z, P0, P1);
  }
}

// Projection records (kProjDoubles per frame) from the frame records and the
// current parameters; one thread per (frame, slot).
__global__ void __launch_bounds__(256) k_frame_proj(int32_t nframes, const FrameDesc* __restrict__ fd,
                                                    const double* __restrict__ frec,
                                                    const double* __restrict__ params, double* __restrict__ prec) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t f = t / kProjDoubles;
  const int q = (int)(t % kProjDoubles);
  if (f >= nframes) return;
  const FrameDesc& F = fd[f];
  double v = 0.0;
  if (q < 12) v = frec[f * kFrameRecDoubles + q];
  else if (q == 12) v = params[F.off[MVBA_BLK_FOCAL]];
  else if (q == 13) v = params[F.off[MVBA_BLK_CENTER]];
  else if (q == 14) v = params[F.off[MVBA_BLK_CENTER] + 1];
  else if (q == 15) v = F.h0;
  else if (q == 16) v = F.h1;
  else if (q == 17) v = (double)F.K;
  else if (q - 18 < F.K) v = params[F.off[MVBA_BLK_DIST] + (q - 18)];
  prec[t] = v;
}

// DEPTH: the problem has BracketedDepthError blocks (their code path is heavy;
// compiled out of the reprojection-only variant to keep its registers down).
// ROWS: a second sweep over the reprojection observations after w_p is known
// (|u_o|^2 for the back-substitution's model cost). Without it pass A only
// accumulates t_p and writes w_p (stride wstride); pass B recomputes u_o from
// the frame direction and w_p, so no per-observation row cache is kept.
template <int MODEL, int DEG, bool DEPTH, bool ROWS>
__global__ void __launch_bounds__(256) k_pass_a(
    const int64_t* __restrict__ pt_begin, int64_t npts, const int32_t* __restrict__ po_frame,
    const double2* __restrict__ po_meas, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const double* __restrict__ dir,
    const double* __restrict__ tinit, const double* __restrict__ V,
    const double* __restrict__ dp, double* __restrict__ zbuf, double* __restrict__ wout, int32_t wstride,
    double* __restrict__ sq_partial, unsigned* __restrict__ counter, double* __restrict__ sq_out,
    int32_t flags, double cauchy_c, PointExtra dc, const double* __restrict__ xcam, double* __restrict__ du,
    const int32_t* __restrict__ gate, const double* __restrict__ prec) {
  if (gate && *gate) return;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = t / kLanesA;
  const int sub = (int)(t % kLanesA);
  const bool valid = p < npts;
  double tv[3] = {0.0, 0.0, 0.0};
  double4 X = make_double4(0, 0, 0, 0);
  int64_t jb = 0, je = 0;
  double zc[kCacheA][8];  // ROWS only (dead otherwise)
  if (valid) {
    X = pts[p];
    jb = pt_begin[p];
    je = pt_begin[p + 1];
    int k = 0;
    for (int64_t j = jb + sub; j < je; j += kLanesA, k++) {
      const int32_t fr = po_frame[j];
      double z[2], P0[3], P1[3];
      pass_a_dispatch<MODEL, DEG>(prec + (int64_t)fr * kProjDoubles, dir ? dir + (int64_t)fr * kDirStride : nullptr,
                                  X, po_meas[j], flags, cauchy_c, z, P0, P1);
#pragma unroll
      for (int q = 0; q < 3; q++) tv[q] += P0[q] * z[0] + P1[q] * z[1];
      if constexpr (!ROWS) continue;
      const double row[8] = {z[0], z[1], P0[0], P0[1], P0[2], P1[0], P1[1], P1[2]};
      bool cached = false;
#pragma unroll
      for (int c = 0; c < kCacheA; c++)
        if (k == c) {
#pragma unroll
          for (int q = 0; q < 8; q++) zc[c][q] = row[q];
          cached = true;
        }
      if (!cached) {
        double* zr = zbuf + 8 * j;
#pragma unroll
        for (int q = 0; q < 8; q++) zr[q] = row[q];
      }
    }
  }
  const double4* dmeas = reinterpret_cast<const double4*>(dc.meas);
  int64_t db = 0, de = 0;
  double dP0 = 0.0;
  if (DEPTH && dc.begin && valid) {
    // BracketedDepthError blocks: z_d = J_cam,d x, t_p += P z_d (J_pt = P I);
    // z_d parked in du until w_p is known
    db = dc.begin[p];
    de = dc.begin[p + 1];
    for (int64_t j = db + sub; j < de; j += kLanesA) {
      const int32_t sl = dc.slot[j];
      const DepthDesc d = dc.dd[sl];
      const double4 m = dmeas[sl];
      DepthCore c;
      depth_core(d, frec + (int64_t)d.frame * kFrameRecDoubles, params, m, X.x, X.y, X.z, flags, cauchy_c, c);
      double z[3] = {0.0, 0.0, 0.0};
      if (dir) depth_jx(d, c, m, dir + (int64_t)d.frame * kDirStride, xcam, z);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        du[3 * (int64_t)sl + r] = z[r];
        if (X.w != 0.0) tv[r] += c.P * z[r];
      }
      if (j == db + sub) dP0 = c.P;  // first entry of this lane: keep P for the second loop
    }
  }
#pragma unroll
  for (int q = 0; q < 3; q++) tv[q] = group_sum_f64<kLanesA>(tv[q]);
  double w[3] = {0.0, 0.0, 0.0};
  double sq = 0.0;
  if (valid && X.w != 0.0) {
    if (tinit)
      for (int q = 0; q < 3; q++) tv[q] += tinit[3 * p + q];
    solve3(V + 6 * p, dp + 3 * p, tv, w);
  }
  if (valid && wout && sub == 0)
    for (int q = 0; q < 3; q++) wout[wstride * p + q] = w[q];
  if (ROWS && valid) {
    int k = 0;
    for (int64_t j = jb + sub; j < je; j += kLanesA, k++) {
      double row[8];
      bool cached = false;
#pragma unroll
      for (int c = 0; c < kCacheA; c++)
        if (k == c) {
#pragma unroll
          for (int q = 0; q < 8; q++) row[q] = zc[c][q];
          cached = true;
        }
      if (!cached) {
        const double* zr = zbuf + 8 * j;
#pragma unroll
        for (int q = 0; q < 8; q++) row[q] = zr[q];
      }
      const double u0 = row[0] - (row[2] * w[0] + row[3] * w[1] + row[4] * w[2]);
      const double u1 = row[1] - (row[5] * w[0] + row[6] * w[1] + row[7] * w[2]);
      sq += u0 * u0 + u1 * u1;
    }
  }
  if (DEPTH && valid && de > db) {
    // u_d = z_d - P w_p  (P = weight * sr depends only on the residual: recompute)
    for (int64_t j = db + sub; j < de; j += kLanesA) {
      const int32_t sl = dc.slot[j];
      double P = dP0;
      if (j != db + sub) {
        const DepthDesc d = dc.dd[sl];
        P = depth_p(d, frec + (int64_t)d.frame * kFrameRecDoubles, params, dmeas[sl], X.x, X.y, X.z, flags,
                    cauchy_c);
      }
#pragma unroll
      for (int r = 0; r < 3; r++) {
        const double u = du[3 * (int64_t)sl + r] - P * w[r];
        du[3 * (int64_t)sl + r] = u;
        sq += u * u;
      }
    }
  }
  if (sq_partial && valid && dc.xbegin && X.w != 0.0) {
    // XYZError priors: no camera columns, u = -P w_p
    const double4* xref = reinterpret_cast<const double4*>(dc.xref);
    for (int64_t j = dc.xbegin[p] + sub; j < dc.xbegin[p + 1]; j += kLanesA) {
      const double4 R = xref[j];
      double hr;
      const double sr = loss_scale3(R.w * (X.x - R.x), R.w * (X.y - R.y), R.w * (X.z - R.z), flags, dc.xcc[j], &hr);
      const double P = R.w * sr;
      sq += P * P * (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    }
  }
  if (sq_partial) grid_sum_finalize(sq, sq_partial, counter, sq_out);
}

// ------------------------------------------------------------ pass A, frame order
// The products of k_pass_a<..., DEPTH = false, ROWS = false> split in two:
// k_pass_a_frame sweeps the observations in frame order like pass B (one wave
// per frame chunk, so the frame's projection record and direction are scalar
// loads instead of per-lane gathers) and stores c_o = J_pt^T z_o per slot;
// k_point_w sums each point's c_o in point order, adds tinit and solves
// (V + D) w = t. Slot-order stores are coalesced; the point kernel gathers.
// One wave per chunk, kPassAWaves waves per block (the solver passes it one
// segment per chunk: nothing is reduced per frame here, and 4x the waves of
// the 4-segment chunks hide the point gathers better).
constexpr int kPassAWaves = 4;
#ifndef MVBA_PASSA_PIPE
#define MVBA_PASSA_PIPE 1  // pipelined slot-record loads (-DMVBA_PASSA_PIPE=0: the plain loop, A/B)
#endif
template <int MODEL, int DEG>
__global__ void __launch_bounds__(64 * kPassAWaves) k_pass_a_frame(
    const int4* __restrict__ chunks, int32_t nchunks, const Segment* __restrict__ segs,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid, const double2* __restrict__ obs_meas,
    const int32_t* __restrict__ slot_po, DirPair dr, double4* __restrict__ cbuf, int32_t flags,
    double cauchy_c,
    const int32_t* __restrict__ gate, const double* __restrict__ prec, const double4* __restrict__ obsX) {
  constexpr int ND = 6 + RowShape<MODEL, DEG>::kIntr;  // direction entries the rows read
  __shared__ double sdir[kPassAWaves][ND];
  const int lane = threadIdx.x & 63;
  const int64_t blk = xcd_block_solver((nchunks + kPassAWaves - 1) / kPassAWaves);
  const int ch = (int)blk * kPassAWaves + (threadIdx.x >> 6);
  if (blk < 0 || ch >= nchunks || (gate && *gate)) return;
  // (first slot, observations, frame, first chunk of the frame): the chunk's
  // segments are consecutive 64-slot runs of one frame, so no segment loads
  const int4 c = chunks[ch];
  const int frame = __builtin_amdgcn_readfirstlane(c.z);
  const int nobs = __builtin_amdgcn_readfirstlane(c.y);
  const double* __restrict__ rec = prec + (int64_t)frame * kProjDoubles;
  // the frame's direction (combined from dz and dp inside CG iterations); the
  // wave of the frame's first segment keeps it for the next product
  double* d = sdir[threadIdx.x >> 6];
  const bool writer = dr.dp_out && c.w;
  stage_dir<ND>(dr, frame, d, writer);
  if (obsX && MVBA_PASSA_PIPE && nobs > 64) {
    // chunks of several segments (c3): the next 64 slot records loaded before
    // this step's arithmetic (a software pipeline; c3 pass A 133 -> 127 us,
    // profiles/r05/r05v/). One-segment chunks (c2) keep the plain loop: the
    // pipelined form measured 1 us slower there (17.3 vs 16.3 us)
    double4 Xn = lane < nobs ? obsX[c.x + lane] : make_double4(0.0, 0.0, 0.0, 0.0);
    for (int s0 = 0; s0 < nobs; s0 += 64) {
      const double4 X = Xn;
      if (s0 + 64 < nobs && lane < nobs - s0 - 64) Xn = obsX[(int64_t)c.x + s0 + 64 + lane];
      if (lane < nobs - s0) {
        const int64_t i = (int64_t)c.x + s0 + lane;
        double z[2], P0[3], P1[3];
        pass_a_obs<MODEL, DEG>(rec, d, X, double2{0.0, 0.0}, flags, cauchy_c, z, P0, P1, X.w);
        cbuf[slot_po ? (int64_t)slot_po[i] : i] = make_double4(P0[0] * z[0] + P1[0] * z[1],
                                                               P0[1] * z[0] + P1[1] * z[1],
                                                               P0[2] * z[0] + P1[2] * z[1], 0.0);
      }
    }
    return;
  }
  for (int s0 = 0; s0 < nobs; s0 += 64) {
    if (lane < nobs - s0) {
      const int64_t i = (int64_t)c.x + s0 + lane;
      double z[2], P0[3], P1[3];
      // obsX (K2's per-slot record): landmark + Cauchy weight, no measurement read
      if (obsX)
        pass_a_obs<MODEL, DEG>(rec, d, obsX[i], double2{0.0, 0.0}, flags, cauchy_c, z, P0, P1, obsX[i].w);
      else
        pass_a_obs<MODEL, DEG>(rec, d, pts[obs_pid[i]], obs_meas[i], flags, cauchy_c, z, P0, P1);
      // plain store: a nontemporal store of these scattered 32-B records
      // doubles the kernel (49 vs 24 us at c2, partial lines go to HBM);
      // slot_po null: stored in slot order (coalesced), k_point_w gathers
      cbuf[slot_po ? (int64_t)slot_po[i] : i] = make_double4(P0[0] * z[0] + P1[0] * z[1], P0[1] * z[0] + P1[1] * z[1],
                                      P0[2] * z[0] + P1[2] * z[1], 0.0);
    }
  }
}

// |J delta|^2 of the back-substitution in frame order (reprojection-only,
// one model group): per observation u_o = z_o - J_pt w_p with z_o = J_cam,o
// delta_c from the frame direction (dr.dz) and w_p from k_point_w (wbuf,
// wstride doubles per point), summed over the grid into sq_out. Replaces the
// point-order k_pass_a<..., ROWS> (4 lanes per point gathering per-frame data)
// after the frame-order pass A + k_point_w.
template <int MODEL, int DEG>
__global__ void __launch_bounds__(64 * kPassAWaves) k_pass_sq(
    const int4* __restrict__ chunks, int32_t nchunks, const int32_t* __restrict__ obs_pid, DirPair dr,
    const double* __restrict__ wbuf, int32_t wstride, const double* __restrict__ prec,
    const double4* __restrict__ obsX, double* __restrict__ partial, unsigned* __restrict__ counter,
    double* __restrict__ sq_out) {
  constexpr int ND = 6 + RowShape<MODEL, DEG>::kIntr;
  __shared__ double sdir[kPassAWaves][ND];
  const int lane = threadIdx.x & 63;
  double sq = 0.0;
  // a bounded grid (1,024 blocks), each wave striding over the chunks: the
  // grid sum's arrival counter takes one atomic per block (39k blocks at c3
  // serialised on it: 534 us; 256 / 512 / 1024 / 2048 blocks: 373 / 225 / 191 /
  // 200 us at c3, 36.8 / 26.2 / 26.7 / 37.2 us at c2). With MVBA_XCD_SOLVER
  // (the grid a multiple of 8) the blocks of XCD x stride over the x-th eighth
  // of the chunks.
  int ch0 = blockIdx.x * kPassAWaves + (threadIdx.x >> 6), cend = nchunks, cstep = gridDim.x * kPassAWaves;
  if (MVBA_XCD_SOLVER) {
    const int per = (nchunks + kXcds - 1) / kXcds, x = (int)(blockIdx.x % kXcds);
    ch0 = x * per + (int)(blockIdx.x / kXcds) * kPassAWaves + (threadIdx.x >> 6);
    cend = min(nchunks, (x + 1) * per);
    cstep = (int)(gridDim.x / kXcds) * kPassAWaves;
  }
  for (int ch = ch0; ch < cend; ch += cstep) {
    const int4 c = chunks[ch];
    const int frame = __builtin_amdgcn_readfirstlane(c.z);
    const int nobs = __builtin_amdgcn_readfirstlane(c.y);
    const double* __restrict__ rec = prec + (int64_t)frame * kProjDoubles;
    double* d = sdir[threadIdx.x >> 6];
    stage_dir<ND>(dr, frame, d, false);
    for (int s0 = 0; s0 < nobs; s0 += 64) {
      if (lane < nobs - s0) {
        const int64_t i = (int64_t)c.x + s0 + lane;
        const double* w = wbuf + (int64_t)wstride * obs_pid[i];
        const double w0 = w[0], w1 = w[1], w2 = w[2];
        const double4 X = obsX[i];
        double z[2], P0[3], P1[3];
        pass_a_obs<MODEL, DEG>(rec, d, X, double2{0.0, 0.0}, 0, 0.0, z, P0, P1, X.w);
        const double u0 = z[0] - (P0[0] * w0 + P0[1] * w1 + P0[2] * w2);
        const double u1 = z[1] - (P1[0] * w0 + P1[1] * w1 + P1[2] * w2);
        sq += u0 * u0 + u1 * u1;
      }
    }
    __builtin_amdgcn_wave_barrier();  // sdir is rewritten by the next chunk of this wave
  }
  grid_sum_finalize(sq, partial, counter, sq_out);
}

// BracketedDepthError / BracketedDepthMeshError blocks in the frame-order CG
// product: one wave per depth segment (one image: the descriptor is read once,
// the point per lane), z_d = J_cam,d x into du (slot order; k_depth_sb forms
// u_d = z_d - P w_p once w is known) and c_d = P z_d at the block's point-order
// position for k_point_w. Replaces the point-order k_pass_a (4 lanes per point
// gathering per-frame data) inside CG iterations.
__global__ void __launch_bounds__(64) k_depth_pa(const Segment* __restrict__ segs, int32_t nseg,
                                                 const DepthDesc* __restrict__ dd, const int32_t* __restrict__ dpid,
                                                 const double4* __restrict__ dmeas, const double* __restrict__ frec,
                                                 const double* __restrict__ params, const double4* __restrict__ pts,
                                                 const double* __restrict__ dir, const double* __restrict__ xcam,
                                                 double* __restrict__ du, const int32_t* __restrict__ dslot_po,
                                                 double4* __restrict__ dcbuf, int32_t flags, double cauchy_c,
                                                 const int32_t* __restrict__ gate) {
  if (gate && *gate) return;
  const int seg = blockIdx.x;
  if (seg >= nseg) return;
  const Segment sg = segs[seg];
  const int lane = threadIdx.x;
  const int count = __builtin_amdgcn_readfirstlane(sg.count);
  const int begin = __builtin_amdgcn_readfirstlane(sg.begin);
  if (lane >= count) return;
  const int64_t i = (int64_t)begin + lane;
  DepthDesc d = dd[begin];
  d.pid = dpid[i];
  const double4 X = pts[d.pid];
  const double4 m = dmeas[i];
  DepthCore c;
  depth_core(d, frec + (int64_t)d.frame * kFrameRecDoubles, params, m, X.x, X.y, X.z, flags, cauchy_c, c);
  double z[3];
  depth_jx(d, c, m, dir + (int64_t)d.frame * kDirStride, xcam, z);
#pragma unroll
  for (int q = 0; q < 3; q++) du[3 * i + q] = z[q];
  dcbuf[dslot_po[i]] = make_double4(c.P * z[0], c.P * z[1], c.P * z[2], 0.0);
}

// w_p = (V + D)^-1 (tinit + sum_o c_o), kLanesW lanes per point gathering its
// c_o (lane-strided, then a butterfly sum); cbuf null: x = 0
#ifndef MVBA_LANES_W
#define MVBA_LANES_W 8
#endif
constexpr int kLanesW = MVBA_LANES_W;
__global__ void __launch_bounds__(256) k_point_w(int64_t npts, const int64_t* __restrict__ pt_begin,
                                                 const int32_t* __restrict__ po_slot, const double4* __restrict__ cbuf,
                                                 const double* __restrict__ tinit, const double* __restrict__ V,
                                                 const double* __restrict__ dp, const double4* __restrict__ pts,
                                                 double* __restrict__ wout, int32_t wstride,
                                                 const int32_t* __restrict__ gate, const int64_t* __restrict__ dbegin,
                                                 const double4* __restrict__ dcbuf, FusedStep fs) {
  if (gate && *gate) return;
  if (fs.dz && (int32_t)blockIdx.x >= fs.point_blocks) {
    // fused CG step: the frame direction d = d_z + beta d_p of this iteration
    // (pass B's records and the next step's d_p), one wave per frame
    const int f = ((int32_t)blockIdx.x - fs.point_blocks) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
    if (f >= fs.nframes) return;
    const int64_t base = (int64_t)f * kDirStride;
    const int nrec = min(9 + fs.fd[f].K, kDirStride);
    const double beta = fs.ctl->beta;
    for (int m = (int)(threadIdx.x & 63); m < nrec; m += 64) fs.dp_out[base + m] = __fma_rn(beta, fs.dp[base + m], fs.dz[base + m]);
    return;
  }
  const int64_t blk = xcd_block_solver((npts * kLanesW + 255) / 256);
  if (blk < 0) return;
  const int64_t t0 = blk * 256 + threadIdx.x;
  const int64_t p = t0 / kLanesW;
  const int sub = (int)(t0 % kLanesW);
  const bool valid = p < npts;
  // the solving lane's point data (free flag, right-hand side, V, damping)
  // loaded before the c_o gathers, so the gathers are its only dependent
  // round trip
  const bool solver = valid && sub == 0;
  double Vp[6], dpp[3], ti[3] = {0.0, 0.0, 0.0};
  double freep = 0.0;
  if (solver) {
    freep = pts[p].w;
#pragma unroll
    for (int q = 0; q < 6; q++) Vp[q] = V[6 * p + q];
#pragma unroll
    for (int q = 0; q < 3; q++) dpp[q] = dp[3 * p + q];
    if (tinit)
#pragma unroll
      for (int q = 0; q < 3; q++) ti[q] = tinit[3 * p + q];
  }
  double t[3] = {0.0, 0.0, 0.0};
  if (valid && cbuf && fs.cbuf2) {
    // fused CG step: t = sum c_z + beta sum c_p (pass A could not know beta)
    double tp[3] = {0.0, 0.0, 0.0};
    const double2* __restrict__ c2 = (const double2*)fs.cbuf2;
    for (int64_t j = pt_begin[p] + sub; j < pt_begin[p + 1]; j += kLanesW) {
      const int64_t o = po_slot ? (int64_t)po_slot[j] : j;
      const double4 cv = cbuf[o];
      const double2 cw = c2[o];
      t[0] += cv.x;
      t[1] += cv.y;
      t[2] += cv.z;
      tp[0] += cv.w;
      tp[1] += cw.x;
      tp[2] += cw.y;
    }
    const double beta = fs.ctl->beta;
#pragma unroll
    for (int q = 0; q < 3; q++) t[q] = __fma_rn(beta, tp[q], t[q]);
  } else if (valid && cbuf)
    for (int64_t j = pt_begin[p] + sub; j < pt_begin[p + 1]; j += kLanesW) {
      // po_slot set: pass A stored c_o in slot order; gather it
      const double4 cv = po_slot ? cbuf[po_slot[j]] : cbuf[j];
      t[0] += cv.x;
      t[1] += cv.y;
      t[2] += cv.z;
    }
  if (valid && dcbuf)  // depth blocks of the point (k_depth_pa), point order
    for (int64_t j = dbegin[p] + sub; j < dbegin[p + 1]; j += kLanesW) {
      const double4 cv = dcbuf[j];
      t[0] += cv.x;
      t[1] += cv.y;
      t[2] += cv.z;
    }
#pragma unroll
  for (int q = 0; q < 3; q++) t[q] = group_sum_f64<kLanesW>(t[q]);
  if (!solver) return;
  double w[3] = {0.0, 0.0, 0.0};
  if (freep != 0.0) {
    if (tinit)
#pragma unroll
      for (int q = 0; q < 3; q++) t[q] += ti[q];
    solve3(Vp, dpp, t, w);
  }
#pragma unroll
  for (int q = 0; q < 3; q++) wout[wstride * p + q] = w[q];
}

// k_point_w as wave tiles of whole tracks (reprojection-only problems): lane l
// of a tile takes one residual of a point (wlane_pid / wlane_idx: the c_o index
// of that residual, -1 for a point without any), so a lane's chain is one round
// trip to its point and c_o index, one to c_o; the point's lanes are consecutive
// and a segmented scan (shuffles, pid equality at each distance) leaves the
// track's sum in its last lane, which loaded the point's V, damping and right-
// hand side alongside the gather and solves. Tracks longer than a wave have a
// tile of their own (lane-strided loop over po_idx, wave sum).
__global__ void __launch_bounds__(256) k_point_w_seg(int32_t ntiles, const int4* __restrict__ tiles,
                                                     const int32_t* __restrict__ wlane_pid,
                                                     const int32_t* __restrict__ wlane_idx,
                                                     const int64_t* __restrict__ pt_begin,
                                                     const int32_t* __restrict__ po_idx,
                                                     const double4* __restrict__ cbuf, const double* __restrict__ tinit,
                                                     const double* __restrict__ V, const double* __restrict__ dp,
                                                     const double4* __restrict__ pts, double* __restrict__ wout,
                                                     int32_t wstride, const int32_t* __restrict__ gate) {
  if (gate && *gate) return;
  const int64_t blk = xcd_block_solver((ntiles + 3) / 4);
  const int tile = (int)blk * 4 + (int)(threadIdx.x >> 6);
  if (blk < 0 || tile >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const int4 T = tiles[tile];
  const int first = __builtin_amdgcn_readfirstlane(T.x);
  const int count = __builtin_amdgcn_readfirstlane(T.y);
  const int lp = __builtin_amdgcn_readfirstlane(T.z);
  auto solve_store = [&](int64_t p, double t0, double t1, double t2) {
    double t[3] = {t0, t1, t2}, w[3] = {0.0, 0.0, 0.0};
    if (pts[p].w != 0.0) {
      if (tinit)
#pragma unroll
        for (int q = 0; q < 3; q++) t[q] += tinit[3 * p + q];
      solve3(V + 6 * p, dp + 3 * p, t, w);
    }
#pragma unroll
    for (int q = 0; q < 3; q++) wout[wstride * p + q] = w[q];
  };
  if (lp >= 0) {  // one long track
    double t[3] = {0.0, 0.0, 0.0};
    for (int64_t j = pt_begin[lp] + lane; j < pt_begin[lp + 1]; j += 64) {
      const double4 cv = cbuf[po_idx ? po_idx[j] : j];
      t[0] += cv.x;
      t[1] += cv.y;
      t[2] += cv.z;
    }
#pragma unroll
    for (int q = 0; q < 3; q++) t[q] = wave_sum_f64(t[q]);
    if (lane == 0) solve_store(lp, t[0], t[1], t[2]);
    return;
  }
  const bool act = lane < count;
  const int32_t pid = act ? wlane_pid[first + lane] : -1 - lane;
  const int32_t idx = act ? wlane_idx[first + lane] : -1;
  const int32_t pid_next = __shfl(pid, lane + 1 < 64 ? lane + 1 : lane, 64);
  const bool last = act && (lane == count - 1 || pid_next != pid);
  // the solving lane's point data, issued beside the gather
  double Vp[6] = {0, 0, 0, 0, 0, 0}, dpp[3] = {0, 0, 0}, ti[3] = {0, 0, 0};
  double freep = 0.0;
  if (last) {
    freep = pts[pid].w;
#pragma unroll
    for (int q = 0; q < 6; q++) Vp[q] = V[6 * (int64_t)pid + q];
#pragma unroll
    for (int q = 0; q < 3; q++) dpp[q] = dp[3 * (int64_t)pid + q];
    if (tinit)
#pragma unroll
      for (int q = 0; q < 3; q++) ti[q] = tinit[3 * (int64_t)pid + q];
  }
  double4 c = make_double4(0.0, 0.0, 0.0, 0.0);
  if (idx >= 0) c = cbuf[idx];
  double t0 = c.x, t1 = c.y, t2 = c.z;
  // segmented inclusive scan over the track's consecutive lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int src = lane >= off ? lane - off : lane;
    const double u0 = __shfl(t0, src, 64), u1 = __shfl(t1, src, 64), u2 = __shfl(t2, src, 64);
    const int32_t pu = __shfl(pid, src, 64);
    if (lane >= off && pu == pid) {
      t0 += u0;
      t1 += u1;
      t2 += u2;
    }
  }
  if (!last) return;
  double t[3] = {t0, t1, t2}, w[3] = {0.0, 0.0, 0.0};
  if (freep != 0.0) {
#pragma unroll
    for (int q = 0; q < 3; q++) t[q] += ti[q];
    solve3(Vp, dpp, t, w);
  }
#pragma unroll
  for (int q = 0; q < 3; q++) wout[wstride * (int64_t)pid + q] = w[q];
}

// ------------------------------------------------------------ pass B, wide rows
// Wide intrinsic blocks (RPC degree >= 4: up to 113 intrinsic columns) do not
// fit per-lane accumulators: the lanes of one half-segment write their row pair
// [Z | I] and u_o straight into LDS ([column][row], as the Gram staging of K2),
// then every lane reduces its columns (lane, lane + 64) over the 64 rows.
constexpr int kPassBRegCols = 48;  // register accumulators up to this many columns
// pass B's end-of-chunk reduction: transposed wave sums (wave_sum_transpose)
// or one full wave_sum_f64 per accumulator (MVBA_PASSB_TRED=0, A/B builds)
#ifndef MVBA_PASSB_TRED
#define MVBA_PASSB_TRED 1
#endif
#ifndef MVBA_RPC_PB_WAVES
#define MVBA_RPC_PB_WAVES 1  // min waves per EU of RPC (degree <= 2) pass B (launch bounds; A/B builds)
#endif
#ifndef MVBA_PASSB_PIPE
#define MVBA_PASSB_PIPE 1  // RPC pass B: software-pipelined gathers (-DMVBA_PASSB_PIPE=0: the plain loop, A/B)
#endif
constexpr int kWideLd = 66;

template <int MODEL, int DEG>
constexpr size_t pass_b_lds() {
  constexpr int NA = 6 + RowShape<MODEL, DEG>::kIntr;
  return NA > kPassBRegCols ? sizeof(double) * (size_t)(NA + 1) * kWideLd : 0;
}

template <int MODEL, int DEG>
__device__ __forceinline__ void pass_b_wide(int4 c, int32_t chunk_id, const Segment* __restrict__ segs,
                                            const FrameDesc* __restrict__ fd, const FrameLin* __restrict__ fl,
                                            const double* __restrict__ frec, const double* __restrict__ params,
                                            const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
                                            const double2* __restrict__ obs_meas, const double* __restrict__ dir,
                                            const double4* __restrict__ wbuf, double* __restrict__ yrep, int64_t ng,
                                            int32_t flags, double cauchy_c, const Slab& sl,
                                            const double4* __restrict__ obsX) {
  using RS = RowShape<MODEL, DEG>;
  constexpr int NA = 6 + RS::kIntr;
  extern __shared__ double st[];  // [NA + 1][kWideLd]: columns, then u
  const int lane = threadIdx.x;
  const int frame = __builtin_amdgcn_readfirstlane(c.z);
  const FrameDesc& F = fd[frame];
  const double* __restrict__ rec = frec + (int64_t)frame * kFrameRecDoubles;
  const double* __restrict__ d = dir ? dir + (int64_t)frame * kDirStride : nullptr;
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  double acc0 = 0.0, acc1 = 0.0;  // columns lane, lane + 64
  const int nobs = __builtin_amdgcn_readfirstlane(c.y);
  for (int s0 = 0; s0 < nobs; s0 += 64) {
    const int count = min(64, nobs - s0);
    for (int half = 0; half < 2 && 32 * half < count; half++) {
      if ((lane >> 5) == half) {
        const int slot = 2 * (lane & 31);
        if (lane < count) {
          const int64_t i = (int64_t)c.x + s0 + lane;
          const int32_t pid = obs_pid[i];
          const double4 w = wbuf[pid];
          const double4 X = obsX ? obsX[i] : pts[pid];
          Proj o;
          project<MODEL, DEG, kFastProj>(rec, X.x, X.y, X.z, f, c0, c1, params + F.off[MVBA_BLK_DIST], F.K, F.h0, F.h1,
                                    o);
          double hr;
          double sr;
          if (obsX) {
            sr = X.w;  // K2's Cauchy weight
          } else {
            const double2 m = obs_meas[i];
            sr = loss_scale(o.d0 - m.x, o.d1 - m.y, flags, cauchy_c, &hr);
          }
          const double fz = fz_of<kFastProj>(f, o, sr);
          const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
          const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
          double a0[3], a1[3];
          cross(o.Xc, G0, a0);
          cross(o.Xc, G1, a1);
          double z0 = 0.0, z1 = 0.0;
          auto put = [&](int q, double v0, double v1) {
            *(dbl2v*)&st[q * kWideLd + slot] = dbl2v{v0, v1};
            if (d) {
              z0 += v0 * d[q];
              z1 += v1 * d[q];
            }
          };
#pragma unroll
          for (int q = 0; q < 3; q++) {
            put(q, a0[q], a1[q]);
            put(3 + q, G0[q], G1[q]);
          }
          put(6, o.df0 * sr, o.df1 * sr);
          const double cc = (MODEL == kModelRpc) ? 0.0 : sr;
          put(7, cc, 0.0);
          put(8, 0.0, cc);
          dist_columns<MODEL, DEG>(o, f, F.K, sr, [&](int q, double v0, double v1) { put(9 + q, v0, v1); });
          double P0[3], P1[3];
#pragma unroll
          for (int q = 0; q < 3; q++) {
            P0[q] = G0[0] * rec[q] + G0[1] * rec[3 + q] + G0[2] * rec[6 + q];
            P1[q] = G1[0] * rec[q] + G1[1] * rec[3 + q] + G1[2] * rec[6 + q];
          }
          const double ux = z0 - (P0[0] * w.x + P0[1] * w.y + P0[2] * w.z);
          const double uy = z1 - (P1[0] * w.x + P1[1] * w.y + P1[2] * w.z);
          *(dbl2v*)&st[NA * kWideLd + slot] = dbl2v{ux, uy};
        } else {
          for (int q = 0; q <= NA; q++) *(dbl2v*)&st[q * kWideLd + slot] = dbl2v{0.0, 0.0};
        }
      }
      __syncthreads();  // one wave per block: a wave barrier with the LDS drained
#pragma unroll 4
      for (int r = 0; r < 64; r++) {
        const double u = st[NA * kWideLd + r];
        if (lane < NA) acc0 += st[lane * kWideLd + r] * u;
        if (lane + 64 < NA) acc1 += st[(lane + 64) * kWideLd + r] * u;
      }
      __syncthreads();
    }
  }
  // Z^T u (columns 0..5, lanes 0..5) to every lane; pose columns through w_k
  double zs[6];
#pragma unroll
  for (int a = 0; a < 6; a++) zs[a] = __shfl(acc0, a, 64);
  const FrameLin& L = fl[frame];
  double* y = yrep + (int64_t)(chunk_id & (kVecReplicas - 1)) * ng;
  if (lane < kPoseCols) {
    const int blk = lane / 7;  // 0 beg, 1 end, 2 ref_to_cam, 3 offset (lane 21)
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    if (L.goff[b] >= 0) {
      const double* wk = rec + 12 + 6 * lane;
      double v = 0.0;
#pragma unroll
      for (int a = 0; a < 6; a++) v += wk[a] * zs[a];
      accumulate(y, L.goff[b] + (lane - 7 * blk), v, sl, chunk_id, lane);
    }
  }
  // intrinsic entries: column 6 + q held by lane (6 + q) mod 64
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int col = lane + 64 * h;
    const int q = col - 6;  // 0 focal, 1..2 center, 3.. distortion
    if (q < 0 || col >= NA) continue;
    int64_t dst = -1;
    if (q == 0) dst = L.goff[MVBA_BLK_FOCAL];
    else if (q < 3) dst = L.goff[MVBA_BLK_CENTER] >= 0 ? L.goff[MVBA_BLK_CENTER] + (q - 1) : -1;
    else if (q - 3 < F.K) dst = L.goff[MVBA_BLK_DIST] >= 0 ? L.goff[MVBA_BLK_DIST] + (q - 3) : -1;
    if (dst >= 0) accumulate(y, dst, h == 0 ? acc0 : acc1, sl, chunk_id, kPoseCols + q);
  }
}

// Pass B's per-observation work for RPC (degree <= 3, register accumulators):
// obs_rows + the loop of k_pass_b with the distortion columns folded through
// the monomials (RpcShape): z takes the four monomial dot products with the
// direction's num / den entries, each accumulator of a distortion column gets
// (row scale * u) * monomial, and the structurally zero rows (the other
// coordinate's half, the centre columns) cost nothing.
template <int DEG>
__device__ __forceinline__ void pass_b_rpc_obs(const FrameDesc& F, const double* __restrict__ rec,
                                               const double* __restrict__ params, double4 X, double2 m,
                                               int32_t flags, double cauchy_c, double sr_given,
                                               const double* __restrict__ d, double4 w, double* acc) {
  using RS = RpcShape<DEG>;
  const double f = params[F.off[MVBA_BLK_FOCAL]];
  const double c0 = params[F.off[MVBA_BLK_CENTER]];
  const double c1 = params[F.off[MVBA_BLK_CENTER] + 1];
  Proj o;
  project<kModelRpc, DEG, kFastProj>(rec, X.x, X.y, X.z, f, c0, c1, params + F.off[MVBA_BLK_DIST], F.K, F.h0, F.h1, o);
  double sr = sr_given;
  if (sr < 0.0) {
    double hr;
    sr = loss_scale(o.d0 - m.x, o.d1 - m.y, flags, cauchy_c, &hr);
  }
  const double fz = fz_of<kFastProj>(f, o, sr);
  const double G0[3] = {fz * o.A00, fz * o.A01, -fz * (o.A00 * o.nx + o.A01 * o.ny)};
  const double G1[3] = {fz * o.A10, fz * o.A11, -fz * (o.A10 * o.nx + o.A11 * o.ny)};
  double a0[3], a1[3];
  cross(o.Xc, G0, a0);
  cross(o.Xc, G1, a1);
  double mono[RS::kNl];
  rpc_monomials<DEG>(o.u0, o.u1, mono);
  const double iDx = o.aux0 * sr, iDy = o.aux1 * sr;
  const double mqx = -o.aux2 * iDx, mqy = -o.aux3 * iDy;
  const double fx = o.df0 * sr, fy = o.df1 * sr;
  double z0 = 0.0, z1 = 0.0;
  if (d) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
      z0 += a0[a] * d[a];
      z1 += a1[a] * d[a];
    }
#pragma unroll
    for (int a = 0; a < 3; a++) {
      z0 += G0[a] * d[3 + a];
      z1 += G1[a] * d[3 + a];
    }
    z0 += fx * d[6];
    z1 += fy * d[6];
    const double* dd = d + 9;
    double snx = mono[0] * dd[RS::kNx], sny = mono[0] * dd[RS::kNy], sdx = 0.0, sdy = 0.0;
#pragma unroll
    for (int k = 1; k < RS::kNl; k++) {
      snx += mono[k] * dd[RS::kNx + k];
      sdx += mono[k] * dd[RS::kDx + k - 1];
      sny += mono[k] * dd[RS::kNy + k];
      sdy += mono[k] * dd[RS::kDy + k - 1];
    }
    z0 += iDx * snx + mqx * sdx;
    z1 += iDy * sny + mqy * sdy;
  }
  double P0[3], P1[3];
#pragma unroll
  for (int q = 0; q < 3; q++) {
    P0[q] = G0[0] * rec[q] + G0[1] * rec[3 + q] + G0[2] * rec[6 + q];
    P1[q] = G1[0] * rec[q] + G1[1] * rec[3 + q] + G1[2] * rec[6 + q];
  }
  const double ux = z0 - (P0[0] * w.x + P0[1] * w.y + P0[2] * w.z);
  const double uy = z1 - (P1[0] * w.x + P1[1] * w.y + P1[2] * w.z);
#pragma unroll
  for (int a = 0; a < 3; a++) {
    acc[a] += a0[a] * ux + a1[a] * uy;
    acc[3 + a] += G0[a] * ux + G1[a] * uy;
  }
  acc[6] += fx * ux + fy * uy;  // focal; the centre columns (7, 8) are zero for RPC
  const double ax = iDx * ux, bx = mqx * ux, ay = iDy * uy, by = mqy * uy;
#pragma unroll
  for (int k = 0; k < RS::kNl; k++) {
    acc[9 + RS::kNx + k] += ax * mono[k];
    acc[9 + RS::kNy + k] += ay * mono[k];
  }
#pragma unroll
  for (int k = 1; k < RS::kNl; k++) {
    acc[9 + RS::kDx + k - 1] += bx * mono[k];
    acc[9 + RS::kDy + k - 1] += by * mono[k];
  }
}

// ------------------------------------------------------------ pass B (frame order)
// One wave per frame chunk: per observation u_o = z_o - J_pt w_p, with
// z_o = J_cam,o x from the frame direction (dir; null: x = 0) and w_p from pass A
// (wbuf, double4 per point); then the sums of Z^T u_o and J_I^T u_o,
// wave-reduced; the lanes map the 6 frame-local sums through the generators
// w_k to the pose columns (y_k = w_k . (Z^T u)) and add pose + intrinsic columns
// into replica (chunk mod kVecReplicas) of the camera-side vector.
template <int MODEL, int DEG>
// (min waves per EU: keeps radtan / none within 128 VGPRs under the 128-thread
// bound, as under the old 64-thread one; FOV needs ~155, RPC more)
#ifndef MVBA_PB_WAVES
#define MVBA_PB_WAVES 4  // radtan / none
#endif
__global__ void __launch_bounds__(128, MODEL == kModelRpc ? (DEG <= 2 ? MVBA_RPC_PB_WAVES : 1) : MODEL == kModelFov ? 3 : MVBA_PB_WAVES) k_pass_b(
    const int4* __restrict__ chunks, int32_t nchunks, int32_t chunk_base,
    const Segment* __restrict__ segs, const FrameDesc* __restrict__ fd, const FrameLin* __restrict__ fl,
    const double* __restrict__ frec, const double* __restrict__ params,
    const double4* __restrict__ pts, const int32_t* __restrict__ obs_pid,
    const double2* __restrict__ obs_meas, const double* __restrict__ dir,
    const double4* __restrict__ wbuf, double* __restrict__ yrep, int64_t ng, int32_t flags, double cauchy_c,
    const int32_t* __restrict__ gate, Slab sl, const double4* __restrict__ obsX) {
  using RS = RowShape<MODEL, DEG>;
  constexpr int NA = 6 + RS::kIntr;
  const int lane = threadIdx.x & 63;
  const int ch = (int)xcd_block_solver(nchunks);
  if (ch < 0 || (gate && *gate)) return;
  if constexpr (NA > kPassBRegCols) {
    pass_b_wide<MODEL, DEG>(chunks[ch], chunk_base + ch, segs, fd, fl, frec, params, pts, obs_pid, obs_meas, dir,
                            wbuf, yrep, ng, flags, cauchy_c, sl, obsX);
    return;
  } else {
  const int4 c = chunks[ch];
  const int frame = __builtin_amdgcn_readfirstlane(c.z);
  const FrameDesc& F = fd[frame];
  const double* __restrict__ rec = frec + (int64_t)frame * kFrameRecDoubles;
  const double* __restrict__ d = dir ? dir + (int64_t)frame * kDirStride : nullptr;
  // RPC (VALU-bound pass B, c3): the transposed reduction, accumulators padded
  // to its power of two (entries NA.. stay 0); the other models keep one
  // wave_sum_f64 per accumulator (the transposed form raises their VGPRs:
  // radtan 112 -> 138, and their pass B is latency-bound, not VALU-bound)
  constexpr bool kTred = MVBA_PASSB_TRED && MODEL == kModelRpc;
  constexpr int NACC = kTred ? TSum<NA>::P : NA;
  double acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; q++) acc[q] = 0.0;
  const int nobs = __builtin_amdgcn_readfirstlane(c.y);
  // 1 or 2 waves per chunk (blockDim; the launcher's choice): with 2, wave w
  // takes segments w, w + 2, ... and wave 1 hands its per-lane accumulators to
  // wave 0 through LDS before the one reduction + atomics of the chunk
  const int nw = (int)(blockDim.x >> 6), wv = (int)(threadIdx.x >> 6);
  if constexpr (MODEL == kModelRpc && MVBA_PASSB_PIPE) {
    // RPC (VALU-heavy, 3 waves per SIMD: too few to hide the gathers, wait_frac
    // 0.52 at c3, profiles/r04/ba_c3.json): a software pipeline over the
    // chunk's 64-observation steps, the next step's slot record, point index
    // and w_p loads issued before this step's arithmetic
    int32_t pid_n = 0;
    double4 w_n = make_double4(0.0, 0.0, 0.0, 0.0), X_n = w_n;
    double2 m_n = make_double2(0.0, 0.0);
    auto fetch = [&](int s) {
      if (lane < nobs - s) {
        const int64_t i = (int64_t)c.x + s + lane;
        pid_n = obs_pid[i];
        if (obsX) X_n = obsX[i];
        else m_n = obs_meas[i];
        w_n = wbuf[pid_n];
        if (!obsX) X_n = pts[pid_n];
      }
    };
    fetch(64 * wv);
    for (int s0 = 64 * wv; s0 < nobs; s0 += 64 * nw) {
      const bool act = lane < nobs - s0;
      const double4 w = w_n, X = X_n;
      const double2 m = m_n;
      if (s0 + 64 * nw < nobs) fetch(s0 + 64 * nw);
      if (act) pass_b_rpc_obs<DEG>(F, rec, params, X, m, flags, cauchy_c, obsX ? X.w : -1.0, d, w, acc);
    }
  } else
  for (int s0 = 64 * wv; s0 < nobs; s0 += 64 * nw) {
    if (lane < nobs - s0) {
      const int64_t i = (int64_t)c.x + s0 + lane;
      const int32_t pid = obs_pid[i];
      const double4 w = wbuf[pid];
      const double4 X = obsX ? obsX[i] : pts[pid];
      if constexpr (MODEL == kModelRpc) {
        pass_b_rpc_obs<DEG>(F, rec, params, X, obsX ? double2{0.0, 0.0} : obs_meas[i], flags, cauchy_c,
                            obsX ? X.w : -1.0, d, w, acc);
        continue;
      }
      double Z0[6], Z1[6], I0[RS::kIntr], I1[RS::kIntr], P0[3], P1[3], r[2], hr;
#pragma unroll
      for (int q = 0; q < RS::kIntr; q++) I0[q] = I1[q] = 0.0;
      // obsX: the Cauchy weight rides in .w (K2), no measurement read
      obs_rows<MODEL, DEG>(F, rec, params, X.x, X.y, X.z, obsX ? double2{0.0, 0.0} : obs_meas[i], flags,
                           cauchy_c, Z0, Z1, I0, I1, P0, P1, r, &hr, obsX ? X.w : -1.0);
      double z0 = 0.0, z1 = 0.0;
      if (d) {
#pragma unroll
        for (int a = 0; a < 6; a++) {
          z0 += Z0[a] * d[a];
          z1 += Z1[a] * d[a];
        }
#pragma unroll
        for (int q = 0; q < RS::kIntr; q++) {
          z0 += I0[q] * d[6 + q];
          z1 += I1[q] * d[6 + q];
        }
      }
      double2 u;
      u.x = z0 - (P0[0] * w.x + P0[1] * w.y + P0[2] * w.z);
      u.y = z1 - (P1[0] * w.x + P1[1] * w.y + P1[2] * w.z);
#pragma unroll
      for (int a = 0; a < 6; a++) acc[a] += Z0[a] * u.x + Z1[a] * u.y;
#pragma unroll
      for (int q = 0; q < RS::kIntr; q++) acc[6 + q] += I0[q] * u.x + I1[q] * u.y;
    }
  }
  if constexpr (MODEL != kModelRpc) {
    __shared__ double comb[NA][64];
    if (nw > 1) {
      if (wv == 1)
#pragma unroll
        for (int q = 0; q < NA; q++) comb[q][lane] = acc[q];
      __syncthreads();
      if (wv == 1) return;
#pragma unroll
      for (int q = 0; q < NA; q++) acc[q] += comb[q][lane];
    }
  }
  const FrameLin& L = fl[frame];
  double* y = yrep + (int64_t)((chunk_base + ch) & (kVecReplicas - 1)) * ng;
  if constexpr (kTred) {
  // transposed wave sums: lane l holds the total of accumulator l >> S; the six
  // Z^T u sums go to every lane through readlane, pose column k on lane k,
  // intrinsic column q on the first lane holding accumulator 6 + q
  {
    constexpr int S = TSum<NA>::kShift;
    const double tv = wave_sum_transpose<NA>(acc, lane);
    double zs[6];
#pragma unroll
    for (int a = 0; a < 6; a++) zs[a] = readlane_f64(tv, a << S);
    if (lane < kPoseCols) {
      const int blk = lane / 7;  // 0 beg, 1 end, 2 ref_to_cam, 3 offset (lane 21)
      const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
      if (L.goff[b] >= 0) {
        const double* wk = rec + 12 + 6 * lane;
        double v = 0.0;
#pragma unroll
        for (int a = 0; a < 6; a++) v += wk[a] * zs[a];
        accumulate(y, L.goff[b] + (lane - 7 * blk), v, sl, chunk_base + ch, lane);
      }
    }
    const int idx = lane >> S;
    const int q = idx - 6;  // 0 focal, 1..2 center, 3.. distortion
    if ((lane & ((1 << S) - 1)) == 0 && q >= 0 && q < RS::kIntr) {
      int64_t dst = -1;
      if (q == 0) dst = L.goff[MVBA_BLK_FOCAL];
      else if (q < 3) dst = L.goff[MVBA_BLK_CENTER] >= 0 ? L.goff[MVBA_BLK_CENTER] + (q - 1) : -1;
      else if (q - 3 < F.K) dst = L.goff[MVBA_BLK_DIST] >= 0 ? L.goff[MVBA_BLK_DIST] + (q - 3) : -1;
      if (dst >= 0) accumulate(y, dst, tv, sl, chunk_base + ch, kPoseCols + q);
    }
  }
  } else {
#pragma unroll
  for (int q = 0; q < NA; q++) acc[q] = wave_sum_f64(acc[q]);
  // every lane holds the totals; lane k < 22 -> pose column k, 22.. -> intrinsics
  int64_t dst = -1;
  double v = 0.0;
  if (lane < kPoseCols) {
    const int blk = lane / 7;  // 0 beg, 1 end, 2 ref_to_cam, 3 offset (lane 21)
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    if (L.goff[b] >= 0) {
      const double* wk = rec + 12 + 6 * lane;
#pragma unroll
      for (int a = 0; a < 6; a++) v += wk[a] * acc[a];
      dst = L.goff[b] + (lane - 7 * blk);
    }
  } else {
    const int q = lane - kPoseCols;  // 0 focal, 1..2 center, 3.. distortion
    if (q < RS::kIntr) {
#pragma unroll
      for (int e = 0; e < RS::kIntr; e++)
        if (e == q) v = acc[6 + e];
      if (q == 0) dst = L.goff[MVBA_BLK_FOCAL];
      else if (q < 3) dst = L.goff[MVBA_BLK_CENTER] >= 0 ? L.goff[MVBA_BLK_CENTER] + (q - 1) : -1;
      else if (q - 3 < F.K) dst = L.goff[MVBA_BLK_DIST] >= 0 ? L.goff[MVBA_BLK_DIST] + (q - 3) : -1;
    }
  }
  if (dst >= 0) accumulate(y, dst, v, sl, chunk_base + ch, lane);
  }
  }
}

// y = sum_r yrep[r] (replicas re-zeroed); with diag: y += diag .* x; with dot_out
// the grid also reduces x.y into dot_out (p'q when no cross-rank exchange follows).
// CG step length (conjugate_gradients_solver.cc [ext]): pq <= 0 -> "Matrix is
// indefinite" (NO_CONVERGENCE, x kept); alpha = rho / pq, inf -> failure
__device__ __forceinline__ void cg_step_length(CgCtl* ctl, double pq) {
  ctl->first = 0;
  if (pq <= 0.0 || isinf(pq) || isnan(pq)) {
    ctl->status = 1;
    ctl->done = 1;
  } else {
    const double alpha = ctl->rho / pq;
    ctl->alpha = alpha;
    if (isinf(alpha)) {
      ctl->status = 2;
      ctl->done = 1;
    }
  }
}

// The finalising block of the x.y reduction. local_dot (sharded solves with a
// library communicator): the dot is this rank's share, summed by the exchange
// that follows; the step length is taken by the update kernel from the summed
// dot and rho_step, the rho snapshot taken here (the update kernel's own
// finalisation overwrites rho for the next iteration while its frame blocks
// may still be reading it).
__device__ __forceinline__ void cg_step_finish(CgCtl* ctl, double pq, int32_t local_dot) {
  if (local_dot) ctl->rho_step = ctl->rho;
  else cg_step_length(ctl, pq);
}

// With lz.z set, x is the CG direction p_new = z (+ beta p_old): formed here
// (first / beta from lz.ctl) and stored to lz.p_new for the update kernel.
__device__ __forceinline__ double x_entry(const double* __restrict__ x, const LazyDir& lz, int64_t e) {
  if (!lz.z) return x[e];
  const double v = lazy_p(lz, lz.ctl->first, lz.ctl->beta, e);
  lz.p_new[e] = v;
  return v;
}

// local_dot 2 (single rank): no finalising block. Each block adds its share of
// x.y to dot_out with one fp64 atomic, block 0 zeroes dot_zero (the other slot of
// the double-buffered accumulator, read by the previous update kernel) and
// snapshots rho; the update kernel takes the step length from the sum (the
// sharded path's form), so the arrival counter and the last block's partial
// loads leave the CG iteration's critical path.
__global__ void __launch_bounds__(256) k_vec_rep_reduce(double* __restrict__ yrep, int64_t n,
                                                        const double* __restrict__ diag,
                                                        const double* __restrict__ x, double* __restrict__ y,
                                                        double* __restrict__ partial, unsigned* __restrict__ counter,
                                                        double* __restrict__ dot_out, const int32_t* __restrict__ gate,
                                                        CgCtl* __restrict__ ctl, LazyDir lz, int32_t local_dot,
                                                        double* __restrict__ dot_zero) {
  if (gate && *gate) return;
  if (local_dot == 2 && blockIdx.x == 0 && threadIdx.x == 0) {
    *dot_zero = 0.0;
    ctl->rho_step = ctl->rho;
  }
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double d = 0.0;
  if (e < n) {
    const double xe = (x || lz.z) ? x_entry(x, lz, e) : 0.0;
    // all replica loads in flight before the first add / zeroing store (the
    // stores go through the same pointer, so a fused loop serialises them)
    double v[kVecReplicas];
#pragma unroll
    for (int r = 0; r < kVecReplicas; r++) v[r] = yrep[r * n + e];
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < kVecReplicas; r++) acc += v[r];
#pragma unroll
    for (int r = 0; r < kVecReplicas; r++) yrep[r * n + e] = 0.0;
    if (diag) acc += diag[e] * xe;
    y[e] = acc;
    d = xe * acc;
  }
  if (local_dot == 2) {
    block_sum<1>(&d);
    if (threadIdx.x == 0) atomicAdd(dot_out, d);
    return;
  }
  if (dot_out && grid_sum_finalize(d, partial, counter, dot_out) && ctl && threadIdx.x == 0)
    cg_step_finish(ctl, dot_out[0], local_dot);
}

// Deterministic mode: y[e] = sum of entry e's slab positions in slab order (CSR
// e -> positions; one wave per entry, lane-strided sums and a fixed butterfly),
// then the same damping, x.y reduction and CG step length as k_vec_rep_reduce.
__global__ void __launch_bounds__(256) k_vec_slab_reduce(SlabTiers tiers, const int64_t* __restrict__ begin,
                                                         const int64_t* __restrict__ pos,
                                                         const double* __restrict__ val,
                                                         const double* __restrict__ diag,
                                                         const double* __restrict__ x, double* __restrict__ y,
                                                         double* __restrict__ partial, unsigned* __restrict__ counter,
                                                         double* __restrict__ dot_out,
                                                         const int32_t* __restrict__ gate, CgCtl* __restrict__ ctl,
                                                         LazyDir lz, int32_t local_dot) {
  if (gate && *gate) return;
  int64_t e;
  double acc;
  double d = 0.0;
  if (slab_gather(tiers, begin, pos, val, &e, &acc)) {
    const double xe = (x || lz.z) ? x_entry(x, lz, e) : 0.0;
    if (diag) acc += diag[e] * xe;
    y[e] = acc;
    d = xe * acc;
  }
  if (dot_out && grid_sum_finalize(d, partial, counter, dot_out) && ctl && threadIdx.x == 0)
    cg_step_finish(ctl, dot_out[0], local_dot);
}

// y += diag .* x; dot_out = x.y (after a cross-rank sum of y); with ctl the
// finalising block also takes the CG step length (sharded device CG), gated
// like the rest of the iteration
__global__ void __launch_bounds__(256) k_add_diag(int64_t n, const double* __restrict__ diag,
                                                  const double* __restrict__ x, double* __restrict__ y,
                                                  double* __restrict__ partial, unsigned* __restrict__ counter,
                                                  double* __restrict__ dot_out, const int32_t* __restrict__ gate,
                                                  CgCtl* __restrict__ ctl, LazyDir lz) {
  if (gate && *gate) return;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double d = 0.0;
  if (e < n) {
    const double xe = x_entry(x, lz, e);
    const double v = y[e] + diag[e] * xe;
    y[e] = v;
    d = xe * v;
  }
  if (dot_out && grid_sum_finalize(d, partial, counter, dot_out) && ctl && threadIdx.x == 0)
    cg_step_length(ctl, dot_out[0]);
}

// r_new(k) and z_i = (M^-1 r_new)_i as the CG update forms them (shared by the
// entry threads and the frame blocks, so both see the same values)
__device__ __forceinline__ double cg_rnew(int32_t mode, double alpha, const double* __restrict__ q,
                                          const double* __restrict__ b, const double* __restrict__ r_in, int64_t k) {
  if (mode & 2) return r_in[k] - alpha * q[k];
  if (mode & 4) return q ? b[k] - q[k] : b[k];
  return r_in[k];
}
__device__ __forceinline__ double cg_zentry(const CgEntry& E, const double* __restrict__ minv, int32_t mode,
                                            double alpha, const double* __restrict__ q, const double* __restrict__ b,
                                            const double* __restrict__ r_in) {
  const double* M = minv + E.moff;
  double zi = 0.0;
  for (int k = 0; k < E.nb; k++) zi += M[k] * cg_rnew(mode, alpha, q, b, r_in, E.o + k);
  return zi;
}

// One CG step on the camera side, one thread per camera entry
// (conjugate_gradients_solver.cc [ext]); r is double-buffered (r_in -> r_out):
//   mode & 1: x += alpha p;  & 2: r = r_in - alpha q;  & 4: r = b - q (q null: r = b);
//   mode & 8: z = M^-1 r (explicit block inverses) and out = [x.b, x.r, r.z].
// With fz.dz (mode & 8), blocks from fz.owner_blocks on are frame blocks, one
// wave per frame: dz_f = W_f z from z recomputed for the frame's camera entries
// (the next product's direction is then dz + beta dp, DirPair): the separate
// direction kernel between this update and pass A is gone.
// The step length of the CG update: from the exchanged (sharded) or
// atomically summed (single rank) p.q, pq_in, and rho_step (every block
// computes the same value; `record`: this thread writes it to ctl), else the
// reduction's ctl->alpha. False: the iteration stops here (indefinite / non-
// finite step; ctl->done set by the recording thread).
__device__ __forceinline__ bool cg_alpha(CgCtl* __restrict__ ctl, const double* __restrict__ pq_in, bool record,
                                         double* alpha) {
  if (!pq_in) {
    *alpha = ctl->alpha;
    return true;
  }
  const double pq = *pq_in;
  const double a = ctl->rho_step / pq;
  const bool indefinite = pq <= 0.0 || isinf(pq) || isnan(pq);
  const bool bad = indefinite || isinf(a);
  if (record) {
    ctl->first = 0;
    if (bad) {
      ctl->status = indefinite ? 1 : 2;
      ctl->done = 1;
    } else {
      ctl->alpha = a;
    }
  }
  *alpha = a;
  return !bad;
}

// One thread: the control block's outcome into the host mirror (CgMirror).
__device__ __forceinline__ void cg_mirror(CgCtl* __restrict__ ctl, CgMirror* __restrict__ mir) {
  const uint32_t q = ++ctl->mseq;
  mir->done = ctl->done;
  mir->status = ctl->status;
  mir->iters = ctl->iters;
  __hip_atomic_store(&mir->seq, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The finalising thread of a CG update: the q-criterion, rho and beta of the
// next iteration (conjugate_gradients_solver.cc [ext]) into ctl, from the
// grid sums [x.b, x.r, r.z].
__device__ __forceinline__ void cg_finalize(CgCtl* __restrict__ ctl, const double* sums, int32_t iter) {
  const double sxb = sums[0], sxr = sums[1];
  const double rho_next = sums[2];
  if (iter == kIterFromCtl) iter = ctl->it++;
  auto bad = [](double v) { return v == 0.0 || isinf(v) || isnan(v); };
  if (iter == 0) {  // r = b, z = M^-1 r: initial rho, Q0 = 0
    if (ctl->bb == 0.0) {  // "Convergence. |b| = 0." (x stays 0)
      ctl->status = 0;
      ctl->iters = 0;
      ctl->done = 1;
      return;
    }
    ctl->Q0 = 0.0;
    ctl->first = 1;
    if (bad(rho_next)) {
      ctl->status = 2;
      ctl->iters = 1;
      ctl->done = 1;
    }
    ctl->rho = rho_next;
    return;
  }
  ctl->iters = iter;
  const double Q1 = -(sxb + sxr);
  const double zeta = iter * (Q1 - ctl->Q0) / Q1;
  if (zeta < ctl->eta && iter >= ctl->min_iter) {
    ctl->status = 0;
    ctl->done = 1;
    return;
  }
  ctl->Q0 = Q1;
  if (iter >= ctl->max_iter) {
    ctl->status = 1;
    ctl->done = 1;
    return;
  }
  // top of the next iteration: rho, beta
  const double last_rho = ctl->rho;
  if (bad(rho_next)) {
    ctl->status = 2;
    ctl->iters = iter + 1;
    ctl->done = 1;
    return;
  }
  const double beta = rho_next / last_rho;
  ctl->rho = rho_next;
  ctl->beta = beta;
  if (bad(beta)) {
    ctl->status = 2;
    ctl->iters = iter + 1;
    ctl->done = 1;
  }
}

// The camera-entry part of a CG update (thread i of blocks [0, nb)): x, r, z
// and, with mode & 8, the [x.b, x.r, r.z] grid sums whose last block takes the
// step control (q-criterion, rho, beta) in ctl and, with mir, mirrors it.
__device__ __forceinline__ void cg_update_entries(int64_t i, int64_t n, const CgEntry* __restrict__ ent,
                                                  const double* __restrict__ minv, int32_t mode, double alpha,
                                                  const double* __restrict__ p, const double* __restrict__ q,
                                                  const double* __restrict__ b, double* __restrict__ x,
                                                  const double* __restrict__ r_in, double* __restrict__ r_out,
                                                  double* __restrict__ z, double* __restrict__ partial,
                                                  unsigned* __restrict__ counters, double* __restrict__ out,
                                                  CgCtl* __restrict__ ctl, int32_t iter, unsigned nb,
                                                  CgMirror* __restrict__ mir = nullptr) {
  double xb = 0.0, xr = 0.0, rz = 0.0;
  if (i < n) {
    const CgEntry E = ent[i];
    double xi = x[i];
    if (mode & 1) {
      xi += alpha * p[i];
      x[i] = xi;
    }
    const double ri = cg_rnew(mode, alpha, q, b, r_in, i);
    if (mode & 6) r_out[i] = ri;  // mode 1 alone (before a residual reset) leaves r to the reset
    if (mode & 8) {
      const double zi = cg_zentry(E, minv, mode, alpha, q, b, r_in);
      z[i] = zi;
      xb = xi * b[i];
      xr = xi * ri;
      rz = ri * zi;
    }
  }
  if (mode & 8) {
    double sums[3];
    if (grid_sum3_finalize(xb, xr, rz, partial, counters, out, sums, nb) && ctl && threadIdx.x == 0) {
      cg_finalize(ctl, sums, iter);
      if (mir) cg_mirror(ctl, mir);
    }
  }
}

__global__ void __launch_bounds__(256) k_cg_update(int64_t n, const CgEntry* __restrict__ ent,
                                                   const double* __restrict__ minv,
                                                   int32_t mode, double alpha, const double* __restrict__ p,
                                                   const double* __restrict__ q, const double* __restrict__ b,
                                                   double* __restrict__ x, const double* __restrict__ r_in,
                                                   double* __restrict__ r_out, double* __restrict__ z,
                                                   double* __restrict__ partial, unsigned* __restrict__ counters,
                                                   double* __restrict__ out, CgCtl* __restrict__ ctl, int32_t iter,
                                                   FrameDirZ fz, const double* __restrict__ pq_in,
                                                   CgMirror* __restrict__ mir) {
  if (ctl) {
    // (a stopped or failed step still mirrors its state: block 0, thread 0)
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (ctl->done) {
      if (mir && lead) cg_mirror(ctl, mir);
      return;
    }
    // sharded / atomic p.q: the step length from the summed p.q (block 0 records it)
    if (!cg_alpha(ctl, pq_in, lead, &alpha)) {
      if (mir && lead) cg_mirror(ctl, mir);
      return;
    }
  }
  if (fz.dz && (int32_t)blockIdx.x >= fz.owner_blocks) {
    const int f = ((int32_t)blockIdx.x - fz.owner_blocks) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
    if (f >= fz.nframes) return;
    const FrameLin& L = ((const FrameLin*)fz.fl)[f];
    const int32_t K = fz.fd[f].K;
    // z_j of camera block b straight from the frame's block offsets (the same
    // entries and block-inverse row the entry threads use, without their
    // CgEntry descriptor load)
    auto Z = [&](int blk, int j) {
      const int nb = blk <= MVBA_BLK_REF_TO_CAM ? 7 : blk == MVBA_BLK_CENTER ? 2 : blk == MVBA_BLK_DIST ? K : 1;
      return cg_zentry(CgEntry{(int32_t)L.goff[blk], nb, L.hoff[blk] + (int64_t)j * nb}, minv, mode, alpha, q, b,
                       r_in);
    };
    frame_dir_body<true>(L, K, fz.frec + (int64_t)f * kFrameRecDoubles, (int)(threadIdx.x & 63), Z,
                         fz.dz + (int64_t)f * kDirStride);
    return;
  }
  cg_update_entries((int64_t)blockIdx.x * blockDim.x + threadIdx.x, n, ent, minv, mode, alpha, p, q, b, x, r_in,
                    r_out, z, partial, counters, out, ctl, iter, fz.dz ? (unsigned)fz.owner_blocks : 0u, mir);
}

// The fused CG step (FusedStep): blocks [0, eb) run the update of iteration
// i - 1 (k_cg_update's entry blocks, mode 1|2|8: x, r, z, the grid sums and
// the step control), blocks from eb on run pass A of iteration i on its frame
// chunks, one wave per chunk. A pass-A wave recomputes z = M^-1 (r - alpha q)
// for its frame's camera entries (the entry blocks' arithmetic, the update's
// frame blocks' form), stages the frame's z record and the previous
// direction's record, and stores both products per slot (c_z | c_p.x in cbuf,
// c_p.y, c_p.z in cbuf2): beta is known only once the entry blocks' grid
// reduction has finished, i.e. in the next launch (k_point_w combines). The
// wave of the frame's first chunk stores the z record (full: pose sums and
// intrinsic entries) for k_point_w's frame blocks. eb is a multiple of 8, so
// the pass-A blocks keep the XCD mapping of k_pass_a_frame. Reprojection-only,
// one model group, obsX records (the host checks).
template <int MODEL, int DEG>
__global__ void __launch_bounds__(256) k_upd_pass_a(
    int64_t n, const CgEntry* __restrict__ ent, const double* __restrict__ minv, const double* __restrict__ p,
    const double* __restrict__ q, const double* __restrict__ b, double* __restrict__ x,
    const double* __restrict__ r_in, double* __restrict__ r_out, double* __restrict__ z,
    double* __restrict__ partial, unsigned* __restrict__ counters, double* __restrict__ out,
    CgCtl* __restrict__ ctl, const double* __restrict__ pq_in, int32_t eb, const int4* __restrict__ chunks,
    int32_t nchunks, const FrameLin* __restrict__ fl, const FrameDesc* __restrict__ fd,
    const double* __restrict__ frec, const double* __restrict__ dp, double* __restrict__ dz_out,
    const int32_t* __restrict__ slot_po, double4* __restrict__ cbuf, double2* __restrict__ cbuf2,
    const double* __restrict__ prec, const double4* __restrict__ obsX) {
  if (ctl->done) return;
  double alpha = 0.0;
  const bool entry = (int32_t)blockIdx.x < eb;
  if (!cg_alpha(ctl, pq_in, entry && blockIdx.x == 0 && threadIdx.x == 0, &alpha)) return;
  if (entry) {
    cg_update_entries((int64_t)blockIdx.x * blockDim.x + threadIdx.x, n, ent, minv, 1 | 2 | 8, alpha, p, q, b, x,
                      r_in, r_out, z, partial, counters, out, ctl, kIterFromCtl, (unsigned)eb);
    return;
  }
  constexpr int ND = 6 + RowShape<MODEL, DEG>::kIntr;
  __shared__ double sz[kPassAWaves][ND];
  __shared__ double sp[kPassAWaves][ND];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t nb = (nchunks + kPassAWaves - 1) / kPassAWaves;
  int64_t blk = -1;
  {
    // xcd_block_solver on the block index past the entry blocks
    const int64_t bb = (int64_t)blockIdx.x - eb;
    if (!MVBA_XCD_SOLVER) {
      blk = bb < nb ? bb : -1;
    } else {
      const int64_t per = (nb + kXcds - 1) / kXcds;
      const int64_t l = (bb % kXcds) * per + bb / kXcds;
      blk = l < nb ? l : -1;
    }
  }
  const int ch = (int)blk * kPassAWaves + wv;
  if (blk < 0 || ch >= nchunks) return;
  const int4 c = chunks[ch];
  const int frame = __builtin_amdgcn_readfirstlane(c.z);
  const int nobs = __builtin_amdgcn_readfirstlane(c.y);
  const double* __restrict__ rec = prec + (int64_t)frame * kProjDoubles;
  const int64_t base = (int64_t)frame * kDirStride;
  double* d1 = sz[wv];
  double* d2 = sp[wv];
  for (int m = lane; m < ND; m += 64) {
    d1[m] = 0.0;  // entries frame_dir_body leaves (past the live distortion columns)
    d2[m] = dp[base + m];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  {
    const FrameLin& L = fl[frame];
    const int32_t K = fd[frame].K;
    auto Z = [&](int bk, int j) {
      const int nbk = bk <= MVBA_BLK_REF_TO_CAM ? 7 : bk == MVBA_BLK_CENTER ? 2 : bk == MVBA_BLK_DIST ? K : 1;
      return cg_zentry(CgEntry{(int32_t)L.goff[bk], nbk, L.hoff[bk] + (int64_t)j * nbk}, minv, 1 | 2 | 8, alpha, q,
                       b, r_in);
    };
    frame_dir_body<false>(L, K, frec + (int64_t)frame * kFrameRecDoubles, lane, Z, d1);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (c.w)
    for (int m = lane; m < ND; m += 64) dz_out[base + m] = d1[m];
  for (int s0 = 0; s0 < nobs; s0 += 64) {
    if (lane < nobs - s0) {
      const int64_t i = (int64_t)c.x + s0 + lane;
      const double4 X = obsX[i];
      double za[2], zb[2], P0[3], P1[3];
      pass_a_obs2<MODEL, DEG>(rec, d1, d2, X, X.w, za, zb, P0, P1);
      const int64_t o = slot_po ? (int64_t)slot_po[i] : i;
      cbuf[o] = make_double4(P0[0] * za[0] + P1[0] * za[1], P0[1] * za[0] + P1[1] * za[1],
                             P0[2] * za[0] + P1[2] * za[1], P0[0] * zb[0] + P1[0] * zb[1]);
      cbuf2[o] = make_double2(P0[1] * zb[0] + P1[1] * zb[1], P0[2] * zb[0] + P1[2] * zb[1]);
    }
  }
}

// ------------------------------------------------------------ vectors / blocks
// out = a*x + b*y (+ c*z)
__global__ void k_axpby(int64_t n, double a, const double* __restrict__ x, double b,
                        const double* __restrict__ y, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = a * x[e] + (y ? b * y[e] : 0.0);
}

// out[0] = x.y (y null: x.x) in one launch: grid-stride partial sums, last-block finalisation
__global__ void __launch_bounds__(256) k_dot_fin(int64_t n, const double* __restrict__ x,
                                                 const double* __restrict__ y, double* __restrict__ partial,
                                                 unsigned* __restrict__ counter, double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    acc += x[e] * (y ? y[e] : x[e]);
  grid_sum_finalize(acc, partial, counter, out);
}

// out[0] = sum partial[0..n)
__global__ void __launch_bounds__(256) k_sum(int64_t n, const double* __restrict__ partial,
                                             double* __restrict__ out) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) acc += partial[e];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// First level of a two-level deterministic sum: block b adds partial[b per ..
// (b + 1) per) in a fixed order (thread-strided, then a fixed tree) into out[b]
__global__ void __launch_bounds__(256) k_sum_level(int64_t n, int64_t per, const double* __restrict__ partial,
                                                   double* __restrict__ out) {
  __shared__ double red[256];
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  double acc = 0.0;
  for (int64_t e = b0 + threadIdx.x; e < b1; e += 256) acc += partial[e];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// Block-Jacobi preconditioner (Ceres' JACOBI for ITERATIVE_SCHUR [ext]:
// blocks of F'F + D^2): one workgroup (one wave) per camera block inverts
// H_bb + diag(d) explicitly by Gauss-Jordan elimination (symmetric positive
// definite: no pivoting; a vanishing pivot = a direction the block does not
// see, inverted as identity), in LDS up to kPrecLds wide, in place in the
// output beyond (RPC distortion of degree >= 4: 116..220 entries); applying it
// is then a block mat-vec. Lane j owns column j: n rank-1 steps with no
// per-lane serial chain. (A column-serial Cholesky with per-lane triangular
// solves kept its solve vector in scratch memory: 282 us per build at c3,
// 3,000 pose blocks; profiles/r03/ab_block_prec/.)
constexpr int kPrecLds = 88;  // 88^2 + 2 * 88 doubles = 62 KB: within the 64 KB of dynamic LDS a plain launch gets
constexpr int kPrecThreads = 256;  // 4 waves per block share the elimination steps
constexpr int kPrecSmall = 8;      // blocks up to this size: k_block_prec_small (one wave each)

__device__ __forceinline__ void block_inverse_gj(int n, const double* __restrict__ H, const double* __restrict__ db,
                                                 double* __restrict__ A, double* colk, double* rowk) {
  // thread t owns column (t mod 64) (+ 64 past 64 columns) and one of the
  // block's row ranges (one per wave): no integer division in the loops, and
  // the n elimination steps spread over every wave of the workgroup
  const int tid = threadIdx.x, lane = tid & 63, nw = blockDim.x >> 6;
  const int rq = (n + nw - 1) / nw, r0 = (tid >> 6) * rq, r1 = min(n, r0 + rq);
  // the lower triangle as stored (coalesced), diagonal damped
  for (int e0 = tid; e0 < n * n; e0 += 8 * (int)blockDim.x) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = e0 + u * (int)blockDim.x;
      v[u] = e < n * n ? H[e] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = e0 + u * (int)blockDim.x;
      if (e < n * n) A[e] = v[u];
    }
  }
  __syncthreads();
  for (int j = lane; j < n; j += 64)
    for (int i = r0; i < r1; i++) {
      if (i < j) A[i * n + j] = A[j * n + i];  // upper triangle from the lower
      else if (i == j) A[i * n + j] += db[i];
    }
  __syncthreads();
  for (int k = 0; k < n; k++) {
    for (int i = tid; i < n; i += blockDim.x) {
      colk[i] = A[i * n + k];
      rowk[i] = A[k * n + i];
    }
    __syncthreads();
    const double piv = colk[k];
    const bool ok = piv > 1e-300;
    const double ip = ok ? 1.0 / piv : 0.0;
    for (int j = lane; j < n; j += 64) {
      const double rj = rowk[j] * ip;
      if (!ok) {
        for (int i = r0; i < r1; i++)
          if (i == k || j == k) A[i * n + j] = (i == j) ? 1.0 : 0.0;
      } else if (j == k) {
        for (int i = r0; i < r1; i++) A[i * n + j] = (i == k) ? ip : -colk[i] * ip;
      } else {
        // 8 rows at a time: every load of the group issued before its stores
        // (A and colk share one LDS array, so the compiler cannot move a load
        // above an earlier store itself)
        for (int i0 = r0; i0 < r1; i0 += 8) {
          double a[8], c[8];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int i = min(i0 + u, r1 - 1);
            a[u] = A[i * n + j];
            c[u] = colk[i];
          }
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int i = i0 + u;
            if (i < r1) A[i * n + j] = (i == k) ? rj : a[u] - c[u] * rj;
          }
        }
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kPrecThreads) k_block_prec(int32_t nblocks, const int64_t* __restrict__ goff,
                                                   const int64_t* __restrict__ hoff,
                                                   const int32_t* __restrict__ bsize,
                                                   const double* __restrict__ hess, const double* __restrict__ d,
                                                   double* __restrict__ minv, int32_t small_done) {
  extern __shared__ double Ls[];  // [n * n | pivot column | pivot row], or the pivot column and row of the wide path
  const int b = blockIdx.x;
  if (b >= nblocks) return;
  const int n = bsize[b];
  if (n <= kPrecSmall && small_done) return;  // k_block_prec_small's
  const int lane = threadIdx.x;
  const double* H = hess + hoff[b];
  const double* db = d + goff[b];
  if (n > kPrecLds) {
    block_inverse_gj(n, H, db, minv + hoff[b], Ls, Ls + n);
    return;
  }
  block_inverse_gj(n, H, db, Ls, Ls + n * n, Ls + n * n + n);
  double* M = minv + hoff[b];
  for (int e = lane; e < n * n; e += blockDim.x) M[e] = Ls[e];
}

// Blocks of at most 8 entries (poses, rig, offsets, focal, centre, radtan /
// FOV distortion: every camera block of c2): one wave per block, lane 8 i + j
// holds A[i][j] in a register and the n Gauss-Jordan steps of
// block_inverse_gj (same formulas, same pivot rule) take the pivot row,
// column and element by lane shuffles: no LDS staging, no block barriers.
// A 256-thread workgroup per 7x7 block spent most of its ~14 us build in the
// barrier-separated steps of mostly idle waves (profiles/r05/r05e/).
__global__ void __launch_bounds__(256) k_block_prec_small(int32_t nblocks, const int64_t* __restrict__ goff,
                                                          const int64_t* __restrict__ hoff,
                                                          const int32_t* __restrict__ bsize,
                                                          const double* __restrict__ hess,
                                                          const double* __restrict__ d, double* __restrict__ minv) {
  const int b = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (b >= nblocks) return;
  const int n = bsize[b];
  if (n > kPrecSmall) return;  // k_block_prec's
  const int lane = threadIdx.x & 63, i = lane >> 3, j = lane & 7;
  const bool act = i < n && j < n;
  const double* H = hess + hoff[b];
  double a = 0.0;
  if (act) {
    a = i >= j ? H[i * n + j] : H[j * n + i];  // the lower triangle as stored
    if (i == j) a += d[goff[b] + i];
  }
  for (int k = 0; k < n; k++) {
    const double colk = __shfl(a, (i << 3) + k, 64);
    const double rowk = __shfl(a, (k << 3) + j, 64);
    const double piv = __shfl(a, (k << 3) + k, 64);
    const bool ok = piv > 1e-300;
    const double ip = ok ? 1.0 / piv : 0.0;
    const double rj = rowk * ip;
    if (!ok) {
      if (i == k || j == k) a = (i == j) ? 1.0 : 0.0;
    } else if (j == k) {
      a = (i == k) ? ip : -colk * ip;
    } else {
      a = (i == k) ? rj : a - colk * rj;
    }
  }
  if (act) minv[hoff[b] + i * n + j] = a;
}

// ---- compact free-parameter vectors: [camera-side entries (layout order) | 3 per point]
// c = diag(J^T J) in compact order (camera blocks' Hessian diagonals, then V_p diagonals)
__global__ void k_extract_diag(int32_t nblocks, const int64_t* __restrict__ goff, const int64_t* __restrict__ hoff,
                               const int32_t* __restrict__ bsize, const double* __restrict__ hess, int64_t npts,
                               const double* __restrict__ V, int64_t ng, double* __restrict__ c) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nblocks) {
    const int n = bsize[t];
    for (int i = 0; i < n; i++) c[goff[t] + i] = hess[hoff[t] + i * n + i];
  } else if (t - nblocks < npts) {
    const int64_t p = t - nblocks;
    c[ng + 3 * p] = V[6 * p];
    c[ng + 3 * p + 1] = V[6 * p + 3];
    c[ng + 3 * p + 2] = V[6 * p + 5];
  }
}

// Jacobi column scaling of Ceres' TrustRegionMinimizer [ext]: s = 1/(1+sqrt(c)),
// computed once from the iteration-0 Jacobian.
__global__ void k_jacobi_scale(int64_t n, const double* __restrict__ c, double* __restrict__ sc) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) sc[e] = 1.0 / (1.0 + sqrt(c[e]));
}

// LevenbergMarquardtStrategy::ComputeStep [ext] on the scaled Jacobian J S:
// D~^2 = clamp(s^2 c, min, max) / radius; unscaled damping = D~^2 / s^2.
// 1/radius from device memory when inv_radius_dev is set (the solver's step
// prologue is a captured graph: its launch arguments cannot change per step)
__global__ void k_lm_diag(int64_t n, const double* __restrict__ c, const double* __restrict__ sc,
                          double inv_radius, const double* __restrict__ inv_radius_dev, double dmin, double dmax,
                          double* __restrict__ d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double ir = inv_radius_dev ? *inv_radius_dev : inv_radius;
  const double s2 = sc ? sc[e] * sc[e] : 1.0;
  d[e] = fmin(fmax(s2 * c[e], dmin), dmax) * ir / s2;
}

// compact <- packed parameters (constant points read as 0)
__global__ void k_gather(int64_t ncam, const int64_t* __restrict__ cam_poff, int64_t npts,
                         const int64_t* __restrict__ pt_off, const uint8_t* __restrict__ pt_free,
                         const double* __restrict__ params, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < ncam) {
    out[e] = params[cam_poff[e]];
  } else if (e < ncam + 3 * npts) {
    const int64_t q = e - ncam, p = q / 3;
    out[e] = pt_free[p] ? params[pt_off[p] + q % 3] : 0.0;
  }
}

// packed parameters <- compact (constant points untouched)
__global__ void k_scatter(int64_t ncam, const int64_t* __restrict__ cam_poff, int64_t npts,
                          const int64_t* __restrict__ pt_off, const uint8_t* __restrict__ pt_free,
                          const double* __restrict__ in, double* __restrict__ params) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < ncam) {
    params[cam_poff[e]] = in[e];
  } else if (e < ncam + 3 * npts) {
    const int64_t q = e - ncam, p = q / 3;
    if (pt_free[p]) params[pt_off[p] + q % 3] = in[e];
  }
}

// out = Plus(x, delta) with bounds (ParameterBlock::Plus + box projection [ext])
__global__ void k_plus(int64_t n, const double* __restrict__ x, const double* __restrict__ delta,
                       const double* __restrict__ lower, const double* __restrict__ upper,
                       double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double v = x[e] + delta[e];
  if (lower) v = fmax(v, lower[e]);
  if (upper) v = fmin(v, upper[e]);
  out[e] = v;
}

// partial[block] = max |x - Plus(x, -g)| (projected gradient, Ceres' gradient_max_norm)
__global__ void __launch_bounds__(256) k_proj_grad_max(int64_t n, const double* __restrict__ x,
                                                       const double* __restrict__ g,
                                                       const double* __restrict__ lower,
                                                       const double* __restrict__ upper,
                                                       double* __restrict__ partial) {
  __shared__ double red[256];
  double m = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    double v = x[e] - g[e];
    if (lower) v = fmax(v, lower[e]);
    if (upper) v = fmin(v, upper[e]);
    m = fmax(m, fabs(x[e] - v));
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_max(int64_t n, const double* __restrict__ partial,
                                             double* __restrict__ out) {
  __shared__ double red[256];
  double m = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) m = fmax(m, partial[e]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// cost only (sum 0.5 rho) of one model group, partial per 256-thread block
template <int MODEL, int DEG>
__global__ void __launch_bounds__(256) k_cost(const Segment* __restrict__ segs, int32_t nseg,
                                              const FrameDesc* __restrict__ fd,
                                              const double* __restrict__ frec,
                                              const double* __restrict__ params,
                                              const double4* __restrict__ pts,
                                              const int32_t* __restrict__ obs_pid,
                                              const double2* __restrict__ obs_meas, int32_t flags,
                                              double cauchy_c, double* __restrict__ partial) {
  __shared__ double red[4];
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  double hr = 0.0;
  if (wave < nseg) {
    const Segment sg = segs[wave];
    const int count = __builtin_amdgcn_readfirstlane(sg.count);
    const int frame = __builtin_amdgcn_readfirstlane(sg.frame);
    if (lane < count) {
      const int64_t i = (int64_t)sg.begin + lane;
      const FrameDesc& F = fd[frame];
      const double* rec = frec + (int64_t)frame * kFrameRecDoubles;
      const double4 X = pts[obs_pid[i]];
      const double2 m = obs_meas[i];
      Proj o;
      project<MODEL, DEG>(rec, X.x, X.y, X.z, params[F.off[MVBA_BLK_FOCAL]], params[F.off[MVBA_BLK_CENTER]],
                          params[F.off[MVBA_BLK_CENTER] + 1], params + F.off[MVBA_BLK_DIST], F.K, F.h0, F.h1, o);
      loss_scale(o.d0 - m.x, o.d1 - m.y, flags, cauchy_c, &hr);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) hr += __shfl_xor(hr, off, 64);
  if (lane == 0) red[threadIdx.x >> 6] = hr;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace mvba

// ------------------------------------------------------------ launchers
#define MVBA_SOLVER_SWITCH(model, deg, CALL)                       \
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

extern "C" {

int mvba_solver_dir_stride(void) { return mvba::kDirStride; }
int mvba_solver_vec_replicas(void) { return mvba::kVecReplicas; }

// lz (nullable): x is the lazily formed CG direction, also stored to lz->p_new
hipError_t mvba_launch_frame_dir(const void* fl, int32_t nframes, const mvba::FrameDesc* fd, const double* frec,
                                 const double* x, double* dir, const int32_t* gate, const mvba::LazyDir* lz,
                                 hipStream_t s) {
  mvba::LazyDir l{};
  if (lz) l = *lz;
  const int64_t fblocks = std::max(nframes, 0), pblocks = lz ? (l.n + 63) / 64 : 0;
  if (fblocks + pblocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_frame_dir, dim3((unsigned)(fblocks + pblocks)), dim3(64), 0, s,
                     (const mvba::FrameLin*)fl, nframes, fd, frec, x, dir, gate, l);
  return hipGetLastError();
}

// model < 0: mixed camera models (runtime dispatch per observation).
// sq_partial/counter/sq_out: optional grid reduction of sum |u_o|^2 into sq_out[0].
hipError_t mvba_launch_pass_a(int model, int deg, const int64_t* pt_begin, int64_t npts, const int32_t* po_frame,
                              const double2* po_meas, const mvba::FrameDesc* fd, const double* frec,
                              const double* params, const double4* pts, const double* dir, const double* tinit,
                              const double* V, const double* dp, double* zbuf, double* wout, int32_t wstride,
                              double* sq_partial, unsigned* counter, double* sq_out, int32_t flags, double cauchy_c,
                              mvba::PointExtra dc, const double* xcam, double* du, const int32_t* gate,
                              const double* prec, hipStream_t s) {
  const unsigned blocks = (unsigned)((npts * mvba::kLanesA + 255) / 256);
  if (npts <= 0) return hipSuccess;
  const bool depth = dc.begin != nullptr, rows = sq_partial != nullptr;
#define MVBA_PA4(M, D, DP, RW)                                                                                 \
  hipLaunchKernelGGL((mvba::k_pass_a<M, D, DP, RW>), dim3(blocks), dim3(256), 0, s, pt_begin, npts, po_frame,   \
                     po_meas, fd, frec, params, pts, dir, tinit, V, dp, zbuf, wout, wstride, sq_partial, counter, \
                     sq_out, flags, cauchy_c, dc, xcam, du, gate, prec)
#define MVBA_PA(M, D)                    \
  if (depth) {                           \
    if (rows) MVBA_PA4(M, D, true, true);   \
    else MVBA_PA4(M, D, true, false);       \
  } else {                               \
    if (rows) MVBA_PA4(M, D, false, true);  \
    else MVBA_PA4(M, D, false, false);      \
  }
  if (model < 0) {
    MVBA_PA(-1, 0)
    return hipGetLastError();
  }
  MVBA_SOLVER_SWITCH(model, deg, MVBA_PA)
#undef MVBA_PA
#undef MVBA_PA4
  return hipGetLastError();
}

// Frame-order pass A (no depth blocks, no |u|^2 sweep) for one model group
hipError_t mvba_launch_pass_a_frame(int model, int deg, const int4* chunks, int32_t nchunks,
                                    const mvba::Segment* segs, const double4* pts, const int32_t* obs_pid,
                                    const double2* obs_meas, const int32_t* slot_po, mvba::DirPair dir,
                                    double4* cbuf, int32_t flags, double cauchy_c, const int32_t* gate,
                                    const double* prec, const double4* obsX, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
#define MVBA_PAF(M, D)                                                                                      \
  hipLaunchKernelGGL((mvba::k_pass_a_frame<M, D>), dim3(mvba::xcd_grid_solver((nchunks + mvba::kPassAWaves - 1) / \
                     mvba::kPassAWaves)), dim3(64 * mvba::kPassAWaves), 0, s, chunks, nchunks,                 \
                     segs, pts, obs_pid, obs_meas, slot_po, dir, cbuf, flags, cauchy_c, gate, prec, obsX)
  MVBA_SOLVER_SWITCH(model, deg, MVBA_PAF)
#undef MVBA_PAF
  return hipGetLastError();
}

hipError_t mvba_launch_pass_sq(int model, int deg, const int4* chunks, int32_t nchunks, const int32_t* obs_pid,
                               mvba::DirPair dir, const double* wbuf, int32_t wstride, const double* prec,
                               const double4* obsX, double* partial, unsigned* counter, double* sq_out,
                               hipStream_t s) {
  if (nchunks <= 0) return hipErrorInvalidValue;  // the grid sum needs a block
  // MVBA_SQ_GRID: the block cap (A/B timing)
  static const int64_t cap = std::getenv("MVBA_SQ_GRID") ? std::atoll(std::getenv("MVBA_SQ_GRID")) : 1024;
  const unsigned grid =
      mvba::xcd_grid_solver(std::min<int64_t>((nchunks + mvba::kPassAWaves - 1) / mvba::kPassAWaves, cap));
#define MVBA_PSQ(M, D)                                                                                      \
  hipLaunchKernelGGL((mvba::k_pass_sq<M, D>), dim3(grid), dim3(64 * mvba::kPassAWaves), 0, s, chunks, nchunks,    \
                     obs_pid, dir, wbuf, wstride, prec, obsX, partial, counter, sq_out)
  MVBA_SOLVER_SWITCH(model, deg, MVBA_PSQ)
#undef MVBA_PSQ
  return hipGetLastError();
}

// fs (nullable): the fused CG step's combination (mvba::FusedStep), with one
// frame wave per frame after the point blocks
hipError_t mvba_launch_point_w(int64_t npts, const int64_t* pt_begin, const int32_t* po_slot, const double4* cbuf,
                               const double* tinit, const double* V, const double* dp, const double4* pts,
                               double* wout, int32_t wstride, const int32_t* gate, const int64_t* dbegin,
                               const double4* dcbuf, const mvba::FusedStep* fs, hipStream_t s) {
  mvba::FusedStep f{};
  const unsigned pb = npts > 0 ? mvba::xcd_grid_solver((npts * mvba::kLanesW + 255) / 256) : 0u;
  unsigned fb = 0;
  if (fs && fs->dz) {
    f = *fs;
    f.point_blocks = (int32_t)pb;
    fb = (unsigned)((fs->nframes + 3) / 4);  // 4 frame waves per 256-thread block
  }
  if (pb + fb == 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_point_w, dim3(pb + fb), dim3(256), 0, s, npts, pt_begin, po_slot, cbuf, tinit, V, dp, pts,
                     wout, wstride, gate, dbegin, dcbuf, f);
  return hipGetLastError();
}

// The fused CG step (k_upd_pass_a): the update of the previous iteration (mode
// 1|2|8, n camera entries) and this iteration's pass A in one launch.
hipError_t mvba_launch_upd_pass_a(int model, int deg, int64_t n, const mvba::CgEntry* ent, const double* minv,
                                  const double* p, const double* q, const double* b, double* x, const double* r_in,
                                  double* r_out, double* z, double* partial, unsigned* counters, double* out,
                                  mvba::CgCtl* ctl, const double* pq_in, const int4* chunks, int32_t nchunks,
                                  const void* fl, const mvba::FrameDesc* fd, const double* frec, const double* dp,
                                  double* dz_out, const int32_t* slot_po, double4* cbuf, double* cbuf2,
                                  const double* prec, const double4* obsX, hipStream_t s) {
  if (n <= 0 || !obsX || !ctl) return hipErrorInvalidValue;
  // entry blocks rounded up to a multiple of 8: the pass-A blocks after them keep
  // k_pass_a_frame's XCD mapping
  const unsigned eb = (unsigned)(((n + 255) / 256 + 7) / 8 * 8);
  const unsigned ab = nchunks > 0 ? mvba::xcd_grid_solver((nchunks + mvba::kPassAWaves - 1) / mvba::kPassAWaves) : 0u;
#define MVBA_UPA(M, D)                                                                                        \
  hipLaunchKernelGGL((mvba::k_upd_pass_a<M, D>), dim3(eb + ab), dim3(64 * mvba::kPassAWaves), 0, s, n, ent, minv, p, \
                     q, b, x, r_in, r_out, z, partial, counters, out, ctl, pq_in, (int32_t)eb, chunks, nchunks,   \
                     (const mvba::FrameLin*)fl, fd, frec, dp, dz_out, slot_po, cbuf, (double2*)cbuf2, prec, obsX)
  MVBA_SOLVER_SWITCH(model, deg, MVBA_UPA)
#undef MVBA_UPA
  return hipGetLastError();
}

hipError_t mvba_launch_point_w_seg(int32_t ntiles, const int4* tiles, const int32_t* wlane_pid,
                                   const int32_t* wlane_idx, const int64_t* pt_begin, const int32_t* po_idx,
                                   const double4* cbuf, const double* tinit, const double* V, const double* dp,
                                   const double4* pts, double* wout, int32_t wstride, const int32_t* gate,
                                   hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_point_w_seg, dim3(mvba::xcd_grid_solver((ntiles + 3) / 4)), dim3(256), 0, s, ntiles,
                     tiles, wlane_pid, wlane_idx, pt_begin, po_idx, cbuf, tinit, V, dp, pts, wout, wstride, gate);
  return hipGetLastError();
}

hipError_t mvba_launch_depth_pa(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                const int32_t* dpid, const double4* dmeas, const double* frec, const double* params,
                                const double4* pts, const double* dir, const double* xcam, double* du,
                                const int32_t* dslot_po, double4* dcbuf, int32_t flags, double cauchy_c,
                                const int32_t* gate, hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_depth_pa, dim3((unsigned)nseg), dim3(64), 0, s, segs, nseg, dd, dpid, dmeas, frec, params,
                     pts, dir, xcam, du, dslot_po, dcbuf, flags, cauchy_c, gate);
  return hipGetLastError();
}

hipError_t mvba_launch_frame_proj(int32_t nframes, const mvba::FrameDesc* fd, const double* frec,
                                  const double* params, double* prec, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  const int64_t n = (int64_t)nframes * mvba::kProjDoubles;
  hipLaunchKernelGGL(mvba::k_frame_proj, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, nframes, fd, frec,
                     params, prec);
  return hipGetLastError();
}

int64_t mvba_pass_a_blocks(int64_t npts) { return (npts * mvba::kLanesA + 255) / 256; }

hipError_t mvba_launch_pass_b(int model, int deg, const int4* chunks, int32_t nchunks, int32_t chunk_base,
                              const mvba::Segment* segs, const mvba::FrameDesc* fd, const void* fl,
                              const double* frec, const double* params, const double4* pts, const int32_t* obs_pid,
                              const double2* obs_meas, const double* dir, const double4* wbuf, double* yrep,
                              int64_t ng, int32_t flags, double cauchy_c, const int32_t* gate, mvba::Slab sl,
                              const double4* obsX, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  // two waves per chunk for the register-accumulator models other than RPC
  // (latency-bound pass B: more waves to cover the gathers, one reduction);
  // RPC (VALU-bound at c3) and the wide rows keep one. MVBA_PASSB_WAVES=1|2
  // (read per call) forces it for the non-RPC models (A/B timing).
  const char* pw = std::getenv("MVBA_PASSB_WAVES");
  const unsigned pb_threads = (model != mvba::kModelRpc && !(pw && pw[0] == '1')) ? 128u : 64u;
#define MVBA_PB(M, D)                                                                                       \
  hipLaunchKernelGGL((mvba::k_pass_b<M, D>), dim3(mvba::xcd_grid_solver(nchunks)),                            \
                     dim3(M == mvba::kModelRpc ? 64u : pb_threads),                                           \
                     (mvba::pass_b_lds<M, D>()), s,                                                           \
                     chunks, nchunks,                                                                         \
                     chunk_base, segs, fd, (const mvba::FrameLin*)fl, frec, params, pts, obs_pid, obs_meas,     \
                     dir, wbuf, yrep, ng, flags, cauchy_c, gate, sl, obsX)
  MVBA_SOLVER_SWITCH(model, deg, MVBA_PB)
#undef MVBA_PB
  return hipGetLastError();
}

// y = sum of replicas (+ diag .* x, and x.y -> dot_out when dot_out != null)
hipError_t mvba_launch_slab_reduce_vec(mvba::SlabTiers t, int64_t grid, const int64_t* begin, const int64_t* pos,
                                       const double* val, const double* diag, const double* x, double* y,
                                       double* partial, unsigned* counter, double* dot_out, const int32_t* gate,
                                       mvba::CgCtl* ctl, const mvba::LazyDir* lz, int32_t local_dot, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  const mvba::LazyDir l = lz ? *lz : mvba::LazyDir{};
  hipLaunchKernelGGL(mvba::k_vec_slab_reduce, dim3((unsigned)grid), dim3(256), 0, s, t, begin, pos, val, diag, x, y,
                     partial, counter, dot_out, gate, ctl, l, local_dot);
  return hipGetLastError();
}

hipError_t mvba_launch_rep_reduce_vec(double* yrep, int64_t ng, const double* diag, const double* x, double* y,
                                      double* partial, unsigned* counter, double* dot_out, const int32_t* gate,
                                      mvba::CgCtl* ctl, const mvba::LazyDir* lz, int32_t local_dot,
                                      double* dot_zero, hipStream_t s) {
  if (ng <= 0) return hipSuccess;
  if (local_dot == 2 && (!dot_out || !dot_zero || !ctl)) return hipErrorInvalidValue;
  const mvba::LazyDir l = lz ? *lz : mvba::LazyDir{};
  // threads per block (MVBA_REP_THREADS=64|128|256, read per call; A/B timing):
  // smaller blocks spread the replica reads (32 per entry) over more CUs
  const char* te = std::getenv("MVBA_REP_THREADS");
  const int nt = te ? std::atoi(te) : 256;
  const unsigned threads = nt == 64 || nt == 128 ? (unsigned)nt : 256u;
  hipLaunchKernelGGL(mvba::k_vec_rep_reduce, dim3((unsigned)((ng + threads - 1) / threads)), dim3(threads), 0, s, yrep,
                     ng, diag, x, y, partial, counter, dot_out, gate, ctl, l, local_dot, dot_zero);
  return hipGetLastError();
}

hipError_t mvba_launch_add_diag(int64_t n, const double* diag, const double* x, double* y, double* partial,
                                unsigned* counter, double* dot_out, const int32_t* gate, mvba::CgCtl* ctl,
                                const mvba::LazyDir* lz, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const mvba::LazyDir l = lz ? *lz : mvba::LazyDir{};
  hipLaunchKernelGGL(mvba::k_add_diag, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, diag, x, y, partial,
                     counter, dot_out, gate, ctl, l);
  return hipGetLastError();
}

// partial needs 3 x ceil(n / 256) doubles, counters 3 (zero-initialised, re-armed by the kernel)
hipError_t mvba_launch_cg_update(int64_t n, const mvba::CgEntry* ent, const double* minv, int32_t mode, double alpha,
                                 const double* p,
                                 const double* q, const double* b, double* x, const double* r_in, double* r_out,
                                 double* z, double* partial, unsigned* counters, double* out, mvba::CgCtl* ctl,
                                 int32_t iter, const mvba::FrameDirZ* fz, const double* pq_in, mvba::CgMirror* mir,
                                 hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  mvba::FrameDirZ f{};
  unsigned fblocks = 0;
  if (fz && fz->dz && (mode & 8) && fz->nframes > 0) {
    f = *fz;
    f.owner_blocks = (int32_t)blocks;
    fblocks = (unsigned)((fz->nframes + 3) / 4);  // 4 frame waves per 256-thread block
  }
  hipLaunchKernelGGL(mvba::k_cg_update, dim3(blocks + fblocks), dim3(256), 0, s, n, ent, minv, mode, alpha,
                     p, q, b, x, r_in, r_out, z, partial, counters, out, ctl, iter, f, pq_in, mir);
  return hipGetLastError();
}

hipError_t mvba_launch_axpby(int64_t n, double a, const double* x, double b, const double* y, double* out,
                             hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_axpby, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, a, x, b, y, out);
  return hipGetLastError();
}

// dot(x, y) -> out (device scalar) via partials[<= 2048] and a counter (zero,
// re-armed). Blocks: about 4 elements per thread, at most 2048 (the round-4
// fixed 256 blocks left one wave per SIMD: c3's 3M-entry point-side dots took
// 14.6 us each, profiles/r05/r05k/)
hipError_t mvba_launch_dot(int64_t n, const double* x, const double* y, double* partial, unsigned* counter,
                           double* out, hipStream_t s) {
  const int64_t want = (n + 1023) / 1024;
  const int blocks = (int)(want < 1 ? 1 : want > 2048 ? 2048 : want);
  hipLaunchKernelGGL(mvba::k_dot_fin, dim3(blocks), dim3(256), 0, s, n, x, y, partial, counter, out);
  return hipGetLastError();
}

// out[0] = sum partial[0..n) in a fixed order; past 4096 partials in two levels
// (blocks of n / 1024+ partials into partial[n ..], then one block): the
// partial array must hold n + 1024 entries. One block over c3's 39k cost
// partials took 40.7 us (profiles/r05/r05k/).
hipError_t mvba_launch_sum(int64_t n, double* partial, double* out, hipStream_t s) {
  if (n <= 4096) {
    hipLaunchKernelGGL(mvba::k_sum, dim3(1), dim3(256), 0, s, n, partial, out);
    return hipGetLastError();
  }
  const int64_t nb2 = std::min<int64_t>(1024, (n + 4095) / 4096);
  const int64_t per = (n + nb2 - 1) / nb2;
  hipLaunchKernelGGL(mvba::k_sum_level, dim3((unsigned)nb2), dim3(256), 0, s, n, per, partial, partial + n);
  hipLaunchKernelGGL(mvba::k_sum, dim3(1), dim3(256), 0, s, nb2, partial + n, out);
  return hipGetLastError();
}

hipError_t mvba_launch_block_prec(int32_t nblocks, int32_t max_bsize, const int64_t* goff, const int64_t* hoff,
                                  const int32_t* bsize, const double* hess, const double* d, double* minv,
                                  hipStream_t s) {
  if (nblocks <= 0) return hipSuccess;
  // MVBA_PREC_SMALL=0: every block by the workgroup form (A/B timing)
  static const bool small = !(std::getenv("MVBA_PREC_SMALL") && std::getenv("MVBA_PREC_SMALL")[0] == '0');
  if (small) {
    hipLaunchKernelGGL(mvba::k_block_prec_small, dim3((unsigned)((nblocks + 3) / 4)), dim3(256), 0, s, nblocks, goff,
                       hoff, bsize, hess, d, minv);
    if (max_bsize <= mvba::kPrecSmall) return hipGetLastError();
  }
  const int m = max_bsize < mvba::kPrecLds ? max_bsize : mvba::kPrecLds;
  const size_t lds = sizeof(double) * (size_t)(m * m + 2 * m > 2 * max_bsize ? m * m + 2 * m : 2 * max_bsize);
  hipLaunchKernelGGL(mvba::k_block_prec, dim3((unsigned)nblocks), dim3(mvba::kPrecThreads), lds, s, nblocks, goff,
                     hoff, bsize, hess,
                     d, minv, small ? 1 : 0);
  return hipGetLastError();
}

static inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t mvba_launch_extract_diag(int32_t nblocks, const int64_t* goff, const int64_t* hoff, const int32_t* bsize,
                                    const double* hess, int64_t npts, const double* V, int64_t ng, double* c,
                                    hipStream_t s) {
  const int64_t n = nblocks + npts;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_extract_diag, grid1(n), dim3(256), 0, s, nblocks, goff, hoff, bsize, hess, npts, V,
                     ng, c);
  return hipGetLastError();
}

hipError_t mvba_launch_jacobi_scale(int64_t n, const double* c, double* sc, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_jacobi_scale, grid1(n), dim3(256), 0, s, n, c, sc);
  return hipGetLastError();
}

hipError_t mvba_launch_lm_diag(int64_t n, const double* c, const double* sc, double inv_radius,
                               const double* inv_radius_dev, double dmin, double dmax, double* d, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_lm_diag, grid1(n), dim3(256), 0, s, n, c, sc, inv_radius, inv_radius_dev, dmin, dmax,
                     d);
  return hipGetLastError();
}

hipError_t mvba_launch_gather(int64_t ncam, const int64_t* cam_poff, int64_t npts, const int64_t* pt_off,
                              const uint8_t* pt_free, const double* params, double* out, hipStream_t s) {
  const int64_t n = ncam + 3 * npts;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_gather, grid1(n), dim3(256), 0, s, ncam, cam_poff, npts, pt_off, pt_free, params, out);
  return hipGetLastError();
}

hipError_t mvba_launch_scatter(int64_t ncam, const int64_t* cam_poff, int64_t npts, const int64_t* pt_off,
                               const uint8_t* pt_free, const double* in, double* params, hipStream_t s) {
  const int64_t n = ncam + 3 * npts;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_scatter, grid1(n), dim3(256), 0, s, ncam, cam_poff, npts, pt_off, pt_free, in, params);
  return hipGetLastError();
}

hipError_t mvba_launch_plus(int64_t n, const double* x, const double* delta, const double* lower,
                            const double* upper, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_plus, grid1(n), dim3(256), 0, s, n, x, delta, lower, upper, out);
  return hipGetLastError();
}

hipError_t mvba_launch_proj_grad_max(int64_t n, const double* x, const double* g, const double* lower,
                                     const double* upper, double* partial, double* out, hipStream_t s) {
  const int64_t want = (n + 1023) / 1024;
  const int blocks = (int)(want < 1 ? 1 : want > 2048 ? 2048 : want);
  hipLaunchKernelGGL(mvba::k_proj_grad_max, dim3(blocks), dim3(256), 0, s, n, x, g, lower, upper, partial);
  hipLaunchKernelGGL(mvba::k_max, dim3(1), dim3(256), 0, s, (int64_t)blocks, partial, out);
  return hipGetLastError();
}

hipError_t mvba_launch_cost(int model, int deg, const mvba::Segment* segs, int32_t nseg, const mvba::FrameDesc* fd,
                            const double* frec, const double* params, const double4* pts, const int32_t* obs_pid,
                            const double2* obs_meas, int32_t flags, double cauchy_c, double* partial, hipStream_t s,
                            int64_t* nblocks_out) {
  const unsigned blocks = (unsigned)((nseg + 3) / 4);
  if (nblocks_out) *nblocks_out = blocks;
  if (nseg <= 0) return hipSuccess;
#define MVBA_CO(M, D)                                                                                       \
  hipLaunchKernelGGL((mvba::k_cost<M, D>), dim3(blocks), dim3(256), 0, s, segs, nseg, fd, frec, params, pts, \
                     obs_pid, obs_meas, flags, cauchy_c, partial)
  MVBA_SOLVER_SWITCH(model, deg, MVBA_CO)
#undef MVBA_CO
  return hipGetLastError();
}

}  // extern "C"
