// mvba_depth.hip — BracketedDepthError residual blocks on gfx950
// (rig_calibrator.cc:522-609, added at :1755-1791 when --depth_tri_weight > 0).
//
//   M  = (depth_to_image with linear *= scale) * meas_depth_xyz     (:558-569)
//   Mw = world_to_cam.inverse() * M                                 (:572)
//   r  = weight * (X - Mw)                                          (:578-580)
//
// world_to_cam is the K0 frame record of the image the depth cloud belongs to
// (same beg/end/ref_to_cam/offset blocks and stamps), so the pose columns reuse
// the frame's generators: with Mw = R^-1 (M - t) and dXc/dp_k = w_k x Xc + v_k,
//   dr_i/dp_k = weight * [ M x Rinv_i ; Rinv_i ] . [w_k ; v_k]
// depth_to_image / scale columns: dr/dtheta = -weight Rinv dM/dtheta; xyz: weight I.
// Device order: depth blocks sorted by frame, line-aligned frame ranges, segments
// of <= 64 blocks of one frame (one wave each), like the reprojection blocks.
#include "mvba_depth.h"

namespace mvba {

constexpr int kDJacBase[7] = {MVBA_DJAC_BASE_BEG, MVBA_DJAC_BASE_END, MVBA_DJAC_BASE_REF_TO_CAM,
                              MVBA_DJAC_BASE_DEPTH_TO_IMAGE, MVBA_DJAC_BASE_SCALE, MVBA_DJAC_BASE_XYZ,
                              MVBA_DJAC_BASE_OFFSET};

// ------------------------------------------------------------ evaluation (K1-depth)
// One lane per depth block, one wave per segment. res[3][ld], J[MVBA_DJAC_ROWS][ld]
// column planes; constant blocks are not written. flags & APPLY_LOSS applies the
// corrector in-kernel.
// OT: double (fp64 output) or float (fp32 output of the same fp64 arithmetic).
// A segment's blocks share one image: their descriptors differ only in the
// point (and its free bit, the point record's w), so the descriptor is read once
// per wave (scalar loads) and the point index per lane from the dense dpid array
// (4 B per block instead of a 64-B descriptor); blocks in XCD-contiguous order.
template <class OT>
__global__ void __launch_bounds__(64) k_depth_obs(const Segment* __restrict__ segs, int32_t nseg,
                                                  const DepthDesc* __restrict__ dd, const int32_t* __restrict__ dpid,
                                                  const double4* __restrict__ dmeas,
                                                  const FrameDesc* __restrict__ fd, const double* __restrict__ frec,
                                                  const double* __restrict__ params, const double4* __restrict__ pts,
                                                  OT* __restrict__ res, OT* __restrict__ J, int64_t ld,
                                                  int32_t flags, double cauchy_c) {
  const int64_t seg = xcd_block(nseg);
  if (seg < 0) return;
  const Segment sg = segs[seg];
  const int lane = threadIdx.x;
  // padding lanes up to the next 128-B line of OT recompute the last block
  // into their padding slots (whole-line stores, as in k_obs)
  constexpr int kLine = 128 / (int)sizeof(OT);
  const int count = __builtin_amdgcn_readfirstlane(sg.count);
  const int begin = __builtin_amdgcn_readfirstlane(sg.begin);
  if (lane >= ((count + kLine - 1) & ~(kLine - 1))) return;
  const int64_t i = (int64_t)begin + lane;
  const int64_t isrc = (int64_t)begin + min(lane, count - 1);
  DepthDesc d = dd[begin];
  d.pid = dpid[isrc];
  const double* rec = frec + (int64_t)d.frame * kFrameRecDoubles;
  const double4 X = pts[d.pid];
  d.free_mask = (d.free_mask & ~(1 << MVBA_DBLK_XYZ)) | (X.w != 0.0 ? (1 << MVBA_DBLK_XYZ) : 0);
  DepthRows o;
  depth_rows(d, rec, params, dmeas[isrc], X.x, X.y, X.z, flags, cauchy_c, o);
  const bool loss = (flags & MVBA_EVAL_APPLY_LOSS) != 0;
  if (res) {
#pragma unroll
    for (int q = 0; q < 3; q++) __builtin_nontemporal_store((OT)(loss ? o.r[q] : o.rr[q]), &res[q * ld + i]);
  }
  if (!J) return;
  // raw (uncorrected) Jacobian unless APPLY_LOSS: divide the corrected rows back
  const double un = loss ? 1.0 : 1.0 / o.sr;
  const int mask = d.free_mask;
  const double* wv = rec + 12;
#pragma unroll
  for (int blk = 0; blk < 4; blk++) {
    const int db = (blk == 3) ? MVBA_DBLK_OFFSET : blk;
    const int ncol = (blk == 3) ? 1 : 7, k0 = blk * 7;
    if (!(mask & (1 << db))) continue;
#pragma unroll
    for (int c = 0; c < 7; c++) {
      if (c >= ncol) break;
      const double* wk = wv + 6 * (k0 + c);
#pragma unroll
      for (int i3 = 0; i3 < 3; i3++) {
        double v = 0.0;
#pragma unroll
        for (int a = 0; a < 6; a++) v += o.Z[i3][a] * wk[a];
        __builtin_nontemporal_store((OT)(v * un), &J[(int64_t)(kDJacBase[db] + i3 * ncol + c) * ld + i]);
      }
    }
  }
  if (mask & (1 << MVBA_DBLK_DEPTH_TO_IMAGE)) {
    const int n = d.dti_n;
#pragma unroll
    for (int i3 = 0; i3 < 3; i3++)
#pragma unroll
      for (int c = 0; c < 12; c++)
        if (c < n)
          __builtin_nontemporal_store((OT)(o.D[i3][c] * un),
                                      &J[(int64_t)(MVBA_DJAC_BASE_DEPTH_TO_IMAGE + i3 * n + c) * ld + i]);
  }
  if (mask & (1 << MVBA_DBLK_SCALE))
#pragma unroll
    for (int i3 = 0; i3 < 3; i3++)
      __builtin_nontemporal_store((OT)(o.S[i3] * un), &J[(int64_t)(MVBA_DJAC_BASE_SCALE + i3) * ld + i]);
  if (mask & (1 << MVBA_DBLK_XYZ))
#pragma unroll
    for (int i3 = 0; i3 < 3; i3++)
#pragma unroll
      for (int c = 0; c < 3; c++)
        __builtin_nontemporal_store((OT)(i3 == c ? o.P * un : 0.0), &J[(int64_t)(MVBA_DJAC_BASE_XYZ + i3 * 3 + c) * ld + i]);
}

// ------------------------------------------------------------ normal equations
// One wave per segment: Gram of B = [Z (6) | D (12) | S | r] over its 3*64 rows
// with fp64 MFMA (rows staged in LDS [column][row]), then the wave expands it:
// pose blocks through the frame's generators, depth_to_image and scale blocks
// directly, into replica (segment mod 32) of [cam_grad | cam_hess | cost].
constexpr int kDW = 20;          // Gram width
constexpr int kDT = 2;           // 16-wide tiles
constexpr int kDRows = 192;      // 3 rows x 64 lanes
// rows are staged 64 at a time (three passes; the MFMA order is the row order
// either way): 17 KB of LDS per wave instead of 50, 2.7x the waves per CU
constexpr int kDStage = 64;
constexpr int kDLd = kDStage + 2; // LDS leading dimension (doubles)
constexpr int kDReplicas = kDepthReplicas;

__global__ void __launch_bounds__(64) k_depth_gram(const Segment* __restrict__ segs, int32_t nseg,
                                                   const DepthDesc* __restrict__ dd, const int32_t* __restrict__ dpid,
                                                   const double4* __restrict__ dmeas, const double* __restrict__ frec,
                                                   const double* __restrict__ params,
                                                   const double4* __restrict__ pts, const FrameLin* __restrict__ fl,
                                                   double* __restrict__ rep, int64_t ng, int64_t nh, int32_t flags,
                                                   double cauchy_c, Slab sl) {
  __shared__ double lds[kDT * 16 * kDLd];
  __shared__ double G[kDW * kDW];
  const int seg = blockIdx.x;
  if (seg >= nseg) return;
  const Segment sg = segs[seg];
  const int lane = threadIdx.x;
  const int frame = __builtin_amdgcn_readfirstlane(sg.frame);
  const double* rec = frec + (int64_t)frame * kFrameRecDoubles;
  double cost = 0.0;
  double row[3][kDW];
#pragma unroll
  for (int i3 = 0; i3 < 3; i3++)
#pragma unroll
    for (int q = 0; q < kDW; q++) row[i3][q] = 0.0;
  DepthDesc d0 = dd[sg.begin];
  if (lane < sg.count) {
    const int64_t i = (int64_t)sg.begin + lane;
    DepthDesc d = d0;  // one image per segment: only the point differs (as k_depth_obs)
    d.pid = dpid[i];
    const double4 X = pts[d.pid];
    DepthRows o;
    depth_rows(d, rec, params, dmeas[i], X.x, X.y, X.z, flags, cauchy_c, o);
    cost = o.half_rho;
#pragma unroll
    for (int i3 = 0; i3 < 3; i3++) {
#pragma unroll
      for (int a = 0; a < 6; a++) row[i3][a] = o.Z[i3][a];
#pragma unroll
      for (int q = 0; q < 12; q++) row[i3][6 + q] = o.D[i3][q];
      row[i3][18] = o.S[i3];
      row[i3][19] = o.r[i3];
    }
  }
  // stage [column][row] (row 3 lane + i3), 64 rows per pass; padding columns
  // 20..31 zero; passes past the segment's last block are all zero rows
  dbl4 acc[3] = {dbl4{0, 0, 0, 0}, dbl4{0, 0, 0, 0}, dbl4{0, 0, 0, 0}};
  const int col = lane & 15, rsub = lane >> 4;
  const int count = __builtin_amdgcn_readfirstlane(sg.count);
  for (int pass = 0; pass < kDRows / kDStage && pass * kDStage < 3 * count; pass++) {
#pragma unroll
    for (int i3 = 0; i3 < 3; i3++) {
      const int r = 3 * lane + i3 - pass * kDStage;
      if (r >= 0 && r < kDStage) {
#pragma unroll
        for (int q = 0; q < kDT * 16; q++) lds[q * kDLd + r] = q < kDW ? row[i3][q] : 0.0;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int st = 0; st < kDStage / 4; st++) {
      const int r = 4 * st + rsub;
      const double v0 = lds[col * kDLd + r], v1 = lds[(16 + col) * kDLd + r];
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, v0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, v1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(v1, v1, acc[2], 0, 0, 0);
    }
    __syncthreads();
  }
  // lane holds G[(lane>>4) + 4r][lane & 15] of tile pairs (0,0), (0,1), (1,1)
  const int pairs[3][2] = {{0, 0}, {0, 1}, {1, 1}};
#pragma unroll
  for (int pidx = 0; pidx < 3; pidx++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int a = pairs[pidx][0] * 16 + (lane >> 4) + 4 * r, b = pairs[pidx][1] * 16 + (lane & 15);
      if (a < kDW && b < kDW) {
        G[a * kDW + b] = acc[pidx][r];
        G[b * kDW + a] = acc[pidx][r];
      }
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cost += __shfl_xor(cost, off, 64);
  __syncthreads();
  // expand (frame-uniform blocks)
  const FrameLin& L = fl[frame];
  double* grad = rep + (int64_t)(seg & (kDReplicas - 1)) * (ng + nh + 1);
  const double* wv = rec + 12;
  for (int blk = 0; blk < 4; blk++) {
    const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
    if (L.goff[b] < 0) continue;
    const int ncol = (blk == 3) ? 1 : 7, k0 = blk * 7;
    for (int e = lane; e < ncol; e += 64) {
      const double* wk = wv + 6 * (k0 + e);
      double g = 0.0;
      for (int a = 0; a < 6; a++) g += wk[a] * G[a * kDW + 19];
      accumulate(grad, L.goff[b] + e, g, sl, seg, 56 * blk + e);
    }
    for (int e = lane; e < ncol * ncol; e += 64) {
      const int kk = e / ncol, kc = e % ncol;
      const double* wa = wv + 6 * (k0 + kk);
      const double* wb = wv + 6 * (k0 + kc);
      double h = 0.0;
      for (int a = 0; a < 6; a++) {
        double t = 0.0;
        for (int c = 0; c < 6; c++) t += G[a * kDW + c] * wb[c];
        h += wa[a] * t;
      }
      accumulate(grad, ng + L.hoff[b] + e, h, sl, seg, 56 * blk + ncol + e);
    }
  }
  // depth_to_image and scale: sensor blocks, the same for the whole segment
  // (one image = one sensor), so take them from the first block's record.
  if (d0.goff_dti >= 0) {
    const int n = d0.dti_n;
    for (int e = lane; e < n; e += 64) accumulate(grad, d0.goff_dti + e, G[(6 + e) * kDW + 19], sl, seg, kSlabDti + e);
    for (int e = lane; e < n * n; e += 64) {
      const int a = e / n, c = e % n;
      accumulate(grad, ng + d0.hoff_dti + e, G[(6 + a) * kDW + 6 + c], sl, seg, kSlabDtiHess + e);
    }
  }
  if (d0.goff_scale >= 0 && lane == 0) {
    accumulate(grad, d0.goff_scale, G[18 * kDW + 19], sl, seg, kSlabScale);
    accumulate(grad, ng + d0.hoff_scale, G[18 * kDW + 18], sl, seg, kSlabScale + 1);
  }
  if (lane == 0) accumulate(grad, ng + nh, cost, sl, seg, (int)(sl.width - 1));
}

// Cost partials (sum 0.5 rho) per 256-thread block over the depth slots.
__global__ void __launch_bounds__(256) k_depth_cost(int64_t nslots, const DepthDesc* __restrict__ dd,
                                                    const int64_t* __restrict__ dorder,
                                                    const double4* __restrict__ dmeas,
                                                    const double* __restrict__ frec,
                                                    const double* __restrict__ params,
                                                    const double4* __restrict__ pts, int32_t flags, double cauchy_c,
                                                    double* __restrict__ partial) {
  __shared__ double red[256];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double c = 0.0;
  if (i < nslots && dorder[i] >= 0) {
    const DepthDesc d = dd[i];
    const double4 X = pts[d.pid];
    DepthRows o;
    depth_rows(d, frec + (int64_t)d.frame * kFrameRecDoubles, params, dmeas[i], X.x, X.y, X.z, flags, cauchy_c,
               o);
    c = o.half_rho;
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// ------------------------------------------------------------ solver pass
// Depth blocks in the implicit Schur product after pass A (which computed, in
// point order, u_d = J_cam,d x - P w_p for every depth block into du):
// y += J_cam,d^T u_d, wave-reduced per segment, mapped through the generators,
// added into replica (segment mod 32) of the camera-side vector.
__global__ void __launch_bounds__(64) k_depth_sb(const Segment* __restrict__ segs, int32_t nseg,
                                                 const DepthDesc* __restrict__ dd, const int32_t* __restrict__ dpid,
                                                 const double4* __restrict__ dmeas,
                                                 const double* __restrict__ frec, const double* __restrict__ params,
                                                 const double4* __restrict__ pts, const FrameLin* __restrict__ fl,
                                                 const double* __restrict__ du, double* __restrict__ yrep, int64_t ng,
                                                 int32_t flags, double cauchy_c, const int32_t* __restrict__ gate,
                                                 Slab sl, const double4* __restrict__ wbuf) {
  if (gate && *gate) return;
  constexpr int NA = 6 + 12 + 1;
  const int seg = blockIdx.x;
  const Segment sg = segs[seg];
  const int lane = threadIdx.x;
  const int frame = __builtin_amdgcn_readfirstlane(sg.frame);
  const double* rec = frec + (int64_t)frame * kFrameRecDoubles;
  double acc[NA];
#pragma unroll
  for (int q = 0; q < NA; q++) acc[q] = 0.0;
  const DepthDesc d0 = dd[sg.begin];
  if (lane < sg.count) {
    const int64_t i = (int64_t)sg.begin + lane;
    DepthDesc d = d0;  // one image per segment: only the point differs
    d.pid = dpid[i];
    const double4 X = pts[d.pid];
    const double4 m = dmeas[i];
    DepthCore c;
    depth_core(d, rec, params, m, X.x, X.y, X.z, flags, cauchy_c, c);
    // du: u_d (point-order pass A), or z_d with wbuf (frame-order k_depth_pa): u_d = z_d - P w_p
    double u[3] = {du[3 * i], du[3 * i + 1], du[3 * i + 2]};
    if (wbuf) {
      const double4 w = wbuf[d.pid];
      u[0] -= c.P * w.x;
      u[1] -= c.P * w.y;
      u[2] -= c.P * w.z;
    }
    depth_jtu(c, m, u, acc, acc + 6, acc + 18);
  }
  {
#pragma unroll
    for (int q = 0; q < NA; q++) acc[q] = wave_sum_f64(acc[q]);
    const FrameLin& L = fl[frame];
    double* y = yrep + (int64_t)(seg & (kDReplicas - 1)) * ng;
    int64_t dst = -1;
    double v = 0.0;
    if (lane < kPoseCols) {
      const int blk = lane / 7;
      const int b = (blk == 3) ? MVBA_BLK_OFFSET : blk;
      if (L.goff[b] >= 0) {
        const double* wk = rec + 12 + 6 * lane;
#pragma unroll
        for (int a = 0; a < 6; a++) v += wk[a] * acc[a];
        dst = L.goff[b] + (lane - 7 * blk);
      }
    } else if (lane < kPoseCols + 12) {
      const int q = lane - kPoseCols;
      if (d0.goff_dti >= 0 && q < d0.dti_n) {
#pragma unroll
        for (int e = 0; e < 12; e++)
          if (e == q) v = acc[6 + e];
        dst = d0.goff_dti + q;
      }
    } else if (lane == kPoseCols + 12 && d0.goff_scale >= 0) {
      v = acc[18];
      dst = d0.goff_scale;
    }
    if (dst >= 0) accumulate(y, dst, v, sl, seg, lane);
  }
}

// ------------------------------------------------------------ XYZError priors
// r = weight (X - ref) (rig_calibrator.cc:720-724), own Cauchy threshold.
// Cost (sum 0.5 rho) over the entries, grid-reduced into out[0].
__global__ void __launch_bounds__(256) k_xyz_cost(int64_t n, const int32_t* __restrict__ xpid,
                                                  const double4* __restrict__ xref, const double* __restrict__ xcc,
                                                  const double4* __restrict__ pts, int32_t flags,
                                                  double* __restrict__ partial, unsigned* __restrict__ counter,
                                                  double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double c = 0.0;
  if (j < n) {
    const double4 X = pts[xpid[j]];
    const double4 R = xref[j];
    double hr;
    loss_scale3(R.w * (X.x - R.x), R.w * (X.y - R.y), R.w * (X.z - R.z), flags, xcc[j], &hr);
    c = hr;
  }
  grid_sum_finalize(c, partial, counter, out);
}

// raw residuals into out[3 * insertion index]
__global__ void k_xyz_eval(int64_t n, const int32_t* __restrict__ xpid, const int64_t* __restrict__ xorder,
                           const double4* __restrict__ xref, const double4* __restrict__ pts,
                           double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double4 X = pts[xpid[j]];
  const double4 R = xref[j];
  const int64_t o = xorder[j];
  out[3 * o] = R.w * (X.x - R.x);
  out[3 * o + 1] = R.w * (X.y - R.y);
  out[3 * o + 2] = R.w * (X.z - R.z);
}

}  // namespace mvba

extern "C" {

size_t mvba_depth_desc_size(void) { return sizeof(mvba::DepthDesc); }

hipError_t mvba_launch_depth_obs(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                 const int32_t* dpid, const double4* dmeas, const mvba::FrameDesc* fd,
                                 const double* frec, const double* params, const double4* pts, void* res, void* J,
                                 int64_t ld, int32_t flags, double cauchy_c, int32_t out_f32, hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  const unsigned grid = mvba::xcd_grid(nseg);
  if (out_f32)
    hipLaunchKernelGGL(mvba::k_depth_obs<float>, dim3(grid), dim3(64), 0, s, segs, nseg, dd, dpid, dmeas, fd, frec,
                       params, pts, (float*)res, (float*)J, ld, flags, cauchy_c);
  else
    hipLaunchKernelGGL(mvba::k_depth_obs<double>, dim3(grid), dim3(64), 0, s, segs, nseg, dd, dpid, dmeas, fd,
                       frec, params, pts, (double*)res, (double*)J, ld, flags, cauchy_c);
  return hipGetLastError();
}

hipError_t mvba_launch_depth_gram(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                  const int32_t* dpid, const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                  const void* fl, double* rep, int64_t ng, int64_t nh, int32_t flags, double cauchy_c,
                                  mvba::Slab sl, hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_depth_gram, dim3((unsigned)nseg), dim3(64), 0, s, segs, nseg, dd, dpid, dmeas, frec, params,
                     pts, (const mvba::FrameLin*)fl, rep, ng, nh, flags, cauchy_c, sl);
  return hipGetLastError();
}

hipError_t mvba_launch_depth_cost(int64_t nslots, const mvba::DepthDesc* dd, const int64_t* dorder,
                                  const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                  int32_t flags, double cauchy_c, double* partial, hipStream_t s,
                                  int64_t* nblocks_out) {
  const int64_t blocks = (nslots + 255) / 256;
  if (nblocks_out) *nblocks_out = blocks;
  if (nslots <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_depth_cost, dim3((unsigned)blocks), dim3(256), 0, s, nslots, dd, dorder, dmeas, frec,
                     params, pts, flags, cauchy_c, partial);
  return hipGetLastError();
}

hipError_t mvba_launch_depth_sb(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                const int32_t* dpid, const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                const void* fl, const double* du, double* yrep, int64_t ng, int32_t flags,
                                double cauchy_c, const int32_t* gate, mvba::Slab sl, const double4* wbuf,
                                hipStream_t s) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_depth_sb, dim3((unsigned)nseg), dim3(64), 0, s, segs, nseg, dd, dpid, dmeas, frec, params, pts,
                     (const mvba::FrameLin*)fl, du, yrep, ng, flags, cauchy_c, gate, sl, wbuf);
  return hipGetLastError();
}

hipError_t mvba_launch_xyz_cost(int64_t n, const int32_t* xpid, const double4* xref, const double* xcc,
                                const double4* pts, int32_t flags, double* partial, unsigned* counter,
                                double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_xyz_cost, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, xpid, xref, xcc, pts,
                     flags, partial, counter, out);
  return hipGetLastError();
}

hipError_t mvba_launch_xyz_eval(int64_t n, const int32_t* xpid, const int64_t* xorder, const double4* xref,
                                const double4* pts, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mvba::k_xyz_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, xpid, xorder, xref,
                     pts, out);
  return hipGetLastError();
}

}  // extern "C"
