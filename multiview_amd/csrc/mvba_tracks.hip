// mvba_tracks.hip — per-pass triangulation and outlier flagging on gfx950
// (SURVEY.md §8 f1).
//
//  k_undistort   one thread per feature: Convert<DISTORTED, UNDISTORTED_C>
//                (camera_params.cc:316-355, :408-410): NONE, FOV, RADTAN through a
//                restatement of OpenCV 3.2 cv::undistortPoints [ext] (5 fixed
//                iterations, then P = undistorted intrinsics), RPC through the
//                undistortion half of the coefficients (compute_rpc,
//                rpc_distortion.cc:116-160, :362-366).
//  k_triangulate one thread per track: multiViewTriangulation
//                (interest_point.cc:649-722) = openMVG Triangulation::compute(3)
//                (triangulation_nview.cc:87-150), P = diag(f, f, 1) [R | t]
//                (interest_point.cc:398-422, projection.cc:35-38).
//  k_flag_angle  one thread per track: max pairwise ray angle among inliers
//                (rig_calibrator.cc:1056-1110).
//  k_flag_reproj one thread per feature: |residual| <= max_reprojection_error
//                (rig_calibrator.cc:1116-1147).
#include <algorithm>
#include <string>
#include <vector>

#include "mvba_depth.h"
#include "mvba_internal.h"

namespace mvba {

struct TrackCams {
  const double* focal;
  const double* center;
  const int32_t* K;
  const int64_t* doff;
  const double* dist;
  const double* dhalf;
  const double* uhalf;
};

// compute_rpc with n coefficients (degree from n = 2 (d+1)(d+2) - 2), in the
// reference's accumulation order.
__device__ void rpc_eval(const double* c, int n, double x, double y, double* ox, double* oy) {
#pragma clang fp contract(off)
  const int d = (int)llround(sqrt(2.0 * n + 5.0) / 2.0 - 1.5);
  double px[kMaxRpcDegree + 1], py[kMaxRpcDegree + 1];
  double vx = 1.0, vy = 1.0;
  for (int k = 0; k <= kMaxRpcDegree; k++) {
    px[k] = vx;
    py[k] = vy;
    if (k < d) {
      vx *= x;
      vy *= y;
    }
  }
  double vals[4] = {0.0, 1.0, 0.0, 1.0};
  int ci = 0;
  for (int count = 0; count < 4; count++) {
    const int start = (count == 1 || count == 3) ? 1 : 0;
    for (int dg = start; dg <= d; dg++)
      for (int i = 0; i <= dg; i++) {
        vals[count] += c[ci] * px[dg - i] * py[i];
        ci++;
      }
  }
  *ox = vals[0] / vals[1];
  *oy = vals[2] / vals[3];
}

__global__ void k_undistort(int64_t nobs, const int32_t* __restrict__ img, const int32_t* __restrict__ image_cam,
                            const double* __restrict__ pix, TrackCams cams, double* __restrict__ upix) {
  // no contraction: the oracle's oracle_undistort bit for bit (the mesh rays
  // are rounded to float from these values)
#pragma clang fp contract(off)
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= nobs) return;
  const int cam = image_cam[img[o]];
  const double f = cams.focal[cam];
  const double cx = cams.center[2 * cam], cy = cams.center[2 * cam + 1];
  const double hx = cams.dhalf[2 * cam], hy = cams.dhalf[2 * cam + 1];
  const int K = cams.K[cam];
  const double* k = cams.dist + cams.doff[cam];
  // DISTORTED -> DISTORTED_C
  const double dx = pix[2 * o] - hx, dy = pix[2 * o + 1] - hy;
  double ux, uy;
  if (K == 0) {
    ux = dx - (cx - hx);
    uy = dy - (cy - hy);
  } else if (K == 1) {
    const double nx = (dx - (cx - hx)) / f, ny = (dy - (cy - hy)) / f;
    const double rd = sqrt(nx * nx + ny * ny);
    const double ru = tan(rd * k[0]) / (2.0 * tan(k[0] / 2.0));
    const double conv = (rd > 1e-5) ? ru / rd : 1.0;
    ux = conv * (nx * f);
    uy = conv * (ny * f);
  } else if (K == 4 || K == 5) {
    // cv::undistortPoints(src = distorted pixel, K_dist = [f 0 c; 0 f c], k,
    //                     R = I, P = [f 0 uh; 0 f uh]), then minus the undistorted half size
    const double sx = dx + hx, sy = dy + hy;
    const double ifx = 1.0 / f, ify = 1.0 / f;
    double x = (sx - cx) * ifx, y = (sy - cy) * ify;
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = (K == 5) ? k[4] : 0.0;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
      const double r2 = x * x + y * y;
      const double icdist = 1.0 / (1.0 + ((k3 * r2 + k2) * r2 + k1) * r2);
      const double deltaX = 2.0 * p1 * x * y + p2 * (r2 + 2.0 * x * x);
      const double deltaY = p1 * (r2 + 2.0 * y * y) + 2.0 * p2 * x * y;
      x = (x0 - deltaX) * icdist;
      y = (y0 - deltaY) * icdist;
    }
    const double uhx = cams.uhalf[2 * cam], uhy = cams.uhalf[2 * cam + 1];
    const double xx = f * x + 0.0 * y + uhx;
    const double yy = 0.0 * x + f * y + uhy;
    ux = xx - uhx;
    uy = yy - uhy;
  } else {
    const int n = K / 2;
    rpc_eval(k + n, n, dx, dy, &ux, &uy);
  }
  upix[2 * o] = ux;
  upix[2 * o + 1] = uy;
}

// Eigen 3x3 inverse (cofactor column 0, adjugate / det), as Matrix3d::inverse [ext].
__device__ __forceinline__ void eigen_inverse3(const double* m, double* o) {
  auto M = [&](int r, int c) { return m[3 * r + c]; };
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
  };
  const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
  const double det = c0[0] * M(0, 0) + c0[1] * M(1, 0) + c0[2] * M(2, 0);
  const double inv = 1.0 / det;
  o[3 * 0 + 0] = c0[0] * inv;
  o[3 * 0 + 1] = c0[1] * inv;
  o[3 * 0 + 2] = c0[2] * inv;
  o[3 * 1 + 0] = cof(0, 1) * inv;
  o[3 * 1 + 1] = cof(1, 1) * inv;
  o[3 * 1 + 2] = cof(2, 1) * inv;
  o[3 * 2 + 0] = cof(0, 2) * inv;
  o[3 * 2 + 1] = cof(1, 2) * inv;
  o[3 * 2 + 2] = cof(2, 2) * inv;
}

// P = diag(f, f, 1) [R | t] (row-major 3x4)
__device__ __forceinline__ void proj_matrix(const double* wc, double f, double* P) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const double s = (r < 2) ? f : 1.0;
#pragma unroll
    for (int c = 0; c < 3; c++) P[4 * r + c] = s * wc[3 * r + c];
    P[4 * r + 3] = s * wc[9 + r];
  }
}

__global__ void k_triangulate(int64_t npts, const int64_t* __restrict__ tb, const int32_t* __restrict__ img,
                              const int32_t* __restrict__ image_cam, const double* __restrict__ wc,
                              const double* __restrict__ focal, const double* __restrict__ upix,
                              uint8_t* __restrict__ inlier, double* __restrict__ xyz) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npts) return;
  const int64_t b = tb[p], e = tb[p + 1];
  int nin = 0;
  for (int64_t o = b; o < e; o++) nin += inlier[o] ? 1 : 0;
  if (nin < 2) {
    for (int64_t o = b; o < e; o++) inlier[o] = 0;
    return;  // xyz stays as initialised (0)
  }
  // openMVG Triangulation::compute(iter = 3): iterated weighted linear LS
  double X[3] = {0.0, 0.0, 0.0};
  for (int it = 0; it < 3; it++) {
    double AtA[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, Atb[3] = {0, 0, 0};
    for (int64_t o = b; o < e; o++) {
      if (!inlier[o]) continue;
      double P[12];
      const int im = img[o];
      proj_matrix(wc + 12 * im, focal[image_cam[im]], P);
      const double u = upix[2 * o], v = upix[2 * o + 1];
      double w = 1.0;
      if (it > 0) {  // weights from the previous solution: 1 / depth
        const double z = P[8] * X[0] + P[9] * X[1] + P[10] * X[2] + P[11];
        w = 1.0 / z;
      }
      double v1[3], v2[3];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        v1[j] = w * (P[j] - u * P[8 + j]);
        v2[j] = w * (P[4 + j] - v * P[8 + j]);
        Atb[j] += w * (v1[j] * (u * P[11] - P[3]) + v2[j] * (v * P[11] - P[7]));
      }
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int j = 0; j <= k; j++) {
          const double val = v1[j] * v1[k] + v2[j] * v2[k];
          AtA[3 * j + k] += val;
          if (j < k) AtA[3 * k + j] += val;
        }
    }
    double Ai[9];
    eigen_inverse3(AtA, Ai);
#pragma unroll
    for (int r = 0; r < 3; r++) X[r] = Ai[3 * r] * Atb[0] + Ai[3 * r + 1] * Atb[1] + Ai[3 * r + 2] * Atb[2];
  }
  xyz[3 * p] = X[0];
  xyz[3 * p + 1] = X[1];
  xyz[3 * p + 2] = X[2];
  if (!isfinite(X[0]) || !isfinite(X[1]) || !isfinite(X[2]))
    for (int64_t o = b; o < e; o++) inlier[o] = 0;
}

// Camera centre (world_to_cam.inverse() * 0): -R^-1 t (Affine3d inverse, Affine mode).
__device__ __forceinline__ void cam_center(const double* wcm, double* C) {
  double Ri[9];
  inverse3(wcm, Ri);
#pragma unroll
  for (int r = 0; r < 3; r++) C[r] = -(Ri[3 * r] * wcm[9] + Ri[3 * r + 1] * wcm[10] + Ri[3 * r + 2] * wcm[11]);
}

__global__ void k_flag_angle(int64_t npts, const int64_t* __restrict__ tb, const int32_t* __restrict__ img,
                             const double* __restrict__ wc, const double* __restrict__ xyz, double min_angle,
                             uint8_t* __restrict__ inlier, unsigned long long* __restrict__ counts) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long n_in = 0, n_out = 0;
  if (p < npts) {
    const int64_t b = tb[p], e = tb[p + 1];
    const double X[3] = {xyz[3 * p], xyz[3 * p + 1], xyz[3 * p + 2]};
    double max_angle = 0.0;
    for (int64_t o1 = b; o1 < e; o1++) {
      if (!inlier[o1]) continue;
      n_in++;
      double C1[3];
      cam_center(wc + 12 * img[o1], C1);
      double r1[3] = {X[0] - C1[0], X[1] - C1[1], X[2] - C1[2]};
      const double n1 = sqrt(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
      if (n1 > 0.0)
        for (int q = 0; q < 3; q++) r1[q] /= n1;
      for (int64_t o2 = b; o2 < e; o2++) {
        if (img[o2] <= img[o1] || !inlier[o2]) continue;
        double C2[3];
        cam_center(wc + 12 * img[o2], C2);
        double r2[3] = {X[0] - C2[0], X[1] - C2[1], X[2] - C2[2]};
        const double n2 = sqrt(r2[0] * r2[0] + r2[1] * r2[1] + r2[2] * r2[2]);
        if (n2 > 0.0)
          for (int q = 0; q < 3; q++) r2[q] /= n2;
        const double ang = (180.0 / M_PI) * acos(r1[0] * r2[0] + r1[1] * r2[1] + r1[2] * r2[2]);
        if (isnan(ang) || isinf(ang)) continue;
        max_angle = fmax(max_angle, ang);
      }
    }
    if (!(max_angle >= min_angle))
      for (int64_t o = b; o < e; o++)
        if (inlier[o]) {
          inlier[o] = 0;
          n_out++;
        }
  }
  // block totals, one atomic per block and counter
  __shared__ unsigned long long s_in, s_out;
  if (threadIdx.x == 0) s_in = s_out = 0;
  __syncthreads();
  atomicAdd(&s_in, n_in);
  atomicAdd(&s_out, n_out);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&counts[0], s_out);
    atomicAdd(&counts[1], s_in);
  }
}

__global__ void k_flag_reproj(int64_t nobs, const double* __restrict__ res, double max_err,
                              uint8_t* __restrict__ inlier, unsigned long long* __restrict__ counts) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long n_in = 0, n_out = 0;
  if (o < nobs && inlier[o]) {
    n_in = 1;
    const double rx = res[2 * o], ry = res[2 * o + 1];
    // NaN never passes, as in the reference's comparison
    const bool good = sqrt(rx * rx + ry * ry) <= max_err;
    if (!good) {
      inlier[o] = 0;
      n_out = 1;
    }
  }
  __shared__ unsigned long long s_in, s_out;
  if (threadIdx.x == 0) s_in = s_out = 0;
  __syncthreads();
  if (n_in) atomicAdd(&s_in, n_in);
  if (n_out) atomicAdd(&s_out, n_out);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&counts[2], s_out);
    atomicAdd(&counts[3], s_in);
  }
}

// meshTriangulations' rays (texture_processing.cc:1448-1468), one thread per
// feature, in double with the reference's operation order (no contraction):
// cam_ray = normalize(u / f, v / f, 1); cam_to_world = world_to_cam^-1 (Eigen
// Affine inverse); world_ray = R^-1 cam_ray; cam_ctr = -R^-1 t; float copies
// for rayint's Ray with the direction normalised again in float. Outliers get a
// zero direction (no ray).
// inverse3 (mvba_depth.h) without contraction: the oracle's affine_inverse bit for bit
__device__ __forceinline__ void inverse3_exact(const double* m, double* o) {
#pragma clang fp contract(off)
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

__global__ void k_mesh_feature_rays(int64_t nobs, const int32_t* __restrict__ img,
                                    const int32_t* __restrict__ image_cam, const double* __restrict__ wc,
                                    const double* __restrict__ focal, const double* __restrict__ upix,
                                    const uint8_t* __restrict__ inlier, float* __restrict__ orig,
                                    float* __restrict__ dir, double* __restrict__ ctr, double* __restrict__ wray) {
#pragma clang fp contract(off)
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= nobs) return;
  if (!inlier[o]) {
    for (int q = 0; q < 3; q++) {
      orig[3 * o + q] = 0.0f;
      dir[3 * o + q] = 0.0f;
    }
    return;
  }
  const int im = img[o];
  const double f = focal[image_cam[im]];
  double cr[3] = {upix[2 * o] / f, upix[2 * o + 1] / f, 1.0};
  const double nrm = sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
  for (int q = 0; q < 3; q++) cr[q] = cr[q] / nrm;
  const double* w = wc + 12 * im;
  double Ri[9];
  inverse3_exact(w, Ri);
  float fd[3];
  for (int r = 0; r < 3; r++) {
    const double wr = Ri[3 * r] * cr[0] + Ri[3 * r + 1] * cr[1] + Ri[3 * r + 2] * cr[2];
    const double c = -(Ri[3 * r] * w[9] + Ri[3 * r + 1] * w[10] + Ri[3 * r + 2] * w[11]);
    wray[3 * o + r] = wr;
    ctr[3 * o + r] = c;
    orig[3 * o + r] = (float)c;
    fd[r] = (float)wr;
  }
  float s = 0.0f;
  s = s + fd[0] * fd[0];
  s = s + fd[1] * fd[1];
  s = s + fd[2] * fd[2];
  const float dn = sqrtf(s);
  for (int q = 0; q < 3; q++) dir[3 * o + q] = fd[q] / dn;
}

// Per track: intersection = cam_ctr + t * world_ray for every hit, summed in
// feature order and divided by the count (bad = 1e100 otherwise).
__global__ void k_mesh_points(int64_t npts, const int64_t* __restrict__ tb, const float* __restrict__ thit,
                              const int32_t* __restrict__ fhit, const double* __restrict__ ctr,
                              const double* __restrict__ wray, double* __restrict__ feat_xyz,
                              double* __restrict__ pt_xyz) {
#pragma clang fp contract(off)
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npts) return;
  const double bad = 1.0e+100;
  double avg[3] = {0.0, 0.0, 0.0};
  int num = 0;
  for (int64_t o = tb[p]; o < tb[p + 1]; o++) {
    double X[3] = {bad, bad, bad};
    if (fhit[o] >= 0) {
      const double t = (double)thit[o];
      for (int q = 0; q < 3; q++) X[q] = ctr[3 * o + q] + t * wray[3 * o + q];
      for (int q = 0; q < 3; q++) avg[q] += X[q];
      num++;
    }
    if (feat_xyz)
      for (int q = 0; q < 3; q++) feat_xyz[3 * o + q] = X[q];
  }
  for (int q = 0; q < 3; q++) pt_xyz[3 * p + q] = num >= 1 ? avg[q] / (double)num : bad;
}

}  // namespace mvba

extern "C" hipError_t mvba_launch_mesh_rays(const mvba_mesh* m, int64_t n, const int64_t* perm, const float* orig,
                                            const float* dir, float tmin, float tmax, float* t_out,
                                            int32_t* face_out, hipStream_t s);
extern "C" int32_t mvba_mesh_device_ordinal(const mvba_mesh* m);

namespace {

thread_local std::string g_tracks_error;

struct DevTracks {
  int64_t nobs = 0, npts = 0;
  int32_t* img = nullptr;
  int32_t* image_cam = nullptr;
  double* wc = nullptr;
  double* focal = nullptr;
  double* center = nullptr;
  int32_t* K = nullptr;
  int64_t* doff = nullptr;
  double* dist = nullptr;
  double* dhalf = nullptr;
  double* uhalf = nullptr;
  int64_t* tb = nullptr;
  double* pix = nullptr;
  double* upix = nullptr;
  uint8_t* inlier = nullptr;
  double* xyz = nullptr;
  double* res = nullptr;
  unsigned long long* counts = nullptr;
  ~DevTracks() {
    void* ptrs[] = {img, image_cam, wc, focal, center, K, doff, dist, dhalf, uhalf, tb, pix, upix, inlier, xyz, res,
                    counts};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
  }
};

template <class T>
hipError_t put(T** p, const T* src, size_t n) {
  hipError_t e = dalloc(p, n);
  if (e == hipSuccess && n && src) e = hipMemcpy(*p, src, n * sizeof(T), hipMemcpyHostToDevice);
  return e;
}

mvba_status fail(mvba_status st, const std::string& m) {
  g_tracks_error = m;
  return st;
}

// Validation + upload shared by both entry points.
mvba_status load(const mvba_tracks_desc* d, int32_t device, DevTracks& t) {
  if (!d) return fail(MVBA_E_INVALID, "null tracks description");
  if (d->num_images < 0 || d->num_cameras < 0 || d->num_points < 0)
    return fail(MVBA_E_INVALID, "negative sizes in tracks description");
  if (d->num_points > 0 && (!d->track_begin || !d->world_to_cam || !d->image_camera))
    return fail(MVBA_E_INVALID, "null array in tracks description");
  const int64_t nobs = d->num_points > 0 ? d->track_begin[d->num_points] : 0;
  if (nobs > 0 && (!d->track_image || !d->track_pix)) return fail(MVBA_E_INVALID, "null array in tracks description");
  if (d->num_cameras > 0 && (!d->focal || !d->center || !d->dist_size || !d->dist_offset || !d->dist_half ||
                             !d->undist_half))
    return fail(MVBA_E_INVALID, "null array in tracks description");
  int64_t dist_len = 0;
  for (int c = 0; c < d->num_cameras; c++) {
    const int K = d->dist_size[c];
    int deg = 0;
    if (mvba_internal::model_of(K, &deg) < 0 || (K > 5 && deg > mvba::kMaxRpcDegree))
      return fail(MVBA_E_BAD_DISTORTION, "Recieved irregular distortion vector size. Size = " + std::to_string(K));
    dist_len = std::max<int64_t>(dist_len, d->dist_offset[c] + K);
  }
  for (int i = 0; i < d->num_images; i++)
    if (d->image_camera[i] < 0 || d->image_camera[i] >= d->num_cameras)
      return fail(MVBA_E_INVALID, "image camera index out of range");
  for (int64_t p = 0; p < d->num_points; p++) {
    if (d->track_begin[p + 1] < d->track_begin[p]) return fail(MVBA_E_INVALID, "track_begin must be non-decreasing");
    for (int64_t o = d->track_begin[p]; o < d->track_begin[p + 1]; o++) {
      if (d->track_image[o] < 0 || d->track_image[o] >= d->num_images)
        return fail(MVBA_E_INVALID, "track image index out of range");
      if (o > d->track_begin[p] && d->track_image[o] <= d->track_image[o - 1])
        return fail(MVBA_E_INVALID, "track images must be increasing within a track (pid_to_cid_fid order)");
    }
  }
  int32_t ndev = 0;
  if (mvba_device_count(&ndev) != MVBA_OK) return fail(MVBA_E_NO_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(MVBA_E_INVALID, "invalid device ordinal");
  if (hipSetDevice(device) != hipSuccess) return fail(MVBA_E_HIP, "hipSetDevice failed");
  t.nobs = nobs;
  t.npts = d->num_points;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (e == hipSuccess && x != hipSuccess) e = x;
  };
  chk(put(&t.img, d->track_image, (size_t)nobs));
  chk(put(&t.image_cam, d->image_camera, (size_t)d->num_images));
  chk(put(&t.wc, d->world_to_cam, (size_t)12 * d->num_images));
  chk(put(&t.focal, d->focal, (size_t)d->num_cameras));
  chk(put(&t.center, d->center, (size_t)2 * d->num_cameras));
  chk(put(&t.K, d->dist_size, (size_t)d->num_cameras));
  chk(put(&t.doff, d->dist_offset, (size_t)d->num_cameras));
  chk(put(&t.dist, d->dist, (size_t)dist_len));
  chk(put(&t.dhalf, d->dist_half, (size_t)2 * d->num_cameras));
  chk(put(&t.uhalf, d->undist_half, (size_t)2 * d->num_cameras));
  chk(put(&t.tb, d->track_begin, (size_t)d->num_points + 1));
  chk(put(&t.pix, d->track_pix, (size_t)2 * nobs));
  chk(dalloc(&t.inlier, (size_t)nobs));
  chk(dalloc(&t.xyz, (size_t)3 * d->num_points));
  chk(dalloc(&t.counts, 4));
  if (e == hipSuccess) chk(hipMemset(t.counts, 0, 4 * sizeof(unsigned long long)));
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  return MVBA_OK;
}

unsigned grid(int64_t n) { return (unsigned)std::max<int64_t>((n + 255) / 256, 1); }

}  // namespace

extern "C" {

const char* mvba_tracks_error(void) { return g_tracks_error.c_str(); }

mvba_status mvba_triangulate(const mvba_tracks_desc* d, int32_t device, uint8_t* inlier, double* xyz) {
  g_tracks_error.clear();
  if (!inlier && d && d->num_points > 0) return fail(MVBA_E_INVALID, "null inlier array");
  if (!xyz && d && d->num_points > 0) return fail(MVBA_E_INVALID, "null xyz array");
  DevTracks t;
  mvba_status st = load(d, device, t);
  if (st != MVBA_OK) return st;
  if (t.npts == 0) return MVBA_OK;
  hipError_t e = hipMemcpy(t.inlier, inlier, (size_t)t.nobs, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(t.xyz, 0, (size_t)3 * t.npts * sizeof(double));
  if (e == hipSuccess) e = dalloc(&t.upix, (size_t)2 * t.nobs);
  if (e == hipSuccess && t.nobs > 0) {
    mvba::TrackCams cams{t.focal, t.center, t.K, t.doff, t.dist, t.dhalf, t.uhalf};
    hipLaunchKernelGGL(mvba::k_undistort, dim3(grid(t.nobs)), dim3(256), 0, nullptr, t.nobs, t.img, t.image_cam, t.pix,
                       cams, t.upix);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mvba::k_triangulate, dim3(grid(t.npts)), dim3(256), 0, nullptr, t.npts, t.tb, t.img,
                       t.image_cam, t.wc, t.focal, t.upix, t.inlier, t.xyz);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(inlier, t.inlier, (size_t)t.nobs, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(xyz, t.xyz, (size_t)3 * t.npts * sizeof(double), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  return MVBA_OK;
}

mvba_status mvba_flag_outliers(const mvba_tracks_desc* d, int32_t device, const double* xyz, const double* residuals,
                               double min_triangulation_angle, double max_reprojection_error, uint8_t* inlier,
                               int64_t* counts) {
  g_tracks_error.clear();
  if (d && d->num_points > 0 && (!xyz || !residuals || !inlier || !counts))
    return fail(MVBA_E_INVALID, "null array");
  DevTracks t;
  mvba_status st = load(d, device, t);
  if (st != MVBA_OK) return st;
  if (counts)
    for (int q = 0; q < 4; q++) counts[q] = 0;
  if (t.npts == 0) return MVBA_OK;
  hipError_t e = hipMemcpy(t.inlier, inlier, (size_t)t.nobs, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(t.xyz, xyz, (size_t)3 * t.npts * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = put(&t.res, residuals, (size_t)2 * t.nobs);
  // angle pass first: the reprojection pass would drop rays that form the points
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mvba::k_flag_angle, dim3(grid(t.npts)), dim3(256), 0, nullptr, t.npts, t.tb, t.img, t.wc,
                       t.xyz, min_triangulation_angle, t.inlier, t.counts);
    e = hipGetLastError();
  }
  if (e == hipSuccess && t.nobs > 0) {
    hipLaunchKernelGGL(mvba::k_flag_reproj, dim3(grid(t.nobs)), dim3(256), 0, nullptr, t.nobs, t.res,
                       max_reprojection_error, t.inlier, t.counts);
    e = hipGetLastError();
  }
  unsigned long long hc[4] = {0, 0, 0, 0};
  if (e == hipSuccess) e = hipMemcpy(inlier, t.inlier, (size_t)t.nobs, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(hc, t.counts, sizeof(hc), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  for (int q = 0; q < 4; q++) counts[q] = (int64_t)hc[q];
  return MVBA_OK;
}

mvba_status mvba_mesh_triangulate(const mvba_tracks_desc* d, mvba_mesh* m, const uint8_t* inlier,
                                  double min_ray_dist, double max_ray_dist, double* feature_xyz, double* point_xyz) {
  g_tracks_error.clear();
  if (!m) return fail(MVBA_E_INVALID, "null mesh handle");
  if (d && d->num_points > 0 && (!inlier || !point_xyz)) return fail(MVBA_E_INVALID, "null array");
  DevTracks t;
  mvba_status st = load(d, mvba_mesh_device_ordinal(m), t);
  if (st != MVBA_OK) return st;
  if (t.npts == 0) return MVBA_OK;
  const int64_t n = t.nobs;
  float *orig = nullptr, *dir = nullptr, *thit = nullptr;
  int32_t* fhit = nullptr;
  double *ctr = nullptr, *wray = nullptr, *fx = nullptr;
  int64_t* perm = nullptr;
  hipError_t e = hipMemcpy(t.inlier, inlier, (size_t)n, hipMemcpyHostToDevice);
  auto chk = [&](hipError_t x) {
    if (e == hipSuccess && x != hipSuccess) e = x;
  };
  chk(dalloc(&t.upix, (size_t)2 * n));
  chk(dalloc(&orig, (size_t)3 * n));
  chk(dalloc(&dir, (size_t)3 * n));
  chk(dalloc(&thit, (size_t)n));
  chk(dalloc(&fhit, (size_t)n));
  chk(dalloc(&ctr, (size_t)3 * n));
  chk(dalloc(&wray, (size_t)3 * n));
  chk(dalloc(&fx, (size_t)3 * n));
  {
    // image-major ray order (counting sort): a wave's rays share a camera centre
    std::vector<int64_t> cnt((size_t)d->num_images + 1, 0), order((size_t)n);
    for (int64_t o = 0; o < n; o++) cnt[(size_t)d->track_image[o] + 1]++;
    for (int32_t i = 0; i < d->num_images; i++) cnt[(size_t)i + 1] += cnt[(size_t)i];
    for (int64_t o = 0; o < n; o++) order[(size_t)cnt[(size_t)d->track_image[o]]++] = o;
    chk(upload(&perm, order));
  }
  if (e == hipSuccess && n > 0) {
    mvba::TrackCams cams{t.focal, t.center, t.K, t.doff, t.dist, t.dhalf, t.uhalf};
    hipLaunchKernelGGL(mvba::k_undistort, dim3(grid(n)), dim3(256), 0, nullptr, n, t.img, t.image_cam, t.pix, cams,
                       t.upix);
    hipLaunchKernelGGL(mvba::k_mesh_feature_rays, dim3(grid(n)), dim3(256), 0, nullptr, n, t.img, t.image_cam, t.wc,
                       t.focal, t.upix, t.inlier, orig, dir, ctr, wray);
    chk(hipGetLastError());
    chk(mvba_launch_mesh_rays(m, n, perm, orig, dir, (float)min_ray_dist, (float)max_ray_dist, thit, fhit, nullptr));
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mvba::k_mesh_points, dim3(grid(t.npts)), dim3(256), 0, nullptr, t.npts, t.tb, thit, fhit, ctr,
                       wray, fx, t.xyz);
    chk(hipGetLastError());
  }
  if (e == hipSuccess) chk(hipMemcpy(point_xyz, t.xyz, (size_t)3 * t.npts * sizeof(double), hipMemcpyDeviceToHost));
  if (e == hipSuccess && feature_xyz) chk(hipMemcpy(feature_xyz, fx, (size_t)3 * n * sizeof(double), hipMemcpyDeviceToHost));
  for (void* p : {(void*)orig, (void*)dir, (void*)thit, (void*)fhit, (void*)ctr, (void*)wray, (void*)fx, (void*)perm})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  return MVBA_OK;
}

}  // extern "C"
