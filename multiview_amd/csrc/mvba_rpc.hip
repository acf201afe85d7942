// mvba_rpc.hip — RPC lens-model fitting on the GPU.
//
// Replaces the nested Ceres fit the calibrator runs after a pass that floated
// RPC distortion: CameraParameters::updateRpcUndistortion (camera_params.cc:
// 214-253) -> fitRpcUndist (rpc_distortion.cc:658-721), and fitRpcDist
// (:622-656, used by the fit_rpc tool):
//   genUndistDistPairs (:519-557): num_samples x num_samples grid over the
//     undistorted image; keep a sample when Convert<UNDISTORTED, DISTORTED>
//     lands inside the distorted crop box; centre both pixels;
//   fitRpcUndist: targets undist_c, inputs compute_rpc(undist_c, dist coeffs);
//   fitRpcDist:   inputs undist_c, targets the camera's distorted pixel;
//   for degree 1..d: start from the identity (degree 1) or the previous
//     solution with zero new terms (increment_degree, :336-356), then
//     fitCurrDegRPC (:559-609): least squares of compute_rpc(in) - target, no
//     loss, Ceres LM, gradient/function tolerance 1e-16, the caller's parameter
//     tolerance and iteration cap;
//   evalRpcDistUndist (:723-737): max |undist(dist(p)) - p| over the samples.
//
// Device work: one kernel generates the pairs (one thread per sample); one
// kernel forms the normal equations of the current coefficients — the x and y
// halves of the coefficient vector are independent (x = Nx/Dx uses only
// num_x, den_x), so J^T J is two m x m blocks (m = (d+1)(d+2) - 1 <= 55). Each
// workgroup stages the Jacobian rows of 128 samples in LDS and every thread
// accumulates its share of the m(m+1)/2 products of each block; per-workgroup
// partials are summed by a second kernel in a fixed order (deterministic).
// The trust-region driver (host, n <= 110 unknowns) follows Ceres 1.14 LM:
// Jacobi scaling fixed at the start, LM diagonal clamp(diag, 1e-6, 1e32)/radius,
// step quality rho > 1e-3, radius / max(1/3, 1 - (2 rho - 1)^3), rejected steps
// radius /= 2^k, parameter tolerance before function tolerance; steps are exact
// (dense Cholesky) where Ceres' solver is iterative: both converge to the same
// least-squares fit (the parity test compares fitted models).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mvba/mvba.h"
#include "mvba_types.h"

namespace mvba_rpc {

constexpr int kChunk = 128;                 // samples staged per LDS pass
constexpr int kMaxM = 55;                   // (d+1)(d+2) - 1 at d = 6
constexpr int kThreads = 256;
constexpr int kMaxPairs = kMaxM * (kMaxM + 1) / 2;
constexpr int kPairsPerThread = (kMaxPairs + kThreads - 1) / kThreads;

__host__ __device__ inline int half_size(int d) { return (d + 1) * (d + 2) - 1; }
__host__ __device__ inline int num_len(int d) { return (d + 1) * (d + 2) / 2; }

// compute_rpc (rpc_distortion.cc:116-160), reference accumulation order.
__device__ void rpc_eval(const double* c, int d, double x, double y, double* ox, double* oy) {
  double px[mvba::kMaxRpcDegree + 1], py[mvba::kMaxRpcDegree + 1];
  double vx = 1.0, vy = 1.0;
#pragma unroll
  for (int k = 0; k <= mvba::kMaxRpcDegree; k++) {
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
      for (int i = 0; i <= dg; i++) vals[count] += c[ci++] * px[dg - i] * py[i];
  }
  *ox = vals[0] / vals[1];
  *oy = vals[2] / vals[3];
}

struct Cam {
  double f, cx, cy, dhx, dhy, uhx, uhy;
  int K, dist_deg;
  double k[5];          // FOV / RADTAN coefficients
  const double* rpc;    // RPC distortion half (device), K > 5
  int W, H, cropW, cropH, uW, uH;
};

// CameraParameters::DistortCentered (camera_params.cc:260-314).
__device__ void distort_centered(const Cam& c, double ux, double uy, double* dx, double* dy) {
  if (c.K == 0) {
    *dx = ux + c.cx - c.dhx;
    *dy = uy + c.cy - c.dhy;
  } else if (c.K == 1) {
    const double nx = ux / c.f, ny = uy / c.f;
    const double ru = sqrt(nx * nx + ny * ny);
    const double rd = atan(ru * (2 * tan(c.k[0] / 2))) * (1 / c.k[0]);
    const double conv = ru > 1e-5 ? rd / ru : 1.0;
    *dx = (c.cx - c.dhx) + conv * nx * c.f;
    *dy = (c.cy - c.dhy) + conv * ny * c.f;
  } else if (c.K == 4 || c.K == 5) {
    const double k1 = c.k[0], k2 = c.k[1], p1 = c.k[2], p2 = c.k[3], k3 = c.K == 5 ? c.k[4] : 0.0;
    const double nx = ux / c.f, ny = uy / c.f;
    const double r2 = nx * nx + ny * ny;
    const double rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2;
    double ox = rad * nx, oy = rad * ny;
    ox += 2 * p1 * nx * ny + p2 * (r2 + 2 * nx * nx);
    oy += p1 * (r2 + 2 * ny * ny) + 2 * p2 * nx * ny;
    *dx = ox * c.f + (c.cx - c.dhx);
    *dy = oy * c.f + (c.cy - c.dhy);
  } else {
    rpc_eval(c.rpc, c.dist_deg, ux, uy, dx, dy);
  }
}

// genUndistDistPairs + the mode's input/target choice. pairs[q] = (in.x, in.y,
// target.x, target.y); valid[q] = inside the distorted crop box. q = ix*S + iy.
__global__ void k_rpc_pairs(Cam cam, int S, int mode, const double* __restrict__ fit_dist, int fit_deg,
                            double4* __restrict__ pairs, uint8_t* __restrict__ valid) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)S * S) return;
  const int ix = (int)(q / S), iy = (int)(q % S);
  const double x = (cam.uW - 1.0) * ix / (S - 1.0);
  const double y = (cam.uH - 1.0) * iy / (S - 1.0);
  const double ux = x - cam.uhx, uy = y - cam.uhy;  // UNDISTORTED -> UNDISTORTED_C
  double dx, dy;
  distort_centered(cam, ux, uy, &dx, &dy);
  dx += cam.dhx;  // DISTORTED_C -> DISTORTED
  dy += cam.dhy;
  const bool in = !(fabs(dx - cam.W / 2.0) > cam.cropW / 2.0 || fabs(dy - cam.H / 2.0) > cam.cropH / 2.0);
  valid[q] = in ? 1 : 0;
  const double dcx = dx - cam.dhx, dcy = dy - cam.dhy;
  if (mode == MVBA_RPC_FIT_DISTORTION) {
    pairs[q] = make_double4(ux, uy, dcx, dcy);
  } else {
    double rx, ry;  // fitRpcUndist: dist_centered = compute_rpc(undist_centered, dist coeffs)
    rpc_eval(fit_dist, fit_deg, ux, uy, &rx, &ry);
    pairs[q] = make_double4(rx, ry, ux, uy);
  }
}

// Normal equations (or the cost only) of coefficients c of degree d over the
// valid pairs. Per-workgroup partial layout: [Hx (P) | Hy (P) | gx (m) | gy (m) | cost].
__global__ __launch_bounds__(kThreads) void k_rpc_normal(int64_t n, const double4* __restrict__ pairs,
                                                         const uint8_t* __restrict__ valid,
                                                         const double* __restrict__ c, int d, int want_jac,
                                                         double* __restrict__ partial) {
  __shared__ double J[kMaxM][kChunk + 1];
  __shared__ double R[kChunk];
  __shared__ double red[kThreads];
  const int tid = threadIdx.x;
  const int m = half_size(d), nl = num_len(d);
  const int P = m * (m + 1) / 2;
  double accH[2][kPairsPerThread];
  double accG[2] = {0.0, 0.0};
  for (int h = 0; h < 2; h++)
    for (int k = 0; k < kPairsPerThread; k++) accH[h][k] = 0.0;
  double cost = 0.0;
  // pair q -> (i, j), j <= i: q = i (i + 1) / 2 + j
  int pi[kPairsPerThread], pj[kPairsPerThread];
  for (int k = 0; k < kPairsPerThread; k++) {
    const int q = tid + k * kThreads;
    int i = (int)((sqrt(8.0 * q + 1.0) - 1.0) / 2.0);
    while (i * (i + 1) / 2 > q) i--;
    while ((i + 1) * (i + 2) / 2 <= q) i++;
    pi[k] = q < P ? i : 0;
    pj[k] = q < P ? q - i * (i + 1) / 2 : 0;
  }
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    for (int h = 0; h < 2; h++) {
      if (tid < kChunk) {
        const int64_t s = ch * kChunk + tid;
        const bool ok = s < n && valid[s];
        double px[mvba::kMaxRpcDegree + 1], py[mvba::kMaxRpcDegree + 1];
        double N = 0.0, D = 1.0, r = 0.0;
        if (ok) {
          const double4 p = pairs[s];
          double vx = 1.0, vy = 1.0;
#pragma unroll
          for (int k = 0; k <= mvba::kMaxRpcDegree; k++) {
            px[k] = vx;
            py[k] = vy;
            if (k < d) {
              vx *= p.x;
              vy *= p.y;
            }
          }
          const double* cn = c + h * m;
          const double* cd = cn + nl;
          int ci = 0;
          for (int dg = 0; dg <= d; dg++)
            for (int i = 0; i <= dg; i++) N += cn[ci++] * px[dg - i] * py[i];
          ci = 0;
          for (int dg = 1; dg <= d; dg++)
            for (int i = 0; i <= dg; i++) D += cd[ci++] * px[dg - i] * py[i];
          r = N / D - (h == 0 ? p.z : p.w);
          cost += r * r;
        }
        if (want_jac) {
          const double inv = ok ? 1.0 / D : 0.0;
          const double nd = ok ? -N / (D * D) : 0.0;
          int k = 0;
          for (int dg = 0; dg <= d; dg++)
            for (int i = 0; i <= dg; i++, k++) {
              const double mono = ok ? px[dg - i] * py[i] : 0.0;
              J[k][tid] = mono * inv;
              if (k > 0) J[nl + k - 1][tid] = mono * nd;
            }
          R[tid] = ok ? r : 0.0;
        }
      }
      if (want_jac) {
        __syncthreads();
        for (int k = 0; k < kPairsPerThread; k++) {
          if (tid + k * kThreads >= P) break;
          const double* a = J[pi[k]];
          const double* b = J[pj[k]];
          double s = 0.0;
          for (int t = 0; t < kChunk; t++) s += a[t] * b[t];
          accH[h][k] += s;
        }
        if (tid < m) {
          double s = 0.0;
          for (int t = 0; t < kChunk; t++) s += J[tid][t] * R[t];
          accG[h] += s;
        }
        __syncthreads();
      }
    }
  }
  const int stride = 2 * P + 2 * m + 1;
  double* out = partial + (int64_t)blockIdx.x * stride;
  if (want_jac) {
    for (int h = 0; h < 2; h++)
      for (int k = 0; k < kPairsPerThread; k++)
        if (tid + k * kThreads < P) out[h * P + tid + k * kThreads] = accH[h][k];
    if (tid < m) {
      out[2 * P + tid] = accG[0];
      out[2 * P + m + tid] = accG[1];
    }
  }
  red[tid] = cost;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) out[stride - 1] = 0.5 * red[0];
}

// Sum the per-workgroup partials in block order (entries [0, len) of each stride).
__global__ void k_rpc_reduce(int nblocks, int stride, int len, int first, const double* __restrict__ partial,
                             double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= len) return;
  double s = 0.0;
  for (int b = 0; b < nblocks; b++) s += partial[(int64_t)b * stride + first + e];
  out[e] = s;
}

// evalRpcDistUndist: per-block max of |undist(dist(p)) - p| over valid samples
// (p = pairs[q].zw in UNDIST mode: the undistorted centred pixel).
__global__ __launch_bounds__(kThreads) void k_rpc_roundtrip(int64_t n, const double4* __restrict__ pairs,
                                                            const uint8_t* __restrict__ valid,
                                                            const double* __restrict__ dist, const double* __restrict__ undist,
                                                            int d, double* __restrict__ block_max) {
  __shared__ double red[kThreads];
  double mx = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    if (!valid[q]) continue;
    const double4 p = pairs[q];
    double ax, ay, bx, by;
    rpc_eval(dist, d, p.z, p.w, &ax, &ay);
    rpc_eval(undist, d, ax, ay, &bx, &by);
    const double ex = p.z - bx, ey = p.w - by;
    mx = fmax(mx, sqrt(ex * ex + ey * ey));
  }
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) block_max[blockIdx.x] = red[0];
}

// -------------------------------------------------------------- host side
thread_local std::string g_error;

struct Dev {
  double4* pairs = nullptr;
  uint8_t* valid = nullptr;
  double* coeffs = nullptr;
  double* partial = nullptr;
  double* sums = nullptr;
  double* aux = nullptr;
  ~Dev() {
    for (void* p : {(void*)pairs, (void*)valid, (void*)coeffs, (void*)partial, (void*)sums, (void*)aux})
      if (p) (void)hipFree(p);
  }
};

struct Normal {
  std::vector<double> H;  // n x n dense (block diagonal)
  std::vector<double> g;  // n
  double cost = 0.0;
};

class Fitter {
 public:
  Fitter(Dev& dv, int64_t n, int nblocks) : dv_(dv), n_(n), nblocks_(nblocks) {}

  // cost (want_jac = 0) or cost + normal equations at coefficients x of degree d
  hipError_t eval(const std::vector<double>& x, int d, bool want_jac, Normal* out) {
    const int m = half_size(d), P = m * (m + 1) / 2, stride = 2 * P + 2 * m + 1;
    hipError_t e = hipMemcpy(dv_.coeffs, x.data(), x.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rpc_normal, dim3((unsigned)nblocks_), dim3(kThreads), 0, 0, n_, dv_.pairs, dv_.valid,
                       dv_.coeffs, d, want_jac ? 1 : 0, dv_.partial);
    const int len = want_jac ? stride : 1, first = want_jac ? 0 : stride - 1;
    hipLaunchKernelGGL(k_rpc_reduce, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, 0, nblocks_, stride, len, first,
                       dv_.partial, dv_.sums);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    std::vector<double> s((size_t)len);
    if ((e = hipMemcpy(s.data(), dv_.sums, s.size() * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess) return e;
    out->cost = s[(size_t)len - 1];
    if (want_jac) {
      const int nn = 2 * m;
      out->H.assign((size_t)nn * nn, 0.0);
      out->g.assign((size_t)nn, 0.0);
      for (int h = 0; h < 2; h++) {
        for (int i = 0, q = 0; i < m; i++)
          for (int j = 0; j <= i; j++, q++) {
            const double v = s[(size_t)(h * P + q)];
            out->H[(size_t)(h * m + i) * nn + (h * m + j)] = v;
            out->H[(size_t)(h * m + j) * nn + (h * m + i)] = v;
          }
        for (int i = 0; i < m; i++) out->g[(size_t)(h * m + i)] = s[(size_t)(2 * P + h * m + i)];
      }
    }
    return hipSuccess;
  }

 private:
  Dev& dv_;
  int64_t n_;
  int nblocks_;
};

// Dense Cholesky solve of A y = b (A symmetric positive definite, n <= 110).
bool chol_solve(std::vector<double> A, int n, std::vector<double>& b) {
  for (int j = 0; j < n; j++) {
    double d = A[(size_t)j * n + j];
    for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    A[(size_t)j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double s = A[(size_t)i * n + j];
      for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
      A[(size_t)i * n + j] = s / d;
    }
  }
  for (int i = 0; i < n; i++) {
    double s = b[(size_t)i];
    for (int k = 0; k < i; k++) s -= A[(size_t)i * n + k] * b[(size_t)k];
    b[(size_t)i] = s / A[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = b[(size_t)i];
    for (int k = i + 1; k < n; k++) s -= A[(size_t)k * n + i] * b[(size_t)k];
    b[(size_t)i] = s / A[(size_t)i * n + i];
  }
  return true;
}

struct DegreeResult {
  double initial_cost = 0, final_cost = 0;
  int iterations = 0;
  int termination = MVBA_NO_CONVERGENCE;
};

// Ceres 1.14 TrustRegionMinimizer + LevenbergMarquardtStrategy on one degree.
hipError_t lm_fit(Fitter& F, int d, std::vector<double>& x, int max_iter, double ptol, DegreeResult* res) {
  const double ftol = 1e-16, gtol = 1e-16;
  const int n = (int)x.size();
  Normal cur;
  hipError_t e = F.eval(x, d, true, &cur);
  if (e != hipSuccess) return e;
  res->initial_cost = res->final_cost = cur.cost;
  std::vector<double> scale((size_t)n);
  for (int j = 0; j < n; j++) scale[(size_t)j] = 1.0 / (1.0 + std::sqrt(cur.H[(size_t)j * n + j]));
  auto grad_max = [&](const Normal& N) {
    double m = 0.0;
    for (double v : N.g) m = std::max(m, std::fabs(v));
    return m;
  };
  if (grad_max(cur) <= gtol) {
    res->termination = MVBA_CONVERGENCE;
    return hipSuccess;
  }
  double radius = 1e4, decrease = 2.0;
  int invalid = 0;
  for (int it = 0; it < max_iter; it++) {
    res->iterations = it + 1;
    // (S H S + diag(clamp(diag(S H S), 1e-6, 1e32) / radius)) y = -S g, delta = S y
    std::vector<double> A((size_t)n * n), b((size_t)n);
    for (int i = 0; i < n; i++) {
      for (int j = 0; j < n; j++) A[(size_t)i * n + j] = scale[(size_t)i] * cur.H[(size_t)i * n + j] * scale[(size_t)j];
      b[(size_t)i] = -scale[(size_t)i] * cur.g[(size_t)i];
    }
    for (int i = 0; i < n; i++) {
      const double dg = std::min(std::max(A[(size_t)i * n + i], 1e-6), 1e32);
      A[(size_t)i * n + i] += dg / radius;
    }
    std::vector<double> delta(b);
    bool ok = chol_solve(A, n, delta);
    double model_change = 0.0;
    if (ok) {
      for (int i = 0; i < n; i++) delta[(size_t)i] *= scale[(size_t)i];
      // model cost change = -(g.delta + 0.5 delta' H delta)
      double gd = 0.0, hd = 0.0;
      for (int i = 0; i < n; i++) {
        gd += cur.g[(size_t)i] * delta[(size_t)i];
        double s = 0.0;
        for (int j = 0; j < n; j++) s += cur.H[(size_t)i * n + j] * delta[(size_t)j];
        hd += delta[(size_t)i] * s;
      }
      model_change = -(gd + 0.5 * hd);
      ok = std::isfinite(model_change) && model_change > 0.0;
    }
    if (!ok) {
      if (++invalid > 5) {
        res->termination = MVBA_FAILURE;
        return hipSuccess;
      }
      radius /= decrease;
      decrease *= 2.0;
      continue;
    }
    invalid = 0;
    std::vector<double> xn((size_t)n);
    double dn = 0.0, xnorm = 0.0;
    for (int i = 0; i < n; i++) {
      xn[(size_t)i] = x[(size_t)i] + delta[(size_t)i];
      dn += delta[(size_t)i] * delta[(size_t)i];
      xnorm += x[(size_t)i] * x[(size_t)i];
    }
    Normal cand;
    if ((e = F.eval(xn, d, false, &cand)) != hipSuccess) return e;
    if (std::sqrt(dn) <= ptol * (std::sqrt(xnorm) + ptol)) {
      res->termination = MVBA_CONVERGENCE;
      return hipSuccess;
    }
    const double change = cur.cost - cand.cost;
    if (std::fabs(change) <= ftol * cur.cost) {
      res->termination = MVBA_CONVERGENCE;
      return hipSuccess;
    }
    const double rho = change / model_change;
    if (std::isfinite(cand.cost) && rho > 1e-3) {
      x = xn;
      if ((e = F.eval(x, d, true, &cur)) != hipSuccess) return e;
      res->final_cost = cur.cost;
      const double t = 2.0 * rho - 1.0;
      radius = std::min(1e16, radius / std::max(1.0 / 3.0, 1.0 - t * t * t));
      decrease = 2.0;
      if (grad_max(cur) <= gtol) {
        res->termination = MVBA_CONVERGENCE;
        return hipSuccess;
      }
    } else {
      radius /= decrease;
      decrease *= 2.0;
      if (radius < 1e-32) {
        res->termination = MVBA_CONVERGENCE;
        return hipSuccess;
      }
    }
  }
  res->termination = MVBA_NO_CONVERGENCE;
  return hipSuccess;
}

// RPCLensDistortion::init_as_identity of degree 1 (rpc_distortion.cc:303-318):
// num_x = (0, 1, 0), num_y = (0, 0, 1), denominators 0.
std::vector<double> identity_deg1() {
  std::vector<double> c(10, 0.0);
  c[1] = 1.0;      // num_x: x
  c[5 + 2] = 1.0;  // num_y: y
  return c;
}

// increment_degree (:336-356): each of the four polynomials gets deg + 2 zero
// coefficients appended.
std::vector<double> increment_degree(const std::vector<double>& c, int d) {
  const int nl = num_len(d), m = half_size(d);
  std::vector<double> out;
  const int add = d + 2;
  for (int h = 0; h < 2; h++) {
    const double* base = c.data() + h * m;
    out.insert(out.end(), base, base + nl);
    out.insert(out.end(), add, 0.0);
    out.insert(out.end(), base + nl, base + m);
    out.insert(out.end(), add, 0.0);
  }
  return out;
}

int rpc_degree_of(int n) { return (int)std::lround(std::sqrt(2.0 * n + 5.0) / 2.0 - 1.5); }

}  // namespace mvba_rpc

extern "C" {

const char* mvba_rpc_error(void) { return mvba_rpc::g_error.c_str(); }

mvba_status mvba_rpc_fit(const mvba_rpc_camera* cam, int32_t mode, int32_t rpc_degree, const double* rpc_dist_coeffs,
                         int32_t num_samples, int32_t num_iterations, double parameter_tolerance, int32_t device,
                         double* coeffs_out, mvba_rpc_fit_report* report) {
  using namespace mvba_rpc;
  auto fail = [](mvba_status s, const std::string& m) {
    g_error = m;
    return s;
  };
  if (!cam || !coeffs_out || (cam->dist_size > 0 && !cam->dist)) return fail(MVBA_E_INVALID, "null argument");
  if (mode != MVBA_RPC_FIT_DISTORTION && mode != MVBA_RPC_FIT_UNDISTORTION)
    return fail(MVBA_E_INVALID, "unknown fit mode");
  if (num_samples < 2) return fail(MVBA_E_INVALID, "The number of samples must be at least 2.");
  const int K = cam->dist_size;
  if (!(K == 0 || K == 1 || K == 4 || K == 5 || (K > 5 && K % 2 == 0)))
    return fail(MVBA_E_BAD_DISTORTION, "Recieved irregular distortion vector size.");
  int cam_deg = 0;
  if (K > 5) {
    cam_deg = rpc_degree_of(K / 2);
    if (cam_deg <= 0 || cam_deg > mvba::kMaxRpcDegree || 2 * (cam_deg + 1) * (cam_deg + 2) - 2 != K / 2)
      return fail(MVBA_E_BAD_DISTORTION, "Recieved irregular distortion vector size.");
  }
  int d = rpc_degree;
  if (mode == MVBA_RPC_FIT_UNDISTORTION) {
    if (!rpc_dist_coeffs) return fail(MVBA_E_INVALID, "rpc_dist_coeffs is required to fit the undistortion");
    if (d <= 0 || d > mvba::kMaxRpcDegree)
      return fail(MVBA_E_INVALID, "Incorrect number of RPC coefficients.");
  } else if (d <= 0 || d > mvba::kMaxRpcDegree) {
    return fail(MVBA_E_INVALID, "The RPC degree must be positive (and at most 6).");
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MVBA_E_NO_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(MVBA_E_INVALID, "device out of range");
  if (hipSetDevice(device) != hipSuccess) return fail(MVBA_E_HIP, "hipSetDevice failed");

  const int64_t n = (int64_t)num_samples * num_samples;
  const int nd = 2 * (d + 1) * (d + 2) - 2;
  Dev dv;
  const int nblocks = (int)std::min<int64_t>((n + kChunk - 1) / kChunk, 1024);
  const int max_stride = 2 * kMaxPairs + 2 * kMaxM + 1;
  hipError_t e = hipMalloc(&dv.pairs, (size_t)n * sizeof(double4));
  if (e == hipSuccess) e = hipMalloc(&dv.valid, (size_t)n);
  if (e == hipSuccess) e = hipMalloc(&dv.coeffs, 4 * sizeof(double) * (size_t)(K + nd + 16));
  if (e == hipSuccess) e = hipMalloc(&dv.partial, (size_t)nblocks * max_stride * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&dv.sums, (size_t)max_stride * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&dv.aux, (size_t)(2 * nd + 1024) * sizeof(double));
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));

  Cam c{};
  c.f = cam->focal;
  c.cx = cam->center[0];
  c.cy = cam->center[1];
  c.W = cam->image_size[0];
  c.H = cam->image_size[1];
  c.cropW = cam->crop_size[0];
  c.cropH = cam->crop_size[1];
  c.uW = cam->undist_size[0];
  c.uH = cam->undist_size[1];
  c.dhx = c.W / 2.0;
  c.dhy = c.H / 2.0;
  c.uhx = c.uW / 2.0;
  c.uhy = c.uH / 2.0;
  c.K = K;
  for (int k = 0; k < K && k < 5; k++) c.k[k] = cam->dist[k];
  c.dist_deg = cam_deg;
  // device copies: [camera RPC distortion half | fit distortion coefficients]
  double* d_cam_rpc = dv.aux;
  double* d_fit_dist = dv.aux + nd + 512;
  if (K > 5) e = hipMemcpy(d_cam_rpc, cam->dist, (size_t)(K / 2) * sizeof(double), hipMemcpyHostToDevice);
  c.rpc = d_cam_rpc;
  if (e == hipSuccess && mode == MVBA_RPC_FIT_UNDISTORTION)
    e = hipMemcpy(d_fit_dist, rpc_dist_coeffs, (size_t)nd * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  if (K > 5 && K / 2 > nd + 512) return fail(MVBA_E_INVALID, "camera RPC degree too large");
  hipLaunchKernelGGL(k_rpc_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, c, num_samples, mode,
                     d_fit_dist, d, dv.pairs, dv.valid);
  if ((e = hipGetLastError()) != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));

  // report: pair count and centred bounding boxes (genUndistDistPairs / fitRpcUndist prints)
  std::vector<double4> hp((size_t)n);
  std::vector<uint8_t> hv((size_t)n);
  e = hipMemcpy(hp.data(), dv.pairs, (size_t)n * sizeof(double4), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(hv.data(), dv.valid, (size_t)n, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  mvba_rpc_fit_report rep{};
  const double big = 1.79769313486231570e+308;
  double ub[4] = {big, big, -big, -big}, db[4] = {big, big, -big, -big};
  for (int64_t q = 0; q < n; q++) {
    if (!hv[(size_t)q]) continue;
    rep.num_samples_used++;
    const double4 p = hp[(size_t)q];
    const double u[2] = {mode == MVBA_RPC_FIT_UNDISTORTION ? p.z : p.x, mode == MVBA_RPC_FIT_UNDISTORTION ? p.w : p.y};
    const double v[2] = {mode == MVBA_RPC_FIT_UNDISTORTION ? p.x : p.z, mode == MVBA_RPC_FIT_UNDISTORTION ? p.y : p.w};
    for (int t = 0; t < 2; t++) {
      ub[t] = std::min(ub[t], u[t]);
      ub[2 + t] = std::max(ub[2 + t], u[t]);
      db[t] = std::min(db[t], v[t]);
      db[2 + t] = std::max(db[2 + t], v[t]);
    }
  }
  std::memcpy(rep.undist_box, ub, sizeof(ub));
  std::memcpy(rep.dist_box, db, sizeof(db));
  if (rep.num_samples_used == 0) return fail(MVBA_E_INVALID, "no samples inside the distorted crop box");

  Fitter F(dv, n, nblocks);
  std::vector<double> x = identity_deg1();
  for (int deg = 1; deg <= d; deg++) {
    if (deg >= 2) x = increment_degree(x, deg - 1);
    DegreeResult r;
    e = lm_fit(F, deg, x, num_iterations, parameter_tolerance, &r);
    if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
    rep.initial_cost[deg - 1] = r.initial_cost;
    rep.final_cost[deg - 1] = r.final_cost;
    rep.iterations[deg - 1] = r.iterations;
    rep.termination[deg - 1] = r.termination;
  }
  std::memcpy(coeffs_out, x.data(), x.size() * sizeof(double));
  rep.max_dist_undist_error = -1.0;
  if (mode == MVBA_RPC_FIT_UNDISTORTION) {
    // evalRpcDistUndist with the fitted undistortion
    double* d_undist = dv.coeffs;
    e = hipMemcpy(d_undist, x.data(), x.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_rpc_roundtrip, dim3((unsigned)nblocks), dim3(kThreads), 0, 0, n, dv.pairs, dv.valid,
                         d_fit_dist, d_undist, d, dv.sums);
      e = hipGetLastError();
    }
    std::vector<double> bm((size_t)nblocks);
    if (e == hipSuccess) e = hipMemcpy(bm.data(), dv.sums, bm.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
    rep.max_dist_undist_error = *std::max_element(bm.begin(), bm.end());
  }
  if (report) *report = rep;
  return MVBA_OK;
}

}  // extern "C"
