// chol_bench.hip — pricing microbench for DESIGN.md §5 "Why the reduced camera
// system is not formed" (X1): a hand-written fp64-MFMA blocked Cholesky of a
// dense SPD matrix of the c3 reduced camera system's size, the same
// factorization by rocSOLVER's dpotrf beside it, and the trailing-update GEMM
// alone. Measurement tooling only (not part of libmvba).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chol_bench.hip -lrocsolver -lrocblas -o tools/chol_bench
//   tools/chol_bench [n]            (n a multiple of 256; default 21248)
//
// Blocked right-looking factorization, column-major lower (A = L L^T):
//   for every 256 columns K0:
//     for every 64 columns k of the panel:
//       k_potrf64   one wave: the 64x64 diagonal block in LDS, and its inverse
//       TRSM        A[k+64:, k:k+64] = A[k+64:, k:k+64] Linv^T     (k_dgemm_nt, K = 64)
//       panel       A[k+64:, k+64:K0+256] -= A[k+64:, k:k+64] A[k+64:K0+256, k:k+64]^T
//     trailing      A[K0+256:, K0+256:] -= P P^T, P = A[K0+256:, K0:K0+256]   (lower tiles, K = 256)
// k_dgemm_nt: 128x128 output tile per 256-thread block, each wave a 64x64
// quarter as 4x4 v_mfma_f64_16x16x4f64 tiles (64 accumulators per lane), the
// K dimension staged through LDS in chunks of 16 (double-buffered, register
// prefetch of the next chunk, row stride 144 doubles: conflict-free fragment
// reads).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

using d4 = __attribute__((ext_vector_type(4))) double;

constexpr int kTile = 128;  // output tile (rows and columns)
constexpr int kKc = 16;     // K chunk staged in LDS
constexpr int kLdsLd = 144; // LDS row stride (doubles): k rows 32 banks apart

// C[M x N] = beta C + alpha A[M x K] B[N x K]^T, column-major. LOWER: only the
// entries with (row + crow0) >= (col + ccol0) are written (tiles entirely above
// that diagonal exit). M, N multiples of 8; K a multiple of 16. The block owns
// the rows of its tile: with N <= 128 the product may run in place (C == A).
template <bool LOWER>
__global__ void __launch_bounds__(256, 2) k_dgemm_nt(int M, int N, int K, double alpha, double beta,
                                                     const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ B, int64_t ldb, double* C,
                                                     int64_t ldc, int64_t crow0, int64_t ccol0) {
  const int m0 = blockIdx.x * kTile, n0 = blockIdx.y * kTile;
  if (LOWER && crow0 + m0 + kTile - 1 < ccol0 + n0) return;
  __shared__ double As[2][kKc][kLdsLd];
  __shared__ double Bs[2][kKc][kLdsLd];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  // staging: thread t moves 8 consecutive rows of column k of the A and B tiles
  const int sk = t >> 4, sm = (t & 15) * 8;
  const bool a_in = m0 + sm < M, b_in = n0 + sm < N;
  double ra[8], rb[8];
  auto load = [&](int k0) {
    const double* a = A + (int64_t)(k0 + sk) * lda + m0 + sm;
    const double* b = B + (int64_t)(k0 + sk) * ldb + n0 + sm;
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
      const double2 va = a_in ? *reinterpret_cast<const double2*>(a + q) : double2{0.0, 0.0};
      const double2 vb = b_in ? *reinterpret_cast<const double2*>(b + q) : double2{0.0, 0.0};
      ra[q] = va.x; ra[q + 1] = va.y;
      rb[q] = vb.x; rb[q + 1] = vb.y;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
      *reinterpret_cast<double2*>(&As[buf][sk][sm + q]) = double2{ra[q], ra[q + 1]};
      *reinterpret_cast<double2*>(&Bs[buf][sk][sm + q]) = double2{rb[q], rb[q + 1]};
    }
  };
  const int nchunks = K / kKc;
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int c = 0; c < nchunks; c++) {
    const int buf = c & 1;
    if (c + 1 < nchunks) load((c + 1) * kKc);
#pragma unroll
    for (int kk = 0; kk < kKc; kk += 4) {
      double fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; i++) fa[i] = As[buf][kk + fk][wm + 16 * i + fr];
#pragma unroll
      for (int j = 0; j < 4; j++) fb[j] = Bs[buf][kk + fk][wn + 16 * j + fr];
      // D[r][c] with r along N (the "A" operand: B's rows) and c along M: the
      // output lanes then run down C's columns (contiguous, column-major)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (c + 1 < nchunks) store(buf ^ 1);
    __syncthreads();
  }
  // acc[i][j] register q: n = wn + 16 j + (lane >> 4) + 4 q, m = wm + 16 i + (lane & 15)
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int m = m0 + wm + 16 * i + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int n = n0 + wn + 16 * j + fk + 4 * q;
        if (n >= N || (LOWER && crow0 + m < ccol0 + n)) continue;
        double* p = C + (int64_t)n * ldc + m;
        const double v = alpha * acc[i][j][q];
        *p = beta == 0.0 ? v : beta * *p + v;
      }
  }
}

// One wave: Cholesky of the 64x64 diagonal block at (k, k) in LDS (lane i owns
// row i), written back in place (lower), and its inverse into linv (64 x 64,
// column-major, lane c forms column c by forward substitution).
__global__ void __launch_bounds__(64) k_potrf64(double* A, int64_t lda, int64_t k, double* __restrict__ linv,
                                               int* __restrict__ info) {
  __shared__ double L[64][65];
  __shared__ double X[64][65];
  const int i = threadIdx.x;
  for (int j = 0; j <= i; j++) L[i][j] = A[(k + j) * lda + k + i];
  for (int j = i + 1; j < 64; j++) L[i][j] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int j = 0; j < 64; j++) {
    const double d = L[j][j];
    if (!(d > 0.0)) {
      if (i == 0) *info = (int)(k + j + 1);
      return;
    }
    const double s = sqrt(d);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (i > j) L[i][j] /= s;
    if (i == j) L[j][j] = s;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (i > j) {
      const double lij = L[i][j];
      for (int l = j + 1; l <= i; l++) L[i][l] -= lij * L[l][j];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // column c = i of L^-1
  const int c = i;
  for (int r = 0; r < c; r++) X[r][c] = 0.0;
  for (int r = c; r < 64; r++) {
    double s = (r == c) ? 1.0 : 0.0;
    for (int l = c; l < r; l++) s -= L[r][l] * X[l][c];
    X[r][c] = s / L[r][r];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int j = 0; j <= i; j++) A[(k + j) * lda + k + i] = L[i][j];
  for (int r = 0; r < 64; r++) linv[(int64_t)i * 64 + r] = X[r][i];  // column i
}

// SPD test matrix: A = S + S^T + 2n I with S uniform in [0, 1) (hash of (i, j)).
__device__ __forceinline__ double uhash(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}
__global__ void k_fill(double* A, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * n) return;
  const int64_t i = t % n, j = t / n;
  double v = uhash((uint64_t)i * 0x9E3779B97F4A7C15ULL + (uint64_t)j) + uhash((uint64_t)j * 0x9E3779B97F4A7C15ULL + (uint64_t)i);
  if (i == j) v += 2.0 * (double)n;
  A[t] = v;
}

// sampled check of L L^T = A0: one thread per sample (i >= j)
__global__ void k_check(const double* L, const double* A0, int64_t n, int ns, double* err) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  int64_t i = (int64_t)(uhash(7ULL * s + 1) * n), j = (int64_t)(uhash(13ULL * s + 5) * n);
  if (i < j) { const int64_t tmp = i; i = j; j = tmp; }
  double v = 0.0;
  for (int64_t l = 0; l <= j; l++) v += L[l * n + i] * L[l * n + j];
  err[s] = fabs(v - A0[j * n + i]) / fabs(A0[j * n + i]);
}

static void gemm(bool lower, int M, int N, int K, double alpha, double beta, const double* A, int64_t lda,
                 const double* B, int64_t ldb, double* C, int64_t ldc, int64_t crow0, int64_t ccol0, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  dim3 grid((M + kTile - 1) / kTile, (N + kTile - 1) / kTile);
  if (lower)
    hipLaunchKernelGGL(k_dgemm_nt<true>, grid, dim3(256), 0, s, M, N, K, alpha, beta, A, lda, B, ldb, C, ldc, crow0, ccol0);
  else
    hipLaunchKernelGGL(k_dgemm_nt<false>, grid, dim3(256), 0, s, M, N, K, alpha, beta, A, lda, B, ldb, C, ldc, crow0, ccol0);
}

static void factor(double* A, int64_t n, double* linv, int* info, hipStream_t s) {
  const int64_t lda = n;
  for (int64_t K0 = 0; K0 < n; K0 += 256) {
    for (int64_t k = K0; k < K0 + 256; k += 64) {
      hipLaunchKernelGGL(k_potrf64, dim3(1), dim3(64), 0, s, A, lda, k, linv, info);
      const int64_t below = n - k - 64;
      double* P = A + k * lda + k + 64;  // A[k+64:, k:k+64]
      gemm(false, (int)below, 64, 64, 1.0, 0.0, P, lda, linv, 64, P, lda, 0, 0, s);  // TRSM as GEMM, in place
      const int64_t pw = K0 + 256 - (k + 64);                                          // rest of the panel
      if (pw > 0)
        gemm(true, (int)below, (int)pw, 64, -1.0, 1.0, P, lda, P, lda, A + (k + 64) * lda + k + 64, lda, k + 64, k + 64,
             s);
    }
    const int64_t rest = n - K0 - 256;
    if (rest > 0) {
      const double* P = A + K0 * lda + K0 + 256;  // A[K0+256:, K0:K0+256]
      gemm(true, (int)rest, (int)rest, 256, -1.0, 1.0, P, lda, P, lda, A + (K0 + 256) * lda + K0 + 256, lda, K0 + 256,
           K0 + 256, s);
    }
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 21248;
  if (n % 256) { std::fprintf(stderr, "n must be a multiple of 256\n"); return 2; }
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  double *A, *A0, *linv, *err;
  int* info;
  const size_t bytes = (size_t)n * n * sizeof(double);
  CHK(hipMalloc(&A, bytes));
  CHK(hipMalloc(&A0, bytes));
  CHK(hipMalloc(&linv, 64 * 64 * sizeof(double)));
  CHK(hipMalloc(&info, sizeof(int)));
  const int ns = 4096;
  CHK(hipMalloc(&err, ns * sizeof(double)));
  const unsigned fb = (unsigned)((n * n + 255) / 256);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, s, A0, n);
  CHK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double flops = (double)n * n * n / 3.0;
  std::printf("n = %lld (%.2f GB fp64), n^3/3 = %.3e flop\n", (long long)n, bytes / 1e9, flops);

  // 1) the trailing-update GEMM alone at the first step's shape (M = N = n - 256, K = 256, lower)
  {
    CHK(hipMemcpyAsync(A, A0, bytes, hipMemcpyDeviceToDevice, s));
    const int64_t m = n - 256;
    for (int rep = 0; rep < 2; rep++) gemm(true, (int)m, (int)m, 256, -1e-9, 1.0, A + 256, n, A + 256, n, A + 256 * n + 256, n, 256, 256, s);
    CHK(hipEventRecord(e0, s));
    const int reps = 5;
    for (int rep = 0; rep < reps; rep++) gemm(true, (int)m, (int)m, 256, -1e-9, 1.0, A + 256, n, A + 256, n, A + 256 * n + 256, n, 256, 256, s);
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double f = (double)m * m * 256;  // lower half of 2 m^2 K
    std::printf("trailing update (lower, M = N = %lld, K = 256): %.3f ms, %.1f TFLOP/s useful (%.1f TFLOP/s issued)\n",
                (long long)m, ms, f / (ms * 1e-3) / 1e12, (f + (double)m * 128 * 256 * 2) / (ms * 1e-3) / 1e12);
  }
  // 2) hand-written blocked Cholesky
  double best_hand = 1e30;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipMemcpyAsync(A, A0, bytes, hipMemcpyDeviceToDevice, s));
    CHK(hipMemsetAsync(info, 0, sizeof(int), s));
    CHK(hipEventRecord(e0, s));
    factor(A, n, linv, info, s);
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    int hinfo = 0;
    CHK(hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost));
    if (hinfo) { std::printf("hand-written: not positive definite at %d\n", hinfo); return 1; }
    best_hand = std::min(best_hand, (double)ms);
    std::printf("hand-written blocked Cholesky (fp64 MFMA): %.2f ms = %.1f TFLOP/s (%.2f of 78.6)\n", ms,
                flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 1e12 / 78.6);
  }
  hipLaunchKernelGGL(k_check, dim3((ns + 255) / 256), dim3(256), 0, s, A, A0, n, ns, err);
  std::vector<double> herr(ns);
  CHK(hipMemcpy(herr.data(), err, ns * sizeof(double), hipMemcpyDeviceToHost));
  double emax = 0;
  for (double v : herr) emax = std::max(emax, v);
  std::printf("hand-written: max relative error of L L^T over %d sampled entries: %.2e\n", ns, emax);

  // 3) rocSOLVER dpotrf on the same matrix
  rocblas_handle rh;
  rocblas_create_handle(&rh);
  rocblas_set_stream(rh, s);
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipMemcpyAsync(A, A0, bytes, hipMemcpyDeviceToDevice, s));
    CHK(hipEventRecord(e0, s));
    rocblas_status st = rocsolver_dpotrf(rh, rocblas_fill_lower, (rocblas_int)n, A, (rocblas_int)n, info);
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    int hinfo = 0;
    CHK(hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost));
    std::printf("rocsolver_dpotrf: status %d info %d, %.2f ms = %.1f TFLOP/s (%.2f of 78.6)\n", (int)st, hinfo, ms,
                flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 1e12 / 78.6);
  }
  hipLaunchKernelGGL(k_check, dim3((ns + 255) / 256), dim3(256), 0, s, A, A0, n, ns, err);
  CHK(hipMemcpy(herr.data(), err, ns * sizeof(double), hipMemcpyDeviceToHost));
  emax = 0;
  for (double v : herr) emax = std::max(emax, v);
  std::printf("rocsolver: max relative error of L L^T over %d sampled entries: %.2e\n", ns, emax);
  rocblas_destroy_handle(rh);
  return 0;
}
