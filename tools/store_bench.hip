// store_bench.hip — write-bandwidth ceilings for K1's output pattern on gfx950.
// Pattern = P column planes of N doubles; each wavefront writes, for every plane,
// its own contiguous chunk (64 lanes x E doubles). Variants: E = 1 (dwordx2) or
// 2 (dwordx4), nontemporal or plain stores, chunk start aligned or misaligned.
// Usage: store_bench [N] [P]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int E, bool NT>
__global__ void __launch_bounds__(256) k_planes(double* __restrict__ J, long ld, int planes, long n, int shift) {
  const long wave = (long)(blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long base = wave * 64 * E + shift;
  const long i = base + (long)lane * E;
  if (i + E > n) return;
  const double v = (double)(i & 1023);
  for (int p = 0; p < planes; p++) {
    double* dst = J + (long)p * ld + i;
    if (E == 1) {
      if (NT) __builtin_nontemporal_store(v + p, dst);
      else *dst = v + p;
    } else {
      typedef double d2 __attribute__((ext_vector_type(2)));
      d2 w = {v + p, v - p};
      if (NT) __builtin_nontemporal_store(w, (d2*)dst);
      else *(d2*)dst = w;
    }
  }
}

// Buffer-store variant with explicit cache-policy bits (aux: 2 = nt, 16 = sc1
// write-through, 18 = sc1 nt); E doubles per lane (1: b64, 2: b128). One
// resource per plane (planes can exceed the 4 GiB reach of one descriptor).
template <int E, int AUX>
__global__ void __launch_bounds__(256) k_planes_buf(double* __restrict__ J, long ld, int planes, long n) {
  const long wave = (long)(blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long base = wave * 64 * E;
  const long i = base + (long)lane * E;
  if (i + E > n) return;
  const double v = (double)(i & 1023);
  for (int p = 0; p < planes; p++) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(J + (long)p * ld + base, 0, 64 * E * 8, 0x00020000);
    if (E == 1) {
      typedef unsigned int u2 __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v + p), rs, lane * 8, 0, AUX);
    } else {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      typedef double d2 __attribute__((ext_vector_type(2)));
      d2 w = {v + p, v - p};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, w), rs, lane * 16, 0, AUX);
    }
  }
}

template <int E, int AUX>
float run_buf(double* J, long ld, int planes, long n, int reps) {
  long waves = n / (64 * E);
  int blocks = (int)((waves * 64 + 255) / 256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_planes_buf<E, AUX>), dim3(blocks), dim3(256), 0, 0, J, ld, planes, n);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((k_planes_buf<E, AUX>), dim3(blocks), dim3(256), 0, 0, J, ld, planes, n);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

// Tiled variant: plane p of slot i at J[(i / 64) * planes * 64 + p * 64 + i % 64]
// (each wave streams one contiguous planes*512-B region).
__global__ void __launch_bounds__(256) k_tiled(double* __restrict__ J, int planes, long n) {
  const long wave = (long)(blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long i = wave * 64 + lane;
  if (i >= n) return;
  const double v = (double)(i & 1023);
  double* dst = J + wave * (long)planes * 64 + lane;
  for (int p = 0; p < planes; p++) __builtin_nontemporal_store(v + p, dst + (long)p * 64);
}

float run_tiled(double* J, int planes, long n, int reps) {
  int blocks = (int)((n + 255) / 256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_tiled, dim3(blocks), dim3(256), 0, 0, J, planes, n);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_tiled, dim3(blocks), dim3(256), 0, 0, J, planes, n);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int E, bool NT>
float run(double* J, long ld, int planes, long n, int shift, int reps) {
  long waves = (n - shift) / (64 * E);
  int blocks = (int)((waves * 64 + 255) / 256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_planes<E, NT>), dim3(blocks), dim3(256), 0, 0, J, ld, planes, n, shift);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((k_planes<E, NT>), dim3(blocks), dim3(256), 0, 0, J, ld, planes, n, shift);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

// Sweep of the plane stride: ld = round_up(n, 64) + pad for pad = 0, 64, ...
// (doubles), dwordx2 nt stores, aligned chunks.
int sweep(long n, int planes, long max_pad, long step) {
  const long ld0 = ((n + 63) / 64) * 64;
  double* J;
  CHECK(hipMalloc(&J, sizeof(double) * (ld0 + max_pad) * planes));
  const double bytes = 8.0 * n * planes;
  for (long pad = 0; pad <= max_pad; pad += step) {
    const long ld = ld0 + pad;
    float ms = run<1, true>(J, ld, planes, n, 0, 20);
    printf("sweep ld %ld (pad %ld, stride %ld B, stride mod 64K %ld) %8.4f ms %7.1f GB/s\n", ld, pad, ld * 8,
           (ld * 8) % 65536, ms, bytes / (ms * 1e-3) / 1e9);
  }
  CHECK(hipFree(J));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 's')
    return sweep(argc > 2 ? atol(argv[2]) : 1000000, argc > 3 ? atoi(argv[3]) : 66, argc > 4 ? atol(argv[4]) : 4096,
                 argc > 5 ? atol(argv[5]) : 64);
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  int planes = argc > 2 ? atoi(argv[2]) : 56;
  long ld = ((n + 255) / 256) * 256;
  double* J;
  CHECK(hipMalloc(&J, sizeof(double) * ld * planes));
  const double bytes = 8.0 * n * planes;
  struct { const char* name; float ms; } res[24];
  int k = 0;
  res[k++] = {"dwordx2 nt   aligned", run<1, true>(J, ld, planes, n, 0, 20)};
  res[k++] = {"dwordx2 plain aligned", run<1, false>(J, ld, planes, n, 0, 20)};
  res[k++] = {"dwordx4 nt   aligned", run<2, true>(J, ld, planes, n, 0, 20)};
  res[k++] = {"dwordx4 plain aligned", run<2, false>(J, ld, planes, n, 0, 20)};
  res[k++] = {"dwordx2 nt   shift 8B", run<1, true>(J, ld, planes, n, 1, 20)};
  res[k++] = {"dwordx4 nt   shift 16B", run<2, true>(J, ld, planes, n, 2, 20)};
  res[k++] = {"tiled 64 x planes nt", run_tiled(J, planes, n, 20)};
  res[k++] = {"buf b64 plain", run_buf<1, 0>(J, ld, planes, n, 20)};
  res[k++] = {"buf b64 nt", run_buf<1, 2>(J, ld, planes, n, 20)};
  res[k++] = {"buf b64 sc1", run_buf<1, 16>(J, ld, planes, n, 20)};
  res[k++] = {"buf b128 plain", run_buf<2, 0>(J, ld, planes, n, 20)};
  res[k++] = {"buf b128 nt", run_buf<2, 2>(J, ld, planes, n, 20)};
  res[k++] = {"buf b128 sc1", run_buf<2, 16>(J, ld, planes, n, 20)};
  res[k++] = {"buf b128 sc1 nt", run_buf<2, 18>(J, ld, planes, n, 20)};
  CHECK(hipFree(J));
  // leading-dimension padding: planes 8 MB apart may share DRAM channels
  const long pads[5] = {64, 512 + 64, 4096 + 64, 32768 + 192, 1 << 16};
  std::vector<double*> keep;
  for (int q = 0; q < 5; q++) {
    const long ldp = ld + pads[q];
    double* Jp;
    CHECK(hipMalloc(&Jp, sizeof(double) * ldp * planes));
    float ms = run<1, true>(Jp, ldp, planes, n, 0, 20);
    printf("dwordx2 nt ld+%-8ld    %8.3f ms  %7.1f GB/s\n", pads[q], ms, bytes / (ms * 1e-3) / 1e9);
    CHECK(hipFree(Jp));
  }
  CHECK(hipMalloc(&J, sizeof(double) * ld * planes));
  for (int i = 0; i < k; i++)
    printf("%-24s %8.3f ms  %7.1f GB/s\n", res[i].name, res[i].ms, bytes / (res[i].ms * 1e-3) / 1e9);
  CHECK(hipFree(J));
  return 0;
}
