// mvba_stats.hip — evalResiduals + calc_residuals_stats on the GPU
// (rig_calibrator.cc:1157-1180, :753-789).
//
// The reference evaluates all residuals (Problem::Evaluate, no loss), divides
// each by its residual scale (1 for pixels, depth_tri_weight for depth
// residuals), groups |r| by residual name (<sensor>_pix_x, <sensor>_pix_y,
// depth_tri_{x,y,z}_m, tri_*, depth_mesh_*, mesh_tri_*), sorts each group and prints vals[int(0.25 len)],
// vals[int(0.5 len)], vals[int(0.75 len)], vals[len - 1].
// Here: one key per residual component (bits of |r|/scale: non-negative doubles
// order like their bit patterns) and its group; two stable LSD radix sorts (by
// value, then by group) leave every group contiguous and sorted; group starts
// come from adjacent-key comparison; the host picks the percentile indices.
#include <hipcub/hipcub.hpp>

#include "mvba_internal.h"

namespace mvba {

// Reprojection slots: group 2*cam + component; padding slots -> sentinel group.
// Depth blocks: groups 2*ncam + k; XYZ priors (--tri_weight): 2*ncam + 3 + k;
// depth_mesh 2*ncam + 6 + k; mesh_tri priors 2*ncam + 9 + k.
__global__ void k_stats_keys_cam(const Segment* __restrict__ segs, int32_t nseg, const FrameDesc* __restrict__ fd,
                                 const double* __restrict__ res, int64_t ld, int64_t nslots,
                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ groups) {
  const int seg = blockIdx.x;
  if (seg >= nseg) return;
  const Segment sg = segs[seg];
  const int lane = threadIdx.x;
  if (lane >= sg.count) return;
  const int64_t i = (int64_t)sg.begin + lane;
  const int cam = fd[sg.frame].cam;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const double v = fabs(res[k * ld + i]);
    keys[k * nslots + i] = __double_as_longlong(v);
    groups[k * nslots + i] = (uint32_t)(2 * cam + k);
  }
}

// Depth slots: group g0 + component (depth_tri), g0 + 6 + component for the
// BracketedDepthMeshError blocks (depth_mesh: their point is a virtual one,
// index >= pid_mesh0); value |r| / weight.
__global__ void k_stats_keys_depth(int64_t nslots, const int64_t* __restrict__ dorder,
                                   const DepthDesc* __restrict__ dd, int32_t pid_mesh0,
                                   const double4* __restrict__ dmeas, const double* __restrict__ dres, int64_t ld,
                                   uint32_t g0, uint64_t* __restrict__ keys, uint32_t* __restrict__ groups) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots || dorder[i] < 0) return;
  const double w = dmeas[i].w;
  const uint32_t gb = g0 + (dd[i].pid >= pid_mesh0 ? 6u : 0u);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const double v = fabs(dres[k * ld + i] / w);
    keys[k * nslots + i] = __double_as_longlong(v);
    groups[k * nslots + i] = gb + k;
  }
}

// XYZError prior blocks: group g0 + component, value |w (X - ref)| / w (the
// reference divides the raw residual by its scale, rig_calibrator.cc:1172-1173).
// mesh_tri priors (kind 1) go to g0 + 6 + component.
__global__ void k_stats_keys_xyz(int64_t n, const int32_t* __restrict__ xpid, const double4* __restrict__ xref,
                                 const uint8_t* __restrict__ xkind, const double4* __restrict__ pts, uint32_t g0,
                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ groups) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double4 X = pts[xpid[j]];
  const double4 R = xref[j];
  const double d[3] = {X.x - R.x, X.y - R.y, X.z - R.z};
  const uint32_t gb = g0 + (xkind[j] ? 6u : 0u);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const double v = fabs((R.w * d[k]) / R.w);
    keys[k * n + j] = __double_as_longlong(v);
    groups[k * n + j] = gb + k;
  }
}

__global__ void k_fill_sentinel(int64_t n, uint64_t* __restrict__ keys, uint32_t* __restrict__ groups,
                                uint32_t sentinel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = 0;
  groups[i] = sentinel;
}

// start[g] = first index of group g in the group-sorted array (ngroups+1 entries,
// pre-set to n); written only at boundaries, so no atomics.
__global__ void k_group_starts(int64_t n, const uint32_t* __restrict__ g, int64_t* __restrict__ start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i == 0 || g[i] != g[i - 1]) start[g[i]] = i;
}

__global__ void k_gather_u64(int32_t m, const int64_t* __restrict__ idx, const uint64_t* __restrict__ v,
                             double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) out[t] = idx[t] >= 0 ? __longlong_as_double((long long)v[idx[t]]) : NAN;
}

__global__ void k_fill_i64(int64_t n, int64_t v, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = v;
}

}  // namespace mvba

extern "C" {

mvba_status mvba_residual_stats(mvba_handle* h, double* out, int64_t* counts, void* stream) {
  if (!h || !out || !counts) return MVBA_E_INVALID;
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  // raw residuals (Problem::Evaluate with apply_loss_function = false)
  mvba_device_view v;
  mvba_status st = mvba_device_buffers(h, &v);
  if (st != MVBA_OK) return st;
  st = mvba_evaluate_device(h, MVBA_EVAL_RESIDUALS, 0.0, v.residuals, nullptr, v.ld, stream);
  if (st != MVBA_OK) return st;
  if (h->ndep > 0) {
    if (!h->d_dres) {
      h->dld = (h->ndep_slots + 63) / 64 * 64;
      hipError_t e = dalloc(&h->d_dres, (size_t)(3 * h->dld));
      if (e == hipSuccess) e = dalloc(&h->d_dJ, (size_t)MVBA_DJAC_ROWS * (size_t)h->dld);
      if (e != hipSuccess) return h->hip_fail(e, "allocating depth outputs");
    }
    st = mvba_evaluate_depth_device(h, MVBA_EVAL_RESIDUALS | MVBA_EVAL_SKIP_PREP, 0.0, h->d_dres, nullptr, h->dld,
                                    stream);
    if (st != MVBA_OK) return st;
  }
  const int32_t ncam_groups = 2 * h->ncams;
  const int32_t ngroups = ncam_groups + 12;
  const uint32_t sentinel = (uint32_t)ngroups;
  const int64_t n_cam = 2 * h->nslots, n_dep = 3 * h->ndep_slots, n_xyz = 3 * h->nxyz, n = n_cam + n_dep + n_xyz;
  hipError_t e = hipSuccess;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *g0 = nullptr, *g1 = nullptr;
  int64_t *start = nullptr, *pick = nullptr;
  double* vals = nullptr;
  void* temp = nullptr;
  size_t tb1 = 0, tb2 = 0;
  auto chk = [&](hipError_t x) {
    if (e == hipSuccess && x != hipSuccess) e = x;
  };
  chk(dalloc(&k0, (size_t)n));
  chk(dalloc(&k1, (size_t)n));
  chk(dalloc(&g0, (size_t)n));
  chk(dalloc(&g1, (size_t)n));
  chk(dalloc(&start, (size_t)ngroups + 2));
  chk(dalloc(&pick, (size_t)4 * ngroups));
  chk(dalloc(&vals, (size_t)4 * ngroups));
  int gbits = 1;
  while ((1u << gbits) <= sentinel) gbits++;
  if (e == hipSuccess) {
    chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tb1, k0, k1, g0, g1, (int)n, 0, 64, s));
    chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, g1, g0, k1, k0, (int)n, 0, gbits, s));
    chk(hipMalloc(&temp, std::max<size_t>(std::max(tb1, tb2), 1)));
  }
  if (e == hipSuccess && n > 0) {
    const unsigned b = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(mvba::k_fill_sentinel, dim3(b), dim3(256), 0, s, n, k0, g0, sentinel);
    if (h->groups.size() && h->nslots)
      hipLaunchKernelGGL(mvba::k_stats_keys_cam, dim3((unsigned)h->nsegs), dim3(64), 0, s, h->d_segs,
                         (int32_t)h->nsegs, h->d_fd, v.residuals, v.ld, h->nslots, k0, g0);
    if (h->ndep > 0)
      hipLaunchKernelGGL(mvba::k_stats_keys_depth, dim3((unsigned)((h->ndep_slots + 255) / 256)), dim3(256), 0, s,
                         h->ndep_slots, h->d_dep_order, h->d_dep_desc, (int32_t)h->npts_user, h->d_dep_meas,
                         h->d_dres, h->dld, (uint32_t)ncam_groups,
                         k0 + n_cam, g0 + n_cam);
    if (h->nxyz > 0)
      hipLaunchKernelGGL(mvba::k_stats_keys_xyz, dim3((unsigned)((h->nxyz + 255) / 256)), dim3(256), 0, s, h->nxyz,
                         h->d_xpid, h->d_xref, h->d_xkind, h->d_pts, (uint32_t)(ncam_groups + 3), k0 + n_cam + n_dep,
                         g0 + n_cam + n_dep);
    size_t t1 = tb1, t2 = tb2;
    chk(hipcub::DeviceRadixSort::SortPairs(temp, t1, k0, k1, g0, g1, (int)n, 0, 64, s));   // by value
    chk(hipcub::DeviceRadixSort::SortPairs(temp, t2, g1, g0, k1, k0, (int)n, 0, gbits, s)); // stable by group
    hipLaunchKernelGGL(mvba::k_fill_i64, dim3((unsigned)((ngroups + 2 + 63) / 64)), dim3(64), 0, s, (int64_t)ngroups + 2, n,
                       start);
    hipLaunchKernelGGL(mvba::k_group_starts, dim3(b), dim3(256), 0, s, n, g0, start);
  }
  std::vector<int64_t> hstart((size_t)ngroups + 2, n);
  if (e == hipSuccess && n > 0)
    chk(hipMemcpyAsync(hstart.data(), start, hstart.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  if (e == hipSuccess) chk(hipStreamSynchronize(s));
  // group g spans [start[g], next start present); absent groups have start == n
  std::vector<int64_t> hpick((size_t)4 * ngroups, -1);
  if (e == hipSuccess) {
    for (int g = 0; g < ngroups; g++) {
      int64_t L = 0;
      if (hstart[g] < n) {
        int64_t hi = n;  // next present group (the sentinel group of padding slots sorts last)
        for (int q = g + 1; q <= ngroups; q++)
          if (hstart[q] < n) {
            hi = hstart[q];
            break;
          }
        L = hi - hstart[g];
      }
      counts[g] = L;
      if (L > 0) {  // calc_residuals_stats: vals[int(0.25 len)], ..., vals[len - 1]
        hpick[4 * g + 0] = hstart[g] + (int64_t)(0.25 * (double)L);
        hpick[4 * g + 1] = hstart[g] + (int64_t)(0.50 * (double)L);
        hpick[4 * g + 2] = hstart[g] + (int64_t)(0.75 * (double)L);
        hpick[4 * g + 3] = hstart[g] + L - 1;
      }
    }
    chk(hipMemcpyAsync(pick, hpick.data(), hpick.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(mvba::k_gather_u64, dim3((unsigned)((4 * ngroups + 255) / 256)), dim3(256), 0, s, 4 * ngroups, pick,
                       k0, vals);
    chk(hipMemcpyAsync(out, vals, (size_t)4 * ngroups * sizeof(double), hipMemcpyDeviceToHost, s));
    chk(hipStreamSynchronize(s));
  }
  for (void* p : {(void*)k0, (void*)k1, (void*)g0, (void*)g1, (void*)start, (void*)pick, (void*)vals, temp})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_residual_stats");
  return mvba_sync_status(h, stream);
}

}  // extern "C"
