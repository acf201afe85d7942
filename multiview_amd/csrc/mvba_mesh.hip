// mvba_mesh.hip — ray–mesh intersection for the --mesh constraints on gfx950
// (SURVEY.md §8 a13 / f4).
//
// The reference loads a PLY mesh, builds rayint's BVHTree over it
// (loadMeshBuildTree, texture_processing.cc:264-285) and per pass intersects
// every inlier feature's ray with it (ray_mesh_intersect, :1436-1479, called by
// meshTriangulations, :1566-1625). rayint itself is an empty submodule here:
// its ray-triangle test is restated from the published algorithm (see
// oracle.cpp, "mesh rays"), in float, with the mve::math::Vec3f operation order,
// and compiled without contraction so the GPU and the oracle agree bit for bit.
//
// Layout in HBM:
//   nodes  32 B each: bounds (lo, hi) + (first child | first triangle, count);
//          children of an inner node are adjacent (c, c + 1);
//   tris   3 x float4 per triangle in leaf order (a, b, c), face id in a.w bits.
// The BVH is built once per mesh on the host (median split of the centroids on
// the longest axis, leaves of <= 4 triangles, depth <= 31: the traversal stack
// of 32 entries per lane lives in LDS, [entry][lane], conflict-free).
// Traversal is latency-bound pointer chasing (a few dozen 32-B node loads and
// 48-B triangle loads per ray, mostly L2 hits for meshes of a few million
// faces); rays are visited in image-major order so a wave's rays share a camera
// centre and similar directions (coherent node sets).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <numeric>
#include <string>
#include <vector>

#include "mvba_internal.h"

namespace mvba {

struct BvhNode {
  float lo[3];
  int32_t first;  // inner: left child (right = first + 1); leaf: first triangle
  float hi[3];
  int32_t count;  // 0 = inner node
};
static_assert(sizeof(BvhNode) == 32, "node layout");

constexpr int kBvhStack = 32;
constexpr int kBvhLeaf = 4;
constexpr int kRayBlock = 256;

#pragma clang fp contract(off)

__device__ __forceinline__ float dot3f(float ax, float ay, float az, float bx, float by, float bz) {
  float s = 0.0f;
  s = s + ax * bx;
  s = s + ay * by;
  s = s + az * bz;
  return s;
}

// rayint's intersect(Ray, Tri) restated (oracle.cpp ray_tri_f, same order).
__device__ __forceinline__ bool ray_tri(float ox, float oy, float oz, float dx, float dy, float dz, float tmin,
                                        float tmax, float4 A, float4 B, float4 Cc, float* tout) {
  const float v0x = B.x - A.x, v0y = B.y - A.y, v0z = B.z - A.z;
  const float v1x = Cc.x - A.x, v1y = Cc.y - A.y, v1z = Cc.z - A.z;
  float nx = v1y * v0z - v1z * v0y, ny = v1z * v0x - v1x * v0z, nz = v1x * v0y - v1y * v0x;
  const float nn = sqrtf(dot3f(nx, ny, nz, nx, ny, nz));
  if (nn < FLT_EPSILON) return false;
  nx = nx / nn;
  ny = ny / nn;
  nz = nz / nn;
  const float cosine = dot3f(nx, ny, nz, dx, dy, dz);
  if (fabsf(cosine) < FLT_EPSILON) return false;
  const float ax = ox - A.x, ay = oy - A.y, az = oz - A.z;
  const float t = -dot3f(nx, ny, nz, ax, ay, az) / cosine;
  if (t < tmin || tmax < t) return false;
  const float v2x = ax + t * dx, v2y = ay + t * dy, v2z = az + t * dz;
  const float d00 = dot3f(v0x, v0y, v0z, v0x, v0y, v0z);
  const float d01 = dot3f(v0x, v0y, v0z, v1x, v1y, v1z);
  const float d11 = dot3f(v1x, v1y, v1z, v1x, v1y, v1z);
  const float d20 = dot3f(v2x, v2y, v2z, v0x, v0y, v0z);
  const float d21 = dot3f(v2x, v2y, v2z, v1x, v1y, v1z);
  const float denom = d00 * d11 - d01 * d01;
  const float bv = (d11 * d20 - d01 * d21) / denom;
  const float bw = (d00 * d21 - d01 * d20) / denom;
  const float bu = 1.0f - bv - bw;
  if (!(bu >= 0.0f && bv >= 0.0f && bw >= 0.0f)) return false;
  *tout = t;
  return true;
}

// Slab test against a node's (host-widened) box over [t0, t1], in double so its
// own rounding is negligible next to the float triangle test's; returns the entry
// parameter or +inf on a miss. It only prunes (the triangle test decides), so
// the caller passes a limit a little above the best hit: a box holding a hit
// whose float t ties or nearly ties the best one is still entered.
__device__ __forceinline__ double box_enter(const BvhNode& n, double ox, double oy, double oz, double ix, double iy,
                                            double iz, double t0, double t1) {
  const double ax = ((double)n.lo[0] - ox) * ix, bx = ((double)n.hi[0] - ox) * ix;
  const double ay = ((double)n.lo[1] - oy) * iy, by = ((double)n.hi[1] - oy) * iy;
  const double az = ((double)n.lo[2] - oz) * iz, bz = ((double)n.hi[2] - oz) * iz;
  const double tn = fmax(fmax(fmin(ax, bx), fmin(ay, by)), fmax(fmin(az, bz), t0));
  const double tf = fmin(fmin(fmax(ax, bx), fmax(ay, by)), fmin(fmax(az, bz), t1));
  return tn <= tf ? tn : (double)INFINITY;
}
__device__ __forceinline__ double prune_limit(float best, float tmax) {
  const double b = (double)fminf(best, tmax);
  return b + 1e-4 * fabs(b) + 1e-6;
}

// Closest hit of ray r (through perm when given). Ties in t keep the lower face id.
__global__ void __launch_bounds__(kRayBlock) k_mesh_rays(int64_t n, const int64_t* __restrict__ perm,
                                                         const float* __restrict__ orig, const float* __restrict__ dir,
                                                         float tmin, float tmax, const BvhNode* __restrict__ nodes,
                                                         const float4* __restrict__ tris, float* __restrict__ t_out,
                                                         int32_t* __restrict__ face_out) {
  __shared__ int32_t stk[kBvhStack][kRayBlock];
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t r = perm ? perm[k] : k;
  const float ox = orig[3 * r], oy = orig[3 * r + 1], oz = orig[3 * r + 2];
  const float dx = dir[3 * r], dy = dir[3 * r + 1], dz = dir[3 * r + 2];
  float best = INFINITY;
  int32_t bf = -1;
  if (!(dx == 0.0f && dy == 0.0f && dz == 0.0f)) {
    const double dox = ox, doy = oy, doz = oz;
    const double ix = 1.0 / (double)dx, iy = 1.0 / (double)dy, iz = 1.0 / (double)dz;
    const double t0 = (double)tmin - 1e-4 * fabs((double)tmin) - 1e-6;
    const int tid = threadIdx.x;
    int sp = 0;
    int32_t node = 0;
    bool recheck = true;  // the root, and every popped entry: test its box against the current best
    while (node >= 0) {
      const BvhNode nd = nodes[node];
      if (recheck && box_enter(nd, dox, doy, doz, ix, iy, iz, t0, prune_limit(best, tmax)) == (double)INFINITY) {
        node = sp > 0 ? stk[--sp][tid] : -1;
        continue;
      }
      if (nd.count > 0) {
        for (int q = 0; q < nd.count; q++) {
          const float4* tp = tris + 3 * (int64_t)(nd.first + q);
          const float4 A = tp[0], B = tp[1], Cc = tp[2];
          float t;
          if (ray_tri(ox, oy, oz, dx, dy, dz, tmin, tmax, A, B, Cc, &t)) {
            const int32_t f = __float_as_int(A.w);
            if (t < best || (t == best && f < bf)) {
              best = t;
              bf = f;
            }
          }
        }
        node = sp > 0 ? stk[--sp][tid] : -1;
        recheck = true;
      } else {
        const double lim = prune_limit(best, tmax);
        const double e0 = box_enter(nodes[nd.first], dox, doy, doz, ix, iy, iz, t0, lim);
        const double e1 = box_enter(nodes[nd.first + 1], dox, doy, doz, ix, iy, iz, t0, lim);
        const bool h0 = e0 != (double)INFINITY, h1 = e1 != (double)INFINITY;
        if (!h0 && !h1) {
          node = sp > 0 ? stk[--sp][tid] : -1;
          recheck = true;
        } else if (h0 != h1) {
          node = h0 ? nd.first : nd.first + 1;
          recheck = false;
        } else {
          const bool near0 = e0 <= e1;
          stk[sp++][tid] = near0 ? nd.first + 1 : nd.first;
          node = near0 ? nd.first : nd.first + 1;
          recheck = false;
        }
      }
    }
  }
  t_out[r] = bf < 0 ? -1.0f : best;
  face_out[r] = bf;
}

}  // namespace mvba

struct mvba_mesh {
  int device = 0;
  int64_t nv = 0, nf = 0, nnodes = 0;
  int32_t depth = 0;
  mvba::BvhNode* d_nodes = nullptr;
  float4* d_tris = nullptr;
  ~mvba_mesh() {
    if (d_nodes) (void)hipFree(d_nodes);
    if (d_tris) (void)hipFree(d_tris);
  }
};

namespace {

thread_local std::string g_mesh_error;

mvba_status mfail(mvba_status st, const std::string& m) {
  g_mesh_error = m;
  return st;
}

// Host BVH: median split of the face centroids on the longest centroid axis.
struct Builder {
  const float* v;
  const uint32_t* f;
  std::vector<float> cen;  // 3 per face
  std::vector<int32_t> idx;
  std::vector<mvba::BvhNode> nodes;
  int32_t depth = 0;

  void bounds(int64_t b, int64_t e, float* lo, float* hi) const {
    for (int q = 0; q < 3; q++) {
      lo[q] = INFINITY;
      hi[q] = -INFINITY;
    }
    for (int64_t k = b; k < e; k++)
      for (int c = 0; c < 3; c++) {
        const float* p = v + 3 * (size_t)f[3 * (size_t)idx[(size_t)k] + c];
        for (int q = 0; q < 3; q++) {
          lo[q] = std::min(lo[q], p[q]);
          hi[q] = std::max(hi[q], p[q]);
        }
      }
    // widen: the slab test in float must never cut a hit the exact test keeps
    for (int q = 0; q < 3; q++) {
      const float pad = 1e-5f * (hi[q] - lo[q]) + 1e-6f * std::max(std::fabs(lo[q]), std::fabs(hi[q])) + 1e-30f;
      lo[q] -= pad;
      hi[q] += pad;
    }
  }

  void build(int64_t nf) {
    cen.resize(3 * (size_t)nf);
    idx.resize((size_t)nf);
    for (int64_t k = 0; k < nf; k++) {
      idx[(size_t)k] = (int32_t)k;
      for (int q = 0; q < 3; q++)
        cen[3 * (size_t)k + q] = (v[3 * (size_t)f[3 * k] + q] + v[3 * (size_t)f[3 * k + 1] + q] +
                                  v[3 * (size_t)f[3 * k + 2] + q]) / 3.0f;
    }
    nodes.reserve((size_t)(2 * (nf / mvba::kBvhLeaf + 1)));
    nodes.emplace_back();
    struct Item {
      int32_t node;
      int64_t b, e;
      int32_t d;
    };
    std::vector<Item> st{{0, 0, nf, 1}};
    while (!st.empty()) {
      const Item it = st.back();
      st.pop_back();
      depth = std::max(depth, it.d);
      mvba::BvhNode& nd = nodes[(size_t)it.node];
      bounds(it.b, it.e, nd.lo, nd.hi);
      if (it.e - it.b <= mvba::kBvhLeaf) {
        nd.first = (int32_t)it.b;
        nd.count = (int32_t)(it.e - it.b);
        continue;
      }
      float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int64_t k = it.b; k < it.e; k++)
        for (int q = 0; q < 3; q++) {
          clo[q] = std::min(clo[q], cen[3 * (size_t)idx[(size_t)k] + q]);
          chi[q] = std::max(chi[q], cen[3 * (size_t)idx[(size_t)k] + q]);
        }
      int ax = 0;
      for (int q = 1; q < 3; q++)
        if (chi[q] - clo[q] > chi[ax] - clo[ax]) ax = q;
      const int64_t mid = (it.b + it.e) / 2;
      std::nth_element(idx.begin() + it.b, idx.begin() + mid, idx.begin() + it.e, [&](int32_t a, int32_t b) {
        const float ca = cen[3 * (size_t)a + ax], cb = cen[3 * (size_t)b + ax];
        return ca < cb || (ca == cb && a < b);
      });
      const int32_t c = (int32_t)nodes.size();
      nodes[(size_t)it.node].first = c;
      nodes[(size_t)it.node].count = 0;
      nodes.emplace_back();
      nodes.emplace_back();
      st.push_back({c + 1, mid, it.e, it.d + 1});
      st.push_back({c, it.b, mid, it.d + 1});
    }
  }
};

}  // namespace

extern "C" {

const char* mvba_mesh_error(void) { return g_mesh_error.c_str(); }

mvba_status mvba_mesh_create(const mvba_mesh_desc* d, int32_t device, mvba_mesh** out) {
  g_mesh_error.clear();
  if (!out) return mfail(MVBA_E_INVALID, "null output handle");
  *out = nullptr;
  if (!d) return mfail(MVBA_E_INVALID, "null mesh description");
  if (d->num_vertices < 0 || d->num_faces < 0) return mfail(MVBA_E_INVALID, "negative sizes in mesh description");
  if (d->num_faces > 0 && (!d->vertices || !d->faces)) return mfail(MVBA_E_INVALID, "null array in mesh description");
  if (d->num_faces >= (int64_t)1 << 30) return mfail(MVBA_E_INVALID, "too many faces for one mesh handle");
  for (int64_t k = 0; k < 3 * d->num_faces; k++)
    if ((int64_t)d->faces[k] >= d->num_vertices) return mfail(MVBA_E_INVALID, "face vertex index out of range");
  int32_t ndev = 0;
  if (mvba_device_count(&ndev) != MVBA_OK) return mfail(MVBA_E_NO_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return mfail(MVBA_E_INVALID, "invalid device ordinal");
  if (hipSetDevice(device) != hipSuccess) return mfail(MVBA_E_HIP, "hipSetDevice failed");
  mvba_mesh* m = new mvba_mesh();
  m->device = device;
  m->nv = d->num_vertices;
  m->nf = d->num_faces;
  Builder B{d->vertices, d->faces, {}, {}, {}, 0};
  if (m->nf > 0) B.build(m->nf);
  if (B.depth > mvba::kBvhStack) {
    delete m;
    return mfail(MVBA_E_INVALID, "BVH deeper than the traversal stack");
  }
  std::vector<float4> tris(3 * (size_t)m->nf);
  for (int64_t k = 0; k < m->nf; k++) {
    const int32_t fid = B.idx[(size_t)k];
    for (int c = 0; c < 3; c++) {
      const float* p = d->vertices + 3 * (size_t)d->faces[3 * (size_t)fid + c];
      tris[3 * (size_t)k + c] = make_float4(p[0], p[1], p[2], c == 0 ? __builtin_bit_cast(float, fid) : 0.0f);
    }
  }
  if (m->nf == 0) {  // one empty leaf: every ray misses
    B.nodes.assign(1, mvba::BvhNode{{INFINITY, INFINITY, INFINITY}, 0, {-INFINITY, -INFINITY, -INFINITY}, 0});
    B.depth = 1;
  }
  m->nnodes = (int64_t)B.nodes.size();
  m->depth = B.depth;
  hipError_t e = upload(&m->d_nodes, B.nodes);
  if (e == hipSuccess) e = upload(&m->d_tris, tris);
  if (e != hipSuccess) {
    delete m;
    return mfail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  }
  *out = m;
  return MVBA_OK;
}

void mvba_mesh_destroy(mvba_mesh* m) { delete m; }

int32_t mvba_mesh_device_ordinal(const mvba_mesh* m) { return m ? m->device : 0; }

mvba_status mvba_mesh_info(const mvba_mesh* m, int64_t* num_nodes, int32_t* depth) {
  if (!m) return mfail(MVBA_E_INVALID, "null mesh handle");
  if (num_nodes) *num_nodes = m->nnodes;
  if (depth) *depth = m->depth;
  return MVBA_OK;
}

// Internal launcher (also used by mvba_mesh_triangulate): optional ray order.
hipError_t mvba_launch_mesh_rays(const mvba_mesh* m, int64_t n, const int64_t* perm, const float* orig,
                                 const float* dir, float tmin, float tmax, float* t_out, int32_t* face_out,
                                 hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + mvba::kRayBlock - 1) / mvba::kRayBlock);
  hipLaunchKernelGGL(mvba::k_mesh_rays, dim3(blocks), dim3(mvba::kRayBlock), 0, s, n, perm, orig, dir, tmin, tmax,
                     m->d_nodes, (const float4*)m->d_tris, t_out, face_out);
  return hipGetLastError();
}

mvba_status mvba_mesh_intersect_device(mvba_mesh* m, int64_t n, const float* d_orig, const float* d_dir, float tmin,
                                       float tmax, float* d_t, int32_t* d_face, void* hip_stream) {
  g_mesh_error.clear();
  if (!m) return mfail(MVBA_E_INVALID, "null mesh handle");
  if (n < 0 || (n > 0 && (!d_orig || !d_dir || !d_t || !d_face))) return mfail(MVBA_E_INVALID, "null ray buffer");
  if (hipSetDevice(m->device) != hipSuccess) return mfail(MVBA_E_HIP, "hipSetDevice failed");
  const hipError_t e = mvba_launch_mesh_rays(m, n, nullptr, d_orig, d_dir, tmin, tmax, d_t, d_face,
                                             (hipStream_t)hip_stream);
  if (e != hipSuccess) return mfail(MVBA_E_HIP, std::string("HIP error: ") + hipGetErrorString(e));
  return MVBA_OK;
}

}  // extern "C"
