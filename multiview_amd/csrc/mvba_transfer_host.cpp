// mvba_transfer_host.cpp — host hand-over of evaluations: mvba_evaluate,
// mvba_evaluate_packed, mvba_evaluate_depth and the pinned-memory helpers.
//
// Replaces what Problem::Evaluate / CostFunction::Evaluate hand to Ceres
// (rig_calibrator.cc:1157-1180 evalResiduals; :1674-1699 the cost functions).
// The device evaluates into column planes (K1), k_rows (mvba_transfer.hip)
// rewrites them as AddResidualBlock-order rows with the Cauchy corrector
// applied, and ONE device-to-host copy moves the rows: straight into the
// destination when it is pinned (mvba_host_alloc, or hipHostRegister'ed by the
// caller), else through two pinned staging buffers whose DMA overlaps the
// host-side copy of the previous chunk.
#include <omp.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "mvba_internal.h"

namespace {

std::mutex g_pinned_mu;
std::map<uintptr_t, size_t> g_pinned;  // mvba_host_alloc'ed ranges

bool registered_pinned(const void* p, size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    auto it = g_pinned.upper_bound((uintptr_t)p);
    if (it != g_pinned.begin()) {
      --it;
      if ((uintptr_t)p >= it->first && (uintptr_t)p + bytes <= it->first + it->second) return true;
    }
  }
  // caller-registered memory (hipHostRegister / hipHostMalloc outside the library)
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost && attr.devicePointer != nullptr;
}

constexpr size_t kStageBytes = size_t(32) << 20;

void par_copy(char* dst, const char* src, size_t n) {
  const size_t kPiece = size_t(1) << 20;
  const int64_t pieces = (int64_t)((n + kPiece - 1) / kPiece);
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < pieces; k++) {
    const size_t off = (size_t)k * kPiece;
    std::memcpy(dst + off, src + off, std::min(kPiece, n - off));
  }
}

}  // namespace

// Device -> host of `bytes` on the default stream; returns when the data is on the host.
static mvba_status copy_to_host(mvba_handle* h, void* dst, const void* src, size_t bytes, const char* what) {
  if (bytes == 0) return MVBA_OK;
  hipError_t e;
  if (registered_pinned(dst, bytes)) {
    e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return h->hip_fail(e, what);
    return MVBA_OK;
  }
  if (!h->h_stage[0]) {
    for (int k = 0; k < 2; k++) {
      e = hipHostMalloc(&h->h_stage[k], kStageBytes, hipHostMallocDefault);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&h->stage_ev[k], hipEventDisableTiming);
      if (e != hipSuccess) return h->hip_fail(e, "allocating pinned staging");
    }
    h->stage_bytes = kStageBytes;
  }
  const size_t C = h->stage_bytes;
  const size_t nchunks = (bytes + C - 1) / C;
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  for (size_t k = 0; k <= nchunks; k++) {
    if (k < nchunks) {
      // stage[k&1] was last used by chunk k-2, copied out during iteration k-1
      e = hipMemcpyAsync(h->h_stage[k & 1], s + k * C, std::min(C, bytes - k * C), hipMemcpyDeviceToHost, nullptr);
      if (e == hipSuccess) e = hipEventRecord(h->stage_ev[k & 1], nullptr);
      if (e != hipSuccess) return h->hip_fail(e, what);
    }
    if (k > 0) {
      const size_t j = k - 1;
      e = hipEventSynchronize(h->stage_ev[j & 1]);
      if (e != hipSuccess) return h->hip_fail(e, what);
      par_copy(d + j * C, static_cast<const char*>(h->h_stage[j & 1]), std::min(C, bytes - j * C));
    }
  }
  return MVBA_OK;
}

static mvba_status ensure_dev(mvba_handle* h, double** p, size_t n, const char* what) {
  if (*p) return MVBA_OK;
  hipError_t e = dalloc(p, n);
  if (e != hipSuccess) return h->hip_fail(e, what);
  return MVBA_OK;
}

static mvba_rows_layout cam_layout(const mvba_handle* h) {
  mvba_rows_layout L;
  L.jac_rows = h->jac_rows;
  L.nres = 2;
  L.nblocks = 8;
  L.var_block = MVBA_BLK_DIST;
  const int base[8] = {MVBA_JAC_BASE_BEG, MVBA_JAC_BASE_END, MVBA_JAC_BASE_REF_TO_CAM, MVBA_JAC_BASE_XYZ,
                       MVBA_JAC_BASE_OFFSET, MVBA_JAC_BASE_FOCAL, MVBA_JAC_BASE_CENTER, MVBA_JAC_BASE_DIST};
  for (int b = 0; b < 8; b++) {
    L.base[b] = base[b];
    L.size[b] = b < 7 ? kFixedSize[b] : 0;
  }
  return L;
}

static double cauchy_c_of(int32_t flags, double thr) { return (flags & MVBA_EVAL_APPLY_LOSS) ? 1.0 / (thr * thr) : 0.0; }

// Evaluate on the device and rewrite the planes as rows (full layout when
// packed == false). Leaves d_tres / d_tcost / d_trows filled, stream synced.
// pinned_dst (packed layout only): the rows are produced in slot-range chunks
// and each chunk's rows (contiguous: device order) are copied to pinned_dst on
// a second stream while the next chunk is transposed; then the copy is done too.
static mvba_status eval_rows(mvba_handle* h, int32_t flags, double thr, bool want_jac, bool packed, bool want_cost,
                             double* pinned_dst = nullptr) {
  const bool loss = (flags & MVBA_EVAL_APPLY_LOSS) != 0;
  if (loss && !(thr > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
  const int32_t dflags = MVBA_EVAL_RESIDUALS | (want_jac ? MVBA_EVAL_JACOBIAN : 0);
  mvba_status st = mvba_evaluate_device(h, dflags, 0.0, nullptr, nullptr, 0, nullptr);
  if (st != MVBA_OK) return st;
  const int64_t N = h->nres;
  if ((st = ensure_dev(h, &h->d_tres, (size_t)(2 * N), "allocating residual rows")) != MVBA_OK) return st;
  if ((st = ensure_dev(h, &h->d_tcost, (size_t)N, "allocating cost rows")) != MVBA_OK) return st;
  if (want_jac) {
    const size_t need = packed ? (size_t)h->xoffsets[(size_t)N] : (size_t)N * (size_t)h->jac_rows;
    if (h->trows_cap < need) {
      if (h->d_trows) (void)hipFree(h->d_trows);
      h->d_trows = nullptr;
      h->trows_cap = 0;
      if ((st = ensure_dev(h, &h->d_trows, need, "allocating Jacobian rows")) != MVBA_OK) return st;
      h->trows_cap = need;
    }
  }
  const mvba_rows_layout L = cam_layout(h);
  const bool pipe = pinned_dst && packed && want_jac;
  constexpr int kChunks = 8;
  hipError_t e = hipSuccess;
  if (pipe && !h->xfer_stream) {
    e = hipStreamCreateWithFlags(&h->xfer_stream, hipStreamNonBlocking);
    for (int c = 0; c < kChunks && e == hipSuccess; c++)
      e = hipEventCreateWithFlags(&h->xfer_ev[c], hipEventDisableTiming);
    if (e != hipSuccess) return h->hip_fail(e, "creating the copy stream");
  }
  const int nch = pipe ? kChunks : 1;
  // chunk boundaries on 64-slot tiles (every k_rows tile size divides 64)
  const int64_t step = (h->nslots + 64 * nch - 1) / (64 * nch) * 64;
  for (int c = 0; c < nch && e == hipSuccess; c++) {
    const int64_t a0 = std::min<int64_t>(h->nslots, c * step), a1 = (c == nch - 1) ? h->nslots
                                                                                   : std::min<int64_t>(h->nslots, (c + 1) * step);
    e = mvba_launch_rows(h->d_res, want_jac ? h->d_J : nullptr, h->ld, a0, a1, &L, cauchy_c_of(flags, thr), h->d_order,
                         h->d_row_written, h->d_varsize, packed ? h->d_xmask : nullptr, packed ? h->d_xoff : nullptr,
                         h->d_tres, want_cost ? h->d_tcost : nullptr, want_jac ? h->d_trows : nullptr, nullptr);
    if (pipe && e == hipSuccess) {
      const int64_t r0 = h->slot_rows[(size_t)a0], r1 = h->slot_rows[(size_t)a1];
      e = hipEventRecord(h->xfer_ev[c], nullptr);
      if (e == hipSuccess) e = hipStreamWaitEvent(h->xfer_stream, h->xfer_ev[c], 0);
      if (e == hipSuccess && r1 > r0)
        e = hipMemcpyAsync(pinned_dst + r0, h->d_trows + r0, (size_t)(r1 - r0) * sizeof(double),
                           hipMemcpyDeviceToHost, h->xfer_stream);
    }
  }
  if (e != hipSuccess) return h->hip_fail(e, "mvba_launch_rows");
  st = mvba_sync_status(h, nullptr);
  if (pipe) {
    e = hipStreamSynchronize(h->xfer_stream);
    if (e != hipSuccess) return h->hip_fail(e, "packed Jacobian copy");
  }
  return st;
}

// cost = sum over blocks in AddResidualBlock order (Problem::Evaluate, one thread).
static mvba_status fetch_cost(mvba_handle* h, const double* d_cost, int64_t n, double* cost) {
  std::vector<double> c((size_t)n);
  mvba_status st = copy_to_host(h, c.data(), d_cost, (size_t)n * sizeof(double), "cost copy");
  if (st != MVBA_OK) return st;
  double total = 0.0;
  for (int64_t i = 0; i < n; i++) total += c[(size_t)i];
  *cost = total;
  return MVBA_OK;
}

extern "C" {

void* mvba_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_pinned_mu);
  g_pinned[(uintptr_t)p] = bytes ? bytes : 1;
  return p;
}

void mvba_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    g_pinned.erase((uintptr_t)p);
  }
  (void)hipHostFree(p);
}

mvba_status mvba_evaluate(mvba_handle* h, int32_t flags, double cauchy_threshold, double* cost, double* residuals,
                          double* jacobian) {
  if (!h) return MVBA_E_INVALID;
  const bool want_jac = jacobian != nullptr && (flags & MVBA_EVAL_JACOBIAN);
  mvba_status st = eval_rows(h, flags, cauchy_threshold, want_jac, false, cost != nullptr);
  if (st != MVBA_OK) return st;
  const int64_t N = h->nres;
  if (residuals &&
      (st = copy_to_host(h, residuals, h->d_tres, (size_t)(2 * N) * sizeof(double), "residual copy")) != MVBA_OK)
    return st;
  if (want_jac && (st = copy_to_host(h, jacobian, h->d_trows, (size_t)N * (size_t)h->jac_rows * sizeof(double),
                                     "Jacobian copy")) != MVBA_OK)
    return st;
  if (cost) return fetch_cost(h, h->d_tcost, N, cost);
  return MVBA_OK;
}

mvba_status mvba_set_transfer_blocks(mvba_handle* h, const uint8_t* transfer, int64_t* offsets) {
  if (!h) return MVBA_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  const int64_t N = h->nres, S = h->nslots;
  // per residual: transferred block mask (insertion order)
  std::vector<uint8_t> rmask((size_t)N);
  for (int64_t i = 0; i < N; i++) {
    const int32_t fr = h->res_frame[(size_t)i];
    int m = 0;
    if (!transfer) {
      m = h->frame_mask[(size_t)fr] | (h->pt_free_h[(size_t)h->res_pt[(size_t)i]] ? (1 << MVBA_BLK_XYZ) : 0);
    } else {
      for (int b = 0; b < 8; b++) {
        const int32_t bid = (b == MVBA_BLK_XYZ) ? h->pt_block_ids[(size_t)h->res_pt[(size_t)i]]
                                                : h->frame_blocks[(size_t)fr][b];
        if (transfer[bid]) m |= 1 << b;
      }
    }
    rmask[(size_t)i] = (uint8_t)m;
  }
  // Rows are laid out in the device's slot order (frame by frame), so each wave
  // of k_rows writes one contiguous range: whole 128-B lines instead of rows
  // scattered in insertion order (a line shared by two rows written by two
  // waves at different times costs HBM a read-modify-write). offsets[i] still
  // locates residual i's row; offsets[N] is the total.
  h->xoffsets.assign((size_t)N + 1, 0);
  std::vector<uint8_t> xm((size_t)S, 0);
  std::vector<int64_t> xo((size_t)S, 0);
  int64_t at = 0;
  h->slot_rows.assign((size_t)S + 1, 0);
  for (int64_t p = 0; p < S; p++) {
    h->slot_rows[(size_t)p] = at;
    const int64_t i = h->order[(size_t)p];
    if (i < 0) continue;
    const int K = h->frame_kdist[(size_t)h->res_frame[(size_t)i]];
    int64_t n = 0;
    for (int b = 0; b < 8; b++)
      if ((rmask[(size_t)i] >> b) & 1) n += 2 * (b < 7 ? kFixedSize[b] : K);
    xm[(size_t)p] = rmask[(size_t)i];
    xo[(size_t)p] = at;
    h->xoffsets[(size_t)i] = at;
    at += n;
  }
  h->xoffsets[(size_t)N] = at;
  h->slot_rows[(size_t)S] = at;
  hipError_t e = hipSuccess;
  if (!h->d_xmask) e = dalloc(&h->d_xmask, (size_t)S);
  if (e == hipSuccess && !h->d_xoff) e = dalloc(&h->d_xoff, (size_t)S);
  if (e == hipSuccess) e = hipMemcpy(h->d_xmask, xm.data(), (size_t)S, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_xoff, xo.data(), (size_t)S * sizeof(int64_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_set_transfer_blocks upload");
  h->packed_set = true;
  if (offsets) std::memcpy(offsets, h->xoffsets.data(), ((size_t)N + 1) * sizeof(int64_t));
  return MVBA_OK;
}

int64_t mvba_packed_size(const mvba_handle* h) {
  return (h && h->packed_set) ? h->xoffsets[(size_t)h->nres] : -1;
}

mvba_status mvba_evaluate_packed(mvba_handle* h, int32_t flags, double cauchy_threshold, double* cost,
                                 double* residuals, double* packed) {
  if (!h) return MVBA_E_INVALID;
  mvba_status st;
  if (!h->packed_set && (st = mvba_set_transfer_blocks(h, nullptr, nullptr)) != MVBA_OK) return st;
  const bool want_jac = packed != nullptr && (flags & MVBA_EVAL_JACOBIAN);
  const int64_t N = h->nres;
  const size_t jbytes = (size_t)h->xoffsets[(size_t)N] * sizeof(double);
  const bool pinned = want_jac && registered_pinned(packed, std::max<size_t>(jbytes, 1));
  st = eval_rows(h, flags, cauchy_threshold, want_jac, true, cost != nullptr, pinned ? packed : nullptr);
  if (st != MVBA_OK) return st;
  if (residuals &&
      (st = copy_to_host(h, residuals, h->d_tres, (size_t)(2 * N) * sizeof(double), "residual copy")) != MVBA_OK)
    return st;
  if (want_jac && !pinned &&
      (st = copy_to_host(h, packed, h->d_trows, jbytes, "packed Jacobian copy")) != MVBA_OK)
    return st;
  if (cost) return fetch_cost(h, h->d_tcost, N, cost);
  return MVBA_OK;
}

mvba_status mvba_evaluate_depth(mvba_handle* h, int32_t flags, double cauchy_threshold, double* cost,
                                double* residuals, double* jacobian) {
  if (!h) return MVBA_E_INVALID;
  const bool want_jac = jacobian != nullptr && (flags & MVBA_EVAL_JACOBIAN);
  const bool loss = (flags & MVBA_EVAL_APPLY_LOSS) != 0;
  if (loss && !(cauchy_threshold > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
  const int64_t ND = h->ndep, S = h->ndep_slots;
  if (ND == 0) {
    if (cost) *cost = 0.0;
    return MVBA_OK;
  }
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipSuccess;
  if (!h->d_dres) {
    h->dld = (S + 63) / 64 * 64;
    e = dalloc(&h->d_dres, (size_t)(3 * h->dld));
    if (e == hipSuccess) e = dalloc(&h->d_dJ, (size_t)MVBA_DJAC_ROWS * (size_t)h->dld);
    if (e != hipSuccess) return h->hip_fail(e, "allocating depth outputs");
  }
  if (!h->d_dwritten) {
    // per-slot written blocks and depth_to_image width, from the device records
    std::vector<mvba::DepthDesc> desc((size_t)S);
    e = hipMemcpy(desc.data(), h->d_dep_desc, (size_t)S * sizeof(mvba::DepthDesc), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return h->hip_fail(e, "depth record copy");
    std::vector<uint8_t> w((size_t)S);
    std::vector<int16_t> n((size_t)S);
    for (int64_t p = 0; p < S; p++) {
      w[(size_t)p] = (uint8_t)desc[(size_t)p].free_mask;
      n[(size_t)p] = (int16_t)desc[(size_t)p].dti_n;
    }
    e = upload(&h->d_dwritten, w);
    if (e == hipSuccess) e = upload(&h->d_dvarsize, n);
    if (e != hipSuccess) return h->hip_fail(e, "depth row tables");
  }
  mvba_status st;
  if ((st = ensure_dev(h, &h->d_tdres, (size_t)(3 * ND), "allocating depth rows")) != MVBA_OK) return st;
  if ((st = ensure_dev(h, &h->d_tdcost, (size_t)ND, "allocating depth rows")) != MVBA_OK) return st;
  if (want_jac && (st = ensure_dev(h, &h->d_tdrows, (size_t)ND * MVBA_DJAC_ROWS, "allocating depth rows")) != MVBA_OK)
    return st;
  // raw residuals / Jacobian on the device; Ceres' corrector applied by k_rows
  st = mvba_evaluate_depth_device(h, MVBA_EVAL_RESIDUALS | (want_jac ? MVBA_EVAL_JACOBIAN : 0), 0.0, h->d_dres,
                                  want_jac ? h->d_dJ : nullptr, h->dld, nullptr);
  if (st != MVBA_OK) return st;
  mvba_rows_layout L;
  L.jac_rows = MVBA_DJAC_ROWS;
  L.nres = 3;
  L.nblocks = 7;
  L.var_block = MVBA_DBLK_DEPTH_TO_IMAGE;
  const int base[7] = {MVBA_DJAC_BASE_BEG, MVBA_DJAC_BASE_END, MVBA_DJAC_BASE_REF_TO_CAM,
                       MVBA_DJAC_BASE_DEPTH_TO_IMAGE, MVBA_DJAC_BASE_SCALE, MVBA_DJAC_BASE_XYZ,
                       MVBA_DJAC_BASE_OFFSET};
  const int size[7] = {7, 7, 7, 0, 1, 3, 1};
  for (int b = 0; b < 8; b++) {
    L.base[b] = b < 7 ? base[b] : MVBA_DJAC_ROWS;
    L.size[b] = b < 7 ? size[b] : 0;
  }
  e = mvba_launch_rows(h->d_dres, want_jac ? h->d_dJ : nullptr, h->dld, 0, S, &L, cauchy_c_of(flags, cauchy_threshold),
                       h->d_dep_order, h->d_dwritten, h->d_dvarsize, nullptr, nullptr, h->d_tdres,
                       cost ? h->d_tdcost : nullptr, want_jac ? h->d_tdrows : nullptr, nullptr);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_launch_rows (depth)");
  if ((st = mvba_sync_status(h, nullptr)) != MVBA_OK) return st;
  if (residuals &&
      (st = copy_to_host(h, residuals, h->d_tdres, (size_t)(3 * ND) * sizeof(double), "depth residual copy")) != MVBA_OK)
    return st;
  if (want_jac && (st = copy_to_host(h, jacobian, h->d_tdrows, (size_t)ND * MVBA_DJAC_ROWS * sizeof(double),
                                     "depth Jacobian copy")) != MVBA_OK)
    return st;
  if (cost) return fetch_cost(h, h->d_tdcost, ND, cost);
  return MVBA_OK;
}

}  // extern "C"
