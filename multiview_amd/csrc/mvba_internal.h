// mvba_internal.h — handle layout shared by the host-side translation units
// (mvba_host.cpp: problem compilation + evaluation; mvba_solve.cpp: the LM driver).
// Not part of the public ABI.
#ifndef MVBA_INTERNAL_H_
#define MVBA_INTERNAL_H_

#include <hip/hip_runtime.h>

#include <array>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mvba/mvba.h"
#include "mvba_types.h"

using mvba::FrameDesc;
using mvba::Segment;

struct SolverState;  // mvba_solve.cpp
void solver_state_free(SolverState* s);

extern "C" {
hipError_t mvba_launch_prep(const FrameDesc* fd, int64_t nframes, const double* params,
                            double* frec, const int64_t* pt_off, const uint8_t* pt_free, int64_t npts,
                            double4* pts, int gen, int* err, hipStream_t s);
int mvba_gram_width(int model, int deg);
size_t mvba_frame_lin_size(void);
hipError_t mvba_launch_frame_lin(int model, int deg, const int4* parts, int32_t nparts, const Segment* segs,
                                 const FrameDesc* fd, const void* fl, const double* frec, const double* params,
                                 const double4* pts, const int32_t* obs_pid, const double2* obs_meas, double* rep,
                                 int64_t ng, int64_t nh, int32_t flags, double cauchy_c, const int64_t* pt_begin,
                                 int64_t npts, const int32_t* po_frame, const double2* po_meas, double* pgrad,
                                 double* phess, mvba::PointExtra dc, mvba::Slab sl, int32_t part_base,
                                 double4* obsx_out, hipStream_t s);
hipError_t mvba_launch_slab_lin(mvba::SlabTiers t, int64_t grid, const int64_t* begin, const int64_t* pos,
                                const double* val, int64_t ng, int64_t nh, double* grad, double* hess, double* cost,
                                hipStream_t s);
hipError_t mvba_launch_rep_reduce(double* rep, int32_t nrep, int64_t ng, int64_t nh, double* grad, double* hess,
                                  double* cost, hipStream_t s);
int mvba_num_replicas(void);
hipError_t mvba_launch_points_lin(int model, int deg, const int64_t* pt_begin, int64_t npts,
                                  const int32_t* po_frame, const double2* po_meas, const FrameDesc* fd,
                                  const double* frec, const double* params, const double4* pts,
                                  double* pgrad, double* phess, int32_t flags, double cauchy_c,
                                  mvba::PointExtra dc, hipStream_t s);
hipError_t mvba_launch_obs(int model, int deg, const Segment* segs, int32_t nseg,
                           const FrameDesc* fd, const double* frec, const double* params,
                           const double4* pts, const int32_t* obs_pid, const double2* obs_meas,
                           void* res, void* J, int64_t ld, int32_t flags, double cauchy_c, int32_t out_f32,
                           hipStream_t s);
int64_t mvba_eval_ready_words(int64_t nframes);
hipError_t mvba_launch_eval_fused(int model, int deg, const Segment* segs, int32_t nseg, const FrameDesc* fd,
                                  int64_t nframes, double* frec, const double* params, const int64_t* pt_off,
                                  const uint8_t* pt_free, int64_t npts, double4* pts, const int32_t* obs_pid,
                                  const double2* obs_meas, void* res, void* J, int64_t ld, int32_t flags,
                                  double cauchy_c, int32_t out_f32, int gen, int* err, unsigned* ready,
                                  unsigned poll_limit, hipStream_t s);
hipError_t mvba_launch_eval_local(int model, int deg, const Segment* segs, int32_t nseg, const FrameDesc* fd,
                                  double* frec, const double* params, const int64_t* pt_off, const uint8_t* pt_free,
                                  int64_t npts, double4* pts, const int32_t* obs_pid, const double2* obs_meas,
                                  void* res, void* J, int64_t ld, int32_t flags, double cauchy_c, int32_t out_f32,
                                  int gen, int* err, hipStream_t s);
}

extern "C" {
size_t mvba_depth_desc_size(void);
hipError_t mvba_launch_depth_obs(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                 const int32_t* dpid, const double4* dmeas, const mvba::FrameDesc* fd,
                                 const double* frec, const double* params, const double4* pts, void* res, void* J,
                                 int64_t ld, int32_t flags, double cauchy_c, int32_t out_f32, hipStream_t s);
hipError_t mvba_launch_depth_gram(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                  const int32_t* dpid, const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                  const void* fl, double* rep, int64_t ng, int64_t nh, int32_t flags, double cauchy_c,
                                  mvba::Slab sl, hipStream_t s);
hipError_t mvba_launch_xyz_cost(int64_t n, const int32_t* xpid, const double4* xref, const double* xcc,
                                const double4* pts, int32_t flags, double* partial, unsigned* counter,
                                double* out, hipStream_t s);
hipError_t mvba_launch_axpby(int64_t n, double a, const double* x, double b, const double* y, double* out,
                             hipStream_t s);
hipError_t mvba_launch_xyz_eval(int64_t n, const int32_t* xpid, const int64_t* xorder, const double4* xref,
                                const double4* pts, double* out, hipStream_t s);
hipError_t mvba_launch_depth_cost(int64_t nslots, const mvba::DepthDesc* dd, const int64_t* dorder,
                                  const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                  int32_t flags, double cauchy_c, double* partial, hipStream_t s,
                                  int64_t* nblocks_out);
// 1 when the communicator's exchange is a plain stream enqueue (RCCL: no host
// rendezvous, no event waits across streams), so a hipGraph capture of the
// solver's stream can hold it (mvba_comm.hip)
int32_t mvba_comm_capturable(const mvba_comm* comm);
// Drops every captured graph (CG runs, step sequences) recorded with this
// communicator's collectives inside, before the communicator goes
// (mvba_comm_destroy; RCCL keeps per-graph resources of a captured
// collective until its graph is destroyed) (mvba_solve.cpp)
void mvba_drop_comm_graphs(const void* comm);
}

// Row layout of a host hand-over (mvba_transfer.hip): residual rows per block,
// parameter blocks, the block with a per-slot width, first plane row and width
// of every block.
struct mvba_rows_layout {
  int32_t jac_rows, nres, nblocks, var_block;
  int32_t base[8], size[8];
};
extern "C" hipError_t mvba_launch_rows(const double* res, const double* J, int64_t ld, int64_t slot0, int64_t nslots,
                                       const mvba_rows_layout* L, double cauchy_c, const int64_t* order,
                                       const uint8_t* written, const int16_t* varsize, const uint8_t* xmask,
                                       const int64_t* xoff, double* out_res, double* out_cost, double* out_rows,
                                       hipStream_t s);

namespace mvba_internal {

// (beg, end, ref_to_cam, offset) block ids + the three stamps: what
// calc_world_to_cam_trans depends on (rig_calibrator.cc:362-390).
struct PoseKey {
  int32_t b[4];
  uint64_t s[3];
  static PoseKey make(int32_t b0, int32_t b1, int32_t b2, int32_t b4, const double* st) {
    PoseKey k;
    k.b[0] = b0; k.b[1] = b1; k.b[2] = b2; k.b[3] = b4;
    std::memcpy(k.s, st, 24);
    return k;
  }
  bool operator==(const PoseKey& o) const {
    return std::memcmp(b, o.b, sizeof(b)) == 0 && s[0] == o.s[0] && s[1] == o.s[1] && s[2] == o.s[2];
  }
};
struct PoseKeyHash {
  size_t operator()(const PoseKey& k) const {
    uint64_t x = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { x = (x ^ v) * 1099511628211ull; };
    for (int q = 0; q < 4; q++) mix((uint64_t)(uint32_t)k.b[q]);
    mix(k.s[0]); mix(k.s[1]); mix(k.s[2]);
    return (size_t)x;
  }
};

constexpr int kFixedSize[7] = {7, 7, 7, 3, 1, 1, 2};

// The device error words (handle::d_err), each raised by atomicMax to the
// generation of the evaluation that failed, so stale words are ignored:
// [0] K0's interpolation check (rig_calibrator.cc:346), [1] a fused-evaluation
// wave that gave up waiting for its frame record (k_eval).
inline mvba_status device_error(const int err[2], int gen) {
  if (gen <= 0) return MVBA_OK;
  if (err[0] >= gen) return MVBA_E_ALPHA_RANGE;
  if (err[1] >= gen) return MVBA_E_DEVICE_WAIT;
  return MVBA_OK;
}
inline const char* device_error_text(mvba_status st) {
  return st == MVBA_E_ALPHA_RANGE ? "Out of bounds in interpolation."
                                  : "fused evaluation: a wave gave up waiting for its frame record (K0 block not "
                                    "run ahead of it); outputs of this evaluation are not valid";
}

inline int rpc_degree(int n) { return static_cast<int>(std::round(std::sqrt(2.0 * n + 5.0) / 2.0 - 1.5)); }
inline int rpc_num_dist_params(int d) { return 2 * (d + 1) * (d + 2) - 2; }

// camera_params.cc:169-208 / rpc_distortion.cc:53-57 size rules.
// Returns model kind, or -1 if SetDistortion would LOG(FATAL).
inline int model_of(int K, int* deg) {
  *deg = 0;
  if (K == 0) return mvba::kModelNone;
  if (K == 1) return mvba::kModelFov;
  if (K == 4 || K == 5) return mvba::kModelRadtan;
  if (K % 2 != 0) return -1;
  const int n = K / 2;
  const int d = rpc_degree(n);
  if (rpc_num_dist_params(d) != n || d <= 0) return -1;
  *deg = d;
  return mvba::kModelRpc;
}

struct Group {
  int model = 0, deg = 0;
  int32_t seg_begin = 0, seg_count = 0;
  int64_t res_begin = 0, res_count = 0;
  // solver passes: chunks of <= 4 segments of one frame (one wave each)
  int32_t chunk_begin = 0, chunk_count = 0;
  int32_t achunk_begin = 0, achunk_count = 0;  // pass A's chunks (<= kChunkSegs segments; d_achunks)
  // linearization (K2): parts of <= kPartSegs segments of one frame (one block each)
  int32_t part_begin = 0, part_count = 0;
  int32_t gram_width = 0, w16 = 0;
};

template <class T>
hipError_t dalloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
}

template <class T>
hipError_t upload(T** p, const std::vector<T>& v) {
  hipError_t e = dalloc(p, v.size());
  if (e != hipSuccess) return e;
  if (v.empty()) return hipSuccess;
  return hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

// Deterministic accumulation plan (mvba::Slab): slab rows of `units` producers,
// `width` doubles each, and the CSR entry -> slab positions (in slab order)
// built once from a record pass.
struct DetPlan {
  int64_t units = 0, width = 0, nout = 0;
  double* val = nullptr;
  int64_t* begin = nullptr;  // [nout + 1]
  int64_t* pos = nullptr;
  int32_t* dst = nullptr;    // record pass only
  int64_t* tiers = nullptr;  // entry ids: heavy | medium | light (mvba::SlabTiers)
  int64_t nheavy = 0, nmedium = 0, nlight = 0;
  bool ready = false;
  mvba::SlabTiers tier_view() const {
    return mvba::SlabTiers{tiers, tiers + nheavy, tiers + nheavy + nmedium, nheavy, nmedium, nlight};
  }
  int64_t grid() const { return nheavy + (nmedium + 3) / 4 + (nlight + 255) / 256; }
  mvba::Slab slab(int64_t unit_base) const { return mvba::Slab{val, ready ? nullptr : dst, width, unit_base}; }
  void release() {
    for (void* p : {(void*)val, (void*)begin, (void*)pos, (void*)dst, (void*)tiers})
      if (p) (void)hipFree(p);
    val = nullptr;
    begin = pos = tiers = nullptr;
    dst = nullptr;
    ready = false;
  }
};
inline mvba::Slab no_slab() { return mvba::Slab{nullptr, nullptr, 0, 0}; }

// Allocate the slab and the record-pass destination array (set to -1).
inline hipError_t det_plan_begin(DetPlan& P, int64_t units, int64_t width, int64_t nout, hipStream_t s) {
  P.units = units;
  P.width = width;
  P.nout = nout;
  const size_t n = (size_t)std::max<int64_t>(units * width, 1);
  hipError_t e = hipSuccess;
  if (!P.val) e = hipMalloc(reinterpret_cast<void**>(&P.val), n * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&P.dst), n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemsetAsync(P.dst, 0xFF, n * sizeof(int32_t), s);
  return e;
}

// After the record pass: CSR of destination entry -> slab positions, positions
// in increasing order (the fixed summation order), uploaded; dst released.
inline hipError_t det_plan_finish(DetPlan& P, hipStream_t s) {
  const size_t n = (size_t)std::max<int64_t>(P.units * P.width, 1);
  std::vector<int32_t> dst(n);
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipMemcpy(dst.data(), P.dst, n * sizeof(int32_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  std::vector<int64_t> begin((size_t)P.nout + 1, 0);
  for (size_t k = 0; k < n; k++)
    if (dst[k] >= 0 && dst[k] < P.nout) begin[(size_t)dst[k] + 1]++;
  for (int64_t k = 0; k < P.nout; k++) begin[(size_t)k + 1] += begin[(size_t)k];
  std::vector<int64_t> fill(begin.begin(), begin.end() - 1), pos((size_t)std::max<int64_t>(begin.back(), 1));
  for (size_t k = 0; k < n; k++)
    if (dst[k] >= 0 && dst[k] < P.nout) pos[(size_t)fill[(size_t)dst[k]]++] = (int64_t)k;
  std::vector<int64_t> heavy, medium, light;
  for (int64_t k = 0; k < P.nout; k++) {
    const int64_t c = begin[(size_t)k + 1] - begin[(size_t)k];
    (c > mvba::kSlabMedium ? heavy : c > mvba::kSlabLight ? medium : light).push_back(k);
  }
  P.nheavy = (int64_t)heavy.size();
  P.nmedium = (int64_t)medium.size();
  P.nlight = (int64_t)light.size();
  heavy.insert(heavy.end(), medium.begin(), medium.end());
  heavy.insert(heavy.end(), light.begin(), light.end());
  e = upload(&P.begin, begin);
  if (e == hipSuccess) e = upload(&P.pos, pos);
  if (e == hipSuccess) e = upload(&P.tiers, heavy);
  if (e == hipSuccess) e = hipFree(P.dst);
  P.dst = nullptr;
  P.ready = e == hipSuccess;
  return e;
}

}  // namespace mvba_internal

using namespace mvba_internal;

struct mvba_handle {
  int device = 0;
  std::string err;
  int64_t nres = 0, nslots = 0, nframes = 0, npts = 0, nparams = 0;
  int64_t npts_user = 0;  // points of the caller's xyz blocks; [npts_user, npts) = mesh blocks' fixed points
  int64_t nsegs = 0;
  int32_t ncams = 0;
  int kmax = 0, jac_rows = 0;
  std::vector<int64_t> order;        // device slot -> insertion index (-1 = padding)
  std::vector<uint8_t> row_written;  // device position -> block bitmask
  std::vector<int16_t> pos_K;        // device position -> distortion length
  std::vector<Group> groups;
  std::vector<int32_t> res_frame;   // AddResidualBlock index -> frame
  double bytes_res = 0.0, bytes_jac = 0.0;

  double* d_params = nullptr;
  FrameDesc* d_fd = nullptr;
  double* d_frec = nullptr;
  int64_t* d_pt_off = nullptr;
  uint8_t* d_pt_free = nullptr;
  double4* d_pts = nullptr;
  // set by mvba_solve for its duration: K2 also writes every reprojection
  // slot's (landmark xyz, Cauchy weight sqrt(rho')) here, the record the
  // frame-order CG passes read instead of the landmark + measurement
  double4* lin_obsx = nullptr;
  int32_t* d_obs_pid = nullptr;
  double2* d_obs_meas = nullptr;
  Segment* d_segs = nullptr;
  int64_t* d_order = nullptr;
  uint8_t* d_row_written = nullptr;
  int* d_err = nullptr;
  unsigned* d_ready = nullptr;  // fused evaluation: per-K0-block ready words (zeroed at creation)
  double* d_res = nullptr;  // library-owned outputs, allocated lazily
  double* d_J = nullptr;
  int64_t ld = 0;
  bool params_set = false;
  bool prep_done = false;
  int gen = 0;  // generation of the last prep launch (error word protocol)

  // host hand-over (mvba_evaluate / mvba_evaluate_packed / mvba_evaluate_depth)
  std::vector<std::array<int32_t, 8>> frame_blocks;  // frame -> block ids (MVBA_BLK_* order)
  std::vector<int32_t> res_pt;     // AddResidualBlock index -> point index
  std::vector<int32_t> frame_mask, frame_kdist;  // frame -> written blocks, distortion length
  std::vector<uint8_t> pt_free_h;  // point index -> not constant
  int16_t* d_varsize = nullptr;    // slot -> K
  double* d_tres = nullptr;        // [2N] corrected residuals, insertion order
  double* d_tcost = nullptr;       // [N] per-block cost, insertion order
  double* d_trows = nullptr;       // rows (full or packed)
  size_t trows_cap = 0;            // doubles
  uint8_t* d_xmask = nullptr;      // packed layout: slot -> transferred blocks
  int64_t* d_xoff = nullptr;       // packed layout: slot -> row offset
  std::vector<int64_t> xoffsets;   // packed layout: insertion index -> row offset (N + 1)
  std::vector<int64_t> slot_rows;  // packed layout: slot -> first row offset at or after it (S + 1)
  hipStream_t xfer_stream = nullptr;  // device-to-host copies overlapping k_rows chunks
  hipEvent_t xfer_ev[8] = {};
  bool packed_set = false;
  uint8_t* d_dwritten = nullptr;   // depth slot -> free blocks
  int16_t* d_dvarsize = nullptr;   // depth slot -> depth_to_image width
  double* d_tdres = nullptr;       // depth: [3 ND] residuals, [ND] cost, rows
  double* d_tdcost = nullptr;
  double* d_tdrows = nullptr;
  void* h_stage[2] = {nullptr, nullptr};  // pinned staging for pageable destinations
  size_t stage_bytes = 0;
  hipEvent_t stage_ev[2] = {nullptr, nullptr};

  // linearization (K2): camera-side compact layout, chunks, point CSR
  bool lin_ok = false;
  std::string lin_err;
  int64_t cam_grad_size = 0, cam_hess_size = 0;
  int32_t nrep = 0;                     // replicas of [cam_grad | cam_hess | cost] in d_rep
  double lin_mfma_flops = 0.0;          // MFMA flops of one camera-side Gram launch set
  std::vector<int32_t> cam_block_ids;   // camera-side blocks in block-id order
  std::vector<int64_t> cam_goff, cam_hoff;
  std::vector<int32_t> pt_block_ids;    // point index -> block id
  int4* d_chunks = nullptr;
  int4* d_segchunks = nullptr;          // one chunk per segment (seg, 1, frame, -)
  int4* d_achunks = nullptr;            // pass A: runs of <= kChunkSegs segments of one frame (direct records)
  void* d_frame_lin = nullptr;
  int4* d_parts = nullptr;              // K2 frame parts (seg_begin, seg_count, frame, -)
  double* d_rep = nullptr;  // nrep copies of [cam_grad | cam_hess | cost], kept zero between calls
  int64_t* d_pt_begin = nullptr;
  int32_t* d_po_frame = nullptr;
  double2* d_po_meas = nullptr;
  int32_t* d_slot_po = nullptr;          // device slot -> point-order index (-1 = padding)
  int32_t* d_po_slot = nullptr;          // point-order index -> device slot
  // k_point_w_seg: wave tiles of whole tracks (first lane, lanes, long-track
  // point or -1, -) and per lane its point, slot (slot-order c_o) and point-order
  // position (point-order c_o); -1 for the one lane of a point without
  // reprojection residuals
  int4* d_wtiles = nullptr;
  int32_t* d_wlane_pid = nullptr;
  int32_t* d_wlane_slot = nullptr;
  int32_t* d_wlane_pos = nullptr;
  int32_t nwtiles = 0;
  std::vector<int64_t> cam_poff;         // camera-side entry -> packed parameter offset
  int32_t nchunks = 0;
  int32_t nparts = 0;                    // K2 frame parts over all model groups
  DetPlan lin_det;                       // deterministic K2 camera side (MVBA_LIN_DETERMINISTIC)

  // BracketedDepthError blocks (device order by frame)
  int64_t ndep = 0, ndep_slots = 0;
  int32_t ndep_segs = 0;
  double bytes_dep = 0.0;
  std::vector<int64_t> dep_order;         // depth slot -> depth insertion index (-1 = padding)
  mvba::DepthDesc* d_dep_desc = nullptr;
  int32_t* d_dep_pid = nullptr;           // depth slot -> point index (dense, for K1-depth)
  double4* d_dep_meas = nullptr;          // (x, y, z, weight)
  Segment* d_dep_segs = nullptr;
  int64_t* d_dep_order = nullptr;
  int64_t* d_dpt_begin = nullptr;         // CSR point -> depth slots
  int32_t* d_dpo_slot = nullptr;
  int32_t* d_dslot_po = nullptr;          // depth slot -> point-order index (inverse of d_dpo_slot)
  mvba::PointExtra point_extra() const {
    mvba::PointExtra c;
    c.begin = ndep > 0 ? d_dpt_begin : nullptr;
    c.slot = d_dpo_slot;
    c.dd = d_dep_desc;
    c.meas = d_dep_meas;
    c.xbegin = nxyz > 0 ? d_xpt_begin : nullptr;
    c.xref = d_xref;
    c.xcc = d_xcc;
    return c;
  }
  // XYZError priors (point order)
  int64_t nxyz = 0;
  std::vector<uint8_t> xfree;             // insertion order: point block free
  int64_t* d_xpt_begin = nullptr;         // CSR point -> prior entries
  double4* d_xref = nullptr;              // (x, y, z, weight)
  double* d_xcc = nullptr;                // Cauchy c = 1/threshold^2
  uint8_t* d_xkind = nullptr;             // entry -> 0 tri prior, 1 mesh_tri prior (stats groups)
  int32_t* d_xpid = nullptr;              // point of each entry
  int64_t* d_xorder = nullptr;            // entry -> insertion index
  double* d_xout = nullptr;               // [3 nxyz] raw residuals (insertion order), lazy
  double* d_xscal = nullptr;              // [1 + partials] prior cost scratch
  unsigned* d_xcnt = nullptr;             // grid-reduction counter (kept zero)
  double* d_dres = nullptr;               // library-owned depth outputs (lazy)
  double* d_dJ = nullptr;
  int64_t dld = 0;

  SolverState* solver = nullptr;         // LM state, allocated by the first mvba_solve

  mvba_status fail(mvba_status st, const std::string& msg) {
    err = msg;
    return st;
  }
  mvba_status hip_fail(hipError_t e, const char* where) {
    err = std::string("HIP error in ") + where + ": " + hipGetErrorString(e);
    return MVBA_E_HIP;
  }
};


#endif  // MVBA_INTERNAL_H_
