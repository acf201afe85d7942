// mvba_host.cpp — C ABI implementation (include/mvba/mvba.h).
//
// mvba_create "compiles" a Ceres-style problem of BracketedCamError residual
// blocks (rig_calibrator.cc:1614-1752 builds exactly this) into an HBM-resident
// structure-of-arrays:
//   * image frames: unique (beg, end, ref_to_cam, offset, focal, center, dist,
//     camera, stamps) tuples — world_to_cam depends only on these
//     (calc_world_to_cam_trans, rig_calibrator.cc:362-390);
//   * points: unique xyz blocks;
//   * residuals reordered into device order = (camera model, frame, insertion),
//     cut into wavefront segments of <= 64 residuals of one frame.
// The product path has no CPU fallback: without a GPU every entry point that
// computes returns MVBA_E_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <string>
#include <unordered_map>
#include <vector>

#include "mvba_internal.h"

namespace {
thread_local std::string g_create_error;
}  // namespace

static void free_all(mvba_handle* h) {
  if (!h) return;
  void* ptrs[] = {h->d_params, h->d_fd,      h->d_frec,  h->d_pt_off, h->d_pt_free,
                  h->d_pts,    h->d_obs_pid, h->d_obs_meas, h->d_segs, h->d_order,
                  h->d_row_written, h->d_err, h->d_ready, h->d_res, h->d_J, h->d_chunks, h->d_segchunks, h->d_achunks, h->d_frame_lin,
                  h->d_parts, h->d_rep, h->d_pt_begin, h->d_po_frame, h->d_po_meas, h->d_slot_po,
                  h->d_po_slot,       h->d_wtiles,  h->d_wlane_pid, h->d_wlane_slot, h->d_wlane_pos,
                  h->d_dep_desc, h->d_dep_pid, h->d_dep_meas, h->d_dep_segs, h->d_dep_order, h->d_dres, h->d_dJ,
                  h->d_dpt_begin, h->d_dpo_slot, h->d_dslot_po, h->d_xpt_begin, h->d_xref, h->d_xcc, h->d_xkind, h->d_xpid,
                  h->d_xorder, h->d_xout, h->d_xscal, h->d_xcnt, h->d_varsize, h->d_tres, h->d_tcost,
                  h->d_trows, h->d_xmask, h->d_xoff, h->d_dwritten, h->d_dvarsize, h->d_tdres,
                  h->d_tdcost, h->d_tdrows};
  solver_state_free(h->solver);
  h->solver = nullptr;
  h->lin_det.release();
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int k = 0; k < 2; k++) {
    if (h->h_stage[k]) (void)hipHostFree(h->h_stage[k]);
    if (h->stage_ev[k]) (void)hipEventDestroy(h->stage_ev[k]);
  }
  for (hipEvent_t ev : h->xfer_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (h->xfer_stream) (void)hipStreamDestroy(h->xfer_stream);
}

extern "C" {

int mvba_abi_version(void) { return MVBA_ABI_VERSION; }

mvba_status mvba_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  if (count) *count = n;
  return n > 0 ? MVBA_OK : MVBA_E_NO_DEVICE;
}

const char* mvba_create_error(void) { return g_create_error.c_str(); }

const char* mvba_last_error(const mvba_handle* h) { return h ? h->err.c_str() : "null handle"; }

void mvba_destroy(mvba_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  free_all(h);
  delete h;
}

mvba_status mvba_create(const mvba_problem_desc* d, const mvba_options* opts, mvba_handle** out) {
  g_create_error.clear();
  if (!out) return MVBA_E_INVALID;
  *out = nullptr;
  auto bad = [&](mvba_status st, const std::string& m) {
    g_create_error = m;
    return st;
  };
  if (!d) return bad(MVBA_E_INVALID, "null problem description");
  if (d->num_residuals < 0 || d->num_blocks < 0 || d->num_cameras < 0)
    return bad(MVBA_E_INVALID, "negative sizes in problem description");
  if (d->num_residuals > std::numeric_limits<int32_t>::max() - 64)
    return bad(MVBA_E_INVALID, "too many residual blocks for one handle (shard the problem)");
  if (d->num_residuals > 0 && (!d->residual_blocks || !d->residual_camera || !d->residual_meas ||
                               !d->residual_stamps || !d->block_size || !d->block_offset ||
                               !d->block_constant || !d->camera_dist_size || !d->camera_half_size))
    return bad(MVBA_E_INVALID, "null array in problem description");

  // Camera models (SetDistortion validation, camera_params.cc:199-206).
  std::vector<int> cam_model(d->num_cameras), cam_deg(d->num_cameras);
  int kmax = 0;
  for (int c = 0; c < d->num_cameras; c++) {
    const int K = d->camera_dist_size[c];
    cam_model[c] = model_of(K, &cam_deg[c]);
    if (cam_model[c] < 0)
      return bad(MVBA_E_BAD_DISTORTION, "Recieved irregular distortion vector size. Size = " +
                                            std::to_string(K) +
                                            "\nAdditional message: Incorrect number of RPC coefficients.");
    if (cam_model[c] == mvba::kModelRpc && cam_deg[c] > mvba::kMaxRpcDegree)
      return bad(MVBA_E_BAD_DISTORTION, "RPC degree " + std::to_string(cam_deg[c]) +
                                            " exceeds the compiled maximum " +
                                            std::to_string(mvba::kMaxRpcDegree));
    kmax = std::max(kmax, K);
  }

  const int64_t N = d->num_residuals;
  // Block-size checks of BracketedCamError's constructor (rig_calibrator.cc:433-443).
  for (int64_t i = 0; i < N; i++) {
    const int32_t* blk = d->residual_blocks + 8 * i;
    const int cam = d->residual_camera[i];
    if (cam < 0 || cam >= d->num_cameras) return bad(MVBA_E_INVALID, "residual camera index out of range");
    for (int b = 0; b < 8; b++)
      if (blk[b] < 0 || blk[b] >= d->num_blocks) return bad(MVBA_E_INVALID, "parameter block index out of range");
    for (int b = 0; b < 7; b++)
      if (d->block_size[blk[b]] != kFixedSize[b])
        return bad(MVBA_E_BLOCK_SIZES, "BracketedCamError: The block sizes were not set up properly.");
    const int K = d->camera_dist_size[cam];
    if (K > 0 && d->block_size[blk[7]] != K)
      return bad(MVBA_E_BLOCK_SIZES, "BracketedCamError: The block sizes were not set up properly.");
  }
  for (int b = 0; b < d->num_blocks; b++)
    if (d->block_offset[b] < 0 || d->block_offset[b] + d->block_size[b] > d->num_param_doubles)
      return bad(MVBA_E_INVALID, "parameter block outside the packed vector");

  // BracketedDepthError blocks: constructor checks (rig_calibrator.cc:534-543) and
  // the image they belong to (a BracketedCamError block with the same pose
  // blocks and stamps, whose world_to_cam they use).
  const int64_t ND = d->num_depth_residuals;
  if (ND < 0) return bad(MVBA_E_INVALID, "negative sizes in problem description");
  if (ND > 0 && (!d->depth_blocks || !d->depth_meas || !d->depth_weight || !d->depth_stamps))
    return bad(MVBA_E_INVALID, "null array in problem description");
  if (ND > std::numeric_limits<int32_t>::max() - 64)
    return bad(MVBA_E_INVALID, "too many depth residual blocks for one handle (shard the problem)");
  std::unordered_map<PoseKey, int64_t, PoseKeyHash> pose_first;  // pose key -> first residual using it
  if (ND > 0) {
    pose_first.reserve(1024);
    for (int64_t i = 0; i < N; i++) {
      const int32_t* blk = d->residual_blocks + 8 * i;
      pose_first.emplace(PoseKey::make(blk[0], blk[1], blk[2], blk[4], d->residual_stamps + 3 * i), i);
    }
  }
  int64_t nmesh = 0;  // BracketedDepthMeshError blocks (xyz block id -1, target in depth_mesh_xyz)
  for (int64_t j = 0; j < ND; j++) {
    const int32_t* blk = d->depth_blocks + 7 * j;
    const bool mesh = blk[MVBA_DBLK_XYZ] == -1;
    if (mesh && !d->depth_mesh_xyz)
      return bad(MVBA_E_INVALID, "depth block without a point block needs depth_mesh_xyz (BracketedDepthMeshError)");
    nmesh += mesh ? 1 : 0;
    for (int b = 0; b < 7; b++)
      if (!(mesh && b == MVBA_DBLK_XYZ) && (blk[b] < 0 || blk[b] >= d->num_blocks))
        return bad(MVBA_E_INVALID, "parameter block index out of range");
    static const int kDepthSize[7] = {7, 7, 7, 7, 1, 3, 1};
    for (int b = 0; b < 7; b++) {
      if (mesh && b == MVBA_DBLK_XYZ) continue;
      const int sz = d->block_size[blk[b]];
      const bool ok = (b == MVBA_DBLK_DEPTH_TO_IMAGE) ? (sz == 7 || sz == 12) : (sz == kDepthSize[b]);
      if (!ok)
        return bad(MVBA_E_DEPTH_BLOCK_SIZES, mesh ? "BracketedDepthMeshError: The block sizes were not set up properly.\n"
                                                  : "BracketedDepthError: The block sizes were not set up properly.\n");
    }
    if (pose_first.find(PoseKey::make(blk[0], blk[1], blk[2], blk[6], d->depth_stamps + 3 * j)) == pose_first.end())
      return bad(MVBA_E_INVALID,
                 "depth residual block without a BracketedCamError block sharing its pose blocks and stamps");
  }

  // XYZError priors: constructor check (rig_calibrator.cc:714-715).
  const int64_t NX = d->num_xyz_residuals;
  if (NX < 0) return bad(MVBA_E_INVALID, "negative sizes in problem description");
  if (NX > 0 && (!d->xyz_block || !d->xyz_ref || !d->xyz_weight || !d->xyz_threshold))
    return bad(MVBA_E_INVALID, "null array in problem description");
  for (int64_t j = 0; j < NX; j++) {
    const int32_t b = d->xyz_block[j];
    if (b < 0 || b >= d->num_blocks) return bad(MVBA_E_INVALID, "parameter block index out of range");
    if (d->block_size[b] != 3) return bad(MVBA_E_XYZ_BLOCK_SIZES, "XYZError: The block sizes were not set up properly.\n");
  }

  // The product path computes on the GPU only: no device, no handle.
  int32_t ndev = 0;
  if (mvba_device_count(&ndev) != MVBA_OK) return bad(MVBA_E_NO_DEVICE, "no HIP device available");
  const int dev = opts ? opts->device : 0;
  if (dev < 0 || dev >= ndev) return bad(MVBA_E_INVALID, "invalid device ordinal");
  if (hipSetDevice(dev) != hipSuccess) return bad(MVBA_E_HIP, "hipSetDevice failed");

  mvba_handle* h = new mvba_handle();
  h->device = dev;
  h->nres = N;
  h->nparams = d->num_param_doubles;
  h->ncams = d->num_cameras;
  h->kmax = kmax;
  h->jac_rows = MVBA_JAC_BASE_DIST + 2 * kmax;

  // ---- points: unique xyz blocks, in order of first use
  std::unordered_map<int32_t, int32_t> pt_index;
  std::vector<int64_t> pt_off;
  std::vector<uint8_t> pt_free;
  std::vector<int32_t> res_pt(N);
  pt_index.reserve(N / 4 + 16);
  for (int64_t i = 0; i < N; i++) {
    const int32_t b = d->residual_blocks[8 * i + MVBA_BLK_XYZ];
    auto it = pt_index.find(b);
    if (it == pt_index.end()) {
      const int32_t id = (int32_t)pt_off.size();
      pt_index.emplace(b, id);
      pt_off.push_back(d->block_offset[b]);
      pt_free.push_back(d->block_constant[b] ? 0 : 1);
      res_pt[i] = id;
    } else {
      res_pt[i] = it->second;
    }
  }
  std::vector<int32_t> dep_pt(ND);
  for (int64_t j = 0; j < ND; j++) {
    const int32_t b = d->depth_blocks[7 * j + MVBA_DBLK_XYZ];
    if (b == -1) continue;  // mesh blocks: virtual points below
    auto it = pt_index.find(b);
    if (it == pt_index.end()) {
      const int32_t id = (int32_t)pt_off.size();
      pt_index.emplace(b, id);
      pt_off.push_back(d->block_offset[b]);
      pt_free.push_back(d->block_constant[b] ? 0 : 1);
      dep_pt[j] = id;
    } else {
      dep_pt[j] = it->second;
    }
  }
  std::vector<int32_t> xyz_pt(NX);
  for (int64_t j = 0; j < NX; j++) {
    const int32_t b = d->xyz_block[j];
    auto it = pt_index.find(b);
    if (it == pt_index.end()) {
      const int32_t id = (int32_t)pt_off.size();
      pt_index.emplace(b, id);
      pt_off.push_back(d->block_offset[b]);
      pt_free.push_back(d->block_constant[b] ? 0 : 1);
      xyz_pt[j] = id;
    } else {
      xyz_pt[j] = it->second;
    }
  }
  // BracketedDepthMeshError (rig_calibrator.cc:615-705) is BracketedDepthError
  // with the landmark replaced by a fixed mesh point: r = w (mesh_xyz - M). Each
  // gets a virtual CONSTANT point after the user's points, backed by a tail of
  // the device parameter vector that mvba_set_params never overwrites, so every
  // depth kernel and solver pass serves it unchanged (constant points contribute
  // camera-side rows only).
  h->npts_user = (int64_t)pt_off.size();
  std::vector<double> mesh_tail;
  mesh_tail.reserve((size_t)(3 * nmesh));
  for (int64_t j = 0; j < ND; j++) {
    if (d->depth_blocks[7 * j + MVBA_DBLK_XYZ] != -1) continue;
    dep_pt[j] = (int32_t)pt_off.size();
    pt_off.push_back(d->num_param_doubles + (int64_t)mesh_tail.size());
    pt_free.push_back(0);
    for (int q = 0; q < 3; q++) mesh_tail.push_back(d->depth_mesh_xyz[3 * j + q]);
  }
  h->npts = (int64_t)pt_off.size();

  // ---- frames: unique (blocks except xyz, camera, stamps)
  struct Key {
    int32_t b[7];
    int32_t cam;
    uint64_t s[3];
    bool operator==(const Key& o) const {
      return std::memcmp(b, o.b, sizeof(b)) == 0 && cam == o.cam && s[0] == o.s[0] &&
             s[1] == o.s[1] && s[2] == o.s[2];
    }
  };
  struct KeyHash {
    size_t operator()(const Key& k) const {
      uint64_t x = 1469598103934665603ull;
      auto mix = [&](uint64_t v) { x = (x ^ v) * 1099511628211ull; };
      for (int q = 0; q < 7; q++) mix((uint64_t)(uint32_t)k.b[q]);
      mix((uint64_t)(uint32_t)k.cam);
      mix(k.s[0]); mix(k.s[1]); mix(k.s[2]);
      return (size_t)x;
    }
  };
  std::unordered_map<Key, int32_t, KeyHash> frame_index;
  frame_index.reserve(1024);
  std::vector<FrameDesc> frames;
  std::vector<std::array<int32_t, 8>> frame_blocks;
  std::vector<int32_t> res_frame(N);
  for (int64_t i = 0; i < N; i++) {
    const int32_t* blk = d->residual_blocks + 8 * i;
    Key k;
    int q = 0;
    for (int b = 0; b < 8; b++)
      if (b != MVBA_BLK_XYZ) k.b[q++] = blk[b];
    k.cam = d->residual_camera[i];
    std::memcpy(&k.s[0], &d->residual_stamps[3 * i], 24);
    auto it = frame_index.find(k);
    if (it != frame_index.end()) {
      res_frame[i] = it->second;
      continue;
    }
    FrameDesc F;
    std::memset(&F, 0, sizeof(F));
    for (int b = 0; b < 8; b++) F.off[b] = d->block_offset[blk[b]];
    F.sb = d->residual_stamps[3 * i];
    F.se = d->residual_stamps[3 * i + 1];
    F.sc = d->residual_stamps[3 * i + 2];
    F.cam = k.cam;
    F.h0 = d->camera_half_size[2 * k.cam];
    F.h1 = d->camera_half_size[2 * k.cam + 1];
    F.K = d->camera_dist_size[k.cam];
    int mask = 0;
    for (int b = 0; b < 8; b++)
      if (b != MVBA_BLK_XYZ && !d->block_constant[blk[b]]) mask |= (1 << b);
    if (F.K == 0) mask &= ~(1 << MVBA_BLK_DIST);
    F.free_mask = mask;
    const int32_t id = (int32_t)frames.size();
    frames.push_back(F);
    std::array<int32_t, 8> fb;
    for (int b = 0; b < 8; b++) fb[b] = blk[b];
    frame_blocks.push_back(fb);
    frame_index.emplace(k, id);
    res_frame[i] = id;
  }
  // Frame numbering in capture order (image timestamp, then camera, then order
  // of first use), not in order of first use: AddResidualBlock order is
  // landmark-major (rig_calibrator.cc:1614-1752), so first use scatters the
  // images of one stretch of the trajectory over the whole frame range. In
  // capture order, frames next to each other see the same landmarks: the
  // landmark numbering below (first use in frame order) becomes a band, the
  // frame-order CG passes of one XCD gather landmark-side vectors (w_p) from an
  // L2-sized window, and the point-order pass gathers each landmark's c_o from
  // a few neighbouring frame ranges. MVBA_FRAME_ORDER=first_use keeps the old
  // numbering (A/B timing).
  {
    const char* fo = std::getenv("MVBA_FRAME_ORDER");
    if (!(fo && !std::strcmp(fo, "first_use")) && frames.size() > 1) {
      const size_t nf = frames.size();
      std::vector<int32_t> ord(nf);
      for (size_t f = 0; f < nf; f++) ord[f] = (int32_t)f;
      std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
        if (frames[a].sc != frames[b].sc) return frames[a].sc < frames[b].sc;
        return frames[a].cam < frames[b].cam;
      });
      std::vector<int32_t> rank(nf);
      for (size_t q = 0; q < nf; q++) rank[ord[q]] = (int32_t)q;
      std::vector<FrameDesc> frames2(nf);
      std::vector<std::array<int32_t, 8>> blocks2(nf);
      for (size_t f = 0; f < nf; f++) {
        frames2[rank[f]] = frames[f];
        blocks2[rank[f]] = frame_blocks[f];
      }
      frames.swap(frames2);
      frame_blocks.swap(blocks2);
      for (auto& v : res_frame) v = rank[v];
    }
  }
  h->nframes = (int64_t)frames.size();
  h->res_frame = res_frame;
  h->frame_blocks = frame_blocks;
  h->res_pt = res_pt;
  h->pt_free_h = pt_free;
  h->frame_mask.resize(frames.size());
  h->frame_kdist.resize(frames.size());
  for (size_t f = 0; f < frames.size(); f++) {
    h->frame_mask[f] = frames[f].free_mask;
    h->frame_kdist[f] = frames[f].K;
  }

  // ---- groups by (model, degree), then device order
  std::vector<int> gkey_of_cam(d->num_cameras);
  std::vector<int> keys;
  for (int c = 0; c < d->num_cameras; c++) {
    gkey_of_cam[c] = cam_model[c] * 16 + cam_deg[c];
    keys.push_back(gkey_of_cam[c]);
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  std::vector<int> grank(d->num_cameras);
  for (int c = 0; c < d->num_cameras; c++)
    grank[c] = (int)(std::lower_bound(keys.begin(), keys.end(), gkey_of_cam[c]) - keys.begin());

  std::vector<int64_t> idx(N);
  for (int64_t i = 0; i < N; i++) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    const int ga = grank[d->residual_camera[a]], gb = grank[d->residual_camera[b]];
    if (ga != gb) return ga < gb;
    return res_frame[a] < res_frame[b];
  });

  // Point numbering in order of first use in DEVICE order (frame order), not in
  // AddResidualBlock order: a frame's landmarks then have nearby indices, so K1's
  // landmark gathers, the solver's point-order scatters (c_o) and gathers
  // (k_point_w) touch a cache-sized window instead of the whole table (tables of
  // 10M+ observations exceed the 256 MB Infinity Cache). Points without a
  // reprojection residual keep their relative order after those; the virtual
  // mesh points stay last. mvba_point_block_map reports the numbering.
  {
    const int64_t np = (int64_t)pt_off.size();
    std::vector<int32_t> perm((size_t)np, -1);
    int32_t next = 0;
    for (int64_t p = 0; p < N; p++) {
      const int32_t q = res_pt[idx[p]];
      if (perm[q] < 0) perm[q] = next++;
    }
    for (int64_t q = 0; q < h->npts_user; q++)
      if (perm[q] < 0) perm[q] = next++;
    for (int64_t q = h->npts_user; q < np; q++) perm[q] = (int32_t)q;  // mesh points: unchanged, last
    std::vector<int64_t> off2((size_t)np);
    std::vector<uint8_t> free2((size_t)np);
    for (int64_t q = 0; q < np; q++) {
      off2[perm[q]] = pt_off[q];
      free2[perm[q]] = pt_free[q];
    }
    pt_off.swap(off2);
    pt_free.swap(free2);
    for (auto& v : res_pt) v = perm[v];
    for (auto& v : dep_pt) v = perm[v];
    for (auto& v : xyz_pt) v = perm[v];
    for (auto& kv : pt_index) kv.second = perm[kv.second];
    h->res_pt = res_pt;
    h->pt_free_h = pt_free;
  }

  // Within a frame, slots in landmark order (stable): the landmarks first used
  // by one earlier frame then sit in one contiguous run of every later frame
  // that sees them, so k_point_w's c_o gathers (points in id order) and the
  // landmark / w_p gathers of K1 and pass B (slots in order) share lines. The
  // numbering above is unchanged by it (a frame's new landmarks keep their
  // relative order and follow the ones numbered before). MVBA_SLOT_ORDER=
  // insertion keeps AddResidualBlock order within frames (A/B timing).
  {
    const char* so = std::getenv("MVBA_SLOT_ORDER");
    if (!(so && !std::strcmp(so, "insertion")))
      for (int64_t a = 0; a < N;) {
        const int64_t ia = idx[a];
        const int ga = grank[d->residual_camera[ia]];
        int64_t b = a + 1;
        while (b < N && res_frame[idx[b]] == res_frame[ia] && grank[d->residual_camera[idx[b]]] == ga) b++;
        std::stable_sort(idx.begin() + a, idx.begin() + b,
                         [&](int64_t x, int64_t y) { return res_pt[x] < res_pt[y]; });
        a = b;
      }
  }

  // Device slots: every frame's residuals start on a 128-byte line of fp32
  // outputs (32 slots; two lines of fp64), so each wavefront's 64-element store
  // chunk per Jacobian plane is line-aligned (misaligned chunks write at ~60% of
  // the aligned rate: tools/store_bench.hip), and K1 fills the frame's last line
  // with padding (Segment::pad bounds it). Measured and not kept:
  // 16-slot alignment (fewer padding slots on thin shards) and frames packed
  // densely into 64-slot windows of several frames.
  constexpr int64_t kAlign = 32;
  int64_t nslots = 0;
  {
    int32_t prev_fr = -1;
    int prev_g = -1;
    for (int64_t p = 0; p < N; p++) {
      const int64_t i = idx[p];
      const int g = grank[d->residual_camera[i]];
      if (res_frame[i] != prev_fr || g != prev_g) nslots = (nslots + kAlign - 1) / kAlign * kAlign;
      prev_fr = res_frame[i];
      prev_g = g;
      nslots++;
    }
    nslots = (nslots + kAlign - 1) / kAlign * kAlign;
  }
  h->nslots = nslots;
  std::vector<int32_t> obs_pid(nslots, 0);
  std::vector<double2> obs_meas(nslots, make_double2(0.0, 0.0));
  h->order.assign(nslots, -1);
  h->row_written.assign(nslots, 0);
  h->pos_K.assign(nslots, 0);
  std::vector<Segment> segs;
  segs.reserve(N / 32 + frames.size() + keys.size() + 1);
  h->groups.resize(keys.size());
  double bytes_res = 0.0, bytes_jac = 0.0;
  for (size_t g = 0; g < keys.size(); g++) {
    h->groups[g].model = keys[g] / 16;
    h->groups[g].deg = keys[g] % 16;
  }
  int cur_group = -1;
  int32_t cur_frame = -1;
  int64_t slot = 0;
  for (int64_t p = 0; p < N; p++) {
    const int64_t i = idx[p];
    const int g = grank[d->residual_camera[i]];
    const int32_t fr = res_frame[i];
    const bool new_group = (g != cur_group);
    if (new_group) {
      if (cur_group >= 0) h->groups[cur_group].seg_count = (int32_t)segs.size() - h->groups[cur_group].seg_begin;
      cur_group = g;
      h->groups[g].seg_begin = (int32_t)segs.size();
    }
    if (new_group || fr != cur_frame) {
      slot = (slot + kAlign - 1) / kAlign * kAlign;
      cur_frame = fr;
    }
    if (new_group) h->groups[g].res_begin = slot;
    h->groups[g].res_count++;
    if (new_group || segs.back().frame != fr || segs.back().count == 64) {
      Segment sg;
      sg.begin = (int32_t)slot;
      sg.count = 0;
      sg.frame = fr;
      sg.pad = 0;
      segs.push_back(sg);
    }
    segs.back().count++;
    obs_pid[slot] = res_pt[i];
    obs_meas[slot] = make_double2(d->residual_meas[2 * i], d->residual_meas[2 * i + 1]);
    h->order[slot] = i;
    const int mask = frames[fr].free_mask | (pt_free[res_pt[i]] ? (1 << MVBA_BLK_XYZ) : 0);
    h->row_written[slot] = (uint8_t)mask;
    h->pos_K[slot] = (int16_t)frames[fr].K;
    // Algorithmic bytes: meas 16 + point index 4 + point 24 + r 16.
    bytes_res += 16.0 + 4.0 + 24.0 + 16.0;
    int cols = 0;
    for (int b = 0; b < 8; b++)
      if (mask & (1 << b)) cols += (b == 7) ? frames[fr].K : kFixedSize[b];
    bytes_jac += 16.0 * cols;
    slot++;
  }
  if (cur_group >= 0) h->groups[cur_group].seg_count = (int32_t)segs.size() - h->groups[cur_group].seg_begin;
  // Segment::pad = the slots this segment's lanes may write (K1's padding lanes
  // fill the frame's last line but never reach the next frame's first slot)
  for (size_t k = 0; k < segs.size(); k++) {
    const int64_t next = k + 1 < segs.size() ? segs[k + 1].begin : nslots;
    segs[k].pad = (int32_t)std::min<int64_t>(64, next - segs[k].begin);
  }
  h->bytes_res = bytes_res;
  h->nsegs = (int64_t)segs.size();
  h->bytes_jac = bytes_jac;

  // ---- linearization structures (K2)
  std::vector<int4> chunks, parts;
  std::vector<mvba::FrameLinHost> flin(frames.size());
  std::vector<int64_t> pt_begin;
  std::vector<int32_t> po_frame, po_slot;
  std::vector<double2> po_meas;
  std::vector<int32_t> slot_po;
  std::vector<int64_t> goff_of(d->num_blocks, -1), hoff_of(d->num_blocks, -1);
  {
    h->lin_ok = true;
    for (const Group& G : h->groups)
      if (G.model == mvba::kModelRpc && G.deg > mvba::kMaxLinRpcDegree) {
        h->lin_ok = false;
        h->lin_err = "linearization supports RPC degree <= " + std::to_string(mvba::kMaxLinRpcDegree);
      }
    // camera-side blocks: not constant, not a point block, in block-id order
    std::vector<uint8_t> is_point(d->num_blocks, 0);
    for (auto& kv : pt_index) is_point[kv.first] = 1;
    h->pt_block_ids.assign(h->npts, -1);  // -1: virtual point of a mesh block
    for (auto& kv : pt_index) h->pt_block_ids[kv.second] = kv.first;
    for (int b = 0; b < d->num_blocks; b++) {
      if (is_point[b] || d->block_constant[b]) continue;
      const int64_t sz = d->block_size[b];
      goff_of[b] = h->cam_grad_size;
      hoff_of[b] = h->cam_hess_size;
      h->cam_block_ids.push_back(b);
      h->cam_goff.push_back(h->cam_grad_size);
      h->cam_hoff.push_back(h->cam_hess_size);
      h->cam_grad_size += sz;
      h->cam_hess_size += sz * sz;
      for (int64_t q = 0; q < sz; q++) h->cam_poff.push_back(d->block_offset[b] + q);
    }
    for (Group& G : h->groups) {
      G.chunk_begin = (int32_t)chunks.size();
      G.part_begin = (int32_t)parts.size();
      G.gram_width = h->lin_ok ? mvba_gram_width(G.model, G.deg) : 0;
      G.w16 = (G.gram_width + 15) / 16 * 16;
      // segments per pass-B chunk (one wave): mvba::kChunkSegs, 2x that where
      // images average 12+ segments (c3, 17 per image: pass B 197 -> 182 us;
      // profiles/r04/r04t/), and halved (8 -> 4 -> 2 -> 1) while the group
      // would have fewer than kMinChunks chunks: thin shards have one or two
      // 8-segment chunks per image, too few waves to cover the gathers' latency
      // (1/8 c2 shard, 470 chunks: pass B 10.5 us with 8-segment chunks, 6.9
      // with 2; whole c2, 3,008 chunks: 21.9 us with 8, 23.0 with 4;
      // profiles/r05/r05g/). MVBA_CHUNK_SEGS overrides it (A/B timing).
      int32_t gframes = 0;
      std::vector<int32_t> fsegs;  // segments per frame run of the group
      for (int32_t sidx = G.seg_begin; sidx < G.seg_begin + G.seg_count; sidx++) {
        if (sidx == G.seg_begin || segs[sidx].frame != segs[sidx - 1].frame) {
          gframes++;
          fsegs.push_back(0);
        }
        fsegs.back()++;
      }
      auto nchunks_of = [&](int cs) {
        int64_t c = 0;
        for (int32_t m : fsegs) c += (m + cs - 1) / cs;
        return c;
      };
      constexpr int64_t kMinChunks = 1024;  // one wave per SIMD
      const int chunk_segs = [&] {
        const char* e = std::getenv("MVBA_CHUNK_SEGS");
        if (e) {
          const int v = std::atoi(e);
          return v >= 1 && v <= 64 ? v : mvba::kChunkSegs;
        }
        if (G.seg_count >= 12 * (int64_t)std::max(gframes, 1)) return 2 * mvba::kChunkSegs;
        int cs = mvba::kChunkSegs;
        while (cs > 1 && nchunks_of(cs) < kMinChunks) cs /= 2;
        return cs;
      }();
      for (int32_t sidx = G.seg_begin; sidx < G.seg_begin + G.seg_count; sidx++) {
        const Segment& sg = segs[sidx];
        if (chunks.size() == (size_t)G.chunk_begin || chunks.back().z != sg.frame ||
            chunks.back().y == chunk_segs) {
          int4 c;
          c.x = sidx;
          c.y = 0;
          c.z = sg.frame;
          c.w = (int32_t)chunks.size() - G.chunk_begin;
          chunks.push_back(c);
          mvba::FrameLinHost& L = flin[sg.frame];
          if (L.chunk_count == 0) L.first_chunk = (int32_t)chunks.size() - 1;
          L.chunk_count++;
          L.width = G.gram_width;
          L.w16 = G.w16;
        }
        chunks.back().y++;
      }
      // K2 parts: a frame's run of segments split evenly into ceil(n / kPartSegs) parts
      for (int32_t r0 = G.seg_begin; r0 < G.seg_begin + G.seg_count;) {
        int32_t r1 = r0;
        while (r1 < G.seg_begin + G.seg_count && segs[r1].frame == segs[r0].frame) r1++;
        const int32_t n = r1 - r0, np = (n + mvba::kPartSegs - 1) / mvba::kPartSegs;
        for (int32_t q = 0, at = r0; q < np; q++) {
          const int32_t len = n / np + (q < n % np ? 1 : 0);
          parts.push_back(make_int4(at, len, segs[r0].frame, 0));
          at += len;
        }
        r0 = r1;
      }
      G.chunk_count = (int32_t)chunks.size() - G.chunk_begin;
      G.part_count = (int32_t)parts.size() - G.part_begin;
      // k_frame_lin: per 32-observation half of a segment, 16 K=4 steps over
      // the T(T+1)/2 tile pairs, 2048 flops per v_mfma_f64_16x16x4
      if (G.gram_width > 0) {
        const int64_t T = (G.gram_width + 15) / 16;
        int64_t halves = 0;
        for (int32_t sidx = G.seg_begin; sidx < G.seg_begin + G.seg_count; sidx++)
          halves += (segs[sidx].count + 31) / 32;
        h->lin_mfma_flops += (double)halves * 16.0 * (double)(T * (T + 1) / 2) * 2048.0;
      }
    }
    for (size_t f = 0; f < frames.size(); f++) {
      for (int b = 0; b < 8; b++) {
        const int32_t bid = frame_blocks[f][b];
        const bool used = (b != MVBA_BLK_XYZ) && (b != MVBA_BLK_DIST || frames[f].K > 0);
        flin[f].goff[b] = used ? goff_of[bid] : -1;
        flin[f].hoff[b] = used ? hoff_of[bid] : -1;
      }
    }
    // point-ordered copy of the observation records (CSR point -> residuals)
    std::vector<int64_t> cnt(h->npts + 1, 0);
    for (int64_t i = 0; i < N; i++) cnt[res_pt[i] + 1]++;
    for (int64_t p = 0; p < h->npts; p++) cnt[p + 1] += cnt[p];
    pt_begin = cnt;
    po_frame.resize(N);
    po_meas.resize(N);
    std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
    std::vector<int32_t> po_of(N);
    for (int64_t i = 0; i < N; i++) {
      const int64_t j = fill[res_pt[i]]++;
      po_of[i] = (int32_t)j;
      po_frame[j] = res_frame[i];
      po_meas[j] = make_double2(d->residual_meas[2 * i], d->residual_meas[2 * i + 1]);
    }
    slot_po.assign(nslots, -1);
    for (int64_t p = 0; p < nslots; p++)
      if (h->order[p] >= 0) slot_po[p] = po_of[h->order[p]];
    po_slot.assign(N, -1);
    for (int64_t p = 0; p < nslots; p++)
      if (slot_po[p] >= 0) po_slot[slot_po[p]] = (int32_t)p;
    h->nchunks = (int32_t)chunks.size();
    h->nparts = (int32_t)parts.size();
  }

  // ---- depth blocks: device order by frame, line-aligned frame ranges, segments
  std::vector<mvba::DepthDesc> ddesc;
  std::vector<double4> dmeas;
  std::vector<Segment> dsegs;
  if (ND > 0) {
    std::unordered_map<PoseKey, int32_t, PoseKeyHash> frame_of_key;
    frame_of_key.reserve(frames.size() * 2);
    for (int64_t i = 0; i < N; i++) {
      const int32_t* blk = d->residual_blocks + 8 * i;
      frame_of_key.emplace(PoseKey::make(blk[0], blk[1], blk[2], blk[4], d->residual_stamps + 3 * i), res_frame[i]);
    }
    std::vector<int32_t> dep_frame(ND);
    for (int64_t j = 0; j < ND; j++) {
      const int32_t* blk = d->depth_blocks + 7 * j;
      dep_frame[j] = frame_of_key.at(PoseKey::make(blk[0], blk[1], blk[2], blk[6], d->depth_stamps + 3 * j));
    }
    std::vector<int64_t> didx(ND);
    for (int64_t j = 0; j < ND; j++) didx[j] = j;
    std::stable_sort(didx.begin(), didx.end(), [&](int64_t a, int64_t b) { return dep_frame[a] < dep_frame[b]; });
    constexpr int64_t kAlign = 32;  // one 128-B line of fp32 outputs (two of fp64)
    int64_t slot = 0;
    int32_t prev = -1;
    std::vector<int64_t> slot_of(ND);
    for (int64_t q = 0; q < ND; q++) {
      const int64_t j = didx[q];
      if (dep_frame[j] != prev) slot = (slot + kAlign - 1) / kAlign * kAlign;
      if (dep_frame[j] != prev || dsegs.back().count == 64) {
        Segment sg;
        sg.begin = (int32_t)slot;
        sg.count = 0;
        sg.frame = dep_frame[j];
        sg.pad = 0;
        dsegs.push_back(sg);
      }
      prev = dep_frame[j];
      dsegs.back().count++;
      slot_of[j] = slot++;
    }
    h->ndep_slots = (slot + kAlign - 1) / kAlign * kAlign;
    h->dep_order.assign(h->ndep_slots, -1);
    ddesc.assign(h->ndep_slots, mvba::DepthDesc{});
    dmeas.assign(h->ndep_slots, make_double4(0, 0, 0, 0));
    for (int64_t j = 0; j < ND; j++) {
      const int32_t* blk = d->depth_blocks + 7 * j;
      const int64_t p = slot_of[j];
      h->dep_order[p] = j;
      mvba::DepthDesc& D = ddesc[p];
      D.dti_off = d->block_offset[blk[MVBA_DBLK_DEPTH_TO_IMAGE]];
      D.scale_off = d->block_offset[blk[MVBA_DBLK_SCALE]];
      D.goff_dti = goff_of[blk[MVBA_DBLK_DEPTH_TO_IMAGE]];
      D.hoff_dti = hoff_of[blk[MVBA_DBLK_DEPTH_TO_IMAGE]];
      D.goff_scale = goff_of[blk[MVBA_DBLK_SCALE]];
      D.hoff_scale = hoff_of[blk[MVBA_DBLK_SCALE]];
      D.frame = dep_frame[j];
      D.pid = dep_pt[j];
      D.dti_n = d->block_size[blk[MVBA_DBLK_DEPTH_TO_IMAGE]];
      const int fm = frames[dep_frame[j]].free_mask;
      int m = 0;
      if (fm & (1 << MVBA_BLK_BEG)) m |= 1 << MVBA_DBLK_BEG;
      if (fm & (1 << MVBA_BLK_END)) m |= 1 << MVBA_DBLK_END;
      if (fm & (1 << MVBA_BLK_REF_TO_CAM)) m |= 1 << MVBA_DBLK_REF_TO_CAM;
      if (fm & (1 << MVBA_BLK_OFFSET)) m |= 1 << MVBA_DBLK_OFFSET;
      if (!d->block_constant[blk[MVBA_DBLK_DEPTH_TO_IMAGE]]) m |= 1 << MVBA_DBLK_DEPTH_TO_IMAGE;
      if (!d->block_constant[blk[MVBA_DBLK_SCALE]]) m |= 1 << MVBA_DBLK_SCALE;
      if (pt_free[dep_pt[j]]) m |= 1 << MVBA_DBLK_XYZ;
      D.free_mask = m;
      dmeas[p] = make_double4(d->depth_meas[3 * j], d->depth_meas[3 * j + 1], d->depth_meas[3 * j + 2],
                              d->depth_weight[j]);
      int cols = 0;
      for (int b = 0; b < 7; b++)
        if (m & (1 << b)) cols += (b == MVBA_DBLK_DEPTH_TO_IMAGE) ? D.dti_n : (b == MVBA_DBLK_SCALE || b == MVBA_DBLK_OFFSET) ? 1 : (b == MVBA_DBLK_XYZ ? 3 : 7);
      // Algorithmic bytes: meas + weight 32 + point 24 + residual 24 + 24 per written column.
      h->bytes_dep += 32.0 + 24.0 + 24.0 + 24.0 * cols;
    }
  }
  h->ndep = ND;
  h->ndep_segs = (int32_t)dsegs.size();
  std::vector<int64_t> dpt_begin;
  std::vector<int32_t> dpo_slot;
  if (ND > 0) {
    dpt_begin.assign(h->npts + 1, 0);
    for (int64_t j = 0; j < ND; j++) dpt_begin[dep_pt[j] + 1]++;
    for (int64_t p = 0; p < h->npts; p++) dpt_begin[p + 1] += dpt_begin[p];
    std::vector<int64_t> fill(dpt_begin.begin(), dpt_begin.end() - 1);
    dpo_slot.resize(ND);
    for (int64_t q = 0; q < h->ndep_slots; q++) {
      const int64_t j = h->dep_order[q];
      if (j >= 0) dpo_slot[fill[dep_pt[j]]++] = (int32_t)q;
    }
  }

  // ---- XYZ priors in point order
  std::vector<int64_t> xpt_begin, xorder;
  std::vector<double4> xref;
  std::vector<double> xcc;
  std::vector<int32_t> xpid;
  std::vector<uint8_t> xkind;
  h->nxyz = NX;
  h->xfree.assign((size_t)NX, 0);
  for (int64_t j = 0; j < NX; j++) h->xfree[(size_t)j] = pt_free[xyz_pt[j]];
  if (NX > 0) {
    xpt_begin.assign(h->npts + 1, 0);
    for (int64_t j = 0; j < NX; j++) xpt_begin[xyz_pt[j] + 1]++;
    for (int64_t p = 0; p < h->npts; p++) xpt_begin[p + 1] += xpt_begin[p];
    std::vector<int64_t> fill(xpt_begin.begin(), xpt_begin.end() - 1);
    xref.resize(NX);
    xcc.resize(NX);
    xpid.resize(NX);
    xorder.resize(NX);
    xkind.resize(NX);
    for (int64_t j = 0; j < NX; j++) {
      const int64_t q = fill[xyz_pt[j]]++;
      xref[q] = make_double4(d->xyz_ref[3 * j], d->xyz_ref[3 * j + 1], d->xyz_ref[3 * j + 2], d->xyz_weight[j]);
      const double t = d->xyz_threshold[j];
      xcc[q] = t > 0.0 ? 1.0 / (t * t) : 0.0;
      xpid[q] = xyz_pt[j];
      xorder[q] = j;
      xkind[q] = d->xyz_kind ? (d->xyz_kind[j] ? 1 : 0) : 0;
    }
  }

  // ---- upload
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (e == hipSuccess && x != hipSuccess) e = x;
  };
  chk(dalloc(&h->d_params, (size_t)std::max<int64_t>(d->num_param_doubles + (int64_t)mesh_tail.size(), 1)));
  if (e == hipSuccess && !mesh_tail.empty())
    chk(hipMemcpy(h->d_params + d->num_param_doubles, mesh_tail.data(), mesh_tail.size() * sizeof(double),
                  hipMemcpyHostToDevice));
  chk(upload(&h->d_fd, frames));
  chk(dalloc(&h->d_frec, (size_t)h->nframes * mvba::kFrameRecDoubles));
  chk(upload(&h->d_pt_off, pt_off));
  chk(upload(&h->d_pt_free, pt_free));
  chk(dalloc(&h->d_pts, (size_t)h->npts));
  chk(upload(&h->d_obs_pid, obs_pid));
  chk(upload(&h->d_obs_meas, obs_meas));
  chk(upload(&h->d_segs, segs));
  chk(upload(&h->d_order, h->order));
  chk(upload(&h->d_row_written, h->row_written));
  chk(upload(&h->d_varsize, h->pos_K));
  chk(dalloc(&h->d_err, 2));  // [0] alpha range (K0), [1] fused-evaluation wait given up
  if (e == hipSuccess) chk(hipMemset(h->d_err, 0, 2 * sizeof(int)));
  {
    const int64_t nw = std::max<int64_t>(mvba_eval_ready_words(h->nframes), 1);
    chk(dalloc(&h->d_ready, (size_t)nw));
    if (e == hipSuccess) chk(hipMemset(h->d_ready, 0, (size_t)nw * sizeof(unsigned)));
  }
  {
    // The CG passes' chunk records carry the slot range directly: (first slot,
    // observations, frame, first chunk of the frame). A chunk's segments are
    // consecutive 64-slot runs of one frame, so the passes load no Segment.
    auto direct = [&](int32_t sidx, int32_t nseg, bool first) {
      int32_t n = 0;
      for (int32_t k = sidx; k < sidx + nseg; k++) n += segs[k].count;
      return make_int4(segs[sidx].begin, n, segs[sidx].frame, first ? 1 : 0);
    };
    std::vector<int4> dc(chunks.size());
    for (size_t k = 0; k < chunks.size(); k++)
      dc[k] = direct(chunks[k].x, chunks[k].y, k == 0 || chunks[k - 1].z != chunks[k].z);
    chk(upload(&h->d_chunks, dc));
    // one-segment chunks: the solver's frame-order pass A takes one segment per
    // wave (it writes per-observation records, nothing per frame to reduce)
    std::vector<int4> sc(segs.size());
    for (size_t k = 0; k < segs.size(); k++) sc[k] = direct((int32_t)k, 1, k == 0 || segs[k - 1].frame != segs[k].frame);
    chk(upload(&h->d_segchunks, sc));
    // pass A's chunks: runs of at most kChunkSegs segments of one frame, also
    // where pass B's chunks are 2x that (c3 pass A: 131 us on 8-segment chunks,
    // 144 on 16-segment ones, profiles/r04/r04w/). MVBA_PASS_A_SEGS overrides
    // the run length (A/B timing).
    const int asegs = [] {
      const char* e = std::getenv("MVBA_PASS_A_SEGS");
      const int v = e ? std::atoi(e) : mvba::kChunkSegs;
      return v >= 1 && v <= 64 ? v : mvba::kChunkSegs;
    }();
    std::vector<int4> ac;
    for (Group& G : h->groups) {
      G.achunk_begin = (int32_t)ac.size();
      for (int32_t a = G.seg_begin; a < G.seg_begin + G.seg_count;) {
        int32_t b = a + 1;
        while (b < G.seg_begin + G.seg_count && b - a < asegs && segs[b].frame == segs[a].frame) b++;
        ac.push_back(direct(a, b - a, a == G.seg_begin || segs[a - 1].frame != segs[a].frame));
        a = b;
      }
      G.achunk_count = (int32_t)ac.size() - G.achunk_begin;
    }
    chk(upload(&h->d_achunks, ac));
  }
  {
    void* p = nullptr;
    chk(hipMalloc(&p, std::max<size_t>(flin.size(), 1) * sizeof(mvba::FrameLinHost)));
    h->d_frame_lin = p;
    if (e == hipSuccess && !flin.empty())
      chk(hipMemcpy(p, flin.data(), flin.size() * sizeof(mvba::FrameLinHost), hipMemcpyHostToDevice));
  }
  chk(upload(&h->d_parts, parts));
  {
    // the depth Gram adds into kDepthReplicas replicas, the camera side into mvba_num_replicas()
    h->nrep = h->ndep > 0 ? std::max(mvba::kDepthReplicas, mvba_num_replicas()) : mvba_num_replicas();
    const size_t nrep = (size_t)h->nrep * (size_t)(h->cam_grad_size + h->cam_hess_size + 1);
    chk(dalloc(&h->d_rep, nrep));
    if (e == hipSuccess) chk(hipMemset(h->d_rep, 0, nrep * sizeof(double)));
  }
  chk(upload(&h->d_pt_begin, pt_begin));
  chk(upload(&h->d_po_frame, po_frame));
  chk(upload(&h->d_po_meas, po_meas));
  chk(upload(&h->d_slot_po, slot_po));
  chk(upload(&h->d_po_slot, po_slot));
  {
    // k_point_w_seg's wave tiles: consecutive points packed whole into <= 64
    // lanes (one lane per reprojection residual, one for a point without any);
    // a track longer than a wave gets a tile of its own (lane-strided loop)
    std::vector<int4> tiles;
    std::vector<int32_t> lpid, lslot, lpos;
    lpid.reserve((size_t)N + (size_t)h->npts / 8 + 64);
    lslot.reserve(lpid.capacity());
    lpos.reserve(lpid.capacity());
    int32_t first = 0, count = 0;
    auto flush = [&]() {
      if (count > 0) tiles.push_back(make_int4(first, count, -1, 0));
      first = (int32_t)lpid.size();
      count = 0;
    };
    for (int64_t p = 0; p < h->npts; p++) {
      const int64_t n = pt_begin[(size_t)p + 1] - pt_begin[(size_t)p];
      if (n > 64) {
        flush();
        tiles.push_back(make_int4(first, 0, (int32_t)p, 0));
        continue;
      }
      const int32_t m = (int32_t)std::max<int64_t>(n, 1);
      if (count + m > 64) flush();
      for (int32_t k = 0; k < m; k++) {
        const int64_t j = n > 0 ? pt_begin[(size_t)p] + k : -1;
        lpid.push_back((int32_t)p);
        lpos.push_back((int32_t)j);
        lslot.push_back(j >= 0 ? po_slot[(size_t)j] : -1);
      }
      count += m;
    }
    flush();
    h->nwtiles = (int32_t)tiles.size();
    chk(upload(&h->d_wtiles, tiles));
    chk(upload(&h->d_wlane_pid, lpid));
    chk(upload(&h->d_wlane_slot, lslot));
    chk(upload(&h->d_wlane_pos, lpos));
  }
  chk(upload(&h->d_dep_desc, ddesc));
  {
    std::vector<int32_t> dpid(ddesc.size());
    for (size_t q = 0; q < ddesc.size(); q++) dpid[q] = ddesc[q].pid;
    chk(upload(&h->d_dep_pid, dpid));
  }
  chk(upload(&h->d_dep_meas, dmeas));
  chk(upload(&h->d_dep_segs, dsegs));
  chk(upload(&h->d_dep_order, h->dep_order));
  chk(upload(&h->d_dpt_begin, dpt_begin));
  chk(upload(&h->d_dpo_slot, dpo_slot));
  {
    std::vector<int32_t> dslot_po((size_t)std::max<int64_t>(h->ndep_slots, 1), -1);
    for (size_t k = 0; k < dpo_slot.size(); k++) dslot_po[(size_t)dpo_slot[k]] = (int32_t)k;
    chk(upload(&h->d_dslot_po, dslot_po));
  }
  chk(upload(&h->d_xpt_begin, xpt_begin));
  chk(upload(&h->d_xref, xref));
  chk(upload(&h->d_xcc, xcc));
  chk(upload(&h->d_xkind, xkind));
  chk(upload(&h->d_xpid, xpid));
  chk(upload(&h->d_xorder, xorder));
  chk(dalloc(&h->d_xscal, (size_t)(1 + std::max<int64_t>((NX + 255) / 256, 1))));
  chk(dalloc(&h->d_xcnt, 1));
  if (e == hipSuccess) chk(hipMemset(h->d_xcnt, 0, sizeof(unsigned)));
  if (e != hipSuccess) {
    g_create_error = std::string("HIP error during mvba_create: ") + hipGetErrorString(e);
    free_all(h);
    delete h;
    return MVBA_E_HIP;
  }
  *out = h;
  return MVBA_OK;
}

mvba_status mvba_set_params(mvba_handle* h, const double* packed) {
  if (!h || !packed) return MVBA_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipMemcpy(h->d_params, packed, (size_t)h->nparams * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_set_params");
  h->params_set = true;
  h->prep_done = false;
  return MVBA_OK;
}

mvba_status mvba_set_params_device(mvba_handle* h, const double* dp, void* stream) {
  if (!h || !dp) return MVBA_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipMemcpyAsync(h->d_params, dp, (size_t)h->nparams * sizeof(double),
                                hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_set_params_device");
  h->params_set = true;
  h->prep_done = false;
  return MVBA_OK;
}

int32_t mvba_jacobian_stride(const mvba_handle* h) { return h ? h->jac_rows : 0; }

mvba_status mvba_residual_order(const mvba_handle* h, int64_t* out) {
  if (!h || !out) return MVBA_E_INVALID;
  std::memcpy(out, h->order.data(), h->order.size() * sizeof(int64_t));  // nslots entries
  return MVBA_OK;
}
int64_t mvba_num_residuals(const mvba_handle* h) { return h ? h->nres : 0; }
int64_t mvba_num_slots(const mvba_handle* h) { return h ? h->nslots : 0; }
int64_t mvba_num_frames(const mvba_handle* h) { return h ? h->nframes : 0; }
int64_t mvba_num_points(const mvba_handle* h) { return h ? h->npts : 0; }

double mvba_eval_bytes(const mvba_handle* h, int32_t flags) {
  if (!h) return 0.0;
  if (flags & MVBA_EVAL_DEPTH) return h->bytes_dep;
  // the prep's algorithmic bytes: per landmark the parameter
  // read 24 + offset 8 + free flag 1 + record store 32; per frame its
  // descriptor 128 + the 22 pose parameters 176 + the record store 1,152
  if (flags & MVBA_EVAL_PREP_ONLY) return 65.0 * (double)h->npts + 1456.0 * (double)h->nframes;
  return h->bytes_res + ((flags & MVBA_EVAL_JACOBIAN) ? h->bytes_jac : 0.0);
}

// Which launch form a full evaluation takes (MVBA_FORM_*); MVBA_SPLIT_PREP=1 /
// MVBA_EVAL_MODE=split|fused|local force one, for A/B timing (read per call).
// One model group: k_eval_local up to kLocalSegsPerFrame segments per frame.
// With frames in capture order it measured faster than the fused form (K0
// blocks handing records to the K1 waves) on the whole c2 (95.5-96.5 vs
// 100.9-101.5 us), equal on c3 (2.14-2.20 vs 2.17 ms), and faster on every
// shard of c2 (N = 2 / 4 / 8: 53.0 / 28.0 / 17.9 vs 57.7 / 35.0 / 24.1 us),
// profiles/r04/r04o, r04p; and against the split form (prep launch + K1) c2
// 95.7 vs 107.2 us, c3 2.14 vs 2.20 ms (profiles/r05/r05m/). Past that every
// frame's K0 runs in too many waves: c4 (~39 segments per frame) split 6.66 /
// 6.67 ms per step, local 7.58 / 7.62, fused 7.78 / 7.79 (same box,
// profiles/r05/r05w/), so the split form takes over there (c3: ~17). With the
// round-6 K0 (split common part, one K0 per frame and block) the gap narrowed
// and held: c4 local 6.35 / 6.37 vs split 6.02 / 6.03 ms, c3 local 2.19 / 2.19
// vs split 2.24 / 2.22 ms (same box, profiles/r06/r06zg/).
static constexpr double kLocalSegsPerFrame = 24.0;
static int eval_form(const mvba_handle* h) {
  const char* sp = std::getenv("MVBA_SPLIT_PREP");
  const char* m = std::getenv("MVBA_EVAL_MODE");
  const int forced = !m ? -1 : !std::strcmp(m, "split") ? 0 : !std::strcmp(m, "fused") ? 1 : !std::strcmp(m, "local") ? 2 : -1;
  if ((sp && sp[0] == '1') || forced == 0 || h->groups.size() != 1) return MVBA_FORM_SPLIT;
  if (forced > 0) return forced == 1 ? MVBA_FORM_FUSED : MVBA_FORM_LOCAL;
  if (h->nframes > 0 && (double)h->groups[0].seg_count > kLocalSegsPerFrame * (double)h->nframes)
    return MVBA_FORM_SPLIT;
  return MVBA_FORM_LOCAL;
}

int32_t mvba_eval_form(const mvba_handle* h) { return h ? eval_form(h) : -1; }

static mvba_status ensure_outputs(mvba_handle* h) {
  if (h->d_res) return MVBA_OK;
  h->ld = ((h->nslots + 63) / 64) * 64;
  if (h->ld == 0) h->ld = 64;
  hipError_t e = dalloc(&h->d_res, (size_t)(2 * h->ld));
  if (e == hipSuccess) e = dalloc(&h->d_J, (size_t)h->jac_rows * (size_t)h->ld);
  if (e != hipSuccess) return h->hip_fail(e, "allocating evaluation outputs");
  return MVBA_OK;
}

static mvba_status evaluate_device_impl(mvba_handle* h, int32_t flags, double cauchy_threshold, void* d_res,
                                        void* d_J, int64_t ld, int32_t out_f32, void* stream);

// Polls of a K0 ready word before a fused-evaluation wave gives up (~0.5 s at
// the default). MVBA_EVAL_POLL_LIMIT (read per call: tests switch it) lowers it;
// 0 makes every wave give up at once, which tests the error path.
static unsigned eval_poll_limit() {
  const char* v = std::getenv("MVBA_EVAL_POLL_LIMIT");
  return v ? (unsigned)std::strtoul(v, nullptr, 10) : (1u << 24);
}

mvba_status mvba_evaluate_device(mvba_handle* h, int32_t flags, double cauchy_threshold,
                                 double* d_res, double* d_J, int64_t ld, void* stream) {
  return evaluate_device_impl(h, flags, cauchy_threshold, d_res, d_J, ld, 0, stream);
}

mvba_status mvba_evaluate_device_f32(mvba_handle* h, int32_t flags, double cauchy_threshold, float* d_res,
                                     float* d_J, int64_t ld, void* stream) {
  if (!h) return MVBA_E_INVALID;
  if (!d_res && !d_J) return h->fail(MVBA_E_INVALID, "fp32 output needs caller-owned buffers");
  return evaluate_device_impl(h, flags, cauchy_threshold, d_res, d_J, ld, 1, stream);
}

static mvba_status evaluate_device_impl(mvba_handle* h, int32_t flags, double cauchy_threshold, void* d_res,
                                        void* d_J, int64_t ld, int32_t out_f32, void* stream) {
  if (!h) return MVBA_E_INVALID;
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  if (!d_res && !d_J) {
    mvba_status st = ensure_outputs(h);
    if (st != MVBA_OK) return st;
    d_res = h->d_res;
    d_J = (flags & MVBA_EVAL_JACOBIAN) ? h->d_J : nullptr;
    ld = h->ld;
  } else if (ld < h->nslots || (ld % 16) != 0) {
    return h->fail(MVBA_E_INVALID, "leading dimension must be >= mvba_num_slots() and a multiple of 16");
  }
  if ((flags & MVBA_EVAL_JACOBIAN) && !d_J)
    return h->fail(MVBA_E_INVALID, "Jacobian requested without a Jacobian buffer");
  if (!(flags & MVBA_EVAL_JACOBIAN)) d_J = nullptr;
  double cauchy_c = 0.0;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    if (!(cauchy_threshold > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
    cauchy_c = 1.0 / (cauchy_threshold * cauchy_threshold);
  }
  hipError_t e = hipSuccess;
  // One model group: one launch. k_eval_local (the default, eval_form): every
  // K1 wave computes its own frame's record in LDS, so neither a prep launch
  // nor a hand-off sits in front of K1. k_eval (MVBA_EVAL_MODE=fused): K0
  // blocks hand their frame records to the K1 waves of the same grid (round 3's
  // choice above four segments per frame; slower once frames are numbered in
  // capture order, profiles/r04/r04p/). Several model groups: the prep launch,
  // then K1 per group. MVBA_SPLIT_PREP=1 forces two launches (A/B timing);
  // mvba_eval_form reports the form.
  const int form = (flags & (MVBA_EVAL_SKIP_PREP | MVBA_EVAL_PREP_ONLY)) ? MVBA_FORM_SPLIT : eval_form(h);
  if (form != MVBA_FORM_SPLIT) {
    h->gen++;
    const Group& G = h->groups[0];
    if (form == MVBA_FORM_FUSED)
      e = mvba_launch_eval_fused(G.model, G.deg, h->d_segs + G.seg_begin, G.seg_count, h->d_fd, h->nframes,
                                 h->d_frec, h->d_params, h->d_pt_off, h->d_pt_free, h->npts, h->d_pts,
                                 h->d_obs_pid, h->d_obs_meas, d_res, d_J, ld, flags, cauchy_c, out_f32, h->gen,
                                 h->d_err, h->d_ready, eval_poll_limit(), s);
    else
      e = mvba_launch_eval_local(G.model, G.deg, h->d_segs + G.seg_begin, G.seg_count, h->d_fd, h->d_frec,
                                 h->d_params, h->d_pt_off, h->d_pt_free, h->npts, h->d_pts, h->d_obs_pid,
                                 h->d_obs_meas, d_res, d_J, ld, flags, cauchy_c, out_f32, h->gen, h->d_err, s);
    h->prep_done = true;
    if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_device launch");
    return MVBA_OK;
  }
  if (!(flags & MVBA_EVAL_SKIP_PREP)) {
    // The error word is never reset: K0 raises it to this evaluation's
    // generation (atomicMax), so a stale error from an earlier call is ignored.
    h->gen++;
    e = mvba_launch_prep(h->d_fd, h->nframes, h->d_params, h->d_frec, h->d_pt_off, h->d_pt_free,
                         h->npts, h->d_pts, h->gen, h->d_err, s);
    h->prep_done = true;
  } else if (!h->prep_done) {
    return h->fail(MVBA_E_INVALID, "MVBA_EVAL_SKIP_PREP before any full evaluation");
  }
  if (flags & MVBA_EVAL_PREP_ONLY) {
    if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_device launch");
    return MVBA_OK;
  }
  for (size_t g = 0; g < h->groups.size() && e == hipSuccess; g++) {
    const Group& G = h->groups[g];
    e = mvba_launch_obs(G.model, G.deg, h->d_segs + G.seg_begin, G.seg_count, h->d_fd, h->d_frec,
                        h->d_params, h->d_pts, h->d_obs_pid, h->d_obs_meas, d_res, d_J, ld, flags,
                        cauchy_c, out_f32, s);
  }
  if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_device launch");
  return MVBA_OK;
}

mvba_status mvba_sync_status(mvba_handle* h, void* stream) {
  if (!h) return MVBA_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_sync_status");
  int err[2] = {0, 0};
  e = hipMemcpy(err, h->d_err, sizeof(err), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_sync_status copy");
  const mvba_status st = device_error(err, h->gen);
  if (st != MVBA_OK) return h->fail(st, device_error_text(st));
  return MVBA_OK;
}

mvba_status mvba_device_buffers(mvba_handle* h, mvba_device_view* v) {
  if (!h || !v) return MVBA_E_INVALID;
  mvba_status st = ensure_outputs(h);
  if (st != MVBA_OK) return st;
  v->num_residuals = h->nres;
  v->num_slots = h->nslots;
  v->ld = h->ld;
  v->jac_rows = h->jac_rows;
  v->max_dist_size = h->kmax;
  v->residuals = h->d_res;
  v->jacobian = h->d_J;
  v->order = h->d_order;
  v->row_written = h->d_row_written;
  return MVBA_OK;
}

mvba_status mvba_lin_layout_info(const mvba_handle* h, mvba_lin_layout* out) {
  if (!h || !out) return MVBA_E_INVALID;
  out->cam_grad_size = h->cam_grad_size;
  out->cam_hess_size = h->cam_hess_size;
  out->num_points = h->npts;
  out->num_cam_blocks = (int32_t)h->cam_block_ids.size();
  out->supported = h->lin_ok ? 1 : 0;
  return MVBA_OK;
}

mvba_status mvba_cam_block_map(const mvba_handle* h, int32_t* block_ids, int64_t* goff, int64_t* hoff) {
  if (!h) return MVBA_E_INVALID;
  const size_t n = h->cam_block_ids.size();
  if (block_ids) std::memcpy(block_ids, h->cam_block_ids.data(), n * sizeof(int32_t));
  if (goff) std::memcpy(goff, h->cam_goff.data(), n * sizeof(int64_t));
  if (hoff) std::memcpy(hoff, h->cam_hoff.data(), n * sizeof(int64_t));
  return MVBA_OK;
}

mvba_status mvba_point_block_map(const mvba_handle* h, int32_t* block_ids) {
  if (!h || !block_ids) return MVBA_E_INVALID;
  std::memcpy(block_ids, h->pt_block_ids.data(), h->pt_block_ids.size() * sizeof(int32_t));
  return MVBA_OK;
}

mvba_status mvba_linearize_device(mvba_handle* h, int32_t flags, double cauchy_threshold,
                                  double* d_cam_grad, double* d_cam_hess, double* d_pt_grad,
                                  double* d_pt_hess, double* d_cost, void* stream) {
  if (!h) return MVBA_E_INVALID;
  if (!h->lin_ok) return h->fail(MVBA_E_INVALID, h->lin_err);
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  const bool cam_side = !(flags & MVBA_LIN_POINTS_ONLY), pt_side = !(flags & MVBA_LIN_CAMERA_ONLY);
  if (!cam_side && !pt_side) return h->fail(MVBA_E_INVALID, "MVBA_LIN_CAMERA_ONLY with MVBA_LIN_POINTS_ONLY");
  if ((cam_side && h->cam_grad_size && (!d_cam_grad || !d_cam_hess)) ||
      (pt_side && h->npts && (!d_pt_grad || !d_pt_hess)))
    return h->fail(MVBA_E_INVALID, "null output buffer");
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  if (mvba_frame_lin_size() != sizeof(mvba::FrameLinHost) || mvba_depth_desc_size() != sizeof(mvba::DepthDesc))
    return h->fail(MVBA_E_INVALID, "record layout mismatch between host and device code");
  hipStream_t s = (hipStream_t)stream;
  double cauchy_c = 0.0;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    if (!(cauchy_threshold > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
    cauchy_c = 1.0 / (cauchy_threshold * cauchy_threshold);
  }
  hipError_t e = hipSuccess;
  if (!(flags & MVBA_EVAL_SKIP_PREP)) {
    h->gen++;
    e = mvba_launch_prep(h->d_fd, h->nframes, h->d_params, h->d_frec, h->d_pt_off, h->d_pt_free,
                         h->npts, h->d_pts, h->gen, h->d_err, s);
    h->prep_done = true;
  } else if (!h->prep_done) {
    return h->fail(MVBA_E_INVALID, "MVBA_EVAL_SKIP_PREP before any full evaluation");
  }
  const int32_t lflags = flags & MVBA_EVAL_APPLY_LOSS;
  // Camera side (K2a) per model group; a single-model problem runs the point
  // side (K2b) as extra blocks of the same launch, so the two overlap on the
  // device without a second stream. Mixed models: a separate point launch.
  const bool single = h->groups.size() == 1;
  const mvba::PointExtra dc = h->point_extra();
  // deterministic camera side: slab rows per frame part / depth segment, then a
  // fixed-order gather; the first call records the slab destinations
  const bool det = cam_side && (flags & MVBA_LIN_DETERMINISTIC);
  DetPlan& D = h->lin_det;
  if (det && !D.ready)
    e = det_plan_begin(D, (int64_t)h->nparts + h->ndep_segs, mvba::lin_slab_width(h->kmax),
                       h->cam_grad_size + h->cam_hess_size + 1, s);
  if (cam_side) {
    for (size_t g = 0; g < h->groups.size() && e == hipSuccess; g++) {
      const Group& G = h->groups[g];
      const bool pts_here = single && pt_side;
      e = mvba_launch_frame_lin(G.model, G.deg, h->d_parts + G.part_begin, G.part_count, h->d_segs, h->d_fd,
                                h->d_frame_lin, h->d_frec, h->d_params, h->d_pts, h->d_obs_pid, h->d_obs_meas,
                                h->d_rep, h->cam_grad_size, h->cam_hess_size, lflags, cauchy_c,
                                pts_here ? h->d_pt_begin : nullptr, h->npts, h->d_po_frame, h->d_po_meas, d_pt_grad,
                                d_pt_hess, dc, det ? D.slab(0) : no_slab(), G.part_begin, h->lin_obsx, s);
    }
  }
  if (pt_side && (!single || !cam_side) && e == hipSuccess)
    e = mvba_launch_points_lin(single ? h->groups[0].model : -1, single ? h->groups[0].deg : 0, h->d_pt_begin,
                               h->npts, h->d_po_frame, h->d_po_meas, h->d_fd, h->d_frec, h->d_params, h->d_pts,
                               d_pt_grad, d_pt_hess, lflags, cauchy_c, dc, s);
  if (cam_side && e == hipSuccess && h->ndep_segs > 0)
    e = mvba_launch_depth_gram(h->d_dep_segs, h->ndep_segs, h->d_dep_desc, h->d_dep_pid, h->d_dep_meas, h->d_frec, h->d_params,
                               h->d_pts, h->d_frame_lin, h->d_rep, h->cam_grad_size, h->cam_hess_size, lflags,
                               cauchy_c, det ? D.slab(h->nparts) : no_slab(), s);
  if (det && e == hipSuccess && !D.ready) e = det_plan_finish(D, s);
  if (det && e == hipSuccess)
    e = mvba_launch_slab_lin(D.tier_view(), D.grid(), D.begin, D.pos, D.val, h->cam_grad_size, h->cam_hess_size,
                             d_cam_grad, d_cam_hess, d_cost, s);
  else if (cam_side && e == hipSuccess)
    e = mvba_launch_rep_reduce(h->d_rep, h->nrep, h->cam_grad_size, h->cam_hess_size, d_cam_grad, d_cam_hess, d_cost,
                               s);
  if (cam_side && e == hipSuccess && h->nxyz > 0 && d_cost) {
    e = mvba_launch_xyz_cost(h->nxyz, h->d_xpid, h->d_xref, h->d_xcc, h->d_pts, lflags, h->d_xscal + 1, h->d_xcnt,
                             h->d_xscal, s);
    if (e == hipSuccess) e = mvba_launch_axpby(1, 1.0, d_cost, 1.0, h->d_xscal, d_cost, s);
  }
  if (e != hipSuccess) return h->hip_fail(e, "mvba_linearize_device launch");
  return MVBA_OK;
}

double mvba_lin_mfma_flops(const mvba_handle* h) { return h ? h->lin_mfma_flops : 0.0; }

int64_t mvba_num_depth_residuals(const mvba_handle* h) { return h ? h->ndep : 0; }
int64_t mvba_num_depth_slots(const mvba_handle* h) { return h ? h->ndep_slots : 0; }

mvba_status mvba_depth_order(const mvba_handle* h, int64_t* out) {
  if (!h || !out) return MVBA_E_INVALID;
  if (!h->dep_order.empty()) std::memcpy(out, h->dep_order.data(), h->dep_order.size() * sizeof(int64_t));
  return MVBA_OK;
}

static mvba_status evaluate_depth_device_impl(mvba_handle* h, int32_t flags, double cauchy_threshold, void* d_res,
                                              void* d_J, int64_t ld, int32_t out_f32, void* stream);

mvba_status mvba_evaluate_depth_device(mvba_handle* h, int32_t flags, double cauchy_threshold, double* d_res,
                                       double* d_J, int64_t ld, void* stream) {
  return evaluate_depth_device_impl(h, flags, cauchy_threshold, d_res, d_J, ld, 0, stream);
}

mvba_status mvba_evaluate_depth_device_f32(mvba_handle* h, int32_t flags, double cauchy_threshold, float* d_res,
                                           float* d_J, int64_t ld, void* stream) {
  return evaluate_depth_device_impl(h, flags, cauchy_threshold, d_res, d_J, ld, 1, stream);
}

static mvba_status evaluate_depth_device_impl(mvba_handle* h, int32_t flags, double cauchy_threshold, void* d_res,
                                              void* d_J, int64_t ld, int32_t out_f32, void* stream) {
  if (!h) return MVBA_E_INVALID;
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  if (mvba_depth_desc_size() != sizeof(mvba::DepthDesc))
    return h->fail(MVBA_E_INVALID, "record layout mismatch between host and device code");
  if (ld < h->ndep_slots || (ld % 16) != 0)
    return h->fail(MVBA_E_INVALID, "leading dimension must be >= mvba_num_depth_slots() and a multiple of 16");
  if ((flags & MVBA_EVAL_JACOBIAN) && !d_J) return h->fail(MVBA_E_INVALID, "Jacobian requested without a Jacobian buffer");
  if (!(flags & MVBA_EVAL_JACOBIAN)) d_J = nullptr;
  double cauchy_c = 0.0;
  if (flags & MVBA_EVAL_APPLY_LOSS) {
    if (!(cauchy_threshold > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
    cauchy_c = 1.0 / (cauchy_threshold * cauchy_threshold);
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (!(flags & MVBA_EVAL_SKIP_PREP)) {
    h->gen++;
    e = mvba_launch_prep(h->d_fd, h->nframes, h->d_params, h->d_frec, h->d_pt_off, h->d_pt_free, h->npts, h->d_pts,
                         h->gen, h->d_err, s);
    h->prep_done = true;
  } else if (!h->prep_done) {
    return h->fail(MVBA_E_INVALID, "MVBA_EVAL_SKIP_PREP before any full evaluation");
  }
  if (e == hipSuccess && !(flags & MVBA_EVAL_PREP_ONLY))
    e = mvba_launch_depth_obs(h->d_dep_segs, h->ndep_segs, h->d_dep_desc, h->d_dep_pid, h->d_dep_meas, h->d_fd, h->d_frec,
                              h->d_params, h->d_pts, d_res, d_J, ld, flags & (MVBA_EVAL_APPLY_LOSS), cauchy_c,
                              out_f32, s);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_depth_device launch");
  return MVBA_OK;
}

int64_t mvba_num_xyz_residuals(const mvba_handle* h) { return h ? h->nxyz : 0; }

mvba_status mvba_evaluate_xyz(mvba_handle* h, int32_t flags, double* cost, double* residuals, double* jacobian) {
  if (!h) return MVBA_E_INVALID;
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  const int64_t NX = h->nxyz;
  if (NX == 0) {
    if (cost) *cost = 0.0;
    return MVBA_OK;
  }
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipSuccess;
  if (!h->d_xout) e = dalloc(&h->d_xout, (size_t)(3 * NX));
  // points gathered by the prep kernel (K0), then raw residuals in insertion order
  h->gen++;
  if (e == hipSuccess)
    e = mvba_launch_prep(h->d_fd, h->nframes, h->d_params, h->d_frec, h->d_pt_off, h->d_pt_free, h->npts, h->d_pts,
                         h->gen, h->d_err, nullptr);
  h->prep_done = true;
  if (e == hipSuccess) e = mvba_launch_xyz_eval(NX, h->d_xpid, h->d_xorder, h->d_xref, h->d_pts, h->d_xout, nullptr);
  std::vector<double> raw((size_t)(3 * NX)), w((size_t)NX), thr((size_t)NX);
  if (e == hipSuccess) e = hipMemcpy(raw.data(), h->d_xout, raw.size() * sizeof(double), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_xyz");
  // weights / thresholds in insertion order (for the Jacobian and the corrector)
  std::vector<double4> xref((size_t)NX);
  std::vector<double> xcc((size_t)NX);
  std::vector<int64_t> xorder((size_t)NX);
  e = hipMemcpy(xref.data(), h->d_xref, xref.size() * sizeof(double4), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(xcc.data(), h->d_xcc, xcc.size() * sizeof(double), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(xorder.data(), h->d_xorder, xorder.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_evaluate_xyz");
  const bool loss = (flags & MVBA_EVAL_APPLY_LOSS) != 0;
  double total = 0.0;
  std::vector<double> cj((size_t)NX);
  for (int64_t q = 0; q < NX; q++) {
    const int64_t j = xorder[q];
    const double c = xcc[q];
    const double* r = &raw[(size_t)(3 * j)];
    const double s2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    double sr = 1.0;
    if (loss) {
      if (!(c > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
      const double sum = 1.0 + s2 * c;
      cj[(size_t)j] = 0.5 * (std::log(sum) / c);
      sr = std::sqrt(std::max(std::numeric_limits<double>::min(), 1.0 / sum));
    } else {
      cj[(size_t)j] = 0.5 * s2;
    }
    if (residuals)
      for (int k = 0; k < 3; k++) residuals[3 * j + k] = r[k] * sr;
    if (jacobian && (flags & MVBA_EVAL_JACOBIAN))  // constant point: NULL jacobian in Ceres -> zeros
      for (int a = 0; a < 3; a++)
        for (int k = 0; k < 3; k++)
          jacobian[9 * j + 3 * a + k] = (a == k && h->xfree[(size_t)j]) ? xref[q].w * sr : 0.0;
  }
  for (int64_t j = 0; j < NX; j++) total += cj[(size_t)j];
  if (cost) *cost = total;
  return mvba_sync_status(h, nullptr);
}

mvba_status mvba_frame_poses(mvba_handle* h, double* out, int32_t* frame_of_residual) {
  if (!h || !out) return MVBA_E_INVALID;
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  mvba_status st = mvba_evaluate_device(h, MVBA_EVAL_PREP_ONLY, 0.0, nullptr, nullptr, 0, nullptr);
  if (st != MVBA_OK) return st;
  st = mvba_sync_status(h, nullptr);
  if (st != MVBA_OK) return st;
  if (h->nframes > 0) {
    hipError_t e = hipMemcpy2D(out, 12 * sizeof(double), h->d_frec, mvba::kFrameRecDoubles * sizeof(double),
                               12 * sizeof(double), (size_t)h->nframes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return h->hip_fail(e, "mvba_frame_poses");
  }
  if (frame_of_residual) std::memcpy(frame_of_residual, h->res_frame.data(), h->res_frame.size() * sizeof(int32_t));
  return MVBA_OK;
}

}  // extern "C"
