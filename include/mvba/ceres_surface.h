// ceres_surface.h — drop-in ceres::CostFunctions for rig_calibrator's residual
// blocks, evaluated in batches on the GPU through the C ABI.
//
// References being replaced (rig_calibrator/bin/rig_calibrator.cc):
//   BracketedCamError::Create(meas, left, right, cam_stamp, block_sizes, cam_params)   :485-505
//   BracketedDepthError::Create(weight, meas_depth_xyz, left, right, cam_stamp,
//                               block_sizes)                                           :586-600
//   BracketedDepthMeshError::Create(weight, meas_depth_xyz, mesh_xyz, left, right,
//                                   cam_stamp, block_sizes)                            :677-693
//   XYZError::Create(ref_xyz, block_sizes, weight)                                     :728-741
//   problem.AddResidualBlock(cost, loss, <blocks>...)      :1695-1699, :1779-1785, :1869-1894
//
// Usage: one BracketedCamBatch per ceres::Problem,
// declared right after the problem; the reference's own statements then change
// only in their namespace qualifier (dense_map:: -> mvba::):
//   ceres::Problem problem;
//   mvba::BracketedCamBatch batch(problem);             // the batch in scope
//   ceres::CostFunction* cost = mvba::BracketedCamError::Create(dist_ip, beg_ref_timestamp,
//       end_ref_timestamp, cam_timestamp, bracketed_cam_block_sizes, cam_params[cam_type]);
//   problem.AddResidualBlock(cost, loss, beg_cam_ptr, end_cam_ptr, ref_to_cam_ptr, &xyz_vec[pid][0],
//       &ref_to_cam_timestamp_offsets[cam_type], &focal_lengths[cam_type],
//       &optical_centers[cam_type][0], distortion_ptr);             // unchanged
//   ... mvba::BracketedDepthError / BracketedDepthMeshError / XYZError::Create likewise ...
//   options.evaluation_callback = batch.callback();   // Ceres 1.14 (2.x: Problem::Options)
// The factories do not see the parameter blocks (the reference passes them to
// AddResidualBlock only): at the first evaluation the batch reads them back from
// the problem (Problem::GetResidualBlocks / GetCostFunctionForResidualBlock /
// GetParameterBlocksForResidualBlock). The member factories below
// (batch.Create(..., blocks)) take the block pointers directly instead.
//
// Semantics: Evaluate() returns what the reference functor + numeric
// differentiation return (raw residuals; row-major num_residuals x size_b
// jacobians; NULL blocks skipped; always true unless the GPU reports an error).
// All residual blocks are evaluated in one GPU pass whenever the parameter
// values change: either in PrepareForEvaluation (solver loop) or lazily on the
// first Evaluate() that sees new values in the user's parameter arrays
// (Problem::Evaluate, which does not fire the callback in Ceres 1.14).
// Thread-safe for Ceres' concurrent Evaluate() calls. There is no CPU fallback.
//
// Transfer: results cross PCIe once per GPU pass into pinned memory
// (mvba_host_alloc). The reprojection Jacobian is packed: after the first
// Jacobian pass only the columns of parameter blocks Ceres has asked for
// (non-NULL jacobians[b], i.e. not SetParameterBlockConstant) are moved; a block
// asked for later makes that pass be redone with every block, and the next
// Jacobian pass moves the blocks asked for so far.
//
// Header-only on purpose: it compiles against whichever Ceres the integrator
// uses (real Ceres first on the include path; include/mvba/ceres_min otherwise).
#ifndef MVBA_CERES_SURFACE_H_
#define MVBA_CERES_SURFACE_H_

#include <ceres/ceres.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mvba.h"

namespace mvba {

class BracketedCamBatch;

// Residual families served by one batch.
enum Family { kCam = 0, kDepth = 1, kXyz = 2 };

class GpuBatchCost : public ceres::CostFunction {
 public:
  GpuBatchCost(BracketedCamBatch* batch, Family fam, int64_t index, int nres, const std::vector<int>& sizes)
      : batch_(batch), fam_(fam), index_(index) {
    set_num_residuals(nres);
    for (int s : sizes) mutable_parameter_block_sizes()->push_back(s);
  }
  bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const override;

 private:
  BracketedCamBatch* batch_;
  Family fam_;
  int64_t index_;
};

// Pinned host buffer from the library (DMA target).
class PinnedDoubles {
 public:
  PinnedDoubles() = default;
  ~PinnedDoubles() { mvba_host_free(p_); }
  PinnedDoubles(const PinnedDoubles&) = delete;
  PinnedDoubles& operator=(const PinnedDoubles&) = delete;
  void reserve(size_t n) {
    if (n <= cap_) return;
    mvba_host_free(p_);
    p_ = static_cast<double*>(mvba_host_alloc(n * sizeof(double)));
    if (!p_) throw std::runtime_error("mvba_host_alloc failed");
    cap_ = n;
  }
  double* data() const { return p_; }
  double operator[](size_t i) const { return p_[i]; }

 private:
  double* p_ = nullptr;
  size_t cap_ = 0;
};

class BracketedCamBatch {
 public:
  // A batch fed through the member factories (block pointers given).
  explicit BracketedCamBatch(int device = 0) : device_(device), callback_(this) { push_current(); }
  // A batch bound to the problem its residual blocks are added to: the static
  // reference-signature factories (mvba::BracketedCamError::Create, ...) feed the
  // batch in scope on this thread, i.e. the most recently constructed one.
  explicit BracketedCamBatch(ceres::Problem& problem, int device = 0)
      : device_(device), problem_(&problem), callback_(this) {
    push_current();
  }
  ~BracketedCamBatch() {
    if (h_) mvba_destroy(h_);
    unlink_current();
  }

  // The batch the static factories feed (throws if none is in scope).
  static BracketedCamBatch& Current() {
    BracketedCamBatch* b = current_slot();
    if (!b) throw std::runtime_error("mvba: no BracketedCamBatch in scope (construct one with the ceres::Problem)");
    return *b;
  }
  BracketedCamBatch(const BracketedCamBatch&) = delete;
  BracketedCamBatch& operator=(const BracketedCamBatch&) = delete;

  // Mirror of BracketedCamError::Create (rig_calibrator.cc:485-505). block_sizes
  // is the caller's [7,7,7,3,1,1,2,1] vector; element 7 is replaced by dist_size
  // exactly as the functor's constructor does (:443). Throws on the reference's
  // fatal conditions (block sizes :433-440; distortion size camera_params.cc:199-206).
  ceres::CostFunction* Create(const double meas_dist_pix[2], double left_ref_stamp, double right_ref_stamp,
                              double cam_stamp, const std::vector<int>& block_sizes, int dist_size,
                              const double dist_half_size[2], const std::array<double*, 8>& blocks) {
    return CreateCam(meas_dist_pix, left_ref_stamp, right_ref_stamp, cam_stamp, block_sizes, dist_size,
                     dist_half_size, blocks.data());
  }

  // blocks == nullptr: the pointers are read back from the problem at the first
  // evaluation (the reference-signature factory's path).
  ceres::CostFunction* CreateCam(const double meas_dist_pix[2], double left_ref_stamp, double right_ref_stamp,
                                 double cam_stamp, const std::vector<int>& block_sizes, int dist_size,
                                 const double dist_half_size[2], double* const* blocks) {
    static const int kFixed[8] = {7, 7, 7, 3, 1, 1, 2, 1};
    if (block_sizes.size() != 8)
      throw std::runtime_error("BracketedCamError: The block sizes were not set up properly.");
    for (int b = 0; b < 8; b++)
      if (block_sizes[b] != kFixed[b])
        throw std::runtime_error("BracketedCamError: The block sizes were not set up properly.");
    check_open();
    std::vector<int> sizes(block_sizes.begin(), block_sizes.end());
    sizes[7] = dist_size;
    const int cam = camera_index(dist_size, dist_half_size);
    Residual r;
    r.nblocks = 8;
    for (int b = 0; b < 8; b++) {
      r.width[b] = sizes[b];
      r.block[b] = blocks ? register_block(blocks[b], b == 7 ? std::max(dist_size, 1) : sizes[b]) : -1;
    }
    r.cam = cam;
    r.meas[0] = meas_dist_pix[0];
    r.meas[1] = meas_dist_pix[1];
    r.stamps[0] = left_ref_stamp;
    r.stamps[1] = right_ref_stamp;
    r.stamps[2] = cam_stamp;
    return add(kCam, r, 2, sizes, blocks == nullptr);
  }

  // Mirror of BracketedDepthError::Create (rig_calibrator.cc:586-600) with the
  // AddResidualBlock blocks (:1779-1785): beg, end, ref_to_cam, depth_to_image
  // (7 rigid or 12 affine), scale, xyz, offset. The image the depth cloud
  // belongs to must also have BracketedCamError blocks in this batch.
  ceres::CostFunction* CreateDepth(double weight, const double meas_depth_xyz[3], double left_ref_stamp,
                                   double right_ref_stamp, double cam_stamp, const std::vector<int>& block_sizes,
                                   const std::array<double*, 7>& blocks) {
    return CreateDepthBlocks(weight, meas_depth_xyz, left_ref_stamp, right_ref_stamp, cam_stamp, block_sizes,
                             blocks.data());
  }
  ceres::CostFunction* CreateDepthBlocks(double weight, const double meas_depth_xyz[3], double left_ref_stamp,
                                         double right_ref_stamp, double cam_stamp,
                                         const std::vector<int>& block_sizes, double* const* blocks) {
    if (block_sizes.size() != 7 || block_sizes[0] != 7 || block_sizes[1] != 7 || block_sizes[2] != 7 ||
        (block_sizes[3] != 7 && block_sizes[3] != 12) || block_sizes[4] != 1 || block_sizes[5] != 3 ||
        block_sizes[6] != 1)
      throw std::runtime_error("BracketedDepthError: The block sizes were not set up properly.");
    check_open();
    Residual r;
    r.nblocks = 7;
    for (int b = 0; b < 7; b++) {
      r.block[b] = blocks ? register_block(blocks[b], block_sizes[b]) : -1;
      r.width[b] = block_sizes[b];
    }
    r.weight = weight;
    for (int k = 0; k < 3; k++) r.xyz[k] = meas_depth_xyz[k];
    r.stamps[0] = left_ref_stamp;
    r.stamps[1] = right_ref_stamp;
    r.stamps[2] = cam_stamp;
    return add(kDepth, r, 3, block_sizes, blocks == nullptr);
  }

  // Mirror of BracketedDepthMeshError::Create (rig_calibrator.cc:677-693) with the
  // AddResidualBlock blocks (:1824-1828): beg, end, ref_to_cam, depth_to_image (7
  // or 12), scale, offset; the mesh point is data (no point block).
  ceres::CostFunction* CreateDepthMesh(double weight, const double meas_depth_xyz[3], const double mesh_xyz[3],
                                       double left_ref_stamp, double right_ref_stamp, double cam_stamp,
                                       const std::vector<int>& block_sizes, const std::array<double*, 6>& blocks) {
    return CreateDepthMeshBlocks(weight, meas_depth_xyz, mesh_xyz, left_ref_stamp, right_ref_stamp, cam_stamp,
                                 block_sizes, blocks.data());
  }
  ceres::CostFunction* CreateDepthMeshBlocks(double weight, const double meas_depth_xyz[3],
                                             const double mesh_xyz[3], double left_ref_stamp,
                                             double right_ref_stamp, double cam_stamp,
                                             const std::vector<int>& block_sizes, double* const* blocks) {
    if (block_sizes.size() != 6 || block_sizes[0] != 7 || block_sizes[1] != 7 || block_sizes[2] != 7 ||
        (block_sizes[3] != 7 && block_sizes[3] != 12) || block_sizes[4] != 1 || block_sizes[5] != 1)
      throw std::runtime_error("BracketedDepthMeshError: The block sizes were not set up properly.");
    check_open();
    Residual r;
    r.nblocks = 6;
    for (int b = 0; b < 6; b++) {
      r.block[b] = blocks ? register_block(blocks[b], block_sizes[b]) : -1;
      r.width[b] = block_sizes[b];
    }
    r.weight = weight;
    r.mesh = true;
    for (int k = 0; k < 3; k++) {
      r.xyz[k] = meas_depth_xyz[k];
      r.mesh_xyz[k] = mesh_xyz[k];
    }
    r.stamps[0] = left_ref_stamp;
    r.stamps[1] = right_ref_stamp;
    r.stamps[2] = cam_stamp;
    return add(kDepth, r, 3, block_sizes, blocks == nullptr);
  }

  // Mirror of XYZError::Create (rig_calibrator.cc:728-741) on one point block.
  ceres::CostFunction* CreateXyz(const double ref_xyz[3], const std::vector<int>& block_sizes, double weight,
                                 double* xyz) {
    if (block_sizes.size() != 1 || block_sizes[0] != 3)
      throw std::runtime_error("XYZError: The block sizes were not set up properly.");
    check_open();
    Residual r;
    r.nblocks = 1;
    r.block[0] = xyz ? register_block(xyz, 3) : -1;
    r.width[0] = 3;
    r.weight = weight;
    for (int k = 0; k < 3; k++) r.xyz[k] = ref_xyz[k];
    return add(kXyz, r, 3, block_sizes, xyz == nullptr);
  }

  ceres::EvaluationCallback* callback() { return &callback_; }

  // Evaluate every residual block at the current contents of the registered
  // parameter arrays (one GPU pass). Thread-safe.
  void Refresh(bool with_jacobian) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    refresh_locked(with_jacobian);
  }

  int64_t num_residuals() const { return (int64_t)res_[kCam].size(); }
  int64_t gpu_evaluations() const { return evaluations_; }
  // Doubles of reprojection Jacobian moved per Jacobian pass (packed layout).
  int64_t transferred_jacobian_doubles() const { return packed_size_; }

  // Used by GpuBatchCost::Evaluate.
  bool Serve(Family f, int64_t i, double const* const* parameters, double* residuals, double** jacobians) {
    const bool want_jac = jacobians != nullptr;
    {
      std::shared_lock<std::shared_mutex> lk(mu_);
      if (want_jac && f == kCam && finalized_) {
        // remember which blocks Ceres wants Jacobians of (not held constant)
        const Residual& r = res_[kCam][(size_t)i];
        for (int b = 0; b < 8; b++)
          if (jacobians[b] && !asked_[(size_t)r.block[b]].load(std::memory_order_relaxed))
            asked_[(size_t)r.block[b]].store(1, std::memory_order_relaxed);
      }
      if (fresh(f, i, parameters, jacobians) == kFresh) return copy_out(f, i, residuals, jacobians);
    }
    std::unique_lock<std::shared_mutex> lk(mu_);
    const Freshness fr = fresh(f, i, parameters, jacobians);
    if (fr != kFresh) {
      // a block missing from the packed transfer: Ceres' constant set changed;
      // move every block this pass, the next Jacobian pass shrinks to the asks
      refresh_locked(want_jac || have_jac_, fr == kMissingBlock);
      if (fresh(f, i, parameters, jacobians) != kFresh) {
        std::fprintf(stderr,
                     "mvba: Evaluate() called at a point that is not in the user's parameter "
                     "arrays; set Solver::Options::evaluation_callback = batch.callback().\n");
        return false;
      }
    }
    return copy_out(f, i, residuals, jacobians);
  }

 private:
  struct Residual {
    int32_t nblocks = 0;
    int32_t block[8];
    int32_t width[8];  // Jacobian columns per block (distortion: K)
    int32_t cam = 0;
    double meas[2] = {0, 0};
    double stamps[3] = {0, 0, 0};
    double weight = 0;
    double xyz[3] = {0, 0, 0};
    bool mesh = false;            // BracketedDepthMeshError (kDepth family, 6 blocks)
    double mesh_xyz[3] = {0, 0, 0};
  };
  struct Callback : public ceres::EvaluationCallback {
    explicit Callback(BracketedCamBatch* b) : batch(b) {}
    void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
      (void)new_evaluation_point;
      batch->Refresh(evaluate_jacobians);
    }
    BracketedCamBatch* batch;
  };

  void check_open() const {
    if (finalized_) throw std::runtime_error("mvba: Create() after the batch was evaluated");
  }

  static BracketedCamBatch*& current_slot() {
    static thread_local BracketedCamBatch* cur = nullptr;
    return cur;
  }
  // Batches need not be destroyed in construction order: a batch leaves the
  // chain from wherever it sits, so no later batch's prev_ points at freed
  // memory (the top of the chain falls back to the next older live batch).
  void unlink_current() {
    BracketedCamBatch** link = &current_slot();
    while (*link && *link != this) link = &(*link)->prev_;
    if (*link == this) *link = prev_;
    prev_ = nullptr;
  }
  void push_current() {
    prev_ = current_slot();
    current_slot() = this;
  }

  ceres::CostFunction* add(Family f, const Residual& r, int nres, const std::vector<int>& sizes, bool deferred) {
    res_[f].push_back(r);
    const int64_t index = (int64_t)res_[f].size() - 1;
    GpuBatchCost* cost = new GpuBatchCost(this, f, index, nres, sizes);
    if (deferred) {
      if (!problem_)
        throw std::runtime_error("mvba: the reference-signature factories need a BracketedCamBatch constructed "
                                 "with the ceres::Problem the residual blocks are added to");
      deferred_.emplace(static_cast<const ceres::CostFunction*>(cost), std::make_pair(f, index));
    }
    return cost;
  }

  // Parameter blocks of the residuals created without them: read back from the
  // problem, in its residual-block order (= AddResidualBlock order).
  void resolve_deferred_locked() {
    if (deferred_.empty()) return;
    std::vector<ceres::ResidualBlockId> ids;
    problem_->GetResidualBlocks(&ids);
    std::vector<double*> ptrs;
    size_t resolved = 0;
    for (ceres::ResidualBlockId id : ids) {
      auto it = deferred_.find(problem_->GetCostFunctionForResidualBlock(id));
      if (it == deferred_.end()) continue;
      Residual& r = res_[it->second.first][(size_t)it->second.second];
      problem_->GetParameterBlocksForResidualBlock(id, &ptrs);
      if ((int)ptrs.size() != r.nblocks)
        throw std::runtime_error("mvba: a residual block was added with the wrong number of parameter blocks");
      for (int b = 0; b < r.nblocks; b++) {
        const bool dist = it->second.first == kCam && b == 7;
        r.block[b] = register_block(ptrs[(size_t)b], dist ? std::max(r.width[b], 1) : r.width[b]);
      }
      resolved++;
    }
    if (resolved != deferred_.size())
      throw std::runtime_error("mvba: a cost function from the batch was never added to its ceres::Problem");
    deferred_.clear();
  }

  int register_block(double* p, int size) {
    auto it = block_index_.find(p);
    if (it != block_index_.end()) {
      if (block_size_[(size_t)it->second] != size)
        throw std::runtime_error("mvba: a parameter block was registered with two sizes");
      return it->second;
    }
    const int id = (int)block_ptr_.size();
    block_index_.emplace(p, id);
    block_ptr_.push_back(p);
    block_size_.push_back(size);
    block_offset_.push_back(num_params_);
    num_params_ += size;
    return id;
  }

  int camera_index(int K, const double* half) {
    for (size_t c = 0; c < cam_K_.size(); c++)
      if (cam_K_[c] == K && cam_half_[2 * c] == half[0] && cam_half_[2 * c + 1] == half[1]) return (int)c;
    cam_K_.push_back(K);
    cam_half_.push_back(half[0]);
    cam_half_.push_back(half[1]);
    return (int)cam_K_.size() - 1;
  }

  void finalize_locked() {
    if (finalized_) return;
    resolve_deferred_locked();
    const std::vector<Residual>& C = res_[kCam];
    const std::vector<Residual>& D = res_[kDepth];
    const std::vector<Residual>& X = res_[kXyz];
    const int64_t n = (int64_t)C.size(), nd = (int64_t)D.size(), nx = (int64_t)X.size();
    std::vector<int32_t> rb(8 * n), rc(n), db(7 * nd), xb(nx);
    std::vector<double> rm(2 * n), rs(3 * n), dm(3 * nd), dw(nd), ds(3 * nd), xr(3 * nx), xw(nx), xt(nx, 1.0);
    std::vector<double> dmesh(3 * nd, 0.0);
    bool any_mesh = false;
    for (int64_t i = 0; i < n; i++) {
      for (int b = 0; b < 8; b++) rb[8 * i + b] = C[i].block[b];
      rc[i] = C[i].cam;
      rm[2 * i] = C[i].meas[0];
      rm[2 * i + 1] = C[i].meas[1];
      for (int k = 0; k < 3; k++) rs[3 * i + k] = C[i].stamps[k];
    }
    for (int64_t j = 0; j < nd; j++) {
      if (D[j].mesh) {  // 6 blocks: the MVBA_DBLK_XYZ slot is -1
        for (int b = 0; b < 7; b++)
          db[7 * j + b] = b < MVBA_DBLK_XYZ ? D[j].block[b] : b == MVBA_DBLK_XYZ ? -1 : D[j].block[b - 1];
        for (int k = 0; k < 3; k++) dmesh[3 * j + k] = D[j].mesh_xyz[k];
        any_mesh = true;
      } else {
        for (int b = 0; b < 7; b++) db[7 * j + b] = D[j].block[b];
      }
      for (int k = 0; k < 3; k++) {
        dm[3 * j + k] = D[j].xyz[k];
        ds[3 * j + k] = D[j].stamps[k];
      }
      dw[j] = D[j].weight;
    }
    for (int64_t j = 0; j < nx; j++) {
      xb[j] = X[j].block[0];
      for (int k = 0; k < 3; k++) xr[3 * j + k] = X[j].xyz[k];
      xw[j] = X[j].weight;
    }
    // Every block is evaluated (the adapter cannot see SetParameterBlockConstant);
    // Evaluate() copies only the non-NULL jacobians Ceres asks for.
    std::vector<uint8_t> constant(block_ptr_.size(), 0);
    mvba_problem_desc d;
    std::memset(&d, 0, sizeof(d));
    d.num_blocks = (int32_t)block_ptr_.size();
    d.block_size = block_size_.data();
    d.block_offset = block_offset_.data();
    d.block_constant = constant.data();
    d.num_param_doubles = num_params_;
    d.num_cameras = (int32_t)cam_K_.size();
    d.camera_dist_size = cam_K_.data();
    d.camera_half_size = cam_half_.data();
    d.num_residuals = n;
    d.residual_blocks = rb.data();
    d.residual_camera = rc.data();
    d.residual_meas = rm.data();
    d.residual_stamps = rs.data();
    d.num_depth_residuals = nd;
    d.depth_blocks = db.data();
    d.depth_meas = dm.data();
    d.depth_weight = dw.data();
    d.depth_stamps = ds.data();
    d.num_xyz_residuals = nx;
    d.xyz_block = xb.data();
    d.xyz_ref = xr.data();
    d.xyz_weight = xw.data();
    d.xyz_threshold = xt.data();
    d.depth_mesh_xyz = any_mesh ? dmesh.data() : nullptr;
    mvba_options o;
    std::memset(&o, 0, sizeof(o));
    o.device = device_;
    mvba_status st = mvba_create(&d, &o, &h_);
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_create: ") + mvba_create_error());
    snapshot_.reserve((size_t)num_params_);
    snapshot_.assign((size_t)num_params_, 0.0);
    r_[kCam].reserve((size_t)(2 * n));
    r_[kDepth].reserve((size_t)(3 * nd));
    r_[kXyz].reserve((size_t)(3 * nx));
    asked_.reset(new std::atomic<uint8_t>[block_ptr_.size()]);
    for (size_t b = 0; b < block_ptr_.size(); b++) asked_[b].store(0);
    finalized_ = true;
  }

  void set_transfer_locked(bool everything) {
    // blocks Ceres has asked Jacobians for; nothing asked yet -> every block
    const size_t nb = block_ptr_.size();
    std::vector<uint8_t> want(nb, 0);
    bool any = false;
    for (size_t b = 0; b < nb; b++) {
      want[b] = asked_[b].load(std::memory_order_relaxed);
      any = any || want[b];
    }
    if (!any || everything) std::fill(want.begin(), want.end(), 1);
    if (xfer_set_ && want == xfer_) return;
    offsets_.resize(res_[kCam].size() + 1);
    mvba_status st = mvba_set_transfer_blocks(h_, want.data(), offsets_.data());
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_set_transfer_blocks: ") + mvba_last_error(h_));
    xfer_ = want;
    xfer_set_ = true;
    packed_size_ = mvba_packed_size(h_);
  }

  void refresh_locked(bool with_jacobian, bool everything = false) {
    finalize_locked();
    for (size_t b = 0; b < block_ptr_.size(); b++)
      std::memcpy(&snapshot_[(size_t)block_offset_[b]], block_ptr_[b], sizeof(double) * block_size_[b]);
    mvba_status st = mvba_set_params(h_, snapshot_.data());
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_set_params: ") + mvba_last_error(h_));
    const int32_t flags = MVBA_EVAL_RESIDUALS | (with_jacobian ? MVBA_EVAL_JACOBIAN : 0);
    const int64_t n = (int64_t)res_[kCam].size(), nd = (int64_t)res_[kDepth].size(),
                  nx = (int64_t)res_[kXyz].size();
    if (n > 0) {
      if (with_jacobian) {
        set_transfer_locked(everything);
        J_[kCam].reserve((size_t)std::max<int64_t>(packed_size_, 1));
      }
      st = mvba_evaluate_packed(h_, flags, 0.0, nullptr, r_[kCam].data(), with_jacobian ? J_[kCam].data() : nullptr);
      if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_evaluate_packed: ") + mvba_last_error(h_));
    }
    if (nd > 0) {
      if (with_jacobian) J_[kDepth].reserve((size_t)nd * MVBA_DJAC_ROWS);
      st = mvba_evaluate_depth(h_, flags, 0.0, nullptr, r_[kDepth].data(), with_jacobian ? J_[kDepth].data() : nullptr);
      if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_evaluate_depth: ") + mvba_last_error(h_));
    }
    if (nx > 0) {
      if (with_jacobian) J_[kXyz].reserve((size_t)nx * 9);
      st = mvba_evaluate_xyz(h_, flags, nullptr, r_[kXyz].data(), with_jacobian ? J_[kXyz].data() : nullptr);
      if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_evaluate_xyz: ") + mvba_last_error(h_));
    }
    have_jac_ = with_jacobian;
    valid_ = true;
    evaluations_++;
  }

  enum Freshness { kFresh = 0, kStale = 1, kMissingBlock = 2 };

  // kFresh: the last pass evaluated this residual at `parameters` with every
  // Jacobian block asked for; kMissingBlock: same point, but a block asked for
  // was left out of the packed transfer.
  Freshness fresh(Family f, int64_t i, double const* const* parameters, double* const* jacobians) const {
    if (!valid_ || (jacobians && !have_jac_)) return kStale;
    const Residual& r = res_[f][(size_t)i];
    bool missing = false;
    for (int b = 0; b < r.nblocks; b++) {
      const int n = r.width[b];
      const double* snap = &snapshot_[(size_t)block_offset_[(size_t)r.block[b]]];
      if (n > 0 && std::memcmp(snap, parameters[b], sizeof(double) * n) != 0) return kStale;
      if (f == kCam && jacobians && jacobians[b] && !xfer_[(size_t)r.block[b]]) missing = true;
    }
    return missing ? kMissingBlock : kFresh;
  }

  bool copy_out(Family f, int64_t i, double* residuals, double** jacobians) const {
    const Residual& r = res_[f][(size_t)i];
    const int nres = f == kCam ? 2 : 3;
    for (int k = 0; k < nres; k++) residuals[k] = r_[f][(size_t)(nres * i + k)];
    if (!jacobians) return true;
    if (f == kCam) {
      // packed row: the transferred blocks in block order
      const double* src = J_[kCam].data() + offsets_[(size_t)i];
      for (int b = 0; b < 8; b++) {
        if (!xfer_[(size_t)r.block[b]]) continue;
        const int n = 2 * r.width[b];
        if (jacobians[b]) std::memcpy(jacobians[b], src, sizeof(double) * n);
        src += n;
      }
    } else if (f == kDepth) {
      static const int base[7] = {MVBA_DJAC_BASE_BEG, MVBA_DJAC_BASE_END, MVBA_DJAC_BASE_REF_TO_CAM,
                                  MVBA_DJAC_BASE_DEPTH_TO_IMAGE, MVBA_DJAC_BASE_SCALE, MVBA_DJAC_BASE_XYZ,
                                  MVBA_DJAC_BASE_OFFSET};
      const double* src = J_[kDepth].data() + (size_t)i * MVBA_DJAC_ROWS;
      for (int b = 0; b < r.nblocks; b++) {
        const int row = base[r.mesh && b >= MVBA_DBLK_XYZ ? b + 1 : b];  // mesh blocks skip the xyz rows
        if (jacobians[b]) std::memcpy(jacobians[b], src + row, sizeof(double) * 3 * r.width[b]);
      }
    } else {
      if (jacobians[0]) std::memcpy(jacobians[0], J_[kXyz].data() + (size_t)i * 9, sizeof(double) * 9);
    }
    return true;
  }

  // residual buffers: pinned, sized at finalize
  struct PinnedVec {
    PinnedDoubles buf;
    void reserve(size_t n) { buf.reserve(std::max<size_t>(n, 1)); }
    double* data() const { return buf.data(); }
    double operator[](size_t k) const { return buf[k]; }
  };

  int device_;
  ceres::Problem* problem_ = nullptr;
  BracketedCamBatch* prev_ = nullptr;
  Callback callback_;
  std::unordered_map<const ceres::CostFunction*, std::pair<Family, int64_t>> deferred_;
  mvba_handle* h_ = nullptr;
  bool finalized_ = false, valid_ = false, have_jac_ = false, xfer_set_ = false;
  int64_t num_params_ = 0;
  int64_t evaluations_ = 0;
  int64_t packed_size_ = 0;
  std::unordered_map<const double*, int> block_index_;
  std::vector<double*> block_ptr_;
  std::vector<int32_t> block_size_;
  std::vector<int64_t> block_offset_;
  std::vector<int32_t> cam_K_;
  std::vector<double> cam_half_;
  std::vector<Residual> res_[3];
  std::vector<double> snapshot_;
  PinnedVec r_[3], J_[3];
  std::vector<uint8_t> xfer_;
  std::vector<int64_t> offsets_;
  std::unique_ptr<std::atomic<uint8_t>[]> asked_;
  mutable std::shared_mutex mu_;
};

inline bool GpuBatchCost::Evaluate(double const* const* parameters, double* residuals, double** jacobians) const {
  return batch_->Serve(fam_, index_, parameters, residuals, jacobians);
}

// ---- The reference's factories, same signatures (rig_calibrator.cc:485-488,
// :586-588, :677-681, :728-730), feeding the batch in scope. Vec2 / Vec3 are
// Eigen::Vector2d / Vector3d (anything indexable); CamParams is
// camera::CameraParameters (GetDistortion().size(), GetDistortedHalfSize()).
struct BracketedCamError {
  template <class Vec2, class CamParams>
  static ceres::CostFunction* Create(Vec2 const& meas_dist_pix, double left_ref_stamp, double right_ref_stamp,
                                     double cam_stamp, std::vector<int> const& block_sizes,
                                     CamParams const& cam_params) {
    const double meas[2] = {meas_dist_pix[0], meas_dist_pix[1]};
    const auto& half = cam_params.GetDistortedHalfSize();
    const double h[2] = {half[0], half[1]};
    return BracketedCamBatch::Current().CreateCam(meas, left_ref_stamp, right_ref_stamp, cam_stamp, block_sizes,
                                                  (int)cam_params.GetDistortion().size(), h, nullptr);
  }
};

struct BracketedDepthError {
  template <class Vec3>
  static ceres::CostFunction* Create(double weight, Vec3 const& meas_depth_xyz, double left_ref_stamp,
                                     double right_ref_stamp, double cam_stamp, std::vector<int> const& block_sizes) {
    const double m[3] = {meas_depth_xyz[0], meas_depth_xyz[1], meas_depth_xyz[2]};
    return BracketedCamBatch::Current().CreateDepthBlocks(weight, m, left_ref_stamp, right_ref_stamp, cam_stamp,
                                                          block_sizes, nullptr);
  }
};

struct BracketedDepthMeshError {
  template <class Vec3>
  static ceres::CostFunction* Create(double weight, Vec3 const& meas_depth_xyz, Vec3 const& mesh_xyz,
                                     double left_ref_stamp, double right_ref_stamp, double cam_stamp,
                                     std::vector<int> const& block_sizes) {
    const double m[3] = {meas_depth_xyz[0], meas_depth_xyz[1], meas_depth_xyz[2]};
    const double x[3] = {mesh_xyz[0], mesh_xyz[1], mesh_xyz[2]};
    return BracketedCamBatch::Current().CreateDepthMeshBlocks(weight, m, x, left_ref_stamp, right_ref_stamp,
                                                              cam_stamp, block_sizes, nullptr);
  }
};

struct XYZError {
  template <class Vec3>
  static ceres::CostFunction* Create(Vec3 const& ref_xyz, std::vector<int> const& block_sizes, double weight) {
    const double x[3] = {ref_xyz[0], ref_xyz[1], ref_xyz[2]};
    return BracketedCamBatch::Current().CreateXyz(x, block_sizes, weight, nullptr);
  }
};

// The reprojection cost's previous name.
using GpuBracketedCamCost = GpuBatchCost;

}  // namespace mvba

#endif  // MVBA_CERES_SURFACE_H_
