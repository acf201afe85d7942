// ceres_surface.h — drop-in ceres::CostFunction for rig_calibrator's
// BracketedCamError, evaluated in batches on the GPU through the C ABI.
//
// Reference being replaced:
//   dense_map::BracketedCamError::Create(meas, left, right, cam_stamp, block_sizes,
//                                        cam_params)        rig_calibrator.cc:485-505
//   problem.AddResidualBlock(cost, loss, beg, end, ref_to_cam, xyz, offset, focal,
//                            center, dist)                  rig_calibrator.cc:1695-1699
//
// Usage: one BracketedCamBatch per ceres::Problem;
//   ceres::CostFunction* cost = batch.Create(meas, left, right, cam, block_sizes,
//       cam_params.GetDistortion().size(), cam_params.GetDistortedHalfSize().data(),
//       {beg, end, ref_to_cam, xyz, offset, focal, center, dist});
//   problem.AddResidualBlock(cost, loss, beg, end, ref_to_cam, xyz, offset, focal, center, dist);
//   options.evaluation_callback = batch.callback();   // Ceres 1.14 (2.x: Problem::Options)
//
// Semantics: Evaluate() returns what BracketedCamError + numeric differentiation
// return (raw residuals; row-major 2 x size_b jacobians; NULL blocks skipped;
// always true unless the GPU reports an error). All residual blocks are
// evaluated in one GPU pass whenever the parameter values change: either in
// PrepareForEvaluation (solver loop) or lazily on the first Evaluate() that
// sees new values in the user's parameter arrays (Problem::Evaluate, which does
// not fire the callback in Ceres 1.14). Thread-safe for Ceres' concurrent
// Evaluate() calls. There is no CPU fallback.
//
// Header-only on purpose: it compiles against whichever Ceres the integrator
// uses (real Ceres first on the include path; include/mvba/ceres_min otherwise).
#ifndef MVBA_CERES_SURFACE_H_
#define MVBA_CERES_SURFACE_H_

#include <ceres/ceres.h>

#include <array>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "mvba.h"

namespace mvba {

class BracketedCamBatch;

class GpuBracketedCamCost : public ceres::CostFunction {
 public:
  GpuBracketedCamCost(BracketedCamBatch* batch, int64_t index, const std::vector<int>& sizes)
      : batch_(batch), index_(index) {
    set_num_residuals(2);
    for (int s : sizes) mutable_parameter_block_sizes()->push_back(s);
  }
  bool Evaluate(double const* const* parameters, double* residuals,
                double** jacobians) const override;

 private:
  BracketedCamBatch* batch_;
  int64_t index_;
};

class BracketedCamBatch {
 public:
  explicit BracketedCamBatch(int device = 0) : device_(device), callback_(this) {}
  ~BracketedCamBatch() {
    if (h_) mvba_destroy(h_);
  }
  BracketedCamBatch(const BracketedCamBatch&) = delete;
  BracketedCamBatch& operator=(const BracketedCamBatch&) = delete;

  // Mirror of BracketedCamError::Create (rig_calibrator.cc:485-505). block_sizes
  // is the caller's [7,7,7,3,1,1,2,1] vector; element 7 is replaced by dist_size
  // exactly as the functor's constructor does (:443). Throws on the reference's
  // fatal conditions (block sizes :433-440; distortion size camera_params.cc:199-206).
  ceres::CostFunction* Create(const double meas_dist_pix[2], double left_ref_stamp,
                              double right_ref_stamp, double cam_stamp,
                              const std::vector<int>& block_sizes, int dist_size,
                              const double dist_half_size[2], const std::array<double*, 8>& blocks) {
    static const int kFixed[8] = {7, 7, 7, 3, 1, 1, 2, 1};
    if (block_sizes.size() != 8)
      throw std::runtime_error("BracketedCamError: The block sizes were not set up properly.");
    for (int b = 0; b < 8; b++)
      if (block_sizes[b] != kFixed[b])
        throw std::runtime_error("BracketedCamError: The block sizes were not set up properly.");
    if (finalized_) throw std::runtime_error("mvba: Create() after the batch was evaluated");
    std::vector<int> sizes(block_sizes.begin(), block_sizes.end());
    sizes[7] = dist_size;
    const int cam = camera_index(dist_size, dist_half_size);
    Residual r;
    for (int b = 0; b < 8; b++) r.block[b] = register_block(blocks[b], b == 7 ? std::max(dist_size, 1) : sizes[b]);
    r.cam = cam;
    r.meas[0] = meas_dist_pix[0];
    r.meas[1] = meas_dist_pix[1];
    r.stamps[0] = left_ref_stamp;
    r.stamps[1] = right_ref_stamp;
    r.stamps[2] = cam_stamp;
    res_.push_back(r);
    return new GpuBracketedCamCost(this, (int64_t)res_.size() - 1, sizes);
  }

  ceres::EvaluationCallback* callback() { return &callback_; }

  // Evaluate every residual block at the current contents of the registered
  // parameter arrays (one GPU pass). Thread-safe.
  void Refresh(bool with_jacobian) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    refresh_locked(with_jacobian);
  }

  int64_t num_residuals() const { return (int64_t)res_.size(); }
  int64_t gpu_evaluations() const { return evaluations_; }

  // Used by GpuBracketedCamCost::Evaluate.
  bool Serve(int64_t i, double const* const* parameters, double* residuals, double** jacobians) {
    const bool want_jac = jacobians != nullptr;
    {
      std::shared_lock<std::shared_mutex> lk(mu_);
      if (fresh(i, parameters, want_jac)) return copy_out(i, residuals, jacobians);
    }
    std::unique_lock<std::shared_mutex> lk(mu_);
    if (!fresh(i, parameters, want_jac)) {
      refresh_locked(want_jac || have_jac_);
      if (!fresh(i, parameters, want_jac)) {
        std::fprintf(stderr,
                     "mvba: Evaluate() called at a point that is not in the user's parameter "
                     "arrays; set Solver::Options::evaluation_callback = batch.callback().\n");
        return false;
      }
    }
    return copy_out(i, residuals, jacobians);
  }

 private:
  struct Residual {
    int32_t block[8];
    int32_t cam;
    double meas[2];
    double stamps[3];
  };
  struct Callback : public ceres::EvaluationCallback {
    explicit Callback(BracketedCamBatch* b) : batch(b) {}
    void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) override {
      (void)new_evaluation_point;
      batch->Refresh(evaluate_jacobians);
    }
    BracketedCamBatch* batch;
  };

  int register_block(double* p, int size) {
    auto it = block_index_.find(p);
    if (it != block_index_.end()) {
      if (block_size_[it->second] != size)
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
    const int64_t n = (int64_t)res_.size();
    std::vector<int32_t> rb(8 * n), rc(n);
    std::vector<double> rm(2 * n), rs(3 * n);
    for (int64_t i = 0; i < n; i++) {
      for (int b = 0; b < 8; b++) rb[8 * i + b] = res_[i].block[b];
      rc[i] = res_[i].cam;
      rm[2 * i] = res_[i].meas[0];
      rm[2 * i + 1] = res_[i].meas[1];
      for (int k = 0; k < 3; k++) rs[3 * i + k] = res_[i].stamps[k];
    }
    // Every block is evaluated (the adapter cannot see SetParameterBlockConstant);
    // Evaluate() copies only the non-NULL jacobians Ceres asks for.
    std::vector<uint8_t> constant(block_ptr_.size(), 0);
    mvba_problem_desc d{};
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
    mvba_options o;
    std::memset(&o, 0, sizeof(o));
    o.device = device_;
    mvba_status st = mvba_create(&d, &o, &h_);
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_create: ") + mvba_create_error());
    stride_ = mvba_jacobian_stride(h_);
    snapshot_.assign((size_t)num_params_, 0.0);
    r_.assign((size_t)(2 * n), 0.0);
    finalized_ = true;
  }

  void refresh_locked(bool with_jacobian) {
    finalize_locked();
    for (size_t b = 0; b < block_ptr_.size(); b++)
      std::memcpy(&snapshot_[(size_t)block_offset_[b]], block_ptr_[b], sizeof(double) * block_size_[b]);
    mvba_status st = mvba_set_params(h_, snapshot_.data());
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_set_params: ") + mvba_last_error(h_));
    if (with_jacobian) J_.resize((size_t)res_.size() * (size_t)stride_);
    st = mvba_evaluate(h_, MVBA_EVAL_RESIDUALS | (with_jacobian ? MVBA_EVAL_JACOBIAN : 0), 0.0,
                       nullptr, r_.data(), with_jacobian ? J_.data() : nullptr);
    if (st != MVBA_OK) throw std::runtime_error(std::string("mvba_evaluate: ") + mvba_last_error(h_));
    have_jac_ = with_jacobian;
    valid_ = true;
    evaluations_++;
  }

  bool fresh(int64_t i, double const* const* parameters, bool want_jac) const {
    if (!valid_ || (want_jac && !have_jac_)) return false;
    const Residual& r = res_[i];
    for (int b = 0; b < 8; b++) {
      const int n = (b == 7) ? cam_K_[r.cam] : block_size_[r.block[b]];
      const double* snap = &snapshot_[(size_t)block_offset_[r.block[b]]];
      if (n > 0 && std::memcmp(snap, parameters[b], sizeof(double) * n) != 0) return false;
    }
    return true;
  }

  bool copy_out(int64_t i, double* residuals, double** jacobians) const {
    residuals[0] = r_[2 * i];
    residuals[1] = r_[2 * i + 1];
    if (!jacobians) return true;
    static const int base[8] = {MVBA_JAC_BASE_BEG, MVBA_JAC_BASE_END, MVBA_JAC_BASE_REF_TO_CAM,
                                MVBA_JAC_BASE_XYZ, MVBA_JAC_BASE_OFFSET, MVBA_JAC_BASE_FOCAL,
                                MVBA_JAC_BASE_CENTER, MVBA_JAC_BASE_DIST};
    static const int fixed[7] = {7, 7, 7, 3, 1, 1, 2};
    const double* J = &J_[(size_t)i * stride_];
    const int K = cam_K_[res_[i].cam];
    for (int b = 0; b < 8; b++) {
      if (!jacobians[b]) continue;
      const int n = 2 * (b == 7 ? K : fixed[b]);
      std::memcpy(jacobians[b], J + base[b], sizeof(double) * n);
    }
    return true;
  }

  int device_;
  Callback callback_;
  mvba_handle* h_ = nullptr;
  bool finalized_ = false, valid_ = false, have_jac_ = false;
  int32_t stride_ = 0;
  int64_t num_params_ = 0;
  int64_t evaluations_ = 0;
  std::unordered_map<const double*, int> block_index_;
  std::vector<double*> block_ptr_;
  std::vector<int32_t> block_size_;
  std::vector<int64_t> block_offset_;
  std::vector<int32_t> cam_K_;
  std::vector<double> cam_half_;
  std::vector<Residual> res_;
  std::vector<double> snapshot_, r_, J_;
  mutable std::shared_mutex mu_;
};

inline bool GpuBracketedCamCost::Evaluate(double const* const* parameters, double* residuals,
                                          double** jacobians) const {
  return batch_->Serve(index_, parameters, residuals, jacobians);
}

}  // namespace mvba

#endif  // MVBA_CERES_SURFACE_H_
