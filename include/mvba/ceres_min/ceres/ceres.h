// Minimal declaration of the parts of the Ceres Solver public interface that the
// mvba adapter implements against (ceres/cost_function.h, ceres/loss_function.h,
// ceres/evaluation_callback.h, and the ceres/problem.h calls the adapter and its
// test make: AddResidualBlock, GetResidualBlocks, GetCostFunctionForResidualBlock,
// GetParameterBlocksForResidualBlock, NumResidualBlocks; Ceres 1.14 / 2.x [ext]). Used ONLY when the real
// Ceres headers are not on the include path (this container has no Ceres).
// With a real Ceres install, put its include directory first and this file is
// never seen.
#ifndef MVBA_CERES_MIN_CERES_H_
#define MVBA_CERES_MIN_CERES_H_

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <memory>
#include <set>
#include <vector>

namespace ceres {

typedef int32_t int32;

class CostFunction {
 public:
  CostFunction() : num_residuals_(0) {}
  virtual ~CostFunction() {}
  virtual bool Evaluate(double const* const* parameters, double* residuals,
                        double** jacobians) const = 0;
  const std::vector<int32>& parameter_block_sizes() const { return parameter_block_sizes_; }
  int num_residuals() const { return num_residuals_; }

 protected:
  std::vector<int32>* mutable_parameter_block_sizes() { return &parameter_block_sizes_; }
  void set_num_residuals(int num_residuals) { num_residuals_ = num_residuals; }

 private:
  std::vector<int32> parameter_block_sizes_;
  int num_residuals_;
};

class LossFunction {
 public:
  virtual ~LossFunction() {}
  virtual void Evaluate(double sq_norm, double out[3]) const = 0;
};

// rho(s) = b log(1 + s/b), b = a^2 (Ceres loss_function.cc [ext]).
class CauchyLoss : public LossFunction {
 public:
  explicit CauchyLoss(double a) : b_(a * a), c_(1.0 / b_) {}
  void Evaluate(double s, double rho[3]) const override {
    const double sum = 1.0 + s * c_;
    const double inv = 1.0 / sum;
    rho[0] = b_ * std::log(sum);
    rho[1] = std::max(std::numeric_limits<double>::min(), inv);
    rho[2] = -c_ * (inv * inv);
  }

 private:
  const double b_, c_;
};

class EvaluationCallback {
 public:
  virtual ~EvaluationCallback() {}
  virtual void PrepareForEvaluation(bool evaluate_jacobians, bool new_evaluation_point) = 0;
};

namespace internal {
struct ResidualBlock {
  CostFunction* cost;
  LossFunction* loss;
  std::vector<double*> blocks;
};
}  // namespace internal
typedef internal::ResidualBlock* ResidualBlockId;

// Residual-block bookkeeping only (no solver). Owns cost and loss functions as
// Problem does by default (Ownership TAKE_OWNERSHIP).
class Problem {
 public:
  Problem() {}
  Problem(const Problem&) = delete;
  Problem& operator=(const Problem&) = delete;
  ~Problem() {
    std::set<CostFunction*> costs;
    std::set<LossFunction*> losses;
    for (auto& r : residuals_) {
      costs.insert(r->cost);
      if (r->loss) losses.insert(r->loss);
    }
    for (CostFunction* c : costs) delete c;
    for (LossFunction* l : losses) delete l;
  }
  template <class... Ts>
  ResidualBlockId AddResidualBlock(CostFunction* cost, LossFunction* loss, double* x0, Ts*... xs) {
    return AddResidualBlock(cost, loss, std::vector<double*>{x0, xs...});
  }
  ResidualBlockId AddResidualBlock(CostFunction* cost, LossFunction* loss, const std::vector<double*>& blocks) {
    residuals_.emplace_back(new internal::ResidualBlock{cost, loss, blocks});
    return residuals_.back().get();
  }
  void SetParameterBlockConstant(double* values) { constant_.insert(values); }
  int NumResidualBlocks() const { return (int)residuals_.size(); }
  void GetResidualBlocks(std::vector<ResidualBlockId>* ids) const {
    ids->clear();
    for (auto& r : residuals_) ids->push_back(r.get());
  }
  const CostFunction* GetCostFunctionForResidualBlock(const ResidualBlockId id) const { return id->cost; }
  const LossFunction* GetLossFunctionForResidualBlock(const ResidualBlockId id) const { return id->loss; }
  void GetParameterBlocksForResidualBlock(const ResidualBlockId id, std::vector<double*>* blocks) const {
    *blocks = id->blocks;
  }

 private:
  std::vector<std::unique_ptr<internal::ResidualBlock>> residuals_;
  std::set<double*> constant_;
};

}  // namespace ceres

#endif  // MVBA_CERES_MIN_CERES_H_
