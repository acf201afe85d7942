// Exercises include/mvba/ceres_surface.h the way Ceres drives a CostFunction.
// Input: a problem dump written by tests/test_ceres_surface_gpu.py. Output: the
// residuals/jacobians Evaluate() returned, for comparison with the oracle.
// Cases: (0) lazy refresh (Problem::Evaluate path, no callback),
// (1) some jacobians NULL, (2) parameters changed in user memory -> refresh,
// (3) evaluation point not in user memory -> Evaluate() returns false,
// (4) callback path, (5) 8 threads evaluating concurrently.
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <thread>
#include <vector>

#include "mvba/ceres_surface.h"

template <class T>
static std::vector<T> read_vec(std::ifstream& f) {
  int64_t n = 0;
  f.read(reinterpret_cast<char*>(&n), 8);
  std::vector<T> v((size_t)n);
  f.read(reinterpret_cast<char*>(v.data()), n * (int64_t)sizeof(T));
  return v;
}
template <class T>
static void write_vec(std::ofstream& f, const std::vector<T>& v) {
  int64_t n = (int64_t)v.size();
  f.write(reinterpret_cast<const char*>(&n), 8);
  f.write(reinterpret_cast<const char*>(v.data()), n * (int64_t)sizeof(T));
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  std::ifstream in(argv[1], std::ios::binary);
  auto block_size = read_vec<int32_t>(in);
  auto block_offset = read_vec<int64_t>(in);
  auto params = read_vec<double>(in);
  auto cam_K = read_vec<int32_t>(in);
  auto cam_half = read_vec<double>(in);
  auto rblocks = read_vec<int32_t>(in);
  auto rcam = read_vec<int32_t>(in);
  auto rmeas = read_vec<double>(in);
  auto rstamps = read_vec<double>(in);
  auto params2 = read_vec<double>(in);  // a second evaluation point
  const int64_t n = (int64_t)rcam.size();

  std::vector<double> user = params;  // the integrator's parameter arrays
  mvba::BracketedCamBatch batch(0);
  std::vector<std::unique_ptr<ceres::CostFunction>> costs;
  const std::vector<int> bs = {7, 7, 7, 3, 1, 1, 2, 1};
  for (int64_t i = 0; i < n; i++) {
    std::array<double*, 8> ptr;
    for (int b = 0; b < 8; b++) ptr[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
    const int c = rcam[i];
    costs.emplace_back(batch.Create(&rmeas[2 * i], rstamps[3 * i], rstamps[3 * i + 1], rstamps[3 * i + 2], bs,
                                    cam_K[c], &cam_half[2 * c], ptr));
  }
  int kmax = 0;
  for (int k : cam_K) kmax = std::max(kmax, k);
  const int stride = 56 + 2 * kmax;
  static const int base[8] = {0, 14, 28, 42, 48, 50, 52, 56};

  auto eval_all = [&](bool jac, std::vector<double>& R, std::vector<double>& J, int null_mask,
                      const std::vector<double>& at) {
    R.assign(2 * n, 0.0);
    J.assign(n * stride, 0.0);
    bool ok = true;
    for (int64_t i = 0; i < n; i++) {
      const double* p[8];
      double* jp[8];
      for (int b = 0; b < 8; b++) {
        p[b] = &at[(size_t)block_offset[rblocks[8 * i + b]]];
        jp[b] = (jac && !(null_mask & (1 << b))) ? &J[i * stride + base[b]] : nullptr;
      }
      ok &= costs[i]->Evaluate(p, &R[2 * i], jac ? jp : nullptr);
    }
    return ok;
  };

  std::ofstream out(argv[2], std::ios::binary);
  std::vector<double> R, J;
  std::vector<int32_t> flags;
  // (0) lazy refresh, all jacobians
  flags.push_back(eval_all(true, R, J, 0, user));
  write_vec(out, R); write_vec(out, J);
  // (1) NULL jacobians for end (1) and distortion (7)
  flags.push_back(eval_all(true, R, J, (1 << 1) | (1 << 7), user));
  write_vec(out, J);
  // (2) new values in user memory -> lazy refresh
  user = params2;
  int64_t before = batch.gpu_evaluations();
  flags.push_back(eval_all(true, R, J, 0, user));
  flags.push_back((int32_t)(batch.gpu_evaluations() - before));
  write_vec(out, R); write_vec(out, J);
  // (3) a point that is not in user memory
  std::vector<double> other = params;
  flags.push_back(eval_all(false, R, J, 0, other));
  // (4) callback path: Ceres copies the point to user memory, then calls the callback
  user = params;
  before = batch.gpu_evaluations();
  batch.callback()->PrepareForEvaluation(true, true);
  flags.push_back(eval_all(true, R, J, 0, user));
  flags.push_back((int32_t)(batch.gpu_evaluations() - before));
  write_vec(out, R); write_vec(out, J);
  // (5) concurrent Evaluate after a change of point
  user = params2;
  std::vector<double> R5(2 * n), J5(n * stride);
  std::atomic<int> bad(0);
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++)
    th.emplace_back([&, t] {
      for (int64_t i = t; i < n; i += 8) {
        const double* p[8];
        double* jp[8];
        for (int b = 0; b < 8; b++) {
          p[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
          jp[b] = &J5[i * stride + base[b]];
        }
        if (!costs[i]->Evaluate(p, &R5[2 * i], jp)) bad++;
      }
    });
  for (auto& t : th) t.join();
  flags.push_back(bad.load());
  write_vec(out, R5); write_vec(out, J5);
  write_vec(out, flags);
  return 0;
}
