// Exercises include/mvba/ceres_surface.h the way Ceres drives a CostFunction.
// Input: a problem dump written by tests/test_ceres_surface_gpu.py. Output: the
// residuals/jacobians Evaluate() returned, for comparison with the oracle.
// Cases: (0) lazy refresh (Problem::Evaluate path, no callback),
// (1) some jacobians NULL, (2) parameters changed in user memory -> refresh,
// (3) evaluation point not in user memory -> Evaluate() returns false,
// (4) callback path, (5) 8 threads evaluating concurrently,
// (6) packed transfer: blocks Ceres never asks for stop crossing PCIe after the
//     first Jacobian pass, and asking for one later extends the set,
// (7) BracketedDepthError + XYZError blocks served from the same batch,
// (8) the reference's own statements (rig_calibrator.cc:1674-1677, :1695-1699,
//     :1762-1785, :1816-1828, :1868-1873) with only the namespace qualifier
//     changed: static Create factories of the batch in scope, blocks read back
//     from the ceres::Problem at the first evaluation.
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "mvba/ceres_surface.h"

// Test stand-ins for the reference's value types (Eigen::Vector2d / Vector3d
// and camera::CameraParameters): the factories only index the vectors and call
// GetDistortion().size() / GetDistortedHalfSize().
struct Vec {
  double v[3] = {0, 0, 0};
  Vec(double a, double b, double c = 0) : v{a, b, c} {}
  double operator[](int i) const { return v[i]; }
};
namespace camera {
class CameraParameters {
 public:
  CameraParameters(int K, const double* half) : dist_((size_t)K, 0.0), half_{half[0], half[1]} {}
  const std::vector<double>& GetDistortion() const { return dist_; }
  const std::array<double, 2>& GetDistortedHalfSize() const { return half_; }

 private:
  std::vector<double> dist_;
  std::array<double, 2> half_;
};
}  // namespace camera

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

// The thread's batch chain when batches are destroyed out of construction
// order (no GPU work: batches create their handle at the first evaluation).
// Under the ASan build a dangling prev_ shows up as a use after free.
static int chain_test() {
  auto* a = new mvba::BracketedCamBatch(0);
  auto* b = new mvba::BracketedCamBatch(0);
  auto* c = new mvba::BracketedCamBatch(0);
  int bad = 0;
  auto expect = [&](mvba::BracketedCamBatch* want, const char* what) {
    mvba::BracketedCamBatch* got = nullptr;
    try { got = &mvba::BracketedCamBatch::Current(); } catch (const std::exception&) {}
    if (got != want) { std::fprintf(stderr, "chain: %s\n", what); bad++; }
  };
  expect(c, "newest batch is current");
  delete b;  // middle first
  expect(c, "current unchanged after deleting the middle batch");
  delete c;
  expect(a, "falls back past the deleted middle batch");
  auto* d = new mvba::BracketedCamBatch(0);
  delete a;  // oldest while a newer one lives
  expect(d, "current unchanged after deleting the oldest batch");
  delete d;
  expect(nullptr, "empty chain");
  std::printf("chain %s\n", bad ? "FAILED" : "ok");
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc == 2 && std::string(argv[1]) == "--chain") return chain_test();
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
  auto dblocks = read_vec<int32_t>(in);  // depth blocks [7 nd]
  auto dsizes = read_vec<int32_t>(in);   // depth_to_image width per depth block
  auto dmeas = read_vec<double>(in);
  auto dweight = read_vec<double>(in);
  auto dstamps = read_vec<double>(in);
  auto xblock = read_vec<int32_t>(in);   // xyz priors
  auto xref = read_vec<double>(in);
  auto xweight = read_vec<double>(in);
  auto dmesh = read_vec<double>(in);     // [3 nd] mesh point of BracketedDepthMeshError rows (xyz block -1)
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

  // (6) a batch whose Ceres never asks for end (1) and distortion (7) Jacobians
  user = params;
  {
    mvba::BracketedCamBatch b6(0);
    std::vector<std::unique_ptr<ceres::CostFunction>> c6;
    for (int64_t i = 0; i < n; i++) {
      std::array<double*, 8> ptr;
      for (int b = 0; b < 8; b++) ptr[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
      const int c = rcam[i];
      c6.emplace_back(b6.Create(&rmeas[2 * i], rstamps[3 * i], rstamps[3 * i + 1], rstamps[3 * i + 2], bs, cam_K[c],
                                &cam_half[2 * c], ptr));
    }
    auto eval6 = [&](int null_mask, std::vector<double>& R6, std::vector<double>& J6) {
      R6.assign(2 * n, 0.0);
      J6.assign(n * stride, 0.0);
      bool ok = true;
      for (int64_t i = 0; i < n; i++) {
        const double* p[8];
        double* jp[8];
        for (int b = 0; b < 8; b++) {
          p[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
          jp[b] = (null_mask & (1 << b)) ? nullptr : &J6[i * stride + base[b]];
        }
        ok &= c6[i]->Evaluate(p, &R6[2 * i], jp);
      }
      return ok;
    };
    std::vector<double> R6, J6;
    const int nulls = (1 << 1) | (1 << 7);
    b6.callback()->PrepareForEvaluation(true, true);
    flags.push_back(eval6(nulls, R6, J6));
    const int64_t full = b6.transferred_jacobian_doubles();
    b6.callback()->PrepareForEvaluation(true, true);
    flags.push_back(eval6(nulls, R6, J6));
    const int64_t packed = b6.transferred_jacobian_doubles();
    write_vec(out, R6); write_vec(out, J6);
    // now a block that was not transferred: one more GPU pass, then served
    before = b6.gpu_evaluations();
    flags.push_back(eval6(0, R6, J6));
    flags.push_back((int32_t)(b6.gpu_evaluations() - before));
    write_vec(out, J6);
    std::vector<int64_t> sizes6 = {full, packed, b6.transferred_jacobian_doubles()};
    write_vec(out, sizes6);
  }

  // (7) depth + xyz blocks next to the reprojection blocks of the same images
  const int64_t nd = (int64_t)dweight.size(), nx = (int64_t)xweight.size();
  {
    mvba::BracketedCamBatch b7(0);
    std::vector<std::unique_ptr<ceres::CostFunction>> c7, d7, x7;
    auto is_mesh = [&](int64_t j) { return dblocks[7 * j + 5] == -1; };
    for (int64_t i = 0; i < n; i++) {
      std::array<double*, 8> ptr;
      for (int b = 0; b < 8; b++) ptr[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
      const int c = rcam[i];
      c7.emplace_back(b7.Create(&rmeas[2 * i], rstamps[3 * i], rstamps[3 * i + 1], rstamps[3 * i + 2], bs, cam_K[c],
                                &cam_half[2 * c], ptr));
    }
    for (int64_t j = 0; j < nd; j++) {
      if (is_mesh(j)) {  // BracketedDepthMeshError: beg, end, ref_to_cam, depth_to_image, scale, offset
        std::array<double*, 6> ptr;
        for (int b = 0; b < 6; b++) ptr[b] = &user[(size_t)block_offset[dblocks[7 * j + (b < 5 ? b : 6)]]];
        const std::vector<int> dbs = {7, 7, 7, dsizes[j], 1, 1};
        d7.emplace_back(b7.CreateDepthMesh(dweight[j], &dmeas[3 * j], &dmesh[3 * j], dstamps[3 * j],
                                           dstamps[3 * j + 1], dstamps[3 * j + 2], dbs, ptr));
        continue;
      }
      std::array<double*, 7> ptr;
      for (int b = 0; b < 7; b++) ptr[b] = &user[(size_t)block_offset[dblocks[7 * j + b]]];
      const std::vector<int> dbs = {7, 7, 7, dsizes[j], 1, 3, 1};
      d7.emplace_back(b7.CreateDepth(dweight[j], &dmeas[3 * j], dstamps[3 * j], dstamps[3 * j + 1],
                                     dstamps[3 * j + 2], dbs, ptr));
    }
    for (int64_t j = 0; j < nx; j++)
      x7.emplace_back(b7.CreateXyz(&xref[3 * j], {3}, xweight[j], &user[(size_t)block_offset[xblock[j]]]));
    static const int dbase[7] = {0, 21, 42, 63, 99, 102, 111};
    std::vector<double> RD(3 * nd), JD(114 * nd, 0.0), RX(3 * nx), JX(9 * nx);
    b7.callback()->PrepareForEvaluation(true, true);
    bool ok = true;
    for (int64_t j = 0; j < nd; j++) {
      const double* p[7];
      double* jp[7];
      int q = 0;
      for (int b = 0; b < 7; b++) {
        if (is_mesh(j) && b == 5) continue;  // no point block: its rows stay zero
        p[q] = &user[(size_t)block_offset[dblocks[7 * j + b]]];
        jp[q++] = &JD[114 * j + dbase[b]];
      }
      ok &= d7[j]->Evaluate(p, &RD[3 * j], jp);
    }
    for (int64_t j = 0; j < nx; j++) {
      const double* p[1] = {&user[(size_t)block_offset[xblock[j]]]};
      double* jp[1] = {&JX[9 * j]};
      ok &= x7[j]->Evaluate(p, &RX[3 * j], jp);
    }
    flags.push_back(ok);
    flags.push_back((int32_t)b7.gpu_evaluations());
    write_vec(out, RD); write_vec(out, JD); write_vec(out, RX); write_vec(out, JX);
  }
  // (8) the reference's statements; parameter blocks as in the reference's
  // arrays (here: slices of `user`), loss functions owned by the problem
  {
    ceres::Problem problem;
    mvba::BracketedCamBatch batch8(problem);
    std::vector<camera::CameraParameters> cam_params;
    for (size_t c = 0; c < cam_K.size(); c++) cam_params.emplace_back(cam_K[c], &cam_half[2 * c]);
    const std::vector<int> bracketed_cam_block_sizes = {7, 7, 7, 3, 1, 1, 2, 1};
    const double FLAGS_robust_threshold = 3.0;
    std::vector<ceres::CostFunction*> c8, d8, x8;
    for (int64_t i = 0; i < n; i++) {
      auto blk = [&](int b) { return &user[(size_t)block_offset[rblocks[8 * i + b]]]; };
      double *beg_cam_ptr = blk(0), *end_cam_ptr = blk(1), *ref_to_cam_ptr = blk(2), *xyz_ptr = blk(3),
             *offset_ptr = blk(4), *focal_ptr = blk(5), *center_ptr = blk(6), *distortion_ptr = blk(7);
      const int cam_type = rcam[i];
      double beg_ref_timestamp = rstamps[3 * i], end_ref_timestamp = rstamps[3 * i + 1],
             cam_timestamp = rstamps[3 * i + 2];
      Vec dist_ip(rmeas[2 * i], rmeas[2 * i + 1]);

      ceres::CostFunction* bracketed_cost_function =
        mvba::BracketedCamError::Create(dist_ip, beg_ref_timestamp, end_ref_timestamp,
                                        cam_timestamp, bracketed_cam_block_sizes,
                                        cam_params[cam_type]);
      ceres::LossFunction* bracketed_loss_function = new ceres::CauchyLoss(FLAGS_robust_threshold);
      problem.AddResidualBlock
        (bracketed_cost_function, bracketed_loss_function,
         beg_cam_ptr, end_cam_ptr, ref_to_cam_ptr, xyz_ptr,
         offset_ptr, focal_ptr, center_ptr, distortion_ptr);
      c8.push_back(bracketed_cost_function);
    }
    auto is_mesh = [&](int64_t j) { return dblocks[7 * j + 5] == -1; };
    for (int64_t j = 0; j < nd; j++) {
      auto blk = [&](int b) { return &user[(size_t)block_offset[dblocks[7 * j + b]]]; };
      double *beg_cam_ptr = blk(0), *end_cam_ptr = blk(1), *ref_to_cam_ptr = blk(2);
      double beg_ref_timestamp = dstamps[3 * j], end_ref_timestamp = dstamps[3 * j + 1],
             cam_timestamp = dstamps[3 * j + 2];
      Vec depth_xyz(dmeas[3 * j], dmeas[3 * j + 1], dmeas[3 * j + 2]);
      ceres::LossFunction* loss = new ceres::CauchyLoss(FLAGS_robust_threshold);
      if (is_mesh(j)) {
        const std::vector<int> bracketed_depth_mesh_block_sizes = {7, 7, 7, dsizes[j], 1, 1};
        Vec mesh_xyz(dmesh[3 * j], dmesh[3 * j + 1], dmesh[3 * j + 2]);
        ceres::CostFunction* bracketed_depth_mesh_cost_function
          = mvba::BracketedDepthMeshError::Create
          (dweight[j], depth_xyz, mesh_xyz, beg_ref_timestamp,
           end_ref_timestamp, cam_timestamp, bracketed_depth_mesh_block_sizes);
        problem.AddResidualBlock
          (bracketed_depth_mesh_cost_function, loss,
           beg_cam_ptr, end_cam_ptr, ref_to_cam_ptr, blk(3), blk(4), blk(6));
        d8.push_back(bracketed_depth_mesh_cost_function);
        continue;
      }
      const std::vector<int> bracketed_depth_block_sizes = {7, 7, 7, dsizes[j], 1, 3, 1};
      ceres::CostFunction* bracketed_depth_cost_function
        = mvba::BracketedDepthError::Create(dweight[j], depth_xyz, beg_ref_timestamp,
                                            end_ref_timestamp, cam_timestamp,
                                            bracketed_depth_block_sizes);
      problem.AddResidualBlock
        (bracketed_depth_cost_function, loss,
         beg_cam_ptr, end_cam_ptr, ref_to_cam_ptr, blk(3), blk(4), blk(5), blk(6));
      d8.push_back(bracketed_depth_cost_function);
    }
    const std::vector<int> xyz_block_sizes = {3};
    for (int64_t j = 0; j < nx; j++) {
      Vec avg_mesh_xyz(xref[3 * j], xref[3 * j + 1], xref[3 * j + 2]);
      ceres::CostFunction* mesh_cost_function =
        mvba::XYZError::Create(avg_mesh_xyz, xyz_block_sizes, xweight[j]);
      problem.AddResidualBlock(mesh_cost_function, new ceres::CauchyLoss(FLAGS_robust_threshold),
                               &user[(size_t)block_offset[xblock[j]]]);
      x8.push_back(mesh_cost_function);
    }
    // Problem::Evaluate-style lazy pass (no callback), then the callback pass
    std::vector<double> R8, J8;
    bool ok = true;
    R8.assign(2 * n, 0.0);
    J8.assign(n * stride, 0.0);
    for (int64_t i = 0; i < n; i++) {
      const double* p[8];
      double* jp[8];
      for (int b = 0; b < 8; b++) {
        p[b] = &user[(size_t)block_offset[rblocks[8 * i + b]]];
        jp[b] = &J8[i * stride + base[b]];
      }
      ok &= c8[(size_t)i]->Evaluate(p, &R8[2 * i], jp);
    }
    static const int dbase[7] = {0, 21, 42, 63, 99, 102, 111};
    std::vector<double> RD(3 * nd), JD(114 * nd, 0.0), RX(3 * nx), JX(9 * nx);
    batch8.callback()->PrepareForEvaluation(true, true);
    for (int64_t j = 0; j < nd; j++) {
      const double* p[7];
      double* jp[7];
      int q = 0;
      for (int b = 0; b < 7; b++) {
        if (is_mesh(j) && b == 5) continue;
        p[q] = &user[(size_t)block_offset[dblocks[7 * j + b]]];
        jp[q++] = &JD[114 * j + dbase[b]];
      }
      ok &= d8[(size_t)j]->Evaluate(p, &RD[3 * j], jp);
    }
    for (int64_t j = 0; j < nx; j++) {
      const double* p[1] = {&user[(size_t)block_offset[xblock[j]]]};
      double* jp[1] = {&JX[9 * j]};
      ok &= x8[(size_t)j]->Evaluate(p, &RX[3 * j], jp);
    }
    flags.push_back(ok);
    flags.push_back((int32_t)batch8.gpu_evaluations());
    flags.push_back((int32_t)problem.NumResidualBlocks());
    write_vec(out, R8); write_vec(out, J8);
    write_vec(out, RD); write_vec(out, JD); write_vec(out, RX); write_vec(out, JX);
  }
  // a static factory whose batch in scope is not bound to a problem (here the
  // first, explicit-pointer batch, already evaluated) throws, not crashes
  {
    camera::CameraParameters cp(0, &cam_half[0]);
    int32_t threw = 0;
    try {
      mvba::BracketedCamError::Create(Vec(1, 2), 0.0, 1.0, 0.5, {7, 7, 7, 3, 1, 1, 2, 1}, cp);
    } catch (const std::runtime_error&) {
      threw = 1;
    }
    flags.push_back(threw);
  }
  write_vec(out, flags);
  return 0;
}
