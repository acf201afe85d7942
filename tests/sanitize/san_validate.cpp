// Host-code sanitizer driver (AddressSanitizer + UBSan build, tests/sanitize/Makefile).
//
// 1. mvba_create's validation paths (rig_calibrator.cc:433-443 block sizes,
//    camera_params.cc:199-206 distortion sizes, :534-543 depth block sizes,
//    :714-715 XYZError) on hand-built descriptions: each must return its status
//    without touching memory it does not own. A valid description returns
//    MVBA_E_NO_DEVICE without a GPU; with one, the handle is exercised through
//    the host hand-over (mvba_evaluate, mvba_set_transfer_blocks,
//    mvba_evaluate_packed into pinned and pageable memory) and destroyed.
// 2. The CLI's file formats (multiview_amd/cli/rig_io.cpp): rig_config, NVM,
//    camera list and depth-cloud round trips, and malformed inputs that must
//    raise the reference's fatal messages.
// Prints one "ok <case>" line per check; exit status = number of failures.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <string>
#include <vector>

#include "mvba/mvba.h"
#include "rig_io.h"

namespace {

int g_fail = 0;

void check(bool ok, const std::string& what) {
  std::printf("%s %s\n", ok ? "ok" : "FAIL", what.c_str());
  if (!ok) g_fail++;
}

// A small valid problem: 2 sensors (radtan K=5, RPC degree 1 K=20), 3 reference
// poses, 4 points, 8 observations; one depth block and one xyz prior.
// RPC degree 1: [num_x(3) den_x(2) num_y(3) den_y(2)] per half, identity = x, y.
struct Problem {
  std::vector<int32_t> block_size;
  std::vector<int64_t> block_offset;
  std::vector<uint8_t> block_constant;
  std::vector<double> params;
  std::vector<int32_t> cam_K{5, 20};
  std::vector<double> cam_half{320, 240, 320, 240};
  std::vector<int32_t> rblocks, rcam;
  std::vector<double> rmeas, rstamps;
  std::vector<int32_t> dblocks;
  std::vector<double> dmeas, dweight, dstamps;
  std::vector<int32_t> xblock;
  std::vector<double> xref, xweight, xthr;

  int add_block(int size, const std::vector<double>& v) {
    block_size.push_back(size);
    block_offset.push_back((int64_t)params.size());
    block_constant.push_back(0);
    for (int k = 0; k < size; k++) params.push_back(k < (int)v.size() ? v[k] : 0.0);
    return (int)block_size.size() - 1;
  }

  Problem() {
    const std::vector<double> I = {0, 0, 0, 0, 0, 0, 1};
    int ref[3];
    for (int k = 0; k < 3; k++) ref[k] = add_block(7, {0.1 * k, 0, 0, 0, 0, 0.01 * k, 1});
    const int ident = add_block(7, I);
    block_constant[ident] = 1;
    const int r2c[2] = {add_block(7, I), add_block(7, {0.1, 0, 0, 0, 0.05, 0, 1})};
    const int off[2] = {add_block(1, {0}), add_block(1, {0.001})};
    block_constant[off[0]] = block_constant[off[1]] = 1;  // no bracket bounds in this driver
    const int foc[2] = {add_block(1, {300}), add_block(1, {310})};
    const int cen[2] = {add_block(2, {320, 240}), add_block(2, {321, 239})};
    std::vector<double> rpc(20, 0.0);
    rpc[1] = rpc[7] = rpc[11] = rpc[17] = 1.0;  // x and y numerators of both halves
    const int dist[2] = {add_block(5, {0.01, -0.001, 0, 0, 0}), add_block(20, rpc)};
    int pts[4];
    for (int p = 0; p < 4; p++) pts[p] = add_block(3, {0.3 * p - 0.4, 0.1 * p, 5.0 + p});
    const int dti = add_block(7, I), scale = add_block(1, {1.0});
    for (int p = 0; p < 4; p++)
      for (int s = 0; s < 2; s++) {
        const int beg = ref[p % 3];
        const bool is_ref = s == 0;
        const int end = is_ref ? ident : ref[(p % 3) + 1 < 3 ? (p % 3) + 1 : 2];
        const int blk[8] = {beg, end == beg ? ident : end, r2c[s], pts[p], off[s], foc[s], cen[s], dist[s]};
        for (int b : blk) rblocks.push_back(b);
        rcam.push_back(s);
        rmeas.push_back(300.0 + 10 * p);
        rmeas.push_back(200.0 + 5 * s);
        const double t0 = 100.0 + (p % 3), t1 = is_ref ? t0 : t0 + 1.0;
        rstamps.push_back(t0);
        rstamps.push_back(t1);
        rstamps.push_back(is_ref ? t0 : t0 + 0.5);
      }
    // a depth block on the first reprojection block's image (sensor 0)
    const int32_t* b0 = &rblocks[0];
    for (int b : {b0[0], b0[1], b0[2], dti, scale, b0[3], b0[4]}) dblocks.push_back(b);
    dmeas = {0.1, 0.2, 5.0};
    dweight = {10.0};
    dstamps = {rstamps[0], rstamps[1], rstamps[2]};
    xblock = {pts[1]};
    xref = {0.0, 0.1, 6.0};
    xweight = {0.5};
    xthr = {0.1};
  }

  mvba_problem_desc desc() {
    mvba_problem_desc d;
    std::memset(&d, 0, sizeof(d));
    d.num_blocks = (int32_t)block_size.size();
    d.block_size = block_size.data();
    d.block_offset = block_offset.data();
    d.block_constant = block_constant.data();
    d.num_param_doubles = (int64_t)params.size();
    d.num_cameras = (int32_t)cam_K.size();
    d.camera_dist_size = cam_K.data();
    d.camera_half_size = cam_half.data();
    d.num_residuals = (int64_t)rcam.size();
    d.residual_blocks = rblocks.data();
    d.residual_camera = rcam.data();
    d.residual_meas = rmeas.data();
    d.residual_stamps = rstamps.data();
    d.num_depth_residuals = (int64_t)dweight.size();
    d.depth_blocks = dblocks.data();
    d.depth_meas = dmeas.data();
    d.depth_weight = dweight.data();
    d.depth_stamps = dstamps.data();
    d.num_xyz_residuals = (int64_t)xweight.size();
    d.xyz_block = xblock.data();
    d.xyz_ref = xref.data();
    d.xyz_weight = xweight.data();
    d.xyz_threshold = xthr.data();
    return d;
  }
};

mvba_status create(Problem& P, mvba_handle** h) {
  mvba_problem_desc d = P.desc();
  mvba_options o;
  std::memset(&o, 0, sizeof(o));
  return mvba_create(&d, &o, h);
}

void expect_status(const std::string& name, std::function<void(Problem&)> mutate, mvba_status want) {
  Problem P;
  mutate(P);
  mvba_handle* h = nullptr;
  const mvba_status st = create(P, &h);
  if (h) mvba_destroy(h);
  check(st == want && h == nullptr, "create rejects " + name + " (status " + std::to_string(st) + ", " +
                                        mvba_create_error() + ")");
}

void validation() {
  expect_status("a 6-wide beg block", [](Problem& P) { P.block_size[P.rblocks[0]] = 6; }, MVBA_E_BLOCK_SIZES);
  expect_status("a distortion block of the wrong size", [](Problem& P) { P.rblocks[7] = P.rblocks[3]; },
                MVBA_E_BLOCK_SIZES);
  expect_status("K = 3", [](Problem& P) { P.cam_K[0] = 3; }, MVBA_E_BAD_DISTORTION);
  expect_status("K = 22 (no RPC degree)", [](Problem& P) { P.cam_K[1] = 22; }, MVBA_E_BAD_DISTORTION);
  expect_status("camera index out of range", [](Problem& P) { P.rcam[2] = 7; }, MVBA_E_INVALID);
  expect_status("block index out of range", [](Problem& P) { P.rblocks[5] = 100000; }, MVBA_E_INVALID);
  expect_status("negative block index", [](Problem& P) { P.rblocks[5] = -1; }, MVBA_E_INVALID);
  expect_status("block outside the packed vector", [](Problem& P) { P.block_offset[3] = (int64_t)P.params.size(); },
                MVBA_E_INVALID);
  expect_status("depth scale block of size 3", [](Problem& P) { P.dblocks[4] = P.dblocks[5]; },
                MVBA_E_DEPTH_BLOCK_SIZES);
  expect_status("depth block without an image", [](Problem& P) { P.dstamps[2] += 0.25; }, MVBA_E_INVALID);
  expect_status("xyz prior on a 7-wide block", [](Problem& P) { P.xblock[0] = P.rblocks[0]; },
                MVBA_E_XYZ_BLOCK_SIZES);
  {
    Problem P;
    mvba_problem_desc d = P.desc();
    d.residual_meas = nullptr;
    mvba_handle* h = nullptr;
    check(mvba_create(&d, nullptr, &h) == MVBA_E_INVALID && !h, "create rejects a null residual array");
    d = P.desc();
    d.num_residuals = -1;
    check(mvba_create(&d, nullptr, &h) == MVBA_E_INVALID && !h, "create rejects negative sizes");
    check(mvba_create(nullptr, nullptr, &h) == MVBA_E_INVALID, "create rejects a null description");
  }
}

void with_device() {
  Problem P;
  mvba_handle* h = nullptr;
  const mvba_status st = create(P, &h);
  int32_t ndev = 0;
  if (mvba_device_count(&ndev) != MVBA_OK) {
    check(st == MVBA_E_NO_DEVICE && h == nullptr, "valid problem without a GPU: MVBA_E_NO_DEVICE");
    return;
  }
  check(st == MVBA_OK && h != nullptr, "valid problem: handle created");
  if (!h) return;
  check(mvba_set_params(h, P.params.data()) == MVBA_OK, "set_params");
  const int64_t n = (int64_t)P.rcam.size();
  const int32_t stride = mvba_jacobian_stride(h);
  std::vector<double> r(2 * n), J((size_t)n * stride);
  double cost = 0;
  check(mvba_evaluate(h, MVBA_EVAL_RESIDUALS | MVBA_EVAL_JACOBIAN | MVBA_EVAL_APPLY_LOSS, 3.0, &cost, r.data(),
                      J.data()) == MVBA_OK && std::isfinite(cost), "evaluate (pageable)");
  std::vector<uint8_t> xfer(P.block_size.size(), 0);
  for (size_t b = 0; b < xfer.size(); b += 2) xfer[b] = 1;
  std::vector<int64_t> offs(n + 1);
  check(mvba_set_transfer_blocks(h, xfer.data(), offs.data()) == MVBA_OK && offs[n] == mvba_packed_size(h),
        "set_transfer_blocks");
  double* pinned = static_cast<double*>(mvba_host_alloc((size_t)std::max<int64_t>(offs[n], 1) * sizeof(double)));
  std::vector<double> r2(2 * n), page((size_t)std::max<int64_t>(offs[n], 1));
  check(pinned && mvba_evaluate_packed(h, MVBA_EVAL_RESIDUALS | MVBA_EVAL_JACOBIAN, 0.0, nullptr, r2.data(),
                                       pinned) == MVBA_OK, "evaluate_packed (pinned)");
  check(mvba_evaluate_packed(h, MVBA_EVAL_RESIDUALS | MVBA_EVAL_JACOBIAN, 0.0, nullptr, r2.data(), page.data()) ==
            MVBA_OK && std::memcmp(pinned, page.data(), (size_t)offs[n] * sizeof(double)) == 0,
        "evaluate_packed (pageable) equals pinned");
  mvba_host_free(pinned);
  std::vector<double> rd(3), Jd(MVBA_DJAC_ROWS);
  check(mvba_evaluate_depth(h, MVBA_EVAL_RESIDUALS | MVBA_EVAL_JACOBIAN, 0.0, &cost, rd.data(), Jd.data()) ==
            MVBA_OK, "evaluate_depth");
  mvba_solver_options o;
  mvba_solver_default_options(&o);
  o.max_num_iterations = 3;
  o.use_loss = 1;
  o.robust_threshold = 3.0;
  o.deterministic = 1;
  mvba_solver_summary s;
  std::memset(&s, 0, sizeof(s));
  const mvba_status sst = mvba_solve(h, &o, &s, nullptr);
  check(sst == MVBA_OK, "solve (deterministic): status " + std::to_string(sst) + " " + mvba_last_error(h) + " / " +
                            s.message);
  mvba_destroy(h);
}

template <class F>
bool throws_with(F f, const std::string& needle) {
  try {
    f();
  } catch (const std::exception& e) {
    return std::string(e.what()).find(needle) != std::string::npos;
  }
  return false;
}

void formats(const std::string& dir) {
  namespace fs = std::filesystem;
  using namespace rigcal;
  fs::create_directories(dir);
  RigConfig rig;
  rig.cam_names = {"nav", "haz", "sci"};
  for (int s = 0; s < 3; s++) {
    CameraParams c;
    c.focal = 600 + s;
    c.center[0] = 320.5;
    c.center[1] = 240.25;
    c.dist = s == 0 ? std::vector<double>{0.1, -0.01, 0.001, 0.002, 0.0003}
             : s == 1 ? std::vector<double>{0.9}
                      : std::vector<double>(20, 0.0);
    if (s == 2) c.dist[1] = c.dist[7] = c.dist[11] = c.dist[17] = 1.0;
    c.image_size[0] = c.crop_size[0] = c.undist_size[0] = 640;
    c.image_size[1] = c.crop_size[1] = c.undist_size[1] = 480;
    rig.params.push_back(c);
    Affine A;
    A.t[0] = 0.1 * s;
    rig.ref_to_cam.push_back(A);
    rig.depth_to_image.push_back(Affine());
    rig.offsets.push_back(0.001 * s);
  }
  write_rig_config(dir, true, rig);
  const RigConfig back = read_rig_config(dir + "/rig_config.txt", true);
  bool same = back.cam_names == rig.cam_names && back.params.size() == 3;
  for (size_t s = 0; same && s < 3; s++)
    same = back.params[s].dist == rig.params[s].dist && back.params[s].focal == rig.params[s].focal &&
           back.offsets[s] == rig.offsets[s] && std::memcmp(back.ref_to_cam[s].t, rig.ref_to_cam[s].t, 24) == 0;
  check(same, "rig_config round trip (radtan, fisheye, rpc)");
  {
    std::ofstream f(dir + "/bad_rig.txt");
    f << "ref_sensor_name: nav\n\nsensor_name: nav\nfocal_length: 600\noptical_center: 320 240\n"
         "distortion_coeffs: 1 2 3\ndistortion_type: radtan\n";
  }
  check(throws_with([&] { read_rig_config(dir + "/bad_rig.txt", true); }, ""),
        "rig_config with a 3-coefficient radtan model is refused");
  check(throws_with([&] { read_rig_config(dir + "/missing.txt", true); }, "Cannot open file for reading"),
        "missing rig_config");

  std::vector<std::vector<std::array<double, 2>>> kp = {{{1.5, 2.5}, {3.0, 4.0}}, {{5.0, 6.0}}, {{7.0, 8.0}}};
  std::vector<std::string> files = {"nav/100.0.jpg", "haz/100.5.jpg", "sci/101.0.jpg"};
  std::vector<std::map<int, int>> tracks = {{{0, 0}, {1, 0}, {2, 0}}, {{0, 1}, {2, 0}}};
  std::vector<std::array<double, 3>> xyz = {{{0.1, 0.2, 3.0}}, {{-0.4, 0.5, 4.0}}};
  std::vector<Affine> w2c(3);
  w2c[1].t[2] = 0.5;
  write_nvm_file(dir + "/m.nvm", kp, files, {600, 601, 602}, tracks, xyz, w2c);
  const NvmData nvm = read_nvm(dir + "/m.nvm");
  check(nvm.cid_to_filename == files && nvm.pid_to_xyz.size() == 2 && nvm.pid_to_cid_fid.size() == 2,
        "NVM round trip");
  {
    std::ofstream f(dir + "/bad.nvm");
    f << "NOT_NVM\n";
  }
  check(throws_with([&] { read_nvm(dir + "/bad.nvm"); }, "NVM token"), "NVM without its token is refused");

  DepthCloud c;
  c.rows = 3;
  c.cols = 4;
  c.xyz.resize(36);
  for (size_t k = 0; k < c.xyz.size(); k++) c.xyz[k] = 0.25f * (float)k;
  save_xyz_image(dir + "/d.pc", c);
  auto c2 = read_xyz_image(dir + "/d.pc");
  check(c2 && c2->rows == 3 && c2->cols == 4 && c2->xyz == c.xyz, "depth cloud round trip");
  {
    std::ofstream f(dir + "/bad.pc", std::ios::binary);
    const int32_t hdr[3] = {2, 2, 9};
    f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  }
  check(throws_with([&] { read_xyz_image(dir + "/bad.pc"); }, "Invalid depth cloud"), "bad depth cloud refused");

  save_camera_poses(dir, files, w2c);
  std::vector<std::string> f2;
  std::vector<Affine> w2;
  read_camera_poses_file(dir + "/cameras.txt", f2, w2);
  check(f2 == files && w2.size() == 3 && w2[1].t[2] == 0.5, "camera list round trip");
}

}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/mvba_san_validate";
  validation();
  with_device();
  try {
    formats(dir);
  } catch (const std::exception& e) {
    check(false, std::string("formats threw: ") + e.what());
  }
  std::printf("%d failure(s)\n", g_fail);
  return g_fail;
}
