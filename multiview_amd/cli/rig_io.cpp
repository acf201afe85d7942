// rig_io.cpp — see rig_io.h for the reference functions each routine follows.
#include "rig_io.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdint>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <stdexcept>

namespace fs = std::filesystem;

namespace rigcal {

const char* const kNoDistortion = "no_distortion";
const char* const kFisheyeDistortion = "fisheye";
const char* const kRadtanDistortion = "radtan";
const char* const kRpcDistortion = "rpc";

namespace {

[[noreturn]] void fatal(const std::string& msg) { throw std::runtime_error(msg); }

// readConfigVals, numeric flavour (dense_map_utils.cc:855-899): text after '#'
// is dropped, empty and whitespace-only lines skipped, the first token must be
// the tag, then as many numbers as parse.
std::vector<double> read_vals(std::istream& f, const std::string& tag, int want) {
  std::string line;
  while (std::getline(f, line)) {
    const size_t hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    if (line.empty()) continue;
    std::istringstream iss(line);
    std::string token;
    iss >> token;
    std::vector<double> vals;
    double v = 0;
    while (iss >> v) vals.push_back(v);
    if (token.empty()) continue;
    if (token != tag) fatal("Could not read value for: " + tag);
    if (want >= 0 && (int)vals.size() != want) fatal("Read an incorrect number of values for: " + tag);
    return vals;
  }
  fatal("Could not read value for: " + tag);
}

// readConfigVals, string flavour (:904-930): only whole-line comments.
std::vector<std::string> read_strs(std::istream& f, const std::string& tag, int want) {
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream iss(line);
    std::string token, v;
    iss >> token;
    std::vector<std::string> vals;
    while (iss >> v) vals.push_back(v);
    if (token != tag) fatal("Could not read value for: " + tag);
    if (want >= 0 && (int)vals.size() != want) fatal("Read an incorrect number of values for: " + tag);
    return vals;
  }
  fatal("Could not read value for: " + tag);
}

int rpc_degree(int n) { return (int)std::round(std::sqrt(2.0 * n + 5.0) / 2.0 - 1.5); }

}  // namespace

bool valid_rpc_size(size_t half) {
  const int d = rpc_degree((int)half);
  return d > 0 && (size_t)(2 * (d + 1) * (d + 2) - 2) == half;
}

void create_dir(const std::string& dir) {
  if (dir.empty()) return;
  std::error_code ec;
  fs::create_directories(dir, ec);
  if (ec && !fs::is_directory(dir)) fatal("Failed to create directory: " + dir);
}

RigConfig read_rig_config(const std::string& path, bool have_rig_transforms) {
  RigConfig rig;
  std::cout << "Reading: " << path << std::endl;
  std::ifstream f(path, std::ios::binary | std::ios::in);
  if (!f.is_open()) fatal("Cannot open file for reading: " + path);
  const std::string ref_name = read_strs(f, "ref_sensor_name:", 1)[0];
  for (int it = 0;; it++) {
    std::vector<std::string> sv;
    try {
      sv = read_strs(f, "sensor_name:", 1);
    } catch (...) {
      // no more sensors; the reference returns here (its trailing identity
      // check, :1047-1051, is never reached)
      return rig;
    }
    const std::string name = sv[0];
    rig.cam_names.push_back(name);
    if ((it == 0 && name != ref_name) || (it != 0 && name == ref_name))
      fatal("The reference sensor must be the first sensor specified in the rig configuration.");
    CameraParams p;
    p.focal = read_vals(f, "focal_length:", 1)[0];
    auto c = read_vals(f, "optical_center:", 2);
    p.center[0] = c[0];
    p.center[1] = c[1];
    p.dist = read_vals(f, "distortion_coeffs:", -1);
    const size_t K = p.dist.size();
    if (K != 0 && K != 1 && K != 4 && K < 5) fatal("Expecting 0, 1, 4, 5, or more distortion coefficients.");
    const std::string type = read_strs(f, "distortion_type:", 1)[0];
    if (K == 0 && type != kNoDistortion)
      fatal(std::string("When there are no distortion coefficients, distortion type must be: ") + kNoDistortion);
    if (K == 1 && type != kFisheyeDistortion)
      fatal(std::string("When there is 1 distortion coefficient, distortion type must be: ") + kFisheyeDistortion);
    if ((K == 4 || K == 5) && type != kRadtanDistortion)
      fatal(std::string("When there are 4 or 5 distortion coefficient, distortion type must be: ") +
            kRadtanDistortion);
    if (K > 5 && type != kRpcDistortion)
      fatal(std::string("When there are more than 5 distortion coefficients, distortion type must be: ") +
            kRpcDistortion);
    // CameraParameters::SetDistortion -> RPCLensDistortion::set_dist_undist_params
    // (camera_params.cc:196-205, rpc_distortion.cc:272-293)
    if (K > 5 && (K % 2 != 0 || !valid_rpc_size(K / 2))) {
      std::ostringstream os;
      os << "Recieved irregular distortion vector size. Size = " << K;
      fatal(os.str());
    }
    auto is = read_vals(f, "image_size:", 2);
    auto cs = read_vals(f, "distorted_crop_size:", 2);
    auto us = read_vals(f, "undistorted_image_size:", 2);
    for (int k = 0; k < 2; k++) {
      p.image_size[k] = (int)is[k];
      p.crop_size[k] = (int)cs[k];
      p.undist_size[k] = (int)us[k];
    }
    rig.params.push_back(p);
    auto t = read_vals(f, "ref_to_sensor_transform:", 12);
    rig.ref_to_cam.push_back(vec12_to_affine(t.data()));
    if (have_rig_transforms) {
      bool all_zero = true;
      for (double v : t) all_zero = all_zero && v == 0.0;
      if (all_zero) fatal("Failed to read valid transforms among the sensors on the rig");
    }
    auto d = read_vals(f, "depth_to_image_transform:", 12);
    rig.depth_to_image.push_back(vec12_to_affine(d.data()));
    rig.offsets.push_back(read_vals(f, "ref_to_sensor_timestamp_offset:", 1)[0]);
  }
}

std::string affine_to_str(const Affine& A) {
  std::ostringstream os;
  os.precision(17);
  os << A.R[0] << " " << A.R[1] << " " << A.R[2] << " " << A.R[3] << " " << A.R[4] << " " << A.R[5] << " " << A.R[6]
     << " " << A.R[7] << " " << A.R[8] << " " << A.t[0] << " " << A.t[1] << " " << A.t[2];
  return os.str();
}

void write_rig_config(const std::string& out_dir, bool model_rig, const RigConfig& rig) {
  create_dir(out_dir);
  const std::string path = out_dir + "/rig_config.txt";
  std::cout << "Writing: " << path << std::endl;
  std::ofstream f(path, std::ios::binary | std::ios::out);
  if (!f.is_open()) fatal("Cannot open file for writing: " + path);
  f.precision(17);
  f << "ref_sensor_name: " << rig.cam_names[0] << "\n";
  for (size_t s = 0; s < rig.params.size(); s++) {
    const CameraParams& p = rig.params[s];
    f << "\n";
    f << "sensor_name: " << rig.cam_names[s] << "\n";
    f << "focal_length: " << p.focal << "\n";
    f << "optical_center: " << p.center[0] << " " << p.center[1] << "\n";
    f << "distortion_coeffs: ";
    for (size_t d = 0; d < p.dist.size(); d++) {
      f << p.dist[d];
      if (d + 1 < p.dist.size()) f << " ";
    }
    f << "\n";
    const size_t K = p.dist.size();
    if (K == 0)
      f << "distortion_type: " << kNoDistortion << "\n";
    else if (K == 1)
      f << "distortion_type: " << kFisheyeDistortion << "\n";
    else if (K >= 4 && K <= 5)
      f << "distortion_type: " << kRadtanDistortion << "\n";
    else if (K > 5)
      f << "distortion_type: " << kRpcDistortion << "\n";
    else
      fatal("Expecting 0, 1, 4, 5, or more distortion coefficients. Got: " + std::to_string(K) + ".");
    f << "image_size: " << p.image_size[0] << ' ' << p.image_size[1] << "\n";
    f << "distorted_crop_size: " << p.crop_size[0] << ' ' << p.crop_size[1] << "\n";
    f << "undistorted_image_size: " << p.undist_size[0] << ' ' << p.undist_size[1] << "\n";
    f << "ref_to_sensor_transform: " << affine_to_str(model_rig ? rig.ref_to_cam[s] : identity()) << "\n";
    f << "depth_to_image_transform: " << affine_to_str(rig.depth_to_image[s]) << "\n";
    f << "ref_to_sensor_timestamp_offset: " << rig.offsets[s] << "\n";
  }
}

NvmData read_nvm(const std::string& path) {
  NvmData nvm;
  std::ifstream f(path, std::ios::in);
  if (!f.is_open()) fatal("Cannot open file for reading: " + path);
  std::string token;
  std::getline(f, token);
  if (token.compare(0, 6, "NVM_V3") != 0) fatal("File doesn't start with NVM token");
  long long ncid = 0;
  f >> ncid;
  if (ncid < 1) fatal("NVM file is missing cameras");
  nvm.cid_to_filename.resize((size_t)ncid);
  nvm.cid_to_keypoint.resize((size_t)ncid);
  nvm.cid_to_cam_t_global.resize((size_t)ncid);
  for (long long cid = 0; cid < ncid; cid++) {
    double focal, d1, d2, q[4], c[3];  // q = w x y z
    f >> token >> focal >> q[0] >> q[1] >> q[2] >> q[3] >> c[0] >> c[1] >> c[2] >> d1 >> d2;
    nvm.cid_to_filename[(size_t)cid] = token;
    // Eigen Quaterniond(w, x, y, z).matrix() (unnormalised input as written), t = -R c
    Affine A;
    quat_to_rot(q[1], q[2], q[3], q[0], A.R);
    for (int r = 0; r < 3; r++) A.t[r] = -(A.R[3 * r] * c[0] + A.R[3 * r + 1] * c[1] + A.R[3 * r + 2] * c[2]);
    nvm.cid_to_cam_t_global[(size_t)cid] = A;
  }
  long long npid = 0;
  f >> npid;
  if (npid < 1) fatal("The NVM file has no triangulated points.");
  nvm.pid_to_cid_fid.resize((size_t)npid);
  nvm.pid_to_xyz.resize((size_t)npid);
  for (long long pid = 0; pid < npid; pid++) {
    std::array<double, 3> xyz;
    int color[3];
    long long nm = 0;
    f >> xyz[0] >> xyz[1] >> xyz[2] >> color[0] >> color[1] >> color[2] >> nm;
    nvm.pid_to_xyz[(size_t)pid] = xyz;
    for (long long m = 0; m < nm; m++) {
      long long cid, fid;
      double px, py;
      f >> cid >> fid >> px >> py;
      if (!f.good() || cid < 0 || cid >= ncid || fid < 0) break;
      nvm.pid_to_cid_fid[(size_t)pid][(int)cid] = (int)fid;
      auto& kp = nvm.cid_to_keypoint[(size_t)cid];
      if ((long long)kp.size() <= fid) kp.resize((size_t)fid + 1, {0.0, 0.0});
      kp[(size_t)fid] = {px, py};
    }
    if (!f.good()) fatal("Unable to correctly read PID: " + std::to_string(pid));
  }
  return nvm;
}

void write_nvm_file(const std::string& path, const std::vector<std::vector<std::array<double, 2>>>& keypoints,
                    const std::vector<std::string>& filenames, const std::vector<double>& focal,
                    const std::vector<std::map<int, int>>& pid_to_cid_fid,
                    const std::vector<std::array<double, 3>>& pid_to_xyz, const std::vector<Affine>& world_to_cam) {
  create_dir(fs::path(path).parent_path().string());
  std::cout << "Writing: " << path << std::endl;
  std::fstream f(path, std::ios::out);
  if (!f.is_open()) fatal("Cannot open file for writing: " + path);
  f.precision(17);
  f << "NVM_V3\n";
  f << filenames.size() << std::endl;
  for (size_t cid = 0; cid < filenames.size(); cid++) {
    const Affine& A = world_to_cam[cid];
    double q[4];  // x y z w
    rot_to_quat(A.R, q);
    double c[3];  // camera center = -R^T t
    for (int k = 0; k < 3; k++) c[k] = -(A.R[k] * A.t[0] + A.R[3 + k] * A.t[1] + A.R[6 + k] * A.t[2]);
    f << filenames[cid] << " " << focal[cid] << " " << q[3] << " " << q[0] << " " << q[1] << " " << q[2] << " "
      << c[0] << " " << c[1] << " " << c[2] << " " << "0 0\n";
  }
  f << pid_to_cid_fid.size() << std::endl;
  for (size_t pid = 0; pid < pid_to_cid_fid.size(); pid++) {
    f << pid_to_xyz[pid][0] << " " << pid_to_xyz[pid][1] << " " << pid_to_xyz[pid][2] << " 0 0 0 "
      << pid_to_cid_fid[pid].size();
    if (pid_to_cid_fid[pid].size() <= 1)
      fatal("PID " + std::to_string(pid) + " has " + std::to_string(pid_to_cid_fid[pid].size()) + " measurements");
    for (const auto& cf : pid_to_cid_fid[pid])
      f << " " << cf.first << " " << cf.second << " " << keypoints[(size_t)cf.first][(size_t)cf.second][0] << " "
        << keypoints[(size_t)cf.first][(size_t)cf.second][1];
    f << std::endl;
  }
}

std::shared_ptr<DepthCloud> read_xyz_image(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::in);
  if (!f.is_open()) fatal("Cannot open file for reading: " + path);
  int32_t hdr[3] = {0, 0, 0};
  f.read(reinterpret_cast<char*>(hdr), sizeof(hdr));
  if (!f || hdr[0] < 0 || hdr[1] < 0 || hdr[2] < 0 || hdr[2] > 3) fatal("Invalid depth cloud: " + path);
  auto c = std::make_shared<DepthCloud>();
  c->rows = hdr[0];
  c->cols = hdr[1];
  c->xyz.assign((size_t)c->rows * (size_t)c->cols * 3, 0.0f);
  const int ch = hdr[2];
  std::vector<float> buf((size_t)c->rows * (size_t)c->cols * (size_t)ch);
  f.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
  if (!f) fatal("Truncated depth cloud: " + path);
  for (size_t p = 0; p < (size_t)c->rows * (size_t)c->cols; p++)
    for (int k = 0; k < ch; k++) c->xyz[3 * p + (size_t)k] = buf[(size_t)ch * p + (size_t)k];
  return c;
}

void save_xyz_image(const std::string& path, const DepthCloud& c) {
  std::ofstream f(path, std::ios::binary | std::ios::out);
  if (!f.is_open()) fatal("Cannot open file for writing: " + path);
  const int32_t hdr[3] = {c.rows, c.cols, 3};
  f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  f.write(reinterpret_cast<const char*>(c.xyz.data()), (std::streamsize)(c.xyz.size() * sizeof(float)));
}

ImageData read_image_entries(const std::vector<std::string>& files, const std::vector<Affine>& world_to_cam,
                             const std::vector<std::string>& cam_names, int ref_cam_type) {
  std::map<int, std::map<double, ImageMessage>> image_maps, depth_maps;
  for (size_t it = 0; it < files.size(); it++) {
    const std::string& image_file = files[it];
    const fs::path p(image_file);
    const std::string cam_name = p.parent_path().filename().string();
    const std::string base = p.filename().string();
    if (base.empty() || base[0] < '0' || base[0] > '9')
      fatal("Image name (without directory) must start with digits. Got: " + base);
    const double timestamp = std::atof(base.c_str());
    int cam_type = -1;
    for (size_t c = 0; c < cam_names.size(); c++)
      if (cam_names[c] == cam_name) {
        cam_type = (int)c;
        break;
      }
    if (cam_type < 0) fatal("Could not determine sensor name from image path: " + image_file);
    auto& im = image_maps[cam_type];
    auto& dm = depth_maps[cam_type];
    std::ostringstream ts;
    ts << std::setprecision(17) << timestamp;
    if (im.count(timestamp)) fatal("Duplicate timestamp " + ts.str() + " for sensor id " + std::to_string(cam_type));
    std::cout << "Reading: " << image_file << std::endl;
    ImageMessage& m = im[timestamp];
    m.name = image_file;
    m.timestamp = timestamp;
    m.world_to_cam = world_to_cam[it];
    if (dm.count(timestamp)) fatal("Duplicate timestamp " + ts.str() + " for sensor id " + std::to_string(cam_type));
    fs::path dp = p;
    dp.replace_extension(".pc");
    if (fs::exists(dp)) {
      std::cout << "Reading: " << dp.string() << std::endl;
      ImageMessage& d = dm[timestamp];
      d.cloud = read_xyz_image(dp.string());
      d.name = dp.string();
      d.timestamp = timestamp;
    }
  }
  // ImageDataToVectors (interest_point.cc:1462-1520)
  ImageData out;
  int max_type = 0;
  for (auto& kv : image_maps) max_type = std::max(max_type, kv.first);
  for (auto& kv : depth_maps) max_type = std::max(max_type, kv.first);
  out.images.resize((size_t)max_type + 1);
  out.depths.resize((size_t)max_type + 1);
  for (int t = 0; t <= max_type; t++) {
    auto ii = image_maps.find(t);
    if (ii != image_maps.end())
      for (auto& kv : ii->second) {
        out.images[(size_t)t].push_back(kv.second);
        if (t == ref_cam_type) {
          out.world_to_ref.push_back(kv.second.world_to_cam);
          out.ref_timestamps.push_back(kv.second.timestamp);
          out.ref_image_files.push_back(kv.second.name);
        }
      }
    auto di = depth_maps.find(t);
    if (di != depth_maps.end())
      for (auto& kv : di->second) out.depths[(size_t)t].push_back(kv.second);
  }
  return out;
}

void read_camera_poses_file(const std::string& path, std::vector<std::string>& files,
                            std::vector<Affine>& world_to_cam) {
  std::cout << "Reading: " << path << std::endl;
  std::ifstream f(path, std::ios::binary | std::ios::in);
  if (!f.is_open()) fatal("Cannot open file for reading: " + path);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream iss(line);
    std::string image_file;
    if (!(iss >> image_file)) fatal("Cannot parse the image file in: " + path);
    double vals[12];
    int count = 0;
    double v = 0;
    while (iss >> v) {
      if (count >= 12) break;
      vals[count++] = v;
    }
    if (count != 12) fatal("Expecting 12 values for the transform on line:\n" + line);
    files.push_back(image_file);
    world_to_cam.push_back(vec12_to_affine(vals));
  }
}

void save_camera_poses(const std::string& out_dir, const std::vector<std::string>& image_names,
                       const std::vector<Affine>& world_to_cam) {
  create_dir(out_dir);
  const std::string path = out_dir + "/cameras.txt";
  std::cout << "Writing: " << path << std::endl;
  std::ofstream f(path, std::ios::binary | std::ios::out);
  if (!f.is_open()) fatal("Cannot open file for writing: " + path);
  f.precision(17);
  f << "# image_file world_to_image_transform\n";
  for (size_t it = 0; it < image_names.size(); it++)
    f << image_names[it] << " " << affine_to_str(world_to_cam[it]) << "\n";
}

// ---------------------------------------------------------------- PLY meshes
namespace {

struct PlyProp {
  std::string name, type, count_type;  // count_type non-empty: list property
};
struct PlyElem {
  std::string name;
  int64_t count = 0;
  std::vector<PlyProp> props;
};

int ply_type_size(const std::string& t) {
  if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
  if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
  if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}

// One scalar of type t from a binary stream (swapping bytes when big endian).
bool ply_read_bin(std::istream& in, const std::string& t, bool big, double* out) {
  unsigned char b[8];
  const int n = ply_type_size(t);
  if (n == 0 || !in.read(reinterpret_cast<char*>(b), n)) return false;
  if (big) std::reverse(b, b + n);
  if (t == "char" || t == "int8") *out = (double)(int8_t)b[0];
  else if (t == "uchar" || t == "uint8") *out = (double)b[0];
  else if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); *out = v; }
  else if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); *out = v; }
  else if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); *out = v; }
  else if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); *out = v; }
  else if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); *out = v; }
  else { double v; std::memcpy(&v, b, 8); *out = v; }
  return true;
}

}  // namespace

bool read_ply_mesh(const std::string& path, std::vector<float>& vertices, std::vector<uint32_t>& faces,
                   std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) {
    err = "Cannot open mesh file: " + path;
    return false;
  }
  std::string line;
  std::getline(in, line);
  if (line.rfind("ply", 0) != 0) {
    err = "Not a PLY file: " + path;
    return false;
  }
  std::string format;
  std::vector<PlyElem> elems;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream is(line);
    std::string key;
    is >> key;
    if (key == "format") {
      is >> format;
    } else if (key == "element") {
      PlyElem e;
      if (!(is >> e.name >> e.count) || e.count < 0) {
        err = "Bad PLY element count in " + path;
        return false;
      }
      elems.push_back(e);
    } else if (key == "property") {
      if (elems.empty()) {
        err = "PLY property before any element: " + path;
        return false;
      }
      PlyProp p;
      std::string t;
      is >> t;
      if (t == "list") {
        is >> p.count_type >> p.type >> p.name;
      } else {
        p.type = t;
        is >> p.name;
      }
      elems.back().props.push_back(p);
    } else if (key == "end_header") {
      break;
    }
  }
  const bool ascii = format == "ascii", big = format == "binary_big_endian";
  if (!ascii && format != "binary_little_endian" && !big) {
    err = "Unsupported PLY format '" + format + "': " + path;
    return false;
  }
  vertices.clear();
  faces.clear();
  for (const PlyElem& e : elems) {
    const bool is_vertex = e.name == "vertex", is_face = e.name == "face";
    int ix = -1, iy = -1, iz = -1, iface = -1;
    for (size_t k = 0; k < e.props.size(); k++) {
      if (e.props[k].name == "x") ix = (int)k;
      if (e.props[k].name == "y") iy = (int)k;
      if (e.props[k].name == "z") iz = (int)k;
      if (!e.props[k].count_type.empty() && (e.props[k].name == "vertex_indices" || e.props[k].name == "vertex_index"))
        iface = (int)k;
    }
    if (is_vertex && (ix < 0 || iy < 0 || iz < 0)) {
      err = "PLY vertices without x, y, z: " + path;
      return false;
    }
    if (is_face && iface < 0) {
      err = "PLY faces without vertex_indices: " + path;
      return false;
    }
    std::vector<double> row;
    for (int64_t r = 0; r < e.count; r++) {
      std::istringstream ls;
      if (ascii) {
        if (!std::getline(in, line)) {
          err = "Truncated PLY file: " + path;
          return false;
        }
        ls.str(line);
      }
      auto scalar = [&](const std::string& t, double* v) -> bool {
        if (ascii) return static_cast<bool>(ls >> *v);
        return ply_read_bin(in, t, big, v);
      };
      float xyz[3] = {0, 0, 0};
      for (size_t k = 0; k < e.props.size(); k++) {
        const PlyProp& p = e.props[k];
        if (p.count_type.empty()) {
          double v;
          if (!scalar(p.type, &v)) {
            err = "Truncated PLY file: " + path;
            return false;
          }
          if ((int)k == ix) xyz[0] = (float)v;
          if ((int)k == iy) xyz[1] = (float)v;
          if ((int)k == iz) xyz[2] = (float)v;
          continue;
        }
        double cnt;
        if (!scalar(p.count_type, &cnt)) {
          err = "Truncated PLY file: " + path;
          return false;
        }
        // list lengths: faces must be triangles; anything else is read and
        // dropped, but a negative, fractional or absurd count is corruption
        if (!(cnt >= 0.0) || cnt > 1024.0 || cnt != (double)(int64_t)cnt) {
          err = "Bad PLY list count in " + path;
          return false;
        }
        row.assign((size_t)cnt, 0.0);
        for (size_t q = 0; q < row.size(); q++)
          if (!scalar(p.type, &row[q])) {
            err = "Truncated PLY file: " + path;
            return false;
          }
        if (is_face && (int)k == iface) {
          if (row.size() != 3) {
            err = "Only triangle faces are supported in " + path;
            return false;
          }
          for (double v : row) faces.push_back((uint32_t)v);
        }
      }
      if (is_vertex) vertices.insert(vertices.end(), xyz, xyz + 3);
    }
  }
  for (uint32_t f : faces)
    if ((size_t)f >= vertices.size() / 3) {
      err = "PLY face index out of range in " + path;
      return false;
    }
  return true;
}

}  // namespace rigcal
