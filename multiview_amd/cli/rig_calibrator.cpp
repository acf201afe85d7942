// rig_calibrator — the reference's calibration driver (rig_calibrator/bin/
// rig_calibrator.cc main(), :1268-2041) over the GPU library (libmvba, C ABI in
// include/mvba/mvba.h). SURVEY.md §8(b) item 3 and row f3.
//
// Same flag names and defaults (:135-316), same validation (:893-955), same
// files in and out (rig_config.txt, NVM_V3 / camera list, cameras.txt,
// cameras.nvm), same pass structure (:1548-1986):
//   world_to_cam -> triangulate (GPU) -> residual blocks -> residual stats (GPU)
//   -> Levenberg-Marquardt (GPU) -> copy back -> residual stats (GPU)
//   -> outlier flagging (GPU).
// The host side here is orchestration (file I/O, bracketing, block wiring);
// every per-observation and per-track computation runs through libmvba. There
// is no CPU compute path: --device=cpu is refused, and a missing GPU is an error.
//
// --mesh (a PLY file): after each triangulation the inlier rays are intersected
// with the mesh on the GPU (meshTriangulations, mvba_mesh_triangulate), which
// feeds --depth_mesh_weight (BracketedDepthMeshError) and --mesh_tri_weight
// (XYZError to the track's mean hit) blocks.
// Out of scope: feature detection/matching (--num_overlaps > 0),
// texturing (--out_texture_dir), registration, voxblox export, saving transformed
// clouds and match files. These flags are parsed and rejected unless left at
// their defaults.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "mvba/mvba.h"
#include "rig_io.h"
#include "rig_math.h"

namespace rigcal {

[[noreturn]] static void fatal(const std::string& msg) { throw std::runtime_error(msg); }

// ---------------------------------------------------------------- flags
// meshTriangulations' marker for "no intersection" (rig_calibrator.cc:1546)
constexpr double kBadXyz = 1.0e+100;

struct Flags {
  double robust_threshold = 3.0;
  int num_iterations = 20;
  double bracket_len = 0.6;
  std::string intrinsics_to_float, rig_transforms_to_float, camera_poses_to_float,
      depth_to_image_transforms_to_float;
  bool float_scale = false, float_timestamp_offsets = false;
  double timestamp_offsets_max_change = 1.0;
  double depth_tri_weight = 0.0;
  std::string mesh;
  double mesh_tri_weight = 0.0, depth_mesh_weight = 0.0, tri_weight = 0.0, tri_robust_threshold = 0.0;
  bool affine_depth_to_image = false;
  int calibrator_num_passes = 2;
  double initial_max_reprojection_error = 300.0, max_reprojection_error = 25.0, min_triangulation_angle = 0.5;
  std::string out_texture_dir;
  double min_ray_dist = 0.0, max_ray_dist = 100.0;
  bool registration = false;
  std::string hugin_file, xyz_file;
  double parameter_tolerance = 1e-12;
  int num_opt_threads = 16, num_match_threads = 8;
  bool no_rig = false;
  std::string out_dir, rig_config, nvm;
  bool no_nvm_matches = false;
  std::string camera_poses;
  int num_overlaps = 0;
  bool use_initial_rig_transforms = false, save_nvm = false, save_matches = false, export_to_voxblox = false,
       save_transformed_depth_clouds = false, verbose = false;
  // this build
  std::string device = "gpu";
  int num_gpus = 1;
  bool profile = false;
};

struct FlagDef {
  const char* name;
  char type;  // b i d s
  void* ptr;
  const char* help;
};

static std::vector<FlagDef> flag_table(Flags& F) {
  return {
      {"robust_threshold", 'd', &F.robust_threshold, "Cauchy loss threshold for pixel and depth residuals."},
      {"num_iterations", 'i', &F.num_iterations, "Solver iterations per pass."},
      {"bracket_len", 'd', &F.bracket_len, "Bracket non-reference images by reference images this close in time."},
      {"intrinsics_to_float", 's', &F.intrinsics_to_float,
       "Intrinsics to float per sensor, e.g. 'cam1:focal_length,optical_center,distortion cam2:focal_length'."},
      {"rig_transforms_to_float", 's', &F.rig_transforms_to_float, "Sensors whose ref-to-sensor transform floats."},
      {"camera_poses_to_float", 's', &F.camera_poses_to_float, "Sensors whose camera poses float."},
      {"depth_to_image_transforms_to_float", 's', &F.depth_to_image_transforms_to_float,
       "Sensors whose depth-to-image transform floats."},
      {"float_scale", 'b', &F.float_scale, "Float the depth-to-image scale."},
      {"float_timestamp_offsets", 'b', &F.float_timestamp_offsets, "Float the timestamp offsets."},
      {"timestamp_offsets_max_change", 'd', &F.timestamp_offsets_max_change,
       "Maximum change of a floated timestamp offset."},
      {"depth_tri_weight", 'd', &F.depth_tri_weight, "Weight of the depth-to-triangulated-point constraint."},
      {"mesh", 's', &F.mesh, "Use this mesh to help constrain the calibration (in .ply format). Must use a "
                             "positive --mesh_tri_weight."},
      {"mesh_tri_weight", 'd', &F.mesh_tri_weight, "Weight of the constraint that triangulated points stay close "
                                                  "to a preexisting mesh."},
      {"depth_mesh_weight", 'd', &F.depth_mesh_weight, "Weight of the constraint that the depth clouds stay close "
                                                      "to the mesh."},
      {"tri_weight", 'd', &F.tri_weight, "Weight keeping triangulated points near their initial values."},
      {"tri_robust_threshold", 'd', &F.tri_robust_threshold, "Cauchy threshold of the --tri_weight constraint."},
      {"affine_depth_to_image", 'b', &F.affine_depth_to_image, "Model depth-to-image as a general affine map."},
      {"calibrator_num_passes", 'i', &F.calibrator_num_passes, "Optimization passes (outliers removed after each)."},
      {"initial_max_reprojection_error", 'd', &F.initial_max_reprojection_error,
       "(feature matching only, not supported in this build)"},
      {"max_reprojection_error", 'd', &F.max_reprojection_error, "Outlier reprojection error after a pass (pixels)."},
      {"min_triangulation_angle", 'd', &F.min_triangulation_angle, "Minimum ray convergence angle (degrees)."},
      {"out_texture_dir", 's', &F.out_texture_dir, "(not supported in this build)"},
      {"min_ray_dist", 'd', &F.min_ray_dist, "Minimum search distance along a ray when intersecting it with "
                                             "the mesh, in meters."},
      {"max_ray_dist", 'd', &F.max_ray_dist, "Maximum search distance along a ray when intersecting it with "
                                             "the mesh, in meters."},
      {"registration", 'b', &F.registration, "(not supported in this build)"},
      {"hugin_file", 's', &F.hugin_file, "(registration only)"},
      {"xyz_file", 's', &F.xyz_file, "(registration only)"},
      {"parameter_tolerance", 'd', &F.parameter_tolerance, "Solver parameter tolerance."},
      {"num_opt_threads", 'i', &F.num_opt_threads, "Accepted for compatibility (the solver runs on the GPU)."},
      {"num_match_threads", 'i', &F.num_match_threads, "(feature matching only)"},
      {"no_rig", 'b', &F.no_rig, "Do not model a rig: every camera pose floats on its own."},
      {"out_dir", 's', &F.out_dir, "Output directory."},
      {"rig_config", 's', &F.rig_config, "Input rig configuration."},
      {"nvm", 's', &F.nvm, "Input NVM_V3 file (camera poses and interest point matches)."},
      {"no_nvm_matches", 'b', &F.no_nvm_matches, "Do not read matches from the nvm file."},
      {"camera_poses", 's', &F.camera_poses, "Input list of images and world-to-camera transforms."},
      {"num_overlaps", 'i', &F.num_overlaps, "(feature matching, not supported in this build)"},
      {"use_initial_rig_transforms", 'b', &F.use_initial_rig_transforms,
       "Use the rig transforms of --rig_config instead of deriving them from the camera poses."},
      {"save_nvm", 'b', &F.save_nvm, "Save the optimized poses and inlier matches as out_dir/cameras.nvm."},
      {"save_matches", 'b', &F.save_matches, "(not supported in this build)"},
      {"export_to_voxblox", 'b', &F.export_to_voxblox, "(not supported in this build)"},
      {"save_transformed_depth_clouds", 'b', &F.save_transformed_depth_clouds, "(not supported in this build)"},
      {"verbose", 'b', &F.verbose, "Verbose output."},
      {"device", 's', &F.device, "Compute device: gpu or gpu:<ordinal> (there is no CPU path)."},
      {"num_gpus", 'i', &F.num_gpus, "Shard the landmarks of each solve over this many GPUs."},
      {"profile", 'b', &F.profile, "Print per-phase timings."},
  };
}

static bool parse_bool(std::string v, bool& out) {
  std::transform(v.begin(), v.end(), v.begin(), ::tolower);
  if (v == "true" || v == "t" || v == "yes" || v == "y" || v == "1") return out = true, true;
  if (v == "false" || v == "f" || v == "no" || v == "n" || v == "0") return out = false, true;
  return false;
}

// gflags command-line syntax: --name=value, --name value, -name..., --name /
// --noname for booleans. Errors exit like gflags ("ERROR: ...", status 1).
static void parse_flags(int argc, char** argv, Flags& F) {
  auto table = flag_table(F);
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "--") break;
    if (a.size() < 2 || a[0] != '-') continue;  // positional arguments are left alone, as gflags does
    a = a.substr(a[1] == '-' ? 2 : 1);
    if (a == "help" || a == "helpfull") {
      std::cout << "rig_calibrator: calibrate a rig of cameras (MI355X build). Flags:\n";
      for (auto& d : table) std::cout << "  --" << d.name << "  " << d.help << "\n";
      std::exit(1);
    }
    std::string name = a, val;
    bool has_val = false;
    const size_t eq = a.find('=');
    if (eq != std::string::npos) {
      name = a.substr(0, eq);
      val = a.substr(eq + 1);
      has_val = true;
    }
    FlagDef* def = nullptr;
    bool negated = false;
    for (auto& d : table)
      if (name == d.name) def = &d;
    if (!def && name.rfind("no", 0) == 0 && !has_val)
      for (auto& d : table)
        if (d.type == 'b' && name.substr(2) == d.name) def = &d, negated = true;
    if (!def) {
      std::cerr << "ERROR: unknown command line flag '" << name << "'\n";
      std::exit(1);
    }
    if (def->type == 'b') {
      bool b = true;
      if (negated)
        b = false;
      else if (has_val && !parse_bool(val, b)) {
        std::cerr << "ERROR: illegal value '" << val << "' specified for bool flag '" << name << "'\n";
        std::exit(1);
      }
      *(bool*)def->ptr = b;
      continue;
    }
    if (!has_val) {
      if (i + 1 >= argc) {
        std::cerr << "ERROR: flag '" << name << "' is missing its argument\n";
        std::exit(1);
      }
      val = argv[++i];
    }
    char* end = nullptr;
    if (def->type == 's') {
      *(std::string*)def->ptr = val;
    } else if (def->type == 'i') {
      errno = 0;
      const long v = std::strtol(val.c_str(), &end, 10);
      if (val.empty() || *end || errno || v < INT32_MIN || v > INT32_MAX) {
        std::cerr << "ERROR: illegal value '" << val << "' specified for int32 flag '" << name << "'\n";
        std::exit(1);
      }
      *(int*)def->ptr = (int)v;
    } else {
      const double v = std::strtod(val.c_str(), &end);
      if (val.empty() || *end) {
        std::cerr << "ERROR: illegal value '" << val << "' specified for double flag '" << name << "'\n";
        std::exit(1);
      }
      *(double*)def->ptr = v;
    }
  }
}

// parameterValidation (rig_calibrator.cc:893-955), then this build's scope.
static void parameter_validation(const Flags& F) {
  if (F.robust_threshold <= 0.0) fatal("The robust threshold must be positive.");
  if (F.bracket_len <= 0.0) fatal("Bracket length must be positive.");
  if (F.num_overlaps < 1 && (F.nvm == "" || F.no_nvm_matches))
    fatal("No nvm file was specified or it is not desired to read its matches. Then must set a positive "
          "--num_overlaps to be able to find new interest point matches.");
  if (F.timestamp_offsets_max_change < 0) fatal("The timestamp offsets must be non-negative.");
  if (F.min_triangulation_angle <= 0.0) fatal("The min triangulation angle must be positive.");
  if (F.depth_tri_weight < 0.0) fatal("The depth weight must non-negative.");
  if (F.mesh_tri_weight < 0.0) fatal("The mesh weight must non-negative.");
  if (F.depth_mesh_weight < 0.0) fatal("The depth mesh weight must non-negative.");
  if (F.tri_weight < 0.0) fatal("The triangulation weight must non-negative.");
  if (F.tri_weight > 0.0 && F.tri_robust_threshold <= 0.0)
    fatal("The triangulation robust threshold must be positive.");
  if (F.registration && (F.xyz_file.empty() || F.hugin_file.empty()))
    fatal("In order to register the map, the hugin and xyz file must be specified.");
  if (F.float_scale && F.affine_depth_to_image)
    fatal("The options --float_scale and --affine_depth_to_image should not be used together. If the latter is "
          "used, the scale is always floated.");
  if (F.no_rig && F.float_timestamp_offsets) fatal("Cannot float timestamps with option --no_rig.");
  if (F.out_dir == "") fatal("The output directory was not specified.");
  if (F.use_initial_rig_transforms && F.no_rig) fatal("Cannot use initial rig transforms if not modeling the rig.");
  if (F.out_texture_dir != "" && F.mesh == "")
    fatal("Cannot project camera images onto a mesh if a mesh was not provided.");
  if (F.rig_config == "") fatal("Must specify the initial rig configuration via --rig_config.");
  if (F.camera_poses != "" && F.nvm != "") fatal("Cannot specify both --nvm and --camera_poses.");
  if (F.camera_poses == "" && F.nvm == "") fatal("Must specify the cameras via --nvm or --camera_poses.");

  // This build's scope: the calibration hot path only.
  auto unsupported = [](const std::string& what) {
    fatal(what + " is outside this build's scope (SURVEY.md §8(b)); leave it at its default.");
  };
  if (F.num_overlaps > 0) unsupported("--num_overlaps > 0 (feature detection and matching)");
  if (F.registration) unsupported("--registration");
  if (F.export_to_voxblox) unsupported("--export_to_voxblox");
  if (F.save_transformed_depth_clouds) unsupported("--save_transformed_depth_clouds");
  if (F.save_matches) unsupported("--save_matches");
  if (F.out_texture_dir != "") unsupported("--out_texture_dir (texturing)");
  if (F.device.rfind("gpu", 0) != 0)
    fatal("--device=" + F.device + ": this build has no CPU compute path; use --device=gpu or gpu:<ordinal>.");
  if (F.num_gpus < 1) fatal("--num_gpus must be positive.");
}

// ---------------------------------------------------------------- name lists
// replace_separators_with_space (dense_map_utils.cc:44-48)
static std::vector<std::string> split_names(std::string s) {
  for (char c : std::string("\\:, \t\r\n")) std::replace(s.begin(), s.end(), c, ' ');
  std::istringstream iss(s);
  std::vector<std::string> out;
  std::string v;
  while (iss >> v) out.push_back(v);
  return out;
}

// parse_intrinsics_to_float (dense_map_utils.cc:54-99)
static std::vector<std::set<std::string>> parse_intrinsics_to_float(const std::string& str,
                                                                    const std::vector<std::string>& names) {
  std::map<std::string, std::set<std::string>> local;
  std::string cur;
  for (const auto& v : split_names(str)) {
    if (std::find(names.begin(), names.end(), v) != names.end()) {
      cur = v;
      continue;
    }
    if (v != "focal_length" && v != "optical_center" && v != "distortion")
      fatal("Unexpected value when parsing intrinsics to float: " + v);
    if (cur == "") fatal("Incorrectly set option for floating intrinsics.");
    local[cur].insert(v);
  }
  std::vector<std::set<std::string>> out(names.size());
  for (size_t i = 0; i < names.size(); i++) out[i] = local[names[i]];
  return out;
}

// parse_camera_names (dense_map_utils.cc:102-137)
static std::set<std::string> parse_camera_names(const std::vector<std::string>& names, const std::string& str) {
  std::set<std::string> out;
  for (const auto& v : split_names(str)) {
    if (std::find(names.begin(), names.end(), v) == names.end())
      fatal("Error: A specified sensor name is not among the known sensors. Offending camera: " + v);
    out.insert(v);
  }
  return out;
}

// ---------------------------------------------------------------- images
struct CameraImage {  // dense_map::cameraImage
  int camera_type = 0;
  double timestamp = 0, ref_timestamp = 0;
  int beg_ref_index = 0, end_ref_index = 0;
  std::string image_name;
  std::shared_ptr<DepthCloud> cloud;
  std::string depth_name;
  double cloud_timestamp = -1.0;
};

// lookupImage (dense_map_utils.cc:702-739): first message at or after desired_time,
// searching forward from start_pos.
static bool lookup_image(double desired_time, const std::vector<ImageMessage>& msgs, int& start_pos,
                         double& found_time, const ImageMessage** found) {
  *found = nullptr;
  found_time = -1.0;
  double prev = -1.0;
  for (int p = start_pos; p < (int)msgs.size(); p++) {
    start_pos = p;
    found_time = msgs[(size_t)p].timestamp;
    if (found_time < prev) fatal("Found images not in chronological order.");
    prev = found_time;
    if (found_time >= desired_time) {
      *found = &msgs[(size_t)p];
      return true;
    }
  }
  return false;
}

static std::string fixed17(double v) {
  std::ostringstream os;
  os << std::fixed << std::setprecision(17) << v;
  return os.str();
}

// lookupImagesAndBrackets / lookupImagesNoBrackets / lookupImages
// (dense_map_utils.cc:1441-1805). Ties in ref_timestamp keep insertion order
// (std::stable_sort; the reference's std::sort leaves them unspecified).
static std::vector<CameraImage> lookup_images(const Flags& F, const std::vector<std::string>& names,
                                              const RigConfig& rig, const ImageData& data,
                                              std::vector<double>& min_off, std::vector<double>& max_off) {
  const int ncam = (int)names.size();
  std::vector<CameraImage> cams;
  min_off.assign((size_t)ncam, -1.0e+100);
  max_off.assign((size_t)ncam, 1.0e+100);
  std::vector<int> img_pos((size_t)ncam, 0), cloud_pos((size_t)ncam, 0);
  auto images_of = [&](int t) -> const std::vector<ImageMessage>& {
    static const std::vector<ImageMessage> none;
    return t < (int)data.images.size() ? data.images[(size_t)t] : none;
  };
  auto depths_of = [&](int t) -> const std::vector<ImageMessage>& {
    static const std::vector<ImageMessage> none;
    return t < (int)data.depths.size() ? data.depths[(size_t)t] : none;
  };
  auto attach_cloud = [&](CameraImage& cam) {
    const ImageMessage* m = nullptr;
    cam.cloud_timestamp = -1.0;
    if (lookup_image(cam.timestamp, depths_of(cam.camera_type), cloud_pos[(size_t)cam.camera_type],
                     cam.cloud_timestamp, &m)) {
      cam.cloud = m->cloud;
      cam.depth_name = m->name;
    }
  };
  if (!F.no_rig) {
    std::cout << "Looking up the images and bracketing the timestamps." << std::endl;
    const int nref = (int)data.ref_timestamps.size();
    for (int beg = 0; beg < nref; beg++) {
      int end = beg + 1;
      const bool last = (end == nref);
      if (last) end = beg;
      for (int t = 0; t < ncam; t++) {
        CameraImage cam;
        if (t == 0) {
          cam.camera_type = 0;
          cam.timestamp = data.ref_timestamps[(size_t)beg];
          cam.ref_timestamp = cam.timestamp;
          cam.beg_ref_index = cam.end_ref_index = beg;
          double found = -1;
          const ImageMessage* m = nullptr;
          if (!lookup_image(cam.timestamp, images_of(t), img_pos[(size_t)t], found, &m) || found != cam.timestamp)
            fatal("Cannot look up camera at time " + fixed17(cam.timestamp) + ".");
          cam.image_name = m->name;
        } else {
          const double off = rig.offsets[(size_t)t];
          const double beg_ts = data.ref_timestamps[(size_t)beg] + off;
          double end_ts = data.ref_timestamps[(size_t)end] + off;
          if (end_ts == beg_ts && last) end_ts = std::nextafter(end_ts, end_ts + 1.0);
          if (end_ts <= beg_ts) fatal("Ref timestamps must be in strictly increasing order.");
          const double mid = (beg_ts + end_ts) / 2.0;
          int start = img_pos[(size_t)t];
          double cur = beg_ts, best_dist = 1.0e+100, best_time = -1.0, found = -1.0;
          std::string best_name;
          while (true) {
            if (found > end_ts) break;
            const ImageMessage* m = nullptr;
            if (!lookup_image(cur, images_of(t), start, found, &m)) break;
            const bool in_bracket = (beg_ts <= found && found < end_ts);
            const double d = std::fabs(found - mid);
            if (d < best_dist && in_bracket) {
              best_dist = d;
              best_time = found;
              img_pos[(size_t)t] = start;
              best_name = m->name;
            }
            cur = std::nextafter(found, found + 1.0);
          }
          if (best_time < 0.0) continue;
          if (best_time > beg_ts && end_ts - beg_ts > F.bracket_len) continue;
          if (best_time < beg_ts || best_time >= end_ts) continue;
          cam.camera_type = t;
          cam.timestamp = best_time;
          cam.ref_timestamp = best_time - off;
          cam.beg_ref_index = beg;
          cam.end_ref_index = end;
          cam.image_name = best_name;
          min_off[(size_t)t] = std::max(min_off[(size_t)t], cam.timestamp - data.ref_timestamps[(size_t)end]);
          max_off[(size_t)t] = std::min(max_off[(size_t)t], cam.timestamp - data.ref_timestamps[(size_t)beg]);
        }
        attach_cloud(cam);
        cams.push_back(cam);
      }
    }
    std::cout << "Timestamp offset allowed ranges based on current bracketing:\n";
    for (int t = 1; t < ncam; t++) {
      min_off[(size_t)t] = std::max(min_off[(size_t)t], rig.offsets[(size_t)t] - F.timestamp_offsets_max_change);
      max_off[(size_t)t] = std::min(max_off[(size_t)t], rig.offsets[(size_t)t] + F.timestamp_offsets_max_change);
      min_off[(size_t)t] += 1.0e-5;
      max_off[(size_t)t] -= 1.0e-5;
      std::cout << std::setprecision(8) << names[(size_t)t] << ": [" << min_off[(size_t)t] << ", "
                << max_off[(size_t)t] << "]\n";
    }
  } else {
    std::cout << "Looking up the images." << std::endl;
    for (int t = 0; t < ncam; t++) {
      const auto& imgs = images_of(t);
      for (size_t k = 0; k < imgs.size(); k++) {
        CameraImage cam;
        cam.camera_type = t;
        cam.timestamp = imgs[k].timestamp;
        cam.ref_timestamp = cam.timestamp;
        cam.beg_ref_index = cam.end_ref_index = (int)k;
        double found = -1;
        const ImageMessage* m = nullptr;
        if (!lookup_image(cam.timestamp, imgs, img_pos[(size_t)t], found, &m) || found != cam.timestamp)
          fatal("Cannot look up camera at time " + fixed17(cam.timestamp) + ".");
        cam.image_name = m->name;
        attach_cloud(cam);
        cams.push_back(cam);
      }
    }
  }
  std::vector<int> count((size_t)ncam, 0);
  for (auto& c : cams) count[(size_t)c.camera_type]++;
  bool good = true;
  for (int t = 0; t < ncam; t++) {
    std::cout << "Number of images for sensor: " << names[(size_t)t] << ": " << count[(size_t)t] << std::endl;
    good = good && count[(size_t)t] > 0;
  }
  if (!good) fatal("Could not find images for all sensors. Cannot continue.");
  std::stable_sort(cams.begin(), cams.end(),
                   [](const CameraImage& a, const CameraImage& b) { return a.ref_timestamp < b.ref_timestamp; });
  return cams;
}

// calc_rig_using_word_to_cam (rig_calibrator.cc:1186-1266): per sensor, the
// entry-wise middle element (vals[size/2], unsorted, as the reference takes it)
// of ref_to_cam over its images, then linear /= det^(1/3).
static std::vector<Affine> rig_from_world_to_cam(int ncam, const std::vector<CameraImage>& cams,
                                                 const std::vector<double>& world_to_ref_vec,
                                                 const std::vector<double>& ref_timestamps,
                                                 const std::vector<double>& offsets,
                                                 const std::vector<Affine>& world_to_cam) {
  std::map<int, std::vector<Affine>> transforms;
  for (size_t k = 0; k < cams.size(); k++) {
    const auto& c = cams[k];
    if (c.camera_type == 0) {
      transforms[0].push_back(identity());
    } else {
      Affine interp = interp_world_to_ref(&world_to_ref_vec[7 * (size_t)c.beg_ref_index],
                                          &world_to_ref_vec[7 * (size_t)c.end_ref_index],
                                          ref_timestamps[(size_t)c.beg_ref_index],
                                          ref_timestamps[(size_t)c.end_ref_index], offsets[(size_t)c.camera_type],
                                          c.timestamp);
      transforms[c.camera_type].push_back(compose(world_to_cam[k], inverse(interp)));
    }
  }
  std::vector<Affine> out((size_t)ncam);
  for (auto& kv : transforms) {
    auto& v = kv.second;
    Affine m = v[v.size() / 2];  // every entry of the 4x4 is vals[size/2]
    const double s = std::pow(det3(m.R), 1.0 / 3.0);
    for (double& r : m.R) r /= s;
    out[(size_t)kv.first] = m;
  }
  return out;
}

// depthValue (dense_map_utils.cc:1364-1391)
static bool depth_value(const DepthCloud* c, double px, double py, double* xyz) {
  xyz[0] = xyz[1] = xyz[2] = 0;
  if (!c || (c->cols == 0 && c->rows == 0)) return false;
  const int col = (int)std::round(px), row = (int)std::round(py);
  if (col < 0 || row < 0 || col > c->cols || row > c->rows) fatal("Out of range in the depth cloud.");
  if (col == c->cols || row == c->rows) return false;
  const float* p = &c->xyz[3 * ((size_t)row * (size_t)c->cols + (size_t)col)];
  if (p[0] == 0 && p[1] == 0 && p[2] == 0) return false;
  for (int k = 0; k < 3; k++) xyz[k] = p[k];
  return true;
}

// ---------------------------------------------------------------- problem
// Parameter blocks keyed by the address of the caller-owned array, as Ceres
// keys them; only blocks some residual references exist (Problem semantics).
struct BlockSet {
  std::vector<int32_t> size;
  std::vector<int64_t> off;
  std::vector<uint8_t> cst;
  std::vector<double> x, lo, hi;
  std::vector<double*> owner;
  std::unordered_map<const double*, int32_t> ids;

  int32_t get(double* p, int n) {
    auto it = ids.find(p);
    if (it != ids.end()) return it->second;
    const int32_t id = (int32_t)size.size();
    ids.emplace(p, id);
    size.push_back(n);
    off.push_back((int64_t)x.size());
    cst.push_back(0);
    owner.push_back(p);
    for (int k = 0; k < n; k++) {
      x.push_back(p[k]);
      lo.push_back(-HUGE_VAL);
      hi.push_back(HUGE_VAL);
    }
    return id;
  }
  void copy_back(const double* packed) const {
    for (size_t b = 0; b < size.size(); b++)
      std::memcpy(owner[b], packed + off[b], sizeof(double) * (size_t)size[b]);
  }
};

// One residual block as main() adds it (:1614-1898), with owner pointers.
struct CamRes {
  double* blk[8];
  int bsize[8];
  int32_t id[8];  // camera-side block ids in the template block set (id[XYZ] unused)
  int cam_type;
  double meas[2];
  double stamps[3];
  int pid;
  int64_t feature;  // index into the track arrays
};
struct DepthRes {
  double* blk[7];
  int bsize[7];
  int32_t id[7];
  double meas[3];
  double stamps[3];
  int pid;
  double weight;
  bool mesh;           // BracketedDepthMeshError (no point block)
  double mesh_xyz[3];
};
struct XyzRes {
  int pid;
  double ref[3];
  double weight, threshold;
  uint8_t kind;  // 0 tri, 1 mesh_tri
};

struct Plan {
  std::vector<CamRes> cam;
  std::vector<DepthRes> depth;
  std::vector<XyzRes> xyz;
  std::unordered_set<const double*> constant;
  std::map<const double*, std::pair<double, double>> bounds;
};

// A shard: the camera-side blocks of the whole problem (same ids on every
// shard) plus the points of a landmark range.
struct Shard {
  int device = 0;
  int index = 0;  // position in the landmark split (shard_of)
  BlockSet blocks;
  std::vector<int32_t> res_blocks, res_cam, dep_blocks, xyz_block;
  std::vector<double> res_meas, res_stamps, dep_meas, dep_weight, dep_stamps, xyz_ref, xyz_weight, xyz_thr;
  std::vector<double> dep_mesh;     // [3 per depth block] mesh point (BracketedDepthMeshError rows)
  std::vector<uint8_t> dep_is_mesh, xyz_kind;
  bool any_mesh = false;
  std::vector<int32_t> cam_dist_size;
  std::vector<double> cam_half;
  std::vector<int64_t> res_feature;  // residual -> feature
  mvba_handle* h = nullptr;
  mvba_solver_summary summary{};
  mvba_status status = MVBA_OK;
  std::string error;
};

static std::string handle_error(mvba_handle* h, mvba_status st) {
  const char* m = h ? mvba_last_error(h) : mvba_create_error();
  std::ostringstream os;
  os << "libmvba status " << (int)st << ": " << (m && *m ? m : "(no message)");
  return os.str();
}

static void check(mvba_handle* h, mvba_status st) {
  if (st != MVBA_OK) fatal(handle_error(h, st));
}

using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

// calc_residuals_stats (rig_calibrator.cc:753-789) output for rows sorted by name.
struct StatRow {
  std::string name;
  double v[4];
  int64_t n;
};
static void print_stats(std::vector<StatRow> rows, const std::string& tag) {
  std::sort(rows.begin(), rows.end(), [](const StatRow& a, const StatRow& b) { return a.name < b.name; });
  std::cout << "The 25, 50, 75, and 100th percentile residual stats " << tag << std::endl;
  for (auto& r : rows) {
    if (r.n == 0)
      std::cout << r.name << ": none";
    else
      std::cout << std::setprecision(5) << r.name << ": " << r.v[0] << ' ' << r.v[1] << ' ' << r.v[2] << ' ' << r.v[3];
    std::cout << " (" << r.n << " residuals)" << std::endl;
  }
}

static std::vector<std::string> group_labels(const std::vector<std::string>& names) {
  std::vector<std::string> labels;
  for (const auto& n : names) {
    labels.push_back(n + "_pix_x");
    labels.push_back(n + "_pix_y");
  }
  // mvba_residual_stats groups: depth_tri, tri, depth_mesh, mesh_tri
  for (const char* kind : {"depth_tri_", "tri_", "depth_mesh_", "mesh_tri_"})
    for (const char* a : {"x", "y", "z"}) labels.push_back(std::string(kind) + a + "_m");
  return labels;
}

// evalResiduals "before/after opt": on the GPU per shard (mvba_residual_stats)
// when there is one shard; with several shards the raw residuals are gathered
// and the percentiles picked on the host (percentiles do not merge).
static void residual_stats(std::vector<Shard>& shards, const std::vector<std::string>& names,
                           const std::string& tag) {
  const size_t ng = 2 * names.size() + 12;
  const auto labels = group_labels(names);
  std::vector<StatRow> rows;
  if (shards.size() == 1) {
    std::vector<double> out(4 * ng);
    std::vector<int64_t> cnt(ng);
    check(shards[0].h, mvba_residual_stats(shards[0].h, out.data(), cnt.data(), nullptr));
    for (size_t g = 0; g < ng; g++)
      if (cnt[g] > 0) rows.push_back({labels[g], {out[4 * g], out[4 * g + 1], out[4 * g + 2], out[4 * g + 3]}, cnt[g]});
  } else {
    std::vector<std::vector<double>> vals(ng);
    for (auto& s : shards) {
      const int64_t nr = mvba_num_residuals(s.h), nd = mvba_num_depth_residuals(s.h),
                    nx = mvba_num_xyz_residuals(s.h);
      std::vector<double> r(2 * (size_t)nr), rd(3 * (size_t)nd), rx(3 * (size_t)nx);
      check(s.h, mvba_evaluate(s.h, MVBA_EVAL_RESIDUALS, 0.0, nullptr, r.data(), nullptr));
      if (nd) check(s.h, mvba_evaluate_depth(s.h, MVBA_EVAL_RESIDUALS, 0.0, nullptr, rd.data(), nullptr));
      if (nx) check(s.h, mvba_evaluate_xyz(s.h, MVBA_EVAL_RESIDUALS, nullptr, rx.data(), nullptr));
      for (int64_t i = 0; i < nr; i++)
        for (int k = 0; k < 2; k++) vals[2 * (size_t)s.res_cam[(size_t)i] + (size_t)k].push_back(std::fabs(r[2 * (size_t)i + (size_t)k]));
      for (int64_t i = 0; i < nd; i++)
        for (int k = 0; k < 3; k++)
          vals[2 * names.size() + (s.dep_is_mesh[(size_t)i] ? 6 : 0) + (size_t)k].push_back(
              std::fabs(rd[3 * (size_t)i + (size_t)k] / s.dep_weight[(size_t)i]));
      for (int64_t i = 0; i < nx; i++)
        for (int k = 0; k < 3; k++)
          vals[2 * names.size() + (s.xyz_kind[(size_t)i] ? 9 : 3) + (size_t)k].push_back(
              std::fabs(rx[3 * (size_t)i + (size_t)k] / s.xyz_weight[(size_t)i]));
    }
    for (size_t g = 0; g < ng; g++) {
      auto& v = vals[g];
      if (v.empty()) continue;
      std::sort(v.begin(), v.end());
      const size_t L = v.size();
      rows.push_back({labels[g], {v[(size_t)(0.25 * (double)L)], v[(size_t)(0.5 * (double)L)], v[(size_t)(0.75 * (double)L)], v[L - 1]},
                      (int64_t)L});
    }
  }
  print_stats(rows, tag);
}

// ---------------------------------------------------------------- main
static int run(int argc, char** argv) {
  Flags F;
  parse_flags(argc, argv, F);
  parameter_validation(F);
  int device0 = 0;
  if (F.device.size() > 4 && F.device[3] == ':') device0 = std::atoi(F.device.c_str() + 4);

  const int ref_cam_type = 0;
  bool use_initial_rig_transforms = F.use_initial_rig_transforms;
  RigConfig rig = read_rig_config(F.rig_config, use_initial_rig_transforms);
  const std::vector<std::string>& cam_names = rig.cam_names;
  const int ncam = (int)rig.params.size();
  if (ncam == 0) fatal("No sensors found in: " + F.rig_config);

  // images and poses
  NvmData nvm;
  std::vector<std::string> files;
  std::vector<Affine> file_w2c;
  if (F.camera_poses != "") {
    read_camera_poses_file(F.camera_poses, files, file_w2c);
  } else {
    nvm = read_nvm(F.nvm);
    files = nvm.cid_to_filename;
    file_w2c = nvm.cid_to_cam_t_global;
  }
  ImageData data = read_image_entries(files, file_w2c, cam_names, ref_cam_type);
  std::vector<double> min_off, max_off;
  std::vector<CameraImage> cams = lookup_images(F, cam_names, rig, data, min_off, max_off);
  const size_t ncams = cams.size();
  const std::vector<double>& ref_timestamps = data.ref_timestamps;
  const int num_ref = (int)data.world_to_ref.size();

  std::vector<double> world_to_ref_vec(7 * (size_t)num_ref);
  for (int c = 0; c < num_ref; c++) rigid_to_array(data.world_to_ref[(size_t)c], &world_to_ref_vec[7 * (size_t)c]);

  std::vector<Affine> world_to_cam(ncams);
  std::vector<Affine> ref_to_cam_trans = rig.ref_to_cam;
  if (use_initial_rig_transforms && !F.no_rig) {
    std::vector<double> r2c(7 * (size_t)ncam);
    for (int t = 0; t < ncam; t++) rigid_to_array(ref_to_cam_trans[(size_t)t], &r2c[7 * (size_t)t]);
    for (size_t k = 0; k < ncams; k++) {
      const auto& c = cams[k];
      world_to_cam[k] = world_to_cam_trans(
          &world_to_ref_vec[7 * (size_t)c.beg_ref_index], &world_to_ref_vec[7 * (size_t)c.end_ref_index],
          &r2c[7 * (size_t)c.camera_type], ref_timestamps[(size_t)c.beg_ref_index],
          ref_timestamps[(size_t)c.end_ref_index], rig.offsets[(size_t)c.camera_type], c.timestamp);
    }
  } else {
    std::vector<size_t> start((size_t)ncam, 0);
    for (size_t k = 0; k < ncams; k++) {
      const int t = cams[k].camera_type;
      const auto& imgs = data.images[(size_t)t];
      for (size_t p = start[(size_t)t]; p < imgs.size(); p++)
        if (cams[k].timestamp == imgs[p].timestamp) {
          world_to_cam[k] = imgs[p].world_to_cam;
          start[(size_t)t] = p;
        }
    }
    ref_to_cam_trans = rig_from_world_to_cam(ncam, cams, world_to_ref_vec, ref_timestamps, rig.offsets, world_to_cam);
  }

  // optimisation state (the reference's *_vec arrays, :1401-1492)
  std::vector<double> ref_to_cam_vec(7 * (size_t)ncam);
  for (int t = 0; t < ncam; t++) rigid_to_array(ref_to_cam_trans[(size_t)t], &ref_to_cam_vec[7 * (size_t)t]);
  std::vector<double> identity_vec(7);
  rigid_to_array(identity(), identity_vec.data());
  auto intrinsics_to_float = parse_intrinsics_to_float(F.intrinsics_to_float, cam_names);
  auto rig_transforms_to_float = parse_camera_names(cam_names, F.rig_transforms_to_float);
  for (const auto& n : rig_transforms_to_float)
    if (n == cam_names[0]) fatal("Cannot float the rig transform from reference camera to itself.");
  auto camera_poses_to_float = parse_camera_names(cam_names, F.camera_poses_to_float);
  auto dti_to_float = parse_camera_names(cam_names, F.depth_to_image_transforms_to_float);
  const int num_depth_params = F.affine_depth_to_image ? 12 : 7;
  std::vector<double> depth_scales((size_t)ncam);
  std::vector<Affine> depth_to_image = rig.depth_to_image;
  for (int t = 0; t < ncam; t++) {
    const double s = std::pow(det3(depth_to_image[(size_t)t].R), 1.0 / 3.0);
    for (double& r : depth_to_image[(size_t)t].R) r /= s;
    depth_scales[(size_t)t] = s;
  }
  std::vector<double> depth_to_image_vec((size_t)ncam * (size_t)num_depth_params);
  for (int t = 0; t < ncam; t++) {
    if (F.affine_depth_to_image)
      affine_to_array(depth_to_image[(size_t)t], &depth_to_image_vec[(size_t)num_depth_params * (size_t)t]);
    else
      rigid_to_array(depth_to_image[(size_t)t], &depth_to_image_vec[(size_t)num_depth_params * (size_t)t]);
  }
  std::vector<double> focal((size_t)ncam);
  std::vector<std::array<double, 2>> center((size_t)ncam);
  std::vector<std::vector<double>> dist((size_t)ncam);
  for (int t = 0; t < ncam; t++) {
    focal[(size_t)t] = rig.params[(size_t)t].focal;
    center[(size_t)t] = {rig.params[(size_t)t].center[0], rig.params[(size_t)t].center[1]};
    dist[(size_t)t] = rig.params[(size_t)t].dist;
  }
  std::vector<double> offsets = rig.offsets;
  std::vector<double> world_to_cam_vec;
  if (F.no_rig) {
    world_to_cam_vec.resize(7 * ncams);
    for (size_t c = 0; c < ncams; c++) rigid_to_array(world_to_cam[c], &world_to_cam_vec[7 * c]);
  }

  // matches (appendMatchesFromNvm, interest_point.cc:1788-1845)
  std::vector<std::vector<std::pair<float, float>>> keypoint_vec(ncams);
  std::vector<std::map<int, int>> pid_to_cid_fid;
  if (!F.no_nvm_matches && F.nvm != "") {
    std::map<std::string, int> name_to_nvm;
    for (size_t c = 0; c < nvm.cid_to_filename.size(); c++) name_to_nvm[nvm.cid_to_filename[c]] = (int)c;
    std::map<int, int> nvm_to_cams;
    for (size_t c = 0; c < ncams; c++) {
      auto it = name_to_nvm.find(cams[c].image_name);
      if (it == name_to_nvm.end())
        fatal("Could not look up image: " + cams[c].image_name + " in the input nvm file.");
      nvm_to_cams[it->second] = (int)c;
    }
    for (size_t pid = 0; pid < nvm.pid_to_cid_fid.size(); pid++) {
      std::map<int, int> out;
      for (const auto& cf : nvm.pid_to_cid_fid[pid]) {
        auto it = nvm_to_cams.find(cf.first);
        if (it == nvm_to_cams.end()) continue;
        const int cid = it->second;
        const auto& kp = nvm.cid_to_keypoint[(size_t)cf.first][(size_t)cf.second];
        const auto& ctr = center[(size_t)cams[(size_t)cid].camera_type];
        const double x = kp[0] + ctr[0], y = kp[1] + ctr[1];
        out[cid] = (int)keypoint_vec[(size_t)cid].size();
        keypoint_vec[(size_t)cid].push_back({(float)x, (float)y});
      }
      if (out.size() > 1) pid_to_cid_fid.push_back(out);
    }
  }
  if (pid_to_cid_fid.empty()) fatal("No interest points were found. Must specify either --nvm or positive --num_overlaps.");

  // tracks in CSR (features of a track in increasing image order, as std::map iterates)
  const int npid = (int)pid_to_cid_fid.size();
  std::vector<int64_t> track_begin((size_t)npid + 1, 0);
  std::vector<int32_t> track_image, track_fid;
  std::vector<double> track_pix;
  for (int p = 0; p < npid; p++) {
    for (const auto& cf : pid_to_cid_fid[(size_t)p]) {
      track_image.push_back(cf.first);
      track_fid.push_back(cf.second);
      const auto& kp = keypoint_vec[(size_t)cf.first][(size_t)cf.second];
      track_pix.push_back(kp.first);
      track_pix.push_back(kp.second);
    }
    track_begin[(size_t)p + 1] = (int64_t)track_image.size();
  }
  const int64_t nobs = (int64_t)track_image.size();
  // flagOutlierByExclusionDist (rig_calibrator.cc:1003-1039)
  std::vector<uint8_t> inlier((size_t)nobs, 1);
  for (int64_t o = 0; o < nobs; o++) {
    const auto& cp = rig.params[(size_t)cams[(size_t)track_image[(size_t)o]].camera_type];
    if (std::fabs(track_pix[2 * (size_t)o] - cp.image_size[0] / 2.0) > cp.crop_size[0] / 2.0 ||
        std::fabs(track_pix[2 * (size_t)o + 1] - cp.image_size[1] / 2.0) > cp.crop_size[1] / 2.0)
      inlier[(size_t)o] = 0;
  }
  std::vector<double> xyz_vec(3 * (size_t)npid, 0.0);
  std::vector<int32_t> image_camera(ncams);
  for (size_t c = 0; c < ncams; c++) image_camera[c] = cams[c].camera_type;

  auto update_world_to_cam = [&]() {  // calc_world_to_cam_rig_or_not (:871-890)
    for (size_t k = 0; k < ncams; k++) {
      const auto& c = cams[k];
      if (F.no_rig) {
        world_to_cam[k] = array_to_rigid(&world_to_cam_vec[7 * k]);
      } else {
        world_to_cam[k] = world_to_cam_trans(
            &world_to_ref_vec[7 * (size_t)c.beg_ref_index], &world_to_ref_vec[7 * (size_t)c.end_ref_index],
            &ref_to_cam_vec[7 * (size_t)c.camera_type], ref_timestamps[(size_t)c.beg_ref_index],
            ref_timestamps[(size_t)c.end_ref_index], offsets[(size_t)c.camera_type], c.timestamp);
      }
    }
  };
  // tracks descriptor at the current cameras and intrinsics
  std::vector<double> td_w2c, td_center, td_dist, td_dhalf, td_uhalf;
  std::vector<int32_t> td_dsize;
  std::vector<int64_t> td_doff;
  auto tracks_desc = [&]() {
    mvba_tracks_desc d{};
    td_w2c.resize(12 * ncams);
    for (size_t k = 0; k < ncams; k++) {
      std::memcpy(&td_w2c[12 * k], world_to_cam[k].R, 9 * sizeof(double));
      std::memcpy(&td_w2c[12 * k + 9], world_to_cam[k].t, 3 * sizeof(double));
    }
    td_center.clear();
    td_dist.clear();
    td_dhalf.clear();
    td_uhalf.clear();
    td_dsize.clear();
    td_doff.clear();
    for (int t = 0; t < ncam; t++) {
      td_center.push_back(center[(size_t)t][0]);
      td_center.push_back(center[(size_t)t][1]);
      td_doff.push_back((int64_t)td_dist.size());
      td_dsize.push_back((int32_t)dist[(size_t)t].size());
      td_dist.insert(td_dist.end(), dist[(size_t)t].begin(), dist[(size_t)t].end());
      const auto& p = rig.params[(size_t)t];
      td_dhalf.push_back(p.image_size[0] / 2.0);
      td_dhalf.push_back(p.image_size[1] / 2.0);
      td_uhalf.push_back(p.undist_size[0] / 2.0);
      td_uhalf.push_back(p.undist_size[1] / 2.0);
    }
    if (td_dist.empty()) td_dist.push_back(0.0);
    d.num_images = (int32_t)ncams;
    d.world_to_cam = td_w2c.data();
    d.image_camera = image_camera.data();
    d.num_cameras = ncam;
    d.focal = focal.data();
    d.center = td_center.data();
    d.dist_size = td_dsize.data();
    d.dist_offset = td_doff.data();
    d.dist = td_dist.data();
    d.dist_half = td_dhalf.data();
    d.undist_half = td_uhalf.data();
    d.num_points = npid;
    d.track_begin = track_begin.data();
    d.track_image = track_image.data();
    d.track_pix = track_pix.data();
    return d;
  };

  const int ngpu = F.num_gpus;
  // --mesh: loadMeshBuildTree (texture_processing.cc:264-285): the PLY file is
  // read (host) before the device check, the BVH is built on the GPU below
  std::vector<float> mv;
  std::vector<uint32_t> mf;
  if (F.mesh != "" && F.calibrator_num_passes > 0) {
    std::cout << "Loading mesh: " << F.mesh << std::endl;
    std::string err;
    if (!read_ply_mesh(F.mesh, mv, mf, err)) fatal(err);
    std::cout << "Number of faces: " << mf.size() / 3 << " faces.\n";
  }
  int32_t ndev = 0;
  if (F.calibrator_num_passes > 0 && (mvba_device_count(&ndev) != MVBA_OK || ndev < 1))
    fatal("No HIP device is available (this build has no CPU compute path).");
  double placeholder = 0.0;  // distortion_placeholder (:1608)
  mvba_mesh* mesh = nullptr;
  std::vector<double> mesh_feat_xyz, mesh_pt_xyz;
  if (F.mesh != "" && F.calibrator_num_passes > 0) {
    const auto tb = Clock::now();
    mvba_mesh_desc md{};
    md.num_vertices = (int64_t)(mv.size() / 3);
    md.vertices = mv.data();
    md.num_faces = (int64_t)(mf.size() / 3);
    md.faces = mf.data();
    if (mvba_mesh_create(&md, device0, &mesh) != MVBA_OK) fatal(std::string("mesh: ") + mvba_mesh_error());
    std::cout << "Building the tree took: " << secs(tb) << " seconds\n";
    mesh_feat_xyz.assign(3 * (size_t)nobs, kBadXyz);
    mesh_pt_xyz.assign(3 * (size_t)npid, kBadXyz);
  }
  double t_tri = 0, t_build = 0, t_create = 0, t_stats = 0, t_solve = 0, t_flag = 0;
  std::vector<double> residuals_after;  // per feature, [2*nobs]
  for (int pass = 0; pass < F.calibrator_num_passes; pass++) {
    std::cout << "\nOptimization pass " << pass + 1 << " / " << F.calibrator_num_passes << "\n";
    update_world_to_cam();
    auto t0 = Clock::now();
    {
      mvba_tracks_desc d = tracks_desc();
      if (mvba_triangulate(&d, device0, inlier.data(), xyz_vec.data()) != MVBA_OK)
        fatal(std::string("triangulation: ") + mvba_tracks_error());
    }
    // where each inlier ray meets the mesh (meshTriangulations, :1581-1588)
    if (mesh) {
      mvba_tracks_desc d = tracks_desc();
      if (mvba_mesh_triangulate(&d, mesh, inlier.data(), F.min_ray_dist, F.max_ray_dist, mesh_feat_xyz.data(),
                                mesh_pt_xyz.data()) != MVBA_OK)
        fatal(std::string("mesh intersection: ") + mvba_tracks_error() + mvba_mesh_error());
    }
    t_tri += secs(t0);
    t0 = Clock::now();
    std::vector<double> xyz_orig = xyz_vec;

    // residual blocks (:1614-1898)
    Plan plan;
    for (int pid = 0; pid < npid; pid++) {
      bool tri_inlier = false;
      for (int64_t o = track_begin[(size_t)pid]; o < track_begin[(size_t)pid + 1]; o++) {
        if (!inlier[(size_t)o]) continue;
        tri_inlier = true;
        const int cid = track_image[(size_t)o];
        const CameraImage& cam = cams[(size_t)cid];
        const int t = cam.camera_type;
        CamRes r{};
        double *beg, *end;
        if (!F.no_rig) {
          beg = &world_to_ref_vec[7 * (size_t)cam.beg_ref_index];
          end = (t == ref_cam_type || cam.beg_ref_index == cam.end_ref_index)
                    ? identity_vec.data()
                    : &world_to_ref_vec[7 * (size_t)cam.end_ref_index];
          r.stamps[0] = ref_timestamps[(size_t)cam.beg_ref_index];
          r.stamps[1] = ref_timestamps[(size_t)cam.end_ref_index];
        } else {
          beg = &world_to_cam_vec[7 * (size_t)cid];
          end = identity_vec.data();
          r.stamps[0] = r.stamps[1] = cam.timestamp;
        }
        r.stamps[2] = cam.timestamp;
        double* r2c = &ref_to_cam_vec[7 * (size_t)t];
        double* distp = dist[(size_t)t].empty() ? &placeholder : dist[(size_t)t].data();
        double* blk[8] = {beg, end, r2c, &xyz_vec[3 * (size_t)pid], &offsets[(size_t)t], &focal[(size_t)t],
                          center[(size_t)t].data(), distp};
        const int bs[8] = {7, 7, 7, 3, 1, 1, 2, dist[(size_t)t].empty() ? 1 : (int)dist[(size_t)t].size()};
        std::memcpy(r.blk, blk, sizeof(blk));
        std::memcpy(r.bsize, bs, sizeof(bs));
        r.cam_type = t;
        r.meas[0] = track_pix[2 * (size_t)o];
        r.meas[1] = track_pix[2 * (size_t)o + 1];
        r.pid = pid;
        r.feature = o;
        plan.cam.push_back(r);
        const auto& itf = intrinsics_to_float[(size_t)t];
        if (!itf.count("focal_length")) plan.constant.insert(&focal[(size_t)t]);
        if (!itf.count("optical_center")) plan.constant.insert(center[(size_t)t].data());
        if (!itf.count("distortion") || dist[(size_t)t].empty()) plan.constant.insert(distp);
        if (!F.no_rig) {
          if (!camera_poses_to_float.count(cam_names[0])) plan.constant.insert(beg);
        } else if (!camera_poses_to_float.count(cam_names[(size_t)t])) {
          plan.constant.insert(beg);
        }
        if (!camera_poses_to_float.count(cam_names[0]) || t == ref_cam_type || F.no_rig) plan.constant.insert(end);
        if (!F.float_timestamp_offsets || t == ref_cam_type || F.no_rig)
          plan.constant.insert(&offsets[(size_t)t]);
        else
          plan.bounds[&offsets[(size_t)t]] = {min_off[(size_t)t], max_off[(size_t)t]};
        if (!rig_transforms_to_float.count(cam_names[(size_t)t]) || t == ref_cam_type || F.no_rig)
          plan.constant.insert(r2c);
        double dxyz[3];
        if (F.depth_tri_weight > 0 && depth_value(cam.cloud.get(), r.meas[0], r.meas[1], dxyz)) {
          DepthRes dr{};
          double* dti = &depth_to_image_vec[(size_t)num_depth_params * (size_t)t];
          double* dblk[7] = {beg, end, r2c, dti, &depth_scales[(size_t)t], &xyz_vec[3 * (size_t)pid],
                             &offsets[(size_t)t]};
          const int dbs[7] = {7, 7, 7, num_depth_params, 1, 3, 1};
          std::memcpy(dr.blk, dblk, sizeof(dblk));
          std::memcpy(dr.bsize, dbs, sizeof(dbs));
          std::memcpy(dr.meas, dxyz, sizeof(dxyz));
          std::memcpy(dr.stamps, r.stamps, sizeof(dr.stamps));
          dr.pid = pid;
          dr.weight = F.depth_tri_weight;
          plan.depth.push_back(dr);
          if (!F.float_scale || F.affine_depth_to_image) plan.constant.insert(&depth_scales[(size_t)t]);
          if (!dti_to_float.count(cam_names[(size_t)t])) plan.constant.insert(dti);
        }
        // depth-to-mesh constraint (:1796-1834): the feature's mesh hit vs its depth point
        if (mesh && F.depth_mesh_weight > 0 && mesh_feat_xyz[3 * (size_t)o] != kBadXyz &&
            depth_value(cam.cloud.get(), r.meas[0], r.meas[1], dxyz)) {
          DepthRes dr{};
          double* dti = &depth_to_image_vec[(size_t)num_depth_params * (size_t)t];
          double* dblk[7] = {beg, end, r2c, dti, &depth_scales[(size_t)t], nullptr, &offsets[(size_t)t]};
          const int dbs[7] = {7, 7, 7, num_depth_params, 1, 0, 1};
          std::memcpy(dr.blk, dblk, sizeof(dblk));
          std::memcpy(dr.bsize, dbs, sizeof(dbs));
          std::memcpy(dr.meas, dxyz, sizeof(dxyz));
          std::memcpy(dr.stamps, r.stamps, sizeof(dr.stamps));
          std::memcpy(dr.mesh_xyz, &mesh_feat_xyz[3 * (size_t)o], sizeof(dr.mesh_xyz));
          dr.pid = pid;
          dr.weight = F.depth_mesh_weight;
          dr.mesh = true;
          plan.depth.push_back(dr);
          if (!F.float_scale || F.affine_depth_to_image) plan.constant.insert(&depth_scales[(size_t)t]);
          if (!dti_to_float.count(cam_names[(size_t)t])) plan.constant.insert(dti);
        }
      }
      // mesh-to-triangulated-point constraint (:1857-1877), then --tri_weight (:1880-1898)
      if (mesh && tri_inlier && F.mesh_tri_weight > 0 && mesh_pt_xyz[3 * (size_t)pid] != kBadXyz) {
        XyzRes x{};
        x.pid = pid;
        std::memcpy(x.ref, &mesh_pt_xyz[3 * (size_t)pid], sizeof(x.ref));
        x.weight = F.mesh_tri_weight;
        x.threshold = F.robust_threshold;
        x.kind = 1;
        plan.xyz.push_back(x);
      }
      if (F.tri_weight > 0.0 && tri_inlier) {
        XyzRes x{};
        x.pid = pid;
        std::memcpy(x.ref, &xyz_orig[3 * (size_t)pid], sizeof(x.ref));
        x.weight = F.tri_weight;
        x.threshold = F.tri_robust_threshold;
        x.kind = 0;
        plan.xyz.push_back(x);
      }
    }
    if (plan.cam.empty()) fatal("No inlier observations are left to optimize.");

    // shards: contiguous landmark ranges of capture order (the timestamp of a
    // landmark's first observing image, then its id), balanced by residual
    // count: each shard then holds the images of one stretch of the trajectory
    // (plus the tracks' reach) instead of observations in every image, so its
    // per-image work shrinks with the split too (bench.py splits the same way,
    // rig.shard_points)
    std::vector<Shard> shards((size_t)ngpu);
    std::vector<int> shard_of((size_t)npid, 0);
    if (ngpu > 1) {
      std::vector<double> first((size_t)npid, std::numeric_limits<double>::infinity());
      std::vector<int64_t> per_pid((size_t)npid, 0);
      for (const auto& r : plan.cam) {
        first[(size_t)r.pid] = std::min(first[(size_t)r.pid], r.stamps[2]);
        per_pid[(size_t)r.pid]++;
      }
      std::vector<int> ord((size_t)npid);
      for (int p = 0; p < npid; p++) ord[(size_t)p] = p;
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return first[(size_t)a] < first[(size_t)b]; });
      const int64_t tot = std::max<int64_t>((int64_t)plan.cam.size(), 1);
      int64_t acc = 0;
      for (int p : ord) {
        shard_of[(size_t)p] = (int)std::min<int64_t>(ngpu - 1, acc * ngpu / tot);
        acc += per_pid[(size_t)p];
      }
    }
    for (int s = 0; s < ngpu; s++) {
      shards[(size_t)s].index = s;
      shards[(size_t)s].device = (device0 + s) % ndev;  // shards share GPUs when there are fewer
    }
    // camera-side blocks first, in the order the whole problem references them,
    // so every shard has the same camera layout; constancy and bounds are
    // properties of the block
    BlockSet tmpl;
    tmpl.ids.reserve(4096);
    for (auto& r : plan.cam)
      for (int b = 0; b < 8; b++)
        if (b != MVBA_BLK_XYZ) r.id[b] = tmpl.get(r.blk[b], r.bsize[b]);
    for (auto& r : plan.depth)
      for (int b = 0; b < 7; b++)
        if (b != MVBA_DBLK_XYZ) r.id[b] = tmpl.get(r.blk[b], r.bsize[b]);
    for (const double* p : plan.constant) {
      auto it = tmpl.ids.find(p);
      if (it != tmpl.ids.end()) tmpl.cst[(size_t)it->second] = 1;
    }
    for (const auto& kv : plan.bounds) {
      auto it = tmpl.ids.find(kv.first);
      if (it == tmpl.ids.end()) continue;
      tmpl.lo[(size_t)tmpl.off[(size_t)it->second]] = kv.second.first;
      tmpl.hi[(size_t)tmpl.off[(size_t)it->second]] = kv.second.second;
    }
    std::vector<int32_t> point_id((size_t)npid);
    for (auto& S : shards) {
      S.blocks = tmpl;
      BlockSet& B = S.blocks;
      std::fill(point_id.begin(), point_id.end(), -1);
      auto point = [&](int pid) {  // point blocks: first use, never constant
        int32_t& id = point_id[(size_t)pid];
        if (id < 0) id = B.get(&xyz_vec[3 * (size_t)pid], 3);
        return id;
      };
      const size_t nres_hint = plan.cam.size() / shards.size() + 16;
      S.res_blocks.reserve(8 * nres_hint);
      S.res_meas.reserve(2 * nres_hint);
      S.res_stamps.reserve(3 * nres_hint);
      for (const auto& r : plan.cam) {
        if (shard_of[(size_t)r.pid] != S.index) continue;
        for (int b = 0; b < 8; b++) S.res_blocks.push_back(b == MVBA_BLK_XYZ ? point(r.pid) : r.id[b]);
        S.res_cam.push_back(r.cam_type);
        S.res_meas.insert(S.res_meas.end(), r.meas, r.meas + 2);
        S.res_stamps.insert(S.res_stamps.end(), r.stamps, r.stamps + 3);
        S.res_feature.push_back(r.feature);
      }
      for (const auto& r : plan.depth) {
        if (shard_of[(size_t)r.pid] != S.index) continue;
        for (int b = 0; b < 7; b++)
          S.dep_blocks.push_back(b == MVBA_DBLK_XYZ ? (r.mesh ? -1 : point(r.pid)) : r.id[b]);
        S.dep_meas.insert(S.dep_meas.end(), r.meas, r.meas + 3);
        S.dep_weight.push_back(r.weight);
        S.dep_stamps.insert(S.dep_stamps.end(), r.stamps, r.stamps + 3);
        S.dep_mesh.insert(S.dep_mesh.end(), r.mesh_xyz, r.mesh_xyz + 3);
        S.dep_is_mesh.push_back(r.mesh ? 1 : 0);
        S.any_mesh = S.any_mesh || r.mesh;
      }
      for (const auto& r : plan.xyz) {
        if (shard_of[(size_t)r.pid] != S.index) continue;
        S.xyz_block.push_back(point(r.pid));
        S.xyz_ref.insert(S.xyz_ref.end(), r.ref, r.ref + 3);
        S.xyz_weight.push_back(r.weight);
        S.xyz_thr.push_back(r.threshold);
        S.xyz_kind.push_back(r.kind);
      }
      for (int t = 0; t < ncam; t++) {
        S.cam_dist_size.push_back((int32_t)dist[(size_t)t].size());
        S.cam_half.push_back(rig.params[(size_t)t].image_size[0] / 2.0);
        S.cam_half.push_back(rig.params[(size_t)t].image_size[1] / 2.0);
      }
      mvba_problem_desc d{};
      d.num_blocks = (int32_t)B.size.size();
      d.block_size = B.size.data();
      d.block_offset = B.off.data();
      d.block_constant = B.cst.data();
      d.num_param_doubles = (int64_t)B.x.size();
      d.num_cameras = ncam;
      d.camera_dist_size = S.cam_dist_size.data();
      d.camera_half_size = S.cam_half.data();
      d.num_residuals = (int64_t)S.res_cam.size();
      d.residual_blocks = S.res_blocks.data();
      d.residual_camera = S.res_cam.data();
      d.residual_meas = S.res_meas.data();
      d.residual_stamps = S.res_stamps.data();
      d.num_depth_residuals = (int64_t)S.dep_weight.size();
      d.depth_blocks = S.dep_blocks.data();
      d.depth_meas = S.dep_meas.data();
      d.depth_weight = S.dep_weight.data();
      d.depth_stamps = S.dep_stamps.data();
      d.num_xyz_residuals = (int64_t)S.xyz_weight.size();
      d.xyz_block = S.xyz_block.data();
      d.xyz_ref = S.xyz_ref.data();
      d.xyz_weight = S.xyz_weight.data();
      d.xyz_threshold = S.xyz_thr.data();
      d.depth_mesh_xyz = S.any_mesh ? S.dep_mesh.data() : nullptr;
      d.xyz_kind = S.xyz_kind.data();
      mvba_options o{};
      o.device = S.device;
      const auto tc = Clock::now();
      check(nullptr, mvba_create(&d, &o, &S.h));
      check(S.h, mvba_set_params(S.h, B.x.data()));
      t_create += secs(tc);
    }
    t_build += secs(t0);
    t0 = Clock::now();
    residual_stats(shards, cam_names, "before opt");
    t_stats += secs(t0);

    // Solve (:1910-1919)
    t0 = Clock::now();
    // --num_gpus > 1: one solver thread and HIP stream per shard; the exchange
    // steps are stream-ordered device all-reduces over a local communicator
    // (mvba_comm_init_local: shards may share a device)
    std::vector<mvba_comm*> comms((size_t)ngpu, nullptr);
    std::vector<hipStream_t> streams((size_t)ngpu, nullptr);
    if (ngpu > 1) {
      std::vector<int32_t> devs((size_t)ngpu);
      for (int s = 0; s < ngpu; s++) devs[(size_t)s] = shards[(size_t)s].device;
      if (mvba_comm_init_local(ngpu, devs.data(), comms.data()) != MVBA_OK)
        fatal(std::string("mvba_comm_init_local: ") + mvba_comm_error());
      for (int s = 0; s < ngpu; s++) {
        if (hipSetDevice(devs[(size_t)s]) != hipSuccess ||
            hipStreamCreateWithFlags(&streams[(size_t)s], hipStreamNonBlocking) != hipSuccess)
          fatal("hipStreamCreate failed");
      }
    }
    auto solve_one = [&](int s) {
      Shard& S = shards[(size_t)s];
      mvba_solver_options o;
      mvba_solver_default_options(&o);
      o.max_num_iterations = F.num_iterations;
      o.gradient_tolerance = 1e-16;
      o.function_tolerance = 1e-16;
      o.parameter_tolerance = F.parameter_tolerance;
      o.use_loss = 1;
      o.robust_threshold = F.robust_threshold;
      o.lower_bounds = S.blocks.lo.data();
      o.upper_bounds = S.blocks.hi.data();
      o.progress_to_stdout = s == 0 ? 1 : 0;
      if (ngpu > 1) {
        o.allreduce = mvba_comm_allreduce;
        o.allreduce_user = comms[(size_t)s];
      }
      S.status = mvba_solve(S.h, &o, &S.summary, streams[(size_t)s]);
      if (S.status != MVBA_OK) {
        S.error = handle_error(S.h, S.status);
        if (comms[(size_t)s]) mvba_comm_abort(comms[(size_t)s]);  // release the other shards
      }
    };
    if (ngpu == 1) {
      solve_one(0);
    } else {
      std::vector<std::thread> th;
      for (int s = 0; s < ngpu; s++) th.emplace_back(solve_one, s);
      for (auto& x : th) x.join();
    }
    for (int s = 0; s < ngpu && ngpu > 1; s++) {
      (void)hipStreamSynchronize(streams[(size_t)s]);
      (void)hipStreamDestroy(streams[(size_t)s]);
      mvba_comm_destroy(comms[(size_t)s]);
    }
    for (auto& S : shards)
      if (S.status != MVBA_OK) fatal(S.error);
    t_solve += secs(t0);
    {
      const auto& sm = shards[0].summary;
      std::cout << "Solver: " << sm.message << " (" << sm.num_iterations << " iterations, "
                << sm.num_successful_steps << " successful; cost " << std::setprecision(10) << sm.initial_cost
                << " -> " << sm.final_cost << ")" << std::endl;
      if (F.profile)
        std::cout << std::setprecision(4) << "Solver time " << sm.total_time_s << " s (linearize "
                  << sm.linearize_time_s << ", linear solver " << sm.linear_solver_time_s << ", evaluation "
                  << sm.eval_time_s << "), " << sm.num_linear_iterations << " CG iterations" << std::endl;
    }

    // copy the optimized state back (:1924-1967); camera-side blocks are equal
    // on every shard, points come from their own shard
    for (size_t s = 0; s < shards.size(); s++) {
      Shard& S = shards[s];
      std::vector<double> x(S.blocks.x.size());
      check(S.h, mvba_get_params(S.h, x.data()));
      for (size_t b = 0; b < S.blocks.size.size(); b++) {
        const bool is_point = S.blocks.size[b] == 3 && S.blocks.owner[b] >= xyz_vec.data() &&
                              S.blocks.owner[b] < xyz_vec.data() + xyz_vec.size();
        if (is_point || s == 0)
          std::memcpy(S.blocks.owner[b], x.data() + S.blocks.off[b], sizeof(double) * (size_t)S.blocks.size[b]);
      }
    }
    // RPC: refit the undistortion half to the optimized distortion half
    // (updateRpcUndistortion, rig_calibrator.cc:1946-1948 -> camera_params.cc:214-253)
    for (int t = 0; t < ncam; t++) {
      auto& D = dist[(size_t)t];
      if (!intrinsics_to_float[(size_t)t].count("distortion") || D.size() <= 5) continue;
      const int num_samples = 400, num_iter = 100;
      std::cout << "Finding RPC undistortion. Using " << num_samples << " samples in width and height, " << num_iter
                << " iterations, and " << F.num_opt_threads << " threads." << std::endl;
      const size_t half = D.size() / 2;
      mvba_rpc_camera rc{};
      rc.focal = focal[(size_t)t];
      rc.center[0] = center[(size_t)t][0];
      rc.center[1] = center[(size_t)t][1];
      rc.dist_size = (int32_t)D.size();
      rc.dist = D.data();
      const auto& cp = rig.params[(size_t)t];
      for (int k = 0; k < 2; k++) {
        rc.image_size[k] = cp.image_size[k];
        rc.crop_size[k] = cp.crop_size[k];
        rc.undist_size[k] = cp.undist_size[k];
      }
      const int deg = (int)std::lround(std::sqrt(2.0 * (double)half + 5.0) / 2.0 - 1.5);
      std::vector<double> undist(half);
      mvba_rpc_fit_report rep{};
      if (mvba_rpc_fit(&rc, MVBA_RPC_FIT_UNDISTORTION, deg, D.data(), num_samples, num_iter, 1e-12, device0,
                       undist.data(), &rep) != MVBA_OK)
        fatal(std::string("RPC undistortion fit: ") + mvba_rpc_error());
      std::copy(undist.begin(), undist.end(), D.begin() + (std::ptrdiff_t)half);
      std::cout << "Max distort_undistort error: " << rep.max_dist_undist_error << std::endl;
    }
    t0 = Clock::now();
    residual_stats(shards, cam_names, "after opt");
    t_stats += secs(t0);

    // residuals of every inlier feature after the solve (evalResiduals output)
    t0 = Clock::now();
    residuals_after.assign(2 * (size_t)nobs, 0.0);
    for (auto& S : shards) {
      std::vector<double> r(2 * S.res_feature.size());
      check(S.h, mvba_evaluate(S.h, MVBA_EVAL_RESIDUALS, 0.0, nullptr, r.data(), nullptr));
      for (size_t i = 0; i < S.res_feature.size(); i++) {
        residuals_after[2 * (size_t)S.res_feature[i]] = r[2 * i];
        residuals_after[2 * (size_t)S.res_feature[i] + 1] = r[2 * i + 1];
      }
    }
    for (auto& S : shards) mvba_destroy(S.h);
    update_world_to_cam();
    {
      mvba_tracks_desc d = tracks_desc();
      int64_t counts[4];
      if (mvba_flag_outliers(&d, device0, xyz_vec.data(), residuals_after.data(), F.min_triangulation_angle,
                             F.max_reprojection_error, inlier.data(), counts) != MVBA_OK)
        fatal(std::string("outlier flagging: ") + mvba_tracks_error());
      std::cout << std::setprecision(4) << "Removed " << counts[0]
                << " outlier features with small angle of convergence, out of " << counts[1] << " ("
                << (counts[1] ? (100.0 * (double)counts[0]) / (double)counts[1] : 0.0) << " %)\n";
      std::cout << std::setprecision(4) << "Removed " << counts[2]
                << " outlier features using reprojection error, out of " << counts[3] << " ("
                << (counts[3] ? (100.0 * (double)counts[2]) / (double)counts[3] : 0.0) << " %)\n";
    }
    t_flag += secs(t0);
  }

  if (mesh) mvba_mesh_destroy(mesh);

  // outputs (:1989-2038)
  for (int t = 0; t < ncam; t++) {
    if (F.affine_depth_to_image)
      depth_to_image[(size_t)t] = array_to_affine(&depth_to_image_vec[(size_t)num_depth_params * (size_t)t]);
    else
      depth_to_image[(size_t)t] = array_to_rigid(&depth_to_image_vec[(size_t)num_depth_params * (size_t)t]);
    for (double& r : depth_to_image[(size_t)t].R) r *= depth_scales[(size_t)t];
  }
  update_world_to_cam();
  std::vector<std::string> image_names(ncams);
  for (size_t c = 0; c < ncams; c++) image_names[c] = cams[c].image_name;
  save_camera_poses(F.out_dir, image_names, world_to_cam);
  RigConfig out = rig;
  for (int t = 0; t < ncam; t++) {
    out.params[(size_t)t].focal = focal[(size_t)t];
    out.params[(size_t)t].center[0] = center[(size_t)t][0];
    out.params[(size_t)t].center[1] = center[(size_t)t][1];
    out.params[(size_t)t].dist = dist[(size_t)t];
    out.ref_to_cam[(size_t)t] = array_to_rigid(&ref_to_cam_vec[7 * (size_t)t]);
  }
  out.depth_to_image = depth_to_image;
  out.offsets = offsets;
  write_rig_config(F.out_dir, !F.no_rig, out);
  if (F.save_nvm) {
    // writeNvm (interest_point.cc:1333-1404): inliers only, keypoints relative
    // to the optical center, tracks with more than two inlier features
    std::vector<std::vector<std::array<double, 2>>> kp(ncams);
    std::vector<double> foc(ncams);
    for (size_t c = 0; c < ncams; c++) foc[c] = focal[(size_t)cams[c].camera_type];
    std::vector<std::map<int, int>> out_tracks;
    std::vector<std::array<double, 3>> out_xyz;
    for (int p = 0; p < npid; p++) {
      std::map<int, int> cf;
      for (int64_t o = track_begin[(size_t)p]; o < track_begin[(size_t)p + 1]; o++) {
        if (!inlier[(size_t)o]) continue;
        const int cid = track_image[(size_t)o];
        const auto& k = keypoint_vec[(size_t)cid][(size_t)track_fid[(size_t)o]];
        const auto& ctr = center[(size_t)cams[(size_t)cid].camera_type];
        cf[cid] = (int)kp[(size_t)cid].size();
        kp[(size_t)cid].push_back({(double)k.first - ctr[0], (double)k.second - ctr[1]});
      }
      if (cf.size() > 2) {
        out_tracks.push_back(cf);
        out_xyz.push_back({xyz_vec[3 * (size_t)p], xyz_vec[3 * (size_t)p + 1], xyz_vec[3 * (size_t)p + 2]});
      }
    }
    write_nvm_file(F.out_dir + "/cameras.nvm", kp, image_names, foc, out_tracks, out_xyz, world_to_cam);
  }
  if (F.profile)
    std::cout << std::setprecision(4) << "Timings (s): triangulation " << t_tri << ", problem setup " << t_build
              << " (mvba_create " << t_create << "), residual stats " << t_stats << ", solve " << t_solve << ", outlier flagging " << t_flag
              << std::endl;
  return 0;
}

}  // namespace rigcal

int main(int argc, char** argv) {
  try {
    return rigcal::run(argc, argv);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
}
