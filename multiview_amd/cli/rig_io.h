// rig_io.h — file formats of the rig_calibrator CLI.
//
//   rig configuration  readRigConfig / writeRigConfig   dense_map_utils.cc:779-1057
//   NVM_V3 sparse map  ReadNVM / WriteNVM / writeNvm      interest_point.cc:1248-1460
//   camera list        readCameraPoses / saveCameraPoses  interest_point.cc:1673-1740,
//                                                         dense_map_utils.cc:753-776
//   image entries      readImageEntry (sensor = parent directory, timestamp =
//                      leading number of the file name, depth cloud = same
//                      name with extension .pc)          interest_point.cc:1611-1671
//   depth clouds       readXyzImage (int32 rows, cols, channels; float32 xyz)
//                                                         interest_point.cc:1585-1609
// Errors are thrown as std::runtime_error carrying the reference's LOG(FATAL)
// text; the CLI prints them and exits non-zero.
#ifndef MVBA_CLI_RIG_IO_H_
#define MVBA_CLI_RIG_IO_H_

#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rig_math.h"

namespace rigcal {

// camera::CameraParameters as far as the calibrator uses it.
struct CameraParams {
  double focal = 0;                 // one focal length (fx = fy, dense_map_utils.cc:988-989)
  double center[2] = {0, 0};        // optical offset
  std::vector<double> dist;         // distortion coefficients (RPC: [dist | undist])
  int image_size[2] = {0, 0};       // distorted size
  int crop_size[2] = {0, 0};        // distorted crop size
  int undist_size[2] = {0, 0};      // undistorted size
};

struct RigConfig {
  std::vector<std::string> cam_names;
  std::vector<CameraParams> params;
  std::vector<Affine> ref_to_cam;
  std::vector<Affine> depth_to_image;
  std::vector<double> offsets;  // ref_to_sensor_timestamp_offset
};

// Distortion type names (dense_map_utils.h).
extern const char* const kNoDistortion;
extern const char* const kFisheyeDistortion;
extern const char* const kRadtanDistortion;
extern const char* const kRpcDistortion;

// Valid RPC coefficient count (one half of [dist | undist]): 2 (d+1)(d+2) - 2.
bool valid_rpc_size(size_t half);

RigConfig read_rig_config(const std::string& path, bool have_rig_transforms);
void write_rig_config(const std::string& out_dir, bool model_rig, const RigConfig& rig);

struct NvmData {
  std::vector<std::string> cid_to_filename;
  std::vector<std::vector<std::array<double, 2>>> cid_to_keypoint;  // [cid][fid]
  std::vector<std::map<int, int>> pid_to_cid_fid;
  std::vector<std::array<double, 3>> pid_to_xyz;
  std::vector<Affine> cid_to_cam_t_global;  // world_to_cam
};

NvmData read_nvm(const std::string& path);
void write_nvm_file(const std::string& path, const std::vector<std::vector<std::array<double, 2>>>& keypoints,
                    const std::vector<std::string>& filenames, const std::vector<double>& focal,
                    const std::vector<std::map<int, int>>& pid_to_cid_fid,
                    const std::vector<std::array<double, 3>>& pid_to_xyz, const std::vector<Affine>& world_to_cam);

struct DepthCloud {
  int rows = 0, cols = 0;
  std::vector<float> xyz;  // rows*cols*3
};
std::shared_ptr<DepthCloud> read_xyz_image(const std::string& path);
void save_xyz_image(const std::string& path, const DepthCloud& c);

struct ImageMessage {
  std::string name;
  double timestamp = 0;
  Affine world_to_cam;
  std::shared_ptr<DepthCloud> cloud;  // depth entries only
};

// Per sensor, chronological (the reference's std::map<double, ...> then vectors).
struct ImageData {
  std::vector<double> ref_timestamps;
  std::vector<Affine> world_to_ref;
  std::vector<std::string> ref_image_files;
  std::vector<std::vector<ImageMessage>> images;  // [cam_type]
  std::vector<std::vector<ImageMessage>> depths;  // [cam_type]
};

// readImageEntry over a list of (image file, world_to_cam), then ImageDataToVectors.
ImageData read_image_entries(const std::vector<std::string>& files, const std::vector<Affine>& world_to_cam,
                             const std::vector<std::string>& cam_names, int ref_cam_type);
// readCameraPoses: "<image> <12 numbers>" lines, '#' comments.
void read_camera_poses_file(const std::string& path, std::vector<std::string>& files,
                            std::vector<Affine>& world_to_cam);

std::string affine_to_str(const Affine& A);
void save_camera_poses(const std::string& out_dir, const std::vector<std::string>& image_names,
                       const std::vector<Affine>& world_to_cam);

void create_dir(const std::string& dir);

// mve::geom::load_ply_mesh as loadMeshBuildTree uses it (texture_processing.cc:268):
// "ply" header, format ascii 1.0 / binary_little_endian 1.0 / binary_big_endian
// 1.0; element vertex with float/double x y z (other properties skipped); element
// face with a list property vertex_indices (or vertex_index) of triangles; other
// elements skipped. False with a message on anything else.
bool read_ply_mesh(const std::string& path, std::vector<float>& vertices, std::vector<uint32_t>& faces,
                   std::string& err);

}  // namespace rigcal

#endif  // MVBA_CLI_RIG_IO_H_
