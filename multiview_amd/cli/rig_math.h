// rig_math.h — host-side rigid/affine transform helpers of the rig_calibrator
// CLI (orchestration only: image poses for triangulation and outlier flagging,
// the initial rig guess, file output). The per-observation math of the hot path
// runs on the GPU (libmvba); these helpers restate the same reference
// conventions for the few hundred/thousand image poses a pass needs.
//
// Conventions (reference):
//   7-array [tx ty tz qx qy qz qw]      dense_map_utils.cc:159-178
//   12-array row-major 3x4 affine        dense_map_utils.cc:181-208
//   Eigen Quaternion(Matrix3d), toRotationMatrix, slerp  [ext Eigen 3.4]
//   linearInterp                         dense_map_utils.cc:315-329
//   calc_interp_world_to_ref             rig_calibrator.cc:322-353
//   calc_world_to_cam_trans              rig_calibrator.cc:362-390
#ifndef MVBA_CLI_RIG_MATH_H_
#define MVBA_CLI_RIG_MATH_H_

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace rigcal {

// Affine transform: linear part row-major, translation.
struct Affine {
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  double t[3] = {0, 0, 0};
};

inline Affine identity() { return Affine(); }

inline Affine compose(const Affine& A, const Affine& B) {  // A * B
  Affine C;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++)
      C.R[3 * r + c] = A.R[3 * r] * B.R[c] + A.R[3 * r + 1] * B.R[3 + c] + A.R[3 * r + 2] * B.R[6 + c];
    C.t[r] = A.R[3 * r] * B.t[0] + A.R[3 * r + 1] * B.t[1] + A.R[3 * r + 2] * B.t[2] + A.t[r];
  }
  return C;
}

inline double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
         m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// General affine inverse (Eigen Transform<Affine>::inverse(): linear part
// inverted through its adjugate, t' = -L^-1 t).
inline Affine inverse(const Affine& A) {
  const double* m = A.R;
  double c[9];
  c[0] = m[4] * m[8] - m[5] * m[7];
  c[1] = m[2] * m[7] - m[1] * m[8];
  c[2] = m[1] * m[5] - m[2] * m[4];
  c[3] = m[5] * m[6] - m[3] * m[8];
  c[4] = m[0] * m[8] - m[2] * m[6];
  c[5] = m[2] * m[3] - m[0] * m[5];
  c[6] = m[3] * m[7] - m[4] * m[6];
  c[7] = m[1] * m[6] - m[0] * m[7];
  c[8] = m[0] * m[4] - m[1] * m[3];
  const double det = m[0] * c[0] + m[1] * c[3] + m[2] * c[6];
  Affine I;
  for (int k = 0; k < 9; k++) I.R[k] = c[k] / det;
  for (int r = 0; r < 3; r++) I.t[r] = -(I.R[3 * r] * A.t[0] + I.R[3 * r + 1] * A.t[1] + I.R[3 * r + 2] * A.t[2]);
  return I;
}

// Eigen QuaternionBase::toRotationMatrix, q = (x, y, z, w), no normalisation.
inline void quat_to_rot(double x, double y, double z, double w, double* R) {
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Eigen Quaternion(const Matrix3&): largest-pivot (Shepperd) extraction, q = x y z w.
inline void rot_to_quat(const double* m, double* q) {
  double t = m[0] + m[4] + m[8];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (m[7] - m[5]) * t;
    q[1] = (m[2] - m[6]) * t;
    q[2] = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[3 * i + i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
    q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
    q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
  }
}

// rigid_transform_to_array: [t, q(x y z w)] with q = Quaterniond(linear()).
inline void rigid_to_array(const Affine& A, double* arr) {
  for (int k = 0; k < 3; k++) arr[k] = A.t[k];
  rot_to_quat(A.R, arr + 3);
}

// array_to_rigid_transform: the quaternion is normalised first.
inline Affine array_to_rigid(const double* arr) {
  double x = arr[3], y = arr[4], z = arr[5], w = arr[6];
  const double n2 = x * x + y * y + z * z + w * w;
  if (n2 > 0) {
    const double n = std::sqrt(n2);
    x /= n; y /= n; z /= n; w /= n;
  }
  Affine A;
  quat_to_rot(x, y, z, w, A.R);
  for (int k = 0; k < 3; k++) A.t[k] = arr[k];
  return A;
}

// affine_transform_to_array / array_to_affine_transform: row-major 3x4.
inline void affine_to_array(const Affine& A, double* arr) {
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) arr[4 * r + c] = A.R[3 * r + c];
    arr[4 * r + 3] = A.t[r];
  }
}
inline Affine array_to_affine(const double* arr) {
  Affine A;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) A.R[3 * r + c] = arr[4 * r + c];
    A.t[r] = arr[4 * r + 3];
  }
  return A;
}

// vecToAffine (transform_utils.cc:44-70): 9 linear entries row-major, then t.
inline Affine vec12_to_affine(const double* v) {
  Affine A;
  for (int k = 0; k < 9; k++) A.R[k] = v[k];
  for (int k = 0; k < 3; k++) A.t[k] = v[9 + k];
  return A;
}

// linearInterp: translation lerp, rotation Eigen slerp of the quaternions
// extracted from both linear parts.
inline Affine linear_interp(double alpha, const Affine& A0, const Affine& A1) {
  double q0[4], q1[4];
  rot_to_quat(A0.R, q0);
  rot_to_quat(A1.R, q1);
  const double d = q0[0] * q1[0] + q0[1] * q1[1] + q0[2] * q1[2] + q0[3] * q1[3];
  const double ad = std::fabs(d);
  double s0, s1;
  if (ad >= 1.0 - 2.220446049250313e-16) {  // 1 - NumTraits<double>::epsilon()
    s0 = 1.0 - alpha;
    s1 = alpha;
  } else {
    const double th = std::acos(ad), st = std::sin(th);
    s0 = std::sin((1.0 - alpha) * th) / st;
    s1 = std::sin(alpha * th) / st;
  }
  if (d < 0) s1 = -s1;
  double q[4];
  for (int k = 0; k < 4; k++) q[k] = s0 * q0[k] + s1 * q1[k];
  Affine R;
  quat_to_rot(q[0], q[1], q[2], q[3], R.R);
  for (int k = 0; k < 3; k++) R.t[k] = (1.0 - alpha) * A0.t[k] + alpha * A1.t[k];
  return R;
}

// calc_interp_world_to_ref; throws on alpha outside [0, 1] (":346" fatal).
inline Affine interp_world_to_ref(const double* beg, const double* end, double beg_stamp, double end_stamp,
                                  double offset, double cam_stamp) {
  Affine b = array_to_rigid(beg), e = array_to_rigid(end);
  if (end_stamp == beg_stamp) return b;
  const double alpha = ((cam_stamp - beg_stamp) - offset) / (end_stamp - beg_stamp);
  if (alpha < 0.0 || alpha > 1.0) throw std::runtime_error("Out of bounds in interpolation.");
  return linear_interp(alpha, b, e);
}

// calc_world_to_cam_trans
inline Affine world_to_cam_trans(const double* beg, const double* end, const double* ref_to_cam, double beg_stamp,
                                 double end_stamp, double offset, double cam_stamp) {
  if (beg_stamp == end_stamp) return array_to_rigid(beg);
  return compose(array_to_rigid(ref_to_cam), interp_world_to_ref(beg, end, beg_stamp, end_stamp, offset, cam_stamp));
}

}  // namespace rigcal

#endif  // MVBA_CLI_RIG_MATH_H_
