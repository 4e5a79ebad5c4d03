// rgbd360/compat.h — source compatibility for the reference's call sites.
//
// The reference's applications (Registration/OdometryRGBD360.cpp, SLAM/SphereGraphSLAM.cpp, ...) include
// RegisterRGBD360.h / Frame360.h / Calib360.h and use the classes in the global namespace with Eigen poses,
// mrpt::format file names and Miscellaneous.h helpers.  Including this header instead lets those call sites
// compile unchanged against the façade:
//
//   Calib360 calib;                        calib.loadExtrinsicCalibration(); calib.loadIntrinsicCalibration();
//   RegisterRGBD360 registerer(mrpt::format("%s/config_files/configLocaliser_sphericalOdometry.ini", PROJECT_SOURCE_PATH));
//   Frame360* f = new Frame360(&calib);    f->loadFrame(file); f->undistort(); f->stitchSphericalImage();
//                                          f->buildSphereCloud(); f->getPlanes();
//   registerer.RegisterPbMap(f1, f2, 25, RegisterRGBD360::PLANAR_3DoF);  registerer.getPose();
//   RegisterPhotoICP align360;             align360.setNumPyr(5); align360.setGrayVariance(3.f/255);
//   align360.setTargetFrame(f1->sphereRGB, f1->sphereDepth);  align360.alignFrames360(T, RegisterPhotoICP::PHOTO_DEPTH);
//
// What it provides, all opt-in through this header only:
//   * Calib360, Frame360, RegisterPhotoICP, RegisterRGBD360, Plane in the global namespace;
//   * Eigen::Matrix4f and Eigen::Matrix<float,6,6> as r360::Matrix4f / Matrix6f when Eigen itself is not used
//     (RGBD360_WITH_EIGEN makes the façade use the real Eigen types instead);
//   * mrpt::format (printf-style std::string) unless MRPT's own header came first;
//   * PROJECT_SOURCE_PATH = r360_data_dir() (data/) unless the build defines it, so the reference's
//     "%s/config_files/..." paths resolve to data/config_files/...;
//   * PI and fexists() of Miscellaneous.h (:44, :120-124).
#pragma once
#include <rgbd360/rgbd360.h>

#include <fstream>
#include <string>

using r360::Calib360;
using r360::Frame360;
using r360::PbMap;
using r360::Plane;
using r360::RegisterPhotoICP;
using r360::RegisterRGBD360;

#if !defined(RGBD360_WITH_EIGEN) && !defined(EIGEN_CORE_H) && !defined(EIGEN_CORE_MODULE_H)
namespace r360 {
template <typename Scalar, int Rows, int Cols>
struct EigenStandIn;                    // only the two fixed-size float matrices of the registration surface
template <> struct EigenStandIn<float, 4, 4> { typedef Matrix4f type; };
template <> struct EigenStandIn<float, 6, 6> { typedef Matrix6f type; };
}  // namespace r360
namespace Eigen {
typedef r360::Matrix4f Matrix4f;
// Eigen::Matrix<float,6,6> (getInfoMat / getHessian, SphereGraphSLAM.cpp:200-201, LoopClosure360.h:314) and
// Eigen::Matrix<float,4,4>
template <typename Scalar, int Rows, int Cols, int Options = 0, int MaxRows = Rows, int MaxCols = Cols>
using Matrix = typename r360::EigenStandIn<Scalar, Rows, Cols>::type;
}  // namespace Eigen
#endif

#if !defined(MRPT_FORMAT_H) && !defined(RGBD360_NO_MRPT_FORMAT)
namespace mrpt {
using r360::format;
}
#endif

namespace r360 {
// the data tree's root: config_files/ and calib/ live under <root>/data here, where the reference has them at its
// PROJECT_SOURCE_PATH root
inline const char* project_source_path() {
    static const std::string p = std::string(r360_data_dir());
    return p.c_str();
}
}  // namespace r360

#ifndef PROJECT_SOURCE_PATH
#define PROJECT_SOURCE_PATH (r360::project_source_path())
#endif

#ifndef PI
#define PI 3.14159265359
#endif

inline bool fexists(const char* filename) {
    std::ifstream ifile(filename);
    return static_cast<bool>(ifile);
}
