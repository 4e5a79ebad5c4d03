// rgbd360/rgbd360.h — C++ façade of librgbd360_hip.so with the reference's class names and method
// signatures for the registration hot path:
//
//   Calib360          include/Calib360.h:44-132
//   Frame360          include/Frame360.h:93-1150   loadFrame / undistort / stitchSphericalImage /
//                                                  buildSphereCloud / getPlanes / planes
//   RegisterPhotoICP  include/RegisterPhotoICP.h   setters :224-269, setSourceFrame/setTargetFrame
//                                                  :480-516, alignFrames360 :4519, getOptimalPose :273,
//                                                  getHessian/getGradient :279-288
//   RegisterRGBD360   include/RegisterRGBD360.h    ctor(ini) :97, setReference/setTarget :111/:161,
//                                                  RegisterPbMap :276, getPose :199, getCovMat :208,
//                                                  getInfoMat :219, calcEntropy :230, getMatchedPlanes :242,
//                                                  getAreaMatched :251, areaSource/areaTarget :91-94,
//                                                  RegisterDensePhotoICP :344, trackingScore :526,
//                                                  Register() = OdometryKeyFrame360.cpp:205-254
//   BatchRegistration  many independent pair registrations on one GPU (§8f-4): SphereGraphSLAM's
//                      tracking loop (SLAM/SphereGraphSLAM.cpp:169-231) and LoopClosure360's candidate
//                      checks (include/LoopClosure360.h:280-366)
//
// Header-only; every body is a call into the C-ABI (include/rgbd360_hip.h).  Matrices are the
// column-major Eigen layout; r360::Matrix4f / Matrix6f are minimal stand-ins with Eigen's (row, col)
// accessors and data() — define RGBD360_WITH_EIGEN to use Eigen::Matrix4f / Matrix<float,6,6>.
// Differences from the reference surface, all forced by the GPU-resident design:
//   * images are r360::Mat (rows, cols, channels, bytes) instead of cv::Mat.  Frame360::sphereRGB /
//     sphereDepth are views of the frame's sphere in HBM: RegisterPhotoICP::setSourceFrame(
//     frame->sphereRGB, frame->sphereDepth) uses the frame's device pyramid without a copy; other images
//     are uploaded and pyramided on the GPU (r360_frame_set_sphere);
//   * objects are bound to an r360::Context (one GPU + HIP stream); errors throw r360::Error.  The constructors with
//     the reference's signatures (Calib360(Resolution), RegisterPhotoICP(), RegisterRGBD360(configFile)) bind to
//     r360::default_context(): one context per host thread on device $R360_DEVICE (default 0), created on first
//     use.  include/rgbd360/compat.h brings the class names into the global namespace for unchanged call sites.
#pragma once
#include <rgbd360_hip.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <ostream>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#ifdef RGBD360_WITH_EIGEN
#include <Eigen/Dense>
#endif

namespace r360 {

struct Error : std::runtime_error {
    explicit Error(const std::string& what) : std::runtime_error(what + ": " + r360_last_error()) {}
};
inline int check(int rc, const char* what) {
    if (rc < 0) throw Error(what);
    return rc;
}

#ifdef RGBD360_WITH_EIGEN
typedef Eigen::Matrix4f Matrix4f;
typedef Eigen::Matrix<float, 6, 6> Matrix6f;
#else
template <int N>
struct MatrixNf {                       // column-major, Eigen's (row, col) and data()
    float v[N * N];
    MatrixNf() { for (int i = 0; i < N * N; ++i) v[i] = (i % (N + 1) == 0) ? 1.f : 0.f; }
    static MatrixNf Identity() { return MatrixNf(); }
    float& operator()(int r, int c) { return v[c * N + r]; }
    float operator()(int r, int c) const { return v[c * N + r]; }
    float* data() { return v; }
    const float* data() const { return v; }
    MatrixNf operator*(const MatrixNf& b) const {
        MatrixNf o;
        for (int c = 0; c < N; ++c)
            for (int r = 0; r < N; ++r) {
                float acc = (*this)(r, 0) * b(0, c);
                for (int k = 1; k < N; ++k) acc += (*this)(r, k) * b(k, c);
                o(r, c) = acc;
            }
        return o;
    }
    // inverse by Gauss-Jordan elimination with partial pivoting in double (Eigen's Matrix4f::inverse() uses
    // cofactors in float: the two agree to float rounding)
    MatrixNf inverse() const {
        double A[N][2 * N];
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < 2 * N; ++c) A[r][c] = c < N ? (*this)(r, c) : (c - N == r ? 1.0 : 0.0);
        for (int k = 0; k < N; ++k) {
            int p = k;
            for (int r = k + 1; r < N; ++r) if (std::fabs(A[r][k]) > std::fabs(A[p][k])) p = r;
            for (int c = 0; c < 2 * N; ++c) { const double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
            const double piv = A[k][k];
            for (int c = 0; c < 2 * N; ++c) A[k][c] /= piv;
            for (int r = 0; r < N; ++r)
                if (r != k) { const double f = A[r][k]; for (int c = 0; c < 2 * N; ++c) A[r][c] -= f * A[k][c]; }
        }
        MatrixNf o;
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < N; ++c) o(r, c) = float(A[r][c + N]);
        return o;
    }
    // block(r0, c0, rows, cols) as a read-only view with Eigen's norm() (e.g. the translation's length,
    // rigidTransf.block(0,3,3,1).norm(), OdometryRGBD360.cpp:228)
    struct Block {
        const MatrixNf* m;
        int r0, c0, rows, cols;
        float operator()(int r, int c) const { return (*m)(r0 + r, c0 + c); }
        float norm() const {
            float s = 0.f;
            for (int c = 0; c < cols; ++c)
                for (int r = 0; r < rows; ++r) s += (*this)(r, c) * (*this)(r, c);
            return std::sqrt(s);
        }
    };
    Block block(int r0, int c0, int rows, int cols) const { return Block{this, r0, c0, rows, cols}; }
};
template <int N>
inline std::ostream& operator<<(std::ostream& os, const MatrixNf<N>& m) {
    for (int r = 0; r < N; ++r) {
        for (int c = 0; c < N; ++c) os << (c ? " " : "") << m(r, c);
        if (r + 1 < N) os << "\n";
    }
    return os;
}
// scalar * matrix (e.g. registerer.getAreaMatched() * registerer.getInfoMat(), KFsphere_SLAM.cpp:454)
template <int N>
inline MatrixNf<N> operator*(float s, const MatrixNf<N>& m) {
    MatrixNf<N> o;
    for (int i = 0; i < N * N; ++i) o.v[i] = s * m.v[i];
    return o;
}
typedef MatrixNf<4> Matrix4f;
typedef MatrixNf<6> Matrix6f;
#endif

class Frame360;

// Host image (cv::Mat stand-in: CV_8UC3 BGR sphereRGB, CV_16UC1 range-mm sphereDepth).  A Mat whose `frame`
// is set is a view of that Frame360's sphere in HBM (no host pixels until Frame360::downloadSphere()).
struct Mat {
    int rows = 0, cols = 0, channels = 1, elem = 1;   // elem: bytes per channel
    std::vector<uint8_t> bytes;
    const Frame360* frame = nullptr;
    Mat() = default;
    Mat(int r, int c, int ch, int e) : rows(r), cols(c), channels(ch), elem(e), bytes(size_t(r) * c * ch * e) {}
    uint8_t* data() { return bytes.data(); }
    const uint8_t* data() const { return bytes.data(); }
    bool empty() const { return rows == 0 || cols == 0; }
};

class Context {
  public:
    explicit Context(int device = 0) { check(r360_ctx_create(device, &h_), "r360_ctx_create"); }
    ~Context() { r360_ctx_destroy(h_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    r360_ctx* get() const { return h_; }
    void sync() { check(r360_ctx_sync(h_), "r360_ctx_sync"); }
  private:
    r360_ctx* h_ = nullptr;
};

// The default contexts of the reference-signature constructors: one per host thread (its own HIP stream), on device
// $R360_DEVICE (default 0), created on first use.  A thread's default context lives as long as its thread or the
// last object built on it, whichever is longer: Calib360(Resolution) and the frames built on it hold a reference, so
// frames built on one thread stay valid after it exits.  RegisterRGBD360(configFile) and RegisterPhotoICP() hold
// no context of their own: each call runs on the CALLING thread's default context, so an object constructed on one
// thread and used on another (LoopClosure360's registerer, constructed by the main thread and used by its loop
// thread, LoopClosure360.h:83-94, 297) never shares a context between threads.  Frames are shared freely: a
// registration on another thread's context waits for the frames' builds on their own streams.
inline int default_device() {
    const char* e = std::getenv("R360_DEVICE");
    return e ? std::atoi(e) : 0;
}
inline const std::shared_ptr<Context>& default_context_ptr() {
    thread_local std::shared_ptr<Context> ctx = std::make_shared<Context>(default_device());
    return ctx;
}
inline Context& default_context() { return *default_context_ptr(); }

// printf-style std::string (the callers' mrpt::format for file names)
inline std::string format(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char buf[4096];
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return std::string(buf);
}
inline std::string data_dir() { return r360_data_dir(); }

// ------------------------------------------------------------------ Calib360
class Calib360 {
  public:
    // Resolution mode of the device (Calib360.h:62-67): per-sensor images of 480/res x 640/res
    enum Resolution { VGA = 1, QVGA = 2, QQVGA = 4 };
    // Calib360(Resolution res = QVGA) (Calib360.h:70), on the thread's default context
    explicit Calib360(Resolution res = QVGA) : Calib360(default_context(), 480 / int(res), 640 / int(res)) {
        keep_ = default_context_ptr();
    }
    // rows x cols per sensor (the reference's QVGA default, Calib360.h:73-77)
    explicit Calib360(Context& ctx, int rows = 240, int cols = 320) : ctx_(ctx) {
        check(r360_calib_create(ctx.get(), rows, cols, &h_), "r360_calib_create");
        resolution = Resolution(cols > 0 && 640 % cols == 0 ? 640 / cols : 0);
    }
    ~Calib360() { r360_calib_destroy(h_); }
    Calib360(const Calib360&) = delete;
    Calib360& operator=(const Calib360&) = delete;
    // "" = the shipped calibration (data/calib/Extrinsics), as the reference's default argument (Calib360.h:122-125)
    void loadExtrinsicCalibration(const std::string& dir = "") {
        check(r360_calib_load_extrinsics(h_, dir.c_str()), "loadExtrinsicCalibration");
    }
    // "" = data/calib/Intrinsics (Calib360.h:104-107)
    void loadIntrinsicCalibration(const std::string& dir = "") {
        check(r360_calib_load_intrinsics(h_, dir.c_str()), "loadIntrinsicCalibration");
    }
    Resolution resolution;
    Matrix4f getRt_id(int sensor_id) const {
        float rt[128];
        check(r360_calib_get_extrinsics(h_, rt, nullptr, nullptr), "getRt_id");
        Matrix4f m;
        std::memcpy(m.data(), rt + 16 * sensor_id, sizeof(float) * 16);
        return m;
    }
    r360_calib* get() const { return h_; }
    Context& ctx() const { return ctx_; }
    // the default context this calibration was built on (null for an explicit Context)
    const std::shared_ptr<Context>& keepAlive() const { return keep_; }
  private:
    Context& ctx_;
    std::shared_ptr<Context> keep_;
    r360_calib* h_ = nullptr;
};

// ------------------------------------------------------------------ Frame360
struct Plane {                          // mrpt::pbmap::Plane fields used on the path
    float v3normal[3], v3center[3], d, areaHull, elongation, curvature, v3PpalDir[3], v3colorNrgb[3],
        dominantIntensity;
    unsigned id;
    int sensor;
    size_t n_inliers;
    std::vector<float> polygonContour;  // closed hull polygon, xyz triples
    std::string label;                  // Plane::label (labelization tools), kept by savePlanes
};

// mrpt::pbmap::PbMap as Frame360::planes holds it (Frame360.h:123): the planes in vPlanes (callers write
// frame360->planes.vPlanes[i], OnlineOdometryRGBD360.cpp:172,330); size() / operator[] / iteration forward to it
struct PbMap {
    std::vector<Plane> vPlanes;
    size_t size() const { return vPlanes.size(); }
    bool empty() const { return vPlanes.empty(); }
    Plane& operator[](size_t i) { return vPlanes[i]; }
    const Plane& operator[](size_t i) const { return vPlanes[i]; }
    std::vector<Plane>::iterator begin() { return vPlanes.begin(); }
    std::vector<Plane>::iterator end() { return vPlanes.end(); }
    std::vector<Plane>::const_iterator begin() const { return vPlanes.begin(); }
    std::vector<Plane>::const_iterator end() const { return vPlanes.end(); }
};

class Frame360 {
  public:
    explicit Frame360(Calib360* calib_) : calib(calib_), keep_(calib_->keepAlive()) {
        check(r360_frame_create(calib->ctx().get(), calib->get(), &h_), "r360_frame_create");
        int r, c, sr, sc;
        check(r360_frame_dims(h_, &r, &c, &sr, &sc), "r360_frame_dims");
        sphereRGB.rows = sphereDepth.rows = sr;
        sphereRGB.cols = sphereDepth.cols = sc;
        sphereRGB.channels = 3; sphereRGB.elem = 1;
        sphereDepth.channels = 1; sphereDepth.elem = 2;
        sphereRGB.frame = sphereDepth.frame = this;
    }
    ~Frame360() { r360_frame_destroy(h_); }
    Frame360(const Frame360&) = delete;
    Frame360& operator=(const Frame360&) = delete;

    void loadFrame(const std::string& path) { check(r360_frame_load_bin(h_, path.c_str()), "loadFrame"); }
    void upload(const uint8_t* bgr8, const uint16_t* depth8) { check(r360_frame_upload(h_, bgr8, depth8), "upload"); }
    void undistort() { check(r360_frame_build(h_, R360_BUILD_UNDISTORT), "undistort"); }
    void stitchSphericalImage() {
        std::lock_guard<std::mutex> lk(build_m_);
        check(r360_frame_build(h_, R360_BUILD_SPHERE | R360_BUILD_PYRAMID), "stitch");
    }
    void buildSphereCloud() { check(r360_frame_build(h_, R360_BUILD_UNDISTORT | R360_BUILD_CLOUD), "buildSphereCloud"); }
    void getPlanes() {
        check(r360_frame_build(h_, R360_BUILD_UNDISTORT | R360_BUILD_PLANES), "getPlanes");
        fetch_planes();
    }
    // ---- keyframe persistence (Frame360.h:181-228, 312-345)
    void serialize(const std::string& fileName) { check(r360_frame_save_bin(h_, fileName.c_str()), "serialize"); }
    void setTimeStamp(uint64_t t) { check(r360_frame_set_timestamp(h_, t), "setTimeStamp"); }
    uint64_t timeStamp() const { uint64_t t = 0; check(r360_frame_get_timestamp(h_, &t), "timeStamp"); return t; }
    void loadCloud(const std::string& pointCloudPath) { check(r360_frame_load_cloud(h_, pointCloudPath.c_str()), "loadCloud"); }
    void loadPbMap(const std::string& pbmapPath) {
        check(r360_frame_load_pbmap(h_, pbmapPath.c_str()), "loadPbMap");
        fetch_planes();
    }
    void load_PbMap_Cloud(const std::string& pointCloudPath, const std::string& pbmapPath) {
        loadCloud(pointCloudPath);
        loadPbMap(pbmapPath);
    }
    void load_PbMap_Cloud(const std::string& path, unsigned index) {
        check(r360_frame_load_pbmap_cloud(h_, path.c_str(), index), "load_PbMap_Cloud");
        fetch_planes();
    }
    // labels edited in `planes` are written with the map
    void savePlanes(const std::string& pathPbMap) {
        push_labels();
        check(r360_frame_save_planes(h_, pathPbMap.c_str()), "savePlanes");
    }
    void save(const std::string& path, unsigned frame) {
        push_labels();
        check(r360_frame_save(h_, path.c_str(), frame), "save");
    }
    // sphereCloud as xyz triples + PointXYZRGBA-packed colours
    void sphereCloud(std::vector<float>& xyz, std::vector<uint32_t>& rgba, int& width, int& height) {
        check(r360_frame_get_sphere_cloud(h_, nullptr, nullptr, 0, &width, &height), "sphereCloud");
        const size_t n = size_t(width) * size_t(height);
        xyz.resize(3 * n);
        rgba.resize(n);
        check(r360_frame_get_sphere_cloud(h_, xyz.data(), rgba.data(), n, &width, &height), "sphereCloud");
    }
    // Frame360::getPlanarArea (Frame360.h:157)
    float getPlanarArea() const {
        float a = 0.f;
        for (const Plane& p : planes) a += p.areaHull;
        return a;
    }
    // sphereRGB / sphereDepth (Frame360.h:104-107): views of the stitched sphere in HBM
    Mat sphereRGB, sphereDepth;
    // copies the sphere's pixels into sphereRGB / sphereDepth (they stay views of this frame)
    void downloadSphere() {
        ensureSpherePyramid();
        sphereRGB.bytes.resize(size_t(sphereRGB.rows) * sphereRGB.cols * 3);
        sphereDepth.bytes.resize(size_t(sphereDepth.rows) * sphereDepth.cols * 2);
        check(r360_frame_get_sphere(h_, sphereRGB.data(), reinterpret_cast<uint16_t*>(sphereDepth.data())),
              "downloadSphere");
    }
    PbMap planes;                       // the frame's PbMap (planes.vPlanes)
    Matrix4f pose;
    unsigned id = 0;
    unsigned node = 0;                  // topological node (submap) of the frame (Frame360.h:101)
    Calib360* calib;                    // the sensor calibration (Frame360.h:97)
    r360_frame* get() const { return h_; }
    // the stitched sphere and its pyramid, built once (stitchSphericalImage, or the first setSourceFrame /
    // setTargetFrame of the frame's sphere views, possibly from another thread)
    void ensureSpherePyramid() {
        std::lock_guard<std::mutex> lk(build_m_);
        unsigned built = 0;
        check(r360_frame_built(h_, &built), "r360_frame_built");
        const unsigned need = R360_BUILD_SPHERE | R360_BUILD_PYRAMID;   // the stitch reads the raw depth
        if ((built & need) != need) check(r360_frame_build(h_, need), "pyramid");
    }

  private:
    void push_labels() {
        for (size_t i = 0; i < planes.size(); ++i)
            check(r360_frame_set_plane_label(h_, int(i), planes[i].label.c_str()), "plane label");
    }
    void fetch_planes() {
        int n = 0;
        check(r360_frame_get_planes(h_, nullptr, 0, &n), "getPlanes");
        std::vector<r360_plane> raw(n > 0 ? n : 1);
        check(r360_frame_get_planes(h_, raw.data(), n, &n), "getPlanes");
        planes.vPlanes.clear();
        for (int i = 0; i < n; ++i) {
            const r360_plane& r = raw[i];
            Plane p;
            std::memcpy(p.v3normal, r.normal, sizeof p.v3normal);
            std::memcpy(p.v3center, r.center, sizeof p.v3center);
            std::memcpy(p.v3PpalDir, r.ppal, sizeof p.v3PpalDir);
            std::memcpy(p.v3colorNrgb, r.nrgb, sizeof p.v3colorNrgb);
            p.d = r.d; p.areaHull = r.area; p.elongation = r.elongation; p.curvature = r.curvature;
            p.dominantIntensity = r.intensity; p.id = unsigned(r.id); p.sensor = r.sensor;
            p.n_inliers = size_t(r.n_inliers);
            p.polygonContour.resize(3 * size_t(r.n_hull));
            int m = 0;
            check(r360_frame_get_plane_hull(h_, i, p.polygonContour.data(), r.n_hull, &m), "getPlanes");
            const int ll = r360_frame_get_plane_label(h_, i, nullptr, 0);
            if (ll > 0) {
                std::vector<char> buf(size_t(ll) + 1);
                r360_frame_get_plane_label(h_, i, buf.data(), ll + 1);
                p.label = buf.data();
            }
            planes.vPlanes.push_back(p);
        }
    }
    std::shared_ptr<Context> keep_;     // the default context the frame was built on (see default_context_ptr)
    std::mutex build_m_;
    r360_frame* h_ = nullptr;
};

// ------------------------------------------------------------------ RegisterPhotoICP
class RegisterPhotoICP {
  public:
    enum costFuncType { PHOTO_CONSISTENCY = 0, DEPTH_CONSISTENCY = 1, PHOTO_DEPTH = 2 };
    explicit RegisterPhotoICP(Context& ctx) : ctx_(&ctx) { r360_icp_default_params(&p_); }
    // RegisterPhotoICP() (RegisterPhotoICP.h:201): every call on the calling thread's default context
    RegisterPhotoICP() { r360_icp_default_params(&p_); }
    ~RegisterPhotoICP() {
        for (auto& o : own_) { r360_frame_destroy(o.frame); r360_calib_destroy(o.calib); }
    }
    RegisterPhotoICP(const RegisterPhotoICP&) = delete;
    RegisterPhotoICP& operator=(const RegisterPhotoICP&) = delete;
    void setNumPyr(int n) { p_.n_pyr = n; }
    void setMinDepth(float d) { p_.min_depth = d; }
    void setMaxDepth(float d) { p_.max_depth = d; }
    void setGrayVariance(float s) { p_.std_dev_photo = s; }   // sets stdDevPhoto (RegisterPhotoICP.h:242-245)
    void setDepthVariance(float s) { p_.std_dev_depth = s; }
    void useSaliency(bool b) {           // the sphere path never subsamples (the saliency code is commented out)
        if (b) throw std::invalid_argument("useSaliency(true) is not supported on the spherical path");
    }
    void setVisualization(bool) {}      // visualizeIterations: OpenCV windows, no display here
    void setSourceFrame(Frame360& f) { ensure_pyramid(f); src_ = f.get(); }
    void setTargetFrame(Frame360& f) { ensure_pyramid(f); trg_ = f.get(); }
    // setSourceFrame / setTargetFrame(cv::Mat& imgRGB, cv::Mat& imgDepth) (:480-516): a frame's own
    // sphereRGB / sphereDepth use its device pyramid; other images (BGR u8, range u16 mm) are uploaded
    void setSourceFrame(Mat& imgRGB, Mat& imgDepth) { src_ = sphere_frame(0, imgRGB, imgDepth); }
    void setTargetFrame(Mat& imgRGB, Mat& imgDepth) { trg_ = sphere_frame(1, imgRGB, imgDepth); }
    // benchmark timing mode: exactly K level-0 iterations (0 = reference schedule)
    void setFixedIterationsLevel0(int k) { p_.fixed_iters_level0 = k; }
    // returns false where the reference prints "ILL-POSED" and returns early (:4682-4690)
    bool alignFrames360(const Matrix4f& pose_guess = Matrix4f::Identity(), costFuncType method = PHOTO_CONSISTENCY,
                        int occlusion = 0) {
        float g[6];
        const int rc = check(r360_align360(ctx().get(), trg_, src_, pose_guess.data(), method, occlusion,
                                           &p_, relPose_.data(), hessian_.data(), g, &st_),
                             "alignFrames360");
        std::memcpy(gradient_, g, sizeof g);
        SSO = st_.sso;
        // the residual members keep their previous value unless the error function assigns them (:183-189)
        if (st_.residuals_set & 1) { avPhotoResidual = st_.av_photo_residual; avDepthResidual = st_.av_depth_residual; }
        if (st_.residuals_set & 2) avResidual = st_.av_residual;
        return rc == 0;
    }
    Matrix4f getOptimalPose() const { return relPose_; }
    Matrix6f getHessian() const { return hessian_; }
    const float* getGradient() const { return gradient_; }
    float SSO = 0.f;
    // public residual members (RegisterPhotoICP.h:183-189; uninitialised in the reference until assigned)
    float avResidual = std::numeric_limits<float>::quiet_NaN();
    double avPhotoResidual = std::numeric_limits<double>::quiet_NaN();
    double avDepthResidual = std::numeric_limits<double>::quiet_NaN();
    const r360_icp_stats& stats() const { return st_; }
    r360_icp_params& params() { return p_; }
  private:
    Context& ctx() const { return ctx_ ? *ctx_ : default_context(); }
    static void ensure_pyramid(Frame360& f) { f.ensureSpherePyramid(); }
    r360_frame* sphere_frame(int role, Mat& rgb, Mat& depth) {
        if (rgb.frame && rgb.frame == depth.frame) {       // the frame's own sphere views
            Frame360& f = const_cast<Frame360&>(*rgb.frame);
            ensure_pyramid(f);
            return f.get();
        }
        if (rgb.channels != 3 || rgb.elem != 1 || depth.channels != 1 || depth.elem != 2 || rgb.rows != depth.rows ||
            rgb.cols != depth.cols || rgb.bytes.size() < size_t(rgb.rows) * rgb.cols * 3 ||
            depth.bytes.size() < size_t(depth.rows) * depth.cols * 2)
            throw std::invalid_argument("sphere images: BGR u8 x 3 and range u16 of the same size");
        Own* o = nullptr;
        for (auto& x : own_)
            if (x.role == role && x.rows == rgb.rows && x.cols == rgb.cols) o = &x;
        if (!o) {
            own_.push_back(Own{role, rgb.rows, rgb.cols, nullptr, nullptr, ctx_ ? nullptr : default_context_ptr()});
            o = &own_.back();
            check(r360_calib_create_sphere(ctx().get(), rgb.rows, rgb.cols, &o->calib), "sphere calibration");
            check(r360_frame_create(ctx().get(), o->calib, &o->frame), "sphere frame");
        }
        check(r360_frame_set_sphere(o->frame, rgb.data(), reinterpret_cast<const uint16_t*>(depth.data()), rgb.rows,
                                    rgb.cols), "setSourceFrame / setTargetFrame");
        return o->frame;
    }
    struct Own { int role, rows, cols; r360_calib* calib; r360_frame* frame; std::shared_ptr<Context> keep; };
    std::vector<Own> own_;
    Context* ctx_ = nullptr;            // null: the calling thread's default context
    r360_icp_params p_;
    r360_icp_stats st_{};
    r360_frame* src_ = nullptr;
    r360_frame* trg_ = nullptr;
    Matrix4f relPose_;
    Matrix6f hessian_;
    float gradient_[6] = {0, 0, 0, 0, 0, 0};
};

// ------------------------------------------------------------------ RegisterRGBD360
class RegisterRGBD360 {
  public:
    enum registrationType { DEFAULT_6DoF = 0, PLANAR_3DoF = 1, ODOMETRY_6DoF = 2, PLANAR_ODOMETRY_3DoF = 3 };
    // matcher.configLocaliser.load_params(configFile) (:97-100): the [global]/[unary]/[binary] thresholds of
    // the mrpt-pbmap ini; without a file, configLocaliser_sphericalOdometry.ini's values
    // RegisterRGBD360(configFile) (RegisterRGBD360.h:97), on the thread's default context
    // every call on the calling thread's default context
    explicit RegisterRGBD360(const std::string& configFile = "") : config_(configFile) { init(); }
    RegisterRGBD360(Context& ctx, const std::string& configFile = "") : ctx_(&ctx), config_(configFile) { init(); }
    r360_match_params& matchParams() { return match_; }
    void setReference(Frame360* ref, size_t max_match_planes = 0) { ref_ = ref; max_ = max_match_planes; done_ = false; }
    void setTarget(Frame360* trg, size_t max_match_planes = 0) { trg_ = trg; max_ = max_match_planes; done_ = false; }
    bool RegisterPbMap(Frame360* frame1 = nullptr, Frame360* frame2 = nullptr, size_t max_match_planes = 0,
                       registrationType registMode = DEFAULT_6DoF) {
        if (frame1) setReference(frame1, max_match_planes);
        if (frame2) setTarget(frame2, max_match_planes);
        mode_ = registMode;
        done_ = true;
        std::vector<int> pairs(512);
        int n = 0;
        check(r360_ctx_set_match_params(ctx().get(), &match_), "matcher thresholds");
        const int rc = check(r360_register_pbmap(ctx().get(), ref_->get(), trg_->get(), max_, registMode,
                                                 rigidTransf_.data(), informationM_.data(), pairs.data(), 256, &n,
                                                 &areaMatched_, &areaSource, &areaTarget),
                             "RegisterPbMap");
        bestMatch_.clear();
        for (int k = 0; k < n && k < 256; ++k) bestMatch_[unsigned(pairs[2 * k])] = unsigned(pairs[2 * k + 1]);
        return rc == 1;                 // false leaves rigidTransf untouched (RegisterRGBD360.h:306-310)
    }
    Matrix4f getPose() { if (!done_) RegisterPbMap(); return rigidTransf_; }
    Matrix6f& getInfoMat() { if (!done_) RegisterPbMap(); return informationM_; }
    // covarianceM = informationM.inverse() (:208-215)
    Matrix6f getCovMat() {
        if (!done_) RegisterPbMap();
        return inverse6(informationM_);
    }
    // differential entropy of the matched planes' Gaussian, 0.5 (DOF (1 + log 2 pi) + log det cov) (:230-238)
    float calcEntropy() {
        const Matrix6f cov = getCovMat();
        double A[36];
        for (int i = 0; i < 36; ++i) A[i] = cov.data()[i];
        return float(0.5 * (6 * (1 + std::log(2 * 3.14159265359)) + std::log(float(det6(A)))));
    }
    // tracking quality from the matched-area ratio (:526-540): 0 GOOD (>= 0.7), 1 WEAK (>= 0.3), 2 BAD
    int trackingScore(float& score) {
        score = getAreaMatched() / areaSource;
        if (score >= 0.7) return 0;
        if (score >= 0.3) return 1;
        return 2;
    }
    std::map<unsigned, unsigned> getMatchedPlanes() { if (!done_) RegisterPbMap(); return bestMatch_; }
    float getAreaMatched() { if (!done_) RegisterPbMap(); return areaMatched_; }
    // Register(): PbMap -> rotOffset conjugation -> alignFrames360 -> back (OdometryKeyFrame360.cpp:205-254);
    // guess is used when the PbMap stage fails.  Returns true when the PbMap stage succeeded.
    bool Register(Frame360* frame1, Frame360* frame2, const r360_icp_params& icp, Matrix4f& pose,
                  const Matrix4f& guess = Matrix4f::Identity(), size_t max_match_planes = 25,
                  registrationType registMode = PLANAR_3DoF) {
        r360_icp_stats st;
        check(r360_ctx_set_match_params(ctx().get(), &match_), "matcher thresholds");
        const int rc = check(r360_register(ctx().get(), frame1->get(), frame2->get(), guess.data(), &icp,
                                           max_match_planes, registMode, pose.data(), informationM_.data(), &st),
                             "Register");
        return rc == 0;
    }
    // RegisterDensePhotoICP (RegisterRGBD360.h:344-520): frame2's 8 sensor images aligned to frame1's, the
    // Jacobians in the rig frame (calcPhotoICPError_robot / calcHessianGradient_robot).  As in the reference,
    // rigidTransf = pose_estim and informationM = the last level's Hessian; false = ILL-POSED.
    bool RegisterDensePhotoICP(Frame360* frame1, Frame360* frame2, Matrix4f pose_estim = Matrix4f::Identity(),
                               RegisterPhotoICP::costFuncType method = RegisterPhotoICP::PHOTO_CONSISTENCY,
                               registrationType registMode = DEFAULT_6DoF) {
        check(r360_frame_build(frame1->get(), R360_BUILD_SENSOR_PYRAMID), "setTargetFrame (sensor pyramids)");
        check(r360_frame_build(frame2->get(), R360_BUILD_SENSOR_PYRAMID), "setSourceFrame (sensor pyramids)");
        const int rc = check(r360_register_dense(ctx().get(), frame1->get(), frame2->get(), pose_estim.data(), method,
                                                 registMode, nullptr, rigidTransf_.data(), informationM_.data(),
                                                 &dense_st_),
                             "RegisterDensePhotoICP");
        done_ = true;                   // bRegistrationDone (:509)
        return rc == 1;
    }
    const r360_dense_stats& denseStats() const { return dense_st_; }
    float areaSource = 0.f, areaTarget = 0.f;
  private:
    void init() {
        std::memset(informationM_.data(), 0, sizeof(float) * 36);
        r360_match_params_default(&match_);
        if (!config_.empty()) check(r360_match_params_load_ini(config_.c_str(), &match_), "load_params");
    }
    Context& ctx() const { return ctx_ ? *ctx_ : default_context(); }
    r360_dense_stats dense_st_{};
    Context* ctx_ = nullptr;            // null: the calling thread's default context
    std::string config_;
    Frame360* ref_ = nullptr;
    Frame360* trg_ = nullptr;
    size_t max_ = 0;
    int mode_ = DEFAULT_6DoF;
    bool done_ = false;
    Matrix4f rigidTransf_;
    Matrix6f informationM_;
    std::map<unsigned, unsigned> bestMatch_;
    float areaMatched_ = 0.f;
    r360_match_params match_{};
    // 6x6 inverse / determinant by Gaussian elimination with partial pivoting (double)
    static double det6(double A[36]) {
        double d = 1.0;
        for (int k = 0; k < 6; ++k) {
            int p = k;
            for (int r = k + 1; r < 6; ++r) if (std::fabs(A[r * 6 + k]) > std::fabs(A[p * 6 + k])) p = r;
            if (A[p * 6 + k] == 0) return 0.0;
            if (p != k) { for (int c = 0; c < 6; ++c) std::swap(A[k * 6 + c], A[p * 6 + c]); d = -d; }
            d *= A[k * 6 + k];
            for (int r = k + 1; r < 6; ++r) {
                const double f = A[r * 6 + k] / A[k * 6 + k];
                for (int c = k; c < 6; ++c) A[r * 6 + c] -= f * A[k * 6 + c];
            }
        }
        return d;
    }
    static Matrix6f inverse6(const Matrix6f& M) {
        double A[6][12];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 12; ++c) A[r][c] = c < 6 ? M(r, c) : (c - 6 == r ? 1.0 : 0.0);
        for (int k = 0; k < 6; ++k) {
            int p = k;
            for (int r = k + 1; r < 6; ++r) if (std::fabs(A[r][k]) > std::fabs(A[p][k])) p = r;
            for (int c = 0; c < 12; ++c) std::swap(A[k][c], A[p][c]);
            const double piv = A[k][k];
            for (int c = 0; c < 12; ++c) A[k][c] /= piv;
            for (int r = 0; r < 6; ++r)
                if (r != k) { const double f = A[r][k]; for (int c = 0; c < 12; ++c) A[r][c] -= f * A[k][c]; }
        }
        Matrix6f out;
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) out(r, c) = float(A[r][c + 6]);
        return out;
    }
};

// ------------------------------------------------------------------ batched registrations (§8f-4)
// Worker lanes (own HIP streams and ICP state) run the pairs of one call concurrently; each pair is the
// single-pair code path, so results equal sequential RegisterRGBD360 / RegisterPhotoICP calls.
class BatchRegistration {
  public:
    BatchRegistration(int device = 0, int lanes = 8) { check(r360_batch_create(device, lanes, &h_), "r360_batch_create"); }
    // the matcher thresholds of every lane (e.g. RegisterRGBD360::matchParams() of an ini file)
    void setMatchParams(const r360_match_params& m) { check(r360_batch_set_match_params(h_, &m), "setMatchParams"); }
    ~BatchRegistration() { r360_batch_destroy(h_); }
    BatchRegistration(const BatchRegistration&) = delete;
    BatchRegistration& operator=(const BatchRegistration&) = delete;
    // generic jobs: RegisterPbMap(ref, trg) and the dense stage each job asks for (R360_JOB_*)
    std::vector<r360_pair_result> registerPairs(const std::vector<r360_pair_job>& jobs, size_t max_match_planes,
                                                RegisterRGBD360::registrationType mode, const r360_icp_params* icp,
                                                int min_matches = 0, float min_area = 0.f) {
        std::vector<r360_pair_result> out(jobs.size());
        check(r360_batch_register(h_, jobs.data(), int(jobs.size()), max_match_planes, mode, min_matches, min_area,
                                  icp, out.data()),
              "registerPairs");
        return out;
    }
    // SphereGraphSLAM tracking step: keyframes oldest first; returns the index of the keyframe the sequential
    // loop registers against (-1: "No registration available"), its result in *winner
    int track(const std::vector<Frame360*>& keyframes, Frame360* frame, r360_pair_result* winner = nullptr,
              int numCheckRegistration = 5, int noAssoc_threshold = 40, size_t max_match_planes = 25,
              RegisterRGBD360::registrationType mode = RegisterRGBD360::PLANAR_ODOMETRY_3DoF) {
        std::vector<r360_frame*> kf;
        for (auto f : keyframes) kf.push_back(f->get());
        int chosen = -1;
        check(r360_track_frame(h_, kf.data(), int(kf.size()), frame->get(), numCheckRegistration, noAssoc_threshold,
                               max_match_planes, mode, &chosen, winner, nullptr),
              "track");
        return chosen;
    }
    // LoopClosure360 candidate checks: RegisterPbMap PLANAR_3DoF, gate n_match > minMatchesThreshold and
    // area_matched > areaThreshold (LoopClosure360.h:114-115), then alignFrames360 (keyframe as source,
    // :309-313) of the pairs that pass
    std::vector<r360_pair_result> loopClosures(const std::vector<std::pair<Frame360*, Frame360*> >& pairs,
                                               const r360_icp_params& icp, int minMatchesThreshold = 5,
                                               float areaThreshold = 15.f) {
        std::vector<r360_pair_job> jobs(pairs.size());
        for (size_t i = 0; i < pairs.size(); ++i) {
            std::memset(&jobs[i], 0, sizeof(r360_pair_job));
            jobs[i].ref = pairs[i].first->get();
            jobs[i].trg = pairs[i].second->get();
            jobs[i].dense = R360_JOB_GATED;
            jobs[i].ref_is_source = 1;
        }
        return registerPairs(jobs, 25, RegisterRGBD360::PLANAR_3DoF, &icp, minMatchesThreshold, areaThreshold);
    }
    r360_batch* get() const { return h_; }
  private:
    r360_batch* h_ = nullptr;
};

}  // namespace r360
