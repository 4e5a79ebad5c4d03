// pbmap.cpp — host side of the plane half of librgbd360_hip.so:
//   * plane-buffer allocation and the device->host hand-over of the segmentation (plane_seg.hip)
//   * Frame360::getPlanesSensor descriptors (include/Frame360.h:940-1075), groupPlanes / mergePlanes
//     (:657-832) — sequential, per-plane work on a few dozen planes, so it stays on the host
//   * RegisterRGBD360::setReference/setTarget (RegisterRGBD360.h:111-196), RegisterPbMap (:276-337)
//     with the interpretation tree on unary/binary tables computed by k_match_tables (plane_match.hip)
//     and the ConsistencyTest pose/information estimate
//   * the Register() alias of OdometryKeyFrame360.cpp:248-254 (PbMap -> rotOffset conjugation ->
//     alignFrames360)
// The MRPT-pbmap definitions (hull, descriptors, same-plane tests, matcher, consistency) are the ones
// documented in DESIGN.md §PbMap; the oracle (oracle/src/pbmap_oracle.cpp) restates them independently.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <zlib.h>
#include <set>
#include <vector>

#include "../r360_internal.h"


int launch_match_tables(r360_ctx* ctx, hipStream_t stream, const float* d_desc, int ns, int nt, int mode,
                        uint8_t* d_unary, unsigned long long* d_bin, int words);

namespace {

struct P3 {
    float x = 0, y = 0, z = 0;
    float at(int k) const { return k == 0 ? x : (k == 1 ? y : z); }
};
inline float dot(const P3& a, const P3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline P3 minus(const P3& a, const P3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float norm2(const P3& a) { return dot(a, a); }
inline P3 affine(const float* T, const P3& p) {
    return {T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12], T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13],
            T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14]};
}
inline P3 linear(const float* T, const P3& p) {
    return {T[0] * p.x + T[4] * p.y + T[8] * p.z, T[1] * p.x + T[5] * p.y + T[9] * p.z, T[2] * p.x + T[6] * p.y + T[10] * p.z};
}

struct HPlane {
    P3 normal, center, ppal;
    float d = 0, area = 0, elongation = 1, curvature = 0;
    float nrgb[3] = {0, 0, 0};
    float intensity = 0;
    int id = 0, sensor = 0;
    std::string label;      // Plane::label (set by the labelization tools, kept by savePlanes)
    std::vector<P3> hull;   // closed polygon
    r360p::Moments st;
};

int axis_of(const P3& n) {
    int k0 = (std::fabs(n.at(0)) > std::fabs(n.at(1))) ? 0 : 1;
    return (std::fabs(n.at(k0)) > std::fabs(n.at(2))) ? k0 : 2;
}

// calcConvexHull: monotone chain on the two coordinates orthogonal to the dominant normal axis.  The points are
// ordered by (a, b, tie), tie = the point's rank in the reference's input order (its position in the contour, its
// voxel index in VoxelGrid's output), which only decides between points of equal (a, b).
struct HullPt { float x, y; long long tie; P3 p; };
// (x, y) as one unsigned key whose integer order is the floats' order (x major; -0 taken as +0, as the float
// comparison does; no NaN reaches the hull)
inline uint32_t ord_bits(float v) {
    uint32_t u;
    v = v + 0.0f;   // -0 -> +0
    std::memcpy(&u, &v, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
void convex_hull_of(HPlane& pl, std::vector<HullPt>& q) {
    pl.hull.clear();
    const int n = int(q.size());
    if (!n) return;
    // sorted by (x, y, tie) through integer keys (round 6: the comparator on the floats was 0.19 ms of a frame's
    // assembly for ~4.8k points)
    struct K { uint64_t k; long long tie; int i; };
    static thread_local std::vector<K> ks;
    static thread_local std::vector<int> ord;
    ks.resize(n);
    for (int i = 0; i < n; ++i) ks[i] = {(uint64_t)ord_bits(q[i].x) << 32 | ord_bits(q[i].y), q[i].tie, i};
    std::sort(ks.begin(), ks.end(), [](const K& u, const K& v) { return u.k < v.k || (u.k == v.k && u.tie < v.tie); });
    ord.resize(n);
    for (int i = 0; i < n; ++i) ord[i] = ks[i].i;
    auto turn = [&](int o, int p, int r) {
        const HullPt &O = q[ord[o]], &Pp = q[ord[p]], &Rr = q[ord[r]];
        const double ox = O.x, oy = O.y;
        return ((double)Pp.x - ox) * ((double)Rr.y - oy) - ((double)Pp.y - oy) * ((double)Rr.x - ox);
    };
    static thread_local std::vector<int> chain;   // positions in the sorted order
    chain.clear();
    chain.reserve(2 * n + 1);
    for (int i = 0; i < n; ++i) {           // lower hull
        while (chain.size() >= 2 && turn(chain[chain.size() - 2], chain.back(), i) <= 0) chain.pop_back();
        chain.push_back(i);
    }
    const size_t lower = chain.size() + 1;
    for (int i = n - 2; i >= 0; --i) {      // upper hull
        while (chain.size() >= lower && turn(chain[chain.size() - 2], chain.back(), i) <= 0) chain.pop_back();
        chain.push_back(i);
    }
    pl.hull.reserve(chain.size());
    for (int c : chain) pl.hull.push_back(q[ord[c]].p);
}

void convex_hull(HPlane& pl, const std::vector<P3>& pts) {
    const int k0 = axis_of(pl.normal), a = (k0 + 1) % 3, b = (k0 + 2) % 3;
    static thread_local std::vector<HullPt> q;
    q.resize(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) q[i] = {pts[i].at(a), pts[i].at(b), (long long)i, pts[i]};
    convex_hull_of(pl, q);
}

// The hull's input is prefiltered on the device (plane_seg.hip k_hullpre, the Akl-Toussaint octagon test that ran here
// until round 6): only the points not strictly inside the octagon of the extreme points in 8 directions reach the host.

// computeMassCenterAndArea
void area_and_center(HPlane& pl) {
    const int k0 = axis_of(pl.normal), k1 = (k0 + 1) % 3, k2 = (k0 + 2) % 3;
    const float ct = std::fabs(pl.normal.at(k0));
    float twice = 0.0f;
    float mc[3] = {0, 0, 0};
    const size_t n = pl.hull.size();
    for (size_t i = 0; i < n; i++) {
        const P3& p = pl.hull[i];
        const P3& q = pl.hull[(i + 1) % n];
        const double cs = p.at(k1) * q.at(k2) - p.at(k2) * q.at(k1);
        twice += cs;
        mc[k1] += (p.at(k1) + q.at(k1)) * cs;
        mc[k2] += (p.at(k2) + q.at(k2)) * cs;
    }
    pl.area = std::fabs(twice) / (2 * ct);
    mc[k1] /= (3 * twice);
    mc[k2] /= (3 * twice);
    const float nc = dot(pl.normal, pl.center);
    mc[k0] = (nc - pl.normal.at(k1) * mc[k1] - pl.normal.at(k2) * mc[k2]) / pl.normal.at(k0);
    pl.center = {mc[0], mc[1], mc[2]};
    pl.d = -dot(pl.normal, pl.center);
}

// symmetric 3x3 eigen-decomposition (cyclic Jacobi), eigenvalues descending, V columns
void sym_eigen3(const double Ain[9], double ev[3], double V[9]) {
    double A[9];
    memcpy(A, Ain, sizeof A);
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    static const int PQ[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int sweep = 0; sweep < 32; ++sweep) {
        if (A[1] * A[1] + A[2] * A[2] + A[5] * A[5] < 1e-300) break;
        for (const auto& pq : PQ) {
            const int p = pq[0], q = pq[1];
            const double apq = A[p * 3 + q];
            if (apq == 0.0) continue;
            const double th = (A[q * 3 + q] - A[p * 3 + p]) / (2.0 * apq);
            const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
            const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {
                const double x = A[k * 3 + p], y = A[k * 3 + q];
                A[k * 3 + p] = c * x - s * y;
                A[k * 3 + q] = s * x + c * y;
            }
            for (int k = 0; k < 3; ++k) {
                const double x = A[p * 3 + k], y = A[q * 3 + k];
                A[p * 3 + k] = c * x - s * y;
                A[q * 3 + k] = s * x + c * y;
            }
            for (int k = 0; k < 3; ++k) {
                const double x = V[k * 3 + p], y = V[k * 3 + q];
                V[k * 3 + p] = c * x - s * y;
                V[k * 3 + q] = s * x + c * y;
            }
        }
    }
    int o[3] = {0, 1, 2};
    const double dg[3] = {A[0], A[4], A[8]};
    std::sort(o, o + 3, [&](int u, int v) { return dg[u] > dg[v] || (dg[u] == dg[v] && u < v); });
    double W[9];
    for (int j = 0; j < 3; ++j) {
        ev[j] = dg[o[j]];
        for (int k = 0; k < 3; ++k) W[k * 3 + j] = V[k * 3 + o[j]];
    }
    memcpy(V, W, sizeof W);
}

// calcElongationAndPpalDir + calcMainColor2 from the exact inlier statistics
void descriptors(HPlane& pl) {
    double mean[3], cov[9];
    r360p::moments_mean_cov(pl.st, mean, cov);
    double ev[3], V[9];
    sym_eigen3(cov, ev, V);
    pl.elongation = float(std::sqrt(ev[0] / ev[1]));
    pl.ppal = {float(V[0]), float(V[3]), float(V[6])};
    const double dn = (double)pl.st.n;
    for (int k = 0; k < 3; ++k) pl.nrgb[k] = float(((double)pl.st.c[k] * 1.1641532182693481e-10) / dn);
    pl.intensity = float((double)pl.st.c[3] / (3.0 * dn));
}

// MRPT dist3D_Segment_to_Segment2
float seg_dist2(const P3& a0, const P3& a1, const P3& b0, const P3& b1) {
    const float SMALL = 0.00000001f;
    const P3 u = minus(a1, a0), v = minus(b1, b0), w = minus(a0, b0);
    const float a = dot(u, u), b = dot(u, v), c = dot(v, v), d = dot(u, w), e = dot(v, w);
    const float D = a * c - b * b;
    float sN, sD = D, tN, tD = D;
    if (D < SMALL) {
        sN = 0.0f; sD = 1.0f; tN = e; tD = c;
    } else {
        sN = (b * e - c * d);
        tN = (a * e - b * d);
        if (sN < 0.0f) { sN = 0.0f; tN = e; tD = c; }
        else if (sN > sD) { sN = sD; tN = e + b; tD = c; }
    }
    if (tN < 0.0f) {
        tN = 0.0f;
        if (-d < 0.0f) sN = 0.0f;
        else if (-d > a) sN = sD;
        else { sN = -d; sD = a; }
    } else if (tN > tD) {
        tN = tD;
        if ((-d + b) < 0.0f) sN = 0;
        else if ((-d + b) > a) sN = sD;
        else { sN = (-d + b); sD = a; }
    }
    const float sc = (std::fabs(sN) < SMALL ? 0.0f : sN / sD);
    const float tc = (std::fabs(tN) < SMALL ? 0.0f : tN / tD);
    const P3 dp = {w.x + (sc * u.x) - (tc * v.x), w.y + (sc * u.y) - (tc * v.y), w.z + (sc * u.z) - (tc * v.z)};
    return dot(dp, dp);
}

// Conservative early-out of the O(|A| |B|) proximity tests below: the distance between the axis-aligned boxes of the
// two point sets (hull vertices and centre) bounds every vertex / vertex and segment / segment distance they compute
// from below (the segment points are convex combinations of the vertices), up to float rounding of a few 1e-6 m on
// coordinates of tens of metres.  Boxes farther apart than the threshold + 1e-4 m therefore give `false` exactly as
// the full loops do, without them (ADVICE / VERDICT r5: host assembly per frame).
struct Box { float lo[3], hi[3]; };
Box box_of(const HPlane& A) {
    Box b;
    for (int k = 0; k < 3; ++k) b.lo[k] = b.hi[k] = A.center.at(k);
    for (const P3& v : A.hull)
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = std::min(b.lo[k], v.at(k));
            b.hi[k] = std::max(b.hi[k], v.at(k));
        }
    return b;
}
bool boxes_apart(const HPlane& A, const HPlane& B, float thr) {
    const Box a = box_of(A), b = box_of(B);
    double g2 = 0;
    for (int k = 0; k < 3; ++k) {
        const double g = std::max({0.0, (double)b.lo[k] - a.hi[k], (double)a.lo[k] - b.hi[k]});
        g2 += g * g;
    }
    const double lim = (double)thr + 1e-4;
    return g2 > lim * lim;
}

// The same bound per segment pair: segments whose boxes are farther apart than lim (threshold + 1e-4 m) have no pair
// of points within the threshold, so their seg_dist2 could not pass the test (round 6: most segment pairs of two
// neighbouring planes that do not touch)
bool segs_apart(const P3& a0, const P3& a1, const P3& b0, const P3& b1, double lim2) {
    double g2 = 0;
    for (int k = 0; k < 3; ++k) {
        const float alo = std::min(a0.at(k), a1.at(k)), ahi = std::max(a0.at(k), a1.at(k));
        const float blo = std::min(b0.at(k), b1.at(k)), bhi = std::max(b0.at(k), b1.at(k));
        const double g = std::max({0.0, (double)blo - ahi, (double)alo - bhi});
        g2 += g * g;
    }
    return g2 > lim2;
}

bool nearby(const HPlane& A, const HPlane& B, float thr) {
    if (boxes_apart(A, B, thr)) return false;
    const float t2 = thr * thr;
    if (norm2(minus(A.center, B.center)) < t2) return true;
    for (size_t i = 1; i < A.hull.size(); i++)
        if (norm2(minus(A.hull[i], B.center)) < t2) return true;
    for (size_t j = 1; j < B.hull.size(); j++)
        if (norm2(minus(A.center, B.hull[j])) < t2) return true;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t j = 1; j < B.hull.size(); j++)
            if (norm2(minus(A.hull[i], B.hull[j])) < t2) return true;
    const double lim = (double)thr + 1e-4, lim2 = lim * lim;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t j = 1; j < B.hull.size(); j++)
            if (!segs_apart(A.hull[i], A.hull[i - 1], B.hull[j], B.hull[j - 1], lim2) &&
                seg_dist2(A.hull[i], A.hull[i - 1], B.hull[j], B.hull[j - 1]) < t2)
                return true;
    return false;
}

bool same_plane(const HPlane& A, const HPlane& B, float cos_angle, float dist, float prox) {
    if (dot(A.normal, B.normal) < cos_angle) return false;
    if (std::fabs(dot(A.normal, minus(B.center, A.center))) > dist) return false;
    return nearby(A, B, prox);
}

// mergePlane2
void merge_into(HPlane& A, const HPlane& B) {
    const P3 n = {A.area * A.normal.x + B.area * B.normal.x, A.area * A.normal.y + B.area * B.normal.y,
                  A.area * A.normal.z + B.area * B.normal.z};
    const float len = std::sqrt(dot(n, n));
    A.normal = {n.x / len, n.y / len, n.z / len};
    std::vector<P3> pts(A.hull);
    pts.insert(pts.end(), B.hull.begin(), B.hull.end());
    convex_hull(A, pts);
    r360p::moments_merge(A.st, B.st);
    area_and_center(A);
    A.d = -dot(A.normal, A.center);
    descriptors(A);
}

const float kMaxCurvature = 0.0013f;   // include/Miscellaneous.h:54
const float kMinArea = 0.12f;          // :57
const float kMaxElongation = 6.0f;     // :60

bool hulls_touch(const HPlane& A, const HPlane& B, float max_dist, float max_normal_off) {
    // the vertex/vertex then segment/segment tests of groupPlanes (:774-808) and mergePlanes (:671-703)
    if (boxes_apart(A, B, max_dist)) return false;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t ii = 1; ii < B.hull.size(); ii++) {
            const P3 diff = minus(A.hull[i], B.hull[ii]);
            if (std::sqrt(norm2(diff)) < max_dist && std::fabs(dot(A.normal, diff)) < max_normal_off) return true;
        }
    const double lim = (double)max_dist + 1e-4, lim2 = lim * lim;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t ii = 1; ii < B.hull.size(); ii++) {
            if (segs_apart(A.hull[i], A.hull[i - 1], B.hull[ii], B.hull[ii - 1], lim2)) continue;
            const float dist = std::sqrt(seg_dist2(A.hull[i], A.hull[i - 1], B.hull[ii], B.hull[ii - 1]));
            if (dist < max_dist) {
                const P3 diff = minus(A.hull[i], B.hull[ii]);
                if (std::fabs(dot(A.normal, diff)) < max_normal_off) return true;
            }
        }
    return false;
}

}  // namespace

struct PbMapHost {
    std::vector<HPlane> planes;
};

// ------------------------------------------------------------------ buffers
int plane_bufs_alloc(r360_frame* f) {
    PlaneBufs& P = f->pl;
    if (P.cloud) return 0;
    P.w = f->cols / 2;
    P.h = f->rows / 2;
    const long N = (long)P.w * P.h, T = 8 * N;
    const long sw = (P.w - 1) / 10 + 5, sh = (P.h - 1) / 10 + 5;
    P.sd_max = 208;
    P.grid_cells = sw * sh * P.sd_max;
    R360_HIP(hipMalloc(&P.cloud, sizeof(float4) * T));
    R360_HIP(hipMalloc(&P.rgb, sizeof(uchar4) * T));
    R360_HIP(hipMalloc(&P.nrm, sizeof(float4) * T));
    R360_HIP(hipMalloc(&P.dist0, sizeof(float) * T));
    R360_HIP(hipMalloc(&P.dist, sizeof(float) * T));
    R360_HIP(hipMalloc(&P.grids, sizeof(float2) * 16 * P.grid_cells));
    R360_HIP(hipMalloc(&P.zmm, sizeof(int) * 16));
    R360_HIP(hipMalloc(&P.parent, sizeof(int) * T));
    R360_HIP(hipMalloc(&P.root, sizeof(int) * T));
    R360_HIP(hipMalloc(&P.lab, sizeof(int) * T));
    R360_HIP(hipMalloc(&P.labf, sizeof(int) * T));
    R360_HIP(hipMalloc(&P.cnt, sizeof(int) * T));
    R360_HIP(hipMalloc(&P.aux, sizeof(int) * 8 * R360_MAX_BIG));
    R360_HIP(hipMalloc(&P.chunk, sizeof(int) * 8 * ((N + 255) / 256)));
    R360_HIP(hipMalloc(&P.gpart, sizeof(RegionPart) * R360_GM_COPIES * 8 * R360_MAX_MODELS));
    R360_HIP(hipMalloc(&P.nlab, sizeof(int) * 8));
    R360_HIP(hipMalloc(&P.big, sizeof(int) * 8 * R360_MAX_BIG));
    R360_HIP(hipMalloc(&P.nbig, sizeof(int) * 8));
    R360_HIP(hipMalloc(&P.mom, sizeof(r360p::Moments) * 8 * R360_MAX_BIG));
    R360_HIP(hipMalloc(&P.models, sizeof(PlaneModel) * 8 * R360_MAX_MODELS));
    R360_HIP(hipMalloc(&P.nmodels, sizeof(int) * 8));
    R360_HIP(hipMalloc(&P.state, T));
    R360_HIP(hipMalloc(&P.state2, T));
    R360_HIP(hipMalloc(&P.rbnd, 8L * R360_REFINE_BANDS * P.w));
    R360_HIP(hipMalloc(&P.rflag, sizeof(int) * 8 * R360_REFINE_BANDS));
    R360_HIP(hipMalloc(&P.mask, sizeof(unsigned long long) * T));
    const long SK = 8L * (P.w + P.h - 1) * P.h;
    R360_HIP(hipMalloc(&P.rcode, sizeof(uint16_t) * SK));
    R360_HIP(hipMalloc(&P.rmsk, sizeof(unsigned long long) * SK));
    R360_HIP(hipMalloc(&P.rf1, SK));
    R360_HIP(hipMalloc(&P.rf2, SK));
    R360_HIP(hipMalloc(&P.out, sizeof(PlaneOut) * 8 * R360_MAX_MODELS));
    P.contour_cap = 2 * T;
    P.vox_cap = T;
    // the contour and voxel outputs are written by the kernels straight into pinned host memory (a
    // few hundred KB per frame), so the host assembly needs no second device->host copy
    R360_HIP(hipHostMalloc(&P.contour, sizeof(float4) * P.contour_cap));
    R360_HIP(hipMalloc(&P.contour_dev, sizeof(float4) * P.contour_cap));
    R360_HIP(hipHostMalloc(&P.vox, sizeof(VoxOut) * P.vox_cap));
    R360_HIP(hipMalloc(&P.vox_dev, sizeof(VoxOut) * P.vox_cap));
    R360_HIP(hipEventCreateWithFlags(&P.done, hipEventDisableTiming | hipEventBlockingSync));
    R360_HIP(hipEventCreateWithFlags(&P.ready, hipEventDisableTiming));
    R360_HIP(hipMalloc(&P.totals, sizeof(long) * 4));
    R360_HIP(hipMalloc(&P.err, sizeof(int)));
    R360_HIP(hipHostMalloc(&P.h_out, sizeof(PlaneOut) * 8 * R360_MAX_MODELS));
    R360_HIP(hipHostMalloc(&P.h_nmodels, sizeof(int) * 16));
    return 0;
}

void plane_bufs_free(r360_frame* f) {
    PlaneBufs& P = f->pl;
    planes_join(f);
    void* dev[] = {P.cloud, P.rgb, P.nrm, P.dist0, P.dist, P.grids, P.zmm, P.parent, P.root, P.lab, P.labf, P.cnt, P.gpart, P.aux, P.chunk, P.nlab,
                   P.big, P.nbig, P.mom, P.models, P.nmodels, P.state, P.state2, P.rbnd, P.rflag, P.mask, P.rcode, P.rmsk, P.rf1, P.rf2, P.out, P.totals, P.err, P.vox_dev, P.contour_dev};
    for (void* p : dev) hipFree(p);
    hipHostFree(P.contour);
    hipHostFree(P.vox);
    hipHostFree(P.h_out);
    hipHostFree(P.h_nmodels);
    if (P.done) hipEventDestroy(P.done);
    if (P.ready) hipEventDestroy(P.ready);
    P = PlaneBufs();
    delete f->pbmap;
    f->pbmap = nullptr;
}

int ctx_vhash_reserve(r360_ctx* ctx, long min_cells, long list_entries, long list_groups) {
    if (ctx->vlist_cap < list_entries || ctx->vcnt_cap < list_groups) {
        hipFree(ctx->d_vlist);
        hipFree(ctx->d_vcnt);
        ctx->d_vlist = nullptr;
        ctx->d_vcnt = nullptr;
        R360_HIP(hipMalloc(&ctx->d_vlist, sizeof(int) * list_entries));
        R360_HIP(hipMalloc(&ctx->d_vcnt, sizeof(int) * list_groups));
        ctx->vlist_cap = list_entries;
        ctx->vcnt_cap = list_groups;
    }
    long cap = 1;
    while (cap < min_cells) cap <<= 1;
    if (ctx->vhash_cap >= cap) return 0;
    hipFree(ctx->d_vhash);
    ctx->d_vhash = nullptr;
    R360_HIP(hipMalloc(&ctx->d_vhash, sizeof(VoxCell) * cap));
    // zero once: k_vox_compact leaves every cell it used zero again (stream order: before the frame's kernels)
    R360_HIP(hipMemsetAsync(ctx->d_vhash, 0, sizeof(VoxCell) * cap, ctx->stream));
    ctx->vhash_cap = cap;
    return 0;
}

int vox_slot_reserve(VoxSlot& s, const PlaneGeom& G, hipStream_t st) {
    long cells, entries, groups;
    vox_scratch_need(G, &cells, &entries, &groups);
    VoxScratch& v = s.v;
    if (s.entries < entries || s.groups < groups) {
        hipFree(v.vlist);
        hipFree(v.vcnt);
        v.vlist = nullptr;
        v.vcnt = nullptr;
        s.entries = s.groups = 0;
        R360_HIP(hipMalloc(&v.vlist, sizeof(int) * entries));
        R360_HIP(hipMalloc(&v.vcnt, sizeof(int) * groups));
        s.entries = entries;
        s.groups = groups;
    }
    long cap = 1;
    while (cap < cells) cap <<= 1;
    if (s.cells < cap) {
        hipFree(v.vhash);
        v.vhash = nullptr;
        s.cells = 0;
        v.cap = 0;
        R360_HIP(hipMalloc(&v.vhash, sizeof(VoxCell) * cap));
        // zeroed once: k_vox_compact leaves every cell it used zero again
        R360_HIP(hipMemsetAsync(v.vhash, 0, sizeof(VoxCell) * cap, st));
        s.cells = cap;
        v.cap = (unsigned long long)cap;
    }
    return 0;
}

void vox_slot_free(VoxSlot& s) {
    hipFree(s.v.vhash);
    hipFree(s.v.vlist);
    hipFree(s.v.vcnt);
    s = VoxSlot();
}

PlaneGeom plane_geom(const r360_frame* f) {
    const PlaneBufs& P = f->pl;
    return PlaneGeom{f->rows, f->cols, P.w, P.h, P.sd_max, P.grid_cells};
}

PlaneDev plane_dev(const r360_frame* f, const VoxScratch& vs) {
    const PlaneBufs& P = f->pl;
    PlaneDev D;
    D.depth_m = f->d_depth_m; D.bgr = f->d_bgr;
    D.cloud = P.cloud; D.rgb = P.rgb; D.nrm = P.nrm; D.dist0 = P.dist0; D.dist = P.dist; D.grids = P.grids; D.zmm = P.zmm;
    D.parent = P.parent; D.root = P.root; D.lab = P.lab; D.labf = P.labf; D.cnt = P.cnt; D.aux = P.aux; D.chunk = P.chunk;
    D.nlab = P.nlab; D.big = P.big; D.nbig = P.nbig; D.mom = P.mom; D.models = P.models; D.nmodels = P.nmodels;
    D.state = P.state; D.state2 = P.state2; D.mask = P.mask; D.rbnd = P.rbnd; D.rflag = P.rflag;
    D.rcode = P.rcode; D.rmsk = P.rmsk; D.rf1 = P.rf1; D.rf2 = P.rf2;
    D.out = P.out; D.gpart = P.gpart; D.contour = P.contour; D.contour_dev = P.contour_dev; D.vox = P.vox; D.vox_dev = P.vox_dev; D.totals = P.totals; D.err = P.err;
    D.h_out = P.h_out; D.h_nmodels = P.h_nmodels; D.rt = f->calib->d_rt;
    D.vhash = vs.vhash; D.vlist = vs.vlist; D.vcnt = vs.vcnt;
    D.contour_cap = P.contour_cap; D.vox_cap = P.vox_cap; D.vhash_cap = vs.cap;
    return D;
}

// the chain of the plane stage (cloud, filter, normals, segmentation, refinement, descriptors' statistics, contours,
// voxel fallback, publication into the frames' pinned host buffers) for F frames of the same size
int planes_launch(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx,
                  const hipEvent_t* bgr_ev) {
    // k_plane_begin (first kernel of launch_cloud_normals) zeroes the error word
    if (launch_cloud_normals(B, F, G, st, tctx)) return -1;
    if (launch_segmentation(B, F, G, st, tctx, bgr_ev)) return -1;
    return launch_plane_publish(B, F, st);
}


// One part of a lone frame's plane stage as a graph (0: cloud, filter, normals, segmentation, refinement; 1: colours,
// statistics, contours, voxels, hull prefilter, publication), captured on first use for the frame's buffers and
// geometry and replayed after: ~40 launches become two, so the stage no longer waits for the host to enqueue it
// behind a split upload's depth copy.  The kernels and their arguments are those planes_launch enqueues.  Captured on
// the ctx's capture stream, not on ctx->stream: an event recorded on a capturing stream cannot be queried, and the
// assembly pool polls the previous frame's `done` event (recorded on ctx->stream) while this frame is captured.
static int plane_graph_launch(r360_ctx* ctx, const PlaneBatch& B, const PlaneGeom& G, int part) {
    std::string key(reinterpret_cast<const char*>(&B.f[0]), sizeof(PlaneDev));
    const long gk[7] = {G.rows, G.cols, G.w, G.h, G.sd_max, G.grid_cells, part};
    key.append(reinterpret_cast<const char*>(gk), sizeof gk);
    ++ctx->graph_clock;
    for (auto& g : ctx->plane_graphs)
        if (g.key == key) {
            g.used = ctx->graph_clock;
            R360_HIP(hipGraphLaunch(g.exec, ctx->stream));
            return 0;
        }
    hipGraph_t graph = nullptr;
    hipStream_t cs = capture_stream(ctx);   // not ctx->stream: the pool polls events recorded there
    if (!cs) return -1;
    R360_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
    const int rc = part == 0 ? (launch_cloud_normals(B, 1, G, cs, nullptr) ? -1 : launch_segmentation_geom(B, 1, G, cs, nullptr))
                             : (launch_segmentation_model(B, 1, G, cs, nullptr) ? -1 : launch_plane_publish(B, 1, cs));
    const hipError_t ec = hipStreamEndCapture(cs, &graph);
    if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
    R360_HIP(ec);
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    R360_HIP(ei);
    constexpr size_t kMaxGraphs = 8;   // two parts for each of a few rotating frame buffers
    if (ctx->plane_graphs.size() >= kMaxGraphs) {
        size_t lru = 0;
        for (size_t i = 1; i < ctx->plane_graphs.size(); ++i)
            if (ctx->plane_graphs[i].used < ctx->plane_graphs[lru].used) lru = i;
        R360_HIP(hipStreamSynchronize(ctx->stream));   // the evicted graph may still be running
        (void)hipGraphExecDestroy(ctx->plane_graphs[lru].exec);
        ctx->plane_graphs.erase(ctx->plane_graphs.begin() + (long)lru);
    }
    ctx->plane_graphs.push_back({std::move(key), exec, ctx->graph_clock});
    R360_HIP(hipGraphLaunch(exec, ctx->stream));
    return 0;
}

// GPU part of getPlanes: cloud, filter, normals, segmentation — enqueued on the frame's ctx stream, or submitted to
// the ctx's plane queue (batched with other frames on the queue's stream)
int planes_enqueue(r360_frame* f) {
    if (plane_bufs_alloc(f)) return -1;
    planes_join(f);
    PlaneBufs& P = f->pl;
    P.ticket.reset();
    if (f->ctx->plane_q) {
        if (plane_queue_submit(f->ctx->plane_q, f)) return -1;
        return planes_spawn_assembly(f);
    }
    const PlaneGeom G = plane_geom(f);
    long cells, entries, groups;
    vox_scratch_need(G, &cells, &entries, &groups);
    r360_ctx* ctx = f->ctx;
    if (ctx_vhash_reserve(ctx, cells, entries, groups)) return -1;
    PlaneBatch B;   // a batch of one (kernel arguments, copied at each launch)
    std::memset(&B, 0, sizeof B);
    B.f[0] = plane_dev(f, VoxScratch{ctx->d_vhash, (unsigned long long)ctx->vhash_cap, ctx->d_vlist, ctx->d_vcnt});
    // experiment builds: R360_NO_PLANE_GRAPH=1 launches a split-upload context's stage kernel by kernel (A/B)
    static const bool no_graph = R360_KNOB("R360_NO_PLANE_GRAPH", 0) != 0;
    if (ctx->split_upload && !ctx->timing && !no_graph) {
        if (plane_graph_launch(ctx, B, G, 0)) return -1;
        if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(ctx->stream, e, 0));
        if (plane_graph_launch(ctx, B, G, 1)) return -1;
    } else {
        const hipEvent_t bev = f->bgr_wait();
        if (planes_launch(B, 1, G, ctx->stream, ctx, &bev)) return -1;
    }
    R360_HIP(hipEventRecord(P.done, f->ctx->stream));
    return planes_spawn_assembly(f);
}

// Frame360::getPlanes of n frames (Frame360.h:615-640) with their plane stages batched: frames of one size go up to
// R360_PLANE_BATCH per launch of the chain, on the stream of frames[0]'s context, each after its own undistortion
// (on its own stream).  The other stages (stitch, pyramids) run on each frame's own stream as r360_frame_build would.
// Every frame's results equal its lone build's.
extern "C" int r360_frames_build(r360_frame* const* frames, int n, unsigned flags) {
    CHECK_ARG(frames && n >= 1, "frames_build: need at least one frame");
    for (int i = 0; i < n; ++i) {
        CHECK_ARG(frames[i], "frames_build: null frame");
        CHECK_ARG(frames[i]->ctx->device == frames[0]->ctx->device, "frames_build: frames of different devices");
        CHECK_ARG(frames[i]->rows > 0 || flags == 0, "a sphere-only frame has no sensor images to build from");
        for (int j = 0; j < i; ++j) CHECK_ARG(frames[j] != frames[i], "frames_build: a frame is listed twice");
    }
    const unsigned plane_flags = R360_BUILD_CLOUD | R360_BUILD_PLANES;
    if (!(flags & plane_flags)) {
        for (int i = 0; i < n; ++i)
            if (int rc = r360_frame_build(frames[i], flags)) return rc;
        return 0;
    }
    r360_ctx* H = frames[0]->ctx;
    if (bind_device(H->device)) return -1;
    for (int i = 0; i < n; ++i)
        if (int rc = r360_frame_build_async(frames[i], R360_BUILD_UNDISTORT)) return rc;
    if ((int)H->bvox.size() < R360_PLANE_BATCH - 1) H->bvox.resize(R360_PLANE_BATCH - 1);
    for (int i = 0; i < n; ++i)
        if (plane_bufs_alloc(frames[i])) return -1;
    std::vector<char> taken(n, 0);
    for (int i0 = 0; i0 < n; ++i0) {
        if (taken[i0]) continue;
        // the next batch: frame i0 and the following frames of its size, up to R360_PLANE_BATCH
        const PlaneGeom G = plane_geom(frames[i0]);
        std::vector<r360_frame*> bf;
        for (int i = i0; i < n && (int)bf.size() < R360_PLANE_BATCH; ++i) {
            const PlaneGeom g = plane_geom(frames[i]);
            if (taken[i] || g.rows != G.rows || g.cols != G.cols || g.w != G.w || g.h != G.h ||
                g.sd_max != G.sd_max || g.grid_cells != G.grid_cells)
                continue;
            taken[i] = 1;
            bf.push_back(frames[i]);
        }
        PlaneBatch B;
        std::memset(&B, 0, sizeof B);
        long cells, entries, groups;
        vox_scratch_need(G, &cells, &entries, &groups);
        if (ctx_vhash_reserve(H, cells, entries, groups)) return -1;
        for (int j = 0; j < (int)bf.size(); ++j) {
            r360_frame* f = bf[j];
            planes_join(f);   // a previous build's assembly still reading the buffers
            f->pl.ticket.reset();
            R360_HIP(hipEventRecord(f->pl.ready, f->ctx->stream));
            R360_HIP(hipStreamWaitEvent(H->stream, f->pl.ready, 0));
            VoxScratch vs{H->d_vhash, (unsigned long long)H->vhash_cap, H->d_vlist, H->d_vcnt};
            if (j > 0) {
                if (vox_slot_reserve(H->bvox[j - 1], G, H->stream)) return -1;
                vs = H->bvox[j - 1].v;
            }
            B.f[j] = plane_dev(f, vs);
        }
        std::vector<hipEvent_t> bev;
        for (r360_frame* f : bf) bev.push_back(f->bgr_wait());
        if (planes_launch(B, (int)bf.size(), G, H->stream, H, bev.data())) return -1;
        for (r360_frame* f : bf) {
            R360_HIP(hipEventRecord(f->pl.done, H->stream));
            if (planes_spawn_assembly(f)) return -1;
            f->built |= R360_BUILD_UNDISTORT | plane_flags;
            delete f->sphere_cloud;   // a cloud set by loadCloud is replaced by the built one
            f->sphere_cloud = nullptr;
        }
    }
    const unsigned rest = flags & ~(R360_BUILD_UNDISTORT | plane_flags);
    for (int i = 0; i < n; ++i)
        if (rest)
            if (int rc = r360_frame_build_async(frames[i], rest)) return rc;
    for (int i = 0; i < n; ++i) {
        if (int rc = planes_finish(frames[i])) return rc;
        R360_HIP(hipStreamSynchronize(frames[i]->ctx->stream));
    }
    return 0;
}

// Host PbMap assembly (A8 + A9: planes_assemble) of the frames whose plane stage is on the GPU, by a persistent pool
// (round 6; a thread per frame before).  One watcher thread sweeps the pending frames in submission order every ~50 us:
// a frame is ready once its plane-queue ticket says its batch is enqueued and its `done` event has completed.  Ready
// frames go to R360_ASM_WORKERS worker threads that sleep on a condition variable.  The per-frame threads each polled
// their event (5 / 20 / 100 us sleeps over the several milliseconds a batched plane stage takes: ~100 wake-ups and
// event queries per frame) and were created and joined per frame; the bench counted 2.04 host cores in them at 1603
// pairs/s.  The pool is created on first use and lives until the process exits.
// R360_PBMAP_PROFILE (experiment builds): per-phase times (us) and sizes of one sensor's assembly
struct AsmProf;
static void planes_assemble_sensor(r360_frame* f, int s, std::vector<HPlane>& local, AsmProf* pf);
static int planes_assemble_group(r360_frame* f, std::vector<std::vector<HPlane>>& local, const AsmProf* pf,
                                 double sensors_us);
static int planes_capacity_ok(r360_frame* f);
struct AsmProf { double pre = 0, hull = 0, desc = 0, local = 0; long in = 0, kept = 0, hullv = 0, models = 0, vox = 0; };

namespace {
constexpr int R360_ASM_WORKERS = 7;   // with a joining thread, one per sensor of a lone frame

// one frame's assembly in flight: its 8 sensor tasks run on any workers; the one that finishes last groups them
struct AsmWork {
    r360_frame* f;
    std::vector<std::vector<HPlane>> local = std::vector<std::vector<HPlane>>(8);
    AsmProf prof[8];
    std::atomic<int> left{8};
    std::atomic<long> ns{0};
    std::chrono::steady_clock::time_point t0;
};

struct AsmPool {
    std::mutex m;
    std::condition_variable cv_watch, cv_work, cv_done;
    std::deque<r360_frame*> pending;
    std::deque<std::pair<AsmWork*, int>> ready;   // (frame, sensor) tasks
    std::vector<std::thread> th;   // never joined: the pool outlives every frame (the process's lifetime)
    long assembled = 0;
};

void asm_finish(AsmPool& A, r360_frame* f, int rc, const std::string& err) {   // under A.m
    f->pl.worker_rc = rc;
    f->pl.worker_err = err;
    f->pl.asm_busy = false;
    ++A.assembled;
}

// Per-sensor tasks (round 6): a frame's sensors are assembled by up to all workers at once and the last one groups
// them, so one frame's assembly takes about a quarter of its CPU time in wall time (the sequential callers wait for
// it; the pipelined runner only gets its PbMaps sooner).  Runs one task taken off A->ready (by a worker or a joining
// thread, planes_join); the thread that completes the frame's last sensor groups them and finishes the frame.
void asm_run(AsmPool* A, const std::pair<AsmWork*, int>& t) {
    AsmWork* W = t.first;
    const auto a0 = std::chrono::steady_clock::now();
    planes_assemble_sensor(W->f, t.second, W->local[t.second], &W->prof[t.second]);
    W->ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - a0).count();
    if (W->left.fetch_sub(1) != 1) return;
    const auto g0 = std::chrono::steady_clock::now();
    const int rc = planes_assemble_group(W->f, W->local,  W->prof,
                                         std::chrono::duration<double, std::micro>(g0 - W->t0).count());
    const std::string err = rc ? std::string(r360_last_error()) : std::string();
    W->ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - g0).count();
    {
        std::lock_guard<std::mutex> lk(A->m);
        W->f->ctx->host_ns[4] += W->ns.load();
        W->f->ctx->host_ns[5] += 1;
        asm_finish(*A, W->f, rc, err);
    }
    delete W;
    A->cv_done.notify_all();
}

void asm_worker(AsmPool* A) {
    for (;;) {
        std::pair<AsmWork*, int> t;
        {
            std::unique_lock<std::mutex> lk(A->m);
            A->cv_work.wait(lk, [&] { return !A->ready.empty(); });
            t = A->ready.front();
            A->ready.pop_front();
        }
        asm_run(A, t);
    }
}

// 1: the frame's GPU part is complete, 0: not yet, -1: it failed (err)
int asm_poll(r360_frame* f, std::string& err) {
    PlaneBufs& P = f->pl;
    if (P.ticket) {
        const int t = plane_ticket_poll(P.ticket, &err);   // the plane queue has not recorded `done` before this
        if (t <= 0) {
            if (t < 0) err = "plane build: " + err;
            return t;
        }
    }
    const hipError_t r = hipEventQuery(P.done);
    if (r == hipSuccess) return 1;
    if (r == hipErrorNotReady) return 0;
    err = "plane build: GPU work failed";
    return -1;
}

// a frame taken off A->pending whose GPU part has ended (st > 0) or failed: its sensor tasks go to A->ready, or it
// finishes with the error.  Under A->m; returns false if the frame failed (the caller notifies cv_done).
bool asm_dispatch(AsmPool* A, r360_frame* f, int st, const std::string& err) {
    if (st > 0 && planes_capacity_ok(f) == 0) {
        auto* W = new AsmWork;
        W->f = f;
        W->t0 = std::chrono::steady_clock::now();
        // heaviest sensors first (hull candidates + a per-plane constant): the frame's wall time is its longest
        // chain of tasks, and the sensors' loads differ several-fold
        const PlaneBufs& P = f->pl;
        int order[8];
        long wt[8];
        for (int s = 0; s < 8; ++s) {
            order[s] = s;
            wt[s] = 0;
            for (int m = 0; m < P.h_nmodels[s]; ++m) wt[s] += P.h_out[s * R360_MAX_MODELS + m].hull_n + 32;
        }
        std::stable_sort(order, order + 8, [&](int a, int b) { return wt[a] > wt[b]; });
        for (int s : order) A->ready.push_back({W, s});
        return true;
    }
    asm_finish(*A, f, -1, st > 0 ? std::string(r360_last_error()) : err);
    return false;
}

void asm_watcher(AsmPool* A) {
    std::vector<r360_frame*> snap;
    std::vector<std::pair<r360_frame*, int>> fin;
    std::vector<std::string> errs;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(A->m);
            A->cv_watch.wait(lk, [&] { return !A->pending.empty(); });
            snap.assign(A->pending.begin(), A->pending.end());
        }
        fin.clear();
        errs.clear();
        for (r360_frame* f : snap) {
            std::string err;
            const int st = asm_poll(f, err);
            if (st != 0) {
                fin.push_back({f, st});
                errs.push_back(err);
            }
        }
        if (fin.empty()) {
            std::this_thread::sleep_for(std::chrono::microseconds(50));
            continue;
        }
        bool failed = false;
        {
            std::lock_guard<std::mutex> lk(A->m);
            for (size_t k = 0; k < fin.size(); ++k) {
                auto it = std::find(A->pending.begin(), A->pending.end(), fin[k].first);
                if (it == A->pending.end()) continue;   // a joining thread took it meanwhile (planes_join)
                A->pending.erase(it);
                failed = !asm_dispatch(A, fin[k].first, fin[k].second, errs[k]) || failed;
            }
        }
        A->cv_work.notify_all();
        if (failed) A->cv_done.notify_all();
    }
}

AsmPool& asm_pool() {
    static AsmPool* A = [] {
        auto* p = new AsmPool;
        p->th.emplace_back(asm_watcher, p);
        for (int k = 0; k < R360_ASM_WORKERS; ++k) p->th.emplace_back(asm_worker, p);
        return p;
    }();
    return *A;
}
}  // namespace

// the frame's host assembly, queued behind its GPU part (the caller has joined any earlier one: planes_enqueue)
int planes_spawn_assembly(r360_frame* f) {
    PlaneBufs& P = f->pl;
    delete f->pbmap;
    f->pbmap = nullptr;
    AsmPool& A = asm_pool();
    {
        std::lock_guard<std::mutex> lk(A.m);
        P.worker_rc = 0;
        P.worker_err.clear();
        P.asm_busy = true;
        A.pending.push_back(f);
    }
    A.cv_watch.notify_one();
    return 0;
}

// Waits until the frame's queued assembly (if any) has finished; any number of threads may wait for one frame.  With
// the frame's ctx->join_help (default) the waiting thread does not leave the frame to the pool's 50 us sweeps and
// wake-ups: it polls the frame's GPU part itself (yielding between queries), dispatches its sensor tasks the moment
// it has ended and runs them beside the workers, so a lone frame's PbMap is ready ~0.1 ms sooner (the sequential
// caller's critical path).  Which thread runs a task does not change its result.
void planes_join(r360_frame* f) {
    PlaneBufs& P = f->pl;
    if (!P.cloud) return;   // never built planes: nothing was queued
    AsmPool& A = asm_pool();
    std::unique_lock<std::mutex> lk(A.m);
    if (f->ctx && f->ctx->join_help) {
        while (P.asm_busy) {
            if (std::find(A.pending.begin(), A.pending.end(), f) != A.pending.end()) {
                lk.unlock();
                std::string err;
                int st;
                while ((st = asm_poll(f, err)) == 0) std::this_thread::yield();
                lk.lock();
                auto it = std::find(A.pending.begin(), A.pending.end(), f);
                if (it == A.pending.end()) continue;   // the watcher took it meanwhile
                A.pending.erase(it);
                const bool ok = asm_dispatch(&A, f, st, err);
                lk.unlock();
                A.cv_work.notify_all();
                if (!ok) A.cv_done.notify_all();
                lk.lock();
                continue;
            }
            auto t = std::find_if(A.ready.begin(), A.ready.end(),
                                  [&](const std::pair<AsmWork*, int>& x) { return x.first->f == f; });
            if (t != A.ready.end()) {
                const std::pair<AsmWork*, int> task = *t;
                A.ready.erase(t);
                lk.unlock();
                asm_run(&A, task);
                lk.lock();
                continue;
            }
            A.cv_done.wait(lk, [&] { return !P.asm_busy; });   // its last tasks run on workers
        }
        return;
    }
    A.cv_done.wait(lk, [&] { return !P.asm_busy; });
}

// Host part of getPlanes: waits for the assembly thread
int planes_finish(r360_frame* f) {
    PlaneBufs& P = f->pl;
    if (!P.cloud && f->pbmap) return 0;   // PbMap loaded from a file (loadPbMap)
    if (!P.cloud) { r360_set_error("planes were not built (R360_BUILD_PLANES)"); return -2; }
    planes_join(f);
    if (P.worker_rc) { r360_set_error("%s", P.worker_err.c_str()); return P.worker_rc; }
    if (!f->pbmap) { r360_set_error("planes were not built (R360_BUILD_PLANES)"); return -2; }
    return 0;
}

// Per-plane host part of getPlanes (A8 + A9), run by the assembly pool once the GPU part (including the pinned
// contour / voxel outputs) is complete: the per-sensor part (getPlanesSensor's hull, area, descriptors, transform and
// same-plane merges, Frame360.h:940-1075) sensor by sensor as independent tasks, then groupPlanes / mergePlanes
// (:657-832) over the sensors' planes.
namespace {
std::chrono::steady_clock::time_point asm_now() { return std::chrono::steady_clock::now(); }
double asm_us(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}
}  // namespace

// the frame's segmentation stayed within the kernels' capacities (else the error, with its code)
static int planes_capacity_ok(r360_frame* f) {
    const int err = f->pl.h_nmodels[8];
    if (!err) return 0;
    r360_set_error("plane segmentation capacity exceeded (code %d: 1 bilateral depth range, 2 labels, 4 models, "
                   "8 contour length, 16 pools)", err);
    return -1;
}

// sensor s's planes (A8) into `local`, independent of the other sensors
static void planes_assemble_sensor(r360_frame* f, int s, std::vector<HPlane>& local, AsmProf* pf) {
    PlaneBufs& P = f->pl;
    static const bool prof = R360_KNOB_STR("R360_PBMAP_PROFILE") != nullptr;
    const float4* contour = P.contour;
    const VoxOut* vox = P.vox;
    static thread_local std::vector<HullPt> hq;
    auto tick = [&](double& acc, std::chrono::steady_clock::time_point& t) {
        if (!prof) return;
        const auto u = asm_now();
        acc += asm_us(t, u);
        t = u;
    };
    const float* Rt = f->calib->rt[s];
    local.clear();
    for (int m = 0; m < P.h_nmodels[s]; ++m) {
        const PlaneOut& O = P.h_out[s * R360_MAX_MODELS + m];
        HPlane pl;
        pl.sensor = s;
        pl.center = {O.model.centroid[0], O.model.centroid[1], O.model.centroid[2]};
        pl.normal = {O.model.v[0], O.model.v[1], O.model.v[2]};
        if (dot(pl.normal, pl.center) > 0) pl.normal = {-pl.normal.x, -pl.normal.y, -pl.normal.z};  // :988-992
        pl.curvature = O.model.curvature;
        pl.st = O.stats;
        const int ax = axis_of(pl.normal), ha = (ax + 1) % 3, hb = (ax + 2) % 3;
        auto tq = prof ? asm_now() : std::chrono::steady_clock::time_point{};
        if (prof) { ++pf->models; pf->in += O.n_contour > 0 ? O.n_contour : O.n_vox; pf->vox += O.n_contour > 0 ? 0 : O.n_vox; }
        // the hull's input: the contour in trace order, or ("HULL 000", :1017-1026) the VoxelGrid centroids from
        // k_vox_* ranked by voxel index (PCL's output order); only the prefilter's survivors, with that rank
        // (both lists arrive prefiltered by k_hullpre: hull_n candidates of the n_contour / n_vox points)
        const bool cont = O.n_contour > 0;
        const int n = O.hull_n;
        const float4* c = contour + O.contour_off;
        const VoxOut* v0 = vox + O.vox_off;
        auto get = [&](int k) { return cont ? P3{c[k].x, c[k].y, c[k].z} : P3{v0[k].x, v0[k].y, v0[k].z}; };
        hq.resize(n);
        for (int k = 0; k < n; ++k) {
            const P3 q = get(k);
            hq[k] = {q.at(ha), q.at(hb), cont ? (long long)k : v0[k].key, q};
        }
        tick(pf->pre, tq);
        if (prof) pf->kept += (long)hq.size();
        convex_hull_of(pl, hq);
        if (prof) pf->hullv += (long)pl.hull.size();
        tick(pf->hull, tq);
        area_and_center(pl);
        if (pl.area < kMinArea) continue;                           // :1034
        pl.d = -dot(pl.normal, pl.center);                          // :1037
        descriptors(pl);
        tick(pf->desc, tq);
        if (pl.elongation > kMaxElongation) continue;               // :1041
        pl.normal = linear(Rt, pl.normal);                          // transform(Rt) :1051
        pl.center = affine(Rt, pl.center);
        pl.d = -dot(pl.normal, pl.center);
        for (P3& v : pl.hull) v = affine(Rt, v);
        bool merged = false;
        if (pl.curvature < kMaxCurvature)
            for (HPlane& q : local)
                if (q.curvature < kMaxCurvature && same_plane(q, pl, 0.99f, 0.05f, 0.2f)) {
                    merge_into(q, pl);
                    merged = true;
                    break;
                }
        if (!merged) {
            pl.id = int(local.size());
            local.push_back(pl);
        }
        tick(pf->local, tq);
    }
}

// groupPlanes (:742-832) and mergePlanes (:657-739) over the sensors' planes: the frame's PbMap.  pf (profile runs):
// the sensors' phase times, sensors_us the wall time from the first sensor task's start
static int planes_assemble_group(r360_frame* f, std::vector<std::vector<HPlane>>& local, const AsmProf* pf,
                                 double sensors_us) {
    static const bool prof = R360_KNOB_STR("R360_PBMAP_PROFILE") != nullptr;
    const auto t3 = asm_now();
    auto* pm = new PbMapHost;
    std::vector<HPlane>& G = pm->planes;
    G = local[0];
    std::set<unsigned> first, prev;
    for (const HPlane& p : G) first.insert(unsigned(p.id));
    prev = first;
    for (int s = 1; s < 8; ++s) {
        std::set<unsigned> next;
        for (HPlane& L : local[s]) {
            bool same = false;
            size_t j = 0;
            if (L.area > 0.5f || L.curvature < kMaxCurvature)
                for (auto it = prev.begin(); it != prev.end() && !same; ++it) {
                    j = *it;
                    if (G[j].area < 0.5f || G[j].curvature > kMaxCurvature) continue;
                    if (std::fabs(G[j].d - L.d) < 0.45f && dot(G[j].normal, L.normal) > 0.99f)
                        same = hulls_touch(G[j], L, 0.5f, 0.09f);
                }
            if (same) {
                next.insert(unsigned(G[j].id));
                merge_into(G[j], L);
            } else {
                next.insert(unsigned(G.size()));
                L.id = int(G.size());
                G.push_back(L);
            }
        }
        prev = next;
        if (s == 6) prev.insert(first.begin(), first.end());
    }
    const auto t4 = asm_now();
    // mergePlanes (:657-739)
    for (size_t j = 0; j < G.size(); j++) {
        if (!(G[j].curvature < kMaxCurvature)) continue;
        for (size_t k = j + 1; k < G.size(); k++) {
            if (!(G[k].curvature < kMaxCurvature)) continue;
            bool same = false;
            if (dot(G[j].normal, G[k].normal) > 0.99f && std::fabs(G[j].d - G[k].d) < 0.45f)
                same = hulls_touch(G[j], G[k], 0.3f, 0.06f);
            if (same) {
                merge_into(G[j], G[k]);
                for (size_t hh = k + 1; hh < G.size(); hh++) --G[hh].id;
                G.erase(G.begin() + long(k));
                j--;
                break;
            }
        }
    }
    f->pbmap = pm;
    if (prof && pf) {
        AsmProf t;
        for (int s = 0; s < 8; ++s) {
            t.pre += pf[s].pre; t.hull += pf[s].hull; t.desc += pf[s].desc; t.local += pf[s].local;
            t.in += pf[s].in; t.kept += pf[s].kept; t.hullv += pf[s].hullv; t.models += pf[s].models; t.vox += pf[s].vox;
        }
        const long* totals = reinterpret_cast<const long*>(f->pl.h_nmodels + 10);
        fprintf(stderr, "[pbmap] pools %ld+%ld pts (voxel table %ld cells, bound %ld) | sensors %.0f us: prefilter %.0f, "
                "hull %.0f, area+desc %.0f, local merges %.0f | groupPlanes %.0f us, mergePlanes %.0f us | models %ld, "
                "points %ld (voxels %ld) -> %ld kept -> %ld hull vertices, planes %zu\n", totals[0], totals[1],
                totals[2] + 1, totals[3], sensors_us, t.pre, t.hull, t.desc, t.local, asm_us(t3, t4),
                asm_us(t4, asm_now()), t.models, t.in, t.vox, t.kept, t.hullv, G.size());
    }
    return 0;
}

// the whole assembly on the calling thread
int planes_assemble(r360_frame* f) {
    if (planes_capacity_ok(f)) return -1;
    std::vector<std::vector<HPlane>> local(8);
    AsmProf pf[8];
    const auto t0 = asm_now();
    for (int s = 0; s < 8; ++s) planes_assemble_sensor(f, s, local[s], &pf[s]);
    return planes_assemble_group(f, local, pf, asm_us(t0, asm_now()));
}

// ------------------------------------------------------------------ RegisterRGBD360
namespace {

// setReference / setTarget (RegisterRGBD360.h:111-196); labels are never set on this path
std::vector<int> subgraph(const std::vector<HPlane>& P, size_t max_match_planes) {
    std::vector<int> ids;
    if (max_match_planes > 0 && P.size() > max_match_planes) {
        std::vector<float> areas(P.size(), 0.f);
        for (size_t i = 0; i < P.size(); i++)
            if (P[i].curvature < kMaxCurvature) areas[i] = P[i].area;
        std::vector<float> sorted(areas);
        std::sort(sorted.begin(), sorted.end());
        const float thr = sorted[P.size() - max_match_planes - 1];
        for (size_t i = 0; i < P.size(); i++)
            if (areas[i] > thr) ids.push_back(P[i].id);
    } else {
        for (size_t i = 0; i < P.size(); i++)
            if (P[i].curvature < kMaxCurvature) ids.push_back(P[i].id);
    }
    std::sort(ids.begin(), ids.end());
    return ids;
}

void pack_desc(const HPlane& p, float* d) {
    const float v[16] = {p.normal.x, p.normal.y, p.normal.z, p.center.x, p.center.y, p.center.z, p.d, p.area,
                         p.elongation, p.nrgb[0], p.nrgb[1], p.nrgb[2], p.intensity, 0, 0, 0};
    memcpy(d, v, sizeof v);
}

struct Tables {
    int ns = 0, nt = 0, words = 0;
    const uint8_t* unary = nullptr;
    const unsigned long long* bin = nullptr;
    bool pair_ok(int i, int j, int k, int l) const {
        const int bit = k * nt + l;
        return (bin[(size_t)(i * nt + j) * words + bit / 64] >> (bit % 64)) & 1;
    }
};

int gpu_tables(r360_ctx* ctx, const std::vector<HPlane>& S, const std::vector<int>& si, const std::vector<HPlane>& T,
               const std::vector<int>& ti, int mode, Tables& tb) {
    const int ns = int(si.size()), nt = int(ti.size());
    const int cap = std::max(ns, nt);
    if (cap > ctx->match_cap) {
        hipFree(ctx->d_match_desc); hipFree(ctx->d_unary); hipFree(ctx->d_bin);
        hipHostFree(ctx->h_unary); hipHostFree(ctx->h_bin);
        ctx->match_cap = std::max(cap, 32);
        const size_t c = ctx->match_cap, np = c * c, words = (np + 63) / 64;
        R360_HIP(hipMalloc(&ctx->d_match_desc, sizeof(float) * 16 * 2 * c));
        R360_HIP(hipMalloc(&ctx->d_unary, np));
        R360_HIP(hipMalloc(&ctx->d_bin, sizeof(unsigned long long) * np * words));
        R360_HIP(hipHostMalloc(&ctx->h_unary, np));
        R360_HIP(hipHostMalloc(&ctx->h_bin, sizeof(unsigned long long) * np * words));
    }
    tb.ns = ns; tb.nt = nt;
    tb.words = (ns * nt + 63) / 64;
    tb.unary = ctx->h_unary;
    tb.bin = ctx->h_bin;
    if (ns == 0 || nt == 0) return 0;
    std::vector<float> desc(16 * (size_t)(ns + nt));
    for (int i = 0; i < ns; ++i) pack_desc(S[si[i]], &desc[16 * i]);
    for (int j = 0; j < nt; ++j) pack_desc(T[ti[j]], &desc[16 * (ns + j)]);
    if (!ctx->mstream) {
        // one stream per device at the highest priority, shared by every context: a few microseconds of work that
        // the calling thread waits for, which at normal priority queued for milliseconds behind the dense queue's
        // launches (2.4 ms per call in the default bench, profiles/r3_host).  Shared, not one per context: a
        // second stream per pipeline would take more hardware queues than GPU_MAX_HW_QUEUES provides.
        static std::mutex m;
        static hipStream_t dev_stream[64] = {};
        std::lock_guard<std::mutex> lk(m);
        if (ctx->device < 0 || ctx->device >= 64) { r360_set_error("device ordinal out of range"); return -2; }
        if (!dev_stream[ctx->device]) {
            int least = 0, greatest = 0;
            R360_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
            R360_HIP(hipStreamCreateWithPriority(&dev_stream[ctx->device], hipStreamNonBlocking, greatest));
        }
        ctx->mstream = dev_stream[ctx->device];
        R360_HIP(hipEventCreateWithFlags(&ctx->mwait_ev, hipEventDisableTiming | hipEventBlockingSync));
    }
    hipStream_t st = ctx->mstream;
    R360_HIP(hipMemcpyAsync(ctx->d_match_desc, desc.data(), sizeof(float) * desc.size(), hipMemcpyHostToDevice, st));
    // the kernel writes the tables straight into the pinned host buffers (no device-to-host copies)
    if (launch_match_tables(ctx, st, ctx->d_match_desc, ns, nt, mode, ctx->h_unary, ctx->h_bin, tb.words)) return -1;
    R360_HIP(hipEventRecord(ctx->mwait_ev, st));
    return event_wait(ctx->mwait_ev);
}

// interpretation tree: depth-first over reference planes (targets ascending, then "no match"); the largest consistent
// set wins, ties by matched reference area, the first one found in that order among equals.  Forward checking: each
// reference plane below the current depth keeps its domain, the targets still consistent (unary, distinct, binary)
// with every assignment above it, so a branch is cut as soon as the planes that can still match cannot beat the best
// set.  Every cut is sound (an upper bound on what the branch can add), so the result is the exhaustive search's;
// the node budget (r360_match_params::max_nodes) only guards against pathological inputs, and a search that
// reaches it is counted (r360_ctx_match_stats) instead of passing silently.
struct Tree {
    const Tables* tb = nullptr;
    std::vector<double> area;
    int W = 1;                            // 64-bit words per target set
    // forward-check rows, built on first use: fc_at[k * nt + l] = offset in fc of the row of assignment k -> l, whose
    // [i][W] words are the targets t of reference i consistent with it.  A search visits a small part of the ns x nt
    // assignments, so rows are appended as they are needed (an eager ns * nt * ns * W table was 256 MB at 200 planes)
    std::vector<uint64_t> fc;
    std::vector<uint32_t> fc_at;
    std::vector<uint64_t> dom;            // [depth][ns][W] domains at each depth
    std::vector<int> cur, best;
    int ns = 0, nt = 0, n_cur = 0, n_best = 0;
    double a_cur = 0, a_best = 0;
    long nodes = 0, budget = 4000000;
    bool truncated = false;
    void init() {
        ns = tb->ns; nt = tb->nt;
        W = std::max(1, (nt + 63) / 64);
        fc.clear();
        fc_at.assign((size_t)ns * nt, UINT32_MAX);
        dom.assign((size_t)(ns + 1) * ns * W, 0);
        for (int i = 0; i < ns; ++i)
            for (int t = 0; t < nt; ++t)
                if (tb->unary[(size_t)i * nt + t]) dom[(size_t)i * W + t / 64] |= 1ull << (t % 64);
        cur.assign(ns, -1);
        best.assign(ns, -1);
    }
    // (the pointer is valid until the next fc_row call: go() reads it before recursing)
    const uint64_t* fc_row(int k, int l) {
        uint32_t& at = fc_at[(size_t)k * nt + l];
        if (at == UINT32_MAX) {
            at = (uint32_t)fc.size();
            fc.resize(fc.size() + (size_t)ns * W, 0);
            uint64_t* r = &fc[at];
            for (int i = k + 1; i < ns; ++i)
                for (int t = 0; t < nt; ++t)
                    if (t != l && tb->pair_ok(i, t, k, l)) r[(size_t)i * W + t / 64] |= 1ull << (t % 64);
        }
        return &fc[at];
    }
    void go(int i) {
        if (++nodes > budget) { truncated = true; return; }
        if (i == ns) {
            if (n_cur > n_best || (n_cur == n_best && a_cur > a_best)) { best = cur; n_best = n_cur; a_best = a_cur; }
            return;
        }
        const uint64_t* D = &dom[(size_t)i * ns * W];   // domains of references i..ns-1 at this depth
        // references with a non-empty domain, and the distinct targets those domains hold, both bound the matches
        // still possible (a reference takes one target, a target one reference)
        int left = 0, targets = 0;
        double rest = 0;
        for (int w = 0; w < W; ++w) {
            uint64_t any = 0;
            for (int r = i; r < ns; ++r) any |= D[(size_t)r * W + w];
            targets += __builtin_popcountll(any);
        }
        for (int r = i; r < ns; ++r) {
            bool any = false;
            for (int w = 0; w < W; ++w) any = any || D[(size_t)r * W + w] != 0;
            if (any) { ++left; rest += area[r]; }
        }
        left = std::min(left, targets);
        if (n_cur + left < n_best) return;
        if (n_cur + left == n_best && a_cur + rest <= a_best) return;
        uint64_t* Dn = &dom[(size_t)(i + 1) * ns * W];
        for (int w = 0; w < W; ++w)
            for (uint64_t m = D[(size_t)i * W + w]; m; m &= m - 1) {
                const int t = w * 64 + __builtin_ctzll(m);
                const uint64_t* F = fc_row(i, t);
                for (size_t x = (size_t)(i + 1) * W; x < (size_t)ns * W; ++x) Dn[x] = D[x] & F[x];
                cur[i] = t; ++n_cur; a_cur += area[i];
                go(i + 1);
                cur[i] = -1; --n_cur; a_cur -= area[i];
                if (truncated) return;
            }
        for (size_t x = (size_t)(i + 1) * W; x < (size_t)ns * W; ++x) Dn[x] = D[x];
        go(i + 1);
    }
};

double det33(const double A[9]) {
    return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) + A[2] * (A[3] * A[7] - A[4] * A[6]);
}

// ConsistencyTest::estimatePoseWithCovariance: Kabsch on area-weighted normals, plane-offset least
// squares for t, information blockdiag(sum w n n^T, sum w (I - n n^T)); false when ill-conditioned
bool estimate_pose(const std::vector<HPlane>& R, const std::vector<HPlane>& T, const std::map<unsigned, unsigned>& m,
                   float pose[16], float info[36]) {
    if (m.size() < 3) return false;
    double M[9] = {0}, Ht[9] = {0}, Hr[9] = {0}, g[3] = {0};
    for (const auto& kv : m) {
        const HPlane& r = R[kv.first];
        const HPlane& t = T[kv.second];
        const double w = t.area;
        const double nr[3] = {r.normal.x, r.normal.y, r.normal.z}, nt[3] = {t.normal.x, t.normal.y, t.normal.z};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                M[a * 3 + b] += w * nt[a] * nr[b];
                Ht[a * 3 + b] += w * nr[a] * nr[b];
                Hr[a * 3 + b] += w * ((a == b ? 1.0 : 0.0) - nr[a] * nr[b]);
            }
        const double e = double(t.d) - double(r.d);
        for (int a = 0; a < 3; ++a) g[a] += w * nr[a] * e;
    }
    double MtM[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += M[k * 3 + a] * M[k * 3 + b];
            MtM[a * 3 + b] = s;
        }
    double lam[3], V[9], U[9], sig[3];
    sym_eigen3(MtM, lam, V);
    for (int k = 0; k < 3; ++k) sig[k] = std::sqrt(std::max(0.0, lam[k]));
    if (!(sig[1] > 1e-6 * sig[0])) return false;
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < 3; ++a) {
            double s = 0;
            for (int b = 0; b < 3; ++b) s += M[a * 3 + b] * V[b * 3 + k];
            U[a * 3 + k] = s / sig[k];
        }
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
    double Rm[9];
    for (int pass = 0; pass < 2; ++pass) {
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += V[a * 3 + k] * U[b * 3 + k];
                Rm[a * 3 + b] = s;
            }
        if (det33(Rm) > 0) break;
        for (int a = 0; a < 3; ++a) V[a * 3 + 2] = -V[a * 3 + 2];
    }
    double lt[3], Vt[9];
    sym_eigen3(Ht, lt, Vt);
    if (!(lt[2] > 0) || lt[0] / lt[2] > 8000.0) return false;   // threshold_conditioning (Miscellaneous.h:76)
    double t[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k) {
        double proj = 0;
        for (int a = 0; a < 3; ++a) proj += Vt[a * 3 + k] * g[a];
        for (int a = 0; a < 3; ++a) t[a] += Vt[a * 3 + k] * proj / lt[k];
    }
    for (int i = 0; i < 16; ++i) pose[i] = (i % 5 == 0) ? 1.f : 0.f;
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) pose[b * 4 + a] = float(Rm[a * 3 + b]);
        pose[12 + a] = float(t[a]);
    }
    for (int i = 0; i < 36; ++i) info[i] = 0.f;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            info[b * 6 + a] = float(Ht[a * 3 + b]);
            info[(b + 3) * 6 + (a + 3)] = float(Hr[a * 3 + b]);
        }
    return true;
}

int ready(r360_frame* f) {
    if (!f) { r360_set_error("null frame"); return -2; }
    if (!(f->built & R360_BUILD_PLANES)) { r360_set_error("frame planes not built (R360_BUILD_PLANES)"); return -2; }
    return planes_finish(f);
}

}  // namespace

// The interpretation tree alone over given tables (host only, no device): best[i] = target of reference i or -1.
// Returns 1 when the node budget stopped the search, 0 when it ran to the end.
extern "C" int r360_match_tree_search(int ns, int nt, const uint8_t* unary, const uint64_t* binary, int words,
                                      const double* area, long max_nodes, int* best, long* nodes) {
    CHECK_ARG(ns >= 0 && nt >= 0 && (ns == 0 || (unary && area && best)) && max_nodes > 0, "bad arguments");
    // the tables' index arithmetic is 32-bit (ns * nt pairs, each a row of ns * nt bits)
    CHECK_ARG(ns <= 1024 && nt <= 1024, "at most 1024 reference and 1024 target planes");
    CHECK_ARG(words == (ns * nt + 63) / 64 && (ns * nt == 0 || binary), "binary table: words != ceil(ns * nt / 64)");
    Tables tb;
    tb.ns = ns; tb.nt = nt; tb.words = words;
    tb.unary = unary;
    tb.bin = reinterpret_cast<const unsigned long long*>(binary);
    Tree tr;
    tr.tb = &tb;
    tr.budget = max_nodes;
    tr.area.assign(area, area + ns);
    tr.init();
    tr.go(0);
    for (int i = 0; i < ns; ++i) best[i] = tr.best[i];
    if (nodes) *nodes = tr.nodes;
    return tr.truncated ? 1 : 0;
}

extern "C" int r360_frame_get_planes(r360_frame* f, r360_plane* out, int cap, int* n) {
    if (int rc = ready(f)) return rc;
    const auto& P = f->pbmap->planes;
    if (n) *n = int(P.size());
    for (int i = 0; i < int(P.size()) && i < cap && out; ++i) {
        const HPlane& p = P[i];
        r360_plane& o = out[i];
        const P3* src[3] = {&p.normal, &p.center, &p.ppal};
        float* dst[3] = {o.normal, o.center, o.ppal};
        for (int k = 0; k < 3; ++k) { dst[k][0] = src[k]->x; dst[k][1] = src[k]->y; dst[k][2] = src[k]->z; }
        o.d = p.d; o.area = p.area; o.elongation = p.elongation; o.curvature = p.curvature;
        for (int k = 0; k < 3; ++k) o.nrgb[k] = p.nrgb[k];
        o.intensity = p.intensity;
        o.id = p.id; o.sensor = p.sensor; o.n_inliers = int(p.st.n); o.n_hull = int(p.hull.size());
    }
    return 0;
}

extern "C" int r360_frame_get_plane_hull(r360_frame* f, int i, float* xyz, int cap, int* n) {
    if (int rc = ready(f)) return rc;
    const auto& P = f->pbmap->planes;
    CHECK_ARG(i >= 0 && i < int(P.size()), "plane index out of range");
    const auto& H = P[i].hull;
    if (n) *n = int(H.size());
    for (int k = 0; k < int(H.size()) && k < cap && xyz; ++k) {
        xyz[3 * k] = H[k].x; xyz[3 * k + 1] = H[k].y; xyz[3 * k + 2] = H[k].z;
    }
    return 0;
}

extern "C" int r360_pbmap_match_tables(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, size_t max_match_planes,
                                       int mode, int* ns, int* nt, int* sid, int* tid, uint8_t* unary,
                                       uint64_t* binary, int cap) {
    CHECK_ARG(ctx && ns && nt, "null arg");
    if (int rc = ready(ref)) return rc;
    if (int rc = ready(trg)) return rc;
    const auto& S = ref->pbmap->planes;
    const auto& T = trg->pbmap->planes;
    const std::vector<int> si = subgraph(S, max_match_planes), ti = subgraph(T, max_match_planes);
    *ns = int(si.size());
    *nt = int(ti.size());
    CHECK_ARG(*ns <= cap && *nt <= cap, "subgraph larger than cap");
    Tables tb;
    if (gpu_tables(ctx, S, si, T, ti, mode, tb)) return -1;
    for (int i = 0; i < *ns; ++i) if (sid) sid[i] = si[i];
    for (int j = 0; j < *nt; ++j) if (tid) tid[j] = ti[j];
    if (unary) memcpy(unary, tb.unary, (size_t)*ns * *nt);
    if (binary) memcpy(binary, tb.bin, sizeof(uint64_t) * (size_t)*ns * *nt * tb.words);
    return tb.words;
}

extern "C" int r360_register_pbmap(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, size_t max_match_planes, int mode,
                                   float pose[16], float info[36], int* match_pairs, int pair_cap, int* n_match,
                                   float* area_matched, float* area_src, float* area_trg) {
    CHECK_ARG(ctx && pose && info, "null arg");
    if (ctx && bind_device(ctx->device)) return -1;
    CHECK_ARG(mode >= 0 && mode <= 3, "registrationType must be 0..3");
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if (int rc = ready(ref)) return rc;
    if (int rc = ready(trg)) return rc;
    const auto t1 = clk::now();
    const auto& S = ref->pbmap->planes;
    const auto& T = trg->pbmap->planes;
    const std::vector<int> si = subgraph(S, max_match_planes), ti = subgraph(T, max_match_planes);
    Tables tb;
    if (gpu_tables(ctx, S, si, T, ti, mode, tb)) return -1;
    const auto t2 = clk::now();
    struct Acct {   // tree + pose time, accounted on every return path
        r360_ctx* c; clk::time_point a, b, s;
        ~Acct() {
            const auto e = clk::now();
            c->host_ns[0] += std::chrono::duration_cast<std::chrono::nanoseconds>(a - s).count();
            c->host_ns[1] += std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
            c->host_ns[2] += std::chrono::duration_cast<std::chrono::nanoseconds>(e - b).count();
            c->host_ns[3] += 1;
        }
    } acct{ctx, t1, t2, t0};
    Tree tr;
    tr.tb = &tb;
    tr.budget = ctx->match.max_nodes;
    tr.area.resize(si.size());
    for (size_t i = 0; i < si.size(); ++i) tr.area[i] = S[si[i]].area;
    tr.init();
    tr.go(0);
    ctx->match_calls.fetch_add(1, std::memory_order_relaxed);
    if (tr.truncated) ctx->match_truncated.fetch_add(1, std::memory_order_relaxed);
    for (long m = ctx->match_nodes_max.load(std::memory_order_relaxed); tr.nodes > m;)
        if (ctx->match_nodes_max.compare_exchange_weak(m, tr.nodes)) break;
    std::map<unsigned, unsigned> best;
    for (size_t i = 0; i < si.size(); ++i)
        if (tr.best[i] >= 0) best[unsigned(si[i])] = unsigned(ti[tr.best[i]]);
    int k = 0;
    float am = 0.f;
    for (const auto& kv : best) {
        if (match_pairs && k < pair_cap) { match_pairs[2 * k] = int(kv.first); match_pairs[2 * k + 1] = int(kv.second); }
        ++k;
        am += S[kv.first].area;                     // calcAreaMatched
    }
    if (n_match) *n_match = int(best.size());
    if (area_matched) *area_matched = am;
    if (best.size() < 3) return 0;                  // "Insuficient matching" (:306-310); pose untouched
    float p[16], inf[36];
    if (!estimate_pose(S, T, best, p, inf)) return 0;
    memcpy(pose, p, sizeof p);
    memcpy(info, inf, sizeof inf);
    float as = 0.f, at = 0.f;                       // :323-334
    for (int id : si) as += S[id].area;
    for (int id : ti) at += T[id].area;
    if (area_src) *area_src = as;
    if (area_trg) *area_trg = at;
    return 1;
}

// ------------------------------------------------------------------ matcher configuration
extern "C" void r360_match_params_default(r360_match_params* m) {
    if (!m) return;
    // config_files/configLocaliser_sphericalOdometry.ini ([global], [unary], [binary])
    m->min_planes_recognition = 3;
    m->dist_d = 0.5f; m->angle = 50.f; m->color_threshold = 0.07f; m->intensity_threshold = 100.f;
    m->elongation_threshold = 2.5f; m->area_threshold = 3.0f;
    m->dist_threshold = 3.0f; m->angle_threshold = 10.f; m->height_threshold = 0.33f; m->cos_angle_parallel = 0.985f;
    m->planar_normal_angle = 10.f;
    m->max_nodes = 4000000;
}

// mrpt-pbmap's config_heuristics::load_params reads the keys of [global], [unary] and [binary] with
// CConfigFile (INI: "key=value", '//' and '%' comments; keys absent from the file keep their defaults)
extern "C" int r360_match_params_load_ini(const char* path, r360_match_params* m) {
    CHECK_ARG(path && m, "null arg");
    FILE* fp = fopen(path, "r");
    if (!fp) { r360_set_error("cannot open %s", path); return -1; }
    char line[1024];
    std::string section;
    while (fgets(line, sizeof line, fp)) {
        std::string l(line);
        const size_t cpos = l.find("//");
        if (cpos != std::string::npos) l.erase(cpos);
        const size_t pct = l.find('%');
        if (pct != std::string::npos) l.erase(pct);
        auto trim = [](std::string x) {
            const size_t a = x.find_first_not_of(" \t\r\n"), b = x.find_last_not_of(" \t\r\n");
            return a == std::string::npos ? std::string() : x.substr(a, b - a + 1);
        };
        l = trim(l);
        if (l.empty()) continue;
        if (l[0] == '[') { section = trim(l.substr(1, l.find(']') - 1)); continue; }
        const size_t eq = l.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = trim(l.substr(0, eq)), v = trim(l.substr(eq + 1));
        const double x = atof(v.c_str());
        if (section == "global" && k == "min_planes_recognition") m->min_planes_recognition = (int)x;
        else if (section == "unary") {
            if (k == "dist_d") m->dist_d = (float)x;
            else if (k == "angle") m->angle = (float)x;
            else if (k == "color_threshold") m->color_threshold = (float)x;
            else if (k == "intensity_threshold") m->intensity_threshold = (float)x;
            else if (k == "elongation_threshold") m->elongation_threshold = (float)x;
            else if (k == "area_threshold") m->area_threshold = (float)x;
        } else if (section == "binary") {
            if (k == "dist_threshold") m->dist_threshold = (float)x;
            else if (k == "angle_threshold") m->angle_threshold = (float)x;
            else if (k == "height_threshold") m->height_threshold = (float)x;
            else if (k == "cos_angle_parallel") m->cos_angle_parallel = (float)x;
        }
    }
    fclose(fp);
    return 0;
}

extern "C" int r360_ctx_set_match_params(r360_ctx* ctx, const r360_match_params* m) {
    CHECK_ARG(ctx && m, "null arg");
    CHECK_ARG(m->max_nodes > 0, "max_nodes must be positive");
    ctx->match = *m;
    return 0;
}

extern "C" int r360_ctx_match_stats(r360_ctx* ctx, long* calls, long* truncated, long* max_nodes) {
    CHECK_ARG(ctx, "null ctx");
    if (calls) *calls = ctx->match_calls.load();
    if (truncated) *truncated = ctx->match_truncated.load();
    if (max_nodes) *max_nodes = ctx->match_nodes_max.load();
    return 0;
}

extern "C" int r360_ctx_get_match_params(const r360_ctx* ctx, r360_match_params* m) {
    CHECK_ARG(ctx && m, "null arg");
    *m = ctx->match;
    return 0;
}

// Register(): PbMap registration, then the dense refinement initialised with the rotOffset-conjugated
// PbMap pose (OdometryKeyFrame360.cpp:167-171, 205, 244-254).  guess = fallback initial pose in the rig
// frame when the PbMap registration fails (the caller's previous relative pose).
// rotOffset: rotation of angleOffset = 157.5 deg about x (OdometryRGBD360.cpp:138-139), column-major
void r360_rot_offset(float Ro[16], float Ri[16]) {
    const float a = 157.5f;
    const float c = (float)cos(a * R360_PI / 180), s = (float)sin(a * R360_PI / 180);
    const float o[16] = {1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1};   // (1,2) = s, (2,1) = -s
    const float t[16] = {1, 0, 0, 0, 0, c, s, 0, 0, -s, c, 0, 0, 0, 0, 1};   // inverse = transpose
    memcpy(Ro, o, sizeof o);
    memcpy(Ri, t, sizeof t);
}
void r360_mul4(const float* A, const float* B, float* C) {   // Eigen Matrix4f product order
    float out[16];
    for (int col = 0; col < 4; ++col)
        for (int r = 0; r < 4; ++r) {
            float acc = A[r] * B[col * 4];
            for (int k = 1; k < 4; ++k) acc += A[k * 4 + r] * B[col * 4 + k];
            out[col * 4 + r] = acc;
        }
    memcpy(C, out, sizeof out);
}

extern "C" int r360_register_async(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, const float guess[16],
                                   const r360_icp_params* p, size_t max_match_planes, int mode) {
    CHECK_ARG(ctx && ref && trg && p, "null arg");
    float pb[16], inf[36];
    for (int i = 0; i < 16; ++i) pb[i] = guess ? guess[i] : ((i % 5 == 0) ? 1.f : 0.f);
    for (int i = 0; i < 36; ++i) inf[i] = 0.f;
    const int good = r360_register_pbmap(ctx, ref, trg, max_match_planes, mode, pb, inf, nullptr, 0, nullptr, nullptr,
                                         nullptr, nullptr);
    if (good < 0) return good;
    float Ro[16], Ri[16], t1[16], init[16];
    r360_rot_offset(Ro, Ri);
    r360_mul4(Ro, pb, t1);
    r360_mul4(t1, Ri, init);                             // rotOffset * pose * rotOffset^-1
    if (int rc = r360_align360_async(ctx, ref, trg, init, R360_PHOTO_DEPTH, 0, p)) return rc;
    ctx->reg_pending = 1;
    ctx->reg_good = good;
    memcpy(ctx->reg_info, inf, sizeof inf);
    return 0;
}

extern "C" int r360_register_result(r360_ctx* ctx, float pose[16], float info[36], r360_icp_stats* st) {
    CHECK_ARG(ctx && ctx->reg_pending && pose, "no registration pending");
    ctx->reg_pending = 0;
    float dense[16];
    const int rc = r360_align360_result(ctx, dense, nullptr, nullptr, st);
    if (rc < 0) return rc;
    float Ro[16], Ri[16], t2[16];
    r360_rot_offset(Ro, Ri);
    r360_mul4(Ri, dense, t2);
    r360_mul4(t2, Ro, pose);                             // rotOffset^-1 * dense * rotOffset
    if (info) memcpy(info, ctx->reg_info, sizeof ctx->reg_info);
    return ctx->reg_good ? 0 : 1;
}

extern "C" int r360_register(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, const float guess[16],
                             const r360_icp_params* p, size_t max_match_planes, int mode, float pose[16],
                             float info[36], r360_icp_stats* st) {
    if (ctx && bind_device(ctx->device)) return -1;
    if (int rc = r360_register_async(ctx, ref, trg, guess, p, max_match_planes, mode)) return rc;
    return r360_register_result(ctx, pose, info, st);
}

// ------------------------------------------------------------------ inspection (parity tests)
extern "C" int r360_frame_get_cloud(r360_frame* f, float* xyz4, uint8_t* rgb4, float* nrm4, float* dist) {
    CHECK_ARG(f && (f->built & R360_BUILD_CLOUD) && f->pl.cloud, "frame cloud not built (R360_BUILD_CLOUD)");
    PlaneBufs& P = f->pl;
    const size_t T = 8 * (size_t)P.w * P.h;
    hipStream_t st = f->ctx->stream;
    if (xyz4) R360_HIP(hipMemcpyAsync(xyz4, P.cloud, sizeof(float4) * T, hipMemcpyDeviceToHost, st));
    if (rgb4) R360_HIP(hipMemcpyAsync(rgb4, P.rgb, sizeof(uchar4) * T, hipMemcpyDeviceToHost, st));
    if (nrm4) R360_HIP(hipMemcpyAsync(nrm4, P.nrm, sizeof(float4) * T, hipMemcpyDeviceToHost, st));
    if (dist) R360_HIP(hipMemcpyAsync(dist, P.dist, sizeof(float) * T, hipMemcpyDeviceToHost, st));
    R360_HIP(hipStreamSynchronize(st));
    return 0;
}

extern "C" int r360_frame_get_labels(r360_frame* f, int* lab, int* labf) {
    CHECK_ARG(f && (f->built & R360_BUILD_PLANES) && f->pl.cloud, "frame planes not built (R360_BUILD_PLANES)");
    PlaneBufs& P = f->pl;
    const size_t T = 8 * (size_t)P.w * P.h;
    hipStream_t st = f->ctx->stream;
    if (lab) R360_HIP(hipMemcpyAsync(lab, P.lab, sizeof(int) * T, hipMemcpyDeviceToHost, st));
    if (labf) R360_HIP(hipMemcpyAsync(labf, P.labf, sizeof(int) * T, hipMemcpyDeviceToHost, st));
    R360_HIP(hipStreamSynchronize(st));
    return 0;
}

extern "C" int r360_frame_get_regions(r360_frame* f, int sensor, r360_region* out, int cap, int* n) {
    if (int rc = ready(f)) return rc;
    CHECK_ARG(f->pl.cloud, "frame planes were loaded, not built: no per-sensor regions");
    CHECK_ARG(sensor >= 0 && sensor < 8, "sensor out of range");
    PlaneBufs& P = f->pl;
    const int nm = P.h_nmodels[sensor];
    if (n) *n = nm;
    for (int m = 0; m < nm && m < cap && out; ++m) {
        const PlaneOut& O = P.h_out[sensor * R360_MAX_MODELS + m];
        r360_region& r = out[m];
        r.label = O.model.label;
        r.count = (int)O.stats.n;
        r.start_idx = O.start;
        r.n_contour = O.n_contour;
        r.n_fit = O.model.n_fit;
        for (int k = 0; k < 3; ++k) r.centroid[k] = O.model.centroid[k];
        for (int k = 0; k < 9; ++k) r.cov[k] = O.model.cov[k];
        for (int k = 0; k < 4; ++k) r.model[k] = O.model.v[k];
        r.curvature = O.model.curvature;
    }
    return 0;
}

// ------------------------------------------------------------------ PbMap persistence
// Frame360::savePlanes / loadPbMap (Frame360.h:195-210, 312-318) stream the mrpt::pbmap::PbMap
// through MRPT's CSerializable into a gzip file.  MRPT is not vendored in the reference, so its byte
// layout cannot be restated here (parity unpinned at the byte level); the file keeps the gzip
// container and carries, per plane, every field the registration path reads, the exact-integer
// moments the same-plane merges use, the label and the convex hull, so a PbMap saved and loaded
// back registers bit-identically to the one built.  Layout (little-endian, inside gzip):
//   "R360PBM1" | u32 version = 1 | u32 n_planes | n_planes x {
//     i32 id, sensor | f32 normal[3], center[3], ppal[3], d, area, elongation, curvature,
//     nrgb[3], intensity | i64 n, s1[3] | i128 s2[6] | i64 c[4] | u32 label_len, label bytes |
//     u32 n_hull, f32 hull[n_hull][3] }
namespace {
const char kPbmMagic[8] = {'R', '3', '6', '0', 'P', 'B', 'M', '1'};

struct GzOut {
    gzFile g;
    bool ok = true;
    void put(const void* p, size_t n) { if (ok && n) ok = gzwrite(g, p, (unsigned)n) == (int)n; }
    template <class T> void val(const T& v) { put(&v, sizeof(T)); }
};
struct GzIn {
    gzFile g;
    bool ok = true;
    void get(void* p, size_t n) { if (ok && n) ok = gzread(g, p, (unsigned)n) == (int)n; }
    template <class T> void val(T& v) { get(&v, sizeof(T)); }
};
}  // namespace

extern "C" int r360_frame_save_planes(r360_frame* f, const char* path) {
    CHECK_ARG(path, "null path");
    if (int rc = ready(f)) return rc;
    GzOut o{gzopen(path, "wb")};
    if (!o.g) { r360_set_error("cannot create %s", path); return -1; }
    const auto& P = f->pbmap->planes;
    o.put(kPbmMagic, 8);
    o.val(uint32_t(1));
    o.val(uint32_t(P.size()));
    for (const HPlane& p : P) {
        o.val(int32_t(p.id)); o.val(int32_t(p.sensor));
        for (const P3* v : {&p.normal, &p.center, &p.ppal}) { o.val(v->x); o.val(v->y); o.val(v->z); }
        o.val(p.d); o.val(p.area); o.val(p.elongation); o.val(p.curvature);
        o.put(p.nrgb, sizeof p.nrgb); o.val(p.intensity);
        o.val(p.st.n); o.put(p.st.s1, sizeof p.st.s1); o.put(p.st.s2, sizeof p.st.s2); o.put(p.st.c, sizeof p.st.c);
        o.val(uint32_t(p.label.size())); o.put(p.label.data(), p.label.size());
        o.val(uint32_t(p.hull.size()));
        for (const P3& q : p.hull) { o.val(q.x); o.val(q.y); o.val(q.z); }
    }
    const bool closed = gzclose(o.g) == Z_OK;
    if (!o.ok || !closed) { r360_set_error("write failed: %s", path); return -1; }
    return 0;
}

extern "C" int r360_frame_load_pbmap(r360_frame* f, const char* path) {
    CHECK_ARG(f && path, "null arg");
    GzIn in{gzopen(path, "rb")};
    if (!in.g) { r360_set_error("cannot open %s", path); return -1; }
    char magic[8] = {};
    uint32_t version = 0, n = 0;
    in.get(magic, 8); in.val(version); in.val(n);
    auto fail = [&](const char* why) { gzclose(in.g); r360_set_error("%s: %s", path, why); return -1; };
    if (!in.ok || memcmp(magic, kPbmMagic, 8) != 0) return fail("not an R360 PbMap file");
    if (version != 1) return fail("unsupported PbMap file version");
    if (n > (1u << 20)) return fail("implausible plane count");
    auto* pm = new PbMapHost;
    pm->planes.resize(n);
    for (HPlane& p : pm->planes) {
        int32_t id = 0, sensor = 0;
        in.val(id); in.val(sensor);
        p.id = id; p.sensor = sensor;
        for (P3* v : {&p.normal, &p.center, &p.ppal}) { in.val(v->x); in.val(v->y); in.val(v->z); }
        in.val(p.d); in.val(p.area); in.val(p.elongation); in.val(p.curvature);
        in.get(p.nrgb, sizeof p.nrgb); in.val(p.intensity);
        in.val(p.st.n); in.get(p.st.s1, sizeof p.st.s1); in.get(p.st.s2, sizeof p.st.s2); in.get(p.st.c, sizeof p.st.c);
        uint32_t ll = 0, nh = 0;
        in.val(ll);
        if (!in.ok || ll > (1u << 20)) { delete pm; return fail("corrupt label"); }
        p.label.resize(ll);
        in.get(&p.label[0], ll);
        in.val(nh);
        if (!in.ok || nh > (1u << 24)) { delete pm; return fail("corrupt hull"); }
        p.hull.resize(nh);
        for (P3& q : p.hull) { in.val(q.x); in.val(q.y); in.val(q.z); }
        if (!in.ok) { delete pm; return fail("truncated"); }
    }
    gzclose(in.g);
    // like `serialize_planes >> planes`, the loaded map replaces the frame's planes
    planes_join(f);
    f->pl.worker_rc = 0;
    delete f->pbmap;
    f->pbmap = pm;
    f->built |= R360_BUILD_PLANES;
    return 0;
}

extern "C" int r360_frame_set_plane_label(r360_frame* f, int i, const char* label) {
    if (int rc = ready(f)) return rc;
    CHECK_ARG(label && i >= 0 && i < int(f->pbmap->planes.size()), "plane index out of range");
    f->pbmap->planes[i].label = label;
    return 0;
}

extern "C" int r360_frame_get_plane_label(r360_frame* f, int i, char* buf, int cap) {
    if (int rc = ready(f)) return rc;
    CHECK_ARG(i >= 0 && i < int(f->pbmap->planes.size()), "plane index out of range");
    const std::string& s = f->pbmap->planes[i].label;
    if (buf && cap > 0) {
        const int k = std::min(cap - 1, int(s.size()));
        memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return int(s.size());
}

// Frame360::save(path, frame) (Frame360.h:320-330): path/sphereCloud_%d.pcd (savePCDFile, ascii)
// and path/spherePlanes_%d.pbmap.
extern "C" int r360_frame_save(r360_frame* f, const char* dir, unsigned index) {
    CHECK_ARG(f && dir, "null arg");
    if (int rc = ready(f)) return rc;
    CHECK_ARG(!f->pbmap->planes.empty(), "save: the frame has no planes (Frame360.h:323 asserts)");
    char a[4096], b[4096];
    snprintf(a, sizeof a, "%s/sphereCloud_%d.pcd", dir, (int)index);
    snprintf(b, sizeof b, "%s/spherePlanes_%d.pbmap", dir, (int)index);
    if (int rc = r360_frame_save_cloud(f, a, 0)) return rc;
    return r360_frame_save_planes(f, b);
}

// Frame360::load_PbMap_Cloud(path, index) (Frame360.h:222-228): %u in the file names.
extern "C" int r360_frame_load_pbmap_cloud(r360_frame* f, const char* dir, unsigned index) {
    CHECK_ARG(f && dir, "null arg");
    char a[4096], b[4096];
    snprintf(a, sizeof a, "%s/sphereCloud_%u.pcd", dir, index);
    snprintf(b, sizeof b, "%s/spherePlanes_%u.pbmap", dir, index);
    if (int rc = r360_frame_load_cloud(f, a)) return rc;
    return r360_frame_load_pbmap(f, b);
}
