// pbmap_oracle.cpp — CPU ORACLE (test infrastructure only) for the per-plane half of the PbMap path:
// plane descriptors (A8, Frame360::getPlanesSensor, include/Frame360.h:940-1075), groupPlanes /
// mergePlanes (A9, :657-832), setReference / setTarget (A11, RegisterRGBD360.h:111-196), the
// SubgraphMatcher interpretation tree (A12) and ConsistencyTest::estimatePoseWithCovariance (A13).
//
// The Frame360 / RegisterRGBD360 logic is vendored reference code and is restated line by line.  The
// mrpt::pbmap::Plane methods, SubgraphMatcher and ConsistencyTest live in the unvendored MRPT-pbmap
// fork (unpinned) and are restated from SURVEY App. C.4/C.5 with the definitions below
// ("parity unpinned"):
//   calcConvexHull      Andrew's monotone chain on the two coordinates orthogonal to the dominant
//                       normal axis, closed polygon (last vertex == first).
//   computeMassCenterAndArea  polygon area / centroid on the dominant-axis projection.
//   calcElongationAndPpalDir  sqrt(l0 / l1) of the inlier covariance (exact moments, rig frame).
//   calcMainColor2      mean normalised rgb and mean intensity of the inliers (hue histogram unused).
//   isSamePlane         normal dot >= cos, |n.(c2-c1)| <= dist, then isPlaneNearby (centre/vertex/
//                       segment distances).
//   mergePlane2         area-weighted normal, hull of both hulls, merged inlier moments.
//   pcl::VoxelGrid      (empty-contour fallback, leaf 0.05) centroids of occupied voxels.
//   SubgraphMatcher     unary (area, elongation, colour, intensity, planar/odometry) and binary
//                       (relative angle, centroid-distance ratio, parallel-plane height) constraints
//                       from configLocaliser_sphericalOdometry.ini; depth-first interpretation tree,
//                       largest set wins, ties by matched source area.
//   ConsistencyTest     Kabsch rotation on area-weighted normals, least-squares translation on plane
//                       offsets, information = blockdiag(sum w n n^T, sum w (I - n n^T)).
#include "oracle360.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <vector>

namespace orc_moments {
typedef __int128 i128;
long long q36(float v);
double i128_to_double(i128 v);
}  // namespace orc_moments

namespace {

using orc_moments::i128;

struct V3 {
    float x = 0, y = 0, z = 0;
    float operator[](int k) const { return k == 0 ? x : (k == 1 ? y : z); }
};
inline float dot3(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 sub3(const V3& a, const V3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float sqn(const V3& a) { return dot3(a, a); }

// exact inlier moments in the rig frame plus colour sums
struct PlaneStats {
    long long n = 0;
    long long s1[3] = {0, 0, 0};
    i128 s2[6] = {0, 0, 0, 0, 0, 0};
    long long c[4] = {0, 0, 0, 0};  // sum of r/(r+g+b), g/.., b/.. (2^-33 fixed point), sum of r+g+b
    void merge(const PlaneStats& o) {
        n += o.n;
        for (int k = 0; k < 3; ++k) s1[k] += o.s1[k];
        for (int k = 0; k < 6; ++k) s2[k] += o.s2[k];
        for (int k = 0; k < 4; ++k) c[k] += o.c[k];
    }
};

void add_point(PlaneStats& S, const V3& p, const uint8_t* rgb) {
    const long long q[3] = {orc_moments::q36(p.x), orc_moments::q36(p.y), orc_moments::q36(p.z)};
    ++S.n;
    for (int k = 0; k < 3; ++k) S.s1[k] += q[k];
    int t = 0;
    for (int a = 0; a < 3; ++a)
        for (int b = a; b < 3; ++b) S.s2[t++] += (i128)q[a] * q[b];
    const int sum = rgb[0] + rgb[1] + rgb[2];
    if (sum != 0) {
        const float inv = 1.0f / float(sum);
        for (int k = 0; k < 3; ++k) S.c[k] += (long long)((double)(float(rgb[k]) * inv) * 8589934592.0);  // 2^33
    }
    S.c[3] += sum;
}

// symmetric 3x3 eigenvalues/vectors (cyclic Jacobi, fixed sweep order), descending
void jacobi3(const double A_in[9], double ev[3], double V[9]) {
    double A[9];
    std::memcpy(A, A_in, sizeof A);
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        if (off < 1e-300) break;
        const int P[3][2] = {{0, 1}, {0, 2}, {1, 2}};
        for (auto& pq : P) {
            const int p = pq[0], q = pq[1];
            const double apq = A[p * 3 + q];
            if (apq == 0.0) continue;
            const double theta = (A[q * 3 + q] - A[p * 3 + p]) / (2.0 * apq);
            const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
            const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {  // A = J^T A J
                const double akp = A[k * 3 + p], akq = A[k * 3 + q];
                A[k * 3 + p] = c * akp - s * akq;
                A[k * 3 + q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; ++k) {
                const double apk = A[p * 3 + k], aqk = A[q * 3 + k];
                A[p * 3 + k] = c * apk - s * aqk;
                A[q * 3 + k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; ++k) {
                const double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
                V[k * 3 + p] = c * vkp - s * vkq;
                V[k * 3 + q] = s * vkp + c * vkq;
            }
        }
    }
    int idx[3] = {0, 1, 2};
    const double d[3] = {A[0], A[4], A[8]};
    std::sort(idx, idx + 3, [&](int a, int b) { return d[a] > d[b] || (d[a] == d[b] && a < b); });
    double Vs[9];
    for (int j = 0; j < 3; ++j) {
        ev[j] = d[idx[j]];
        for (int k = 0; k < 3; ++k) Vs[k * 3 + j] = V[k * 3 + idx[j]];
    }
    std::memcpy(V, Vs, sizeof Vs);
}

struct Plane {
    V3 normal, center, ppal;
    float d = 0, area = 0, elongation = 1, curvature = 0;
    float nrgb[3] = {0, 0, 0};
    float intensity = 0;
    int id = 0, sensor = 0;
    std::vector<V3> hull;       // closed polygon
    PlaneStats st;
};

inline int dominant_axis(const V3& n) {
    int k0 = (std::fabs(n[0]) > std::fabs(n[1])) ? 0 : 1;
    k0 = (std::fabs(n[k0]) > std::fabs(n[2])) ? k0 : 2;
    return k0;
}

// Plane::calcConvexHull — Andrew's monotone chain, closed output
void calc_convex_hull(Plane& pl, const std::vector<V3>& pts) {
    const int k0 = dominant_axis(pl.normal), k1 = (k0 + 1) % 3, k2 = (k0 + 2) % 3;
    const int n = int(pts.size());
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) {
        const float ax = pts[a][k1], bx = pts[b][k1], ay = pts[a][k2], by = pts[b][k2];
        return ax < bx || (ax == bx && (ay < by || (ay == by && a < b)));
    });
    auto cross = [&](int o, int a, int b) {
        const double ox = pts[o][k1], oy = pts[o][k2];
        return ((double)pts[a][k1] - ox) * ((double)pts[b][k2] - oy) - ((double)pts[a][k2] - oy) * ((double)pts[b][k1] - ox);
    };
    pl.hull.clear();
    if (n == 0) return;
    std::vector<int> H(2 * n + 1);
    int k = 0;
    for (int i = 0; i < n; ++i) {
        while (k >= 2 && cross(H[k - 2], H[k - 1], ord[i]) <= 0) k--;
        H[k++] = ord[i];
    }
    for (int i = n - 2, t = k + 1; i >= 0; i--) {
        while (k >= t && cross(H[k - 2], H[k - 1], ord[i]) <= 0) k--;
        H[k++] = ord[i];
    }
    for (int i = 0; i < k; ++i) pl.hull.push_back(pts[H[i]]);
}

// Plane::computeMassCenterAndArea
void mass_center_and_area(Plane& pl) {
    const int k0 = dominant_axis(pl.normal), k1 = (k0 + 1) % 3, k2 = (k0 + 2) % 3;
    const float ct = std::fabs(pl.normal[k0]);
    float AreaX2 = 0.0f;
    float mc[3] = {0, 0, 0};
    const size_t n = pl.hull.size();
    for (size_t i = 0; i < n; i++) {
        const V3& pi = pl.hull[i];
        const V3& pj = pl.hull[(i + 1) % n];
        const double cross_segment = pi[k1] * pj[k2] - pi[k2] * pj[k1];   // float expression
        AreaX2 += cross_segment;
        mc[k1] += (pi[k1] + pj[k1]) * cross_segment;
        mc[k2] += (pi[k2] + pj[k2]) * cross_segment;
    }
    pl.area = std::fabs(AreaX2) / (2 * ct);
    mc[k1] /= (3 * AreaX2);
    mc[k2] /= (3 * AreaX2);
    const float nc = dot3(pl.normal, pl.center);
    mc[k0] = (nc - pl.normal[k1] * mc[k1] - pl.normal[k2] * mc[k2]) / pl.normal[k0];
    pl.center = {mc[0], mc[1], mc[2]};
    pl.d = -dot3(pl.normal, pl.center);
}

// Plane::calcElongationAndPpalDir + calcMainColor2 from the exact statistics
void descriptors_from_stats(Plane& pl) {
    const PlaneStats& S = pl.st;
    const double dn = (double)S.n;
    double cov[9];
    int t = 0;
    for (int a = 0; a < 3; ++a)
        for (int b = a; b < 3; ++b, ++t) {
            const i128 num = (i128)S.n * S.s2[t] - (i128)S.s1[a] * S.s1[b];
            cov[a * 3 + b] = cov[b * 3 + a] = orc_moments::i128_to_double(num) * 2.117582368135751e-22 / (dn * dn);
        }
    double ev[3], V[9];
    jacobi3(cov, ev, V);
    pl.elongation = float(std::sqrt(ev[0] / ev[1]));
    pl.ppal = {float(V[0]), float(V[3]), float(V[6])};
    for (int k = 0; k < 3; ++k) pl.nrgb[k] = float(((double)S.c[k] * 1.1641532182693481e-10) / dn);  // 2^-33
    pl.intensity = float((double)S.c[3] / (3.0 * dn));
}

// MRPT geometry: dist3D_Segment_to_Segment2 (squared distance between segments)
float seg_seg2(const V3& a0, const V3& a1, const V3& b0, const V3& b1) {
    const float SMALL_NUM = 0.00000001f;
    const V3 u = sub3(a1, a0), v = sub3(b1, b0), w = sub3(a0, b0);
    const float a = dot3(u, u), b = dot3(u, v), c = dot3(v, v), d = dot3(u, w), e = dot3(v, w);
    const float D = a * c - b * b;
    float sc, sN, sD = D, tc, tN, tD = D;
    if (D < SMALL_NUM) {
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
    sc = (std::fabs(sN) < SMALL_NUM ? 0.0f : sN / sD);
    tc = (std::fabs(tN) < SMALL_NUM ? 0.0f : tN / tD);
    const V3 dP = {w.x + (sc * u.x) - (tc * v.x), w.y + (sc * u.y) - (tc * v.y), w.z + (sc * u.z) - (tc * v.z)};
    return dot3(dP, dP);
}

bool is_plane_nearby(const Plane& A, const Plane& B, float thr) {
    const float t2 = thr * thr;
    if (sqn(sub3(A.center, B.center)) < t2) return true;
    for (size_t i = 1; i < A.hull.size(); i++)
        if (sqn(sub3(A.hull[i], B.center)) < t2) return true;
    for (size_t j = 1; j < B.hull.size(); j++)
        if (sqn(sub3(A.center, B.hull[j])) < t2) return true;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t j = 1; j < B.hull.size(); j++)
            if (sqn(sub3(A.hull[i], B.hull[j])) < t2) return true;
    for (size_t i = 1; i < A.hull.size(); i++)
        for (size_t j = 1; j < B.hull.size(); j++)
            if (seg_seg2(A.hull[i], A.hull[i - 1], B.hull[j], B.hull[j - 1]) < t2) return true;
    return false;
}

bool is_same_plane(const Plane& A, const Plane& B, float cos_angle, float dist, float prox) {
    if (dot3(A.normal, B.normal) < cos_angle) return false;
    const float dn = dot3(A.normal, sub3(B.center, A.center));
    if (std::fabs(dn) > dist) return false;
    return is_plane_nearby(A, B, prox);
}

// Plane::mergePlane2
void merge_plane2(Plane& A, const Plane& B) {
    V3 n = {A.area * A.normal.x + B.area * B.normal.x, A.area * A.normal.y + B.area * B.normal.y,
            A.area * A.normal.z + B.area * B.normal.z};
    const float len = std::sqrt(dot3(n, n));
    A.normal = {n.x / len, n.y / len, n.z / len};
    std::vector<V3> pts = A.hull;
    pts.insert(pts.end(), B.hull.begin(), B.hull.end());
    calc_convex_hull(A, pts);
    A.st.merge(B.st);
    mass_center_and_area(A);
    A.d = -dot3(A.normal, A.center);
    descriptors_from_stats(A);
}

// pcl::VoxelGrid (leaf 0.05) centroids, voxels in increasing index order
std::vector<V3> voxel_grid(const std::vector<V3>& pts) {
    std::vector<V3> out;
    if (pts.empty()) return out;
    const float inv = 1.0f / 0.05f;
    V3 mn = pts[0], mx = pts[0];
    for (const V3& p : pts) {
        mn = {std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z)};
        mx = {std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z)};
    }
    const long long minb[3] = {(long long)std::floor(mn.x * inv), (long long)std::floor(mn.y * inv),
                               (long long)std::floor(mn.z * inv)};
    const long long maxb[3] = {(long long)std::floor(mx.x * inv), (long long)std::floor(mx.y * inv),
                               (long long)std::floor(mx.z * inv)};
    const long long divb0 = maxb[0] - minb[0] + 1, divb1 = maxb[1] - minb[1] + 1;
    std::vector<std::pair<long long, int>> key(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) {
        const V3& p = pts[i];
        const long long ijk0 = (long long)std::floor(p.x * inv) - minb[0];
        const long long ijk1 = (long long)std::floor(p.y * inv) - minb[1];
        const long long ijk2 = (long long)std::floor(p.z * inv) - minb[2];
        key[i] = {ijk0 + ijk1 * divb0 + ijk2 * divb0 * divb1, int(i)};
    }
    std::sort(key.begin(), key.end());
    for (size_t i = 0; i < key.size();) {
        size_t j = i;
        double s[3] = {0, 0, 0};
        while (j < key.size() && key[j].first == key[i].first) {
            const V3& p = pts[key[j].second];
            s[0] += p.x; s[1] += p.y; s[2] += p.z;
            ++j;
        }
        const double c = double(j - i);
        out.push_back({float(s[0] / c), float(s[1] / c), float(s[2] / c)});
        i = j;
    }
    return out;
}

inline V3 xform(const float* T, const V3& p) {  // Eigen Affine3f * Vector3f (col-major T)
    return {T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12], T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13],
            T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14]};
}
inline V3 rot(const float* T, const V3& p) {
    return {T[0] * p.x + T[4] * p.y + T[8] * p.z, T[1] * p.x + T[5] * p.y + T[9] * p.z,
            T[2] * p.x + T[6] * p.y + T[10] * p.z};
}

const float max_curvature_plane = 0.0013f;   // include/Miscellaneous.h:54
const float min_area_plane = 0.12f;          // :57
const float max_elongation_plane = 6.0f;     // :60

struct PbMap {
    std::vector<Plane> planes;
};

}  // namespace

// ------------------------------------------------------------------------------------------------
// Public oracle entry points
extern "C" {

struct orc_pbmap_s { PbMap m; };

void* orc_pbmap_from_segments(int n_sensors, int w, int h, const float* xyz4_all, const uint8_t* rgb4_all,
                              const int* labels_final_all, const orc_region* regions, const int* n_regions,
                              const int* contour_all, const int* contour_base, const float* rt8) {
    auto* out = new orc_pbmap_s;
    std::vector<std::vector<Plane>> local(n_sensors);
    const size_t N = size_t(w) * h;
    int roff = 0;
    for (int s = 0; s < n_sensors; ++s) {
        const float* xyz4 = xyz4_all + 4 * N * s;
        const uint8_t* rgb4 = rgb4_all + 4 * N * s;
        const int* lf = labels_final_all + N * s;
        const int* contour = contour_all + contour_base[s];
        const float* Rt = rt8 + 16 * s;
        for (int i = 0; i < n_regions[s]; ++i) {
            const orc_region& R = regions[roff + i];
            Plane pl;
            pl.sensor = s;
            pl.center = {R.centroid[0], R.centroid[1], R.centroid[2]};
            pl.normal = {R.model[0], R.model[1], R.model[2]};
            if (dot3(pl.normal, pl.center) > 0) pl.normal = {-pl.normal.x, -pl.normal.y, -pl.normal.z};  // :988-992
            pl.curvature = R.curvature;
            // inliers = pixels whose final label is this region's label (refinement grows only into
            // non-planar labels, so inlier_indices[i] == {final label == label_i})
            std::vector<V3> inl;
            for (size_t p = 0; p < N; ++p)
                if (lf[p] == R.label) {
                    const V3 q = {xyz4[4 * p], xyz4[4 * p + 1], xyz4[4 * p + 2]};
                    inl.push_back(q);
                    add_point(pl.st, xform(Rt, q), rgb4 + 4 * p);
                }
            std::vector<V3> cpts;
            if (R.n_contour > 0) {
                for (int k = 0; k < R.n_contour; ++k) {
                    const int p = contour[R.contour_off + k];
                    cpts.push_back({xyz4[4 * p], xyz4[4 * p + 1], xyz4[4 * p + 2]});
                }
            } else {
                cpts = voxel_grid(inl);                    // "HULL 000" fallback, :1017-1026
            }
            calc_convex_hull(pl, cpts);
            mass_center_and_area(pl);
            if (pl.area < min_area_plane) continue;       // :1034
            pl.d = -dot3(pl.normal, pl.center);            // :1037
            descriptors_from_stats(pl);                    // elongation (rig frame moments) + colour
            if (pl.elongation > max_elongation_plane) continue;  // :1041
            // transform(Rt) (:1051): normal, centre, hull (inlier stats are already in the rig frame)
            pl.normal = rot(Rt, pl.normal);
            pl.center = xform(Rt, pl.center);
            pl.d = -dot3(pl.normal, pl.center);
            for (V3& v : pl.hull) v = xform(Rt, v);
            bool same = false;
            if (pl.curvature < max_curvature_plane)
                for (size_t j = 0; j < local[s].size(); j++)
                    if (local[s][j].curvature < max_curvature_plane &&
                        is_same_plane(local[s][j], pl, 0.99f, 0.05f, 0.2f)) {
                        same = true;
                        merge_plane2(local[s][j], pl);
                        break;
                    }
            if (!same) {
                pl.id = int(local[s].size());
                local[s].push_back(pl);
            }
        }
        roff += n_regions[s];
    }
    // groupPlanes (:742-832)
    std::vector<Plane>& P = out->m.planes;
    const float maxDistHull = 0.5f, maxDistParallelHull = 0.09f;
    P = local[0];
    std::set<unsigned> prev_planes, first_planes;
    for (size_t i = 0; i < P.size(); i++) first_planes.insert(unsigned(P[i].id));
    prev_planes = first_planes;
    for (int s = 1; s < n_sensors; ++s) {
        size_t j = 0;
        std::set<unsigned> next_prev;
        for (size_t k = 0; k < local[s].size(); k++) {
            Plane& L = local[s][k];
            bool same = false;
            if (L.area > 0.5f || L.curvature < max_curvature_plane)
                for (auto it = prev_planes.begin(); it != prev_planes.end() && !same; it++) {
                    j = *it;
                    if (P[j].area < 0.5f || P[j].curvature > max_curvature_plane) continue;
                    if (std::fabs(P[j].d - L.d) < 0.45f)
                        if (dot3(P[j].normal, L.normal) > 0.99f) {
                            for (size_t i = 1; i < P[j].hull.size() && !same; i++)
                                for (size_t ii = 1; ii < L.hull.size(); ii++) {
                                    const V3 diff = sub3(P[j].hull[i], L.hull[ii]);
                                    const float dist = std::sqrt(sqn(diff));
                                    if (dist < maxDistHull && std::fabs(dot3(P[j].normal, diff)) < maxDistParallelHull) {
                                        same = true;
                                        break;
                                    }
                                }
                            if (!same)
                                for (size_t i = 1; i < P[j].hull.size() && !same; i++)
                                    for (size_t ii = 1; ii < L.hull.size(); ii++) {
                                        const float dist = std::sqrt(seg_seg2(P[j].hull[i], P[j].hull[i - 1], L.hull[ii], L.hull[ii - 1]));
                                        if (dist < maxDistHull) {
                                            const V3 diff = sub3(P[j].hull[i], L.hull[ii]);
                                            if (std::fabs(dot3(P[j].normal, diff)) < maxDistParallelHull) {
                                                same = true;
                                                break;
                                            }
                                        }
                                    }
                        }
                    if (same) break;
                }
            if (same) {
                next_prev.insert(unsigned(P[j].id));
                merge_plane2(P[j], L);
            } else {
                next_prev.insert(unsigned(P.size()));
                L.id = int(P.size());
                P.push_back(L);
            }
        }
        prev_planes = next_prev;
        if (s == 6) prev_planes.insert(first_planes.begin(), first_planes.end());
    }
    // mergePlanes (:657-739)
    for (size_t j = 0; j < P.size(); j++)
        if (P[j].curvature < max_curvature_plane)
            for (size_t k = j + 1; k < P.size(); k++)
                if (P[k].curvature < max_curvature_plane) {
                    bool same = false;
                    if (dot3(P[j].normal, P[k].normal) > 0.99f)
                        if (std::fabs(P[j].d - P[k].d) < 0.45f) {
                            for (size_t i = 1; i < P[j].hull.size() && !same; i++)
                                for (size_t ii = 1; ii < P[k].hull.size(); ii++) {
                                    const V3 diff = sub3(P[j].hull[i], P[k].hull[ii]);
                                    const float dist = std::sqrt(sqn(diff));
                                    if (dist < 0.3f && std::fabs(dot3(P[j].normal, diff)) < 0.06f) {
                                        same = true;
                                        break;
                                    }
                                }
                            if (!same)
                                for (size_t i = 1; i < P[j].hull.size() && !same; i++)
                                    for (size_t ii = 1; ii < P[k].hull.size(); ii++) {
                                        const float dist = std::sqrt(seg_seg2(P[j].hull[i], P[j].hull[i - 1], P[k].hull[ii], P[k].hull[ii - 1]));
                                        if (dist < 0.3f) {
                                            const V3 diff = sub3(P[j].hull[i], P[k].hull[ii]);
                                            if (std::fabs(dot3(P[j].normal, diff)) < 0.06f) {
                                                same = true;
                                                break;
                                            }
                                        }
                                    }
                        }
                    if (same) {
                        merge_plane2(P[j], P[k]);
                        for (size_t hh = k + 1; hh < P.size(); hh++) --P[hh].id;
                        P.erase(P.begin() + long(k));
                        j--;
                        k = P.size();
                    }
                }
    return out;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Frame-level pipeline (Frame360::buildSphereCloud + getPlanes, include/Frame360.h:467-510, 615-640)
namespace {

struct MatchCfg {                       // config_files/configLocaliser_sphericalOdometry.ini
    float dist_d = 0.5f, cos_angle_unary = 0.64278761f /* cos 50 deg */, color_threshold = 0.07f,
          intensity_threshold = 100.f, elongation_threshold = 2.5f, area_threshold = 3.0f;
    float dist_threshold = 3.0f, cos_angle_binary = 0.98480775f /* cos 10 deg */, height_threshold = 0.33f,
          cos_angle_parallel = 0.985f, planar_normal_tol = 0.17364818f /* sin 10 deg */;
    int min_planes_recognition = 3;
    long max_nodes = 4000000;           // interpretation-tree node budget (deterministic cut-off)
    MatchCfg() = default;
    explicit MatchCfg(const orc_match_params* p) {
        if (!p) return;
        const double PI = 3.14159265359;        // include/Miscellaneous.h:44
        dist_d = p->dist_d;
        cos_angle_unary = (float)std::cos(p->angle * PI / 180);
        color_threshold = p->color_threshold;
        intensity_threshold = p->intensity_threshold;
        elongation_threshold = p->elongation_threshold;
        area_threshold = p->area_threshold;
        dist_threshold = p->dist_threshold;
        cos_angle_binary = (float)std::cos(p->angle_threshold * PI / 180);
        height_threshold = p->height_threshold;
        cos_angle_parallel = p->cos_angle_parallel;
        planar_normal_tol = (float)std::sin(p->planar_normal_angle * PI / 180);
        min_planes_recognition = p->min_planes_recognition;
        max_nodes = p->max_nodes;
    }
};

enum { DEFAULT_6DoF = 0, PLANAR_3DoF = 1, ODOMETRY_6DoF = 2, PLANAR_ODOMETRY_3DoF = 3 };

bool unary_ok(const Plane& s, const Plane& t, int mode, const MatchCfg& c) {
    if (s.area > c.area_threshold * t.area || t.area > c.area_threshold * s.area) return false;
    if (s.elongation > c.elongation_threshold * t.elongation || t.elongation > c.elongation_threshold * s.elongation)
        return false;
    for (int k = 0; k < 3; ++k)
        if (std::fabs(s.nrgb[k] - t.nrgb[k]) > c.color_threshold) return false;
    if (std::fabs(s.intensity - t.intensity) > c.intensity_threshold) return false;
    if (mode == PLANAR_3DoF || mode == PLANAR_ODOMETRY_3DoF) {
        // planar motion about the vertical rig axis x: the vertical normal component is preserved and
        // horizontal planes keep their height
        if (std::fabs(s.normal.x - t.normal.x) > c.planar_normal_tol) return false;
        if (std::fabs(s.normal.x) > c.cos_angle_parallel && std::fabs(s.d - t.d) > c.dist_d) return false;
    }
    if (mode == ODOMETRY_6DoF || mode == PLANAR_ODOMETRY_3DoF) {
        if (dot3(s.normal, t.normal) < c.cos_angle_unary) return false;
        if (std::fabs(s.d - t.d) > c.dist_d) return false;
    }
    return true;
}

bool binary_ok(const Plane& s1, const Plane& t1, const Plane& s2, const Plane& t2, const MatchCfg& c) {
    const float a = dot3(s1.normal, s2.normal), b = dot3(t1.normal, t2.normal);
    const float sa = std::sqrt(std::max(0.0f, 1.0f - a * a)), sb = std::sqrt(std::max(0.0f, 1.0f - b * b));
    if (a * b + sa * sb < c.cos_angle_binary) return false;
    const float ds2 = sqn(sub3(s1.center, s2.center)), dt2 = sqn(sub3(t1.center, t2.center));
    const float r2 = c.dist_threshold * c.dist_threshold;
    if (ds2 > r2 * dt2 || dt2 > r2 * ds2) return false;
    if (std::fabs(a) > c.cos_angle_parallel) {
        const float hs = dot3(s1.normal, sub3(s2.center, s1.center));
        const float ht = dot3(t1.normal, sub3(t2.center, t1.center));
        if (std::fabs(hs - ht) > c.height_threshold) return false;
    }
    return true;
}

// RegisterRGBD360::setReference / setTarget (RegisterRGBD360.h:111-196): subgraph plane ids
std::vector<int> select_planes(const std::vector<Plane>& P, size_t max_match_planes) {
    std::vector<int> ids;
    if (max_match_planes > 0 && P.size() > max_match_planes) {
        std::vector<float> areas(P.size(), 0);
        for (size_t i = 0; i < P.size(); i++)
            if (P[i].curvature < max_curvature_plane) areas[i] = P[i].area;   // label == "" always
        std::vector<float> sorted = areas;
        std::sort(sorted.begin(), sorted.end());
        const float thr = sorted[P.size() - max_match_planes - 1];
        for (size_t i = 0; i < P.size(); i++)
            if (areas[i] > thr) ids.push_back(P[i].id);
    } else {
        for (size_t i = 0; i < P.size(); i++)
            if (P[i].curvature < max_curvature_plane) ids.push_back(P[i].id);
    }
    std::sort(ids.begin(), ids.end());   // std::set<unsigned> iteration order
    return ids;
}

struct Tables {
    int ns = 0, nt = 0;
    std::vector<uint8_t> unary;          // [ns][nt]
    std::vector<uint64_t> bin;           // [(i*nt+j)][words] bit (k*nt+l)
    int words = 0;
    bool b(int i, int j, int k, int l) const {
        const size_t r = size_t(i * nt + j) * words;
        const int bit = k * nt + l;
        return (bin[r + bit / 64] >> (bit % 64)) & 1;
    }
};

Tables build_tables(const std::vector<Plane>& S, const std::vector<int>& sid, const std::vector<Plane>& T,
                    const std::vector<int>& tid, int mode, const MatchCfg& c) {
    Tables tb;
    tb.ns = int(sid.size());
    tb.nt = int(tid.size());
    tb.unary.assign(size_t(tb.ns) * tb.nt, 0);
    for (int i = 0; i < tb.ns; ++i)
        for (int j = 0; j < tb.nt; ++j) tb.unary[size_t(i) * tb.nt + j] = unary_ok(S[sid[i]], T[tid[j]], mode, c);
    const int np = tb.ns * tb.nt;
    tb.words = (np + 63) / 64;
    tb.bin.assign(size_t(np) * tb.words, 0);
    for (int i = 0; i < tb.ns; ++i)
        for (int j = 0; j < tb.nt; ++j)
            for (int k = 0; k < tb.ns; ++k)
                for (int l = 0; l < tb.nt; ++l) {
                    if (k == i || l == j) continue;
                    if (binary_ok(S[sid[i]], T[tid[j]], S[sid[k]], T[tid[l]], c)) {
                        const int bit = k * tb.nt + l;
                        tb.bin[size_t(i * tb.nt + j) * tb.words + bit / 64] |= 1ull << (bit % 64);
                    }
                }
    return tb;
}

// Interpretation tree (App. C.4): references in order, each tries its targets ascending and then "unmatched";
// best = most matches, ties by matched reference area, first found among equals.  Forward checking keeps, per
// reference below the current depth, the set of targets still allowed by the unary table and by the binary table
// against every assignment made above it; the bound counts only references whose set is non-empty.  The cuts are
// sound, so the search returns the exhaustive optimum unless the node budget stops it (then `truncated`).
struct Search {
    const Tables* tb;
    std::vector<double> area_s;
    std::vector<std::vector<std::vector<bool>>> doms;   // doms[depth][ref][target]
    std::vector<int> cur, best;         // cur[i] = target index or -1
    int n_cur = 0, n_best = 0;
    double a_cur = 0, a_best = 0;
    long nodes = 0, max_nodes = 0;
    bool truncated = false;
    void start() {
        const int ns = tb->ns, nt = tb->nt;
        doms.assign(ns + 1, std::vector<std::vector<bool>>(ns, std::vector<bool>(nt, false)));
        for (int i = 0; i < ns; ++i)
            for (int t = 0; t < nt; ++t) doms[0][i][t] = tb->unary[size_t(i) * nt + t] != 0;
        cur.assign(ns, -1);
        best.assign(ns, -1);
        rec(0);
    }
    void rec(int i) {
        if (++nodes > max_nodes) { truncated = true; return; }
        const int ns = tb->ns, nt = tb->nt;
        if (i == ns) {
            if (n_cur > n_best || (n_cur == n_best && a_cur > a_best)) {
                best = cur; n_best = n_cur; a_best = a_cur;
            }
            return;
        }
        const auto& D = doms[i];
        int open = 0, free_targets = 0;
        double open_area = 0;
        for (int r = i; r < ns; ++r)
            if (std::find(D[r].begin(), D[r].end(), true) != D[r].end()) { ++open; open_area += area_s[r]; }
        for (int u = 0; u < nt; ++u) {
            bool any = false;
            for (int r = i; r < ns && !any; ++r) any = D[r][u];
            free_targets += any ? 1 : 0;
        }
        open = std::min(open, free_targets);      // each target can still take one reference
        if (n_cur + open < n_best) return;
        if (n_cur + open == n_best && a_cur + open_area <= a_best) return;
        auto& N = doms[i + 1];
        for (int t = 0; t < nt; ++t) {
            if (!D[i][t]) continue;
            for (int r = i + 1; r < ns; ++r)
                for (int u = 0; u < nt; ++u) N[r][u] = D[r][u] && u != t && tb->b(r, u, i, t);
            cur[i] = t; n_cur++; a_cur += area_s[i];
            rec(i + 1);
            cur[i] = -1; n_cur--; a_cur -= area_s[i];
            if (truncated) return;
        }
        for (int r = i + 1; r < ns; ++r) N[r] = D[r];
        rec(i + 1);
    }
};

// ConsistencyTest::estimatePoseWithCovariance (App. C.5)
bool consistency(const std::vector<Plane>& R, const std::vector<Plane>& T, const std::map<unsigned, unsigned>& m,
                 float pose[16], float info[36]) {
    if (m.size() < 3) return false;
    double M[9] = {0}, Ht[9] = {0}, Hr[9] = {0}, g[3] = {0};
    for (auto& kv : m) {
        const Plane& pr = R[kv.first];
        const Plane& pt = T[kv.second];
        const double w = pt.area;
        const double nr[3] = {pr.normal.x, pr.normal.y, pr.normal.z}, nt[3] = {pt.normal.x, pt.normal.y, pt.normal.z};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                M[a * 3 + b] += w * nt[a] * nr[b];
                Ht[a * 3 + b] += w * nr[a] * nr[b];
                Hr[a * 3 + b] += w * ((a == b ? 1.0 : 0.0) - nr[a] * nr[b]);
            }
        const double e = double(pt.d) - double(pr.d);
        for (int a = 0; a < 3; ++a) g[a] += w * nr[a] * e;
    }
    // SVD of M via the eigen-decomposition of M^T M
    double MtM[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += M[k * 3 + a] * M[k * 3 + b];
            MtM[a * 3 + b] = s;
        }
    double lam[3], V[9];
    jacobi3(MtM, lam, V);
    double sig[3], U[9];
    for (int k = 0; k < 3; ++k) sig[k] = std::sqrt(std::max(0.0, lam[k]));
    if (!(sig[1] > 1e-6 * sig[0])) return false;     // fewer than two independent normals
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < 3; ++a) {
            double s = 0;
            for (int b = 0; b < 3; ++b) s += M[a * 3 + b] * V[b * 3 + k];
            U[a * 3 + k] = s / sig[k];
        }
    U[0 * 3 + 2] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
    U[1 * 3 + 2] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
    U[2 * 3 + 2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
    auto det3 = [](const double A[9]) {
        return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) + A[2] * (A[3] * A[7] - A[4] * A[6]);
    };
    double Rm[9];
    for (int pass = 0; pass < 2; ++pass) {
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += V[a * 3 + k] * U[b * 3 + k];
                Rm[a * 3 + b] = s;
            }
        if (det3(Rm) > 0) break;
        for (int a = 0; a < 3; ++a) V[a * 3 + 2] = -V[a * 3 + 2];
    }
    // translation: Ht t = g, conditioning test (threshold_conditioning, Miscellaneous.h:76)
    double lt[3], Vt[9];
    jacobi3(Ht, lt, Vt);
    if (!(lt[2] > 0) || lt[0] / lt[2] > 8000.0) return false;
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

}  // namespace

extern "C" {

void* orc_pbmap_build(const float* depth_m8, const uint8_t* bgr8, int rows, int cols, const float* rt8) {
    const int w = cols / 2, h = rows / 2;
    const size_t N = size_t(w) * h;
    std::vector<float> xyz(8 * N * 4), nrm(8 * N * 4), dist(8 * N);
    std::vector<uint8_t> rgb(8 * N * 4);
    std::vector<int> lc(8 * N), lf(8 * N);
    const int max_regions = 1024, cap = int(16 * N);
    std::vector<orc_region> regs(8 * size_t(max_regions));
    std::vector<int> contour(8 * size_t(cap));
    int nreg[8] = {0};
    int fail = 0;
#pragma omp parallel for num_threads(8) schedule(static, 1)
    for (int s = 0; s < 8; ++s) {      // include/Frame360.h:476-499 (one OpenMP thread per sensor)
        float* x = xyz.data() + 4 * N * s;
        orc_cloud_downsample(depth_m8 + size_t(rows) * cols * s, bgr8 + size_t(rows) * cols * 3 * s, rows, cols, x,
                             rgb.data() + 4 * N * s);
        orc_bilateral(x, w, h);
        orc_normals(x, w, h, nrm.data() + 4 * N * s, dist.data() + N * s);
        nreg[s] = orc_segment(x, nrm.data() + 4 * N * s, w, h, lc.data() + N * s, lf.data() + N * s,
                              regs.data() + size_t(max_regions) * s, max_regions, contour.data() + size_t(cap) * s, cap);
        if (nreg[s] < 0) {
#pragma omp atomic write
            fail = 1;
        }
    }
    if (fail) return nullptr;
    // pack the regions contiguously as orc_pbmap_from_segments expects
    std::vector<orc_region> packed;
    int base[8];
    for (int s = 0; s < 8; ++s) {
        base[s] = cap * s;
        for (int i = 0; i < nreg[s]; ++i) packed.push_back(regs[size_t(max_regions) * s + i]);
    }
    return orc_pbmap_from_segments(8, w, h, xyz.data(), rgb.data(), lf.data(), packed.data(), nreg, contour.data(),
                                   base, rt8);
}

void orc_pbmap_free(void* h) { delete static_cast<orc_pbmap_s*>(h); }

int orc_pbmap_count(const void* h) { return int(static_cast<const orc_pbmap_s*>(h)->m.planes.size()); }

int orc_pbmap_get(const void* h, int i, orc_plane* out, float* hull_xyz, int hull_cap) {
    const auto& P = static_cast<const orc_pbmap_s*>(h)->m.planes;
    if (i < 0 || i >= int(P.size())) return -1;
    const Plane& p = P[size_t(i)];
    const V3* v3[3] = {&p.normal, &p.center, &p.ppal};
    float* o3[3] = {out->normal, out->center, out->ppal};
    for (int k = 0; k < 3; ++k) { o3[k][0] = v3[k]->x; o3[k][1] = v3[k]->y; o3[k][2] = v3[k]->z; }
    out->d = p.d; out->area = p.area; out->elongation = p.elongation; out->curvature = p.curvature;
    for (int k = 0; k < 3; ++k) out->nrgb[k] = p.nrgb[k];
    out->intensity = p.intensity;
    out->id = p.id; out->sensor = p.sensor; out->n_inliers = int(p.st.n); out->n_hull = int(p.hull.size());
    for (int k = 0; k < int(p.hull.size()) && k < hull_cap; ++k) {
        hull_xyz[3 * k] = p.hull[k].x; hull_xyz[3 * k + 1] = p.hull[k].y; hull_xyz[3 * k + 2] = p.hull[k].z;
    }
    return 0;
}

int orc_match_tables(const void* href, const void* htrg, size_t max_match_planes, int mode, int* ns, int* nt,
                     int* sid, int* tid, uint8_t* unary, uint64_t* binary, int cap, const orc_match_params* mp) {
    const auto& S = static_cast<const orc_pbmap_s*>(href)->m.planes;
    const auto& T = static_cast<const orc_pbmap_s*>(htrg)->m.planes;
    MatchCfg c(mp);
    const std::vector<int> si = select_planes(S, max_match_planes), ti = select_planes(T, max_match_planes);
    *ns = int(si.size());
    *nt = int(ti.size());
    if (*ns > cap || *nt > cap) return -1;
    const Tables tb = build_tables(S, si, T, ti, mode, c);
    for (int i = 0; i < *ns; ++i) sid[i] = si[i];
    for (int j = 0; j < *nt; ++j) tid[j] = ti[j];
    std::memcpy(unary, tb.unary.data(), tb.unary.size());
    std::memcpy(binary, tb.bin.data(), tb.bin.size() * 8);
    return tb.words;
}

// The search alone over given tables (unary [ns][nt], binary [(i*nt+j)][words], reference areas)
int orc_tree_search(int ns, int nt, const uint8_t* unary, const uint64_t* binary, int words, const double* area,
                    long max_nodes, int* best, long* nodes) {
    Tables tb;
    tb.ns = ns; tb.nt = nt; tb.words = words;
    tb.unary.assign(unary, unary + size_t(ns) * nt);
    tb.bin.assign(binary, binary + size_t(ns) * nt * words);
    Search sr;
    sr.tb = &tb;
    sr.max_nodes = max_nodes;
    sr.area_s.assign(area, area + ns);
    sr.start();
    for (int i = 0; i < ns; ++i) best[i] = sr.best[i];
    *nodes = sr.nodes;
    return sr.truncated ? 1 : 0;
}

// nodes visited by the last orc_register_pbmap search on this thread and whether the budget stopped it
static thread_local long g_last_nodes = 0;
static thread_local int g_last_truncated = 0;
void orc_last_match_stats(long* nodes, int* truncated) {
    if (nodes) *nodes = g_last_nodes;
    if (truncated) *truncated = g_last_truncated;
}

int orc_register_pbmap(const void* href, const void* htrg, size_t max_match_planes, int mode, float pose[16],
                       float info[36], int* pairs, int pair_cap, int* n_match, float* area_matched, float* area_src,
                       float* area_trg, const orc_match_params* mp) {
    const auto& S = static_cast<const orc_pbmap_s*>(href)->m.planes;
    const auto& T = static_cast<const orc_pbmap_s*>(htrg)->m.planes;
    MatchCfg c(mp);
    const std::vector<int> si = select_planes(S, max_match_planes), ti = select_planes(T, max_match_planes);
    const Tables tb = build_tables(S, si, T, ti, mode, c);
    Search sr;
    sr.tb = &tb;
    sr.max_nodes = c.max_nodes;
    sr.area_s.resize(si.size());
    for (size_t i = 0; i < si.size(); ++i) sr.area_s[i] = S[si[i]].area;
    sr.start();
    g_last_nodes = sr.nodes;
    g_last_truncated = sr.truncated ? 1 : 0;
    std::map<unsigned, unsigned> best;
    for (size_t i = 0; i < si.size(); ++i)
        if (sr.best[i] >= 0) best[unsigned(si[i])] = unsigned(ti[sr.best[i]]);
    *n_match = int(best.size());
    int k = 0;
    float am = 0;
    for (auto& kv : best) {
        if (k < pair_cap) { pairs[2 * k] = int(kv.first); pairs[2 * k + 1] = int(kv.second); }
        ++k;
        am += S[kv.first].area;                       // SubgraphMatcher::calcAreaMatched
    }
    *area_matched = am;
    if (int(best.size()) < c.min_planes_recognition) return 0;   // RegisterRGBD360.h:306-310
    const bool good = consistency(S, T, best, pose, info);
    if (good) {                                                     // :323-334
        float as = 0, at = 0;
        for (int id : si) as += S[id].area;
        for (int id : ti) at += T[id].area;
        *area_src = as;
        *area_trg = at;
    }
    return good ? 1 : 0;
}

}  // extern "C"
