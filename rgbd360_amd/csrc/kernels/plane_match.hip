// plane_match.hip — SubgraphMatcher constraint tables on gfx950.
// The interpretation tree (host, pbmap.cpp) only reads two tables:
//   unary[i][j]          plane i of the reference subgraph may match plane j of the target one
//   binary[(i,j)][(k,l)] the pairs (i->j) and (k->l) are geometrically consistent
// k_match_tables evaluates all ns*nt*ns*nt binary constraints, one per thread, and packs them with
// wave ballots into 64-bit words.  Constraint definitions: DESIGN.md §PbMap (configLocaliser_
// sphericalOdometry.ini thresholds); the oracle's build_tables is the CPU statement of the same.
#include "../r360_internal.h"

namespace {

// descriptor layout, 16 floats per plane
enum { D_NX = 0, D_CX = 3, D_D = 6, D_AREA = 7, D_ELONG = 8, D_RGB = 9, D_INT = 12, D_STRIDE = 16 };

struct MatchCfg {
    float dist_d, cos_angle_unary, color_threshold, intensity_threshold, elongation_threshold, area_threshold;
    float dist_threshold, cos_angle_binary, height_threshold, cos_angle_parallel, planar_normal_tol;
};

__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ bool unary_ok(const float* s, const float* t, int mode, const MatchCfg& c) {
    if (s[D_AREA] > c.area_threshold * t[D_AREA] || t[D_AREA] > c.area_threshold * s[D_AREA]) return false;
    if (s[D_ELONG] > c.elongation_threshold * t[D_ELONG] || t[D_ELONG] > c.elongation_threshold * s[D_ELONG]) return false;
    for (int k = 0; k < 3; ++k)
        if (fabsf(s[D_RGB + k] - t[D_RGB + k]) > c.color_threshold) return false;
    if (fabsf(s[D_INT] - t[D_INT]) > c.intensity_threshold) return false;
    if (mode == 1 || mode == 3) {   // PLANAR_3DoF, PLANAR_ODOMETRY_3DoF: rotation about the vertical x axis
        if (fabsf(s[D_NX] - t[D_NX]) > c.planar_normal_tol) return false;
        if (fabsf(s[D_NX]) > c.cos_angle_parallel && fabsf(s[D_D] - t[D_D]) > c.dist_d) return false;
    }
    if (mode == 2 || mode == 3) {   // ODOMETRY_6DoF, PLANAR_ODOMETRY_3DoF: small displacement
        if (dot3(s + D_NX, t + D_NX) < c.cos_angle_unary) return false;
        if (fabsf(s[D_D] - t[D_D]) > c.dist_d) return false;
    }
    return true;
}

__device__ bool binary_ok(const float* s1, const float* t1, const float* s2, const float* t2, const MatchCfg& c) {
    const float a = dot3(s1 + D_NX, s2 + D_NX), b = dot3(t1 + D_NX, t2 + D_NX);
    const float sa = sqrtf(fmaxf(0.0f, 1.0f - a * a)), sb = sqrtf(fmaxf(0.0f, 1.0f - b * b));
    if (a * b + sa * sb < c.cos_angle_binary) return false;      // |angle(s1,s2) - angle(t1,t2)| <= 10 deg
    float ds[3], dt[3];
    for (int k = 0; k < 3; ++k) { ds[k] = s1[D_CX + k] - s2[D_CX + k]; dt[k] = t1[D_CX + k] - t2[D_CX + k]; }
    const float ds2 = dot3(ds, ds), dt2 = dot3(dt, dt);
    const float r2 = c.dist_threshold * c.dist_threshold;
    if (ds2 > r2 * dt2 || dt2 > r2 * ds2) return false;          // centroid-distance ratio <= 3
    if (fabsf(a) > c.cos_angle_parallel) {                        // parallel planes: relative height
        float es[3], et[3];
        for (int k = 0; k < 3; ++k) { es[k] = s2[D_CX + k] - s1[D_CX + k]; et[k] = t2[D_CX + k] - t1[D_CX + k]; }
        const float hs = dot3(s1 + D_NX, es), ht = dot3(t1 + D_NX, et);
        if (fabsf(hs - ht) > c.height_threshold) return false;
    }
    return true;
}

__global__ void k_match_tables(const float* __restrict__ desc, int ns, int nt, int mode, MatchCfg cfg,
                               uint8_t* __restrict__ unary, unsigned long long* __restrict__ bin, int words) {
    const float* S = desc;
    const float* T = desc + (long)ns * D_STRIDE;
    const int np = ns * nt;
    const long row_bits = (long)words * 64;
    const long total = (long)np * row_bits;
    for (long t0 = blockIdx.x * (long)blockDim.x; t0 < total; t0 += (long)gridDim.x * blockDim.x) {
        const long t = t0 + threadIdx.x;
        bool ok = false;
        long row = 0, bit = 0;
        if (t < total) {
            row = t / row_bits;
            bit = t - row * row_bits;
            if (bit < np) {
                const int i = (int)(row / nt), j = (int)(row - (long)i * nt);
                const int k = (int)(bit / nt), l = (int)(bit - (long)k * nt);
                if (k != i && l != j)
                    ok = binary_ok(S + i * D_STRIDE, T + j * D_STRIDE, S + k * D_STRIDE, T + l * D_STRIDE, cfg);
            }
        }
        const unsigned long long b = __ballot(ok);
        // blockDim.x and row_bits are multiples of 64: a wave covers one aligned word
        if ((threadIdx.x & 63) == 0 && t < total) bin[t / 64] = b;
        if (t < total && bit == 0 && row < np) {
            const int i = (int)(row / nt), j = (int)(row - (long)i * nt);
            unary[row] = unary_ok(S + i * D_STRIDE, T + j * D_STRIDE, mode, cfg) ? 1 : 0;
        }
    }
}

}  // namespace

int launch_match_tables(r360_ctx* ctx, hipStream_t stream, const float* d_desc, int ns, int nt, int mode,
                        uint8_t* d_unary, unsigned long long* d_bin, int words) {
    // the ctx's thresholds (r360_match_params, the ini keys); angles become the cosines / sine the
    // constraints compare against (configLocaliser_sphericalOdometry.ini: cos 50, cos 10, sin 10 deg)
    const r360_match_params& m = ctx->match;
    const MatchCfg cfg = {m.dist_d, (float)cos(m.angle * R360_PI / 180), m.color_threshold, m.intensity_threshold,
                          m.elongation_threshold, m.area_threshold, m.dist_threshold,
                          (float)cos(m.angle_threshold * R360_PI / 180), m.height_threshold, m.cos_angle_parallel,
                          (float)sin(m.planar_normal_angle * R360_PI / 180)};
    const long total = (long)ns * nt * words * 64;
    if (total == 0) return 0;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_match_tables, dim3(blocks), dim3(256), 0, stream, d_desc, ns, nt, mode, cfg, d_unary,
                       d_bin, words);
    R360_HIP(hipGetLastError());
    return 0;
}
