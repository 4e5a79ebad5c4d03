// frame_kernels.hip — Frame360 construction on gfx950:
//   k_undistort : loadDepthEigen + CLAMS undistort           (Frame360.h:254-258, 293-310)
//   k_stitch(_t): stitchSphericalImage + cvtColor + depth m   (Frame360.h:1099-1148,
//                 RegisterPhotoICP.h:485-486, 316-317)
//   k_pyramid   : pyrDown (gray) + buildPyramidRange (depth)  (RegisterPhotoICP.h:292-354)
//   k_gradient  : calcGradientXY for gray and depth + the alignFrames360 seam mask
//                 (RegisterPhotoICP.h:365-398, 4538-4549)
// All are HBM-streaming, one thread per output pixel.  Compiled with -ffp-contract=off so each
// float expression rounds exactly as the reference's scalar C++ does.
#include "../r360_internal.h"

namespace {

constexpr int TPB = 256;

// ------------------------------------------------------------------ undistort
__global__ void k_undistort(const uint16_t* __restrict__ depth, float* __restrict__ depth_m, int rows, int cols,
                            const float* __restrict__ mult, const float* __restrict__ counts, int nx, int bin_w,
                            int bin_h, int nb, double bin_depth, int apply) {
    const long n = (long)R360_NUM_SENSORS * rows * cols;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        float z = (float)depth[i] * 0.001f;                       // convertTo(CV_32FC1, 0.001)
        if (apply && z != 0) {                                    // discrete_depth_distortion_model.cpp:175-186
            const int s = (int)(i / ((long)rows * cols));
            const int pix = (int)(i - (long)s * rows * cols);
            const int v = pix / cols, u = pix - v * cols;
            const long fr = ((long)s * (rows / bin_h) * nx + (long)(v / bin_h) * nx + (u / bin_w)) * nb;
            int idx = (int)floor(z / bin_depth);
            idx = idx < nb - 1 ? idx : nb - 1;
            float start = (float)(bin_depth * idx);
            int idx1 = (z - start < bin_depth / 2) ? idx : idx + 1;  // interpolatedUndistort :48-68
            int idx0 = idx1 - 1;
            if (idx0 < 0 || idx1 >= nb || counts[fr + idx0] < 50 || counts[fr + idx1] < 50) {
                z *= mult[fr + idx];
            } else {
                double z0 = (idx0 + 1) * bin_depth - bin_depth * 0.5;
                double c1 = (z - z0) / bin_depth;
                double c0 = 1.0 - c1;
                double m = c0 * mult[fr + idx0] + c1 * mult[fr + idx1];
                z = (float)(z * m);
            }
        }
        depth_m[i] = z;
    }
}

// k_undistort with 4 consecutive pixels of one sensor row per thread (cols % 4 == 0): one 8-byte load and one 16-byte
// store per thread instead of a 2-byte load and a 4-byte store per pixel, the same per-pixel expressions
__device__ __forceinline__ float undistort_px(float z, int s, int v, int u, int rows, int cols,
                                              const float* __restrict__ mult, const float* __restrict__ counts, int nx,
                                              int bin_w, int bin_h, int nb, double bin_depth) {
    const long fr = ((long)s * (rows / bin_h) * nx + (long)(v / bin_h) * nx + (u / bin_w)) * nb;
    int idx = (int)floor(z / bin_depth);
    idx = idx < nb - 1 ? idx : nb - 1;
    float start = (float)(bin_depth * idx);
    int idx1 = (z - start < bin_depth / 2) ? idx : idx + 1;  // interpolatedUndistort :48-68
    int idx0 = idx1 - 1;
    if (idx0 < 0 || idx1 >= nb || counts[fr + idx0] < 50 || counts[fr + idx1] < 50) return z * mult[fr + idx];
    double z0 = (idx0 + 1) * bin_depth - bin_depth * 0.5;
    double c1 = (z - z0) / bin_depth;
    double c0 = 1.0 - c1;
    double m = c0 * mult[fr + idx0] + c1 * mult[fr + idx1];
    return (float)(z * m);
}

__global__ void k_undistort4(const uint16_t* __restrict__ depth, float* __restrict__ depth_m, int rows, int cols,
                             const float* __restrict__ mult, const float* __restrict__ counts, int nx, int bin_w,
                             int bin_h, int nb, double bin_depth, int apply) {
    const long nq = (long)R360_NUM_SENSORS * rows * cols / 4;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < nq; q += (long)gridDim.x * blockDim.x) {
        const uint2 d4 = reinterpret_cast<const uint2*>(depth)[q];
        const unsigned dv[4] = {d4.x & 0xffffu, d4.x >> 16, d4.y & 0xffffu, d4.y >> 16};
        float z[4];
        // the quad's sensor, row and first column (one row: cols % 4 == 0; 32-bit: a sensor image < 2^31 pixels)
        const int pq = rows * cols / 4;
        const int qi = (int)q;
        const int s = qi / pq;
        const int pix = (qi - s * pq) * 4;
        const int v = pix / cols, u0 = pix - v * cols;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            z[e] = (float)dv[e] * 0.001f;                          // convertTo(CV_32FC1, 0.001)
            if (apply && z[e] != 0)                                // discrete_depth_distortion_model.cpp:175-186
                z[e] = undistort_px(z[e], s, v, u0 + e, rows, cols, mult, counts, nx, bin_w, bin_h, nb, bin_depth);
        }
        reinterpret_cast<float4*>(depth_m)[q] = make_float4(z[0], z[1], z[2], z[3]);
    }
}

// ------------------------------------------------------------------ stitch
// One thread per sphere pixel.  Sensor k owns columns [(7-k)*rows, (8-k)*rows)  (:1119-1120).
__global__ void k_stitch(const uint8_t* __restrict__ bgr8, const uint16_t* __restrict__ depth8, int rows, int cols,
                         int H, int W, const float* __restrict__ sinphi, const float* __restrict__ cosphi,
                         const float* __restrict__ sinth, const float* __restrict__ costh,
                         const float* __restrict__ rt_inv, float fx, float fy, float cx, float cy,
                         uint8_t* __restrict__ sph_bgr, uint16_t* __restrict__ sph_depth, float2* __restrict__ p0,
                         uint32_t* __restrict__ pk) {
    const long n = (long)H * W;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int row = (int)(i / W), col = (int)(i - (long)row * W);
        const int k = 7 - col / rows;
        const float* T = rt_inv + 16 * k;
        const float v0 = sinphi[row], cos_phi = cosphi[row];
        const float v1 = cos_phi * sinth[col];
        const float v2 = cos_phi * costh[col];
        float p0x = T[0] * v0 + T[4] * v1 + T[8] * v2;
        float p1 = T[1] * v0 + T[5] * v1 + T[9] * v2;
        float p2 = T[2] * v0 + T[6] * v1 + T[10] * v2;
        p0x = p0x + T[12]; p1 = p1 + T[13]; p2 = p2 + T[14];
        const float u = fx * p0x / p2 + cx;                          // :1133
        const float v = fy * p1 / p2 + cy;                           // :1134
        uint8_t b = 0, g = 0, r = 0;
        uint16_t dd = 0;
        if (u >= 0 && u < cols && v >= 0 && v < rows) {
            const int iu = (int)u, iv = (int)v;
            const long si = (long)k * rows * cols + (long)iv * cols + iu;
            b = bgr8[si * 3 + 0]; g = bgr8[si * 3 + 1]; r = bgr8[si * 3 + 2];
            const double du = (double)((u - cx) / fx), dv = (double)((v - cy) / fy);
            dd = (uint16_t)(depth8[si] * sqrt(1 + du * du + dv * dv));  // :1142 (range in mm)
        }
        sph_bgr[i * 3 + 0] = b; sph_bgr[i * 3 + 1] = g; sph_bgr[i * 3 + 2] = r;
        sph_depth[i] = dd;
        // setSourceFrame / setTargetFrame level 0: CV_RGB2GRAY on BGR data, /255; depth *0.001
        const int y = (b * 4899 + g * 9617 + r * 1868 + (1 << 13)) >> 14;
        p0[i] = make_float2((float)y * (float)(1. / 255), (float)dd * 0.001f);
        pk[i] = dd | ((unsigned)y << 16);
    }
}

// k_stitch with 4 consecutive sphere pixels of one row per thread (W % 4 == 0): the same per-pixel expressions,
// with the 4 pixels' BGR bytes, ranges and level-0 {gray, depth} written as 3 + 2 + 8 dwords (byte-granular
// stores of one pixel per lane were a third of the kernel's memory instructions)
__global__ void k_stitch4(const uint8_t* __restrict__ bgr8, const uint16_t* __restrict__ depth8, int rows, int cols,
                          int H, int W, const float* __restrict__ sinphi, const float* __restrict__ cosphi,
                          const float* __restrict__ sinth, const float* __restrict__ costh,
                          const float* __restrict__ rt_inv, float fx, float fy, float cx, float cy,
                          uint8_t* __restrict__ sph_bgr, uint16_t* __restrict__ sph_depth, float2* __restrict__ p0,
                          uint32_t* __restrict__ pk) {
    const long nq = (long)H * W / 4;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < nq; q += (long)gridDim.x * blockDim.x) {
        const long i0 = 4 * q;
        const int row = (int)(i0 / W), col0 = (int)(i0 - (long)row * W);
        const float v0 = sinphi[row], cos_phi = cosphi[row];
        // the four columns' tables as 16-byte loads (col0 % 4 == 0), and the sensor's pose loaded once when the four
        // pixels share a sensor (every sensor width that is a multiple of 4)
        const float4 st4 = *reinterpret_cast<const float4*>(sinth + col0);
        const float4 ct4 = *reinterpret_cast<const float4*>(costh + col0);
        const float st_[4] = {st4.x, st4.y, st4.z, st4.w}, ct_[4] = {ct4.x, ct4.y, ct4.z, ct4.w};
        const int kA = 7 - col0 / rows;
        const bool one_sensor = kA == 7 - (col0 + 3) / rows;
        const float4* TA4 = reinterpret_cast<const float4*>(rt_inv + 16 * kA);
        const float4 ta0 = TA4[0], ta1 = TA4[1], ta2 = TA4[2], ta3 = TA4[3];
        const float TA[16] = {ta0.x, ta0.y, ta0.z, ta0.w, ta1.x, ta1.y, ta1.z, ta1.w,
                              ta2.x, ta2.y, ta2.z, ta2.w, ta3.x, ta3.y, ta3.z, ta3.w};
        unsigned char px[12];
        unsigned short dd4[4];
        unsigned pk4[4];
        float2 o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int col = col0 + e;
            const int k = 7 - col / rows;
            float T[16];
            if (one_sensor) {
#pragma unroll
                for (int t = 0; t < 16; ++t) T[t] = TA[t];
            } else {
#pragma unroll
                for (int t = 0; t < 16; ++t) T[t] = rt_inv[16 * k + t];
            }
            const float v1 = cos_phi * st_[e];
            const float v2 = cos_phi * ct_[e];
            float p0x = T[0] * v0 + T[4] * v1 + T[8] * v2;
            float p1 = T[1] * v0 + T[5] * v1 + T[9] * v2;
            float p2 = T[2] * v0 + T[6] * v1 + T[10] * v2;
            p0x = p0x + T[12]; p1 = p1 + T[13]; p2 = p2 + T[14];
            const float u = fx * p0x / p2 + cx;                          // :1133
            const float v = fy * p1 / p2 + cy;                           // :1134
            uint8_t b = 0, g = 0, r = 0;
            uint16_t dd = 0;
            if (u >= 0 && u < cols && v >= 0 && v < rows) {
                const int iu = (int)u, iv = (int)v;
                const long si = (long)k * rows * cols + (long)iv * cols + iu;
                b = bgr8[si * 3 + 0]; g = bgr8[si * 3 + 1]; r = bgr8[si * 3 + 2];
                const double du = (double)((u - cx) / fx), dv = (double)((v - cy) / fy);
                dd = (uint16_t)(depth8[si] * sqrt(1 + du * du + dv * dv));  // :1142 (range in mm)
            }
            px[3 * e] = b; px[3 * e + 1] = g; px[3 * e + 2] = r;
            dd4[e] = dd;
            const int y = (b * 4899 + g * 9617 + r * 1868 + (1 << 13)) >> 14;
            o[e] = make_float2((float)y * (float)(1. / 255), (float)dd * 0.001f);
            pk4[e] = dd | ((unsigned)y << 16);
        }
        uint3 wb;
        wb.x = px[0] | (px[1] << 8) | (px[2] << 16) | ((unsigned)px[3] << 24);
        wb.y = px[4] | (px[5] << 8) | (px[6] << 16) | ((unsigned)px[7] << 24);
        wb.z = px[8] | (px[9] << 8) | (px[10] << 16) | ((unsigned)px[11] << 24);
        *reinterpret_cast<uint3*>(sph_bgr + 12 * q) = wb;
        *reinterpret_cast<uint2*>(sph_depth + i0) = make_uint2(dd4[0] | ((unsigned)dd4[1] << 16),
                                                                 dd4[2] | ((unsigned)dd4[3] << 16));
        *reinterpret_cast<float4*>(p0 + i0) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
        *reinterpret_cast<float4*>(p0 + i0 + 2) = make_float4(o[2].x, o[2].y, o[3].x, o[3].y);
        *reinterpret_cast<uint4*>(pk + i0) = make_uint4(pk4[0], pk4[1], pk4[2], pk4[3]);
    }
}

// k_stitch with the sphere walked in 64-row x 16-column tiles, one wave per sphere column: a sphere column maps onto
// one sensor row (the sensors are mounted on their side: sphere rows run along sensor columns), so a wave's 64 gathers
// of BGR bytes and ranges read a few consecutive cache lines of one sensor row, where k_stitch4's row-major waves read
// 64 sensor rows (a line per byte).  The tile goes through LDS and is stored row-major as k_stitch4 stores it.  Per
// pixel the expressions of k_stitch (the sensor pose loaded once per column, which is one sensor), bit for bit.
constexpr int STT_R = 64, STT_C = 16;
__global__ void __launch_bounds__(256) k_stitch_t(const uint8_t* __restrict__ bgr8, const uint16_t* __restrict__ depth8,
                                                  int rows, int cols, int H, int W, const float* __restrict__ sinphi,
                                                  const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                                  const float* __restrict__ costh, const float* __restrict__ rt_inv,
                                                  float fx, float fy, float cx, float cy, uint8_t* __restrict__ sph_bgr,
                                                  uint16_t* __restrict__ sph_depth, float2* __restrict__ p0,
                                                  uint32_t* __restrict__ pk) {
    __shared__ uint32_t s_pk[STT_C][STT_R + 1];    // range mm | luma << 16
    __shared__ uint32_t s_bgr[STT_C][STT_R + 1];   // b | g << 8 | r << 16
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tiles_x = W / STT_C;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int row = ty * STT_R + lane;
    const bool in = row < H;
    const float v0 = in ? sinphi[row] : 0.f, cos_phi = in ? cosphi[row] : 0.f;
#pragma unroll
    for (int j = 0; j < STT_C / 4; ++j) {
        const int cl = w * (STT_C / 4) + j;
        const int col = __builtin_amdgcn_readfirstlane(tx * STT_C + cl);
        const int k = 7 - col / rows;
        const float* T = rt_inv + 16 * k;
        const float v1 = cos_phi * sinth[col];
        const float v2 = cos_phi * costh[col];
        float p0x = T[0] * v0 + T[4] * v1 + T[8] * v2;
        float p1 = T[1] * v0 + T[5] * v1 + T[9] * v2;
        float p2 = T[2] * v0 + T[6] * v1 + T[10] * v2;
        p0x = p0x + T[12]; p1 = p1 + T[13]; p2 = p2 + T[14];
        const float u = fx * p0x / p2 + cx;                          // :1133
        const float v = fy * p1 / p2 + cy;                           // :1134
        unsigned b = 0, g = 0, r = 0, dd = 0;
        if (in && u >= 0 && u < cols && v >= 0 && v < rows) {
            const int iu = (int)u, iv = (int)v;
            const long si = (long)k * rows * cols + (long)iv * cols + iu;
            b = bgr8[si * 3 + 0]; g = bgr8[si * 3 + 1]; r = bgr8[si * 3 + 2];
            const double du = (double)((u - cx) / fx), dv = (double)((v - cy) / fy);
            dd = (uint16_t)(depth8[si] * sqrt(1 + du * du + dv * dv));  // :1142 (range in mm)
        }
        const unsigned y = (b * 4899 + g * 9617 + r * 1868 + (1 << 13)) >> 14;
        s_pk[cl][lane] = dd | (y << 16);
        s_bgr[cl][lane] = b | (g << 8) | (r << 16);
    }
    __syncthreads();
    // row-major stores: thread t writes 4 consecutive pixels of tile row t / 4
    const int tr = threadIdx.x >> 2, c0 = (threadIdx.x & 3) * 4;
    const int grow = ty * STT_R + tr;
    if (grow >= H) return;
    const long i0 = (long)grow * W + tx * STT_C + c0;
    unsigned pk4[4], px[12];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        pk4[e] = s_pk[c0 + e][tr];
        const unsigned q = s_bgr[c0 + e][tr];
        px[3 * e] = q & 255; px[3 * e + 1] = (q >> 8) & 255; px[3 * e + 2] = q >> 16;
    }
    uint3 wb;
    wb.x = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
    wb.y = px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24);
    wb.z = px[8] | (px[9] << 8) | (px[10] << 16) | (px[11] << 24);
    *reinterpret_cast<uint3*>(sph_bgr + 3 * i0) = wb;
    *reinterpret_cast<uint2*>(sph_depth + i0) = make_uint2((pk4[0] & 0xffffu) | (pk4[1] << 16),
                                                            (pk4[2] & 0xffffu) | (pk4[3] << 16));
    float2 o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)   // setSourceFrame / setTargetFrame level 0: gray /255, depth * 0.001
        o[e] = make_float2((float)(pk4[e] >> 16) * (float)(1. / 255), (float)(pk4[e] & 0xffffu) * 0.001f);
    *reinterpret_cast<float4*>(p0 + i0) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
    *reinterpret_cast<float4*>(p0 + i0 + 2) = make_float4(o[2].x, o[2].y, o[3].x, o[3].y);
    *reinterpret_cast<uint4*>(pk + i0) = make_uint4(pk4[0], pk4[1], pk4[2], pk4[3]);
}

__device__ __forceinline__ int refl101(int p, int n) {
    p = p < 0 ? -p : p;
    return p >= n ? 2 * n - p - 2 : p;
}

// ------------------------------------------------------------------ pyramid (level l -> l+1)
// Level l's {gray, depth} through a loader: the float2 image, or level 0's packed image (4 B per pixel instead of
// 8: luma * (float)(1/255) and range * 0.001f are the stitch's own expressions, so the values are those of p0).
struct LvF2 {
    const float2* p;
    __device__ __forceinline__ float g(long i) const { return p[i].x; }
    __device__ __forceinline__ float d(long i) const { return p[i].y; }
    __device__ __forceinline__ float2 gd(long i) const { return p[i]; }
};
struct LvPk {
    const uint32_t* p;
    __device__ __forceinline__ float g(long i) const { return (float)(p[i] >> 16) * (float)(1. / 255); }
    __device__ __forceinline__ float d(long i) const { return (float)(p[i] & 0xffffu) * 0.001f; }
    __device__ __forceinline__ float2 gd(long i) const {
        const uint32_t v = p[i];
        return make_float2((float)(v >> 16) * (float)(1. / 255), (float)(v & 0xffffu) * 0.001f);
    }
};

// nimg images of R x C stored back to back (the sphere: 1; the per-sensor pyramids: 8)
// (32-bit index arithmetic: nimg * R * C < 2^31, checked by the launchers)
template <class IN>
__global__ void k_pyramid(const IN in_all, int R, int C, float2* __restrict__ out_all, float min_d, float max_d,
                          int nimg) {
    const int dr = R / 2, dc = C / 2;
    const unsigned per = (unsigned)(dr * dc), n = per * (unsigned)nimg;
    for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const unsigned img = nimg > 1 ? j / per : 0u;
        const unsigned i = j - img * per;
        const long in0 = (long)img * R * C;
        float2* out = out_all + (long)img * per;
        const int y = (int)(i / (unsigned)dc), x = (int)(i - (unsigned)y * dc);
        // cv::pyrDown: horizontal [1 4 6 4 1] per source row, then the vertical SSE order.
        const int sx = 2 * x;
        const int xa = refl101(sx - 2, C), xb = refl101(sx - 1, C), xd = refl101(sx + 1, C), xe = refl101(sx + 2, C);
        float h[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int yy = refl101(2 * y - 2 + k, R);
            const long s = in0 + (long)yy * C;
            const float a = in_all.g(s + xa), b = in_all.g(s + xb), c = in_all.g(s + sx), d = in_all.g(s + xd),
                        e = in_all.g(s + xe);
            h[k] = c * 6 + (b + d) * 4 + a + e;
        }
        float t0 = h[0] + h[4];
        const float t1 = (h[1] + h[3]) + h[2];
        t0 = t0 + (h[2] + h[2]);
        t0 = t0 + t1 * 4.f;
        const float gray = t0 * (1.f / 256);
        // buildPyramidRange: mean of the 2x2 depths in (minDepth, maxDepth) (:330-348)
        float av = 0.f; unsigned nv = 0;
        const long s0 = in0 + (long)(2 * y) * C + sx;
        const long s1 = s0 + C;
        const float z0 = in_all.d(s0), z1 = in_all.d(s0 + 1), z2 = in_all.d(s1), z3 = in_all.d(s1 + 1);
        if (z0 > min_d && z0 < max_d) { av += z0; ++nv; }
        if (z1 > min_d && z1 < max_d) { av += z1; ++nv; }
        if (z2 > min_d && z2 < max_d) { av += z2; ++nv; }
        if (z3 > min_d && z3 < max_d) { av += z3; ++nv; }
        out[i] = make_float2(gray, nv > 0 ? av / nv : 0.f);
    }
}

// ------------------------------------------------------------------ gradients + seam mask
__device__ __forceinline__ float harm(float fl, float f, float fr) {
    if ((f > fr && f < fl) || (f < fr && f > fl)) return 2.f / (1 / (fr - f) + 1 / (f - fl));
    return 0.f;
}

// seam = 1: the sphere (alignFrames360's seam mask); 0: per-sensor images (alignFrames has none)
__global__ void k_gradient(const float2* __restrict__ p0, int R, int C, float4* __restrict__ tg, int nimg,
                           int mask_seams) {
    const long per = (long)R * C, n = per * nimg;
    const int ws = C / 8;   // >= 1: calib_build_tables stops the pyramid before a level narrower than 8
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const long li = i % per;
        const int r = (int)(li / C), c = (int)(li - (long)r * C);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        // seam columns s*ws-1 and s*ws, s = 1..7, are zeroed by alignFrames360 (:4538-4549)
        const int m = ws > 0 ? c % ws : 1;
        const bool seam = mask_seams && ws > 0 && (c >= ws - 1) && (c < 7 * ws + 1) && (m == 0 || m == ws - 1);
        if (!seam && r >= 1 && r < R - 1 && c >= 1 && c < C - 1) {
            const float2 f = p0[i], fl = p0[i - 1], fr = p0[i + 1], fu = p0[i - C], fd = p0[i + C];
            o.x = harm(fl.x, f.x, fr.x);
            o.y = harm(fu.x, f.x, fd.x);
            o.z = harm(fl.y, f.y, fr.y);
            o.w = harm(fu.y, f.y, fd.y);
        }
        tg[i] = o;
    }
}

// all sphere levels' gradients in one launch (the levels are independent once the pyramid is built): block b
// belongs to the level l with blk0[l] <= b < blk0[l + 1], one pixel per thread
struct GradLevels {
    const float2* p0[R360_MAX_PYR];
    const uint32_t* pk0;   // level 0's packed image (read instead of p0[0] when set)
    float4* tg[R360_MAX_PYR];
    int rows[R360_MAX_PYR], cols[R360_MAX_PYR];
    int blk0[R360_MAX_PYR + 1];
    int nl;
};

// GRAD_PPT pixels per thread: a wave covers GRAD_PPT x 64 consecutive pixels, pixel k of a lane at i0 + 64 k (every
// load and store coalesced across the wave); the row and column of the first pixel come from one 32-bit division and
// are stepped by 64 columns for the others (one level search and one division per 4 pixels instead of per pixel:
// in the pipeline the launch had 12.8 k single-pixel-per-thread workgroups per frame)
constexpr int GRAD_PPT = 4;

template <class IN>
__device__ __forceinline__ void gradient_run(const IN p0, int i0, int R, int C, float4* __restrict__ tg) {
    const int ws = C / 8;   // >= 1: calib_build_tables stops the pyramid before a level narrower than 8
    const int n = R * C;
    int r = i0 / C, c = i0 - r * C;
#pragma unroll
    for (int k = 0; k < GRAD_PPT; ++k) {
        const int i = i0 + 64 * k;
        if (i >= n) break;
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        const int m = ws > 0 ? c % ws : 1;   // seam columns as k_gradient (alignFrames360 :4538-4549)
        const bool seam = ws > 0 && (c >= ws - 1) && (c < 7 * ws + 1) && (m == 0 || m == ws - 1);
        if (!seam && r >= 1 && r < R - 1 && c >= 1 && c < C - 1) {
            const float2 f = p0.gd(i), fl = p0.gd(i - 1), fr = p0.gd(i + 1), fu = p0.gd(i - C), fd = p0.gd(i + C);
            o.x = harm(fl.x, f.x, fr.x);
            o.y = harm(fu.x, f.x, fd.x);
            o.z = harm(fl.y, f.y, fr.y);
            o.w = harm(fu.y, f.y, fd.y);
        }
        tg[i] = o;
        c += 64;   // the lane's next pixel (C may be below 64 on the small levels: several rows on)
        while (c >= C) { c -= C; ++r; }
    }
}

__global__ void k_gradient_levels(GradLevels G) {
    int l = 0;
    while (l + 1 < G.nl && (int)blockIdx.x >= G.blk0[l + 1]) ++l;
    const int R = G.rows[l], C = G.cols[l];
    const int i0 = (int)((blockIdx.x - G.blk0[l]) * blockDim.x * GRAD_PPT + (threadIdx.x & ~63u) * GRAD_PPT +
                         (threadIdx.x & 63u));
    if (i0 >= R * C) return;
    if (l == 0 && G.pk0) gradient_run(LvPk{G.pk0}, i0, R, C, G.tg[0]);
    else gradient_run(LvF2{G.p0[l]}, i0, R, C, G.tg[l]);
}

// setSourceFrame / setTargetFrame level 0 of each sensor's raw images (:480-516): CV_RGB2GRAY on the
// BGR-stored data /255, and the u16 depth * 0.001 (buildPyramidRange :316-317)
// pk (optional): the packed level-0 image of the sphere (LevelBufs::pk)
__global__ void k_sensor_level0(const uint8_t* __restrict__ bgr8, const uint16_t* __restrict__ depth8, long n,
                                float2* __restrict__ p0, uint32_t* __restrict__ pk) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int b = bgr8[3 * i], g = bgr8[3 * i + 1], r = bgr8[3 * i + 2];
        const int y = (b * 4899 + g * 9617 + r * 1868 + (1 << 13)) >> 14;
        p0[i] = make_float2((float)y * (float)(1. / 255), (float)depth8[i] * 0.001f);
        if (pk) pk[i] = depth8[i] | ((unsigned)y << 16);
    }
}

inline int grid_for(long n) {
    long b = (n + TPB - 1) / TPB;
    return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

// ------------------------------------------------------------------ launchers
int launch_undistort(r360_frame* f) {
    const r360_calib* c = f->calib;
    const long n = (long)R360_NUM_SENSORS * f->rows * f->cols;
    const bool apply = c->has_intrinsics && c->clams.width == f->cols && c->clams.height == f->rows;
    if (f->cols % 4 == 0) {
        hipLaunchKernelGGL(k_undistort4, dim3(grid_for(n / 4)), dim3(TPB), 0, f->ctx->stream, f->d_depth, f->d_depth_m,
                           f->rows, f->cols, c->clams.d_mult, c->clams.d_counts, c->clams.nx, c->clams.bin_w,
                           c->clams.bin_h, c->clams.num_bins, c->clams.bin_depth, apply ? 1 : 0);
        R360_HIP(hipGetLastError());
        return 0;
    }
    hipLaunchKernelGGL(k_undistort, dim3(grid_for(n)), dim3(TPB), 0, f->ctx->stream, f->d_depth, f->d_depth_m, f->rows,
                       f->cols, c->clams.d_mult, c->clams.d_counts, c->clams.nx, c->clams.bin_w, c->clams.bin_h,
                       c->clams.num_bins, c->clams.bin_depth, apply ? 1 : 0);
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_stitch(r360_frame* f) {
    const r360_calib* c = f->calib;
    const long n = (long)f->sph_rows * f->sph_cols;
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(f->ctx->stream, e, 0));   // a split upload's BGR copy
    const int slot = timing_begin(f->ctx, "k_stitch");
    // experiment builds: R360_STITCH=4 forces the row-major k_stitch4
    static const int form = R360_KNOB("R360_STITCH", 0);
    if (f->sph_cols % STT_C == 0 && form != 4)
        hipLaunchKernelGGL(k_stitch_t, dim3((f->sph_cols / STT_C) * ((f->sph_rows + STT_R - 1) / STT_R)), dim3(256), 0,
                           f->ctx->stream, f->d_bgr, f->d_depth, f->rows, f->cols, f->sph_rows, f->sph_cols,
                           c->d_st_sinphi, c->d_st_cosphi, c->d_st_sinth, c->d_st_costh, c->d_rt_inv, c->K[0], c->K[4],
                           c->K[6], c->K[7], f->d_sph_bgr, f->d_sph_depth, f->lv[0].p0, f->lv[0].pk);
    else if (f->sph_cols % 4 == 0)
        hipLaunchKernelGGL(k_stitch4, dim3(grid_for(n / 4)), dim3(TPB), 0, f->ctx->stream, f->d_bgr, f->d_depth,
                           f->rows, f->cols, f->sph_rows, f->sph_cols, c->d_st_sinphi, c->d_st_cosphi, c->d_st_sinth,
                           c->d_st_costh, c->d_rt_inv, c->K[0], c->K[4], c->K[6], c->K[7], f->d_sph_bgr,
                           f->d_sph_depth, f->lv[0].p0, f->lv[0].pk);
    else
        hipLaunchKernelGGL(k_stitch, dim3(grid_for(n)), dim3(TPB), 0, f->ctx->stream, f->d_bgr, f->d_depth, f->rows,
                           f->cols, f->sph_rows, f->sph_cols, c->d_st_sinphi, c->d_st_cosphi, c->d_st_sinth,
                           c->d_st_costh, c->d_rt_inv, c->K[0], c->K[4], c->K[6], c->K[7], f->d_sph_bgr,
                           f->d_sph_depth, f->lv[0].p0, f->lv[0].pk);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}

// ------------------------------------------------------------------ ICP source points
// The source side of errorPhotoICP_sphere / calcHessGrad_sphere reads, per pixel with
// minDepth < depth < maxDepth, the LUT_xyz_sphere point (RegisterPhotoICP.h:4553-4587, the same float
// expressions) and the gray value; both are fixed for a source frame.  They are compacted here once per
// frame, in raster order (a deterministic two-kernel scan), so the pass streams only valid pixels.
// A block covers R360_SRC_BLOCK consecutive pixels, SRC_PPT consecutive ones per thread (256-thread workgroups: a
// 1024-thread one had to find 16 free wave slots on one CU, which under load delayed the frame's build).
constexpr int SRC_PPT = 16, SRC_TPB = R360_SRC_BLOCK / SRC_PPT;

// flattened (level, block) grid: level l owns blocks [blk0[l], blk0[l + 1]) (the coarse levels need a quarter, a
// sixteenth ... of level 0's blocks; a 2D grid sized for level 0 dispatched thousands of empty workgroups)
struct SrcGrid { int blk0[R360_MAX_PYR + 1]; int nl; };
__device__ __forceinline__ void src_block(const SrcGrid& G, int& level, int& b) {
    const int bid = blockIdx.x;
    level = 0;
    while (level + 1 < G.nl && bid >= G.blk0[level + 1]) ++level;
    b = bid - G.blk0[level];
}

__device__ __forceinline__ bool src_valid(float d, float min_d, float max_d) { return min_d < d && d < max_d; }

__global__ void __launch_bounds__(SRC_TPB) k_src_count(const SrcLevel* __restrict__ L, SrcGrid G, float min_d, float max_d,
                                                      int* __restrict__ cnt, int stride) {
    int lvl, bx;
    src_block(G, lvl, bx);
    const SrcLevel S = L[lvl];
    const long n = (long)S.rows * S.cols;
    const long b0 = (long)bx * R360_SRC_BLOCK;
    if (b0 >= n) return;
    int c = 0;
#pragma unroll
    for (int k = 0; k < SRC_PPT; ++k) {
        const long i = b0 + k * SRC_TPB + threadIdx.x;
        c += (i < n && src_valid(S.p0[i].y, min_d, max_d)) ? 1 : 0;
    }
    __shared__ int sh[SRC_TPB / 64];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < SRC_TPB / 64; ++w) t += sh[w];
        cnt[lvl * stride + bx] = t;
    }
}

__global__ void __launch_bounds__(SRC_TPB) k_src_compact(const SrcLevel* __restrict__ L, SrcGrid G, float min_d,
                                                        float max_d, const int* __restrict__ cnt, int stride,
                                                        int* __restrict__ npts) {
    int lvl, bx;
    src_block(G, lvl, bx);
    const SrcLevel S = L[lvl];
    const long n = (long)S.rows * S.cols;
    const long b0 = (long)bx * R360_SRC_BLOCK;
    if (b0 >= n) return;
    __shared__ int sh[SRC_TPB / 64 + 1];
    // this block's output offset: the counts of the blocks before it
    int base = 0;
    for (int b = threadIdx.x; b < bx; b += SRC_TPB) base += cnt[lvl * stride + b];
    for (int o = 32; o > 0; o >>= 1) base += __shfl_xor(base, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = base;
    __syncthreads();
    base = 0;
    for (int w = 0; w < SRC_TPB / 64; ++w) base += sh[w];
    __syncthreads();
    // raster order: the block's pixels as SRC_PPT rows of SRC_TPB, pixel b0 + k SRC_TPB + t (coalesced loads); a
    // pixel's slot = the valid pixels of the rows before k, then of the waves before this one in row k, then of the
    // lanes before it (ballot masks: one LDS round for the whole block)
    __shared__ int s_cnt[SRC_PPT][SRC_TPB / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    float2 a[SRC_PPT];
    unsigned long long m[SRC_PPT];
#pragma unroll
    for (int k = 0; k < SRC_PPT; ++k) {
        const long i = b0 + (long)k * SRC_TPB + threadIdx.x;
        a[k] = i < n ? S.p0[i] : make_float2(0.f, 0.f);
        m[k] = __ballot(i < n && src_valid(a[k].y, min_d, max_d));
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < SRC_PPT; ++k) s_cnt[k][wid] = __popcll(m[k]);
    __syncthreads();
    int pos = base;
#pragma unroll
    for (int k = 0; k < SRC_PPT; ++k) {
        int before = pos, row = 0;
#pragma unroll
        for (int w = 0; w < SRC_TPB / 64; ++w) {
            const int cw = s_cnt[k][w];
            before += w < wid ? cw : 0;
            row += cw;
        }
        if ((m[k] >> lane) & 1ull) {
            const long i = b0 + (long)k * SRC_TPB + threadIdx.x;
            const int r = (int)(i / S.cols), cc = (int)(i - (long)r * S.cols);
            const float d = a[k].y;
            // LUT_xyz_sphere (:4580-4582): x = d sin(phi), y = -d cos(phi) sin(theta), z = -d cos(phi) cos(theta)
            S.pts[before + __popcll(m[k] & lt)] =
                make_float4(d * S.sinphi[r], -d * S.cosphi[r] * S.sinth[cc], -d * S.cosphi[r] * S.costh[cc], a[k].x);
        }
        pos += row;
    }
    if (bx == (int)((n - 1) / R360_SRC_BLOCK) && threadIdx.x == SRC_TPB - 1) npts[lvl] = pos;
}

int launch_sphere_level0(r360_frame* f) {
    const long n = (long)f->sph_rows * f->sph_cols;
    // cvtColor(CV_RGB2GRAY) / 255 and convertTo(CV_32F, 0.001): the stitch kernel's level-0 expressions
    hipLaunchKernelGGL(k_sensor_level0, dim3(grid_for(n)), dim3(TPB), 0, f->ctx->stream, f->d_sph_bgr, f->d_sph_depth,
                       n, f->lv[0].p0, f->lv[0].pk);
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_pyramid(r360_frame* f) {
    // RegisterPhotoICP constructor defaults minDepth 0.3 / maxDepth 6.0 (:202-203)
    const float min_d = 0.3f, max_d = 6.0f;
    if ((long)f->lv[0].rows * f->lv[0].cols > 0x7fffffffL - 4096) {   // 32-bit pixel indices
        r360_set_error("sphere of %d x %d pixels is too large", f->lv[0].rows, f->lv[0].cols);
        return -1;
    }
    static const bool pyr_f2 = R360_KNOB("R360_PYR_F2", 0) != 0;   // experiment builds: level 0 read as float2
    for (int l = 1; l < f->n_levels; ++l) {
        const long n = (long)f->lv[l].rows * f->lv[l].cols;
        // level 1 from level 0's packed image (half the bytes of its float2 image, the same values)
        if (l == 1 && f->lv[0].pk && !pyr_f2)
            hipLaunchKernelGGL(k_pyramid<LvPk>, dim3(grid_for(n)), dim3(TPB), 0, f->ctx->stream, LvPk{f->lv[0].pk},
                               f->lv[0].rows, f->lv[0].cols, f->lv[1].p0, min_d, max_d, 1);
        else
            hipLaunchKernelGGL(k_pyramid<LvF2>, dim3(grid_for(n)), dim3(TPB), 0, f->ctx->stream, LvF2{f->lv[l - 1].p0},
                               f->lv[l - 1].rows, f->lv[l - 1].cols, f->lv[l].p0, min_d, max_d, 1);
    }
    {
        GradLevels GL{};
        GL.nl = f->n_levels;
        GL.pk0 = pyr_f2 ? nullptr : f->lv[0].pk;
        for (int l = 0; l < f->n_levels; ++l) {
            GL.p0[l] = f->lv[l].p0;
            GL.tg[l] = f->lv[l].tg;
            GL.rows[l] = f->lv[l].rows;
            GL.cols[l] = f->lv[l].cols;
            GL.blk0[l + 1] = GL.blk0[l] + (int)(((long)f->lv[l].rows * f->lv[l].cols + TPB * GRAD_PPT - 1) / (TPB * GRAD_PPT));
        }
        hipLaunchKernelGGL(k_gradient_levels, dim3(GL.blk0[f->n_levels]), dim3(TPB), 0, f->ctx->stream, GL);
    }
    // the compacted points feed a lone alignment's passes (PF 5); batched passes stream the images (PF 6 at level 0
    // where its rows split into whole waves, PF 8 on levels of >= 64 columns), so frames that only enter batches
    // (f->compact_all unset: the sequence runner's queued ring) skip the levels a batched pass streams (built on
    // request: r360_frame_get_points, or a form forced by R360_ICP_PF)
    static const int pf_env = R360_KNOB("R360_ICP_PF", -1);
    const bool skip_ok = !f->compact_all && !(pf_env == 4 || pf_env == 5);
    unsigned need = 0;
    for (int l = 0; l < f->n_levels; ++l) {
        static const bool coarse_pf5 = R360_KNOB("R360_COARSE_PF5", 0) != 0;   // experiment builds (icp_kernels.hip)
        const bool streamed = l == 0 && f->lv[0].pk ? f->lv[0].cols % 64 == 0 : f->lv[l].cols >= 64 && !coarse_pf5;
        if (!skip_ok || !streamed) need |= 1u << l;
    }
    f->compacted = need;
    return launch_src_compaction(f, need);
}

// The compaction of the levels in `levels` (bit l: level l), one count + one compact launch over a flattened
// (level, block) grid
int launch_src_compaction(r360_frame* f, unsigned levels) {
    const float min_d = 0.3f, max_d = 6.0f;
    int l1 = 0;
    for (int l = 0; l < f->n_levels; ++l)
        if ((levels >> l) & 1u) l1 = l + 1;
    if (l1 == 0) return 0;
    SrcGrid G{};
    G.nl = l1;
    for (int l = 0; l < l1; ++l)
        G.blk0[l + 1] = G.blk0[l] + (((levels >> l) & 1u) ? (int)(((long)f->lv[l].rows * f->lv[l].cols + R360_SRC_BLOCK - 1) /
                                                                      R360_SRC_BLOCK) : 0);
    const dim3 g(G.blk0[l1]);
    hipLaunchKernelGGL(k_src_count, g, dim3(SRC_TPB), 0, f->ctx->stream, f->d_src_levels, G, min_d, max_d, f->d_src_cnt,
                       f->src_blocks);
    hipLaunchKernelGGL(k_src_compact, g, dim3(SRC_TPB), 0, f->ctx->stream, f->d_src_levels, G, min_d, max_d,
                       f->d_src_cnt, f->src_blocks, f->d_npts);
    R360_HIP(hipGetLastError());
    return 0;
}

// The 8 sensors' pinhole pyramids (RegisterPhotoICP::setSourceFrame / setTargetFrame on
// frameRGBD_[k].getRGBImage() / getDepthImage(), MethodsRegisterRGBD360.cpp:337-338), all sensors per
// launch.  Levels are allocated on first use.
int launch_sensor_pyramid(r360_frame* f) {
    const float min_d = 0.3f, max_d = 6.0f;
    if (!f->n_slevels) {
        int R = f->rows, C = f->cols, nl = 0;
        while (nl < R360_MAX_PYR) {
            f->sp[nl].rows = R; f->sp[nl].cols = C;
            R360_HIP(hipMalloc(&f->sp[nl].p0, sizeof(float2) * 8 * (size_t)R * C));
            R360_HIP(hipMalloc(&f->sp[nl].tg, sizeof(float4) * 8 * (size_t)R * C));
            ++nl;
            if ((R & 1) || (C & 1) || R < 8 || C < 8) break;   // cv::pyrDown halves exactly only even sizes
            R /= 2; C /= 2;
        }
        f->n_slevels = nl;
    }
    hipStream_t st = f->ctx->stream;
    const long n0 = 8L * f->rows * f->cols;
    if (n0 > 0x7fffffffL) {   // k_pyramid's 32-bit pixel indices
        r360_set_error("sensor images of %d x %d pixels are too large", f->rows, f->cols);
        return -1;
    }
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(st, e, 0));   // a split upload's BGR copy
    hipLaunchKernelGGL(k_sensor_level0, dim3(grid_for(n0)), dim3(TPB), 0, st, f->d_bgr, f->d_depth, n0, f->sp[0].p0,
                       (uint32_t*)nullptr);
    for (int l = 1; l < f->n_slevels; ++l) {
        const long n = 8L * f->sp[l].rows * f->sp[l].cols;
        hipLaunchKernelGGL(k_pyramid<LvF2>, dim3(grid_for(n)), dim3(TPB), 0, st, LvF2{f->sp[l - 1].p0}, f->sp[l - 1].rows,
                           f->sp[l - 1].cols, f->sp[l].p0, min_d, max_d, 8);
    }
    for (int l = 0; l < f->n_slevels; ++l) {
        const long n = 8L * f->sp[l].rows * f->sp[l].cols;
        hipLaunchKernelGGL(k_gradient, dim3(grid_for(n)), dim3(TPB), 0, st, f->sp[l].p0, f->sp[l].rows, f->sp[l].cols,
                           f->sp[l].tg, 8, 0);
    }
    R360_HIP(hipGetLastError());
    return 0;
}
