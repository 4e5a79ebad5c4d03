// plane_kernels.hip — the per-pixel plane half of Frame360 on gfx950:
//   k_cloud       back-projection + 2x2 upper-median downsample   (CloudRGBD_Ext.h:78-139,
//                 DownsampleRGBD.h:209-311)
//   k_bil_*       pcl::FastBilateralFilter (sigma_s 10, sigma_r 0.05): splat / fused blur / slice
//   k_dcm         depth-change map + distance-map init            (IntegralImageNormalEstimation)
//   k_distmap     two-pass chamfer distance map, row bands with halos (exact below the 9.5 cap)
//   k_normals     AVERAGE_3D_GRADIENT normals from exact window sums + plane offset d = p.n
//   CCL, plane fit, refinement, boundary trace and statistics: plane_seg.hip
//
// Every float expression is the oracle's (oracle/src/planes_oracle.cpp), compiled with
// -ffp-contract=off, so the outputs are bit-identical.  Layout: per frame, 8 organized clouds of
// w x h = (cols/2) x (rows/2) points, sensor after sensor; float4 {x, y, z, 0}, uchar4 {r, g, b, 0}.
#include "../r360_internal.h"

namespace {

__device__ __forceinline__ bool isfin(float v) { return __builtin_isfinite(v); }

// ------------------------------------------------------------------ A3
// order-preserving float <-> int map for integer atomic min / max
__device__ __forceinline__ int f2ord(float f) {
    const int b = __float_as_int(f);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int e) { return __int_as_float(e >= 0 ? e : e ^ 0x7fffffff); }
constexpr int kOrdMinInit = 0x7f7f7f7f;            // memset byte 0x7f: above every finite float
constexpr int kOrdMaxInit = (int)0x80808080;       // memset byte 0x80: below every finite float

// one output point of k_cloud; returns its z
__device__ __forceinline__ float cloud_point_impl(const float* __restrict__ depth_m, int rows, int cols, float inv_f,
                                                  float ox, float oy, float4* __restrict__ cloud, long i, int w, long N,
                                                  float nan) {
    {
        const int s = (int)(i / N);
        const int j = (int)(i - (long)s * N);
        const int r2 = j / w, c2 = j - (j / w) * w;
        const int r = 2 * r2, c = 2 * c2;
        const float* D = depth_m + (long)s * rows * cols;
        float xs[4], ys[4], zs[4];
        int n = 0;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const float z = D[(long)(r + rr) * cols + c + cc];
                if (z > 0 && z >= 0.3f && z <= 10.0f && 0.3f < z && z < 5.0f) {
                    xs[n] = ((float)(c + cc) - ox) * z * inv_f;
                    ys[n] = ((float)(r + rr) - oy) * z * inv_f;
                    zs[n] = z;
                    ++n;
                }
            }
        float4 o;
        if (n > 0) {
            // insertion sorts; element n/2 is the upper median (std::sort + [n/2])
            for (int a = 1; a < n; ++a)
                for (int b = a; b > 0; --b) {
                    if (xs[b - 1] > xs[b]) { const float t = xs[b]; xs[b] = xs[b - 1]; xs[b - 1] = t; }
                    if (ys[b - 1] > ys[b]) { const float t = ys[b]; ys[b] = ys[b - 1]; ys[b - 1] = t; }
                    if (zs[b - 1] > zs[b]) { const float t = zs[b]; zs[b] = zs[b - 1]; zs[b - 1] = t; }
                }
            o = make_float4(xs[n / 2], ys[n / 2], zs[n / 2], 0.f);
        } else {  // copy the centre point (r+1, c+1), possibly finite with 5 <= z <= 10
            const float z = D[(long)(r + 1) * cols + c + 1];
            if (z > 0 && z >= 0.3f && z <= 10.0f)
                o = make_float4(((float)(c + 1) - ox) * z * inv_f, ((float)(r + 1) - oy) * z * inv_f, z, 0.f);
            else
                o = make_float4(nan, nan, nan, 0.f);
        }
        cloud[i] = o;   // its colour: k_rgb (the BGR images may still be on their way, r360_ctx::split_upload)
        return o.z;
    }
}

__device__ __forceinline__ void d_cloud(const float* __restrict__ depth_m, int rows, int cols, float inv_f, float ox,
                                        float oy, float4* __restrict__ cloud, int* __restrict__ zmm, int* __restrict__ wmm) {
    const int w = cols / 2, h = rows / 2;
    const long N = (long)w * h, total = 8 * N;
    const float nan = __builtin_nanf("");
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i0 = blockIdx.x * (long)blockDim.x + (threadIdx.x & ~63); i0 < total; i0 += stride) {
        const long i = i0 + (threadIdx.x & 63);
        // per-sensor min / max of the finite depths (the bilateral filter's range), wave-reduced
        int emin = kOrdMinInit, emax = kOrdMaxInit;
        const int s0 = (int)(i0 / N);
        if (i < total) {
            const float z = cloud_point_impl(depth_m, rows, cols, inv_f, ox, oy, cloud, i, w, N, nan);
            if (isfin(z)) { emin = f2ord(z); emax = emin; }
        }
        const bool one_sensor = (i0 + 63 < total) && ((i0 + 63) / N == s0);
        if (one_sensor) {   // per-wave partial, reduced per sensor by k_zrange (no contended atomics)
            for (int o = 32; o > 0; o >>= 1) {
                emin = min(emin, __shfl_xor(emin, o, 64));
                emax = max(emax, __shfl_xor(emax, o, 64));
            }
            if ((threadIdx.x & 63) == 0) {
                wmm[2 * (i0 >> 6)] = emin;
                wmm[2 * (i0 >> 6) + 1] = emax;
            }
        } else if (i < total && emin != kOrdMinInit) {
            const int s = (int)(i / N);
            atomicMin(zmm + s, emin);
            atomicMax(zmm + 8 + s, emax);
        }
    }
}
__global__ void k_cloud(const PlaneBatch B, int rows, int cols, float inv_f, float ox, float oy) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_cloud(D.depth_m, rows, cols, inv_f, ox, oy, D.cloud, D.zmm, reinterpret_cast<int*>(D.dist0));
}

// the organized clouds' colours: point (r2, c2) of a sensor takes the BGR pixel (2 r2 + 1, 2 c2 + 1) as {r, g, b, 0}
// (CloudRGBD_Ext.h:78-139, DownsampleRGBD.h:209-311: the centre pixel of the 2x2 block)
__global__ void k_rgb(const PlaneBatch B, int rows, int cols) {
    const PlaneDev& D = B.f[blockIdx.z];
    const int w = cols / 2, h = rows / 2;
    const long N = (long)w * h, total = 8 * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        const int j = (int)(i - (long)s * N);
        const int r2 = j / w, c2 = j - r2 * w;
        const uint8_t* b = D.bgr + ((long)s * rows * cols + (long)(2 * r2 + 1) * cols + 2 * c2 + 1) * 3;
        D.rgb[i] = make_uchar4(b[2], b[1], b[0], 0);
    }
}



// the frame's plane stage starts: depth-range accumulators and the error word (one launch instead of memsets)
__device__ __forceinline__ void d_plane_begin(int* __restrict__ zmm, int* __restrict__ err) {
    const int t = threadIdx.x;
    if (t < 8) zmm[t] = kOrdMinInit;
    else if (t < 16) zmm[t] = kOrdMaxInit;
    if (t == 0) *err = 0;
}
__global__ void k_plane_begin(const PlaneBatch B) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_plane_begin(D.zmm, D.err);
}


// per-sensor depth range from k_cloud's per-wave partials (waves inside one sensor)
__device__ __forceinline__ void d_zrange(const int* __restrict__ wmm, long N, int* __restrict__ zmm) {
    __shared__ int smin[16], smax[16];
    const int s = blockIdx.x;
    const long w0 = (s * N + 63) / 64, w1 = ((s + 1) * N) / 64;   // waves starting inside the sensor
    int emin = kOrdMinInit, emax = kOrdMaxInit;
    for (long w = w0 + threadIdx.x; w < w1; w += blockDim.x) {
        if ((w * 64 + 63) / N != s) continue;                      // straddling wave: atomics in k_cloud
        emin = min(emin, wmm[2 * w]);
        emax = max(emax, wmm[2 * w + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        emin = min(emin, __shfl_xor(emin, o, 64));
        emax = max(emax, __shfl_xor(emax, o, 64));
    }
    if ((threadIdx.x & 63) == 0) { smin[threadIdx.x >> 6] = emin; smax[threadIdx.x >> 6] = emax; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < (int)(blockDim.x >> 6); ++q) { emin = min(emin, smin[q]); emax = max(emax, smax[q]); }
        if (emin != kOrdMinInit) {
            atomicMin(zmm + s, emin);
            atomicMax(zmm + 8 + s, emax);
        }
    }
}
__global__ void __launch_bounds__(1024) k_zrange(const PlaneBatch B, long N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_zrange(reinterpret_cast<const int*>(D.dist0), N, D.zmm);
}


// ------------------------------------------------------------------ A4
// pcl::FastBilateralFilter as four fully parallel kernels over the 8 sensors:
//   splat  one thread per (sx, sy) grid column, the column's sd cells accumulated in LDS in the
//          reference's x-major / y-minor pixel order (so every cell sum has the reference's order);
//   blur   per axis the two [1 2 1]/4 iterations fused (each output cell recomputes the three
//          first-iteration cells it needs, with the same float expressions), boundaries zero;
//   slice  trilinear interpolation, z <- D0 / D1.
// Grids are stored z-major ([sz][sy][sx]); the depth range comes from k_cloud's atomics.
constexpr int BIL_SD_MAX = 208;
constexpr int BIL_COLS = 64;

// depth range and grid depth of sensor s; false when the filter does not run (no finite depth, or
// a range beyond the grid capacity, which is flagged)
__device__ __forceinline__ bool bil_params(const int* __restrict__ zmm, int s, int sd_max, float& bmin, float& bmax,
                                           long& sd, bool& over) {
    over = false;
    const int emax = zmm[8 + s];
    if (emax == kOrdMaxInit) return false;
    bmin = ord2f(zmm[s]);
    bmax = ord2f(emax);
    const float base_delta = bmax - bmin;
    sd = (long)(unsigned long)(base_delta / 0.05f) + 5;
    over = sd > sd_max;
    return !over;
}

__device__ __forceinline__ void d_bil_splat(const float4* __restrict__ cloud_all, int w, int h, long sw,
                                                       long sh, const int* __restrict__ zmm, int sd_max,
                                                       float2* __restrict__ grids, long grid_cells,
                                                       int* __restrict__ err) {
    __shared__ float cx[BIL_SD_MAX][BIL_COLS], cy[BIL_SD_MAX][BIL_COLS];
    const int s = blockIdx.y, t = threadIdx.x;
    float bmin, bmax;
    long sd;
    bool over;
    if (!bil_params(zmm, s, sd_max, bmin, bmax, sd, over)) {
        if (over && blockIdx.x == 0 && t == 0) atomicOr(err, 1);
        return;
    }
    const float sigma_s = 10.0f, sigma_r = 0.05f;
    const long ncol = sw * sh;
    const long col = (long)blockIdx.x * BIL_COLS + t;
    if (col >= ncol) return;
    for (long z = 0; z < sd; ++z) { cx[z][t] = 0.f; cy[z][t] = 0.f; }
    const float4* cloud = cloud_all + (long)s * w * h;
    const int sx = (int)(col % sw), sy = (int)(col / sw);
    const int x0 = max(0, 10 * (sx - 2) - 6), x1 = min(w - 1, 10 * (sx - 2) + 6);
    const int y0 = max(0, 10 * (sy - 2) - 6), y1 = min(h - 1, 10 * (sy - 2) + 6);
    for (int x = x0; x <= x1; ++x) {
        if ((long)(unsigned long)((float)x / sigma_s + 0.5f) + 2 != sx) continue;
        // the column's depths of this x, all loads in flight before the ordered accumulation (y1 - y0 <= 12)
        float zr[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) zr[k] = y0 + k <= y1 ? cloud[(long)(y0 + k) * w + x].z : 0.f;
#pragma unroll
        for (int k = 0; k < 13; ++k) {
            const int y = y0 + k;
            if (y > y1 || (long)(unsigned long)((float)y / sigma_s + 0.5f) + 2 != sy) continue;
            float Z = zr[k];
            if (!isfin(Z)) Z = bmax;                           // NaN depths take the range maximum
            const float z = Z - bmin;
            const long sz = (long)(unsigned long)(z / sigma_r + 0.5f) + 2;
            cx[sz][t] += Z;
            cy[sz][t] += 1.0f;
        }
    }
    float2* A = grids + (long)s * 2 * grid_cells;
    for (long z = 0; z < sd; ++z) A[z * ncol + col] = make_float2(cx[z][t], cy[z][t]);
}
__global__ void __launch_bounds__(BIL_COLS) k_bil_splat(const PlaneBatch B, int w, int h, long sw, long sh, int sd_max, long grid_cells) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_bil_splat(D.cloud, w, h, sw, sh, D.zmm, sd_max, D.grids, grid_cells, D.err);
}


template <int AX>
__device__ __forceinline__ void d_bil_blur(float2* __restrict__ grids, long grid_cells, int src_slot, long sw, long sh,
                           const int* __restrict__ zmm, int sd_max) {
    const int s = blockIdx.y;
    float bmin, bmax;
    long sd;
    bool over;
    if (!bil_params(zmm, s, sd_max, bmin, bmax, sd, over)) return;
    const long ncol = sw * sh, cells = sd * ncol;
    const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cells) return;
    const float2* src = grids + (long)s * 2 * grid_cells + (long)src_slot * grid_cells;
    float2* dst = grids + (long)s * 2 * grid_cells + (long)(1 - src_slot) * grid_cells;
    const long z = c / ncol, col = c - z * ncol, y = col / sw, x = col - y * sw;
    const long o = AX == 0 ? 1 : (AX == 1 ? sw : ncol);
    const long a0 = AX == 0 ? x : (AX == 1 ? y : z);           // coordinate along the axis
    const long an = AX == 0 ? sw : (AX == 1 ? sh : sd);
    const bool other_bnd = AX == 0 ? (y <= 0 || y >= sh - 1 || z <= 0 || z >= sd - 1)
                                   : AX == 1 ? (x <= 0 || x >= sw - 1 || z <= 0 || z >= sd - 1)
                                             : (x <= 0 || x >= sw - 1 || y <= 0 || y >= sh - 1);
    if (other_bnd || a0 <= 0 || a0 >= an - 1) { dst[c] = make_float2(0.f, 0.f); return; }
    // first iteration at axis offsets -1, 0, +1 (zero on the boundary)
    float2 b1[3];
#pragma unroll
    for (int k = -1; k <= 1; ++k) {
        const long ak = a0 + k;
        if (ak <= 0 || ak >= an - 1) { b1[k + 1] = make_float2(0.f, 0.f); continue; }
        const long q = c + k * o;
        const float2 a = src[q - o], b = src[q + o], m = src[q];
        b1[k + 1] = make_float2((a.x + b.x + 2.0f * m.x) / 4.0f, (a.y + b.y + 2.0f * m.y) / 4.0f);
    }
    dst[c] = make_float2((b1[0].x + b1[2].x + 2.0f * b1[1].x) / 4.0f, (b1[0].y + b1[2].y + 2.0f * b1[1].y) / 4.0f);
}
template <int AX>
__global__ void k_bil_blur(const PlaneBatch B, long grid_cells, int src_slot, long sw, long sh, int sd_max) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_bil_blur<AX>(D.grids, grid_cells, src_slot, sw, sh, D.zmm, sd_max);
}


// The three axis passes in one launch: a workgroup stages a BT_X x BT_Y x BT_Z tile of the splat grid with a 2-cell
// halo in LDS, blurs along x over the tile's y / z halo, then along y over its z halo, then along z, and writes the
// tile once (the three launches read and wrote the whole grid three times).  Every cell is computed by d_bil_blur's
// expressions from the same inputs, so the result is that of the three passes bit for bit; a halo cell outside the
// grid is staged as zero and never enters an interior cell's value (a pass reads only in-grid neighbours of interior
// cells, and every boundary cell of every pass is zero).
constexpr int BT_X = 16, BT_Y = 8, BT_Z = 4, BT_TPB = 256;
constexpr int BT_SX = BT_X + 4, BT_SY = BT_Y + 4, BT_SZ = BT_Z + 4;

__device__ __forceinline__ float2 bil_121(float2 a, float2 b, float2 m) {
    return make_float2((a.x + b.x + 2.0f * m.x) / 4.0f, (a.y + b.y + 2.0f * m.y) / 4.0f);
}
// one pass's output at axis coordinate a0 (extent an) from the five values v[0..4] at a0 - 2 .. a0 + 2; zero when the
// cell is on a boundary of the grid (bnd: of the other two axes, or of this one)
__device__ __forceinline__ float2 bil_pass(const float2 (&v)[5], long a0, long an, bool bnd) {
    if (bnd || a0 <= 0 || a0 >= an - 1) return make_float2(0.f, 0.f);
    float2 b1[3];
#pragma unroll
    for (int k = -1; k <= 1; ++k) {
        const long ak = a0 + k;
        b1[k + 1] = (ak <= 0 || ak >= an - 1) ? make_float2(0.f, 0.f) : bil_121(v[k + 1], v[k + 3], v[k + 2]);
    }
    return make_float2((b1[0].x + b1[2].x + 2.0f * b1[1].x) / 4.0f, (b1[0].y + b1[2].y + 2.0f * b1[1].y) / 4.0f);
}

__global__ void __launch_bounds__(BT_TPB) k_bil_blur3(const PlaneBatch B, long grid_cells, long sw, long sh, int sd_max) {
    __shared__ float2 S[BT_SZ][BT_SY][BT_SX];   // source tile + halo
    __shared__ float2 XB[BT_SZ][BT_SY][BT_X];   // after the x pass
    __shared__ float2 YB[BT_SZ][BT_Y][BT_X];    // after the y pass
    const PlaneDev& D = B.f[blockIdx.z / 8];
    const int s = blockIdx.z & 7;
    float bmin, bmax;
    long sd;
    bool over;
    if (!bil_params(D.zmm, s, sd_max, bmin, bmax, sd, over)) return;
    const long ntx = (sw + BT_X - 1) / BT_X;
    const long x0 = (long)(blockIdx.x % ntx) * BT_X, y0 = (long)(blockIdx.x / ntx) * BT_Y, z0 = (long)blockIdx.y * BT_Z;
    if (z0 >= sd) return;
    const long ncol = sw * sh;
    const float2* src = D.grids + (long)s * 2 * grid_cells;            // slot 0
    float2* dst = D.grids + (long)s * 2 * grid_cells + grid_cells;     // slot 1
    const int t = threadIdx.x;
    for (int k = t; k < BT_SZ * BT_SY * BT_SX; k += BT_TPB) {
        const int lx = k % BT_SX, ly = (k / BT_SX) % BT_SY, lz = k / (BT_SX * BT_SY);
        const long x = x0 - 2 + lx, y = y0 - 2 + ly, z = z0 - 2 + lz;
        S[lz][ly][lx] = (x >= 0 && x < sw && y >= 0 && y < sh && z >= 0 && z < sd) ? src[z * ncol + y * sw + x]
                                                                                    : make_float2(0.f, 0.f);
    }
    __syncthreads();
    for (int k = t; k < BT_SZ * BT_SY * BT_X; k += BT_TPB) {   // x pass
        const int lx = k % BT_X, ly = (k / BT_X) % BT_SY, lz = k / (BT_X * BT_SY);
        const long x = x0 + lx, y = y0 - 2 + ly, z = z0 - 2 + lz;
        float2 v[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) v[j] = S[lz][ly][lx + j];
        XB[lz][ly][lx] = bil_pass(v, x, sw, y <= 0 || y >= sh - 1 || z <= 0 || z >= sd - 1);
    }
    __syncthreads();
    for (int k = t; k < BT_SZ * BT_Y * BT_X; k += BT_TPB) {    // y pass
        const int lx = k % BT_X, ly = (k / BT_X) % BT_Y, lz = k / (BT_X * BT_Y);
        const long x = x0 + lx, y = y0 + ly, z = z0 - 2 + lz;
        float2 v[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) v[j] = XB[lz][ly + j][lx];
        YB[lz][ly][lx] = bil_pass(v, y, sh, x <= 0 || x >= sw - 1 || z <= 0 || z >= sd - 1);
    }
    __syncthreads();
    for (int k = t; k < BT_Z * BT_Y * BT_X; k += BT_TPB) {     // z pass and the tile's write
        const int lx = k % BT_X, ly = (k / BT_X) % BT_Y, lz = k / (BT_X * BT_Y);
        const long x = x0 + lx, y = y0 + ly, z = z0 + lz;
        if (x >= sw || y >= sh || z >= sd) continue;
        float2 v[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) v[j] = YB[lz + j][ly][lx];
        dst[z * ncol + y * sw + x] = bil_pass(v, z, sd, x <= 0 || x >= sw - 1 || y <= 0 || y >= sh - 1);
    }
}


__device__ __forceinline__ void d_bil_slice(float4* __restrict__ cloud_all, int w, int h, long sw, long sh,
                            const int* __restrict__ zmm, int sd_max, const float2* __restrict__ grids, long grid_cells,
                            int slot) {
    const long N = (long)w * h, total = 8 * N;
    const float sigma_s = 10.0f, sigma_r = 0.05f;
    const long ncol = sw * sh;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        float bmin, bmax;
        long sd;
        bool over;
        if (!bil_params(zmm, s, sd_max, bmin, bmax, sd, over)) continue;
        const float2* G = grids + (long)s * 2 * grid_cells + (long)slot * grid_cells;
        const int j = (int)(i - (long)s * N);
        const int y = j / w, x = j - (j / w) * w;
        float Z = cloud_all[i].z;
        if (!isfin(Z)) Z = bmax;
        const float z = Z - bmin;
        const float fx = (float)x / sigma_s + 2.0f, fy = (float)y / sigma_s + 2.0f, fz = z / sigma_r + 2.0f;
        long xi = (long)(unsigned long)fx, yi = (long)(unsigned long)fy, zi = (long)(unsigned long)fz;
        xi = xi < 0 ? 0 : (xi > sw - 1 ? sw - 1 : xi);
        yi = yi < 0 ? 0 : (yi > sh - 1 ? sh - 1 : yi);
        zi = zi < 0 ? 0 : (zi > sd - 1 ? sd - 1 : zi);
        const long xxi = xi + 1 > sw - 1 ? sw - 1 : xi + 1;
        const long yyi = yi + 1 > sh - 1 ? sh - 1 : yi + 1;
        const long zzi = zi + 1 > sd - 1 ? sd - 1 : zi + 1;
        const float xa = fx - (float)xi, ya = fy - (float)yi, za = fz - (float)zi;
        auto V = [&](long a, long b, long c) { return G[c * ncol + a + sw * b]; };
        const float2 v000 = V(xi, yi, zi), v100 = V(xxi, yi, zi), v010 = V(xi, yyi, zi), v110 = V(xxi, yyi, zi);
        const float2 v001 = V(xi, yi, zzi), v101 = V(xxi, yi, zzi), v011 = V(xi, yyi, zzi), v111 = V(xxi, yyi, zzi);
        const float w000 = (1.0f - xa) * (1.0f - ya) * (1.0f - za), w100 = xa * (1.0f - ya) * (1.0f - za);
        const float w010 = (1.0f - xa) * ya * (1.0f - za), w110 = xa * ya * (1.0f - za);
        const float w001 = (1.0f - xa) * (1.0f - ya) * za, w101 = xa * (1.0f - ya) * za;
        const float w011 = (1.0f - xa) * ya * za, w111 = xa * ya * za;
        const float D0 = w000 * v000.x + w100 * v100.x + w010 * v010.x + w110 * v110.x + w001 * v001.x +
                         w101 * v101.x + w011 * v011.x + w111 * v111.x;
        const float D1 = w000 * v000.y + w100 * v100.y + w010 * v010.y + w110 * v110.y + w001 * v001.y +
                         w101 * v101.y + w011 * v011.y + w111 * v111.y;
        cloud_all[i].z = D0 / D1;
    }
}
__global__ void k_bil_slice(const PlaneBatch B, int w, int h, long sw, long sh, int sd_max, long grid_cells, int slot) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_bil_slice(D.cloud, w, h, sw, sh, D.zmm, sd_max, D.grids, grid_cells, slot);
}


// ------------------------------------------------------------------ A6: depth-change map
__device__ __forceinline__ bool dc_fail(float depth, float other) {
    const float ddc = 0.02f * (fabsf(depth) + 1.0f) * 2.0f;
    return fabsf(depth - other) > ddc || !isfin(depth) || !isfin(other);
}

__device__ __forceinline__ void d_dcm(const float4* __restrict__ cloud, int w, int h, float* __restrict__ dist) {
    const long N = (long)w * h, total = 8 * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        const int j = (int)(i - (long)s * N);
        const int r = j / w, c = j - (j / w) * w;
        const float4* P = cloud + (long)s * N;
        const float z = P[j].z;
        bool edge = false;
        if (r < h - 1 && c < w - 1) edge = dc_fail(z, P[j + 1].z) || dc_fail(z, P[j + w].z);
        if (c >= 1 && r < h - 1) edge = edge || dc_fail(P[j - 1].z, z);        // right test of (r, c-1)
        if (r >= 1 && c < w - 1) edge = edge || dc_fail(P[j - w].z, z);        // down test of (r-1, c)
        dist[i] = edge ? 0.0f : (float)(w + h);
    }
}
__global__ void k_dcm(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_dcm(D.cloud, w, h, D.dist0);
}


// ------------------------------------------------------------------ A6: distance map
// The reference runs a forward and a backward chamfer pass over the whole image (1.0 / 1.4 steps).
// Its result is consumed only as min(dist, 8 + z/10) <= 9, so only values < 9.5 must be exact: such a
// value comes from an edge within 9 rows / 9 columns, so a band of rows with a 10-row halo on each side
// and a 10-term window for the within-row chain reproduce every value below the cap bit for bit
// (rounding is monotone: fl(min(a,b)+1) = min(fl(a+1), fl(b+1))).  Values at or above the cap are
// upper bounds of the true ones and never win the min.
// DM_BAND output rows per workgroup, which also sweeps DM_HALO rows above and below: 4 rows kept the isolated
// latency lowest (38 row steps per workgroup), 8 halves the redundant halo sweeps (1590-1596 -> 1614-1615 pairs/s
// in the batched plane stage, profiles/r5_dm; 16 / 32 within noise of 8)
constexpr int DM_BAND = 8, DM_HALO = 10, DM_TPB = 512;
// (one wave per band measured 2.3x slower: the 10-term chain windows of 5 columns per lane serialise); a thread per
// column at VGA (w = 320): 256 threads 64 us, 320 41 us, 512 39 us per frame; bands of 2 / 3 / 6 / 8 rows slower

__device__ __forceinline__ void dm_sync() { __syncthreads(); }

__device__ __forceinline__ void d_distmap(const float* __restrict__ init, int w, int h, int band,
                                                   float* __restrict__ out) {
    extern __shared__ float sm[];   // (band + 2*DM_HALO + 2) rows x w, plus two temp rows
    const int s = blockIdx.y;
    const int r0 = blockIdx.x * band;
    if (r0 >= h) return;
    const long N = (long)w * h;
    const float* I = init + s * N;
    const int R1 = max(1, r0 - DM_HALO), R2 = min(h - 1, r0 + band + DM_HALO);
    const int base = R1 - 1;                       // LDS row 0 = image row R1-1
    const int nrows = R2 - base + 1;
    float* tmp = sm + (long)nrows * w;
    auto L = [&](int row) { return sm + (long)(row - base) * w; };
    for (int k = threadIdx.x; k < nrows * w; k += blockDim.x) sm[k] = I[(long)base * w + k];
    dm_sync();
    // forward pass rows R1..R2
    for (int r = R1; r <= R2; ++r) {
        const float* prev = L(r - 1);
        float* cur = L(r);
        for (int c = 1 + threadIdx.x; c < w; c += blockDim.x) {
            const float upRight = (c + 1 < w ? prev[c + 1] : cur[0]) + 1.4f;   // prev[w] == cur[0]
            float m = fminf(fminf(prev[c - 1] + 1.4f, prev[c] + 1.0f), upRight);
            tmp[c] = fminf(cur[c], m);
        }
        dm_sync();
        // the chain reads tmp (and cur[0], never updated), so its results go straight into the row
        for (int c = 1 + threadIdx.x; c < w; c += blockDim.x) {
            const int k0 = c - 10 > 1 ? c - 10 : 1;
            float v = (k0 == 1) ? cur[0] : 1e30f;          // chain start (cur[0] is never updated)
            for (int k = k0; k <= c; ++k) v = fminf(tmp[k], v + 1.0f);
            cur[c] = v;
        }
        dm_sync();
    }
    // backward pass rows Rb..r0
    const int Rb = min(h - 2, r0 + band + DM_HALO - 1);
    for (int r = Rb; r >= r0; --r) {
        const float* next = L(r + 1);
        float* cur = L(r);
        for (int c = threadIdx.x; c <= w - 2; c += blockDim.x) {
            const float lowerLeft = (c >= 1 ? next[c - 1] : cur[w - 1]) + 1.4f;   // next[-1] == cur[w-1]
            const float m = fminf(fminf(lowerLeft, next[c] + 1.0f), next[c + 1] + 1.4f);
            tmp[c] = fminf(cur[c], m);
        }
        dm_sync();
        for (int c = threadIdx.x; c <= w - 2; c += blockDim.x) {
            const int k0 = c + 10 < w - 2 ? c + 10 : w - 2;
            float v = (k0 == w - 2) ? cur[w - 1] : 1e30f;   // cur[w-1] is never updated
            for (int k = k0; k >= c; --k) v = fminf(tmp[k], v + 1.0f);
            cur[c] = v;
        }
        dm_sync();
    }
    const int rend = min(h, r0 + band);
    for (int k = threadIdx.x; k < (rend - r0) * w; k += blockDim.x) out[s * N + (long)r0 * w + k] = L(r0)[k];
}
__global__ void __launch_bounds__(DM_TPB) k_distmap(const PlaneBatch B, int w, int h, int band) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_distmap(D.dist0, w, h, band, D.dist);
}


// ------------------------------------------------------------------ A6: normals
// Window sums of the central differences are sums of floats whose ulps are >= 2^-36 and whose
// magnitudes stay far below 2^17, so they are exact in double in any order: a direct sum over the
// (<= 9 x 9) window equals the reference's integral-image differences bit for bit.
//
// One workgroup = a tile of NT_R x NT_C output pixels of one sensor.  The central differences of the tile
// plus a NT_H-pixel halo are computed once into LDS as {dx, finite}, {dy, finite} (a non-finite difference is
// stored as zero and not counted, which is what skipping it does to an exact sum); each pixel then sums its
// window from LDS.  Windows wider than the halo (smoothing >= 10, only for points beyond ~20 m) are summed from
// global memory as before.
constexpr int NT_R = 16, NT_C = 64, NT_H = 4, NT_TPB = 256;
constexpr int NT_SR = NT_R + 2 * NT_H, NT_SC = NT_C + 2 * NT_H;

__device__ __forceinline__ void normal_out(const double (&gx)[3], const double (&gy)[3], unsigned cx, unsigned cy,
                                           const float4& p, float4& o) {
    if (cx != 0 && cy != 0) {
        const double n0 = gy[1] * gx[2] - gy[2] * gx[1];
        const double n1 = gy[2] * gx[0] - gy[0] * gx[2];
        const double n2 = gy[0] * gx[1] - gy[1] * gx[0];
        const double len = n0 * n0 + n1 * n1 + n2 * n2;
        if (len != 0.0) {
            const double sl = sqrt(len);
            float nx = (float)(n0 / sl), ny = (float)(n1 / sl), nz = (float)(n2 / sl);
            const float vx = 0.f - p.x, vy = 0.f - p.y, vz = 0.f - p.z;
            if (vx * nx + vy * ny + vz * nz < 0) { nx *= -1; ny *= -1; nz *= -1; }
            o = make_float4(nx, ny, nz, p.x * nx + p.y * ny + p.z * nz);
        }
    }
}

__device__ __forceinline__ void d_normals(const float4* __restrict__ cloud, const float* __restrict__ dist,
                                                   int w, int h, float4* __restrict__ nrm) {
    __shared__ float4 sdx[NT_SR * NT_SC], sdy[NT_SR * NT_SC];
    const int s = blockIdx.z & 7;   // sensor (blockIdx.z / 8: the frame of the batch)
    const int r0 = blockIdx.y * NT_R, c0 = blockIdx.x * NT_C;
    const long N = (long)w * h;
    const float4* P = cloud + (long)s * N;
    // differences of the staged pixels (image rows r0 - NT_H .., columns c0 - NT_H ..); positions outside
    // [1, h-2] x [1, w-2] are zero and counted, as the reference's border handling (never read by pixels that
    // pass the 8-pixel border test)
    for (int k = threadIdx.x; k < NT_SR * NT_SC; k += NT_TPB) {
        const int yy = r0 - NT_H + k / NT_SC, xx = c0 - NT_H + k % NT_SC;
        float4 a = make_float4(0.f, 0.f, 0.f, 1.f), b = a;
        if (yy >= 1 && yy <= h - 2 && xx >= 1 && xx <= w - 2) {
            const int q = yy * w + xx;
            const float4 pr = P[q + 1], pl = P[q - 1], pu = P[q - w], pd = P[q + w];
            const float dx0 = pr.x - pl.x, dx1 = pr.y - pl.y, dx2 = pr.z - pl.z;
            const float dy0 = pd.x - pu.x, dy1 = pd.y - pu.y, dy2 = pd.z - pu.z;
            a = isfin(dx0 + dx1 + dx2) ? make_float4(dx0, dx1, dx2, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
            b = isfin(dy0 + dy1 + dy2) ? make_float4(dy0, dy1, dy2, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        sdx[k] = a;
        sdy[k] = b;
    }
    __syncthreads();
    const float nan = __builtin_nanf("");
    const int c = c0 + (threadIdx.x & (NT_C - 1));
    for (int rr = threadIdx.x / NT_C; rr < NT_R; rr += NT_TPB / NT_C) {
        const int r = r0 + rr;
        if (r >= h || c >= w) continue;
        const int j = r * w + c;
        const long i = (long)s * N + j;
        float4 o = make_float4(nan, nan, nan, nan);
        const int border = 8;
        const float4 p = P[j];
        if (r >= border && r < h - border && c >= border && c < w - border && isfin(p.z)) {
            const float dm = dist[i];
            const float lim = 8.0f + p.z / 10.0f;
            const float smoothing = dm < lim ? dm : lim;
            if (smoothing > 2.0f) {
                const int rs = (int)smoothing, rs2 = rs / 2;
                const int sx = c - rs2, sy = r - rs2;
                double gx[3] = {0, 0, 0}, gy[3] = {0, 0, 0};
                unsigned cx = 0, cy = 0;
                if (rs <= 2 * NT_H + 1) {
                    float fcx = 0.f, fcy = 0.f;   // counts of <= 81 ones: exact in float
                    for (int yy = sy; yy < sy + rs; ++yy) {
                        const int rowb = (yy - (r0 - NT_H)) * NT_SC - (c0 - NT_H);
                        for (int xx = sx; xx < sx + rs; ++xx) {
                            const float4 a = sdx[rowb + xx], b = sdy[rowb + xx];
                            gx[0] += a.x; gx[1] += a.y; gx[2] += a.z; fcx += a.w;
                            gy[0] += b.x; gy[1] += b.y; gy[2] += b.z; fcy += b.w;
                        }
                    }
                    cx = (unsigned)fcx;
                    cy = (unsigned)fcy;
                } else {
                    for (int yy = sy; yy < sy + rs; ++yy)
                        for (int xx = sx; xx < sx + rs; ++xx) {
                            if (yy < 1 || yy > h - 2 || xx < 1 || xx > w - 2) { ++cx; ++cy; continue; }  // zero, finite
                            const int q = yy * w + xx;
                            const float4 a = P[q + 1], b = P[q - 1], u = P[q - w], d = P[q + w];
                            const float dx0 = a.x - b.x, dx1 = a.y - b.y, dx2 = a.z - b.z;
                            const float dy0 = d.x - u.x, dy1 = d.y - u.y, dy2 = d.z - u.z;
                            if (isfin(dx0 + dx1 + dx2)) { gx[0] += dx0; gx[1] += dx1; gx[2] += dx2; ++cx; }
                            if (isfin(dy0 + dy1 + dy2)) { gy[0] += dy0; gy[1] += dy1; gy[2] += dy2; ++cy; }
                        }
                }
                normal_out(gx, gy, cx, cy, p, o);
            }
        }
        nrm[i] = o;
    }
}
__global__ void __launch_bounds__(NT_TPB) k_normals(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z >> 3];
    d_normals(D.cloud, D.dist, w, h, D.nrm);
}



// k_normals with the window sums read from summed-area tables of the staged tile instead of summed over the
// window: a table entry is a sum of at most (NT_SR x NT_SC) = 1728 central differences, each a multiple of 2^-36
// below 2^5 in magnitude, so every entry (< 2^16) and every rectangle of entries is exact in double, and a window
// sum S(y1,x1) - S(y0,x1) - S(y1,x0) + S(y0,x0) equals the direct sum bit for bit.  Per output pixel that is 4
// lookups per channel instead of up to 81 float4 reads per difference image.  The tables (3 doubles + a count per
// entry, leading zero row / column) are built for dx, used, then rebuilt for dy in the same 51 KB.
constexpr int NS_W = NT_SC + 1, NS_H = NT_SR + 1;   // table size with the leading zero row / column
struct SatShared { double v[3][NS_H * NS_W]; int c[NS_H * NS_W]; };

__device__ __forceinline__ void d_normals_sat(const float4* __restrict__ cloud, const float* __restrict__ dist,
                                                       int w, int h, float4* __restrict__ nrm) {
    __shared__ SatShared T;
    const int s = blockIdx.z & 7;   // sensor (blockIdx.z / 8: the frame of the batch)
    const int r0 = blockIdx.y * NT_R, c0 = blockIdx.x * NT_C;
    const long N = (long)w * h;
    const float4* P = cloud + (long)s * N;
    const float nan = __builtin_nanf("");
    // the thread's output pixels (column c, rows r0 + rr, rr = thread / NT_C + 4 j) and their windows
    constexpr int PER = NT_R / (NT_TPB / NT_C);
    const int c = c0 + (threadIdx.x & (NT_C - 1));
    int rs_[PER];         // window size (0: no normal from the table path; -1: the global-memory path)
    float4 pt[PER];
    double g[2][PER][3];
    unsigned cnt[2][PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int r = r0 + threadIdx.x / NT_C + j * (NT_TPB / NT_C);
        rs_[j] = 0;
        pt[j] = make_float4(nan, nan, nan, nan);
        if (r >= h || c >= w) continue;
        const int border = 8;
        const float4 p = P[r * w + c];
        pt[j] = p;
        if (r >= border && r < h - border && c >= border && c < w - border && isfin(p.z)) {
            const float dm = dist[(long)s * N + r * w + c];
            const float lim = 8.0f + p.z / 10.0f;
            const float smoothing = dm < lim ? dm : lim;
            if (smoothing > 2.0f) {
                const int rs = (int)smoothing;
                rs_[j] = rs <= 2 * NT_H + 1 ? rs : -1;
            }
        }
    }
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {   // 0: x differences (right - left), 1: y differences (down - up)
        // stage the differences at table position (y + 1, x + 1); row 0 and column 0 are zero.  NT_STG entries per
        // thread at a time: their point loads are issued together before any of them is used
        constexpr int NT_STG = 4;
        for (int k0 = 0; k0 < NS_H * NS_W; k0 += NT_STG * NT_TPB) {
            float4 a[NT_STG], b[NT_STG];
            int st[NT_STG];   // 0: outside the table, 1: zero and counted, 2: a difference
#pragma unroll
            for (int u = 0; u < NT_STG; ++u) {
                const int k = k0 + u * NT_TPB + threadIdx.x;
                const int ty = k / NS_W, tx = k - ty * NS_W;
                st[u] = 0;
                a[u] = b[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (k < NS_H * NS_W && ty > 0 && tx > 0) {
                    const int yy = r0 - NT_H + ty - 1, xx = c0 - NT_H + tx - 1;
                    st[u] = 1;   // outside [1, h-2] x [1, w-2]: zero and counted, as k_normals
                    if (yy >= 1 && yy <= h - 2 && xx >= 1 && xx <= w - 2) {
                        const int q = yy * w + xx;
                        a[u] = ph ? P[q + w] : P[q + 1];
                        b[u] = ph ? P[q - w] : P[q - 1];
                        st[u] = 2;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < NT_STG; ++u) {
                const int k = k0 + u * NT_TPB + threadIdx.x;
                if (k >= NS_H * NS_W) continue;
                double d0 = 0.0, d1 = 0.0, d2 = 0.0;
                int n = st[u] ? 1 : 0;
                if (st[u] == 2) {
                    const float e0 = a[u].x - b[u].x, e1 = a[u].y - b[u].y, e2 = a[u].z - b[u].z;
                    if (isfin(e0 + e1 + e2)) { d0 = e0; d1 = e1; d2 = e2; } else n = 0;
                }
                T.v[0][k] = d0; T.v[1][k] = d1; T.v[2][k] = d2; T.c[k] = n;
            }
        }
        __syncthreads();
        // row prefix sums (one thread per (row, channel)), then column prefix sums (one per (column, channel))
        for (int t = threadIdx.x; t < NS_H * 4; t += NT_TPB) {
            const int row = t >> 2, ch = t & 3;
            if (ch < 3) {
                double* v = T.v[ch] + row * NS_W;
                double acc = 0.0;
                for (int x = 0; x < NS_W; ++x) { acc += v[x]; v[x] = acc; }
            } else {
                int* v = T.c + row * NS_W;
                int acc = 0;
                for (int x = 0; x < NS_W; ++x) { acc += v[x]; v[x] = acc; }
            }
        }
        __syncthreads();
        for (int t = threadIdx.x; t < NS_W * 4; t += NT_TPB) {
            const int col = t >> 2, ch = t & 3;
            if (ch < 3) {
                double* v = T.v[ch] + col;
                double acc = 0.0;
                for (int y = 0; y < NS_H; ++y) { acc += v[y * NS_W]; v[y * NS_W] = acc; }
            } else {
                int* v = T.c + col;
                int acc = 0;
                for (int y = 0; y < NS_H; ++y) { acc += v[y * NS_W]; v[y * NS_W] = acc; }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            g[ph][j][0] = g[ph][j][1] = g[ph][j][2] = 0.0;
            cnt[ph][j] = 0;
            const int rs = rs_[j];
            if (rs <= 0) continue;
            const int r = r0 + threadIdx.x / NT_C + j * (NT_TPB / NT_C);
            // window rows [r - rs/2, +rs), columns [c - rs/2, +rs) in table coordinates (+ NT_H - r0 / c0)
            const int y0 = r - rs / 2 - (r0 - NT_H), x0 = c - rs / 2 - (c0 - NT_H);
            const int i00 = y0 * NS_W + x0, i01 = y0 * NS_W + x0 + rs, i10 = (y0 + rs) * NS_W + x0,
                      i11 = (y0 + rs) * NS_W + x0 + rs;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const double* v = T.v[ch];
                g[ph][j][ch] = ((v[i11] - v[i01]) - v[i10]) + v[i00];
            }
            cnt[ph][j] = (unsigned)(((T.c[i11] - T.c[i01]) - T.c[i10]) + T.c[i00]);
        }
        __syncthreads();   // the tables are rebuilt for the next phase
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int r = r0 + threadIdx.x / NT_C + j * (NT_TPB / NT_C);
        if (r >= h || c >= w) continue;
        float4 o = make_float4(nan, nan, nan, nan);
        const float4 p = pt[j];
        if (rs_[j] > 0) {
            normal_out(g[0][j], g[1][j], cnt[0][j], cnt[1][j], p, o);
        } else if (rs_[j] < 0) {   // window wider than the halo: summed from global memory as k_normals
            const float dm = dist[(long)s * N + r * w + c];
            const float lim = 8.0f + p.z / 10.0f;
            const int rs = (int)(dm < lim ? dm : lim), rs2 = rs / 2;
            const int sx = c - rs2, sy = r - rs2;
            double gx[3] = {0, 0, 0}, gy[3] = {0, 0, 0};
            unsigned cx = 0, cy = 0;
            for (int yy = sy; yy < sy + rs; ++yy)
                for (int xx = sx; xx < sx + rs; ++xx) {
                    if (yy < 1 || yy > h - 2 || xx < 1 || xx > w - 2) { ++cx; ++cy; continue; }  // zero, finite
                    const int q = yy * w + xx;
                    const float4 a = P[q + 1], b = P[q - 1], u = P[q - w], d = P[q + w];
                    const float dx0 = a.x - b.x, dx1 = a.y - b.y, dx2 = a.z - b.z;
                    const float dy0 = d.x - u.x, dy1 = d.y - u.y, dy2 = d.z - u.z;
                    if (isfin(dx0 + dx1 + dx2)) { gx[0] += dx0; gx[1] += dx1; gx[2] += dx2; ++cx; }
                    if (isfin(dy0 + dy1 + dy2)) { gy[0] += dy0; gy[1] += dy1; gy[2] += dy2; ++cy; }
                }
            normal_out(gx, gy, cx, cy, p, o);
        }
        nrm[(long)s * N + r * w + c] = o;
    }
}
__global__ void __launch_bounds__(NT_TPB) k_normals_sat(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z >> 3];
    d_normals_sat(D.cloud, D.dist, w, h, D.nrm);
}


}  // namespace

// ------------------------------------------------------------------ launchers
int launch_rgb(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st) {
    const long tot = 8L * G.w * G.h;
    const int blocks = (int)std::min<long>((tot + 255) / 256, 4096);
    hipLaunchKernelGGL(k_rgb, dim3(blocks, 1, (unsigned)F), dim3(256), 0, st, B, G.rows, G.cols);
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_cloud_normals(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx) {
    const int w = G.w, h = G.h;
    const long tot = 8L * w * h;
    const int blocks = (int)((tot + 255) / 256);
    const unsigned nf = (unsigned)F;   // grid z: the batch's frames
    // CloudRGBD_Ext.h:97-102 constants, evaluated as the reference writes them
    const float res_factor_VGA = G.cols / 640.0;
    const float focal_length = 525 * res_factor_VGA;
    const float inv_f = 1.f / focal_length;
    const float ox = G.cols / 2 - 0.5, oy = G.rows / 2 - 0.5;
    int slot = timing_begin(tctx, "k_cloud");
    hipLaunchKernelGGL(k_plane_begin, dim3(1, 1, nf), dim3(64), 0, st, B);
    hipLaunchKernelGGL(k_cloud, dim3(blocks, 1, nf), dim3(256), 0, st, B, G.rows, G.cols, inv_f, ox, oy);
    hipLaunchKernelGGL(k_zrange, dim3(8, 1, nf), dim3(1024), 0, st, B, (long)w * h);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_bilateral");
    {
        // grid extent (FastBilateralFilter): sw, sh from the image size; sd per sensor on the device
        const long sw = (long)(unsigned long)((float)(w - 1) / 10.0f) + 5;
        const long sh = (long)(unsigned long)((float)(h - 1) / 10.0f) + 5;
        if (G.sd_max != BIL_SD_MAX || sw * sh * G.sd_max > G.grid_cells) {
            r360_set_error("bilateral grid configuration mismatch");
            return -1;
        }
        const long ncol = sw * sh;
        hipLaunchKernelGGL(k_bil_splat, dim3((ncol + BIL_COLS - 1) / BIL_COLS, 8, nf), dim3(BIL_COLS), 0, st, B, w, h,
                           sw, sh, G.sd_max, G.grid_cells);
        // the three axis passes fused (k_bil_blur3; R360_BIL_FUSED=0, experiment builds: one launch per axis)
        static const int fused = R360_KNOB("R360_BIL_FUSED", 1);
        if (fused) {
            const long ntile = ((sw + BT_X - 1) / BT_X) * ((sh + BT_Y - 1) / BT_Y);
            hipLaunchKernelGGL(k_bil_blur3, dim3((unsigned)ntile, (unsigned)((G.sd_max + BT_Z - 1) / BT_Z), 8 * nf),
                               dim3(BT_TPB), 0, st, B, G.grid_cells, sw, sh, G.sd_max);
        } else {
            const dim3 gb((unsigned)((ncol * G.sd_max + 255) / 256), 8, nf);
            hipLaunchKernelGGL(k_bil_blur<0>, gb, dim3(256), 0, st, B, G.grid_cells, 0, sw, sh, G.sd_max);
            hipLaunchKernelGGL(k_bil_blur<1>, gb, dim3(256), 0, st, B, G.grid_cells, 1, sw, sh, G.sd_max);
            hipLaunchKernelGGL(k_bil_blur<2>, gb, dim3(256), 0, st, B, G.grid_cells, 0, sw, sh, G.sd_max);
        }
        hipLaunchKernelGGL(k_bil_slice, dim3(blocks, 1, nf), dim3(256), 0, st, B, w, h, sw, sh, G.sd_max, G.grid_cells, 1);
    }
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_dcm");
    hipLaunchKernelGGL(k_dcm, dim3(blocks, 1, nf), dim3(256), 0, st, B, w, h);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    // experiment builds: R360_DM_BAND rows per workgroup (each workgroup also sweeps 2 x DM_HALO halo rows)
    static const int dm_band = R360_KNOB("R360_DM_BAND", DM_BAND);
    const int band = dm_band >= 1 && dm_band <= 64 ? dm_band : DM_BAND;
    const int nb = (h + band - 1) / band;
    const int max_rows = band + 2 * DM_HALO + 2;
    const size_t lds = sizeof(float) * ((size_t)max_rows + 2) * w;
    if (lds > 160 * 1024) { r360_set_error("distance map: cloud width %d too large", w); return -1; }
    slot = timing_begin(tctx, "k_distmap");
    hipLaunchKernelGGL(k_distmap, dim3(nb, 8, nf), dim3(DM_TPB), lds, st, B, w, h, band);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_normals");
    // summed-area-table windows (default; R360_NORMALS_SAT=0: the direct window sums of k_normals); grid z = 8 sensors
    // x the batch's frames
    static const int nsat = R360_KNOB("R360_NORMALS_SAT", 1);
    const dim3 gn((w + NT_C - 1) / NT_C, (h + NT_R - 1) / NT_R, 8 * nf);
    if (nsat) hipLaunchKernelGGL(k_normals_sat, gn, dim3(NT_TPB), 0, st, B, w, h);
    else hipLaunchKernelGGL(k_normals, gn, dim3(NT_TPB), 0, st, B, w, h);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}
