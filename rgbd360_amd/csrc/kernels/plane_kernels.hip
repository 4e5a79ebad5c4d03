// plane_kernels.hip — the per-pixel plane half of Frame360 on gfx950:
//   k_cloud       back-projection + 2x2 upper-median downsample   (CloudRGBD_Ext.h:78-139,
//                 DownsampleRGBD.h:209-311)
//   k_bilateral   pcl::FastBilateralFilter (sigma_s 10, sigma_r 0.05), one workgroup per sensor
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
__global__ void k_cloud(const float* __restrict__ depth_m, const uint8_t* __restrict__ bgr, int rows, int cols,
                        float inv_f, float ox, float oy, float4* __restrict__ cloud, uchar4* __restrict__ rgb) {
    const int w = cols / 2, h = rows / 2;
    const long N = (long)w * h, total = 8 * N;
    const float nan = __builtin_nanf("");
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
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
        cloud[i] = o;
        const uint8_t* b = bgr + ((long)s * rows * cols + (long)(r + 1) * cols + c + 1) * 3;
        rgb[i] = make_uchar4(b[2], b[1], b[0], 0);
    }
}

// ------------------------------------------------------------------ A4
// One workgroup per sensor.  grid0/grid1: 2 x (sw*sh*sd) float2 cells each, zeroed here.
constexpr int BIL_TPB = 1024;

__device__ float block_reduce_minmax(float v, bool is_max, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const float o = __shfl_xor(v, m, 64);
        v = is_max ? (o > v ? o : v) : (o < v ? o : v);
    }
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = is_max ? (red[k] > r ? red[k] : r) : (red[k] < r ? red[k] : r);
        red[16] = r;
    }
    __syncthreads();
    return red[16];
}

__global__ void __launch_bounds__(BIL_TPB) k_bilateral(float4* __restrict__ cloud_all, int w, int h,
                                                      float2* __restrict__ grids, long grid_cells, int sd_max,
                                                      int* __restrict__ err) {
    __shared__ float red[17];
    const int s = blockIdx.x;
    float4* cloud = cloud_all + (long)s * w * h;
    float2* A = grids + (long)s * 2 * grid_cells;
    float2* B = A + grid_cells;
    const int n = w * h;
    const float sigma_s = 10.0f, sigma_r = 0.05f;
    float lmax = -3.40282347e38f, lmin = 3.40282347e38f;
    int lfound = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float z = cloud[i].z;
        if (isfin(z)) {
            lmax = lmax < z ? z : lmax;
            lmin = lmin > z ? z : lmin;
            lfound = 1;
        }
    }
    const float base_max = block_reduce_minmax(lmax, true, red);
    const float base_min = block_reduce_minmax(lmin, false, red);
    const int found = __syncthreads_or(lfound);
    if (!found) return;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (!isfin(cloud[i].z)) cloud[i].z = base_max;
    const float base_delta = base_max - base_min;
    const long sw = (long)(unsigned long)((float)(w - 1) / sigma_s) + 5;
    const long sh = (long)(unsigned long)((float)(h - 1) / sigma_s) + 5;
    const long sd = (long)(unsigned long)(base_delta / sigma_r) + 5;
    if (sd > sd_max) {
        if (threadIdx.x == 0) atomicOr(err, 1);
        return;
    }
    const long cells = sw * sh * sd;
    for (long i = threadIdx.x; i < cells; i += blockDim.x) {
        A[i] = make_float2(0.f, 0.f);
        B[i] = make_float2(0.f, 0.f);
    }
    __syncthreads();
    // splat: one thread per (sx, sy) column, points in the oracle's x-major, y-minor order
    for (long col = threadIdx.x; col < sw * sh; col += blockDim.x) {
        const int sx = (int)(col % sw), sy = (int)(col / sw);
        const int x0 = max(0, 10 * (sx - 2) - 6), x1 = min(w - 1, 10 * (sx - 2) + 6);
        const int y0 = max(0, 10 * (sy - 2) - 6), y1 = min(h - 1, 10 * (sy - 2) + 6);
        for (int x = x0; x <= x1; ++x) {
            if ((long)(unsigned long)((float)x / sigma_s + 0.5f) + 2 != sx) continue;
            for (int y = y0; y <= y1; ++y) {
                if ((long)(unsigned long)((float)y / sigma_s + 0.5f) + 2 != sy) continue;
                const float Z = cloud[(long)y * w + x].z;
                const float z = Z - base_min;
                const long sz = (long)(unsigned long)(z / sigma_r + 0.5f) + 2;
                float2& d = A[(sx + sw * sy) * sd + sz];
                d.x += Z;
                d.y += 1.0f;
            }
        }
    }
    __syncthreads();
    // 3 axes x 2 iterations of [1 2 1]/4 over the interior; boundaries stay zero
    const long off[3] = {sd, sw * sd, 1};
    float2* src = A;
    float2* dst = B;
    const long inner = (sw - 2) * (sh - 2) * (sd - 2);
    for (int pass = 0; pass < 6; ++pass) {
        const long o = off[pass >> 1];
        for (long t = threadIdx.x; t < inner; t += blockDim.x) {
            const long z = t % (sd - 2) + 1;
            const long rest = t / (sd - 2);
            const long y = rest % (sh - 2) + 1;
            const long x = rest / (sh - 2) + 1;
            const long p = (x + sw * y) * sd + z;
            const float2 a = src[p - o], b = src[p + o], c = src[p];
            dst[p] = make_float2((a.x + b.x + 2.0f * c.x) / 4.0f, (a.y + b.y + 2.0f * c.y) / 4.0f);
        }
        __syncthreads();
        float2* t = src; src = dst; dst = t;
    }
    // slice (trilinear) and z <- D0 / D1; src holds the result after 6 passes
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int y = i / w, x = i - (i / w) * w;
        const float Z = cloud[i].z;
        const float z = Z - base_min;
        const float fx = (float)x / sigma_s + 2.0f, fy = (float)y / sigma_s + 2.0f, fz = z / sigma_r + 2.0f;
        long xi = (long)(unsigned long)fx, yi = (long)(unsigned long)fy, zi = (long)(unsigned long)fz;
        xi = xi < 0 ? 0 : (xi > sw - 1 ? sw - 1 : xi);
        yi = yi < 0 ? 0 : (yi > sh - 1 ? sh - 1 : yi);
        zi = zi < 0 ? 0 : (zi > sd - 1 ? sd - 1 : zi);
        const long xxi = xi + 1 > sw - 1 ? sw - 1 : xi + 1;
        const long yyi = yi + 1 > sh - 1 ? sh - 1 : yi + 1;
        const long zzi = zi + 1 > sd - 1 ? sd - 1 : zi + 1;
        const float xa = fx - (float)xi, ya = fy - (float)yi, za = fz - (float)zi;
        auto V = [&](long a, long b, long c) { return src[(a + sw * b) * sd + c]; };
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
        cloud[i].z = D0 / D1;
    }
}

// ------------------------------------------------------------------ A6: depth-change map
__device__ __forceinline__ bool dc_fail(float depth, float other) {
    const float ddc = 0.02f * (fabsf(depth) + 1.0f) * 2.0f;
    return fabsf(depth - other) > ddc || !isfin(depth) || !isfin(other);
}

__global__ void k_dcm(const float4* __restrict__ cloud, int w, int h, float* __restrict__ dist) {
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

// ------------------------------------------------------------------ A6: distance map
// The reference runs a forward and a backward chamfer pass over the whole image (1.0 / 1.4 steps).
// Its result is consumed only as min(dist, 8 + z/10) <= 9, so only values < 9.5 must be exact: such a
// value comes from an edge within 9 rows / 9 columns, so a band of rows with a 10-row halo on each side
// and a 10-term window for the within-row chain reproduce every value below the cap bit for bit
// (rounding is monotone: fl(min(a,b)+1) = min(fl(a+1), fl(b+1))).  Values at or above the cap are
// upper bounds of the true ones and never win the min.
constexpr int DM_BAND = 16, DM_HALO = 10, DM_TPB = 256;

__global__ void __launch_bounds__(DM_TPB) k_distmap(const float* __restrict__ init, int w, int h,
                                                   float* __restrict__ out) {
    extern __shared__ float sm[];   // (DM_BAND + 2*DM_HALO + 2) rows x w, plus one temp row
    const int s = blockIdx.y;
    const int r0 = blockIdx.x * DM_BAND;
    if (r0 >= h) return;
    const long N = (long)w * h;
    const float* I = init + s * N;
    const int R1 = max(1, r0 - DM_HALO), R2 = min(h - 1, r0 + DM_BAND + DM_HALO);
    const int base = R1 - 1;                       // LDS row 0 = image row R1-1
    const int nrows = R2 - base + 1;
    float* tmp = sm + (long)nrows * w;
    auto L = [&](int row) { return sm + (long)(row - base) * w; };
    for (int k = threadIdx.x; k < nrows * w; k += blockDim.x) sm[k] = I[(long)base * w + k];
    __syncthreads();
    // forward pass rows R1..R2
    for (int r = R1; r <= R2; ++r) {
        const float* prev = L(r - 1);
        float* cur = L(r);
        for (int c = 1 + threadIdx.x; c < w; c += blockDim.x) {
            const float upRight = (c + 1 < w ? prev[c + 1] : cur[0]) + 1.4f;   // prev[w] == cur[0]
            float m = fminf(fminf(prev[c - 1] + 1.4f, prev[c] + 1.0f), upRight);
            tmp[c] = fminf(cur[c], m);
        }
        __syncthreads();
        float res[4];
        int nres = 0;
        for (int c = 1 + threadIdx.x; c < w; c += blockDim.x) {
            const int k0 = c - 10 > 1 ? c - 10 : 1;
            float v = (k0 == 1) ? cur[0] : 1e30f;          // chain start (cur[0] is never updated)
            for (int k = k0; k <= c; ++k) v = fminf(tmp[k], v + 1.0f);
            res[nres++] = v;
        }
        __syncthreads();
        nres = 0;
        for (int c = 1 + threadIdx.x; c < w; c += blockDim.x) cur[c] = res[nres++];
        __syncthreads();
    }
    // backward pass rows Rb..r0
    const int Rb = min(h - 2, r0 + DM_BAND + DM_HALO - 1);
    for (int r = Rb; r >= r0; --r) {
        const float* next = L(r + 1);
        float* cur = L(r);
        for (int c = threadIdx.x; c <= w - 2; c += blockDim.x) {
            const float lowerLeft = (c >= 1 ? next[c - 1] : cur[w - 1]) + 1.4f;   // next[-1] == cur[w-1]
            const float m = fminf(fminf(lowerLeft, next[c] + 1.0f), next[c + 1] + 1.4f);
            tmp[c] = fminf(cur[c], m);
        }
        __syncthreads();
        float res[4];
        int nres = 0;
        for (int c = threadIdx.x; c <= w - 2; c += blockDim.x) {
            const int k0 = c + 10 < w - 2 ? c + 10 : w - 2;
            float v = (k0 == w - 2) ? cur[w - 1] : 1e30f;
            for (int k = k0; k >= c; --k) v = fminf(tmp[k], v + 1.0f);
            res[nres++] = v;
        }
        __syncthreads();
        nres = 0;
        for (int c = threadIdx.x; c <= w - 2; c += blockDim.x) cur[c] = res[nres++];
        __syncthreads();
    }
    const int rend = min(h, r0 + DM_BAND);
    for (int k = threadIdx.x; k < (rend - r0) * w; k += blockDim.x) out[s * N + (long)r0 * w + k] = L(r0)[k];
}

// ------------------------------------------------------------------ A6: normals
// Window sums of the central differences are sums of floats whose ulps are >= 2^-36 and whose
// magnitudes stay far below 2^17, so they are exact in double in any order: a direct sum over the
// (<= 9 x 9) window equals the reference's integral-image differences bit for bit.
__global__ void k_normals(const float4* __restrict__ cloud, const float* __restrict__ dist, int w, int h,
                          float4* __restrict__ nrm) {
    const long N = (long)w * h, total = 8 * N;
    const float nan = __builtin_nanf("");
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        const int j = (int)(i - (long)s * N);
        const int r = j / w, c = j - (j / w) * w;
        const float4* P = cloud + (long)s * N;
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
        }
        nrm[i] = o;
    }
}

}  // namespace

// ------------------------------------------------------------------ launchers
int launch_cloud_normals(r360_frame* f) {
    PlaneBufs& P = f->pl;
    hipStream_t st = f->ctx->stream;
    const int w = P.w, h = P.h;
    const long tot = 8L * w * h;
    const int blocks = (int)((tot + 255) / 256);
    // CloudRGBD_Ext.h:97-102 constants, evaluated as the reference writes them
    const float res_factor_VGA = f->cols / 640.0;
    const float focal_length = 525 * res_factor_VGA;
    const float inv_f = 1.f / focal_length;
    const float ox = f->cols / 2 - 0.5, oy = f->rows / 2 - 0.5;
    int slot = timing_begin(f->ctx, "k_cloud");
    hipLaunchKernelGGL(k_cloud, dim3(blocks), dim3(256), 0, st, f->d_depth_m, f->d_bgr, f->rows, f->cols, inv_f, ox, oy,
                       P.cloud, P.rgb);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(f->ctx, "k_bilateral");
    hipLaunchKernelGGL(k_bilateral, dim3(8), dim3(BIL_TPB), 0, st, P.cloud, w, h, P.grids, P.grid_cells, P.sd_max,
                       P.err);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(f->ctx, "k_dcm");
    hipLaunchKernelGGL(k_dcm, dim3(blocks), dim3(256), 0, st, P.cloud, w, h, P.dist0);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    const int nb = (h + DM_BAND - 1) / DM_BAND;
    const int max_rows = DM_BAND + 2 * DM_HALO + 2;
    const size_t lds = sizeof(float) * ((size_t)max_rows + 1) * w;
    if (lds > 160 * 1024) { r360_set_error("distance map: cloud width %d too large", w); return -1; }
    slot = timing_begin(f->ctx, "k_distmap");
    hipLaunchKernelGGL(k_distmap, dim3(nb, 8), dim3(DM_TPB), lds, st, P.dist0, w, h, P.dist);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(f->ctx, "k_normals");
    hipLaunchKernelGGL(k_normals, dim3(blocks), dim3(256), 0, st, P.cloud, P.dist, w, h, P.nrm);
    timing_end(f->ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}
