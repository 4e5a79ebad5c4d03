// plane_seg.hip — OrganizedMultiPlaneSegmentation::segmentAndRefine on gfx950 and the
// per-plane statistics the PbMap descriptors need (A8):
//   k_ccl_*        4-connected components under PlaneCoefficientComparator (LDS union-find per row
//                  band, then lock-free global union of the band-crossing edges; roots = smallest
//                  raster index, labels numbered in raster order of their roots — the reference's
//                  run-id compaction order)
//   k_big_list     labels with > 80 points, in order
//   k_gm<false>    exact moments per large label (int64/int128 sums), pixel order, no pixel lists
//   k_plane_fit    eigen33 plane fit, curvature test and the accumulating viewpoint of segment()
//   k_refine       the two raster sweeps of refine(): one wave per sensor walks the rows; within a row
//                  the left-to-right (right-to-left) label chains are resolved with wave scans over
//                  per-lane chunk summaries; closeness to every model is precomputed per pixel as a
//                  bit mask (k_refine_init)
//   k_gm<true>     final inlier moments (rig frame) + colour sums + bounds per refined region (folded by k_nbmask)
//   k_trace        findLabeledRegionBoundary (Moore-neighbour trace) over per-pixel neighbour masks
//   k_vox_*        VoxelGrid of regions without a contour (Frame360.h:1017-1026): (region, voxel) hash
//                  table with exact double sums, compacted into per-region voxel lists
// Arithmetic follows oracle/src/planes_oracle.cpp and pbmap_oracle.cpp; see rgbd360_amd/csrc/plane_math.h.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include "../r360_internal.h"
#include "../plane_math.h"

namespace {

__device__ __forceinline__ bool isfin(float v) { return __builtin_isfinite(v); }

// ------------------------------------------------------------------ CCL
__device__ __forceinline__ int ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// with path halving (see lds_find); the re-points are agent-scope atomic stores, like the CAS links
__device__ int find_root(int* parent, int x) {
    int p = ld(parent + x);
    while (p != x) {
        const int gp = ld(parent + p);
        if (gp != p) __hip_atomic_store(parent + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x = gp;
        p = ld(parent + x);
    }
    return x;
}

__device__ void unite(int* parent, int a, int b) {
    while (true) {
        a = find_root(parent, a);
        b = find_root(parent, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(parent + a, a, b);
        if (old == a) return;
        a = old;
    }
}

// PlaneCoefficientComparator::compare(a, b), depth dependent (threshold 0.02 * z_a^2)
__device__ __forceinline__ bool plane_cmp(const float4& pa, const float4& na, const float4& nb, float ang_thr) {
    float thr = 0.02f;
    const float z = pa.x * 0.f + pa.y * 0.f + pa.z * 1.f;
    thr *= z * z;
    const float nd = na.x * nb.x + na.y * nb.y + na.z * nb.z;
    return fabsf(na.w - nb.w) < thr && nd > ang_thr;
}

// Two-level CCL: each workgroup labels a band of CCL_ROWS full rows with an LDS union-find (min-index
// roots, the same representative the global union-find produces), writes every pixel's parent as
// the global index of its band-local root, then k_ccl_border unites only the edges that cross band
// boundaries in global memory.
constexpr int CCL_ROWS = 16, CCL_TPB = 1024;

// path halving: every other node on the walk is re-pointed at its grandparent.  Parents only ever point at
// smaller indices of the same component, so a racing re-point installs another ancestor and the roots (the
// components' smallest indices) are unchanged.
__device__ int lds_find(int* lp, int x) {
    int p = lp[x];
    while (p != x) {
        const int gp = lp[p];
        if (gp != p) lp[x] = gp;
        x = gp;
        p = lp[x];
    }
    return x;
}

__device__ void lds_unite(int* lp, int a, int b) {
    while (true) {
        a = lds_find(lp, a);
        b = lds_find(lp, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(lp + a, a, b);
        if (old == a) return;
        a = old;
    }
}

__device__ __forceinline__ void d_ccl_local(const float4* __restrict__ cloud, const float4* __restrict__ nrm,
                                                      int w, int h, float ang_thr, int* __restrict__ parent) {
    extern __shared__ int lp[];
    const int s = blockIdx.y, r0 = blockIdx.x * CCL_ROWS;
    if (r0 >= h) return;
    const int rows = min(CCL_ROWS, h - r0), n = rows * w;
    const long base = (long)s * w * h + (long)r0 * w;
    for (int k = threadIdx.x; k < n; k += CCL_TPB) lp[k] = isfin(cloud[base + k].x) ? k : -1;
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += CCL_TPB) {
        if (lp[k] < 0) continue;                   // invalid pixels never change
        const int rr = k / w, c = k - rr * w;
        const float4 p = cloud[base + k], nn = nrm[base + k];
        if (c >= 1 && lp[k - 1] >= 0 && plane_cmp(p, nn, nrm[base + k - 1], ang_thr)) lds_unite(lp, k, k - 1);
        if (rr >= 1 && lp[k - w] >= 0 && plane_cmp(p, nn, nrm[base + k - w], ang_thr)) lds_unite(lp, k, k - w);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += CCL_TPB) {
        const int v = lp[k];
        parent[base + k] = v < 0 ? -1 : (int)(base + lds_find(lp, k));
    }
}
__global__ void __launch_bounds__(CCL_TPB) k_ccl_local(const PlaneBatch B, int w, int h, float ang_thr) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_ccl_local(D.cloud, D.nrm, w, h, ang_thr, D.parent);
}


__device__ __forceinline__ void d_ccl_border(const float4* __restrict__ cloud, const float4* __restrict__ nrm, int w, int h,
                             float ang_thr, int* __restrict__ parent) {
    const int nb = (h - 1) / CCL_ROWS;                          // band boundaries per sensor
    const long total = 8L * nb * w;
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        const int s = (int)(t / ((long)nb * w));
        const int q = (int)(t - (long)s * nb * w);
        const int b = q / w, c = q - b * w;
        const long i = (long)s * w * h + (long)(b + 1) * CCL_ROWS * w + c;
        if (ld(parent + i) < 0 || ld(parent + i - w) < 0) continue;
        if (plane_cmp(cloud[i], nrm[i], nrm[i - w], ang_thr)) unite(parent, (int)i, (int)(i - w));
    }
}
__global__ void k_ccl_border(const PlaneBatch B, int w, int h, float ang_thr) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_ccl_border(D.cloud, D.nrm, w, h, ang_thr, D.parent);
}


// Roots, and the root count of every chunk of NUMC pixels of a sensor (grid (chunks, 8)) for k_ccl_number; also
// zeroes the label counts k_ccl_label accumulates (one launch instead of a memset).
constexpr int NUMC = 256;   // elements per chunk = threads per workgroup of the chunked numbering kernels

__device__ __forceinline__ void d_ccl_flatten(int* __restrict__ parent, int N, int* __restrict__ root,
                                                     int* __restrict__ cnt, int* __restrict__ ccnt) {
    const int s = blockIdx.y, j = blockIdx.x * NUMC + threadIdx.x;
    const long i = (long)s * N + j;
    bool is_root = false;
    if (j < N) {
        const int r = parent[i] < 0 ? -1 : find_root(parent, (int)i);
        root[i] = r;
        cnt[i] = 0;
        is_root = r == (int)i;
    }
    const int c = __syncthreads_count(is_root);
    if (threadIdx.x == 0) ccnt[s * gridDim.x + blockIdx.x] = c;
}
__global__ void __launch_bounds__(NUMC) k_ccl_flatten(const PlaneBatch B, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_ccl_flatten(D.parent, N, D.root, D.cnt, D.chunk);
}


// Exclusive rank of this thread's flag within its chunk, the chunk's offset (the sum of the counts of the chunks
// before it in the sensor) and the chunk's total; one workgroup of NUMC threads per chunk.
__device__ __forceinline__ int chunk_rank(bool flag, const int* __restrict__ ccnt_s, int chunk, int& off, int& tot) {
    __shared__ int s_w[NUMC / 64], s_off[NUMC / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int a = 0;
    for (int k = threadIdx.x; k < chunk; k += NUMC) a += ccnt_s[k];
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    const unsigned long long m = __ballot(flag);
    if (lane == 0) { s_off[wid] = a; s_w[wid] = __popcll(m); }
    __syncthreads();
    int o = 0, before = 0, t = 0;
    for (int w = 0; w < NUMC / 64; ++w) { o += s_off[w]; before += w < wid ? s_w[w] : 0; t += s_w[w]; }
    off = o;
    tot = t;
    return before + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// roots -> label ids in raster order; rank stored at the root's slot.  Grid (chunks, 8): a chunk's offset is the
// sum of k_ccl_flatten's root counts of the chunks before it, its roots are ranked with a ballot scan.
__device__ __forceinline__ void d_ccl_number(const int* __restrict__ root, int N, const int* __restrict__ ccnt,
                                                    int* __restrict__ rank, int* __restrict__ nlab) {
    const int s = blockIdx.y, j = blockIdx.x * NUMC + threadIdx.x;
    const long i = (long)s * N + j;
    const bool is_root = j < N && root[i] == (int)i;
    int off, tot;
    const int r = chunk_rank(is_root, ccnt + s * gridDim.x, blockIdx.x, off, tot);
    if (is_root) rank[i] = off + r;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) nlab[s] = off + tot;
}
__global__ void __launch_bounds__(NUMC) k_ccl_number(const PlaneBatch B, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_ccl_number(D.root, N, D.chunk, D.parent, D.nlab);
}


__device__ __forceinline__ void d_ccl_label(const int* __restrict__ root, const int* __restrict__ rank, int N, int* __restrict__ lab,
                            int* __restrict__ cnt) {
    const long total = 8L * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int rt = root[i];
        const int L = rt < 0 ? -1 : rank[rt];
        lab[i] = L;
        // wave-aggregated label counts
        const int s = (int)(i / N);
        long key = L < 0 ? -1 : (long)s * N + L;
        bool pending = key >= 0;
        while (__any(pending)) {
            const unsigned long long act = __ballot(pending);
            const int leader = __ffsll((long long)act) - 1;
            const long lk = __shfl(key, leader, 64);
            const bool mine = pending && key == lk;
            const unsigned long long same = __ballot(mine);
            if (mine && (int)(threadIdx.x & 63) == leader) atomicAdd(cnt + lk, __popcll(same));
            if (mine) pending = false;
        }
    }
}
__global__ void k_ccl_label(const PlaneBatch B, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_ccl_label(D.root, D.parent, N, D.lab, D.cnt);
}


// ------------------------------------------------------------------ moments
// float min / max through integer atomics (the accumulators start at +inf / -inf; -0 orders below +0)
__device__ __forceinline__ void atomic_fmin(float* p, float v) {
    if (v >= 0.f) atomicMin(reinterpret_cast<int*>(p), __float_as_int(v));
    else atomicMax(reinterpret_cast<unsigned*>(p), __float_as_uint(v));
}
__device__ __forceinline__ void atomic_fmax(float* p, float v) {
    if (v >= 0.f) atomicMax(reinterpret_cast<int*>(p), __float_as_int(v));
    else atomicMin(reinterpret_cast<unsigned*>(p), __float_as_uint(v));
}

__device__ __forceinline__ void add128(unsigned long long* p, r360p::i128 v) {
    const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
    const unsigned long long old = atomicAdd(p, lo);
    atomicAdd(p + 1, hi + (old + lo < old ? 1ull : 0ull));
}

// labels with more than min_inliers points, in increasing label order, and the label -> large-label index map
// (-1 for the others).  Grid (chunks of label ids, 8): k_big_count counts each chunk's large labels, k_big_list
// ranks them after the chunks before; the sensor's last chunk also zeroes the large labels' moment accumulators
// k_gm<false> adds into.
__device__ __forceinline__ void d_big_count(const int* __restrict__ cnt, const int* __restrict__ nlab, int N,
                                                   int min_inliers, int* __restrict__ bmap, int* __restrict__ ccnt) {
    const int s = blockIdx.y, j = blockIdx.x * NUMC + threadIdx.x;
    const long i = (long)s * N + j;
    bool big = false;
    if (j < nlab[s]) {
        big = cnt[i] > min_inliers;
        if (!big) bmap[i] = -1;
    }
    const int c = __syncthreads_count(big);
    if (threadIdx.x == 0) ccnt[s * gridDim.x + blockIdx.x] = c;
}
__global__ void __launch_bounds__(NUMC) k_big_count(const PlaneBatch B, int N, int min_inliers) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_big_count(D.cnt, D.nlab, N, min_inliers, D.parent, D.chunk);
}


__device__ __forceinline__ void d_big_list(const int* __restrict__ cnt, const int* __restrict__ nlab, int N,
                                                  int min_inliers, const int* __restrict__ ccnt, int* __restrict__ big,
                                                  int* __restrict__ nbig, int maxbig, int* __restrict__ err,
                                                  int* __restrict__ bmap, r360p::Moments* __restrict__ mom,
                                                  int* __restrict__ bfirst) {
    const int s = blockIdx.y, j = blockIdx.x * NUMC + threadIdx.x;
    const long i = (long)s * N + j;
    const bool is_big = j < nlab[s] && cnt[i] > min_inliers;
    int off, tot;
    const int r = chunk_rank(is_big, ccnt + s * gridDim.x, blockIdx.x, off, tot);
    if (is_big) {
        const int b = off + r;
        bmap[i] = b < maxbig ? b : -1;
        if (b < maxbig) big[s * maxbig + b] = j;
    }
    if (blockIdx.x == gridDim.x - 1) {
        const int all = off + tot, nb = all < maxbig ? all : maxbig;
        if (threadIdx.x == 0) {
            nbig[s] = nb;
            if (all > maxbig) atomicOr(err, 2);
        }
        for (int q = threadIdx.x; q < nb; q += NUMC) {
            r360p::moments_zero(mom[s * maxbig + q]);
            bfirst[s * maxbig + q] = N;
        }
    }
}
__global__ void __launch_bounds__(NUMC) k_big_list(const PlaneBatch B, int N, int min_inliers, int maxbig) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_big_list(D.cnt, D.nlab, N, min_inliers, D.chunk, D.big, D.nbig, maxbig, D.err, D.parent, D.mom, D.aux);
}


// ------------------------------------------------------------------ pixel-order grouped moments
// The moments of every large label (k_gm<false>) and of every refined model region (k_gm<true>) straight from the
// label images, with no grouped pixel list: a workgroup streams a contiguous pixel range, each wave a contiguous
// quarter of it in chunks of 64 consecutive pixels, whose labels, keys and points it loads up front.  A chunk's
// pixels form runs of equal keys (raster order: a few per chunk); one segmented inclusive scan across the wave sums
// every run at once, and the last lane of each run adds the run's sums into a workgroup table in LDS (so one LDS
// deposit per run instead of a conflicting atomic per pixel).  The table (GM_SLOTS open-addressed slots) goes to
// the global accumulators at the end, 14 lanes per slot; a key that finds no free slot is merged into the global
// accumulators directly.  Global atomics execute at the memory side, and a planar region spans hundreds of
// workgroups: the region accumulators are kept in GM_COPIES copies (workgroup x adds into copy x % GM_COPIES) that
// k_nbmask folds into the region records, so that no word takes more than 1/8 of the adds.  Exact integer sums
// (int128 as a low / high pair whose carry each adder derives from the old low word it got back) and min / max: the
// result is independent of the grouping, bit for bit the same as summing each region's pixels in any order.
constexpr int GM_TPB = 256, GM_SLOTS = 64, GM_PX = 512, GM_COPIES = R360_GM_COPIES;


struct GmShared {
    int key[GM_SLOTS];
    unsigned long long w[GM_SLOTS][20];   // n, s1[3], s2 (lo, hi) x 6, c[4]
    float b[GM_SLOTS][6];                 // model regions: local-frame min xyz, max xyz
    int first[GM_SLOTS];                  // large labels: first pixel
};

struct GmAcc {   // one lane's sums for one key
    long long n, s1[3], c[4];
    r360p::i128 s2[6];
    float b[6];
    int first;
};

__device__ __forceinline__ void gm_zero(GmAcc& a) {
    a.n = 0;
    a.first = 0x7fffffff;
    for (int k = 0; k < 3; ++k) a.s1[k] = 0;
    for (int k = 0; k < 4; ++k) a.c[k] = 0;
    for (int k = 0; k < 6; ++k) { a.s2[k] = 0; a.b[k] = k < 3 ? 3.4e38f : -3.4e38f; }
}


// one lane's sums of key into the workgroup table (or, with the table full, into the global accumulators)
template <bool MODEL>
__device__ __forceinline__ void gm_deposit(GmShared* sh, int key, const GmAcc& a, r360p::Moments* gmom, int* gfirst,
                                           RegionPart* gout) {
    int h = key & (GM_SLOTS - 1), t = 0;
#pragma unroll 1
    for (; t < GM_SLOTS; ++t, h = (h + 1) & (GM_SLOTS - 1)) {
        const int old = atomicCAS(&sh->key[h], -1, key);
        if (old == -1 || old == key) break;
    }
    if (t < GM_SLOTS) {
        unsigned long long* d = sh->w[h];
        if (a.n) {
            atomicAdd(d + 0, (unsigned long long)a.n);
            for (int k = 0; k < 3; ++k) atomicAdd(d + 1 + k, (unsigned long long)a.s1[k]);
            for (int k = 0; k < 6; ++k) add128(d + 4 + 2 * k, a.s2[k]);
        }
        if (MODEL) {
            for (int k = 0; k < 4; ++k) atomicAdd(d + 16 + k, (unsigned long long)a.c[k]);
            for (int k = 0; k < 3; ++k) { atomic_fmin(&sh->b[h][k], a.b[k]); atomic_fmax(&sh->b[h][k + 3], a.b[k + 3]); }
        } else {
            atomicMin(&sh->first[h], a.first);
        }
        return;
    }
    r360p::Moments* dst = MODEL ? &gout[key].m : &gmom[key];
    if (a.n) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&dst->n), (unsigned long long)a.n);
        for (int k = 0; k < 3; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(&dst->s1[k]), (unsigned long long)a.s1[k]);
        for (int k = 0; k < 6; ++k) add128(reinterpret_cast<unsigned long long*>(&dst->s2[k]), a.s2[k]);
    }
    if (MODEL) {
        for (int k = 0; k < 4; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(&dst->c[k]), (unsigned long long)a.c[k]);
        for (int k = 0; k < 3; ++k) { atomic_fmin(&gout[key].bmin[k], a.b[k]); atomic_fmax(&gout[key].bmax[k], a.b[k + 3]); }
    } else {
        atomicMin(gfirst + key, a.first);
    }
}

// Segmented inclusive scan of the lanes' contributions within runs of lanes (head: the first lane of this lane's
// run), on DPP lane moves (no LDS): row_shr 1, 2, 4, 8 inside each row of 16 lanes, then row_bcast:15 (rows 1 and 3
// take the last lane of the row before) and row_bcast:31 (rows 2 and 3 take lane 31); a lane takes a moved value
// only when the source lane lies in its run.  The pixel counts and first pixels are not scanned (run lengths and
// ballots give them).
template <int CTRL>
__device__ __forceinline__ unsigned dpp32(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ long long dpp64(long long v) {
    const unsigned lo = dpp32<CTRL>((unsigned)(unsigned long long)v), hi = dpp32<CTRL>((unsigned)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
template <int CTRL>
__device__ __forceinline__ r360p::i128 dpp128(r360p::i128 v) {
    const unsigned long long lo = (unsigned long long)dpp64<CTRL>((long long)(unsigned long long)v);
    const unsigned long long hi = (unsigned long long)dpp64<CTRL>((long long)(unsigned long long)(v >> 64));
    return (r360p::i128)(((unsigned __int128)hi << 64) | lo);
}
template <bool MODEL, int CTRL>
__device__ __forceinline__ void gm_scan_step(GmAcc& v, bool take) {
    long long s1[3];
    r360p::i128 s2[6];
    for (int k = 0; k < 3; ++k) s1[k] = dpp64<CTRL>(v.s1[k]);
    for (int k = 0; k < 6; ++k) s2[k] = dpp128<CTRL>(v.s2[k]);
    if (MODEL) {
        long long c[4];
        float b[6];
        for (int k = 0; k < 4; ++k) c[k] = dpp64<CTRL>(v.c[k]);
        for (int k = 0; k < 6; ++k) b[k] = __uint_as_float(dpp32<CTRL>(__float_as_uint(v.b[k])));
        if (take) {
            for (int k = 0; k < 4; ++k) v.c[k] += c[k];
            for (int k = 0; k < 3; ++k) { v.b[k] = fminf(v.b[k], b[k]); v.b[k + 3] = fmaxf(v.b[k + 3], b[k + 3]); }
        }
    }
    if (take) {
        for (int k = 0; k < 3; ++k) v.s1[k] += s1[k];
        for (int k = 0; k < 6; ++k) v.s2[k] += s2[k];
    }
}
template <bool MODEL>
__device__ __forceinline__ void gm_seg_scan(GmAcc& v, int lane, int head) {
    const int r = lane & 15, row = lane >> 4;
    gm_scan_step<MODEL, 0x111>(v, r >= 1 && head <= lane - 1);   // row_shr:1
    gm_scan_step<MODEL, 0x112>(v, r >= 2 && head <= lane - 2);   // row_shr:2
    gm_scan_step<MODEL, 0x114>(v, r >= 4 && head <= lane - 4);   // row_shr:4
    gm_scan_step<MODEL, 0x118>(v, r >= 8 && head <= lane - 8);   // row_shr:8
    gm_scan_step<MODEL, 0x142>(v, (row & 1) && head <= (lane & ~15) - 1);   // row_bcast:15
    gm_scan_step<MODEL, 0x143>(v, row >= 2 && head <= 31);                   // row_bcast:31
}

// MODEL = false (large labels): key = s * R360_MAX_BIG + bmap[label], moments of the finite points, first pixel into
//   bfirst; also clears the label -> model map (mmap) k_plane_fit fills.
// MODEL = true (refined regions): key = s * R360_MAX_MODELS + mmap[labf], moments of the points in the rig frame
//   (Eigen Affine3f * Vector3f with the sensor's column-major pose, pcl::transformPointCloud) and of the colours, and
//   the local-frame bounds, into copy blockIdx.x % GM_COPIES.  The accumulators were zeroed (bounds at -+3.4e38) by
//   k_big_list / k_plane_fit.
template <bool MODEL, int CPW>   // CPW: chunks of 64 pixels per wave (a workgroup takes 256 * CPW pixels)
__device__ __forceinline__ void d_gm(const float4* __restrict__ cloud, const uchar4* __restrict__ rgb,
                                             const int* __restrict__ lab, int N, const int* __restrict__ kmap,
                                             int* __restrict__ mmap_clear, const float* __restrict__ rt8,
                                             r360p::Moments* __restrict__ gmom, int* __restrict__ gfirst,
                                             RegionPart* __restrict__ gpart, int exp) {
    __shared__ GmShared sh;
    RegionPart* const gout = MODEL ? gpart + (blockIdx.x % GM_COPIES) * 8 * R360_MAX_MODELS : nullptr;
    for (int q = threadIdx.x; q < GM_SLOTS; q += GM_TPB) {
        sh.key[q] = -1;
        sh.first[q] = 0x7fffffff;
        for (int k = 0; k < 20; ++k) sh.w[q][k] = 0;
        for (int k = 0; k < 6; ++k) sh.b[q][k] = k < 3 ? 3.4e38f : -3.4e38f;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long total = 8L * N;
    const long w0 = ((long)blockIdx.x * GM_TPB * CPW) + (long)wid * 64 * CPW + lane;   // this lane's first pixel
    // the wave's chunks' labels, keys and points loaded up front (three rounds of CPW independent loads)
    int key[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const long i = w0 + 64 * c;
        key[c] = i < total ? lab[i] : -1;
        if (!MODEL && i < total) mmap_clear[i] = -1;
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const long i = w0 + 64 * c;
        const int s = (int)(i / N);
        const int m = key[c] >= 0 ? kmap[(long)s * N + key[c]] : -1;
        key[c] = m >= 0 ? s * (MODEL ? R360_MAX_MODELS : R360_MAX_BIG) + m : -1;
    }
    float4 pt[CPW];
    uchar4 col[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const long i = w0 + 64 * c;
        pt[c] = key[c] >= 0 ? cloud[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (MODEL) col[c] = key[c] >= 0 ? rgb[i] : make_uchar4(0, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const long i = w0 + 64 * c;
        const int s = (int)(i / N);
        GmAcc p;                       // this pixel's contribution
        gm_zero(p);
        if (key[c] >= 0) {
            const float4 q = pt[c];
            float x = q.x, y = q.y, z = q.z;
            bool add = true;
            if (MODEL) {
                p.b[0] = q.x; p.b[1] = q.y; p.b[2] = q.z; p.b[3] = q.x; p.b[4] = q.y; p.b[5] = q.z;
                const float* T = rt8 + 16 * s;
                x = T[0] * q.x + T[4] * q.y + T[8] * q.z + T[12];
                y = T[1] * q.x + T[5] * q.y + T[9] * q.z + T[13];
                z = T[2] * q.x + T[6] * q.y + T[10] * q.z + T[14];
                const uchar4 cc = col[c];
                const int sum = cc.x + cc.y + cc.z;
                if (sum != 0) {   // r360p::moments_add_rgb
                    const float inv = 1.0f / float(sum);
                    p.c[0] = (long long)((double)(float(cc.x) * inv) * 8589934592.0);
                    p.c[1] = (long long)((double)(float(cc.y) * inv) * 8589934592.0);
                    p.c[2] = (long long)((double)(float(cc.z) * inv) * 8589934592.0);
                }
                p.c[3] = sum;
            } else {
                p.first = (int)(i - (long)s * N);
                add = isfin(q.x) && isfin(q.y) && isfin(q.z);
            }
            if (add) {   // r360p::moments_add_xyz
                const long long qv[3] = {r360p::q36(x), r360p::q36(y), r360p::q36(z)};
                p.n = 1;
                for (int k = 0; k < 3; ++k) p.s1[k] = qv[k];
                p.s2[0] = (r360p::i128)qv[0] * qv[0];
                p.s2[1] = (r360p::i128)qv[0] * qv[1];
                p.s2[2] = (r360p::i128)qv[0] * qv[2];
                p.s2[3] = (r360p::i128)qv[1] * qv[1];
                p.s2[4] = (r360p::i128)qv[1] * qv[2];
                p.s2[5] = (r360p::i128)qv[2] * qv[2];
            }
        }
        // one segmented inclusive scan over the chunk's runs of equal keys; the last lane of a run deposits it
        const unsigned long long heads = __ballot(lane == 0 || key[c] != __shfl_up(key[c], 1, 64));
        const unsigned long long le = lane == 63 ? ~0ull : (2ull << lane) - 1;
        const int head = 63 - __clzll((long long)(heads & le));
        const unsigned long long fin = __ballot(p.n != 0);   // pixels with moments (labels: finite points)
        if (!(exp & 4)) gm_seg_scan<MODEL>(p, lane, head);
        const bool tail = lane == 63 || ((heads >> (lane + 1)) & 1ull);
        if (!(exp & 2) && tail && key[c] >= 0) {
            const unsigned long long run = le & ~((1ull << head) - 1);
            p.n = __popcll(fin & run);
            p.first -= lane - head;   // the run's first pixel (consecutive pixels of one sensor)
            gm_deposit<MODEL>(&sh, key[c], p, gmom, gfirst, gout);
        }
    }
    __syncthreads();
    // the table into the global accumulators: slot q by 32 lanes (14 words, 6 bounds or the first pixel)
    for (int q = threadIdx.x >> 5; q < GM_SLOTS; q += GM_TPB / 32) {
        const int key = sh.key[q];
        if (key < 0 || (exp & 1)) continue;
        const int l = threadIdx.x & 31;
        r360p::Moments* dst = MODEL ? &gout[key].m : &gmom[key];
        if (l < 6) {
            unsigned long long* d = reinterpret_cast<unsigned long long*>(&dst->s2[l]);
            const unsigned long long lo = sh.w[q][4 + 2 * l], hi = sh.w[q][5 + 2 * l];
            const unsigned long long old = atomicAdd(d, lo);
            atomicAdd(d + 1, hi + (old + lo < old ? 1ull : 0ull));
        } else if (l < 14) {
            const int k = l - 6;   // n, s1[0..2], c[0..3]
            if (k < 4 || MODEL) {
                long long* d = k == 0 ? &dst->n : k < 4 ? &dst->s1[k - 1] : &dst->c[k - 4];
                atomicAdd(reinterpret_cast<unsigned long long*>(d), sh.w[q][k == 0 ? 0 : k < 4 ? k : 12 + k]);
            }
        } else if (MODEL && l < 20) {
            const int k = l - 14;
            if (k < 3) atomic_fmin(&gout[key].bmin[k], sh.b[q][k]);
            else atomic_fmax(&gout[key].bmax[k - 3], sh.b[q][k]);
        } else if (!MODEL && l == 14) {
            atomicMin(gfirst + key, sh.first[q]);
        }
    }
}
template <bool MODEL, int CPW>
__global__ void __launch_bounds__(GM_TPB) k_gm(const PlaneBatch B, int N, int exp) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_gm<MODEL, CPW>(D.cloud, MODEL ? D.rgb : nullptr, MODEL ? D.labf : D.lab, N, MODEL ? D.root : D.parent, MODEL ? nullptr : D.root, MODEL ? D.rt : nullptr, MODEL ? nullptr : D.mom, MODEL ? nullptr : D.aux, MODEL ? D.gpart : nullptr, exp);
}


// OrganizedMultiPlaneSegmentation::segment plane fit, one thread per sensor over its large labels in
// label order (the viewpoint vp accumulates across labels, as in PCL 1.7)
// One workgroup per sensor.  The eigen33 fits of the large labels are independent (one thread each); the only
// order dependence of segment() is the viewpoint vp, which accumulates the centroids of all previous labels in
// float — four sequential subtraction chains, one lane per component — and decides each label's flip; the
// planar labels are then numbered in label order.
constexpr int PF_TPB = 256;

__device__ __forceinline__ void d_plane_fit(const r360p::Moments* __restrict__ mom, const int* __restrict__ big,
                                                     const int* __restrict__ nbig, int maxbig, float max_curvature,
                                                     PlaneModel* __restrict__ models, int* __restrict__ nmodels,
                                                     int* __restrict__ err, int N, int* __restrict__ mmap,
                                                     const int* __restrict__ bfirst, PlaneOut* __restrict__ out,
                                                     RegionPart* __restrict__ gpart) {
    __shared__ float s_c[R360_MAX_BIG][4], s_pp[R360_MAX_BIG][4], s_vp[R360_MAX_BIG][4];
    __shared__ float s_curv[R360_MAX_BIG];
    __shared__ int s_idx[R360_MAX_BIG];
    const int s = blockIdx.x;
    const int nb = min(nbig[s], maxbig);
    for (int b = threadIdx.x; b < nb; b += PF_TPB) {
        const r360p::Moments m = mom[s * maxbig + b];
        double mean[3], cv[9];
        r360p::moments_mean_cov(m, mean, cv);
        float centroid[4] = {(float)mean[0], (float)mean[1], (float)mean[2], 1.f};
        float cov[9];
        for (int k = 0; k < 9; ++k) cov[k] = (float)cv[k];
        float eval, evec[3];
        r360p::eigen33_min(cov, eval, evec);
        float pp[4] = {evec[0], evec[1], evec[2], 0};
        pp[3] = -1 * r360p::dot4(pp, centroid);
        const float eig_sum = cov[0] + cov[4] + cov[8];
        s_curv[b] = eig_sum != 0 ? fabsf(eval / eig_sum) : 0.f;
        for (int k = 0; k < 4; ++k) { s_c[b][k] = centroid[k]; s_pp[b][k] = pp[k]; }
    }
    __syncthreads();
    if (threadIdx.x < 4) {   // vp after label b: vp -= centroid, in label order
        const int k = threadIdx.x;
        float v = 0.f;
        for (int b = 0; b < nb; ++b) { v -= s_c[b][k]; s_vp[b][k] = v; }
    }
    if (threadIdx.x == 32) {   // planar labels numbered in label order (wave 0, lane 32: beside the vp chains)
        int nm = 0;
        for (int b = 0; b < nb; ++b) s_idx[b] = s_curv[b] < max_curvature ? nm++ : -1;
        if (nm > R360_MAX_MODELS) atomicOr(err, 4);
        nmodels[s] = nm < R360_MAX_MODELS ? nm : R360_MAX_MODELS;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += PF_TPB) {
        const int nm = s_idx[b];
        if (nm < 0 || nm >= R360_MAX_MODELS) continue;
        float centroid[4], pp[4], vp[4];
        for (int k = 0; k < 4; ++k) { centroid[k] = s_c[b][k]; pp[k] = s_pp[b][k]; vp[k] = s_vp[b][k]; }
        const float cos_theta = r360p::dot4(vp, pp);
        if (cos_theta < 0) {
            for (int k = 0; k < 4; ++k) pp[k] *= -1;
            pp[3] = -1 * r360p::dot4(pp, centroid);
        }
        // the label's covariance again (cheap next to the eigen solve; keeps the LDS small)
        const r360p::Moments m = mom[s * maxbig + b];
        double mean[3], cv[9];
        r360p::moments_mean_cov(m, mean, cv);
        PlaneModel& M = models[s * R360_MAX_MODELS + nm];
        M.label = big[s * maxbig + b];
        M.big = b;
        mmap[(long)s * N + M.label] = nm;
        M.n_fit = (int)m.n;
        for (int k = 0; k < 4; ++k) M.v[k] = pp[k];
        for (int k = 0; k < 3; ++k) M.centroid[k] = centroid[k];
        for (int k = 0; k < 9; ++k) M.cov[k] = (float)cv[k];
        M.curvature = s_curv[b];
        // the region record, and the copies of its accumulators k_gm<true> adds into (bounds at -+3.4e38: a region
        // left without pixels after the refinement keeps them, as the reference's min / max over an empty cloud)
        PlaneOut& O = out[s * R360_MAX_MODELS + nm];
        O.model = M;
        O.start = bfirst[s * maxbig + b];
        for (int c = 0; c < GM_COPIES; ++c) {
            RegionPart& G = gpart[(c * 8 + s) * R360_MAX_MODELS + nm];
            r360p::moments_zero(G.m);
            for (int k = 0; k < 3; ++k) { G.bmin[k] = 3.4e38f; G.bmax[k] = -3.4e38f; }
        }
        O.n_contour = 0;
        O.contour_off = 0;
        O.n_vox = 0;
        O.vox_fill = 0;
        O.vox_off = 0;
    }
}
__global__ void __launch_bounds__(PF_TPB) k_plane_fit(const PlaneBatch B, int maxbig, float max_curvature, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_plane_fit(D.mom, D.big, D.nbig, maxbig, max_curvature, D.models, D.nmodels, D.err, N, D.root, D.aux, D.out, D.gpart);
}


// ------------------------------------------------------------------ refine
// state: -1 no label, -2 non-planar label, m >= 0 planar model m.  mask bit m: |model_m . p| < 0.02
__device__ __forceinline__ void d_refine_init(const float4* __restrict__ cloud, const int* __restrict__ lab, int N,
                              const PlaneModel* __restrict__ models, const int* __restrict__ nmodels,
                              int8_t* __restrict__ state, unsigned long long* __restrict__ mask) {
    const long total = 8L * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        const int L = lab[i];
        const int nm = nmodels[s];
        const PlaneModel* M = models + s * R360_MAX_MODELS;
        int st = L < 0 ? -1 : -2;
        unsigned long long bits = 0;
        const float4 p = cloud[i];
        for (int m = 0; m < nm; ++m) {
            if (L >= 0 && M[m].label == L) st = m;
            const double ptp = fabs((double)(M[m].v[0] * p.x + M[m].v[1] * p.y + M[m].v[2] * p.z + M[m].v[3]));
            if (ptp < (double)0.02f) bits |= 1ull << m;
        }
        state[i] = (int8_t)st;
        mask[i] = bits;
    }
}
__global__ void k_refine_init(const PlaneBatch B, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_init(D.cloud, D.lab, N, D.models, D.nmodels, D.state, D.mask);
}


// Chain resolution of one row.  The row is laid out in walking order across the wave: lane l holds
// the K consecutive walking positions l*K .. l*K+K-1 (left-to-right in the first sweep, right-to-left
// in the second).  L[k]: states, M[k]: closeness masks; F receives the states after the chain.
template <int K>
__device__ void resolve_chain(const int (&L)[K], const unsigned long long (&M)[K], int (&F)[K]) {
    const int lane = threadIdx.x & 63;
    // lane summary: anchored (some non-chain state) -> outgoing value fixed; else AND of masks
    bool anch = false;
    unsigned long long am = ~0ull;
    int out = -2;
    {
        int v = -2;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (L[k] != -2) { anch = true; v = L[k]; }
            else if (anch) v = (v >= 0 && ((M[k] >> v) & 1)) ? v : -2;
            else am &= M[k];
        }
        out = v;
    }
    // inclusive max-scan of anchor lanes and segmented AND-scan of masks since the last anchor
    int apos = anch ? lane : -1;
    unsigned long long segm = anch ? ~0ull : am;
    int segf = anch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int pa = __shfl_up(apos, o, 64);
        const unsigned long long pm = __shfl_up(segm, o, 64);
        const int pf = __shfl_up(segf, o, 64);
        if (lane >= o) {
            apos = pa > apos ? pa : apos;
            if (!segf) { segm &= pm; segf = pf; }
        }
    }
    const int a_prev = __shfl_up(apos, 1, 64);                 // last anchor lane before this lane
    const unsigned long long m_prev = __shfl_up(segm, 1, 64);  // AND of masks after that anchor
    const int o_anchor = __shfl(out, a_prev < 0 ? 0 : a_prev, 64);
    int in = -2;
    if (lane > 0 && a_prev >= 0 && o_anchor >= 0 && ((m_prev >> o_anchor) & 1)) in = o_anchor;
    int v = in;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        F[k] = (L[k] == -2 && v >= 0 && ((M[k] >> v) & 1)) ? v : L[k];
        v = F[k];
    }
}

// One wave per sensor walks the rows.  Rows are loaded two ahead into three register sets used in
// rotation (the loop is unrolled by three), so no loop-carried copy of an in-flight load forces a
// vmcnt(0) per row, and every load is unconditional (clamped column, value masked afterwards).
template <int K>
__device__ void refine_sweeps(int8_t* __restrict__ state_all, const unsigned long long* __restrict__ mask_all, int w,
                              int h, int s, int sweeps, int r_top = -1) {
    if (r_top < 0) r_top = h - 1;   // the second sweep's first source row (rows above it are already swept)
    const int lane = threadIdx.x & 63;
    const long N = (long)w * h;
    int8_t* S = state_all + s * N;
    const unsigned long long* MK = mask_all + s * N;
    auto col = [&](int k, int dir) { return dir > 0 ? lane * K + k : (63 - lane) * K + (K - 1 - k); };
    auto load = [&](int r, int (&L)[K], unsigned long long (&M)[K], int dir) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            // walking order: dir>0 -> column lane*K + k; dir<0 -> column (63-lane)*K + (K-1-k)
            const int c = col(k, dir);
            const int cc = c < w ? c : w - 1;
            const int v = S[(long)r * w + cc];
            const unsigned long long m = MK[(long)r * w + cc];
            L[k] = c < w ? v : -1;
            M[k] = c < w ? m : 0ull;
        }
    };
    auto store = [&](int r, const int (&L)[K], int dir) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int c = col(k, dir);
            if (c < w) S[(long)r * w + c] = (int8_t)L[k];
        }
    };
    int A[K], B[K], C[K];
    unsigned long long Am[K], Bm[K], Cm[K];
    // ---------------- first sweep: top->bottom, left->right; right and down checks
    if (sweeps & 1) {
        auto step = [&](int r, int (&cur)[K], unsigned long long (&cm)[K], int (&nxt)[K], unsigned long long (&nm)[K],
                        int (&nn)[K], unsigned long long (&nnm)[K]) {
            if (r + 2 < h) load(r + 2, nn, nnm, +1);     // consumed two steps later
            int F[K];
            resolve_chain<K>(cur, cm, F);
            // original state of the column to the right of each of this lane's columns
            const int right_of_last = __shfl(cur[0], (lane + 1) & 63, 64);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int c = lane * K + k;
                if (c >= w - 1) continue;
                const int rl = k + 1 < K ? cur[k + 1] : (lane < 63 ? right_of_last : -1);
                if (F[k] == -1 || rl == -1) continue;
                if (nxt[k] == -1) continue;
                if (F[k] >= 0 && nxt[k] == -2 && ((nm[k] >> F[k]) & 1)) nxt[k] = F[k];
            }
            store(r, F, +1);
        };
        load(0, A, Am, +1);
        if (h > 1) load(1, B, Bm, +1);
        int r = 0;
        for (; r + 3 <= h - 1; r += 3) {
            step(r, A, Am, B, Bm, C, Cm);
            step(r + 1, B, Bm, C, Cm, A, Am);
            step(r + 2, C, Cm, A, Am, B, Bm);
        }
        const int rem = (h - 1) - r;
        if (rem == 0) store(h - 1, A, +1);
        else if (rem == 1) { step(r, A, Am, B, Bm, C, Cm); store(h - 1, B, +1); }
        else { step(r, A, Am, B, Bm, C, Cm); step(r + 1, B, Bm, C, Cm, A, Am); store(h - 1, C, +1); }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // ---------------- second sweep: bottom->top, right->left; left and up checks
    if (sweeps & 2) {
        const int cl = w - 1;                                    // owner of column w-1 (walking order)
        const int own_lane = 63 - cl / K, own_k = K - 1 - cl % K;
        auto step = [&](int r, int (&cur)[K], unsigned long long (&cm)[K], int (&up)[K], unsigned long long (&um)[K],
                        int (&uu)[K], unsigned long long (&uum)[K]) {
            if (r - 2 >= 0) load(r - 2, uu, uum, -1);    // consumed two steps later
            int F[K];
            resolve_chain<K>(cur, cm, F);
            // original state of the column to the left (walking order: the next element)
            const int left_of_last = __shfl(cur[0], (lane + 1) & 63, 64);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int c = (63 - lane) * K + (K - 1 - k);
                if (c >= w || c == 0) continue;
                const int ll = k + 1 < K ? cur[k + 1] : (lane < 63 ? left_of_last : -1);
                if (F[k] == -1 || ll == -1) continue;
                if (up[k] == -1) continue;
                if (F[k] >= 0 && up[k] == -2 && ((um[k] >> F[k]) & 1)) up[k] = F[k];
            }
            // column 0: its "left" neighbour is the last pixel of the row above (flat-index wrap)
            int upw = -1;
            unsigned long long upw_m = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k == own_k) { upw = up[k]; upw_m = um[k]; }
            upw = __shfl(upw, own_lane, 64);
            upw_m = __shfl(upw_m, own_lane, 64);
            const int f0 = __shfl(F[K - 1], 63, 64);             // column 0 = lane 63, k = K-1
            const int up0 = __shfl(up[K - 1], 63, 64);
            const unsigned long long um0 = __shfl(um[K - 1], 63, 64);
            int new_upw = upw, new_up0 = up0;
            if (f0 != -1 && upw != -1) {
                if (f0 >= 0 && upw == -2 && ((upw_m >> f0) & 1)) new_upw = f0;
                if (up0 != -1 && f0 >= 0 && up0 == -2 && ((um0 >> f0) & 1)) new_up0 = f0;
            }
            if (w - 1 == 0) new_upw = new_up0;                   // degenerate single-column image
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (lane == own_lane && k == own_k) up[k] = new_upw;
                if (lane == 63 && k == K - 1) up[k] = new_up0;
            }
            store(r, F, -1);
        };
        load(r_top, A, Am, -1);
        if (r_top >= 1) load(r_top - 1, B, Bm, -1);
        int r = r_top;
        for (; r - 3 >= 0; r -= 3) {
            step(r, A, Am, B, Bm, C, Cm);
            step(r - 1, B, Bm, C, Cm, A, Am);
            step(r - 2, C, Cm, A, Am, B, Bm);
        }
        if (r == 0) store(0, A, -1);
        else if (r == 1) { step(1, A, Am, B, Bm, C, Cm); store(0, B, -1); }
        else { step(2, A, Am, B, Bm, C, Cm); step(1, B, Bm, C, Cm, A, Am); store(0, C, -1); }
    }
}

template <int K>
__device__ __forceinline__ void d_refine(int8_t* __restrict__ state_all,
                                              const unsigned long long* __restrict__ mask_all, int w, int h) {
    refine_sweeps<K>(state_all, mask_all, w, h, blockIdx.x, 3);
}
template <int K>
__global__ void __launch_bounds__(64) k_refine(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine<K>(D.state, D.mask, w, h);
}


// ------------------------------------------------------------------ banded refine
// The sweeps are sequential along rows (row r's swept states change row r+1 in the first sweep, row r-1
// in the second), but the change only travels through non-planar (-2) pixels close to a model, so it dies
// out within a few rows.  Each sweep therefore runs in two phases over row bands of rb rows:
//   phase 1  every (sensor, band) in parallel, one wave each, assuming no incoming assignment into the
//            band's first row; the band's assignments into the next band's first row are kept (rbnd) with
//            a flag telling whether they changed that row;
//   phase 2  one wave per sensor walks the bands in sweep order: a band whose incoming row was changed
//            (flag of the previous band) is swept again from the true incoming row until a swept row equals
//            its phase-1 result — every later row of the band (and its boundary) is then unchanged.
// The result is the sequential sweep's, bit for bit.  The sweeps read Sin (unchanged) and write Sout.
//
// One band of one sweep: DIR = +1 rows top->bottom, columns left->right, right/down checks (rows 0..h-2
// swept, row h-1 only receives); DIR = -1 rows bottom->top, columns right->left, left/up checks with the
// flat-index wrap of column 0 (rows h-1..1 swept, row 0 only receives).
template <int K, int DIR>
__device__ void refine_band(const int8_t* __restrict__ Sin, int8_t* __restrict__ Sout,
                            const unsigned long long* __restrict__ MK, int w, int h, int r0, int r1,
                            const int8_t* __restrict__ init, int8_t* __restrict__ bnd_out, int* __restrict__ flag_out,
                            bool conv) {
    const int lane = threadIdx.x & 63;
    auto col = [&](int k) { return DIR > 0 ? lane * K + k : (63 - lane) * K + (K - 1 - k); };
    auto load = [&](const int8_t* src, int r, int (&L)[K], unsigned long long (&M)[K]) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int c = col(k);
            const int cc = c < w ? c : w - 1;
            const int v = src[(long)r * w + cc];
            const unsigned long long m = MK[(long)r * w + cc];
            L[k] = c < w ? v : -1;
            M[k] = c < w ? m : 0ull;
        }
    };
    const int first = DIR > 0 ? r0 : r1 - 1, last = DIR > 0 ? r1 - 1 : r0;
    int cur[K];
    unsigned long long cm[K];
    if (init) {
        int dummy[K];
        load(Sin, first, dummy, cm);
#pragma unroll
        for (int k = 0; k < K; ++k) { const int c = col(k); cur[k] = c < w ? (int)init[c] : -1; }
    } else {
        load(Sin, first, cur, cm);
    }
    const int cl = w - 1;                                    // owner of column w-1 in walking order (DIR < 0)
    const int own_lane = 63 - cl / K, own_k = K - 1 - cl % K;
    // conv: the phase-1 states of the current row, loaded one row ahead like the inputs
    auto load_out = [&](int r, int (&P)[K]) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int c = col(k);
            P[k] = (int)Sout[(long)r * w + (c < w ? c : w - 1)];
        }
    };
    int po[K];
    if (conv) load_out(first, po);
    for (int r = first;; r += DIR) {
        const int nr = r + DIR;
        const bool has_nr = nr >= 0 && nr < h;
        int nxt[K], nxt0[K], pn[K];
        unsigned long long nm[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { nxt[k] = -1; nm[k] = 0ull; pn[k] = 0; }
        if (has_nr) load(Sin, nr, nxt, nm);
        if (conv && has_nr && r != last) load_out(nr, pn);
#pragma unroll
        for (int k = 0; k < K; ++k) nxt0[k] = nxt[k];
        int F[K];
        const bool swept = DIR > 0 ? r <= h - 2 : r >= 1;
        if (swept) {
            resolve_chain<K>(cur, cm, F);
            // original state of the next column in walking order (right in the first sweep, left in the second)
            const int next_of_last = __shfl(cur[0], (lane + 1) & 63, 64);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int c = col(k);
                if (DIR > 0 ? c >= w - 1 : (c >= w || c == 0)) continue;
                const int nl = k + 1 < K ? cur[k + 1] : (lane < 63 ? next_of_last : -1);
                if (F[k] == -1 || nl == -1) continue;
                if (nxt[k] == -1) continue;
                if (F[k] >= 0 && nxt[k] == -2 && ((nm[k] >> F[k]) & 1)) nxt[k] = F[k];
            }
            if (DIR < 0) {
                // column 0: its "left" neighbour is the last pixel of the row above (flat-index wrap)
                int upw = -1;
                unsigned long long upw_m = 0;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (k == own_k) { upw = nxt[k]; upw_m = nm[k]; }
                upw = __shfl(upw, own_lane, 64);
                upw_m = __shfl(upw_m, own_lane, 64);
                const int f0 = __shfl(F[K - 1], 63, 64);     // column 0 = lane 63, k = K-1
                const int up0 = __shfl(nxt[K - 1], 63, 64);
                const unsigned long long um0 = __shfl(nm[K - 1], 63, 64);
                int new_upw = upw, new_up0 = up0;
                if (f0 != -1 && upw != -1) {
                    if (f0 >= 0 && upw == -2 && ((upw_m >> f0) & 1)) new_upw = f0;
                    if (up0 != -1 && f0 >= 0 && up0 == -2 && ((um0 >> f0) & 1)) new_up0 = f0;
                }
                if (w - 1 == 0) new_upw = new_up0;           // degenerate single-column image
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (lane == own_lane && k == own_k) nxt[k] = new_upw;
                    if (lane == 63 && k == K - 1) nxt[k] = new_up0;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) F[k] = cur[k];
        }
        if (conv) {   // converged onto the phase-1 sweep: the rest of the band is unchanged
            bool same = true;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int c = col(k);
                if (c < w) same = same && po[k] == F[k];
            }
            if (__all(same)) return;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int c = col(k);
            if (c < w) Sout[(long)r * w + c] = (int8_t)F[k];
        }
        if (r == last) {
            if (has_nr && bnd_out) {
                bool diff = false;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int c = col(k);
                    if (c < w) { bnd_out[c] = (int8_t)nxt[k]; diff = diff || nxt[k] != nxt0[k]; }
                }
                const bool any = __any(diff);
                if (lane == 0) *flag_out = any ? 1 : 0;
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) { cur[k] = nxt[k]; cm[k] = nm[k]; po[k] = pn[k]; }
    }
}

template <int K, int DIR>
__device__ __forceinline__ void d_refine_p1(const int8_t* __restrict__ Sin, int8_t* __restrict__ Sout,
                                                 const unsigned long long* __restrict__ MK, int w, int h, int rb,
                                                 int8_t* __restrict__ bnd, int* __restrict__ flag) {
    const int b = blockIdx.x, s = blockIdx.y;
    const long N = (long)w * h;
    const int r0 = b * rb, r1 = min(h, r0 + rb);
    refine_band<K, DIR>(Sin + s * N, Sout + s * N, MK + s * N, w, h, r0, r1, nullptr,
                        bnd + ((long)s * R360_REFINE_BANDS + b) * w, flag + s * R360_REFINE_BANDS + b, false);
}
template <int K, int DIR>
__global__ void __launch_bounds__(64) k_refine_p1(const PlaneBatch B, int w, int h, int rb) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_p1<K, DIR>(DIR > 0 ? D.state : D.state2, DIR > 0 ? D.state2 : D.state, D.mask, w, h, rb, D.rbnd, D.rflag);
}


template <int K, int DIR>
__device__ __forceinline__ void d_refine_p2(const int8_t* __restrict__ Sin, int8_t* __restrict__ Sout,
                                                 const unsigned long long* __restrict__ MK, int w, int h, int rb,
                                                 int nb, int8_t* __restrict__ bnd, int* __restrict__ flag) {
    const int s = blockIdx.x;
    const long N = (long)w * h;
    int8_t* B = bnd + (long)s * R360_REFINE_BANDS * w;
    int* Fl = flag + s * R360_REFINE_BANDS;
    for (int i = 1; i < nb; ++i) {
        const int b = DIR > 0 ? i : nb - 1 - i;
        const int prev = b - DIR;
        // flags and boundary rows were written by phase 1 or by this wave's previous band
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (!__builtin_amdgcn_readfirstlane(Fl[prev])) continue;
        const int r0 = b * rb, r1 = min(h, r0 + rb);
        refine_band<K, DIR>(Sin + s * N, Sout + s * N, MK + s * N, w, h, r0, r1, B + (long)prev * w, B + (long)b * w,
                            Fl + b, true);
    }
}
template <int K, int DIR>
__global__ void __launch_bounds__(64) k_refine_p2(const PlaneBatch B, int w, int h, int rb, int nb) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_p2<K, DIR>(DIR > 0 ? D.state : D.state2, DIR > 0 ? D.state2 : D.state, D.mask, w, h, rb, nb, D.rbnd, D.rflag);
}


// ------------------------------------------------------------------ wavefront refine
// The sweeps as anti-diagonal wavefronts.  In the first sweep a pixel's state depends only on the pixel above
// (the down push of the row above, applied first) and the pixel to its left (the row's chain), both on the
// previous anti-diagonal k - 1 (k = row + column); the second sweep mirrors it (the pixel below, the pixel to
// the right; diagonals in decreasing order).  So one thread per row walks its row while the diagonals advance:
// at step k thread r handles column k - r, takes the left/right neighbour from its own previous step and the
// upper/lower neighbour's from thread r -/+ 1 (DPP wave shift inside a wave, LDS between waves, one barrier
// per diagonal).  h + w - 1 steps instead of h dependent row scans.
//
// Per pixel (O = state before the sweep, only O == -2 pixels change, M = closeness mask):
//   sweep 1   D = up push:  r >= 1, c <= w-2, O(r-1, c+1) != -1, a = F(r-1, c) >= 0, M bit a  -> a
//             chain:        D == -2, r <= h-2, c >= 1, b = F(r, c-1) >= 0, M bit b           -> b
//   sweep 2   D = push:     r <= h-2, O(r+1, c-1) != -1 (c >= 1) or O(r, w-1) != -1 (c == 0),
//                           a = F(r+1, c) >= 0, M bit a                                        -> a
//             chain:        D == -2, r >= 1, c <= w-2, b = F(r, c+1) >= 0, M bit b            -> b
// The second sweep has one edge the wavefront cannot order: column 0 of row r+1 also pushes into (r, w-1)
// when the push from below left it at -2 (the flat-index wrap of PCL's "left" neighbour), but (r+1, 0) is
// reached only after row r has started.  The wavefront runs as if that push never happens and checks it when
// thread r reaches column 0 (where a = F(r+1, 0)); if it would have fired for any row, the sensor's fallback
// flag is set and k_refine_fb redoes the second sweep with the single-wave kernel.  Without such a row every
// pixel satisfies the sequential recurrences, so the states are the sequential sweep's bit for bit.
//
// Inputs in skewed layout (k_refine_skew): slot k * h + r of diagonal k holds pixel (r, k - r), so a step's
// loads are coalesced; code = state | static push conditions << 8.
constexpr int RW_PF = 8;   // diagonals prefetched ahead

__device__ __forceinline__ void d_refine_skew(const int8_t* __restrict__ S, const unsigned long long* __restrict__ MK, int w, int h,
                              uint16_t* __restrict__ code, unsigned long long* __restrict__ msk, int* __restrict__ fb) {
    // one thread per skewed slot (coalesced stores; the raster reads walk down-left diagonals, which reuse
    // each cache line for the next diagonals); slots outside the image are never used
    const long N = (long)w * h, SK = (long)(h + w - 1) * h, total = 8 * SK;
    if (blockIdx.x == 0 && threadIdx.x < 24) fb[threadIdx.x] = 0;
    for (long d = blockIdx.x * (long)blockDim.x + threadIdx.x; d < total; d += (long)gridDim.x * blockDim.x) {
        const int s = (int)(d / SK);
        const long q = d - (long)s * SK;
        const int k = (int)(q / h), r = (int)(q - (long)k * h);
        const int c = k - r;
        if (c < 0 || c >= w) continue;
        const int j = r * w + c;
        const long i = (long)s * N + j;
        const int8_t* O = S + (long)s * N;
        const bool c1 = r >= 1 && c <= w - 2 && O[(r - 1) * w + c + 1] != -1;
        const bool c2 = r <= h - 2 && (c >= 1 ? O[(r + 1) * w + c - 1] != -1 : O[r * w + w - 1] != -1);
        code[d] = (uint16_t)((uint8_t)O[j] | (c1 ? 0x100 : 0) | (c2 ? 0x200 : 0));
        msk[d] = MK[i];
    }
}
__global__ void k_refine_skew(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_skew(D.state, D.mask, w, h, D.rcode, D.rmsk, D.rflag);
}


__device__ __forceinline__ bool mbit(unsigned long long m, int v) { return (v >= 0) & (((m >> (v & 63)) & 1ull) != 0); }

// DIR = +1: first sweep, F written to f1 (skewed).  DIR = -1: second sweep over f1, F written to S (raster).
// blockDim.x = 64 * ceil(h / 64), grid = 8 sensors.
//
// Second sweep, wrap pushes: the wavefront runs with an assumed wrap value per row (none at first); when thread
// r reaches column 0 it records the value the wrap push into (r, w-1) really takes given the states now known
// (wdet[r]).  Rows are swept bottom-up, so the last row (largest r) whose record differs from its assumption is
// the earliest point where the sweep went wrong: everything on diagonals above r + w - 1 is exact.  Every
// differing row takes its record as the new assumption (that row's record is exact, the others are the best
// guess) and the wavefront is re-run from diagonal r + w - 1 downwards, comparing every state with the
// previous pass's; once it is below the lowest changed assumption, a whole diagonal that comes out unchanged
// means every later diagonal would too, and the pass stops.  Repeat until no row's record differs from its
// assumption: then every pixel satisfies the sequential recurrences and the states are the sequential sweep's
// (each pass makes the last differing row exact, so this ends).  After RW_MAX_REDO re-runs the sensor is handed
// to k_refine_fb (fb[s] = first differing row + 1).
constexpr int RW_MAX_REDO = 64;

template <int DIR>
__device__ __forceinline__ void d_refine_wave(const uint16_t* __restrict__ code_all,
                                                      const unsigned long long* __restrict__ msk_all,
                                                      int8_t* __restrict__ f1_all, int8_t* __restrict__ f2_all,
                                                      int* __restrict__ fb, int w, int h) {
    __shared__ int xch[2][16];
    __shared__ int8_t wasm[1024], wdet[1024];   // DIR < 0: assumed / detected wrap value per row (-2: none)
    __shared__ int s_red, s_min;
    __shared__ int chg[2][16];   // re-runs: whether a wave changed any state at a step
    const int s = blockIdx.x;
    const int r = threadIdx.x, lane = r & 63, wv = r >> 6, nw = blockDim.x >> 6;
    const long SK = (long)(h + w - 1) * h;
    const uint16_t* code = code_all + s * SK;
    const unsigned long long* msk = msk_all + s * SK;
    int8_t* f1 = f1_all + s * SK;
    int8_t* f2 = f2_all + s * SK;                 // DIR < 0: the second sweep's states, skewed (coalesced stores)
    const int KS = h + w - 1;
    const int rr = r < h ? r : h - 1;             // loads of rows >= h are clamped (never used)
    auto kof = [&](int t) { return DIR > 0 ? t : KS - 1 - t; };
    auto tc = [&](int t) { return t < KS ? t : KS - 1; };
    // inputs of RW_PF diagonals per chunk: the next chunk's loads are issued when a chunk starts and consumed
    // RW_PF steps later (kept as loaded; combining them at load time would wait for them there): code = state |
    // push conditions, the mask, for DIR < 0 the first sweep's state and, in a re-run, the previous pass's
    struct In { unsigned short code; unsigned char f1, old; unsigned long long m; };
    auto ld = [&](int t, bool redo, In& x) {
        const int k = kof(tc(t));
        const long q = (long)k * h + rr;
        x.code = code[q];
        x.m = msk[q];
        if (DIR < 0) x.f1 = (unsigned char)f1[q];
        if (DIR < 0 && redo) x.old = (unsigned char)f2[q];
    };
    if (DIR < 0) {
        for (int q = threadIdx.x; q < 1024; q += blockDim.x) { wasm[q] = -2; wdet[q] = -2; }
    }
    bool upw_free = false;     // DIR < 0: (r, w-1) was left at -2 by the push from below
    unsigned long long mw = 0; //   and its mask
    int t_start = 0, t_guard = 0;   // re-runs may stop only at steps after t_guard
    // one pass of the wavefront from step t_start; REDO: a re-run (compares with the previous pass, may stop)
    auto run = [&](auto redo_tag) {
        constexpr bool REDO = decltype(redo_tag)::value;
        int prev = -1;         // this row's state at the previous step
        if (REDO) {            // resume from the previous pass's states on the diagonal before t_start
            const int k = kof(t_start - 1), c = k - r;
            if (r < h && c >= 0 && c < w) prev = f2[(long)k * h + r];
        }
        const int my_wasm = DIR < 0 && r < h ? (int)wasm[r] : -2;   // this row's assumed wrap push
        int my_wdet = DIR < 0 && r < h ? (int)wdet[r] : -2;         // and the one it detects
        In cur[RW_PF];
#pragma unroll
        for (int d = 0; d < RW_PF; ++d) ld(t_start + d, REDO, cur[d]);
        __syncthreads();
        if (lane == (DIR > 0 ? 63 : 0)) xch[(t_start + 1) & 1][wv] = prev;
        if (threadIdx.x < 16) { chg[0][threadIdx.x] = 1; chg[1][threadIdx.x] = 1; }
        __syncthreads();
        bool stop = false;
        for (int t0 = t_start; t0 < KS && !stop; t0 += RW_PF) {
            In nxt[RW_PF];
#pragma unroll
            for (int d = 0; d < RW_PF; ++d) ld(t0 + RW_PF + d, REDO, nxt[d]);
#pragma unroll
            for (int d = 0; d < RW_PF; ++d) {
                const int t = t0 + d;
                if (t >= KS) break;
                if (REDO && t - 1 > t_guard) {
                    // the previous diagonal came out equal to the previous pass's: so would every later one
                    int any = 0;
                    for (int q = 0; q < nw; ++q) any |= chg[(t + 1) & 1][q];
                    if (!any) { stop = true; break; }
                }
                const int k = kof(t);
                const int c = k - r;
                const bool act = (r < h) & (c >= 0) & (c < w);
                const int o = DIR > 0 ? (int)(int8_t)(cur[d].code & 0xff) : (int)(int8_t)cur[d].f1;
                const bool cond = (cur[d].code >> (DIR > 0 ? 8 : 9)) & 1;
                const unsigned long long m = cur[d].m;
                // the neighbour row's state at the previous step: thread r - 1 (DIR > 0) / r + 1 (DIR < 0)
                const int pw = DIR > 0 ? (wv > 0 ? xch[(t + 1) & 1][wv - 1] : -1)
                                       : (wv + 1 < nw ? xch[(t + 1) & 1][wv + 1] : -1);
                int a = DIR > 0 ? __builtin_amdgcn_update_dpp(pw, prev, 0x138, 0xf, 0xf, false)    // wave_shr:1
                                : __builtin_amdgcn_update_dpp(pw, prev, 0x130, 0xf, 0xf, false);   // wave_shl:1
                if (DIR < 0 && r == h - 1) a = -1;
                // branch-free: only o == -2 pixels change
                int D = (cond & mbit(m, a)) ? a : -2;
                if (DIR < 0) {
                    const bool first = (c == w - 1) & (o == -2);   // (r, w-1): the wrap push's target
                    const bool uf = (D == -2) & (r <= h - 2);
                    upw_free = first ? uf : upw_free;
                    mw = first ? m : mw;
                    D = (first & uf & act) ? my_wasm : D;          // the assumed wrap push (-2: none)
                }
                const bool ch = DIR > 0 ? ((r <= h - 2) & (c >= 1)) : ((r >= 1) & (c <= w - 2));
                D = ((D == -2) & ch & mbit(m, prev)) ? prev : D;
                const int F = o == -2 ? D : o;
                if (DIR < 0) {
                    const bool last = act & (c == 0) & (r <= h - 2);  // a = F(r+1, 0): the wrap push's source
                    my_wdet = last ? ((upw_free & mbit(mw, a)) ? a : -2) : my_wdet;
                }
                if (act) {
                    if (DIR > 0) f1[(long)k * h + r] = (int8_t)F;
                    else f2[(long)k * h + r] = (int8_t)F;
                }
                const bool changed = REDO & act & (F != (int)(int8_t)cur[d].old);
                prev = act ? F : prev;
                if (lane == (DIR > 0 ? 63 : 0)) xch[t & 1][wv] = prev;
                if (REDO) {
                    const bool wchg = __any(changed);
                    if (lane == 0) chg[t & 1][wv] = wchg;
                }
                // LDS-only barrier: the exchange slots are the only shared state (no wait for the prefetches)
                __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
                __builtin_amdgcn_s_barrier();
            }
#pragma unroll
            for (int d = 0; d < RW_PF; ++d) cur[d] = nxt[d];
        }
        if (DIR < 0 && r < h) wdet[r] = (int8_t)my_wdet;
        __syncthreads();
    };
    for (int pass = 0;; ++pass) {
        if (pass == 0) run(std::integral_constant<bool, false>{});
        else run(std::integral_constant<bool, true>{});
        if (DIR > 0) break;
        // the last row (first in sweep order) whose detected wrap push differs from the assumed one
        if (threadIdx.x == 0) { s_red = -1; s_min = h; }
        __syncthreads();
        const bool mis = r <= h - 2 && wdet[r] != wasm[r];
        if (mis) { atomicMax(&s_red, r); atomicMin(&s_min, r); }
        __syncthreads();
        const int rs = s_red;
        if (rs < 0) {
            if (threadIdx.x == 0 && pass > 0) fb[8 + s] = pass;   // re-runs this sensor needed (inspection)
            break;
        }
        if (pass >= RW_MAX_REDO) {   // give up: the single-wave kernel finishes the sweep from that row
            if (threadIdx.x == 0) { fb[s] = rs + 1; fb[8 + s] = pass; }
            break;
        }
        if (mis) wasm[r] = wdet[r];
        t_start = KS - 1 - (rs + w - 1);      // the step of diagonal rs + w - 1
        t_guard = KS - 1 - (s_min + w - 1);   // the step of the lowest changed assumption
        __syncthreads();
    }
}
template <int DIR>
__global__ void __launch_bounds__(1024) k_refine_wave(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_wave<DIR>(D.rcode, D.rmsk, D.rf1, DIR > 0 ? D.state : D.rf2, D.rflag, w, h);
}


// ------------------------------------------------------------------ pipelined wavefront
// The same wavefront with no workgroup barrier per diagonal: wave g owns the 64-row band r0 = 64 g .. r0 + 63
// and walks its own diagonals r0 .. r0 + 63 + w - 1 at its own pace (inside the band the neighbour row's state
// still comes by DPP from the neighbouring lane).  The one row that crosses a band edge is handed over in LDS:
// the producing band (DIR > 0 the band above, DIR < 0 the band below) writes its edge row's states, in sweep
// order u, to bnd[band][u] and publishes how many are valid (prog); the consuming band waits, every RP_BC steps,
// until the values of its next RP_BC steps are there.  A band's step then costs its own dependency chain only,
// not an LDS round trip plus a barrier over all bands, and the bands run as a pipeline one band's lead apart.
//
// Re-runs (DIR < 0, wrap pushes, as k_refine_wave): a band may stop early once its previous diagonal came out
// unchanged, the lowest changed wrap assumption is behind it, and the band it consumes from has finished this
// pass with every value it changed already consumed (lchg).  Values a band does not recompute in a re-run stay
// in bnd from the previous pass, so prog starts at the band's first recomputed u.
constexpr int RP_BC = 8;           // steps per chunk (hand-off check); loads run two chunks ahead
constexpr int RP_MAXB = 8;         // bands (waves): h <= 512
constexpr int RP_MAXW = 640;       // widest sensor
constexpr int RP_PAD = 8;          // bnd rows are padded on both sides: a chunk stores its RP_BC edge values whole
constexpr unsigned RP_SPIN = 1u << 22;

struct PipeShared {
    int8_t bnd[RP_MAXB][RP_MAXW + 2 * RP_PAD];   // each band's edge row (DIR > 0 its last, DIR < 0 its first), by u
    int prog[RP_MAXB];              // bnd[g][u] valid this pass for u < prog[g] (w: the band is done)
    int lchg[RP_MAXB];              // re-runs: the largest u of bnd[g] changed this pass (-1: none)
    int8_t wasm[64 * RP_MAXB], wdet[64 * RP_MAXB];   // DIR < 0: assumed / detected wrap value per row
    int s_red, s_min, s_fail;
};

// NARROW: every label and closeness bit of the sensor is below 30, so a mask test is one 32-bit bit-field
// extract whose offset wraps -1 / -2 onto the always-clear bits 31 / 30 (no sign test), and the step's
// dependency chain is DPP -> extract -> compare -> select.  The skewed arrays are read and written through
// buffer resources: a step's diagonal offset is wave-uniform (scalar), the lane's row the vector offset.
template <int DIR, bool NARROW>
__device__ __forceinline__ void refine_pipe_body(const uint16_t* __restrict__ code_all,
                                                 const unsigned long long* __restrict__ msk_all,
                                                 int8_t* __restrict__ f1_all, int8_t* __restrict__ f2_all,
                                                 int* __restrict__ fb, int w, int h, PipeShared& P) {
    auto& bnd = P.bnd;
    auto& prog = P.prog;
    auto& lchg = P.lchg;
    auto& wasm = P.wasm;
    auto& wdet = P.wdet;
    const int s = blockIdx.x;
    const int r = threadIdx.x, lane = r & 63, nw = blockDim.x >> 6;
    const int g = __builtin_amdgcn_readfirstlane(r >> 6);
    const int SK = (h + w - 1) * h;
    const auto rcode = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(code_all) + (long)s * SK, 0, SK * 2, 0x00020000);
    const auto rmsk = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned long long*>(msk_all) + (long)s * SK, 0, SK * 8,
                                                        0x00020000);
    const auto rf1 = __builtin_amdgcn_make_buffer_rsrc(f1_all + (long)s * SK, 0, SK, 0x00020000);
    const auto rf2 = __builtin_amdgcn_make_buffer_rsrc(f2_all + (long)s * SK, 0, SK, 0x00020000);
    const int KS = h + w - 1;
    const int rr = r < h ? r : h - 1;             // loads of rows >= h are clamped (never used)
    const int r0 = g * 64, nr = min(64, h - r0);
    // this band's diagonals r0 .. r0 + nr + w - 2 as steps [tlo, thi]
    const int tlo = DIR > 0 ? r0 : KS - 1 - (r0 + nr + w - 2), thi = DIR > 0 ? r0 + nr + w - 2 : KS - 1 - r0;
    const int up = DIR > 0 ? g - 1 : g + 1;       // the band whose edge row this one consumes
    const bool has_up = up >= 0 && up < nw;
    const bool has_out = DIR > 0 ? g < nw - 1 : g > 0;   // a band consumes this one's edge row
    const int plane = DIR > 0 ? 63 : 0;           // the lane whose row is this band's edge row
    // u of the consuming lane (DIR > 0 lane 0, DIR < 0 lane 63) and of the edge lane at step t
    auto ucons = [&](int t) { return DIR > 0 ? t - r0 : t + r0 + 64 - h; };
    auto uprod = [&](int t) { return DIR > 0 ? t - r0 - 63 : t + r0 + 1 - h; };
    auto kof = [&](int t) { return DIR > 0 ? t : KS - 1 - t; };
    struct In { unsigned code, f1, old; unsigned long long m; };
    // DIR < 0 keeps fewer scalar registers live with plain 32-bit-offset loads (its wrap bookkeeping needs them)
    constexpr bool BUF = DIR > 0;
    const uint16_t* cs = code_all + (long)s * SK;
    const unsigned long long* ms = msk_all + (long)s * SK;
    const int8_t* f1s = f1_all + (long)s * SK;
    int8_t* f2s = f2_all + (long)s * SK;
    auto ld = [&](int t, bool redo, In& x) {
        const int so = kof(t <= thi ? t : thi) * h;   // the diagonal's first slot
        if (!BUF) {
            const unsigned q = (unsigned)(so + rr);
            x.code = cs[q];
            x.m = NARROW ? (unsigned long long)reinterpret_cast<const unsigned*>(ms)[2 * q] : ms[q];
            x.f1 = (unsigned char)f1s[q];
            if (redo) x.old = (unsigned char)f2s[q];
            return;
        }
        x.code = __builtin_amdgcn_raw_buffer_load_b16(rcode, rr * 2, so * 2, 0);
        if (NARROW) {
            x.m = __builtin_amdgcn_raw_buffer_load_b32(rmsk, rr * 8, so * 8, 0);
        } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rmsk, rr * 8, so * 8, 0);
            x.m = (unsigned long long)v[0] | ((unsigned long long)v[1] << 32);
        }
        if (DIR < 0) x.f1 = __builtin_amdgcn_raw_buffer_load_b8(rf1, rr, so, 0);
        if (DIR < 0 && redo) x.old = __builtin_amdgcn_raw_buffer_load_b8(rf2, rr, so, 0);
    };
    if (DIR < 0) {
        for (int q = threadIdx.x; q < 64 * RP_MAXB; q += blockDim.x) { wasm[q] = -2; wdet[q] = -2; }
    }
    if (threadIdx.x == 0) P.s_fail = 0;
    bool upw_free = false;     // DIR < 0: (r, w-1) was left at -2 by the push from below
    unsigned long long mw = 0; //   and its mask
    int t_start = 0, t_guard = 0;   // re-runs may stop only at steps after t_guard
    auto run = [&](auto redo_tag) {
        constexpr bool REDO = decltype(redo_tag)::value;
        const int tb = max(t_start, tlo);
        int prev = -1;         // this row's state at the previous step
        if (REDO) {            // resume from the previous pass's states on the diagonal before tb
            const int k = kof(tb - 1), c = k - r;
            if (r < h && c >= 0 && c < w) prev = f2_all[(long)s * SK + (long)k * h + r];
        }
        const int my_wasm = DIR < 0 && r < h ? (int)wasm[r] : -2;   // this row's assumed wrap push
        int my_wdet = DIR < 0 && r < h ? (int)wdet[r] : -2;         // and the one it detects
        // three register sets of RP_BC diagonals used in rotation: a chunk's loads are issued two chunks ahead and
        // no loop-carried copy of an in-flight load forces a wait
        In A[RP_BC], B[RP_BC], C[RP_BC];
#pragma unroll
        for (int d = 0; d < RP_BC; ++d) { ld(tb + d, REDO, A[d]); ld(tb + RP_BC + d, REDO, B[d]); }
        if (lane == 0) { lchg[g] = -1; prog[g] = min(max(uprod(tb), 0), w); }
        __syncthreads();
        bool pchg = true;
        int lchg_r = -1;       // edge lane: the largest u it changed this pass
        unsigned spins = 0;
        // one chunk of RP_BC steps from t0 over inputs cur, issuing the loads of chunk t0 + 2 RP_BC into nn; FULL:
        // every step is inside the band's range.  True when the pass ends in it.
        auto chunk = [&](int t0, In (&cur)[RP_BC], In (&nn)[RP_BC], auto full_tag) -> bool {
            constexpr bool FULL = decltype(full_tag)::value;
#pragma unroll
            for (int d = 0; d < RP_BC; ++d) ld(t0 + 2 * RP_BC + d, REDO, nn[d]);
            // the upstream band's edge values of these steps
            int bv[RP_BC];
            if (has_up) {
                const int need = min(ucons(t0 + RP_BC - 1), w - 1);
                if (need >= 0) {
                    while (__hip_atomic_load(&prog[up], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= need) {
                        if (++spins > RP_SPIN) { P.s_fail = 1; break; }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                asm volatile("" ::: "memory");
#pragma unroll
                for (int e = 0; e < RP_BC; ++e) {
                    const int u = ucons(t0 + e);
                    bv[e] = bnd[up][RP_PAD + (u < 0 ? 0 : (u < w ? u : w - 1))];
                }
            } else {
#pragma unroll
                for (int e = 0; e < RP_BC; ++e) bv[e] = -1;
            }
            int Fv[RP_BC];     // the edge lane's states of this chunk (pass 0: stored to bnd at its end)
            bool ended = false;
#pragma unroll
            for (int d = 0; d < RP_BC; ++d) {
                const int t = t0 + d;
                if (!FULL && t > thi) {
                    ended = true;
#pragma unroll
                    for (int e = d; e < RP_BC; ++e) Fv[e] = -1;   // lands in the row's back padding
                    break;
                }
                if (REDO && t > tb && !pchg && t - 1 > t_guard) {
                    // the previous diagonal came out as in the previous pass: so does every later one once the
                    // upstream band is done and its changed values are consumed
                    if (!has_up || (__hip_atomic_load(&prog[up], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= w &&
                                    __hip_atomic_load(&lchg[up], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < ucons(t)))
                        return true;
                }
                const int k = kof(t);
                const int c = k - r;
                const bool act = (r < h) & ((unsigned)c < (unsigned)w);
                // this step's inputs become visible here, not earlier: otherwise the scheduler hoists their uses
                // to the chunk start and waits there for loads issued for two chunks later
                unsigned xcode = cur[d].code, xf1 = cur[d].f1, xold = cur[d].old;
                unsigned long long xm = cur[d].m;
                asm volatile("" : "+v"(xcode), "+v"(xm));
                if (DIR < 0) asm volatile("" : "+v"(xf1));
                if (REDO) asm volatile("" : "+v"(xold));
                const int o = DIR > 0 ? (int)(int8_t)(xcode & 0xff) : (int)(int8_t)xf1;
                const bool cond = (xcode >> (DIR > 0 ? 8 : 9)) & 1;
                const bool ch = DIR > 0 ? ((r <= h - 2) & (c >= 1)) : ((r >= 1) & (c <= w - 2));
                const int pw = bv[d];
                int F;
                if (NARROW) {
                    // off the chain: the candidate masks of the push (from the neighbour row) and of the chain
                    // (from the left / right), and the value when neither applies
                    const unsigned mlo = (unsigned)xm;
                    const bool fixed = o != -2;
                    const unsigned mp = (cond & !fixed) ? mlo : 0u, mc = (ch & !fixed) ? mlo : 0u;
                    int base = o;
                    bool first = false;
                    if (DIR < 0) {
                        first = (c == w - 1) & !fixed;                          // (r, w-1): the wrap push's target
                        base = (first & (r <= h - 2)) ? my_wasm : base;        // the assumed wrap push
                    }
                    const int a = DIR > 0 ? __builtin_amdgcn_update_dpp(pw, prev, 0x138, 0xf, 0xf, false)
                                          : __builtin_amdgcn_update_dpp(pw, prev, 0x130, 0xf, 0xf, false);
                    const int alt = __builtin_amdgcn_ubfe(mc, (unsigned)prev, 1) ? prev : base;
                    const bool pok = __builtin_amdgcn_ubfe(mp, (unsigned)a, 1) != 0;
                    F = pok ? a : alt;
                    if (DIR < 0) {
                        // the wrap bookkeeping touches one lane per step at most: branches, not selects per step
                        if (first) {
                            upw_free = !pok & (r <= h - 2);
                            mw = mlo;
                        }
                        if (act & (c == 0) & (r <= h - 2))   // a = F(r+1, 0): the wrap push's source
                            my_wdet = (upw_free & (__builtin_amdgcn_ubfe((unsigned)mw, (unsigned)a, 1) != 0)) ? a : -2;
                    }
                } else {
                    const unsigned long long m = xm;
                    int a = DIR > 0 ? __builtin_amdgcn_update_dpp(pw, prev, 0x138, 0xf, 0xf, false)    // wave_shr:1
                                    : __builtin_amdgcn_update_dpp(pw, prev, 0x130, 0xf, 0xf, false);   // wave_shl:1
                    if (DIR < 0 && r == h - 1) a = -1;
                    int D = (cond & mbit(m, a)) ? a : -2;
                    if (DIR < 0) {
                        const bool first = (c == w - 1) & (o == -2);   // (r, w-1): the wrap push's target
                        const bool uf = (D == -2) & (r <= h - 2);
                        upw_free = first ? uf : upw_free;
                        mw = first ? m : mw;
                        D = (first & uf & act) ? my_wasm : D;          // the assumed wrap push (-2: none)
                    }
                    D = ((D == -2) & ch & mbit(m, prev)) ? prev : D;
                    F = o == -2 ? D : o;
                    if (DIR < 0) {
                        const bool last = act & (c == 0) & (r <= h - 2);  // a = F(r+1, 0): the wrap push's source
                        my_wdet = last ? ((upw_free & mbit(mw, a)) ? a : -2) : my_wdet;
                    }
                }
                if (act) {
                    if (BUF) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)F, rf1, r, k * h, 0);
                    else f2s[(unsigned)(k * h + r)] = (int8_t)F;
                }
                Fv[d] = F;
                prev = act ? F : prev;
                if (REDO || DIR < 0) {   // DIR < 0: per-step edge stores keep fewer registers live
                    const bool changed = REDO & act & (F != (int)(int8_t)xold);
                    if (lane == plane && act) {
                        const int u = uprod(t);
                        bnd[g][RP_PAD + u] = (int8_t)F;
                        if (changed) lchg_r = u;
                    }
                    if (REDO) pchg = __any(changed);
                }
            }
            if (lane == plane) {   // publish this chunk's edge values
                if (!REDO && DIR > 0 && has_out) {
                    const int u0 = uprod(t0);
                    if (u0 + RP_BC - 1 >= 0) {
#pragma unroll
                        for (int d = 0; d < RP_BC; ++d) bnd[g][RP_PAD + u0 + d] = (int8_t)Fv[d];
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the values before their count
                lchg[g] = lchg_r;
                __hip_atomic_store(&prog[g], min(max(uprod(min(t0 + RP_BC - 1, thi)) + 1, 0), w), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            return ended;
        };
        using T = std::integral_constant<bool, true>;
        using Fl = std::integral_constant<bool, false>;
        int t0 = tb;
        bool ended = false;
        for (; DIR > 0 && t0 + 3 * RP_BC - 1 <= thi; t0 += 3 * RP_BC) {   // whole rotations inside the range
            if (chunk(t0, A, C, T{}) || chunk(t0 + RP_BC, B, A, T{}) || chunk(t0 + 2 * RP_BC, C, B, T{})) {
                ended = true;
                break;
            }
        }
        if (DIR > 0) {
            if (!ended && t0 <= thi && !chunk(t0, A, C, Fl{}) && t0 + RP_BC <= thi && !chunk(t0 + RP_BC, B, A, Fl{}) &&
                t0 + 2 * RP_BC <= thi)
                chunk(t0 + 2 * RP_BC, C, B, Fl{});
        } else {   // DIR < 0: every chunk checks the range end (one copy of the step code per rotation slot)
            for (; t0 <= thi; t0 += 3 * RP_BC) {
                if (chunk(t0, A, C, Fl{}) || chunk(t0 + RP_BC, B, A, Fl{}) || chunk(t0 + 2 * RP_BC, C, B, Fl{})) break;
            }
        }
        if (lane == plane) {   // done: every value of bnd[g] is this pass's
            __builtin_amdgcn_s_waitcnt(0xc07f);
            lchg[g] = lchg_r;
            __hip_atomic_store(&prog[g], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (DIR < 0 && r < h) wdet[r] = (int8_t)my_wdet;
        __syncthreads();
    };
    for (int pass = 0;; ++pass) {
        if (pass == 0) run(std::integral_constant<bool, false>{});
        else run(std::integral_constant<bool, true>{});
        if (P.s_fail) {   // a hand-off wait gave up: k_refine_fb redoes this sensor (both sweeps after a first-sweep failure)
            if (threadIdx.x == 0) {
                fb[s] = h - 1;
                if (DIR > 0) fb[16 + s] = 1;
            }
            break;
        }
        if (DIR > 0) break;
        if (threadIdx.x == 0) { P.s_red = -1; P.s_min = h; }
        __syncthreads();
        const bool mis = r <= h - 2 && wdet[r] != wasm[r];
        if (mis) { atomicMax(&P.s_red, r); atomicMin(&P.s_min, r); }
        __syncthreads();
        const int rs = __builtin_amdgcn_readfirstlane(P.s_red);
        if (rs < 0) {
            if (threadIdx.x == 0 && pass > 0) fb[8 + s] = pass;
            break;
        }
        if (pass >= RW_MAX_REDO) {
            if (threadIdx.x == 0) { fb[s] = rs + 1; fb[8 + s] = pass; }
            break;
        }
        if (mis) wasm[r] = wdet[r];
        t_start = KS - 1 - (rs + w - 1);
        t_guard = KS - 1 - (__builtin_amdgcn_readfirstlane(P.s_min) + w - 1);
        __syncthreads();
    }
}

// NW: the most waves (bands) it is launched with; 4 (h <= 256) leaves each wave up to 512 VGPRs
template <int DIR, int NW>
__device__ __forceinline__ void d_refine_pipe(const uint16_t* __restrict__ code_all,
                                                             const unsigned long long* __restrict__ msk_all,
                                                             int8_t* __restrict__ f1_all, int8_t* __restrict__ f2_all,
                                                             const int* __restrict__ nmodels, int* __restrict__ fb,
                                                             int w, int h, int narrow_max) {
    __shared__ PipeShared P;
    if (nmodels[blockIdx.x] <= narrow_max) refine_pipe_body<DIR, true>(code_all, msk_all, f1_all, f2_all, fb, w, h, P);
    else refine_pipe_body<DIR, false>(code_all, msk_all, f1_all, f2_all, fb, w, h, P);
}
template <int DIR, int NW>
__global__ void __launch_bounds__(64 * NW) k_refine_pipe(const PlaneBatch B, int w, int h, int narrow_max) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_pipe<DIR, NW>(D.rcode, D.rmsk, D.rf1, D.rf2, D.nmodels, D.rflag, w, h, narrow_max);
}


// the second sweep's states back to raster order (sensors handed to k_refine_fb are written by it)
__device__ __forceinline__ void d_refine_unskew(const int8_t* __restrict__ f2_all, int8_t* __restrict__ S_all,
                                const int* __restrict__ fb, int w, int h) {
    const long N = (long)w * h, SK = (long)(h + w - 1) * h, total = 8 * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        if (fb[s]) continue;
        const int j = (int)(i - (long)s * N), r = j / w, c = j - r * w;
        S_all[i] = f2_all[s * SK + (long)(r + c) * h + r];
    }
}
__global__ void k_refine_unskew(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_unskew(D.rf2, D.state, D.rflag, w, h);
}


// The exact second sweep for a sensor whose wavefront saw the wrap push fire, first at target row r0 = fb - 1:
// rows below r0 are exact (nothing they depend on fired), so rows 0..r0 get the first sweep's states back and
// the single-wave sweep resumes at source row r0 + 1 (re-chaining a swept row leaves it unchanged).
template <int K>
__device__ __forceinline__ void d_refine_fb(const int8_t* __restrict__ f1_all, const int8_t* __restrict__ f2_all,
                                                 int8_t* __restrict__ S_all,
                                                 const unsigned long long* __restrict__ MK, const int* __restrict__ fb,
                                                 int w, int h) {
    const int s = blockIdx.x;
    if (fb[16 + s]) {   // the pipelined first sweep gave up: both sweeps from the original states
        refine_sweeps<K>(S_all, MK, w, h, s, 3);
        return;
    }
    const int r0 = fb[s] - 1;
    if (r0 < 0) return;
    const long N = (long)w * h, SK = (long)(h + w - 1) * h;
    // rows 0..r0 from the first sweep, rows below from the wavefront's (exact) second sweep
    for (long j = threadIdx.x; j < N; j += 64) {
        const int r = (int)(j / w), c = (int)(j - (long)r * w);
        S_all[s * N + j] = (r <= r0 ? f1_all : f2_all)[s * SK + (long)(r + c) * h + r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    refine_sweeps<K>(S_all, MK, w, h, s, 2, r0 + 1);
}
template <int K>
__global__ void __launch_bounds__(64) k_refine_fb(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_fb<K>(D.rf1, D.rf2, D.state, D.mask, D.rflag, w, h);
}


__device__ __forceinline__ void d_refine_final(const int8_t* __restrict__ state, const int* __restrict__ lab, int N,
                               const PlaneModel* __restrict__ models, int* __restrict__ labf) {
    const long total = 8L * N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N);
        const int st = state[i];
        labf[i] = st >= 0 ? models[s * R360_MAX_MODELS + st].label : (st == -2 ? lab[i] : -1);
    }
}
__global__ void k_refine_final(const PlaneBatch B, int N) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_refine_final(D.state, D.lab, N, D.models, D.labf);
}


// findLabeledRegionBoundary (Moore-neighbour trace), all regions of a sensor in one workgroup.
// k_nbmask first stores, per pixel, the 8-bit mask of the neighbours carrying the same refined label
// (bit d = direction d of {W, NW, N, NE, E, SE, S, SW}; out-of-image neighbours are 0).  A trace only
// ever stands on member pixels of its region, so that mask is exactly the region-membership
// neighbourhood of the reference's trace, and one step is one LDS byte read plus a rotate /
// find-first-set.  k_trace loads the masks of its sensor into LDS, lane m of wave 0 walks region m
// (all regions of the sensor in parallel), appending the visited pixel indices to 32-entry chunks of
// an LDS list; then the whole workgroup writes the contour points to the pool in trace order.
// Threads 0 .. 20 * 8 * R360_MAX_MODELS - 1 also fold the region accumulators' copies of k_gm<true> into the region
// records, one word each (exact integer sums, min / max), for k_alloc and the host.
__device__ __forceinline__ void d_nbmask(const int* __restrict__ labf, int w, int h, uint8_t* __restrict__ nb,
                         const RegionPart* __restrict__ gpart, const int* __restrict__ nmodels,
                         PlaneOut* __restrict__ out) {
    const int N = w * h;
    const long total = 8L * N;
    {   // thread (q, w): word w of region q summed over the copies
        const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
        const int q = (int)(t / 20), w = (int)(t % 20);
        if (q < 8 * R360_MAX_MODELS && q % R360_MAX_MODELS < nmodels[q / R360_MAX_MODELS]) {
            const RegionPart* G = gpart + q;
            PlaneOut& O = out[q];
            constexpr int C = GM_COPIES, S = 8 * R360_MAX_MODELS;
            if (w < 6) {
                r360p::i128 v = 0;
#pragma unroll
                for (int c = 0; c < C; ++c) v += G[c * S].m.s2[w];
                O.stats.s2[w] = v;
            } else if (w < 14) {
                const int k = w - 6;   // n, s1[0..2], c[0..3]
                long long v = 0;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const r360p::Moments& m = G[c * S].m;
                    v += k == 0 ? m.n : k < 4 ? m.s1[k - 1] : m.c[k - 4];
                }
                if (k == 0) O.stats.n = v;
                else if (k < 4) O.stats.s1[k - 1] = v;
                else O.stats.c[k - 4] = v;
            } else {
                const int k = w - 14;   // bmin[0..2], bmax[0..2]
                float v = k < 3 ? 3.4e38f : -3.4e38f;
#pragma unroll
                for (int c = 0; c < C; ++c) v = k < 3 ? fminf(v, G[c * S].bmin[k]) : fmaxf(v, G[c * S].bmax[k - 3]);
                if (k < 3) O.bmin[k] = v;
                else O.bmax[k - 3] = v;
            }
        }
    }
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int s = (int)(i / N), p = (int)(i - (long)s * N);
        const int* Lb = labf + (long)s * N;
        const int y = p / w, x = p - y * w;
        const int L = Lb[p];
        unsigned m = 0;
        if (L >= 0) {
            const bool l = x > 0, r = x < w - 1, u = y > 0, d = y < h - 1;
            if (l && Lb[p - 1] == L) m |= 1u;
            if (l && u && Lb[p - w - 1] == L) m |= 2u;
            if (u && Lb[p - w] == L) m |= 4u;
            if (r && u && Lb[p - w + 1] == L) m |= 8u;
            if (r && Lb[p + 1] == L) m |= 16u;
            if (r && d && Lb[p + w + 1] == L) m |= 32u;
            if (d && Lb[p + w] == L) m |= 64u;
            if (l && d && Lb[p + w - 1] == L) m |= 128u;
        }
        nb[i] = (uint8_t)m;
    }
}
__global__ void k_nbmask(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_nbmask(D.labf, w, h, reinterpret_cast<uint8_t*>(D.mask), D.gpart, D.nmodels, D.out);
}


constexpr int TR_TPB = 1024;
constexpr int TR_CHUNK = 32;
constexpr int TR_LIST = 12288;                 // contour pixel indices per sensor held in LDS
constexpr int TR_NCH = TR_LIST / TR_CHUNK;

constexpr int TR_NB_MAX = 96 * 1024;          // largest sensor (w*h) whose masks are staged in LDS

// Moore step: next direction = first neighbour in the mask clockwise after dir (the d = 1..8 scan of
// the reference loop); an empty mask keeps nd = dir (the scan's last candidate), as the reference does.
__device__ __forceinline__ int trace_next(unsigned m8, int dir) {
    const unsigned r = ((m8 * 0x101u) >> ((dir + 1) & 7)) & 0xffu;
    // v_ffbl of 0 is -1, which leaves nd = dir for an empty mask with no compare / select
    int tz;
    asm("v_ffbl_b32 %0, %1" : "=v"(tz) : "v"(r));
    return (dir + 1 + tz) & 7;
}

template <bool LDS>
__device__ __forceinline__ void d_trace(const uint8_t* __restrict__ nbg, const float4* __restrict__ cloud,
                                                 int w, int h, const int* __restrict__ nmodels,
                                                 PlaneOut* __restrict__ out, float4* __restrict__ pool, long pool_cap,
                                                 int* __restrict__ err) {
    // static LDS (a workgroup may hold all 160 KiB): masks, index list, chunk tables
    __shared__ __attribute__((aligned(16))) unsigned char sm[LDS ? TR_NB_MAX : 16];
    __shared__ int list[TR_LIST], link[TR_NCH], cout_[TR_NCH], cown[TR_NCH];
    __shared__ int s_nch, s_len[R360_MAX_MODELS], s_head[R360_MAX_MODELS], s_over;
    __shared__ long s_off[R360_MAX_MODELS];
    const int s = blockIdx.x, N = w * h;
    const uint8_t* nbs = nbg + (long)s * N;
    const int nm = nmodels[s];
    if (LDS) {
        const uint4* src4 = reinterpret_cast<const uint4*>(nbs);
        uint4* dst4 = reinterpret_cast<uint4*>(sm);
        if ((N & 15) == 0 && ((reinterpret_cast<uintptr_t>(nbs) & 15) == 0)) {
            for (int q = threadIdx.x; q < N / 16; q += TR_TPB) dst4[q] = src4[q];
        } else {
            for (int q = threadIdx.x; q < N; q += TR_TPB) sm[q] = nbs[q];
        }
    }
    if (threadIdx.x == 0) { s_nch = 0; s_over = 0; }
    // a chain can end with an allocated but empty chunk (length a multiple of TR_CHUNK): unowned
    for (int c = threadIdx.x; c < TR_NCH; c += TR_TPB) cown[c] = -1;
    __syncthreads();
    const uint8_t* nb = LDS ? sm : nbs;
    // Moore directions {W, NW, N, NE, E, SE, S, SW} as 2-bit fields of two constants (a dynamically indexed
    // local table would be a global-memory load on the trace's dependency chain)
    auto dxs = [](int d) { return (int)((0x1A90U >> (2 * d)) & 3u) - 1; };
    auto dys = [](int d) { return (int)((0xA901U >> (2 * d)) & 3u) - 1; };
    // the step's index offset dy * w + dx with a 24-bit multiply of the raw (0..2) fields
    const int wp1 = w + 1;
    auto step_off = [&](int d) {
        return (int)__umul24((0xA901U >> (2 * d)) & 3u, (unsigned)w) + (int)((0x1A90U >> (2 * d)) & 3u) - wp1;
    };
    const int max_len = 8 * N;
    const int m = threadIdx.x;
    int dir0 = -1, start = 0;
    if (m < nm) {
        PlaneOut& O = out[s * R360_MAX_MODELS + m];
        start = O.start;
        const int cx = start % w, cy = start / w;
        const unsigned m8 = nb[start];
        for (int d = 0; d < 8; ++d) {
            const int x = cx + dxs(d), y = cy + dys(d);
            if (x >= 0 && x < w && y >= 0 && y < h && !((m8 >> d) & 1)) { dir0 = d; break; }
        }
        int n = 0;
        if (dir0 >= 0) {
            int chunk = atomicAdd(&s_nch, 1), pos = 0;
            s_head[m] = chunk;
            auto append = [&](int idx) {
                // past the list's end the chunk index is clamped instead of branched on: s_nch > TR_NCH then, the
                // whole list is discarded (s_over) and the overflow walk below writes the points
                list[min(chunk, TR_NCH - 1) * TR_CHUNK + pos] = idx;
                if (++pos == TR_CHUNK) {
                    const int nc = atomicAdd(&s_nch, 1);
                    if (chunk < TR_NCH) link[chunk] = nc;
                    chunk = nc;
                    pos = 0;
                }
            };
            append(start);
            n = 1;
            int cidx = start, dir = dir0;
            unsigned mc = nb[cidx];
            do {
                const int nd = trace_next(mc, dir);
                dir = (nd + 4) & 7;
                cidx += step_off(nd);
                mc = nb[cidx];   // the next step's mask (cidx is a member pixel): in flight under the bookkeeping
                append(cidx);
                if (++n > max_len) { atomicOr(err, 8); break; }
            } while (cidx != start);
        }
        s_len[m] = (int)n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // contour pool partitioned per sensor: sensor s owns [s, s+1) * pool_cap / 8
        const long base = s * (pool_cap / 8), cap = pool_cap / 8;
        long o = 0;
        for (int k = 0; k < nm; ++k) { s_off[k] = base + o; o += s_len[k]; }
        if (o > cap) atomicOr(err, 16);
        if (s_nch > TR_NCH) s_over = 1;
        for (int k = 0; k < nm; ++k) {
            PlaneOut& O = out[s * R360_MAX_MODELS + k];
            O.n_contour = s_len[k];
            O.contour_off = s_off[k];
        }
    }
    __syncthreads();
    if (!s_over) {
        // chunk -> (region, output position), one lane per region walking its chain
        if (m < nm && s_len[m] > 0) {
            int c = s_head[m];
            for (int j = 0; j * TR_CHUNK < s_len[m]; ++j) {
                cout_[c] = j * TR_CHUNK;
                cown[c] = m;
                if ((j + 1) * TR_CHUNK < s_len[m]) c = link[c];
            }
        }
        __syncthreads();
        const float4* P = cloud + (long)s * N;
        const long cap_end = (s + 1) * (pool_cap / 8);
        for (int e = threadIdx.x; e < s_nch * TR_CHUNK; e += TR_TPB) {
            const int c = e / TR_CHUNK;
            const int r = cown[c];
            if (r < 0) continue;
            const int k = cout_[c] + (e - c * TR_CHUNK);
            if (k < s_len[r]) {
                const long dst = s_off[r] + k;
                if (dst < cap_end) pool[dst] = P[list[e]];
            }
        }
    } else if (m < nm && dir0 >= 0) {
        // more contour pixels than the LDS list holds: walk again, writing the points directly
        const float4* P = cloud + (long)s * N;
        const long cap_end = (s + 1) * (pool_cap / 8);
        long n = 0, dst = s_off[m];
        int cidx = start, dir = dir0;
        if (dst < cap_end) pool[dst] = P[start];
        ++n;
        do {
            const int nd = trace_next(nb[cidx], dir);
            dir = (nd + 4) & 7;
            cidx += step_off(nd);
            if (dst + n < cap_end) pool[dst + n] = P[cidx];
        } while (++n <= max_len && cidx != start);
    }
}
template <bool LDS>
__global__ void __launch_bounds__(TR_TPB) k_trace(const PlaneBatch B, int w, int h) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_trace<LDS>(reinterpret_cast<const uint8_t*>(D.mask), D.cloud, w, h, D.nmodels, D.out, D.contour_dev, D.contour_cap, D.err);
}


// contour total of the frame (profiling / pool accounting), and the voxel hash table size for this
// frame: a power of two >= 2x a bound on the distinct voxels of the regions without a contour (per region the
// smaller of its inliers and its bounding box's voxels), capped by the allocation
// one workgroup of 512 threads, thread = (sensor, model)
__device__ __forceinline__ void d_alloc(const int* __restrict__ nmodels, const PlaneOut* __restrict__ out,
                                               unsigned long long cap,
                                               long* __restrict__ totals) {
    __shared__ long sco[8], sca[8];
    const int q = threadIdx.x, s = q / R360_MAX_MODELS, m = q % R360_MAX_MODELS;
    long co = 0, cand = 0;
    if (m < nmodels[s]) {
        const int nc = out[q].n_contour;
        co = nc;
        if (nc == 0) {
            // distinct voxels of the region: at most its inliers and at most the voxels of its bounding box
            const float inv = 1.0f / 0.05f;
            double vol = 1.0;
            for (int k = 0; k < 3; ++k)
                vol *= (double)((long long)floorf(out[q].bmax[k] * inv) - (long long)floorf(out[q].bmin[k] * inv) + 1);
            cand = out[q].stats.n;
            if (vol >= 1.0 && vol < (double)cand) cand = (long)vol;
        }
    }
    for (int o = 32; o > 0; o >>= 1) { co += __shfl_xor(co, o, 64); cand += __shfl_xor(cand, o, 64); }
    if ((q & 63) == 0) { sco[q >> 6] = co; sca[q >> 6] = cand; }
    __syncthreads();
    if (q != 0) return;
    co = 0; cand = 0;
    for (int w = 0; w < 8; ++w) { co += sco[w]; cand += sca[w]; }
    totals[0] = co;
    unsigned long long t = 1024;
    while (t < 2ull * (unsigned long long)cand && t < cap) t <<= 1;
    totals[2] = (long)(t - 1);   // hash mask
    totals[3] = cand;            // bound on the voxels of the regions without a contour (0: no voxel stage work)
}
__global__ void __launch_bounds__(512) k_alloc(const PlaneBatch B) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_alloc(D.nmodels, D.out, D.vhash_cap, D.totals);
}



// pcl::VoxelGrid (leaf 0.05) of the inliers of regions without a contour (Frame360.h:1017-1026):
// points are hashed by (region, voxel index); voxel sums of <= a few hundred coordinates with ulps
// >= 2^-36 are exact in double, so atomic accumulation is order-free and equals the sequential sum.
__device__ __forceinline__ unsigned long long vhash(unsigned long long tag, unsigned long long mask) {
    return (tag * 0x9E3779B97F4A7C15ull >> 20) & mask;
}

// Only the inliers of regions without a contour are hashed.  A workgroup takes VOX_PX consecutive pixels (a few
// rows of a sensor, so its points fall into a few dozen voxels), sums them per (region, voxel) in an LDS hash
// table (exact double sums: order-free), then flushes one update per voxel it touched into the global table.
// New voxels are counted per region in LDS and flushed once per workgroup.
constexpr int VOX_TPB = 256, VOX_PX = 1024, VOX_LT = 512;   // VOX_PX: default pixels per workgroup (2048: 3.4x, 4096:
                                                            // 15x slower, profiles/r3_planes)

// a cell this workgroup claims is appended to its list (vlist_b, count in LDS *nclaim) for k_vox_compact
__device__ __forceinline__ void vox_global_add(VoxCell* __restrict__ tab, unsigned long long mask,
                                               unsigned long long tag, double x, double y, double z, unsigned n,
                                               int* __restrict__ nnew_slot, int* __restrict__ err,
                                               int* __restrict__ nclaim, int* __restrict__ vlist_b) {
    unsigned long long hsh = vhash(tag, mask);
    for (unsigned long long probe = 0;; ++probe) {
        const unsigned long long prev = atomicCAS(&tab[hsh].tag, 0ull, tag);
        if (prev == 0ull) {
            atomicAdd(nnew_slot, 1);
            vlist_b[atomicAdd(nclaim, 1)] = (int)hsh;
            break;
        }
        if (prev == tag) break;
        hsh = (hsh + 1) & mask;
        if (probe > mask) { atomicOr(err, 16); return; }
    }
    atomicAdd(&tab[hsh].s[0], x);
    atomicAdd(&tab[hsh].s[1], y);
    atomicAdd(&tab[hsh].s[2], z);
    atomicAdd(&tab[hsh].cnt, n);
}

__device__ __forceinline__ void d_vox_hash(const float4* __restrict__ cloud, const int8_t* __restrict__ state,
                                                     int N, const int* __restrict__ nmodels, PlaneOut* __restrict__ out,
                                                     VoxCell* __restrict__ tab, const long* __restrict__ totals,
                                                     int* __restrict__ err, int px, int* __restrict__ vlist,
                                                     int* __restrict__ vcnt) {
    if (totals[3] == 0) return;
    __shared__ int s_nclaim;
    int* const vlist_b = vlist + (long)blockIdx.x * px;
    __shared__ int nnew_[2 * R360_MAX_MODELS];
    __shared__ unsigned char cand_[2 * R360_MAX_MODELS];
    __shared__ long long bnd_[2 * R360_MAX_MODELS][5];   // voxel origin b0..b2 and extents d0, d1 of a region
    __shared__ unsigned long long ltag[VOX_LT];
    __shared__ double lsum[3][VOX_LT];
    __shared__ unsigned lcnt[VOX_LT];
    __shared__ int any;
    const long total = 8L * N;
    const long i0 = (long)blockIdx.x * px;
    const int s0 = (int)(i0 / N), s1 = (int)(min(total, i0 + px) - 1) / N;   // sensors of this block (px <= N)
    // the block's regions, indexed by (sensor, model) - s0 * R360_MAX_MODELS
    int* nnew = nnew_ - s0 * R360_MAX_MODELS;
    unsigned char* cand = cand_ - s0 * R360_MAX_MODELS;
    long long (*bnd)[5] = bnd_ - s0 * R360_MAX_MODELS;
    const float inv = 1.0f / 0.05f;
    if (threadIdx.x == 0) { any = 0; s_nclaim = 0; }
    for (int q = threadIdx.x; q < VOX_LT; q += VOX_TPB) {
        ltag[q] = 0ull; lsum[0][q] = 0.0; lsum[1][q] = 0.0; lsum[2][q] = 0.0; lcnt[q] = 0u;
    }
    for (int q = threadIdx.x; q < (s1 - s0 + 1) * R360_MAX_MODELS; q += VOX_TPB) {
        const int sm = s0 * R360_MAX_MODELS + q;
        const PlaneOut& O = out[sm];
        const bool c = (q % R360_MAX_MODELS) < nmodels[sm / R360_MAX_MODELS] && O.n_contour == 0;
        cand[sm] = c;
        nnew[sm] = 0;
        if (c) {
            bnd[sm][0] = (long long)floorf(O.bmin[0] * inv);
            bnd[sm][1] = (long long)floorf(O.bmin[1] * inv);
            bnd[sm][2] = (long long)floorf(O.bmin[2] * inv);
            bnd[sm][3] = (long long)floorf(O.bmax[0] * inv) - bnd[sm][0] + 1;
            bnd[sm][4] = (long long)floorf(O.bmax[1] * inv) - bnd[sm][1] + 1;
            any = 1;
        }
    }
    __syncthreads();
    if (!any) {
        if (threadIdx.x == 0) vcnt[blockIdx.x] = 0;
        return;
    }
    const unsigned long long mask = (unsigned long long)totals[2];
    for (int k = threadIdx.x; k < px; k += VOX_TPB) {
        const long i = i0 + k;
        if (i >= total) break;
        const int m = state[i];
        if (m < 0) continue;
        const int s = (int)(i / N);
        const int sm = s * R360_MAX_MODELS + m;
        if (!cand[sm]) continue;
        const float4 p = cloud[i];
        const long long* B = bnd[sm];
        const long long key = ((long long)floorf(p.x * inv) - B[0]) + ((long long)floorf(p.y * inv) - B[1]) * B[3] +
                              ((long long)floorf(p.z * inv) - B[2]) * B[3] * B[4];
        const unsigned long long tag = ((unsigned long long)(sm + 1) << 48) | (unsigned long long)key;
        unsigned q = (unsigned)vhash(tag, VOX_LT - 1);
        bool ok = false;
        for (int probe = 0; probe < VOX_LT; ++probe) {
            const unsigned long long prev = atomicCAS(&ltag[q], 0ull, tag);
            if (prev == 0ull || prev == tag) { ok = true; break; }
            q = (q + 1) & (VOX_LT - 1);
        }
        if (ok) {
            atomicAdd(&lsum[0][q], (double)p.x);
            atomicAdd(&lsum[1][q], (double)p.y);
            atomicAdd(&lsum[2][q], (double)p.z);
            atomicAdd(&lcnt[q], 1u);
        } else {   // more distinct voxels than VOX_LT in one block: straight to the global table
            vox_global_add(tab, mask, tag, p.x, p.y, p.z, 1u, &nnew[sm], err, &s_nclaim, vlist_b);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < VOX_LT; q += VOX_TPB) {
        const unsigned long long tag = ltag[q];
        if (tag) vox_global_add(tab, mask, tag, lsum[0][q], lsum[1][q], lsum[2][q], lcnt[q], &nnew[(int)(tag >> 48) - 1], err,
                                &s_nclaim, vlist_b);
    }
    __syncthreads();
    if (threadIdx.x == 0) vcnt[blockIdx.x] = s_nclaim;
    for (int q = threadIdx.x; q < (s1 - s0 + 1) * R360_MAX_MODELS; q += VOX_TPB) {
        const int sm = s0 * R360_MAX_MODELS + q;
        if (nnew[sm]) atomicAdd(&out[sm].n_vox, nnew[sm]);
    }
}
__global__ void __launch_bounds__(VOX_TPB) k_vox_hash(const PlaneBatch B, int N, int px) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_vox_hash(D.cloud, D.state, N, D.nmodels, D.out, D.vhash, D.totals, D.err, px, D.vlist, D.vcnt);
}


// voxel list offsets per region in (sensor, model) order: one workgroup of 512 threads, exclusive scan
__device__ __forceinline__ void d_vox_alloc(const int* __restrict__ nmodels, PlaneOut* __restrict__ out,
                                                   long* __restrict__ totals, long vox_cap, int* __restrict__ err) {
    __shared__ long sw[8];
    const int q = threadIdx.x, lane = q & 63, wid = q >> 6;
    const bool live = (q % R360_MAX_MODELS) < nmodels[q / R360_MAX_MODELS];
    const long v = live ? out[q].n_vox : 0;
    long x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const long y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sw[wid] = x;
    __syncthreads();
    long pre = 0;
    for (int w = 0; w < wid; ++w) pre += sw[w];
    if (live) out[q].vox_off = pre + x - v;
    if (q == 511) {
        totals[1] = pre + x;
        if (pre + x > vox_cap) atomicOr(err, 16);
    }
}
__global__ void __launch_bounds__(512) k_vox_alloc(const PlaneBatch B) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_vox_alloc(D.nmodels, D.out, D.totals, D.vox_cap, D.err);
}


// one workgroup per k_vox_hash workgroup: the cells that workgroup claimed (its list) are counted per region in LDS
// (one LDS atomic per (wave, region)), one global atomic per (workgroup, region) reserves the slots, then the cells
// are written — and cleared, so that the table is all zero again for the next frame of this context (no clearing
// kernel, and no pass over the cells nobody claimed).
constexpr int VOXC_TPB = 256;

// runs of equal region keys within a wave: per distinct key the lanes' mask (the leader adds the count)
template <typename F>
__device__ __forceinline__ void wave_by_key(int key, F&& f) {
    bool pending = key >= 0;
    while (__any(pending)) {
        const unsigned long long act = __ballot(pending);
        const int leader = __ffsll((long long)act) - 1;
        const int lk = __shfl(key, leader, 64);
        const bool mine = pending && key == lk;
        f(lk, __ballot(mine), leader, mine);
        if (mine) pending = false;
    }
}

__device__ __forceinline__ void d_vox_compact(VoxCell* __restrict__ tab,
                                                         const long* __restrict__ totals, PlaneOut* __restrict__ out,
                                                         VoxOut* __restrict__ pool, long pool_cap,
                                                         const int* __restrict__ vlist, const int* __restrict__ vcnt,
                                                         int px) {
    if (totals[3] == 0) return;
    const int n = vcnt[blockIdx.x];
    if (n == 0) return;
    __shared__ int cnt[8 * R360_MAX_MODELS], base[8 * R360_MAX_MODELS];
    for (int q = threadIdx.x; q < 8 * R360_MAX_MODELS; q += VOXC_TPB) cnt[q] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int* L = vlist + (long)blockIdx.x * px;
    for (int kb = 0; kb < n; kb += VOXC_TPB) {
        const int k = kb + threadIdx.x;
        const unsigned long long tag = k < n ? tab[L[k]].tag : 0ull;
        wave_by_key(tag ? (int)(tag >> 48) - 1 : -1, [&](int key, unsigned long long m, int leader, bool) {
            if (lane == leader) atomicAdd(&cnt[key], __popcll(m));
        });
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 8 * R360_MAX_MODELS; q += VOXC_TPB) {
        base[q] = cnt[q] ? atomicAdd(&out[q].vox_fill, cnt[q]) : 0;
        cnt[q] = 0;
    }
    __syncthreads();
    for (int kb = 0; kb < n; kb += VOXC_TPB) {
        const int k = kb + threadIdx.x;
        const int c = k < n ? L[k] : 0;
        const unsigned long long tag = k < n ? tab[c].tag : 0ull;
        const int sm = tag ? (int)(tag >> 48) - 1 : -1;
        int pos = 0;
        wave_by_key(sm, [&](int key, unsigned long long m, int leader, bool mine) {
            int o = 0;
            if (lane == leader) o = atomicAdd(&cnt[key], __popcll(m));
            o = __shfl(o, leader, 64);
            if (mine) pos = base[key] + o + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        });
        if (sm < 0) continue;
        const PlaneOut& O = out[sm];
        const double cn = (double)tab[c].cnt;
        VoxOut v;
        v.key = (long long)(tag & ((1ull << 48) - 1));
        v.x = (float)(tab[c].s[0] / cn);
        v.y = (float)(tab[c].s[1] / cn);
        v.z = (float)(tab[c].s[2] / cn);
        v.pad = 0.f;
        if (O.vox_off + pos < pool_cap) pool[O.vox_off + pos] = v;
        tab[c].tag = 0;
        tab[c].s[0] = tab[c].s[1] = tab[c].s[2] = 0.0;
        tab[c].cnt = 0;
    }
}
__global__ void __launch_bounds__(VOXC_TPB) k_vox_compact(const PlaneBatch B, int px) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_vox_compact(D.vhash, D.totals, D.out, D.vox_dev, D.vox_cap, D.vlist, D.vcnt, px);
}

// The convex hull's Akl-Toussaint prefilter, on the device (round 6: on the host it was 0.67 of the 0.91 ms a synthetic
// frame's PbMap assembly took, 49k points per frame, and the full point lists crossed PCIe into pinned memory).  One
// workgroup per region, over its traced contour (k_trace, in trace order) or, for a region without one, its VoxelGrid
// centroids (k_vox_compact): the extreme points in 8 directions of the hull plane's two coordinates form an octagon (a
// convex polygon of input points, so inside the hull); every point strictly inside it by the margin 1e-7 (|e_x| + |e_y|) S
// (S = the box width + height of the region's points; far above the rounding of the host's double turn test) is dropped,
// and the survivors are compacted, in list order, into the pinned pool at the region's contour_off / vox_off; hull_n
// becomes their count.  The host's monotone chain over the survivors gives the hull of all points (its output does not
// depend on points strictly inside the hull; regions of fewer than 64 points keep all).  Contour survivors keep their
// relative order (the host ranks ties by it); voxel survivors are ranked by voxel index on the host, as before.
constexpr int VOXH_TPB = 256;
template <class PT>
__device__ __forceinline__ float pt_coord(const PT& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : v.z; }

template <class PT>
__device__ __forceinline__ int d_hullpre(const PT* __restrict__ src, PT* __restrict__ dst, int n, const PlaneModel& model) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // the hull plane: the two coordinates other than the normal's dominant axis (pbmap.cpp axis_of)
    const float n0 = fabsf(model.v[0]), n1 = fabsf(model.v[1]), n2 = fabsf(model.v[2]);
    int k0 = n0 > n1 ? 0 : 1;
    k0 = (k0 == 0 ? n0 : n1) > n2 ? k0 : 2;
    const int ca = (k0 + 1) % 3, cb = (k0 + 2) % 3;
    __shared__ double s_v[VOXH_TPB];
    __shared__ int s_i[VOXH_TPB];
    __shared__ double s_best[8], s_ex[8], s_ey[8], s_vx[8], s_vy[8], s_M[8];
    __shared__ int s_idx[8], s_all, s_wc[VOXH_TPB / 64], s_base;
    // pass 1: per direction the largest value, the first point among equals
    double best[8];
    int bi[8];
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0x7fffffff; }
    for (int i = tid; i < n; i += VOXH_TPB) {
        const double x = pt_coord(src[i], ca), y = pt_coord(src[i], cb);
        const double v[8] = {-x, -x - y, -y, x - y, x, x + y, y, y - x};
        for (int k = 0; k < 8; ++k)
            if (v[k] > best[k]) { best[k] = v[k]; bi[k] = i; }
    }
    for (int k = 0; k < 8; ++k) {
        s_v[tid] = best[k];
        s_i[tid] = bi[k];
        __syncthreads();
        for (int o = VOXH_TPB / 2; o > 0; o >>= 1) {
            if (tid < o) {
                const double a = s_v[tid], b = s_v[tid + o];
                const int ia = s_i[tid], ib = s_i[tid + o];
                if (b > a || (b == a && ib < ia)) { s_v[tid] = b; s_i[tid] = ib; }
            }
            __syncthreads();
        }
        if (tid == 0) { s_best[k] = s_v[0]; s_idx[k] = s_i[0]; }
        __syncthreads();
    }
    // the octagon (consecutive equal vertices merged) and its edges' constants
    if (tid == 0) {
        double vx[8], vy[8];
        int mm = 0;
        for (int k = 0; k < 8; ++k) {
            const double x = pt_coord(src[s_idx[k]], ca), y = pt_coord(src[s_idx[k]], cb);
            if (mm && x == vx[mm - 1] && y == vy[mm - 1]) continue;
            vx[mm] = x; vy[mm] = y; ++mm;
        }
        if (mm > 1 && vx[mm - 1] == vx[0] && vy[mm - 1] == vy[0]) --mm;
        s_all = (n < 64 || mm < 3) ? 1 : 0;
        const double S = (s_best[4] + s_best[0]) + (s_best[6] + s_best[2]);
        for (int k = 0; k < 8; ++k) {
            const int e = k < mm ? k : 0, e1 = mm > 0 ? (e + 1) % mm : 0;
            s_ex[k] = mm > 0 ? vx[e1] - vx[e] : 0.0;
            s_ey[k] = mm > 0 ? vy[e1] - vy[e] : 0.0;
            s_vx[k] = mm > 0 ? vx[e] : 0.0;
            s_vy[k] = mm > 0 ? vy[e] : 0.0;
            s_M[k] = 1e-7 * (fabs(s_ex[k]) + fabs(s_ey[k])) * S;
        }
        s_base = 0;
    }
    __syncthreads();
    const bool all = s_all != 0;
    // pass 2: the survivors, compacted in list order
    for (int i0 = 0; i0 < n; i0 += VOXH_TPB) {
        const int i = i0 + tid;
        bool keep = false;
        PT v;
        if (i < n) {
            v = src[i];
            keep = true;
            if (!all) {
                const double x = pt_coord(v, ca), y = pt_coord(v, cb);
                bool inside = true;
                for (int k = 0; k < 8; ++k) inside = inside && (s_ex[k] * (y - s_vy[k]) - s_ey[k] * (x - s_vx[k])) > s_M[k];
                keep = !inside;
            }
        }
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) s_wc[wid] = __popcll(bal);
        __syncthreads();
        int off = s_base;
        for (int w = 0; w < wid; ++w) off += s_wc[w];
        if (keep) dst[off + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] = v;
        __syncthreads();
        if (tid == 0) for (int w = 0; w < VOXH_TPB / 64; ++w) s_base += s_wc[w];
        __syncthreads();
    }
    return s_base;
}

__global__ void __launch_bounds__(VOXH_TPB) k_hullpre(const PlaneBatch B) {
    const PlaneDev& D = B.f[blockIdx.z];
    const int q = blockIdx.x, s = q / R360_MAX_MODELS, m = q % R360_MAX_MODELS;
    if (m >= D.nmodels[s]) return;
    PlaneOut& O = D.out[q];
    int kept = 0;
    if (O.n_contour > 0)
        kept = d_hullpre(D.contour_dev + O.contour_off, D.contour + O.contour_off, O.n_contour, O.model);
    else if (O.n_vox > 0 && D.totals[3] != 0)
        kept = d_hullpre(D.vox_dev + O.vox_off, D.vox + O.vox_off, O.n_vox, O.model);
    if (threadIdx.x == 0) O.hull_n = kept;
}
}  // namespace


// refinement mode: -1 the wavefront sweeps (default; pipelined bands for h <= 512), -2 the wavefront sweeps with a
// barrier per diagonal, 0 the single-wave sweeps, rb > 0 banded with rb rows per band (R360_REFINE_ROWS overrides)
int refine_band_rows(int h) {
    static const int env = R360_KNOB("R360_REFINE_ROWS", -99);
    int rb = env >= -2 ? env : -1;
    if (rb < 0) return h <= 1024 ? rb : 0;
    if (rb > 0 && (h + rb - 1) / rb > R360_REFINE_BANDS) rb = (h + R360_REFINE_BANDS - 1) / R360_REFINE_BANDS;
    return rb;
}

// refine()'s two sweeps over 8 sensors' states (PlaneDev::state, in place) and closeness masks (mask) of each frame of
// the batch.  rb > 0: banded (phases 1 and 2 per sweep; state2 holds the first sweep's output); rb = 0: one wave per
// sensor walks every row (k_refine); rb < 0: the wavefront sweeps (rcode / rmsk / rf1 / rf2, rflag).
int launch_refine_sweeps(const PlaneBatch& B, int F, hipStream_t st, int w, int h, int rb, bool wave_bufs) {
    const int K = (w + 63) / 64;
    const unsigned nf = (unsigned)F;
    if (rb < 0 && (w < 2 || h > 1024 || !wave_bufs)) rb = 0;
    if (rb < 0) {
        const long slots = 8L * (h + w - 1) * h;
        hipLaunchKernelGGL(k_refine_skew, dim3((unsigned)((slots + 255) / 256), 1, nf), dim3(256), 0, st, B, w, h);
        const int tpb = 64 * ((h + 63) / 64);
        // R360_REFINE_NARROW=0: the 64-bit mask path for every sensor (inspection)
        static const int narrow_max = R360_KNOB("R360_REFINE_NARROW", 1) == 0 ? -1 : 30;
        if (rb == -1 && h <= 64 * RP_MAXB && w <= RP_MAXW) {
            if (h <= 256) {
                hipLaunchKernelGGL((k_refine_pipe<1, 4>), dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h, narrow_max);
                hipLaunchKernelGGL((k_refine_pipe<-1, 4>), dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h, narrow_max);
            } else {
                hipLaunchKernelGGL((k_refine_pipe<1, RP_MAXB>), dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h, narrow_max);
                hipLaunchKernelGGL((k_refine_pipe<-1, RP_MAXB>), dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h, narrow_max);
            }
        } else {
            hipLaunchKernelGGL(k_refine_wave<1>, dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h);
            hipLaunchKernelGGL(k_refine_wave<-1>, dim3(8, 1, nf), dim3(tpb), 0, st, B, w, h);
        }
        hipLaunchKernelGGL(k_refine_unskew, dim3((unsigned)((8L * w * h + 255) / 256), 1, nf), dim3(256), 0, st, B, w, h);
        switch (K) {
#define R360_FB_CASE(k) case k: hipLaunchKernelGGL(k_refine_fb<k>, dim3(8, 1, nf), dim3(64), 0, st, B, w, h); break;
            R360_FB_CASE(1) R360_FB_CASE(2) R360_FB_CASE(3) R360_FB_CASE(4) R360_FB_CASE(5)
            R360_FB_CASE(6) R360_FB_CASE(7) R360_FB_CASE(8) R360_FB_CASE(9) R360_FB_CASE(10)
#undef R360_FB_CASE
            default: r360_set_error("refine: cloud width %d > 640 unsupported", w); return -1;
        }
        R360_HIP(hipGetLastError());
        return 0;
    }
    if (rb > 0 && (h + rb - 1) / rb > R360_REFINE_BANDS) { r360_set_error("refine: %d rows per band too few", rb); return -2; }
    const int nb = rb > 0 ? (h + rb - 1) / rb : 0;
    switch (K) {
#define R360_REFINE_CASE(k)                                                                                     \
    case k:                                                                                                     \
        if (rb == 0) { hipLaunchKernelGGL(k_refine<k>, dim3(8, 1, nf), dim3(64), 0, st, B, w, h); break; }      \
        hipLaunchKernelGGL((k_refine_p1<k, 1>), dim3(nb, 8, nf), dim3(64), 0, st, B, w, h, rb);                 \
        hipLaunchKernelGGL((k_refine_p2<k, 1>), dim3(8, 1, nf), dim3(64), 0, st, B, w, h, rb, nb);              \
        hipLaunchKernelGGL((k_refine_p1<k, -1>), dim3(nb, 8, nf), dim3(64), 0, st, B, w, h, rb);                \
        hipLaunchKernelGGL((k_refine_p2<k, -1>), dim3(8, 1, nf), dim3(64), 0, st, B, w, h, rb, nb);             \
        break;
        R360_REFINE_CASE(1) R360_REFINE_CASE(2) R360_REFINE_CASE(3) R360_REFINE_CASE(4) R360_REFINE_CASE(5)
        R360_REFINE_CASE(6) R360_REFINE_CASE(7) R360_REFINE_CASE(8) R360_REFINE_CASE(9) R360_REFINE_CASE(10)
#undef R360_REFINE_CASE
        default: r360_set_error("refine: cloud width %d > 640 unsupported", w); return -1;
    }
    R360_HIP(hipGetLastError());
    return 0;
}

// ------------------------------------------------------------------ launcher
template <bool MODEL>
int launch_gm(int px, long total, const PlaneBatch& B, int F, hipStream_t st, int N) {
    const unsigned blocks = (unsigned)((total + px - 1) / px);
    static const int exp = R360_KNOB("R360_EXP_GM", 0);   // timing experiments only
    switch (px) {
#define R360_GM_CASE(cpw)                                                                                         \
    case 256 * cpw:                                                                                               \
        hipLaunchKernelGGL((k_gm<MODEL, cpw>), dim3(blocks, 1, (unsigned)F), dim3(GM_TPB), 0, st, B, N, exp);    \
        return 0;
        R360_GM_CASE(1) R360_GM_CASE(2) R360_GM_CASE(4) R360_GM_CASE(8) R360_GM_CASE(16)
#undef R360_GM_CASE
    }
    r360_set_error("segmentation: R360_GM_PX=%d (256, 512, 1024, 2048 or 4096)", px);
    return -1;
}

// the geometric part: connected components, plane fits, refinement (depth / normals only)
int launch_segmentation_geom(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx) {
    const int w = G.w, h = G.h, N = w * h;
    const long total = 8L * N;
    const int blocks = (int)((total + 255) / 256);
    const unsigned nf = (unsigned)F;
    // PlaneCoefficientComparator::setAngularThreshold stores cosf(angle) (angle 0.039812, Frame360.h:959)
    const float ang_thr = cosf((float)0.039812);
    int slot = timing_begin(tctx, "k_ccl");
    hipLaunchKernelGGL(k_ccl_local, dim3((h + CCL_ROWS - 1) / CCL_ROWS, 8, nf), dim3(CCL_TPB), sizeof(int) * CCL_ROWS * w,
                       st, B, w, h, ang_thr);
    {
        const long edges = 8L * ((h - 1) / CCL_ROWS) * w;
        if (edges > 0)
            hipLaunchKernelGGL(k_ccl_border, dim3((unsigned)((edges + 255) / 256), 1, nf), dim3(256), 0, st, B, w, h, ang_thr);
    }
    const int nch = (N + NUMC - 1) / NUMC;   // numbering chunks per sensor; their counts in chunk [8][nch]
    hipLaunchKernelGGL(k_ccl_flatten, dim3(nch, 8, nf), dim3(NUMC), 0, st, B, N);
    hipLaunchKernelGGL(k_ccl_number, dim3(nch, 8, nf), dim3(NUMC), 0, st, B, N);
    hipLaunchKernelGGL(k_ccl_label, dim3(blocks, 1, nf), dim3(256), 0, st, B, N);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_plane_fit");
    // aux: the large labels' first pixels [8][MAX_BIG].  parent / root are free after the labelling and hold the
    // label -> large-label and label -> model maps (the kernels' PlaneDev mapping, k_big_* / k_gm / k_plane_fit).
    hipLaunchKernelGGL(k_big_count, dim3(nch, 8, nf), dim3(NUMC), 0, st, B, N, 80);
    hipLaunchKernelGGL(k_big_list, dim3(nch, 8, nf), dim3(NUMC), 0, st, B, N, 80, R360_MAX_BIG);
    // pixels per workgroup of the grouped-moment kernels (R360_GM_PX, experiments)
    static const int gm_px = R360_KNOB("R360_GM_PX", GM_PX);
    if (launch_gm<false>(gm_px, total, B, F, st, N)) return -1;
    hipLaunchKernelGGL(k_plane_fit, dim3(8, 1, nf), dim3(PF_TPB), 0, st, B, R360_MAX_BIG, 0.001f, N);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_refine");
    hipLaunchKernelGGL(k_refine_init, dim3(blocks, 1, nf), dim3(256), 0, st, B, N);
    if (launch_refine_sweeps(B, F, st, w, h, refine_band_rows(h), true)) return -1;
    hipLaunchKernelGGL(k_refine_final, dim3(blocks, 1, nf), dim3(256), 0, st, B, N);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}

// the model part: the clouds' colours (the first kernel of the stage that reads the BGR images), the regions'
// statistics, contours, the voxel fallback and the hull prefilter
int launch_segmentation_model(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx) {
    const int w = G.w, h = G.h, N = w * h;
    const long total = 8L * N;
    const int blocks = (int)((total + 255) / 256);
    const unsigned nf = (unsigned)F;
    static const int gm_px = R360_KNOB("R360_GM_PX", GM_PX);
    int slot = timing_begin(tctx, "k_model_stats");
    if (launch_rgb(B, F, G, st)) return -1;
    if (launch_gm<true>(gm_px, total, B, F, st, N)) return -1;
    // the refinement's closeness masks are dead here: their storage holds the neighbour masks
    hipLaunchKernelGGL(k_nbmask, dim3(std::max(blocks, 20 * 8 * R360_MAX_MODELS / 256), 1, nf), dim3(256), 0, st, B, w, h);
    if (N <= TR_NB_MAX) hipLaunchKernelGGL(k_trace<true>, dim3(8, 1, nf), dim3(TR_TPB), 0, st, B, w, h);
    else hipLaunchKernelGGL(k_trace<false>, dim3(8, 1, nf), dim3(TR_TPB), 0, st, B, w, h);
    long cells, entries, groups;
    vox_scratch_need(G, &cells, &entries, &groups);
    const int vox_px = (int)(entries / groups);
    hipLaunchKernelGGL(k_alloc, dim3(1, 1, nf), dim3(512), 0, st, B);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    slot = timing_begin(tctx, "k_voxel");
    // the voxel kernels exit at entry when no region lacks a contour (totals[3] == 0, the usual case); the table is
    // zero on allocation and k_vox_compact clears every cell it reads
    hipLaunchKernelGGL(k_vox_hash, dim3((unsigned)groups, 1, nf), dim3(VOX_TPB), 0, st, B, N, vox_px);
    hipLaunchKernelGGL(k_vox_alloc, dim3(1, 1, nf), dim3(512), 0, st, B);
    hipLaunchKernelGGL(k_vox_compact, dim3((unsigned)groups, 1, nf), dim3(VOXC_TPB), 0, st, B, vox_px);
    hipLaunchKernelGGL(k_hullpre, dim3(8 * R360_MAX_MODELS, 1, nf), dim3(VOXH_TPB), 0, st, B);
    timing_end(tctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_segmentation(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx,
                        const hipEvent_t* bgr_ev) {
    if (launch_segmentation_geom(B, F, G, st, tctx)) return -1;
    // a split upload copies the BGR images beside the geometric part
    for (int j = 0; bgr_ev && j < F; ++j)
        if (bgr_ev[j]) R360_HIP(hipStreamWaitEvent(st, bgr_ev[j], 0));
    return launch_segmentation_model(B, F, G, st, tctx);
}

// hash cells (a bound on a frame's distinct (region, voxel) cells, k_alloc), and the claimed-cell lists of
// k_vox_hash: one per workgroup of vox_px pixels (R360_VOX_PX in experiment builds)
void vox_scratch_need(const PlaneGeom& G, long* cells, long* entries, long* groups) {
    const int N = G.w * G.h;
    static const int vox_px_env = R360_KNOB("R360_VOX_PX", VOX_PX);   // experiments
    const int vox_px = std::min(vox_px_env, N);   // a block spans at most two sensors
    const long vox_blocks = (8L * N + vox_px - 1) / vox_px;
    *cells = 12L * N;
    *entries = vox_blocks * vox_px;
    *groups = vox_blocks;
}

namespace {
// the plane stage's outputs for the host assembly, written straight into pinned host memory (one launch
// instead of four device-to-host copies): the region records, models per sensor, error word, totals
__device__ __forceinline__ void d_plane_publish(const PlaneOut* __restrict__ out, const int* __restrict__ nmodels,
                                const int* __restrict__ err, const long* __restrict__ totals, PlaneOut* __restrict__ h_out,
                                int* __restrict__ h_nm, int nwords) {
    // only the sensors' live region records (slots [0, nmodels[s]) of each sensor; ~48 of the 512): the rest would
    // be written over PCIe for nothing (round 6: the kernel's stores to pinned host memory hold its completion)
    const int* src = reinterpret_cast<const int*>(out);
    int* dst = reinterpret_cast<int*>(h_out);
    constexpr int per = (int)(sizeof(PlaneOut) / 4);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += gridDim.x * blockDim.x) {
        const int slot = i / per;
        if (slot % R360_MAX_MODELS < nmodels[slot / R360_MAX_MODELS]) dst[i] = src[i];
    }
    if (blockIdx.x == 0 && threadIdx.x < 14 && threadIdx.x != 9) {
        const int t = threadIdx.x;
        h_nm[t] = t < 8 ? nmodels[t] : t == 8 ? *err : reinterpret_cast<const int*>(totals)[t - 10];
    }
}
__global__ void k_plane_publish(const PlaneBatch B, int nwords) {
    const PlaneDev& D = B.f[blockIdx.z];
    d_plane_publish(D.out, D.nmodels, D.err, D.totals, D.h_out, D.h_nmodels, nwords);
}

}  // namespace

int launch_plane_publish(const PlaneBatch& B, int F, hipStream_t st) {
    static_assert(sizeof(PlaneOut) % 4 == 0, "PlaneOut is copied as 32-bit words");
    const int nwords = (int)(sizeof(PlaneOut) * 8 * R360_MAX_MODELS / 4);
    hipLaunchKernelGGL(k_plane_publish, dim3((nwords + 255) / 256, 1, (unsigned)F), dim3(256), 0, st, B, nwords);
    R360_HIP(hipGetLastError());
    return 0;
}

// Test hook: refine()'s two sweeps on given states / closeness masks of 8 sensors (w x h each): rb = -1 the
// wavefront sweeps (pipelined bands for h <= 512), -2 the barrier-per-diagonal wavefront, 0 the single-wave sweeps, rb > 0 banded with rb rows per band; out receives the swept
// states.  Returns the number of sensors whose wavefront second sweep needed wrap-push corrections (re-runs
// or the single-wave fallback; rb < 0), else 0.
extern "C" int r360_refine_eval(const int8_t* state, const uint64_t* mask, int w, int h, int rb, int8_t* out) {
    if (!state || !mask || !out || w < 1 || h < 1 || w > 640) { r360_set_error("r360_refine_eval: bad arguments"); return -2; }
    const size_t T = 8 * (size_t)w * h;
    int8_t *S, *S2, *bnd;
    unsigned long long* MK;
    int* flag;
    R360_HIP(hipMalloc(&S, T));
    R360_HIP(hipMalloc(&S2, T));
    R360_HIP(hipMalloc(&MK, sizeof(unsigned long long) * T));
    R360_HIP(hipMalloc(&bnd, 8L * R360_REFINE_BANDS * w));
    R360_HIP(hipMalloc(&flag, sizeof(int) * 8 * R360_REFINE_BANDS));
    R360_HIP(hipMemcpy(S, state, T, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(MK, mask, sizeof(unsigned long long) * T, hipMemcpyHostToDevice));
    uint16_t* code; unsigned long long* msk; int8_t *f1, *f2;
    const size_t SK = 8 * (size_t)(h + w - 1) * h;
    R360_HIP(hipMalloc(&code, sizeof(uint16_t) * SK));
    R360_HIP(hipMalloc(&msk, sizeof(unsigned long long) * SK));
    R360_HIP(hipMalloc(&f1, SK));
    R360_HIP(hipMalloc(&f2, SK));
    // models per sensor as the pipeline's k_plane_fit counts them: above every label and closeness bit
    int nmh[8], *nm;
    for (int s = 0; s < 8; ++s) {
        int top = 0;
        for (size_t i = (size_t)s * w * h; i < (size_t)(s + 1) * w * h; ++i) {
            if (state[i] + 1 > top) top = state[i] + 1;
            if (mask[i]) top = std::max(top, 64 - __builtin_clzll(mask[i]));
        }
        nmh[s] = top;
    }
    R360_HIP(hipMalloc(&nm, sizeof(nmh)));
    R360_HIP(hipMemcpy(nm, nmh, sizeof(nmh), hipMemcpyHostToDevice));
    PlaneBatch B;
    std::memset(&B, 0, sizeof B);
    PlaneDev& D = B.f[0];
    D.state = S; D.state2 = S2; D.mask = MK; D.rbnd = bnd; D.rflag = flag;
    D.rcode = code; D.rmsk = msk; D.rf1 = f1; D.rf2 = f2; D.nmodels = nm;
    int rc = launch_refine_sweeps(B, 1, 0, w, h, rb, true);
    if (rc == 0) {
        R360_HIP(hipMemcpy(out, S, T, hipMemcpyDeviceToHost));
        if (rb < 0 && w >= 2 && h <= 1024) {
            int fbh[16];
            R360_HIP(hipMemcpy(fbh, flag, sizeof(fbh), hipMemcpyDeviceToHost));
            for (int k = 0; k < 8; ++k) rc += (fbh[k] != 0 || fbh[8 + k] != 0);
            if (R360_KNOB_STR("R360_REFINE_TRACE"))
                for (int k = 0; k < 8; ++k) fprintf(stderr, "refine sensor %d: re-runs %d fallback row %d\n", k, fbh[8 + k], fbh[k] - 1);
        }
    }
    (void)hipFree(S); (void)hipFree(S2); (void)hipFree(MK); (void)hipFree(bnd); (void)hipFree(flag); (void)hipFree(nm);
    (void)hipFree(code); (void)hipFree(msk); (void)hipFree(f1); (void)hipFree(f2);
    return rc;
}
