// io_oracle.cpp — ORACLE (test infrastructure only, see oracle360.h).
// Restates the reference's frame I/O, CLAMS depth undistortion and spherical stitching.
#include "oracle360.h"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

static const double REF_PI = 3.14159265359;  // include/Miscellaneous.h:44

// ---------------------------------------------------------------------------
// A1 — Boost binary_iarchive of 8 x {RGB CV_8UC3, depth CV_16UC1} + timestamp mat.
// Reader: include/Frame360.h:236-249; per-mat layout: cvmat_serialization.h:39-55
// (int cols, int rows, size_t elem_size, size_t elem_type, raw bytes).
// The archive prologue is 45 bytes (verified on samples/*.bin).
// ---------------------------------------------------------------------------
static const int kArchivePrologue = 45;

static bool read_file(const char* path, std::vector<uint8_t>& buf) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    size_t n = (size_t)f.tellg();
    f.seekg(0);
    buf.resize(n);
    f.read((char*)buf.data(), n);
    return (bool)f;
}

struct MatHdr { int32_t cols, rows; uint64_t esz, etype; };

extern "C" int orc_bin_dims(const char* path, int* rows, int* cols) {
    std::vector<uint8_t> b;
    if (!read_file(path, b) || b.size() < kArchivePrologue + 24) return -1;
    MatHdr h; memcpy(&h, b.data() + kArchivePrologue, sizeof(h));
    *rows = h.rows; *cols = h.cols;
    return 0;
}

extern "C" int orc_bin_load(const char* path, uint8_t* bgr8, uint16_t* depth8) {
    std::vector<uint8_t> b;
    if (!read_file(path, b)) return -1;
    size_t off = kArchivePrologue;
    int rows = -1, cols = -1;
    for (int s = 0; s < 8; ++s) {
        for (int m = 0; m < 2; ++m) {
            if (off + 24 > b.size()) return -2;
            MatHdr h; memcpy(&h, b.data() + off, sizeof(h)); off += 24;
            if (rows < 0) { rows = h.rows; cols = h.cols; }
            if (h.rows != rows || h.cols != cols) return -3;
            size_t n = (size_t)h.cols * h.rows * h.esz;
            if (off + n > b.size()) return -4;
            if (m == 0) {  // RGB (stored BGR), CV_8UC3 = type 16
                if (h.esz != 3 || h.etype != 16) return -5;
                memcpy(bgr8 + (size_t)s * rows * cols * 3, b.data() + off, n);
            } else {       // depth mm, CV_16UC1 = type 2
                if (h.esz != 2 || h.etype != 2) return -6;
                memcpy(depth8 + (size_t)s * rows * cols, b.data() + off, n);
            }
            off += n;
        }
    }
    return 0;
}

// Writer mirror of Frame360::serialize (include/Frame360.h:333-345); timestamp = empty mat.
extern "C" int orc_bin_write(const char* path, const uint8_t* bgr8, const uint16_t* depth8, int rows, int cols) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return -1;
    uint64_t len = 22;
    f.write((const char*)&len, 8);
    f.write("serialization::archive", 22);
    const uint8_t tail[15] = {9, 0, 4, 8, 4, 8, 1, 0, 0, 0, 0, 0, 0, 0, 0};
    f.write((const char*)tail, 15);
    for (int s = 0; s < 8; ++s) {
        MatHdr h{cols, rows, 3, 16};
        f.write((const char*)&h, 24);
        f.write((const char*)(bgr8 + (size_t)s * rows * cols * 3), (size_t)rows * cols * 3);
        MatHdr hd{cols, rows, 2, 2};
        f.write((const char*)&hd, 24);
        f.write((const char*)(depth8 + (size_t)s * rows * cols), (size_t)rows * cols * 2);
    }
    MatHdr ht{0, 0, 0, 0};
    f.write((const char*)&ht, 24);
    return f ? 0 : -2;
}

// ---------------------------------------------------------------------------
// A2 — CLAMS DiscreteDepthDistortionModel
// deserialize: discrete_depth_distortion_model.cpp:259-280 (+ DiscreteFrustum :82-91)
// downsampleParams(2): :313-320 ; undistort: :175-186 ; interpolatedUndistort: :48-68
// ---------------------------------------------------------------------------
struct Frustum {
    double max_dist; int num_bins; double bin_depth;
    std::vector<float> counts, mult;
};
struct ClamsModel {
    int width, height, bin_w, bin_h, nx, ny; double bin_depth;
    std::vector<Frustum> fr;  // [ny][nx]
};

template <class T> static bool rd(std::istream& in, T* v) { in.read((char*)v, sizeof(T)); return (bool)in; }
static bool rd_vecf(std::istream& in, std::vector<float>& v) {
    int bytes, rows, cols;
    if (!rd(in, &bytes) || !rd(in, &rows) || !rd(in, &cols) || bytes != 4) return false;
    v.resize((size_t)rows * cols);
    in.read((char*)v.data(), v.size() * 4);
    return (bool)in;
}

extern "C" void* orc_clams_load(const char* path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return nullptr;
    std::string line;
    std::getline(in, line);
    ClamsModel* m = new ClamsModel;
    if (line == "R360CLAMS1") {  // compact table written by tools/compact_clams.py (counts + multipliers)
        int nb;
        rd(in, &m->width); rd(in, &m->height); rd(in, &m->bin_w); rd(in, &m->bin_h);
        rd(in, &m->nx); rd(in, &m->ny); rd(in, &nb); rd(in, &m->bin_depth);
        m->fr.resize((size_t)m->nx * m->ny);
        std::vector<float> c((size_t)m->nx * m->ny * nb), mu((size_t)m->nx * m->ny * nb);
        in.read((char*)c.data(), 4 * c.size());
        in.read((char*)mu.data(), 4 * mu.size());
        if (!in) { delete m; return nullptr; }
        for (size_t i = 0; i < m->fr.size(); ++i) {
            Frustum& f = m->fr[i];
            f.max_dist = 10; f.num_bins = nb; f.bin_depth = m->bin_depth;
            f.counts.assign(c.begin() + i * nb, c.begin() + (i + 1) * nb);
            f.mult.assign(mu.begin() + i * nb, mu.begin() + (i + 1) * nb);
        }
    } else if (line == "DiscreteDepthDistortionModel v01") {
        rd(in, &m->width); rd(in, &m->height); rd(in, &m->bin_w); rd(in, &m->bin_h);
        rd(in, &m->bin_depth); rd(in, &m->nx); rd(in, &m->ny);
        m->fr.resize((size_t)m->nx * m->ny);
        std::vector<float> tn, td;
        for (auto& f : m->fr) {
            rd(in, &f.max_dist); rd(in, &f.num_bins); rd(in, &f.bin_depth);
            if (!rd_vecf(in, f.counts) || !rd_vecf(in, tn) || !rd_vecf(in, td) || !rd_vecf(in, f.mult)) {
                delete m; return nullptr;
            }
        }
    } else {
        delete m;
        return nullptr;
    }
    // Calib360::loadIntrinsicCalibration -> downsampleParams(2) (include/Calib360.h:115)
    m->width /= 2; m->height /= 2; m->bin_w /= 2; m->bin_h /= 2;
    return m;
}

extern "C" void orc_clams_free(void* model) { delete (ClamsModel*)model; }

// hdr = {width, height, bin_w, bin_h, nx, ny, num_bins, 0}; mult/counts = [ny*nx*num_bins]
extern "C" int orc_clams_export(const void* model, int* hdr, float* mult, float* counts) {
    const ClamsModel* m = (const ClamsModel*)model;
    int nb = m->fr[0].num_bins;
    hdr[0] = m->width; hdr[1] = m->height; hdr[2] = m->bin_w; hdr[3] = m->bin_h;
    hdr[4] = m->nx; hdr[5] = m->ny; hdr[6] = nb; hdr[7] = 0;
    if (mult) {
        for (size_t i = 0; i < m->fr.size(); ++i)
            for (int b = 0; b < nb; ++b) {
                mult[i * nb + b] = m->fr[i].mult[b];
                counts[i * nb + b] = m->fr[i].counts[b];
            }
    }
    return nb;
}

static inline int fr_index(const Frustum& f, float z) {           // :42-45
    int i = (int)std::floor(z / f.bin_depth);
    return i < f.num_bins - 1 ? i : f.num_bins - 1;
}

static inline void interpolated_undistort(const Frustum& f, float* z) {  // :48-68
    int idx = fr_index(f, *z);
    float start = (float)(f.bin_depth * idx);
    int idx1 = (*z - start < f.bin_depth / 2) ? idx : idx + 1;
    int idx0 = idx1 - 1;
    if (idx0 < 0 || idx1 >= f.num_bins || f.counts[idx0] < 50 || f.counts[idx1] < 50) {
        *z *= f.mult[fr_index(f, *z)];                                   // DiscreteFrustum::undistort :47-50
        return;
    }
    double z0 = (idx0 + 1) * f.bin_depth - f.bin_depth * 0.5;
    double coeff1 = (*z - z0) / f.bin_depth;
    double coeff0 = 1.0 - coeff1;
    double mult = coeff0 * f.mult[idx0] + coeff1 * f.mult[idx1];
    *z = (float)(*z * mult);
}

extern "C" void orc_clams_undistort(const void* model, float* depth, int rows, int cols) {
    const ClamsModel* m = (const ClamsModel*)model;
    // The reference hard-codes 240x320 (:178-179), i.e. the downsampled model size.
    if (rows != m->height || cols != m->width) return;
    for (int v = 0; v < m->height; ++v)
        for (int u = 0; u < m->width; ++u) {
            float* z = depth + (size_t)v * cols + u;
            if (*z == 0) continue;
            const Frustum& f = m->fr[(size_t)(v / m->bin_h) * m->nx + (u / m->bin_w)];
            interpolated_undistort(f, z);
        }
}

// ---------------------------------------------------------------------------
// A10 — Frame360::stitchSphericalImage / stitchImage (include/Frame360.h:386-405, 1099-1148)
// ---------------------------------------------------------------------------
extern "C" void orc_stitch(const uint8_t* bgr8, const uint16_t* depth8, int rows, int cols,
                           const float* rt_inv8, const float* K, uint8_t* sph_bgr, uint16_t* sph_depth) {
    const int W = rows * 8;                                    // :391
    const int H = (int)(W * 0.5 * 60.0 / 180);                 // :392
    memset(sph_bgr, 0, (size_t)W * H * 3);
    memset(sph_depth, 0, (size_t)W * H * 2);
    const float fx = K[0], fy = K[4], cx = K[6], cy = K[7];    // col-major 3x3
    #pragma omp parallel for num_threads(8)
    for (int k = 0; k < 8; ++k) {
        const float* T = rt_inv8 + 16 * k;                     // Rt_inv[k] col-major
        const uint8_t* img = bgr8 + (size_t)k * rows * cols * 3;
        const uint16_t* dep = depth8 + (size_t)k * rows * cols;
        const float offsetPhi = H / 2 - 0.5;                   // :1104
        const float offsetTheta = -rows * 15 / 2 + 0.5;        // :1105
        const float angle_pixel = 2 * REF_PI / W;              // :1106
        for (int row_phi = 0; row_phi < H; ++row_phi) {
            float phi_i = (offsetPhi - row_phi) * angle_pixel;
            float v0 = std::sin(phi_i);
            float cos_phi = std::cos(phi_i);
            int c0 = (7 - k) * rows, c1 = (8 - k) * rows;      // :1119-1120
            for (int col = c0; col < c1; ++col) {
                float theta_i = (col + offsetTheta) * angle_pixel;
                float v1 = cos_phi * std::sin(theta_i);
                float v2 = cos_phi * std::cos(theta_i);
                float p0 = T[0] * v0 + T[4] * v1 + T[8] * v2;
                float p1 = T[1] * v0 + T[5] * v1 + T[9] * v2;
                float p2 = T[2] * v0 + T[6] * v1 + T[10] * v2;
                p0 = p0 + T[12]; p1 = p1 + T[13]; p2 = p2 + T[14];
                float u = fx * p0 / p2 + cx;                    // :1133
                float v = fy * p1 / p2 + cy;                    // :1134
                if (u >= 0 && u < cols && v >= 0 && v < rows) {
                    int iu = (int)u, iv = (int)v;
                    size_t si = (size_t)iv * cols + iu, di = (size_t)row_phi * W + col;
                    sph_bgr[di * 3 + 0] = img[si * 3 + 0];
                    sph_bgr[di * 3 + 1] = img[si * 3 + 1];
                    sph_bgr[di * 3 + 2] = img[si * 3 + 2];
                    double du = (double)((u - cx) / fx), dv = (double)((v - cy) / fy);
                    sph_depth[di] = (uint16_t)(dep[si] * std::sqrt(1 + std::pow(du, 2) + std::pow(dv, 2)));  // :1142
                }
            }
        }
    }
}
