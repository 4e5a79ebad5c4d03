// io.cpp — Frame360 .bin archive reader (Frame360::loadFrame, include/Frame360.h:231-266).
// The file is a Boost binary_iarchive of 8 x {cv::Mat RGB CV_8UC3, cv::Mat depth CV_16UC1}
// followed by a timestamp mat; each mat is {int cols, int rows, size_t elem_size,
// size_t elem_type, bytes} (cvmat_serialization.h:39-55).  No Boost here: the 45-byte archive
// prologue is checked and skipped.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <numeric>
#include <sstream>
#include <vector>

#include "../r360_internal.h"

// Timestamp <-> 1 x D CV_8U matrix of decimal digits, most significant first
// (OpenNI2_Grabber/FrameRGBD/SerializeFrameRGBD.h:47-89, used by Frame360.h:247 and :340).
static uint64_t timestamp_from_digits(const uint8_t* d, int n) {
    uint64_t v = 0, p10 = 1;
    for (int i = n - 1; i >= 0; --i) { v += p10 * uint64_t(d[i]); p10 *= 10; }
    return v;
}

static std::vector<uint8_t> timestamp_to_digits(uint64_t v) {
    std::vector<uint8_t> d;
    for (; v > 0; v /= 10) d.push_back(uint8_t(v % 10));
    return std::vector<uint8_t>(d.rbegin(), d.rend());
}

// The calling thread's page-locked staging buffer for .bin files (grown as needed, freed with the thread): a file
// is read into it in one call and its mats go to the device images by DMA.  Byte-wise stream reads and copies out of
// pageable memory were 4.9 ms of the 5.6 ms a QVGA loadFrame took (BASELINE configs[0]'s loadFrame).
namespace {
struct PinnedFileBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~PinnedFileBuf() { if (p) hipHostFree(p); }
    int reserve(size_t n) {
        if (n <= cap) return 0;
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        R360_HIP(hipHostMalloc(&p, n, hipHostMallocDefault));
        cap = n;
        return 0;
    }
};
thread_local PinnedFileBuf t_file;
}  // namespace

// Frame360::loadFrame (Frame360.h:231-266): the archive prologue is checked and skipped, the 8 x {RGB, depth} mats
// checked against the calibration's sensor size and copied to the frame's images, the timestamp mat decoded.
extern "C" int r360_frame_load_bin(r360_frame* f, const char* path) {
    if (f && bind_device(f->ctx->device)) return -1;
    if (!f || !path) { r360_set_error("null arg"); return -2; }
    CHECK_ARG(f->rows > 0, "a sphere-only frame has no sensor images");
    FILE* fp = fopen(path, "rb");
    if (!fp) { r360_set_error("cannot open %s", path); return -1; }
    fseek(fp, 0, SEEK_END);
    const long len = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    if (len < 0 || t_file.reserve((size_t)len + 1)) { fclose(fp); if (len < 0) r360_set_error("cannot size %s", path); return -1; }
    const size_t got = fread(t_file.p, 1, (size_t)len, fp);
    fclose(fp);
    if (got != (size_t)len) { r360_set_error("%s: short read", path); return -1; }
    const uint8_t* b = t_file.p;
    const size_t size = (size_t)len;
    static const char kTag[] = "serialization::archive";
    if (size < 45 + 24 || memcmp(b + 8, kTag, 22) != 0) {
        r360_set_error("%s: not a boost binary archive", path);
        return -1;
    }
    // every mat checked before any is copied (a malformed file leaves the frame as it was)
    size_t off = 45;
    size_t moff[8][2];
    const size_t npx = (size_t)f->rows * f->cols;
    for (int s = 0; s < 8; ++s)
        for (int m = 0; m < 2; ++m) {
            if (off + 24 > size) { r360_set_error("%s: truncated", path); return -1; }
            int32_t c, r; uint64_t esz, et;
            memcpy(&c, b + off, 4); memcpy(&r, b + off + 4, 4); memcpy(&esz, b + off + 8, 8); memcpy(&et, b + off + 16, 8);
            off += 24;
            if (r != f->rows || c != f->cols) {
                r360_set_error("%s: sensor %d is %dx%d, calib expects %dx%d", path, s, r, c, f->rows, f->cols);
                return -1;
            }
            const size_t n = (size_t)r * c * esz;
            if (off + n > size) { r360_set_error("%s: truncated payload", path); return -1; }
            if (m == 0 && (esz != 3 || et != 16)) { r360_set_error("%s: RGB mat type %llu", path, (unsigned long long)et); return -1; }
            if (m == 1 && (esz != 2 || et != 2)) { r360_set_error("%s: depth mat type %llu", path, (unsigned long long)et); return -1; }
            moff[s][m] = off;
            off += n;
        }
    planes_join(f);   // a plane stage still reading the images (a plane queue's batch) ends first
    hipStream_t st = f->ctx->stream;
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(st, e, 0));   // a split upload's copy in flight
    for (int s = 0; s < 8; ++s) {
        R360_HIP(hipMemcpyAsync(f->d_bgr + s * npx * 3, b + moff[s][0], npx * 3, hipMemcpyHostToDevice, st));
        R360_HIP(hipMemcpyAsync(f->d_depth + s * npx, b + moff[s][1], npx * 2, hipMemcpyHostToDevice, st));
    }
    f->bgr_split = false;
    // the timestamp mat (Frame360.h:244-247); loadFrame swallows archive errors here, so a missing
    // or malformed one leaves the timestamp at 0
    uint64_t ts = 0;
    if (off + 24 <= size) {
        int32_t c, r; uint64_t esz, et;
        memcpy(&c, b + off, 4); memcpy(&r, b + off + 4, 4); memcpy(&esz, b + off + 8, 8); memcpy(&et, b + off + 16, 8);
        off += 24;
        const size_t n = (c > 0 && r > 0) ? (size_t)c * r * esz : 0;
        if (n && esz == 1 && off + n <= size) ts = timestamp_from_digits(b + off, (int)n);
    }
    R360_HIP(hipStreamSynchronize(st));   // the staging buffer is the thread's next file's
    f->built = 0;
    f->timestamp = ts;
    return 0;
}

extern "C" int r360_frame_set_timestamp(r360_frame* f, uint64_t ts) {
    if (!f) { r360_set_error("null frame"); return -2; }
    f->timestamp = ts;
    return 0;
}

extern "C" int r360_frame_get_timestamp(const r360_frame* f, uint64_t* ts) {
    if (!f || !ts) { r360_set_error("null arg"); return -2; }
    *ts = f->timestamp;
    return 0;
}

// Frame360::serialize (Frame360.h:332-345): the Boost binary_oarchive prologue, 8 x {RGB, depth}
// as they were loaded (the raw sensor images, before undistortion), then the timestamp as a
// 1 x D CV_8U digit matrix.  A zero timestamp is written as the empty mat the sample captures
// carry (header {0,0,0,0}), so those files round-trip byte-identically.
extern "C" int r360_frame_save_bin(r360_frame* f, const char* path) {
    if (!f || !path) { r360_set_error("null arg"); return -2; }
    const size_t npx = (size_t)f->rows * f->cols;
    std::vector<uint8_t> bgr(8 * npx * 3);
    std::vector<uint16_t> depth(8 * npx);
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(f->ctx->stream, e, 0));
    R360_HIP(hipMemcpyAsync(bgr.data(), f->d_bgr, bgr.size(), hipMemcpyDeviceToHost, f->ctx->stream));
    R360_HIP(hipMemcpyAsync(depth.data(), f->d_depth, depth.size() * 2, hipMemcpyDeviceToHost, f->ctx->stream));
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    std::ofstream o(path, std::ios::binary);
    if (!o) { r360_set_error("cannot create %s", path); return -1; }
    // boost::archive prologue: string length, signature, library version 9, the sizes of
    // int/long/float/double, the endianness flag, then the cv::Mat class info (tracking 0,
    // version 0) — the 45 bytes every sample capture starts with
    const uint64_t len = 22;
    o.write((const char*)&len, 8);
    o.write("serialization::archive", 22);
    const uint8_t tail[15] = {9, 0, 4, 8, 4, 8, 1, 0, 0, 0, 0, 0, 0, 0, 0};
    o.write((const char*)tail, 15);
    auto mat = [&](int32_t c, int32_t r, uint64_t esz, uint64_t et, const void* data) {
        o.write((const char*)&c, 4); o.write((const char*)&r, 4);
        o.write((const char*)&esz, 8); o.write((const char*)&et, 8);
        if (data) o.write((const char*)data, (std::streamsize)((size_t)c * r * esz));
    };
    for (int s = 0; s < 8; ++s) {
        mat(f->cols, f->rows, 3, 16, &bgr[s * npx * 3]);   // CV_8UC3
        mat(f->cols, f->rows, 2, 2, &depth[s * npx]);      // CV_16UC1
    }
    const std::vector<uint8_t> dig = timestamp_to_digits(f->timestamp);
    if (dig.empty()) mat(0, 0, 0, 0, nullptr);
    else mat((int32_t)dig.size(), 1, 1, 0, dig.data());   // CV_8U
    o.close();
    if (!o) { r360_set_error("write failed: %s", path); return -1; }
    return 0;
}

// ------------------------------------------------------------------ Frame360::sphereCloud
// buildSphereCloud (Frame360.h:467-519): the per-sensor organized clouds (downsampled and
// bilaterally filtered, as the plane stage holds them in HBM) transformed by Rt_[sensor] with
// pcl::transformPointCloud, concatenated sensor by sensor, then height = cloud_[0]->width and
// width = 8 * cloud_[0]->height.
#pragma clang fp contract(off)
static int sphere_cloud_from_device(r360_frame* f, SphereCloudHost& sc) {
    const PlaneBufs& P = f->pl;
    planes_join(f);   // a plane queue builds the cloud on its own stream: its frame's assembly has waited for it
    const size_t per = (size_t)P.w * P.h, n = 8 * per;
    std::vector<float4> xyz(n);
    std::vector<uchar4> rgb(n);
    R360_HIP(hipMemcpyAsync(xyz.data(), P.cloud, sizeof(float4) * n, hipMemcpyDeviceToHost, f->ctx->stream));
    R360_HIP(hipMemcpyAsync(rgb.data(), P.rgb, sizeof(uchar4) * n, hipMemcpyDeviceToHost, f->ctx->stream));
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    sc.width = 8 * P.h;
    sc.height = P.w;
    sc.xyz.resize(3 * n);
    sc.rgba.resize(n);
    for (int s = 0; s < 8; ++s) {
        const float* m = f->calib->rt[s];  // column-major: m(r, c) = m[c * 4 + r]
        for (size_t i = s * per; i < (s + 1) * per; ++i) {
            const float x = xyz[i].x, y = xyz[i].y, z = xyz[i].z;
            float* o = &sc.xyz[3 * i];
            if (!std::isfinite(x) || !std::isfinite(y) || !std::isfinite(z)) {
                // transformPointCloud leaves non-finite points of a non-dense cloud as they were
                o[0] = x; o[1] = y; o[2] = z;
            } else {
                // pcl/common/impl/transforms.hpp: m(k,0)*x + m(k,1)*y + m(k,2)*z + m(k,3), float
                for (int k = 0; k < 3; ++k) {
                    float a = m[k] * x;
                    a = a + m[4 + k] * y;
                    a = a + m[8 + k] * z;
                    o[k] = a + m[12 + k];
                }
            }
            const uchar4 c = rgb[i];  // {r, g, b, a}
            sc.rgba[i] = uint32_t(c.z) | uint32_t(c.y) << 8 | uint32_t(c.x) << 16 | uint32_t(c.w) << 24;
        }
    }
    return 0;
}
#pragma clang fp contract(on)

static int sphere_cloud(r360_frame* f, const SphereCloudHost** out, SphereCloudHost& tmp) {
    if (f->sphere_cloud) { *out = f->sphere_cloud; return 0; }
    if (!(f->built & R360_BUILD_CLOUD)) {
        r360_set_error("no sphere cloud: build the frame with R360_BUILD_CLOUD or load one (loadCloud)");
        return -2;
    }
    if (int rc = sphere_cloud_from_device(f, tmp)) return rc;
    *out = &tmp;
    return 0;
}

extern "C" int r360_frame_get_sphere_cloud(r360_frame* f, float* xyz, uint32_t* rgba, size_t cap, int* width,
                                           int* height) {
    if (!f) { r360_set_error("null frame"); return -2; }
    SphereCloudHost tmp;
    const SphereCloudHost* sc = nullptr;
    if (int rc = sphere_cloud(f, &sc, tmp)) return rc;
    if (width) *width = sc->width;
    if (height) *height = sc->height;
    const size_t n = std::min(cap, sc->rgba.size());
    if (xyz) memcpy(xyz, sc->xyz.data(), sizeof(float) * 3 * n);
    if (rgba) memcpy(rgba, sc->rgba.data(), sizeof(uint32_t) * n);
    return 0;
}

// ------------------------------------------------------------------ PCD (PCL .pcd v0.7)
// pcl::io::savePCDFile (Frame360.h:326) and PCDReader::read (Frame360.h:190-192) for
// pcl::PointXYZRGBA, restated from PCL 1.7's pcd_io.cpp (third-party, not vendored in the
// reference): header from PCDWriter::generateHeader, DATA ascii (writeASCII: precision 8,
// "nan", fields space-separated), binary (packed fields per point) and binary_compressed
// (fields de-interleaved, then LZF).
namespace {

// LZF (liblzf 3.x, the codec PCL vendors as pcl/common/src/lzf.cpp): control byte < 32 = literal
// run of ctrl+1 bytes; else a back-reference of length (ctrl>>5)+2 (+ next byte when 7) at
// offset ((ctrl&31)<<8 | next) + 1.  The compressor is a greedy one-entry-hash matcher; any
// valid stream decodes identically, the compressed bytes need not match liblzf's.
std::vector<uint8_t> lzf_compress(const uint8_t* in, size_t n) {
    std::vector<uint8_t> out;
    out.reserve(n + n / 32 + 16);
    std::vector<int64_t> table(1 << 14, -1);
    size_t lit_start = 0, i = 0;
    auto flush_literals = [&](size_t end) {
        while (lit_start < end) {
            const size_t run = std::min<size_t>(32, end - lit_start);
            out.push_back(uint8_t(run - 1));
            out.insert(out.end(), in + lit_start, in + lit_start + run);
            lit_start += run;
        }
    };
    while (i + 2 < n) {
        const uint32_t h = ((uint32_t(in[i]) << 16 | uint32_t(in[i + 1]) << 8 | in[i + 2]) * 2654435761u) >> 18;
        const int64_t ref = table[h];
        table[h] = (int64_t)i;
        if (ref >= 0 && i - (size_t)ref <= 8192 && in[ref] == in[i] && in[ref + 1] == in[i + 1] && in[ref + 2] == in[i + 2]) {
            size_t len = 3;
            const size_t maxlen = std::min<size_t>(264, n - i);
            while (len < maxlen && in[ref + len] == in[i + len]) ++len;
            flush_literals(i);
            const size_t off = i - (size_t)ref - 1, l = len - 2;
            if (l < 7) {
                out.push_back(uint8_t((off >> 8) + (l << 5)));
            } else {
                out.push_back(uint8_t((off >> 8) + (7 << 5)));
                out.push_back(uint8_t(l - 7));
            }
            out.push_back(uint8_t(off & 255));
            i += len;
            lit_start = i;
        } else {
            ++i;
        }
    }
    flush_literals(n);
    return out;
}

bool lzf_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_n) {
    size_t ip = 0, op = 0;
    while (ip < n) {
        const unsigned c = in[ip++];
        if (c < 32) {
            const size_t run = c + 1;
            if (ip + run > n || op + run > out_n) return false;
            memcpy(out + op, in + ip, run);
            ip += run; op += run;
        } else {
            size_t len = c >> 5;
            if (len == 7) { if (ip >= n) return false; len += in[ip++]; }
            if (ip >= n) return false;
            const size_t back = ((size_t)(c & 31) << 8) + in[ip++] + 1;
            len += 2;
            if (back > op || op + len > out_n) return false;
            for (size_t k = 0; k < len; ++k, ++op) out[op] = out[op - back];
        }
    }
    return op == out_n;
}

struct PcdField { std::string name; int size = 4, count = 1; char type = 'F'; };

// one field value -> double (for x/y/z) or raw uint32 bits (for rgb/rgba)
double field_value(const uint8_t* p, const PcdField& F) {
    switch (F.type) {
        case 'F': { if (F.size == 8) { double v; memcpy(&v, p, 8); return v; } float v; memcpy(&v, p, 4); return v; }
        case 'U': { if (F.size == 1) return *p; if (F.size == 2) { uint16_t v; memcpy(&v, p, 2); return v; }
                    if (F.size == 8) { uint64_t v; memcpy(&v, p, 8); return (double)v; }
                    uint32_t v; memcpy(&v, p, 4); return v; }
        default:  { if (F.size == 1) return (int8_t)*p; if (F.size == 2) { int16_t v; memcpy(&v, p, 2); return v; }
                    if (F.size == 8) { int64_t v; memcpy(&v, p, 8); return (double)v; }
                    int32_t v; memcpy(&v, p, 4); return v; }
    }
}

}  // namespace

// Writes width*height points: xyz [n][3] float, rgba [n] packed as PointXYZRGBA (may be NULL = 0).
// mode 0 = ascii (savePCDFile's default, the reference's call), 1 = binary, 2 = binary_compressed.
extern "C" int r360_pcd_write(const char* path, const float* xyz, const uint32_t* rgba, int width, int height,
                              int mode) {
    if (!path || !xyz || width < 0 || height < 0 || mode < 0 || mode > 2) { r360_set_error("bad argument"); return -2; }
    const size_t n = (size_t)width * height;
    std::ofstream o(path, std::ios::binary);
    if (!o) { r360_set_error("cannot create %s", path); return -1; }
    o << "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgba\nSIZE 4 4 4 4\n"
         "TYPE F F F U\nCOUNT 1 1 1 1\nWIDTH " << width << "\nHEIGHT " << height << "\n"
         "VIEWPOINT 0 0 0 1 0 0 0\nPOINTS " << n << "\n";
    if (mode == 0) {
        o << "DATA ascii\n";
        std::string line;
        char buf[32];
        for (size_t i = 0; i < n; ++i) {
            line.clear();
            for (int k = 0; k < 3; ++k) {
                const float v = xyz[3 * i + k];
                if (std::isnan(v)) line += "nan";
                else { snprintf(buf, sizeof buf, "%.8g", (double)v); line += buf; }
                line += ' ';
            }
            snprintf(buf, sizeof buf, "%u\n", rgba ? rgba[i] : 0u);
            line += buf;
            o.write(line.data(), (std::streamsize)line.size());
        }
    } else if (mode == 1) {
        o << "DATA binary\n";
        std::vector<uint8_t> rec(16 * n);
        for (size_t i = 0; i < n; ++i) {
            memcpy(&rec[16 * i], &xyz[3 * i], 12);
            const uint32_t c = rgba ? rgba[i] : 0u;
            memcpy(&rec[16 * i + 12], &c, 4);
        }
        o.write((const char*)rec.data(), (std::streamsize)rec.size());
    } else {
        o << "DATA binary_compressed\n";
        std::vector<uint8_t> soa(16 * n);
        for (size_t i = 0; i < n; ++i) {
            for (int k = 0; k < 3; ++k) memcpy(&soa[4 * (k * n + i)], &xyz[3 * i + k], 4);
            const uint32_t c = rgba ? rgba[i] : 0u;
            memcpy(&soa[4 * (3 * n + i)], &c, 4);
        }
        const std::vector<uint8_t> z = lzf_compress(soa.data(), soa.size());
        const uint32_t zs = (uint32_t)z.size(), us = (uint32_t)soa.size();
        o.write((const char*)&zs, 4);
        o.write((const char*)&us, 4);
        o.write((const char*)z.data(), (std::streamsize)z.size());
    }
    o.close();
    if (!o) { r360_set_error("write failed: %s", path); return -1; }
    return 0;
}

// Reads a .pcd into xyz [cap][3] / rgba [cap] (either may be NULL; a cloud without an rgb/rgba
// field reads as 0).  *n = points in the file, *width / *height as in its header.
extern "C" int r360_pcd_read(const char* path, float* xyz, uint32_t* rgba, size_t cap, size_t* n_out, int* width,
                             int* height) {
    if (!path) { r360_set_error("null path"); return -2; }
    std::ifstream f(path, std::ios::binary);
    if (!f) { r360_set_error("cannot open %s", path); return -1; }
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<PcdField> F;
    long W = -1, H = 1, N = -1;
    std::string data;
    size_t off = 0;
    while (off < b.size() && data.empty()) {
        size_t e = off;
        while (e < b.size() && b[e] != '\n') ++e;
        std::string line((const char*)&b[off], e - off);
        off = e + 1;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty() || line[0] == '#') continue;
        std::istringstream ls(line);
        std::string key;
        ls >> key;
        if (key == "FIELDS" || key == "COLUMNS") { std::string s; while (ls >> s) { PcdField p; p.name = s; F.push_back(p); } }
        else if (key == "SIZE") { for (auto& p : F) ls >> p.size; }
        else if (key == "TYPE") { for (auto& p : F) ls >> p.type; }
        else if (key == "COUNT") { for (auto& p : F) ls >> p.count; }
        else if (key == "WIDTH") ls >> W;
        else if (key == "HEIGHT") ls >> H;
        else if (key == "POINTS") ls >> N;
        else if (key == "DATA") ls >> data;
    }
    if (F.empty() || W < 0 || data.empty()) { r360_set_error("%s: incomplete PCD header", path); return -1; }
    if (N < 0) N = W * H;
    if (N != W * H) { r360_set_error("%s: POINTS %ld != WIDTH*HEIGHT %ld", path, N, W * H); return -1; }
    int ix = -1, iy = -1, iz = -1, ic = -1;
    std::vector<size_t> foff(F.size());
    size_t rec = 0;
    for (size_t k = 0; k < F.size(); ++k) {
        const PcdField& p = F[k];
        if (!(p.size == 1 || p.size == 2 || p.size == 4 || p.size == 8) || p.count < 1 ||
            !(p.type == 'F' || p.type == 'U' || p.type == 'I')) {
            r360_set_error("%s: unsupported field %s", path, p.name.c_str());
            return -1;
        }
        foff[k] = rec;
        rec += (size_t)p.size * p.count;
        if (p.name == "x") ix = (int)k; else if (p.name == "y") iy = (int)k; else if (p.name == "z") iz = (int)k;
        else if (p.name == "rgba" || p.name == "rgb") ic = (int)k;
    }
    if (ix < 0 || iy < 0 || iz < 0) { r360_set_error("%s: no x/y/z fields", path); return -1; }
    const size_t n = (size_t)N;
    if (n_out) *n_out = n;
    if (width) *width = (int)W;
    if (height) *height = (int)H;
    const size_t m = std::min(cap, n);
    auto store = [&](size_t i, const double* v, uint32_t c) {
        if (i >= m) return;
        if (xyz) for (int k = 0; k < 3; ++k) xyz[3 * i + k] = (float)v[k];
        if (rgba) rgba[i] = c;
    };
    auto color_bits = [&](const uint8_t* p) -> uint32_t {
        if (ic < 0) return 0;
        uint32_t c = 0;
        memcpy(&c, p, std::min(4, F[ic].size));  // rgb is a float holding the packed bytes
        return c;
    };
    if (data == "ascii") {
        size_t i = 0;
        std::string text((const char*)b.data() + std::min(off, b.size()), b.size() - std::min(off, b.size()));
        std::istringstream ts(text);
        std::string tok;
        const size_t ntok = rec ? std::accumulate(F.begin(), F.end(), size_t(0), [](size_t a, const PcdField& p) { return a + p.count; }) : 0;
        std::vector<std::string> toks(ntok);
        for (; i < n; ++i) {
            for (size_t t = 0; t < ntok; ++t)
                if (!(ts >> toks[t])) { r360_set_error("%s: truncated ascii data at point %zu", path, i); return -1; }
            double v[3];
            uint32_t c = 0;
            size_t t = 0;
            for (size_t k = 0; k < F.size(); ++k) {
                const std::string& s = toks[t];
                if ((int)k == ix || (int)k == iy || (int)k == iz)
                    v[(int)k == ix ? 0 : (int)k == iy ? 1 : 2] = (s == "nan" || s == "NaN") ? NAN : strtod(s.c_str(), nullptr);
                else if ((int)k == ic) {
                    if (F[k].type == 'F') { const float fv = strtof(s.c_str(), nullptr); memcpy(&c, &fv, 4); }
                    else c = (uint32_t)strtoul(s.c_str(), nullptr, 10);
                }
                t += F[k].count;
            }
            store(i, v, c);
        }
    } else if (data == "binary" || data == "binary_compressed") {
        std::vector<uint8_t> soa;
        const uint8_t* base = nullptr;
        const bool compressed = data == "binary_compressed";
        if (compressed) {
            if (off + 8 > b.size()) { r360_set_error("%s: truncated", path); return -1; }
            uint32_t zs, us;
            memcpy(&zs, &b[off], 4); memcpy(&us, &b[off + 4], 4);
            if (off + 8 + zs > b.size() || us != rec * n) { r360_set_error("%s: bad compressed block", path); return -1; }
            soa.resize(us);
            if (!lzf_decompress(&b[off + 8], zs, soa.data(), us)) { r360_set_error("%s: LZF stream corrupt", path); return -1; }
            base = soa.data();
        } else {
            if (off + rec * n > b.size()) { r360_set_error("%s: truncated binary data", path); return -1; }
            base = &b[off];
        }
        // binary_compressed stores each field for all points contiguously (field-major)
        auto at = [&](size_t i, int k) -> const uint8_t* {
            const size_t fs = (size_t)F[k].size * F[k].count;
            return compressed ? base + foff[k] * n + i * fs : base + i * rec + foff[k];
        };
        for (size_t i = 0; i < m; ++i) {
            const double v[3] = {field_value(at(i, ix), F[ix]), field_value(at(i, iy), F[iy]), field_value(at(i, iz), F[iz])};
            store(i, v, ic >= 0 ? color_bits(at(i, ic)) : 0u);
        }
    } else {
        r360_set_error("%s: unknown DATA %s", path, data.c_str());
        return -1;
    }
    return 0;
}

extern "C" int r360_frame_save_cloud(r360_frame* f, const char* path, int mode) {
    if (!f || !path) { r360_set_error("null arg"); return -2; }
    SphereCloudHost tmp;
    const SphereCloudHost* sc = nullptr;
    if (int rc = sphere_cloud(f, &sc, tmp)) return rc;
    return r360_pcd_write(path, sc->xyz.data(), sc->rgba.data(), sc->width, sc->height, mode);
}

extern "C" int r360_frame_load_cloud(r360_frame* f, const char* path) {
    if (!f || !path) { r360_set_error("null arg"); return -2; }
    size_t n = 0;
    int w = 0, h = 0;
    if (int rc = r360_pcd_read(path, nullptr, nullptr, 0, &n, &w, &h)) return rc;
    auto* sc = new SphereCloudHost;
    sc->width = w; sc->height = h;
    sc->xyz.resize(3 * n);
    sc->rgba.resize(n);
    if (int rc = r360_pcd_read(path, sc->xyz.data(), sc->rgba.data(), n, &n, &w, &h)) { delete sc; return rc; }
    delete f->sphere_cloud;
    f->sphere_cloud = sc;
    return 0;
}
