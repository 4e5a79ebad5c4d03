// synth.cpp — deterministic synthetic Frame360 generator: a procedural indoor
// room (8 x 6 x 3 m, 4 walls + floor + ceiling + 6 boxes) rendered by the 8 rig cameras with the
// rig's own extrinsics and the generalised pinhole (f = 525*cols/640).  Vertical axis = x, as in
// the rig/sphere convention of the reference (RegisterPhotoICP.h:4580-4582).  Depth is u16 mm with
// Kinect-like noise sigma = 1.2e-3 z^2 m and 12-35 % holes; colour is BGR u8 value-noise + checker
// texture attached to the surfaces, so frames of one scene are photometrically consistent.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../r360_internal.h"

namespace {

inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
inline uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return mix32(a * 0x9E3779B1U ^ mix32(b + 0x85EBCA77U * c)); }
inline float u01(uint32_t h) { return (h >> 8) * (1.0f / 16777216.0f); }

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ULL + 1) {}
    float next() {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        return (float)((s >> 40) * (1.0 / 16777216.0));
    }
};

struct Box { float lo[3], hi[3]; uint32_t id; };
struct Scene { Box room; std::vector<Box> boxes; uint32_t seed; };

Scene make_scene(uint32_t seed) {
    Scene sc;
    sc.seed = seed;
    sc.room = {{-1.3f, -4.0f, -3.0f}, {1.7f, 4.0f, 3.0f}, 0};
    Rng rng(seed);
    for (int i = 0; i < 6; ++i) {
        Box b;
        const float h = 0.4f + 1.2f * rng.next();
        const float sy = 0.4f + 0.8f * rng.next(), sz = 0.4f + 0.8f * rng.next();
        const int side = i % 4;
        float cy, cz;
        if (side == 0) { cy = -3.45f; cz = -2.4f + 4.8f * rng.next(); }
        else if (side == 1) { cy = 3.45f; cz = -2.4f + 4.8f * rng.next(); }
        else if (side == 2) { cz = -2.55f; cy = -3.2f + 6.4f * rng.next(); }
        else { cz = 2.55f; cy = -3.2f + 6.4f * rng.next(); }
        const bool hanging = (i == 4);
        b.lo[0] = hanging ? 1.7f - 0.5f : -1.3f;
        b.hi[0] = hanging ? 1.7f : -1.3f + h;
        b.lo[1] = cy - sy / 2; b.hi[1] = cy + sy / 2;
        b.lo[2] = cz - sz / 2; b.hi[2] = cz + sz / 2;
        b.id = 7 + i;
        sc.boxes.push_back(b);
    }
    return sc;
}

inline float smooth(float t) { return t * t * (3 - 2 * t); }
float vnoise(float x, float y, uint32_t salt) {
    const float fx = std::floor(x), fy = std::floor(y);
    const int ix = (int)fx, iy = (int)fy;
    const float tx = smooth(x - fx), ty = smooth(y - fy);
    const float a = u01(hash3(ix, iy, salt)), b = u01(hash3(ix + 1, iy, salt));
    const float c = u01(hash3(ix, iy + 1, salt)), d = u01(hash3(ix + 1, iy + 1, salt));
    return (a + (b - a) * tx) + ((c + (d - c) * tx) - (a + (b - a) * tx)) * ty;
}

// Surface texture: value-noise fBm + 0.5 m checker on the two in-plane coordinates.
void shade(uint32_t sid, int axis, const float p[3], uint8_t bgr[3]) {
    const int a1 = (axis + 1) % 3, a2 = (axis + 2) % 3;
    const float u = p[a1], v = p[a2];
    float n = 0.f, amp = 0.5f, fr = 1.7f;
    for (int o = 0; o < 5; ++o) {
        n += amp * vnoise(u * fr + 13.1f * o, v * fr - 7.3f * o, sid * 31u + o);
        amp *= 0.5f; fr *= 2.13f;
    }
    const int chk = ((int)std::floor(u * 2.f) + (int)std::floor(v * 2.f)) & 1;
    const float m = (0.45f + 1.1f * n) * (chk ? 0.8f : 1.0f) * (0.85f + 0.05f * axis);
    const uint32_t h = mix32(sid * 7919u + 17u);
    const float base[3] = {70.f + (h & 127), 70.f + ((h >> 8) & 127), 70.f + ((h >> 16) & 127)};
    for (int c = 0; c < 3; ++c) bgr[c] = (uint8_t)std::min(255.f, std::max(0.f, base[c] * m));
}

float gauss(uint32_t h1, uint32_t h2) {
    const float a = std::max(u01(h1), 1e-7f), b = u01(h2);
    return std::sqrt(-2.f * std::log(a)) * std::cos(6.2831853f * b);
}

}  // namespace

extern "C" int r360_synth_path_pose(uint32_t seed, int frame, float pose_out[16]) {
    (void)seed;
    const double w = 2 * R360_PI * frame / 256.0;
    const double y = 2.4 * std::sin(w), z = 1.6 * std::sin(2 * w);
    const double yaw = 0.35 * std::sin(w + 0.7);
    const double c = std::cos(yaw), s = std::sin(yaw);
    // rotation about the vertical x axis
    const float T[16] = {1, 0, 0, 0, 0, (float)c, (float)s, 0, 0, (float)-s, (float)c, 0, 0, (float)y, (float)z, 1};
    memcpy(pose_out, T, sizeof(T));
    return 0;
}

// rig_pose: column-major 4x4 rig -> room.  noise seed = scene seed ^ hash(rig pose bits) unless
// the caller varies the scene seed; depth noise uses (seed, sensor, pixel).
static int synth_impl(int rows, int cols, const float (*rt)[16], uint32_t seed, const float rig_pose[16],
                      uint8_t* bgr8, uint16_t* depth8) {
    const Scene sc = make_scene(seed >> 16);
    // cameraMatrix convention of r360_calib_create (CloudRGBD_Ext.h:97-102)
    const float f = 525 * (float)(cols / 640.0);
    const float cx = cols / 2 - 0.5, cy = rows / 2 - 0.5;
    uint32_t pose_h = seed;
    for (int i = 0; i < 16; ++i) { uint32_t b; memcpy(&b, &rig_pose[i], 4); pose_h = mix32(pose_h ^ b); }
    const float* P = rig_pose;
#pragma omp parallel for schedule(dynamic, 4)
    for (int job = 0; job < 8 * rows; ++job) {
        const int k = job / rows, v = job % rows;
        const float* Rt = rt[k];
        for (int u = 0; u < cols; ++u) {
            const float dc[3] = {(u - cx) / f, (v - cy) / f, 1.f};
            float dr[3], orr[3], dw[3], ow[3];
            for (int r = 0; r < 3; ++r) {
                dr[r] = Rt[r] * dc[0] + Rt[4 + r] * dc[1] + Rt[8 + r] * dc[2];
                orr[r] = Rt[12 + r];
            }
            for (int r = 0; r < 3; ++r) {
                dw[r] = P[r] * dr[0] + P[4 + r] * dr[1] + P[8 + r] * dr[2];
                ow[r] = P[r] * orr[0] + P[4 + r] * orr[1] + P[8 + r] * orr[2] + P[12 + r];
            }
            // room interior
            float tbest = 1e30f; int axis = 0; uint32_t sid = 0;
            for (int a = 0; a < 3; ++a) {
                if (dw[a] > 1e-9f) { float t = (sc.room.hi[a] - ow[a]) / dw[a]; if (t < tbest) { tbest = t; axis = a; sid = 2 * a + 1; } }
                else if (dw[a] < -1e-9f) { float t = (sc.room.lo[a] - ow[a]) / dw[a]; if (t < tbest) { tbest = t; axis = a; sid = 2 * a; } }
            }
            for (const Box& b : sc.boxes) {
                float t0 = -1e30f, t1 = 1e30f; int ax = 0;
                bool miss = false;
                for (int a = 0; a < 3 && !miss; ++a) {
                    if (std::fabs(dw[a]) < 1e-9f) { if (ow[a] < b.lo[a] || ow[a] > b.hi[a]) miss = true; continue; }
                    float ta = (b.lo[a] - ow[a]) / dw[a], tb = (b.hi[a] - ow[a]) / dw[a];
                    if (ta > tb) std::swap(ta, tb);
                    if (ta > t0) { t0 = ta; ax = a; }
                    if (tb < t1) t1 = tb;
                }
                if (!miss && t0 <= t1 && t0 > 1e-4f && t0 < tbest) { tbest = t0; axis = ax; sid = b.id; }
            }
            const float p[3] = {ow[0] + tbest * dw[0], ow[1] + tbest * dw[1], ow[2] + tbest * dw[2]};
            const size_t pi = ((size_t)k * rows + v) * cols + u;
            shade(sid, axis, p, &bgr8[pi * 3]);
            const uint32_t hp = hash3(pose_h, (uint32_t)k, (uint32_t)(v * cols + u));
            for (int c = 0; c < 3; ++c) {
                const int nz = (int)(mix32(hp + 11u * c) % 5u) - 2;
                bgr8[pi * 3 + c] = (uint8_t)std::min(255, std::max(0, bgr8[pi * 3 + c] + nz));
            }
            // depth = camera z (the ray parameter, since dc_z == 1)
            float z = tbest;
            const float nrm = std::sqrt(dw[0] * dw[0] + dw[1] * dw[1] + dw[2] * dw[2]);
            const float cosang = std::fabs(dw[axis]) / nrm;
            const float sigma = 1.2e-3f * z * z;
            z += sigma * gauss(mix32(hp ^ 0xA511E9B3U), mix32(hp ^ 0x63D83595U));
            bool hole = (z < 0.4f || z > 8.0f || cosang < 0.12f);
            hole |= vnoise(u / 37.f, v / 37.f, mix32(pose_h + k)) > 0.8f;
            hole |= u01(mix32(hp ^ 0x1234567U)) < 0.04f;
            depth8[pi] = hole ? 0 : (uint16_t)std::lrint(z * 1000.f);
        }
    }
    return 0;
}

extern "C" int r360_synth_frame(const r360_calib* calib, uint32_t seed, const float rig_pose[16], uint8_t* bgr8,
                                uint16_t* depth8) {
    if (!calib || !rig_pose || !bgr8 || !depth8) { r360_set_error("null arg"); return -2; }
    return synth_impl(calib->rows, calib->cols, calib->rt, seed, rig_pose, bgr8, depth8);
}

extern "C" int r360_synth_frame_rt(int rows, int cols, const float* rt8, uint32_t seed, const float rig_pose[16],
                                   uint8_t* bgr8, uint16_t* depth8) {
    if (!rt8 || !rig_pose || !bgr8 || !depth8 || rows <= 0 || cols <= 0) { r360_set_error("null arg"); return -2; }
    float rt[8][16];
    memcpy(rt, rt8, sizeof(rt));
    return synth_impl(rows, cols, rt, seed, rig_pose, bgr8, depth8);
}
