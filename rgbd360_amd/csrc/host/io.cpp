// io.cpp — Frame360 .bin archive reader (Frame360::loadFrame, include/Frame360.h:231-266).
// The file is a Boost binary_iarchive of 8 x {cv::Mat RGB CV_8UC3, cv::Mat depth CV_16UC1}
// followed by a timestamp mat; each mat is {int cols, int rows, size_t elem_size,
// size_t elem_type, bytes} (cvmat_serialization.h:39-55).  No Boost here: the 45-byte archive
// prologue is checked and skipped.
#include <cstring>
#include <fstream>
#include <vector>

#include "../r360_internal.h"

int parse_bin_file(const char* path, int rows, int cols, std::vector<uint8_t>& bgr, std::vector<uint16_t>& depth) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { r360_set_error("cannot open %s", path); return -1; }
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    static const char kTag[] = "serialization::archive";
    if (b.size() < 45 + 24 || memcmp(b.data() + 8, kTag, 22) != 0) {
        r360_set_error("%s: not a boost binary archive", path);
        return -1;
    }
    size_t off = 45;
    const size_t npx = (size_t)rows * cols;
    bgr.resize(8 * npx * 3);
    depth.resize(8 * npx);
    for (int s = 0; s < 8; ++s)
        for (int m = 0; m < 2; ++m) {
            if (off + 24 > b.size()) { r360_set_error("%s: truncated", path); return -1; }
            int32_t c, r; uint64_t esz, et;
            memcpy(&c, &b[off], 4); memcpy(&r, &b[off + 4], 4); memcpy(&esz, &b[off + 8], 8); memcpy(&et, &b[off + 16], 8);
            off += 24;
            if (r != rows || c != cols) {
                r360_set_error("%s: sensor %d is %dx%d, calib expects %dx%d", path, s, r, c, rows, cols);
                return -1;
            }
            const size_t n = (size_t)r * c * esz;
            if (off + n > b.size()) { r360_set_error("%s: truncated payload", path); return -1; }
            if (m == 0) {
                if (esz != 3 || et != 16) { r360_set_error("%s: RGB mat type %llu", path, (unsigned long long)et); return -1; }
                memcpy(&bgr[s * npx * 3], &b[off], n);
            } else {
                if (esz != 2 || et != 2) { r360_set_error("%s: depth mat type %llu", path, (unsigned long long)et); return -1; }
                memcpy(&depth[s * npx], &b[off], n);
            }
            off += n;
        }
    return 0;
}
