// oracle_la.h — ORACLE (test infrastructure only): the small dense linear algebra of the GN / LM
// steps, shared by the spherical (photo_icp_oracle.cpp) and pinhole (pinhole_oracle.cpp) paths.
#pragma once
#include <cmath>
#include <cstring>
#include <utility>

// ---------------------------------------------------------------------------
// small dense linear algebra for the GN step
// ---------------------------------------------------------------------------
static inline void matmul4f(const float A[16], const float B[16], float C[16]) {  // col-major, float like Eigen
    float out[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            float s = A[r] * B[c * 4];
            for (int k = 1; k < 4; ++k) s += A[k * 4 + r] * B[c * 4 + k];
            out[c * 4 + r] = s;
        }
    memcpy(C, out, sizeof(out));
}

// Eigen FullPivLU::rank() with the default threshold (eps * diagonalSize) (:4682)
static inline int rank6(const double M_in[36]) {
    double M[36]; memcpy(M, M_in, sizeof(M));
    double maxpiv = 0; int rk = 0;
    double piv[6];
    for (int k = 0; k < 6; ++k) {
        int br = k, bc = k; double bv = -1;
        for (int r = k; r < 6; ++r)
            for (int c = k; c < 6; ++c)
                if (std::fabs(M[r * 6 + c]) > bv) { bv = std::fabs(M[r * 6 + c]); br = r; bc = c; }
        for (int c = 0; c < 6; ++c) std::swap(M[k * 6 + c], M[br * 6 + c]);
        for (int r = 0; r < 6; ++r) std::swap(M[r * 6 + k], M[r * 6 + bc]);
        piv[k] = M[k * 6 + k];
        if (piv[k] != 0)
            for (int r = k + 1; r < 6; ++r) {
                double f = M[r * 6 + k] / piv[k];
                for (int c = k; c < 6; ++c) M[r * 6 + c] -= f * M[k * 6 + c];
            }
    }
    maxpiv = std::fabs(piv[0]);
    const double thr = 1.1920928955078125e-07 * 6;
    for (int k = 0; k < 6; ++k) if (std::fabs(piv[k]) > thr * maxpiv) ++rk;
    return rk;
}

// x = -H^-1 g by Gaussian elimination with partial pivoting (double)
static inline bool solve6(const double H_in[36], const double g[6], double x[6]) {
    double A[6][7];
    for (int r = 0; r < 6; ++r) { for (int c = 0; c < 6; ++c) A[r][c] = H_in[r * 6 + c]; A[r][6] = -g[r]; }
    for (int k = 0; k < 6; ++k) {
        int p = k;
        for (int r = k + 1; r < 6; ++r) if (std::fabs(A[r][k]) > std::fabs(A[p][k])) p = r;
        if (A[p][k] == 0) return false;
        for (int c = 0; c < 7; ++c) std::swap(A[k][c], A[p][c]);
        for (int r = k + 1; r < 6; ++r) {
            double f = A[r][k] / A[k][k];
            for (int c = k; c < 7; ++c) A[r][c] -= f * A[k][c];
        }
    }
    for (int r = 5; r >= 0; --r) {
        double s = A[r][6];
        for (int c = r + 1; c < 6; ++c) s -= A[r][c] * x[c];
        x[r] = s / A[r][r];
    }
    return true;
}

