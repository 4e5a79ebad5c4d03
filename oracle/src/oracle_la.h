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

// Eigen FullPivLU<Matrix<float,6,6>>::rank() with the default threshold (:4682, :4345, RegisterRGBD360.h:443):
// the reference's matrices are float, so the decomposition runs in float.  Per step the biggest |.| of the
// remaining corner is found in Eigen's visiting order (column-major, first strictly greater, starting at the
// corner's first coefficient); m_maxpivot is the largest of those maxima; rank = #pivots with
// |pivot| > |maxpivot| * (FLT_EPSILON * 6).  M_in: row-major, values already rounded to float.
static inline int rank6(const double M_in[36]) {
    float M[36];
    for (int k = 0; k < 36; ++k) M[k] = (float)M_in[k];
    float maxpiv = 0.f, piv[6];
    int nz = 6;
    for (int k = 0; k < 6; ++k) {
        int br = k, bc = k;
        float bv = std::fabs(M[k * 6 + k]);
        for (int c = k; c < 6; ++c)
            for (int r = (c == k ? k + 1 : k); r < 6; ++r)
                if (std::fabs(M[r * 6 + c]) > bv) { bv = std::fabs(M[r * 6 + c]); br = r; bc = c; }
        if (bv == 0.f) { nz = k; break; }
        if (bv > maxpiv) maxpiv = bv;
        for (int c = 0; c < 6; ++c) std::swap(M[k * 6 + c], M[br * 6 + c]);
        for (int r = 0; r < 6; ++r) std::swap(M[r * 6 + k], M[r * 6 + bc]);
        piv[k] = M[k * 6 + k];
        for (int r = k + 1; r < 6; ++r) M[r * 6 + k] = M[r * 6 + k] / piv[k];
        for (int r = k + 1; r < 6; ++r)
            for (int c = k + 1; c < 6; ++c) M[r * 6 + c] = M[r * 6 + c] - M[r * 6 + k] * M[k * 6 + c];
    }
    const float thr = maxpiv * (1.1920928955078125e-07f * 6.0f);
    int rk = 0;
    for (int k = 0; k < nz; ++k) if (std::fabs(piv[k]) > thr) ++rk;
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

