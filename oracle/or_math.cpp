// oracle/or_math.cpp — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
#include "or_math.h"
#include "oracle.h"
#include <algorithm>
#include <cstring>

namespace orc {

// float4x4::getInverse, Source/SiftGPU/cuda_SimpleMatrixUtil.h:980-1090, term for term.
m4 inverse(const m4& m) {
    const float* e = m.e;
    float inv[16];
    inv[0] = e[5] * e[10] * e[15] - e[5] * e[11] * e[14] - e[9] * e[6] * e[15] + e[9] * e[7] * e[14] + e[13] * e[6] * e[11] - e[13] * e[7] * e[10];
    inv[4] = -e[4] * e[10] * e[15] + e[4] * e[11] * e[14] + e[8] * e[6] * e[15] - e[8] * e[7] * e[14] - e[12] * e[6] * e[11] + e[12] * e[7] * e[10];
    inv[8] = e[4] * e[9] * e[15] - e[4] * e[11] * e[13] - e[8] * e[5] * e[15] + e[8] * e[7] * e[13] + e[12] * e[5] * e[11] - e[12] * e[7] * e[9];
    inv[12] = -e[4] * e[9] * e[14] + e[4] * e[10] * e[13] + e[8] * e[5] * e[14] - e[8] * e[6] * e[13] - e[12] * e[5] * e[10] + e[12] * e[6] * e[9];
    inv[1] = -e[1] * e[10] * e[15] + e[1] * e[11] * e[14] + e[9] * e[2] * e[15] - e[9] * e[3] * e[14] - e[13] * e[2] * e[11] + e[13] * e[3] * e[10];
    inv[5] = e[0] * e[10] * e[15] - e[0] * e[11] * e[14] - e[8] * e[2] * e[15] + e[8] * e[3] * e[14] + e[12] * e[2] * e[11] - e[12] * e[3] * e[10];
    inv[9] = -e[0] * e[9] * e[15] + e[0] * e[11] * e[13] + e[8] * e[1] * e[15] - e[8] * e[3] * e[13] - e[12] * e[1] * e[11] + e[12] * e[3] * e[9];
    inv[13] = e[0] * e[9] * e[14] - e[0] * e[10] * e[13] - e[8] * e[1] * e[14] + e[8] * e[2] * e[13] + e[12] * e[1] * e[10] - e[12] * e[2] * e[9];
    inv[2] = e[1] * e[6] * e[15] - e[1] * e[7] * e[14] - e[5] * e[2] * e[15] + e[5] * e[3] * e[14] + e[13] * e[2] * e[7] - e[13] * e[3] * e[6];
    inv[6] = -e[0] * e[6] * e[15] + e[0] * e[7] * e[14] + e[4] * e[2] * e[15] - e[4] * e[3] * e[14] - e[12] * e[2] * e[7] + e[12] * e[3] * e[6];
    inv[10] = e[0] * e[5] * e[15] - e[0] * e[7] * e[13] - e[4] * e[1] * e[15] + e[4] * e[3] * e[13] + e[12] * e[1] * e[7] - e[12] * e[3] * e[5];
    inv[14] = -e[0] * e[5] * e[14] + e[0] * e[6] * e[13] + e[4] * e[1] * e[14] - e[4] * e[2] * e[13] - e[12] * e[1] * e[6] + e[12] * e[2] * e[5];
    inv[3] = -e[1] * e[6] * e[11] + e[1] * e[7] * e[10] + e[5] * e[2] * e[11] - e[5] * e[3] * e[10] - e[9] * e[2] * e[7] + e[9] * e[3] * e[6];
    inv[7] = e[0] * e[6] * e[11] - e[0] * e[7] * e[10] - e[4] * e[2] * e[11] + e[4] * e[3] * e[10] + e[8] * e[2] * e[7] - e[8] * e[3] * e[6];
    inv[11] = -e[0] * e[5] * e[11] + e[0] * e[7] * e[9] + e[4] * e[1] * e[11] - e[4] * e[3] * e[9] - e[8] * e[1] * e[7] + e[8] * e[3] * e[5];
    inv[15] = e[0] * e[5] * e[10] - e[0] * e[6] * e[9] - e[4] * e[1] * e[10] + e[4] * e[2] * e[9] + e[8] * e[1] * e[6] - e[8] * e[2] * e[5];
    float det = e[0] * inv[0] + e[1] * inv[4] + e[2] * inv[8] + e[3] * inv[12];
    float detr = 1.0f / det;
    m4 r;
    for (int i = 0; i < 16; i++) r.e[i] = inv[i] * detr;
    return r;
}

}  // namespace orc

extern "C" void or_matrix_inverse(const float M[16], float out[16]) {
    orc::m4 m;
    std::memcpy(m.e, M, 64);
    orc::m4 r = orc::inverse(m);
    std::memcpy(out, r.e, 64);
}

// Host memory bandwidth probe for bench.py's cpu_baseline (SURVEY.md §8(d) asks for the host's
// achieved memory GB/s next to the CPU timing): an OpenMP copy of `bytes` bytes, best of `reps`,
// counted as read + write bytes. Returns GB/s and the thread count used.
#include <chrono>
#include <omp.h>
extern "C" double or_host_membw(size_t bytes, int reps, int* threadsOut) {
    const size_t n = bytes / sizeof(double);
    double* a = new double[n];
    double* b = new double[n];
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) { a[i] = (double)i; b[i] = 0.0; }
    double best = 0.0;
    for (int r = 0; r < reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < n; i++) b[i] = a[i];
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = std::max(best, 2.0 * (double)(n * sizeof(double)) / s / 1e9);
    }
    if (threadsOut) *threadsOut = omp_get_max_threads();
    volatile double sink = b[n / 2];
    (void)sink;
    delete[] a;
    delete[] b;
    return best;
}

// The oracle's OpenMP thread count, set explicitly by bench.py's cpu_baseline (returns the count in
// effect afterwards).
extern "C" int or_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
}
