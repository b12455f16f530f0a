// Exhaustive check of csrc/tsdf.hip deint_channel (the batch pass's de-integrate colour) against the
// reference expression u8(clamp(roundf((oc w - cu) / (w - 1)), 0, 254.5)) (CUDASceneRepHashSDF.cu:420-521).
// gcc -O2 -fopenmp -ffp-contract=off tools/check_deint_color.c -lm && ./a.out   (~30 s on 8 cores)
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static float ref(int oc, int cu, float w) {
    volatile float a = (float)oc * w;      // oc0 * w0
    volatile float b = (float)cu * 1.0f;   // cu0 * wUpd
    volatile float x = a - b;
    volatile float d = w - 1.0f;
    volatile float q = x / d;
    float r = roundf(q);
    r = fmaxf(0.0f, fminf(r, 254.5f));
    return (float)(uint8_t)r;
}
static float fast(int oc, int cu, float w, int rcpv) {
    float d = w - 1.0f;
    float den = 2.0f * d;
    float rc = 1.0f / den;
    if (rcpv == 1) rc = nextafterf(rc, INFINITY);
    if (rcpv == 2) rc = nextafterf(rc, 0.0f);
    if (d > 510.0f) rc = 0.0f;
    float o = (float)oc, c = (float)cu;
    float delta = o - c;
    float num = fmaf(delta, 2.0f, d);
    float q = num * rc;
    float k = floorf(q + 5e-4f);
    float r = o + k;
    r = fmaxf(0.0f, fminf(r, 254.0f));  // med3
    return r;
}
int main(void) {
    long bad = 0, n = 0;
    #pragma omp parallel for reduction(+:bad,n) schedule(dynamic, 64)
    for (int wi = 2; wi <= 140000; wi++) {
        float w = (float)wi;
        for (int oc = 0; oc < 256; oc++)
            for (int cu = 0; cu < 256; cu++) {
                float r0 = ref(oc, cu, w);
                for (int v = 0; v < (wi <= 600 ? 3 : 1); v++) {
                    n++;
                    if (fast(oc, cu, w, v) != r0) { bad++; if (bad < 10) printf("bad w=%d oc=%d cu=%d v=%d ref=%g fast=%g\n", wi, oc, cu, v, r0, fast(oc,cu,w,v)); }
                }
            }
    }
    // large weights up to weightMax, sampled
    for (long wi = 140000; wi <= 99999999; wi = wi * 1.01 + 1) {
        float w = (float)wi;
        for (int oc = 0; oc < 256; oc += 3)
            for (int cu = 0; cu < 256; cu += 5) { n++; if (fast(oc, cu, w, 0) != ref(oc, cu, w)) { bad++; if (bad < 20) printf("bad large w=%ld\n", wi); } }
    }
    printf("checked %ld, mismatches %ld\n", n, bad);
    return bad != 0;
}
