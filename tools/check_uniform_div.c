// Check of csrc/tsdf.hip div_by_uniform: a / b as two residual corrections of a * RN(1/b), against the
// IEEE quotient, for the divisor range the host admits ([2^-20, 2^20]) and |a| <= 2^100 (the range the
// voxel-coordinate guard admits; the depth-to-camera numerators are pixel offsets, far inside it).
// Bit-identical for 2^-100 <= |a| <= 2^100 and a = 0; below 2^-100 (residuals underflow) the result is
// checked to stay a finite number of |value| < 2^-60 with a's sign, which world_to_vvox's
// f2i(p + sgn(p) 0.5) maps to 0 exactly as it does the IEEE quotient.
// gcc -O2 -fopenmp -ffp-contract=off -mfma tools/check_uniform_div.c -lm && ./a.out   (~20 s on 8 cores)
// Exit status 0 = no disagreement. tests/test_oracle_tsdf.py runs a reduced sample (argument 13).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float fast(float a, float b, float rb) {
    const float q0 = a * rb;
    const float q1 = fmaf(fmaf(-b, q0, a), rb, q0);
    return fmaf(fmaf(-b, q1, a), rb, q1);
}
static uint64_t rng(uint64_t* s) {  // splitmix64
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static float from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
// a random float with |x| in [2^elo, 2^ehi), random sign and mantissa
static float rand_float(uint64_t* s, int elo, int ehi) {
    const uint64_t r = rng(s);
    const int e = elo + (int)(r % (uint64_t)(ehi - elo));
    const uint32_t m = (uint32_t)(r >> 20) & 0x7FFFFF;
    const uint32_t sg = (uint32_t)(r >> 63) << 31;
    return from_bits(sg | ((uint32_t)(e + 127) << 23) | m);
}

int main(int argc, char** argv) {
    // divisors: the scene / camera values the tests and bench use, then random ones over the range
    const float fixed[] = {0.004f, 0.005f, 0.01f, 0.02f, 0.04f, 0.05f, 0.06f, 0.1f, 1.0f / 3.0f,
                           525.0f, 577.871f, 580.8f, 583.0f, 50.0f, 100.0f, 0x1p-20f, 0x1.fffffep19f};
    const int nFixed = (int)(sizeof fixed / sizeof fixed[0]);
    const int nRandB = 4096;
    const long perB = 1L << (argc > 1 ? atoi(argv[1]) : 21);  // numerators per divisor (the test runs 2^13)
    long bad = 0, total = 0;
#pragma omp parallel for reduction(+ : bad, total) schedule(dynamic)
    for (int bi = 0; bi < nFixed + nRandB; bi++) {
        uint64_t s = 0x1234567ull + (uint64_t)bi * 7919u;
        float b = bi < nFixed ? fixed[bi] : fabsf(rand_float(&s, -20, 20));
        const float rb = 1.0f / b;
        for (long i = 0; i < perB; i++) {
            float a;
            const int kind = (int)(i & 7);
            if (kind == 4 || kind == 5) {  // below 2^-100, denormals included
                a = kind == 4 ? rand_float(&s, -126, -100) : from_bits((uint32_t)(rng(&s) & 0x807FFFFFu));
                const float f = fast(a, b, rb);
                total++;
                if (!(fabsf(f) < 0x1p-60f) || (a != 0.0f && f != 0.0f && signbit(a) != signbit(f))) {
#pragma omp critical
                    printf("tiny a=%a b=%a fast=%a\n", a, b, f);
                    bad++;
                }
                continue;
            }
            if (kind == 0 || kind >= 6) a = rand_float(&s, -100, 100);  // anything the guard admits
            else if (kind == 1) a = rand_float(&s, -8, 8);            // metres and voxel coordinates
            else if (kind == 2) a = (float)(int)(rng(&s) % 2048) - 1023.5f + (float)(int)(rng(&s) % 3) * 0.25f;  // pixel offsets
            else {  // quotients near a half-integer (the f2i(p +- 0.5) steps of world_to_vvox)
                const float t = (float)((int)(rng(&s) % 20001) - 10000) + 0.5f;
                a = t * b;
                const int nudge = (int)(rng(&s) % 5) - 2;
                for (int k = 0; k < nudge; k++) a = nextafterf(a, INFINITY);
                for (int k = 0; k > nudge; k--) a = nextafterf(a, -INFINITY);
            }
            const float q = a / b, f = fast(a, b, rb);
            total++;
            if (bits(q) != bits(f) && !(q == 0.0f && f == 0.0f)) {
#pragma omp critical
                printf("a=%a b=%a ieee=%a fast=%a\n", a, b, q, f);
                bad++;
            }
        }
    }
    printf("%ld cases, %ld disagreements (signed zeros compared equal; tiny numerators checked for range and sign)\n", total, bad);
    return bad != 0;
}
