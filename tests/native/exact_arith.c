/* Host restatement of the device division formulas of custom-k8s-scheduler_amd/csrc/qs_device.hpp
 * (spec/semantics.md S10), checked against true integer / IEEE division.
 *   floor_div(n, y = RN(1/d)) == n / d           (LeastAllocated, normalize, weight combine)
 *   fraction(a, r, y = RN(1/a)) == min(RN(r/a),1) (BalancedAllocation, Markstein quotient)
 *   wide layout (memory in f64 bytes, 1 <= a <= 2^46):
 *   least_requested_w(a, reqd, RN(1/a)) == ((a - reqd) * 100) / a   (f64 quotient + one fma-exact
 *                                                                      integer correction)
 *   fraction_w(a, r, RN(1/a)) == min(RN(r/a), 1)                     (the same Markstein quotient)
 *   div_count(x, c) == RN(x / c), c in {3, 4}: BalancedAllocation's mean and variance over three or
 *   four resources (x >= 0 normal or zero; c = 4 an exact scaling, c = 3 Markstein's correction
 *   fma(fma(-q0, 3, x), RN(1/3), q0) of q0 = RN(x RN(1/3)))
 * Usage: exact_arith <mode> ; prints "ok <count>" or the first counter-example.  Test infra. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint32_t floor_div(uint32_t n, double y) { return (uint32_t)fma((double)n, y, 0x1p-30); }
static double fraction(int32_t a, int32_t r, double y) {
    double R = (double)r, A = (double)a;
    double q0 = R * y;
    double rem = fma(-q0, A, R);
    double q = fma(rem, y, q0);
    return r >= a ? 1.0 : q;
}
/* RN(1/a), 1 <= a < 2^24, as the scan kernel computes it (qs_device.hpp rcp_int): an f32 reciprocal
 * estimate (v_rcp_f32, within 1 ulp) refined by two fma Newton steps in f64.  y0 is passed in so the
 * check covers every estimate within +-2 f32 ulps of 1/a. */
static double rcp_int(int32_t a, float y0f) {
    const double A = (double)a;
    double y = (double)y0f;
    double e = fma(-A, y, 1.0);
    y = fma(y, e, y);
    e = fma(-A, y, 1.0);
    return fma(y, e, y);
}
static uint32_t least_requested_w(double a, double reqd, double ya) {
    const double rq = reqd < a ? reqd : a;
    const double n = (a - rq) * 100.0;
    double q = trunc(n * ya);
    const double r = fma(-q, a, n); /* exact: an integer below 2a in magnitude */
    q = r < 0.0 ? q - 1.0 : q;
    q = (r >= a && a > 0.0) ? q + 1.0 : q;
    return reqd > a ? 0u : (uint32_t)q;
}
static double fraction_w(double a, double r, double y) {
    const double q0 = r * y;
    const double rem = fma(-q0, a, r);
    const double q = fma(rem, y, q0);
    return r >= a ? 1.0 : q;
}
static uint64_t sm = 0x5EED1234ULL;
static uint64_t rnd(void) {
    uint64_t z = (sm += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static long long checks = 0;
static int check_la(int32_t a, int32_t r) { /* ((a - r) * 100) / a for 0 <= r <= a */
    double y = 1.0 / (double)a;
    uint32_t n = (uint32_t)(a - r) * 100u;
    checks++;
    if (floor_div(n, y) != n / (uint32_t)a) { printf("LA a=%d r=%d got %u want %u\n", a, r, floor_div(n, y), n / (uint32_t)a); return 1; }
    return 0;
}
static int check_frac(int32_t a, int32_t r) {
    double y = 1.0 / (double)a;
    volatile double want = (double)r / (double)a;
    double w = want > 1 ? 1 : want;
    checks++;
    if (fraction(a, r, y) != w) { printf("FRAC a=%d r=%d got %.17g want %.17g\n", a, r, fraction(a, r, y), w); return 1; }
    return 0;
}
static int check_wide(int64_t a, int64_t r) {
    double A = (double)a, R = (double)r, y = 1.0 / A;
    checks += 2;
    if (r <= a) {
        uint32_t want = (uint32_t)(((a - r) * 100) / a);
        uint32_t got = least_requested_w(A, R, y);
        if (got != want) { printf("LAW a=%lld r=%lld got %u want %u\n", (long long)a, (long long)r, got, want); return 1; }
    }
    volatile double want = R / A;
    double w = want > 1 ? 1 : want;
    if (fraction_w(A, R, y) != w) { printf("FRACW a=%lld r=%lld\n", (long long)a, (long long)r); return 1; }
    return 0;
}
static double div_count(double x, uint32_t c) {
    const double y3 = 0x1.5555555555555p-2; /* RN(1/3) */
    const double q0 = x * y3;
    const double r = fma(-q0, 3.0, x);
    const double q3 = fma(r, y3, q0);
    return c == 4u ? x * 0.25 : q3;
}
static uint64_t rbits(void);
int main(int argc, char **argv) {
    int mode = argc > 1 ? atoi(argv[1]) : 0;
    if (mode == 0) { /* exhaustive over every allocatable value of spec/synth.md (cpu m, memory MiB) */
        static const int32_t cpu[6] = {4000, 8000, 16000, 32000, 64000, 96000};
        for (int i = 0; i < 6; i++) {
            int32_t a = cpu[i];
            for (int32_t r = 0; r <= a + 10; r++) { if (r <= a && check_la(a, r)) return 1; if (check_frac(a, r)) return 1; }
            for (int m = 2; m <= 8; m *= 2) {
                int32_t am = (a / 1000) * m * 1024; /* MiB */
                for (int32_t r = 0; r <= am + 10; r++) { if (r <= am && check_la(am, r)) return 1; if (check_frac(am, r)) return 1; }
            }
        }
    } else if (mode == 1) { /* random over the whole compacted range [1, 2^24) */
        for (int k = 0; k < 20000000; k++) {
            int32_t a = (int32_t)(1 + rnd() % ((1u << 24) - 1));
            int32_t r = (int32_t)(rnd() % ((uint64_t)a + 1));
            if (check_la(a, r) || check_frac(a, r)) return 1;
        }
    } else if (mode == 3) { /* rcp_int == IEEE 1/a for every a in [1, 2^24), estimates +-2 ulp */
        for (int32_t a = 1; a < (1 << 24); a++) {
            volatile double want = 1.0 / (double)a;
            float f = 1.0f / (float)a;
            float lo = nextafterf(nextafterf(f, 0.0f), 0.0f), hi = nextafterf(nextafterf(f, 2.0f), 2.0f);
            for (float y0 = lo; y0 <= hi; y0 = nextafterf(y0, 2.0f)) {
                checks++;
                if (rcp_int(a, y0) != want) { printf("RCP a=%d y0=%.9g got %.17g want %.17g\n", a, y0, rcp_int(a, y0), want); return 1; }
            }
        }
    } else if (mode == 4) { /* wide layout: random a over every binade up to 2^46, r near a, near
                               multiples of a / 100, and uniform; all-ones significands */
        for (int k = 0; k < 12000000; k++) {
            int e = 1 + (int)(rnd() % 46);
            int64_t a = (int64_t)((rnd() & ((1ULL << e) - 1)) | (1ULL << (e - 1)));
            if (k % 8 == 0) a = (int64_t)((1ULL << e) - 1);
            if (a < 1) a = 1;
            int64_t r;
            switch (k % 4) {
                case 0: r = (int64_t)(rnd() % ((uint64_t)a + 1)); break;
                case 1: r = a - (int64_t)(rnd() % 3); break;
                case 2: { int64_t m = (int64_t)(rnd() % 101); r = a - (a * m) / 100 + (int64_t)(rnd() % 3) - 1; break; }
                default: r = (int64_t)(rnd() % 1024); break;
            }
            if (r < 0) r = 0;
            if (check_wide(a, r)) return 1;
        }
    } else if (mode == 5) { /* div_count: random doubles over every binade of [2^-60, 4), the sums and
                               squared deviations of fractions of small integers, neighbours of
                               multiples of 1/3, and all-ones significands */
        for (long k = 0; k < 40000000; k++) {
            double x;
            switch (k % 5) {
                case 0: { int e = -60 + (int)(rnd() % 62); x = ldexp(1.0 + (double)(rbits() >> 12) * 0x1p-52, e); break; }
                case 1: { double a = (double)(1 + rnd() % 1000), b = (double)(1 + rnd() % 1000);
                          x = (double)(rnd() % 1001) / a + (double)(rnd() % 1001) / b + (double)(rnd() % 1001) / 997.0; break; }
                case 2: { double m = (double)(rnd() % 4000) / 1000.0; x = nextafter(m / 3.0 * 3.0, (k & 8) ? 4.0 : 0.0); break; }
                case 3: { int e = -40 + (int)(rnd() % 42); x = ldexp(2.0 - 0x1p-52, e); break; }
                default: { double f0 = (double)(rnd() % 100001) / 100000.0, f1 = (double)(rnd() % 100001) / 100000.0;
                           double f2 = (double)(rnd() % 100001) / 100000.0; double mu = (f0 + f1 + f2) / 3.0;
                           x = (f0 - mu) * (f0 - mu) + (f1 - mu) * (f1 - mu) + (f2 - mu) * (f2 - mu); break; }
            }
            if (!(x < 4.0)) x = fmod(x, 4.0);
            for (uint32_t c = 3; c <= 4; c++) {
                checks++;
                volatile double want = x / (double)c;
                if (div_count(x, c) != want) { printf("DIVC x=%a c=%u got %a want %a\n", x, c, div_count(x, c), want); return 1; }
            }
        }
        checks += 2;
        if (div_count(0.0, 3) != 0.0 || div_count(0.0, 4) != 0.0) { printf("DIVC zero\n"); return 1; }
    } else { /* small divisors (weight sums, normalize maxima): n/d <= 100 exhaustive */
        for (uint32_t d = 1; d <= 131070; d += (d < 2048 ? 1 : 97)) {
            double y = 1.0 / (double)d;
            for (uint32_t n = 0; n <= 100 * d; n += (d < 256 ? 1 : 1 + d / 64)) {
                checks++;
                if (floor_div(n, y) != n / d) { printf("DIV n=%u d=%u\n", n, d); return 1; }
            }
        }
    }
    printf("ok %lld\n", checks);
    return 0;
}
static uint64_t rbits(void) { return ((uint64_t)rnd() << 32) ^ (uint64_t)rnd(); }
