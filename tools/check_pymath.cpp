// Bulk check of pymath.h's glibc pow(x, 2.0) emulation against the live libm pow.
// Usage: check_pymath N   (prints "n=.. bad=..")
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "pymath.h"

static const uint64_t LH[] = GLIBC_POW_LOG_HDR, LT[] = GLIBC_POW_LOG_TAB, EH[] = GLIBC_EXP_HDR,
                      ET[] = GLIBC_EXP_TAB;
static double (*volatile P)(double, double) = pow;

int main(int argc, char** argv) {
    const pym::PowTables T{LH, LT, EH, ET};
    std::mt19937_64 g(123);
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    long bad = 0, diffsq = 0;
    for (long i = 0; i < n; i++) {
        double x;
        switch (i % 4) {
            case 0: x = std::uniform_real_distribution<double>(-1, 1)(g); break;
            case 1: {
                uint64_t u = g() & 0x7fffffffffffffffULL;
                memcpy(&x, &u, 8);
                if (!std::isfinite(x)) continue;
                break;
            }
            case 2: x = std::uniform_real_distribution<double>(-1e-3, 1e-3)(g); break;
            default: x = ldexp(std::uniform_real_distribution<double>(0.5, 1)(g), (int)(g() % 2100) - 1074);
        }
        int st;
        const double a = pym::py_pow2(x, T, &st);
        const double b = (x == 0 || fabs(x) == 1) ? (x == 0 ? 0 : 1) : P(fabs(x), 2.0);
        if (memcmp(&a, &b, 8) != 0 && !(std::isnan(a) && std::isnan(b))) {
            if (bad < 5) printf("x=%a got %a want %a\n", x, a, b);
            bad++;
        }
        if (a != fabs(x) * fabs(x)) diffsq++;
    }
    printf("n=%ld bad=%ld (pow != x*x: %ld)\n", n, bad, diffsq);
    return bad != 0;
}
