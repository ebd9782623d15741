/* Emulation for VERDICT r5 item 2: can k_lpc's Tukey rectangle (the samples with window
 * weight exactly 1.0, where every product x_j * x_{j+lag} is an exact integer) be computed as
 * an exact integer sum plus a closed-form rounding of the running fraction, instead of one
 * f64 FMA per term, while staying bit-identical to the reference's sequential float sum
 * (encoder.py:443-450, autocorrelation via sum() of a generator)?
 *
 * Theory ("Why the Tukey rectangle stays on fp64 FMAs"): inside the rectangle the
 * chain is acc_j = RN(acc_{j-1} + p_j) with integer p_j.  Write acc = I + phi, I integer, phi in
 * [0, 1).  While |acc| < 2^53 an add is exact unless the exact sum reaches a binade whose ulp is
 * coarser than every ulp seen so far (the grid G of phi); then phi is rounded to that ulp (ties
 * to even; the integer part is a multiple of any grid <= 1/2).  So the rectangle's result is
 * floor(acc0) + S + phi', S the exact integer sum, phi' = phi0 rounded once per new record
 * binade in the order they are reached.
 *
 * This program checks, per (unit, lag), on the bench's synthetic units:
 *   1. the closed form computed from the exact prefix sums equals the sequential chain (the
 *      theory, bit for bit);
 *   2. the share of (unit, lag) pairs whose record-binade sequence is NOT provable from
 *      B-product block sums: per block, the exact block sum S_b and sum|p| A_b; the walk's
 *      maximum inside the block lies in [max(|I_start|, |I_end|), |I_start| + A_b + 1]; it is
 *      proven when that interval holds no relevant binade boundary, or when its upper end is
 *      already in the binade of max(|I_start|, |I_end|) (the record then moves one binade at a
 *      time up to there: every |p| <= max|x|^2 < 2^31 cannot skip a relevant binade above G).
 *      Otherwise that pair would need the sequential fallback.
 *
 * Test infrastructure only (links oracle/liboracle.so for the synthetic units and the window).
 *   gcc -O2 -ffp-contract=off -o /tmp/rect_emul tools/experiments/rect_emul.c -Loracle -loracle -lm
 *   LD_LIBRARY_PATH=oracle /tmp/rect_emul UNITS [n bits L open8]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_tukey(int32_t n, double* w);
void oracle_synth_unit_mix(int64_t unit, int32_t len, int32_t bits, uint64_t seed, int32_t open_eighths, int32_t* out);

static int binade_i64(int64_t v) { /* floor(log2 |v|), v != 0 */
    uint64_t a = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
    return 63 - __builtin_clzll(a);
}

/* binade of I + phi, phi in [0, 1]; -1075 for 0 (no relevant ulp) */
static int binade_val(int64_t I, double phi) {
    if (I >= 1) return binade_i64(I);
    if (I == 0) return phi > 0 ? ilogb(phi) : -1075;
    /* I <= -1: |v| = |I| - phi */
    uint64_t a = (uint64_t)(-I);
    if (phi == 0.0) return binade_i64(I);
    if ((a & (a - 1)) == 0) return a == 1 ? ilogb(1.0 - phi) : binade_i64(I) - 1;
    return binade_i64(I);
}

/* phi rounded to the grid 2^g, ties to even (exact in double) */
static double round_grid(double phi, int g) { return ldexp(nearbyint(ldexp(phi, -g)), g); }

int main(int argc, char** argv) {
    int units = argc > 1 ? atoi(argv[1]) : 200, n = argc > 2 ? atoi(argv[2]) : 4608, bits = argc > 3 ? atoi(argv[3]) : 16;
    int L = argc > 4 ? atoi(argv[4]) : 12, open8 = argc > 5 ? atoi(argv[5]) : 0;
    const int nb = 4, blocks[4] = {16, 32, 64, 128};
    double* w = malloc(sizeof(double) * n);
    double* xw = malloc(sizeof(double) * n);
    int32_t* x = malloc(sizeof(int32_t) * n);
    oracle_tukey(n, w);
    int lo = 0, hi = 0;
    for (int i = 0; i < n;) {
        if (w[i] != 1.0) { ++i; continue; }
        int j = i;
        while (j < n && w[j] == 1.0) ++j;
        if (j - i > hi - lo) lo = i, hi = j;
        i = j;
    }
    long pairs = 0, theory_bad = 0, no_rect = 0, phi_zero = 0, amb[4] = {0, 0, 0, 0}, amb_units[4] = {0, 0, 0, 0};
    long rect_terms = 0, all_terms = 0;
    for (int u = 0; u < units; ++u) {
        oracle_synth_unit_mix(u, n, bits, 2024, open8, x);
        int64_t xm = 0;
        for (int i = 0; i < n; ++i) {
            xw[i] = (double)x[i] * w[i];
            int64_t a = x[i] < 0 ? -(int64_t)x[i] : x[i];
            xm = a > xm ? a : xm;
        }
        int unit_amb[4] = {0, 0, 0, 0};
        for (int l = 0; l <= L; ++l) {
            const int m = n - l - 1; /* terms j = 0 .. m - 1 */
            const int rlo = lo, rhi = hi - l < m ? hi - l : m;
            ++pairs;
            all_terms += m;
            if (rhi <= rlo) { ++no_rect; continue; }
            rect_terms += rhi - rlo;
            /* the taper chain up to the rectangle.  Its products are not integers, so after the
             * accumulator drops to a lower binade the next add leaves bits at that binade's ulp:
             * phi0 is a multiple of ulp(acc0), not of the coarsest ulp the taper reached */
            double acc = 0.0;
            for (int j = 0; j < rlo; ++j) acc = acc + xw[j] * xw[j + l];
            const double acc0 = acc;
            const int grid = acc0 != 0.0 ? ilogb(acc0) - 52 : -1100; /* phi0 is a multiple of 2^grid */
            /* truth: the sequential rectangle */
            for (int j = rlo; j < rhi; ++j) acc = acc + xw[j] * xw[j + l];
            const double truth = acc;
            /* closed form from the exact prefixes */
            int64_t I = (int64_t)floor(acc0);
            double phi = acc0 - (double)I;
            int g = grid;
            for (int j = rlo; j < rhi; ++j) {
                I += (int64_t)x[j] * (int64_t)x[j + l];
                int e = binade_val(I, phi);
                if (e - 52 > g) {
                    g = e - 52;
                    phi = round_grid(phi, g);
                    if (phi == 1.0) { I += 1; phi = 0.0; }
                    int e2 = binade_val(I, phi); /* a round-up onto a power of two */
                    if (e2 - 52 > g) g = e2 - 52;
                }
            }
            const double closed = (double)I + phi;
            if (memcmp(&closed, &truth, sizeof(double)) != 0) {
                ++theory_bad;
                if (getenv("RECT_VERBOSE"))
                    printf("  miss unit %d lag %d: acc0 %.17g grid 2^%d truth %.17g closed %.17g max|x|^2 2^%.1f\n", u, l, acc0,
                           grid, truth, closed, log2((double)xm * (double)xm));
            }
            const double phi0 = acc0 - floor(acc0);
            if (phi0 == 0.0) { ++phi_zero; continue; }
            /* provability from block sums */
            for (int b = 0; b < nb; ++b) {
                const int B = blocks[b];
                int64_t Is = (int64_t)floor(acc0);
                double ph = phi0;
                int gg = grid, bad = 0;
                for (int j0 = rlo; j0 < rhi && !bad; j0 += B) {
                    const int j1 = j0 + B < rhi ? j0 + B : rhi;
                    int64_t S = 0, A = 0;
                    for (int j = j0; j < j1; ++j) {
                        int64_t p = (int64_t)x[j] * (int64_t)x[j + l];
                        S += p;
                        A += p < 0 ? -p : p;
                    }
                    const int64_t Ie = Is + S;
                    const int64_t as = Is < 0 ? -Is : Is, ae = Ie < 0 ? -Ie : Ie;
                    const int64_t Ub = as + A + 1;
                    const int eU = binade_i64(Ub);
                    if (eU - 52 <= gg) { Is = Ie; continue; } /* no relevant record in the block */
                    const int elo = binade_i64((as > ae ? as : ae) + 1) ; /* conservative: |v| <= |I| + 1 */
                    const int elo2 = (as > ae ? as : ae) > 0 ? binade_i64(as > ae ? as : ae) : -1075;
                    if (elo2 == eU && elo == eU && xm * xm < (1LL << (gg + 53))) {
                        /* the record reaches exactly binade eU, one binade at a time */
                        int64_t carry = 0;
                        for (int e = gg + 53; e <= eU; ++e) {
                            ph = round_grid(ph, e - 52);
                            if (ph == 1.0) { carry += 1; ph = 0.0; }
                        }
                        gg = eU - 52;
                        Is = Ie + carry;
                        continue;
                    }
                    if (ph == 0.0) { Is = Ie; continue; } /* phi is 0: every later add is exact */
                    bad = 1;
                }
                if (bad) { ++amb[b]; unit_amb[b] = 1; }
            }
        }
        for (int b = 0; b < nb; ++b) amb_units[b] += unit_amb[b];
    }
    printf("n %d bits %d L %d open8 %d units %d: rectangle [%d, %d) = %d samples; rectangle terms %.1f%% of all\n", n, bits, L,
           open8, units, lo, hi, hi - lo, 100.0 * rect_terms / all_terms);
    printf("(unit, lag) pairs %ld: closed form != sequential chain: %ld; no rectangle: %ld; phi0 == 0: %ld\n", pairs,
           theory_bad, no_rect, phi_zero);
    for (int b = 0; b < nb; ++b)
        printf("  block %3d: pairs needing the sequential fallback %ld (%.2f%%), units with any %ld (%.1f%%)\n", blocks[b],
               amb[b], 100.0 * amb[b] / pairs, amb_units[b], 100.0 * amb_units[b] / units);
    return 0;
}
