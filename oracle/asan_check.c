/* asan_check.c — TEST INFRASTRUCTURE: drives every oracle entry point over edge shapes
 * under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "ASan host build"; make -C
 * oracle asan, run by tests/test_asan.py).  It checks memory safety and defined behaviour
 * of the CPU restatement, not results (tests/test_oracle_golden.py pins those). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flac_oracle.h"

static uint64_t rng = 0x243F6A8885A308D3ull;
static uint64_t next(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

/* kinds: 0 zeros, 1 constant, 2 alternating full scale, 3 random, 4 synthetic tones, 5 ramp */
static void fill(int64_t* x, int n, int bits, int kind) {
    const int64_t hi = (bits >= 64) ? INT64_MAX : (int64_t)((1ull << (bits - 1)) - 1), lo = -hi - 1;
    int32_t* tmp = kind == 4 ? malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1)) : NULL;
    if (tmp) oracle_synth_unit(7, n, bits, 2024, tmp);
    for (int i = 0; i < n; ++i) {
        int64_t v = 0;
        switch (kind) {
            case 1: v = hi / 3; break;
            case 2: v = (i & 1) ? hi : lo; break;
            case 3: v = lo + (int64_t)(next() % (uint64_t)(hi - lo + 1)); break;
            case 4: v = tmp[i]; break;
            case 5: v = lo + (hi - lo) / (n ? n : 1) * i; break;
        }
        x[i] = v;
    }
    free(tmp);
}

static int unit(const int64_t* x, int n, int L, int q, int rmin, int rmax, int mode, int rorder) {
    flacmi_params p;
    memset(&p, 0, sizeof p);
    p.max_lpc_order = L;
    p.qlp_precision = q;
    p.rice_min = rmin;
    p.rice_max = rmax;
    p.mode = mode;
    p.reserved[0] = rorder;
    flacmi_unit_meta m;
    const int pr = (1 << (rmax > 0 ? rmax : 0)) + 2;
    int32_t* rp = calloc((size_t)pr, sizeof(int32_t));
    uint64_t* res = calloc((size_t)(n > 0 ? n : 1), sizeof(uint64_t));
    double acf[33];
    int64_t fs[5], ls[32];
    int32_t rec[FLACMI_LPC_REC_WORDS(32)];
    const int rc = oracle_analyze_unit(x, n, &p, &m, rp, res, acf, fs, ls, rec);
    free(rp);
    free(res);
    return rc;
}

int main(void) {
    long units = 0;
    const int ns[] = {0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 192, 576, 1152, 4608, 16384};
    const int bitss[] = {2, 8, 16, 20, 24, 32};
    for (size_t a = 0; a < sizeof ns / sizeof ns[0]; ++a) {
        const int n = ns[a];
        int64_t* x = malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
        for (size_t b = 0; b < sizeof bitss / sizeof bitss[0]; ++b)
            for (int kind = 0; kind < 6; ++kind) {
                fill(x, n, bitss[b], kind);
                const int Ls[] = {0, 1, 2, 8, 12, 32};
                for (int li = 0; li < 6; ++li) {
                    if (n > 4608 && Ls[li] != 32 && Ls[li] != 0) continue; /* keep the run short */
                    const int q = (bitss[b] >= 24) ? 15 : (li & 1 ? 5 : 14);
                    unit(x, n, Ls[li], q, 0, n > 4608 ? 8 : 5, FLACMI_MODE_REFERENCE, 0);
                    units++;
                }
                if (n <= 4608) {
                    unit(x, n, 0, 5, 0, 15, FLACMI_MODE_FIXED_ONLY, 0);
                    unit(x, n, 12, 5, 2, 3, FLACMI_MODE_LPC_ONLY, 0);
                    unit(x, n, 0, 5, 0, 4, FLACMI_MODE_RICE_ONLY, n > 2 ? 2 : 0);
                    unit(x, n, 0, 5, 3, 1, FLACMI_MODE_REFERENCE, 0); /* empty Rice range */
                    units += 4;
                }
            }
        free(x);
    }
    /* batch entry point: int16 and int32 rows, tail units, several threads */
    for (int sb = 2; sb <= 4; sb += 2) {
        const int n = 4608, nu = 24, stride = n + 8;
        void* s = calloc((size_t)nu * stride, (size_t)sb);
        for (int u = 0; u < nu; ++u)
            for (int i = 0; i < n; ++i) {
                const int64_t v = (int64_t)(next() % 20001) - 10000;
                if (sb == 2) ((int16_t*)s)[(size_t)u * stride + i] = (int16_t)v;
                else ((int32_t*)s)[(size_t)u * stride + i] = (int32_t)v * 300;
            }
        flacmi_batch b;
        memset(&b, 0, sizeof b);
        b.samples = s;
        b.sample_bytes = sb;
        b.sample_bits = sb == 2 ? 16 : 24;
        b.unit_stride = stride;
        b.n_units = nu;
        b.block_len = n;
        b.tail_len = 1000;
        b.n_tail_units = 2;
        flacmi_params p;
        memset(&p, 0, sizeof p);
        p.max_lpc_order = 12;
        p.qlp_precision = 12;
        p.rice_max = 6;
        flacmi_unit_meta* m = calloc(nu, sizeof *m);
        int32_t* rp = calloc((size_t)nu * 65, sizeof(int32_t));
        uint64_t* res = calloc((size_t)nu * stride, sizeof(uint64_t));
        double* acf = calloc((size_t)nu * 33, sizeof(double));
        int64_t* fs = calloc((size_t)nu * 5, sizeof(int64_t));
        int64_t* ls = calloc((size_t)nu * 32, sizeof(int64_t));
        int32_t* rec = calloc((size_t)nu * FLACMI_LPC_REC_WORDS(32), sizeof(int32_t));
        oracle_analyze_batch(&b, &p, m, rp, 65, res, stride, acf, fs, ls, rec, 4);
        units += nu;
        free(m), free(rp), free(res), free(acf), free(fs), free(ls), free(rec), free(s);
    }
    /* the individual functions on edge values */
    const double vals[] = {0.0, -0.0, 1.0, -1.0, 1e-310, -1e-310, 1e154, 1.35e154, -1.34e154, 1e308, INFINITY,
                           -INFINITY, NAN, 0.5, 2.0, 0x1.fffffffffffffp-1, 0x1p-1074};
    for (size_t i = 0; i < sizeof vals / sizeof vals[0]; ++i) {
        int32_t st;
        (void)oracle_pypow2(vals[i], &st);
        (void)oracle_floor_log2(vals[i], &st);
        double r[4] = {vals[i], vals[(i + 1) % 17], vals[(i + 3) % 17], vals[(i + 5) % 17]}, c[3];
        int32_t site, qv[4], nq, sh;
        oracle_levinson(r, 3, c, &site);
        oracle_quantize(r, 4, 5, qv, &nq, &sh, &site);
        oracle_quantize(r, 0, 15, qv, &nq, &sh, &site);
    }
    for (int n = 0; n < 40; ++n) {
        double w[40];
        oracle_tukey(n, w);
        if (n > 1) (void)oracle_autocorrelation(w, n, n / 2);
    }
    printf("asan_check: %ld units, every oracle entry point, no sanitizer report\n", units);
    return 0;
}
