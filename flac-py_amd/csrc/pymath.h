/*
 * pymath.h — the few Python float operations of flac-py's LPC path, bit-exact on host
 * and device.
 *
 *   py_pow2(x)          float `x ** 2` (flac/encoder.py:476): CPython 3.10 float_pow
 *                       special cases, then glibc 2.35 __pow_fma(|x|, 2.0) instruction for
 *                       instruction (ARM optimized-routines algorithm: log_inline +
 *                       exp_inline with 128-entry tables, every FMA where that build has
 *                       one, every separate add/mul where it does not).
 *   py_floor_log2(x)    math.floor(math.log2(x)) for finite x > 0 (encoder.py:503, :753),
 *                       via a per-exponent threshold table built from the host libm log2.
 *
 * Everything else in the path is plain IEEE add/sub/mul/div/rint, which the device
 * executes exactly as x86-64 SSE2 does provided no contraction happens: every
 * translation unit including this header is compiled with -ffp-contract=off, and the
 * FMAs below are explicit __builtin_fma calls.
 */
#pragma once
#include <stdint.h>
#include <string.h>

#include "glibc_pow_tables.h"

#if defined(__HIPCC__)
#define PYM_HD __host__ __device__ __forceinline__
#else
#define PYM_HD static inline
#endif

namespace pym {

PYM_HD double as_double(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}
PYM_HD uint64_t as_u64(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}

struct PowTables {
    const uint64_t* log_hdr;  /* ln2hi, ln2lo, A[0..6] */
    const uint64_t* log_tab;  /* 128 x {invc, pad, logc, logctail} */
    const uint64_t* exp_hdr;  /* invln2N, shift, negln2hiN, negln2loN, C2..C5 */
    const uint64_t* exp_tab;  /* 2*128 */
};

enum { PYM_OK = 0, PYM_OVERFLOW = 4 };

/* glibc __pow_fma(x, 2.0) for finite x > 0 (x != 1.0 excluded by the caller).
 * *ovf is set when glibc would set errno = ERANGE with an infinite result. */
PYM_HD double glibc_pow2_pos(double x, const PowTables& T, int* ovf) {
    const double Y = 2.0;
    uint64_t ix = as_u64(x);
    if ((ix >> 52) == 0) { /* subnormal: normalise (pow.c "topx == 0") */
        ix = as_u64(x * 0x1p52) & 0x7fffffffffffffffULL;
        ix -= 52ULL << 52;
    }
    /* ---- log_inline(ix, &tail) ---- */
    const uint64_t tmp = ix - 0x3fe6955500000000ULL;
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffULL << 52));
    const double z = as_double(iz);
    const double kd = (double)k;
    const double invc = as_double(T.log_tab[4 * i + 0]);
    const double logc = as_double(T.log_tab[4 * i + 2]);
    const double logctail = as_double(T.log_tab[4 * i + 3]);
    const double Ln2hi = as_double(T.log_hdr[0]), Ln2lo = as_double(T.log_hdr[1]);
    const double A0 = as_double(T.log_hdr[2]), A1 = as_double(T.log_hdr[3]),
                 A2 = as_double(T.log_hdr[4]), A3 = as_double(T.log_hdr[5]),
                 A4 = as_double(T.log_hdr[6]), A5 = as_double(T.log_hdr[7]),
                 A6 = as_double(T.log_hdr[8]);
    const double r = __builtin_fma(z, invc, -1.0);
    const double t1 = __builtin_fma(kd, Ln2hi, logc);
    const double t2 = t1 + r;
    const double lo1 = __builtin_fma(kd, Ln2lo, logctail);
    const double lo2 = (t1 - t2) + r;
    const double ar = A0 * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = __builtin_fma(ar, r, -ar2);
    const double lo4 = (t2 - hi) + ar2;
    const double p1 = __builtin_fma(r, A2, A1);
    const double p3 = __builtin_fma(r, A4, A3);
    const double p5 = __builtin_fma(r, A6, A5);
    const double q = __builtin_fma(ar2, p5, p3);
    const double q2 = __builtin_fma(ar2, q, p1);
    double lo = lo1 + lo2;
    lo = lo + lo3;
    lo = lo + lo4;
    lo = __builtin_fma(ar3, q2, lo);
    const double ly = hi + lo;
    const double ltail = (hi - ly) + lo;
    /* ---- pow: ehi/elo ---- */
    const double ehi = Y * ly;
    const double elo = __builtin_fma(Y, ltail, __builtin_fma(ly, Y, -ehi));
    /* ---- exp_inline(ehi, elo, sign_bias = 0) ---- */
    uint32_t abstop = (uint32_t)((as_u64(ehi) >> 52) & 0x7ff);
    if (abstop - 0x3c9u > 0x3eu) {
        if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + ehi; /* |ehi| < 2^-54 */
        if (abstop > 0x408u) {
            if (as_u64(ehi) >> 63) return 0.0;                 /* __math_uflow: errno cleared by CPython */
            *ovf = 1;
            return __builtin_inf();                             /* __math_oflow */
        }
        abstop = 0; /* large |ehi|: specialcase below */
    }
    const double InvLn2N = as_double(T.exp_hdr[0]), Shift = as_double(T.exp_hdr[1]);
    const double NegLn2hiN = as_double(T.exp_hdr[2]), NegLn2loN = as_double(T.exp_hdr[3]);
    const double C2 = as_double(T.exp_hdr[4]), C3 = as_double(T.exp_hdr[5]),
                 C4 = as_double(T.exp_hdr[6]), C5 = as_double(T.exp_hdr[7]);
    double kd2 = __builtin_fma(ehi, InvLn2N, Shift);
    const uint64_t ki = as_u64(kd2);
    kd2 = kd2 - Shift;
    double er = __builtin_fma(kd2, NegLn2hiN, ehi);
    er = __builtin_fma(kd2, NegLn2loN, er);
    er = elo + er;
    const uint64_t idx = 2 * (ki & 127);
    const uint64_t top = ki << 45;
    const double etail = as_double(T.exp_tab[idx]);
    uint64_t sbits = T.exp_tab[idx + 1] + top;
    const double p23 = __builtin_fma(er, C3, C2);
    const double tr = er + etail;
    const double r2 = er * er;
    const double p45 = __builtin_fma(er, C5, C4);
    double etmp = __builtin_fma(r2, p23, tr);
    const double r4 = r2 * r2;
    etmp = __builtin_fma(r4, p45, etmp);
    if (abstop == 0) { /* specialcase(tmp, sbits, ki) */
        if ((ki & 0x80000000ULL) == 0) {
            sbits -= 1009ULL << 52;
            const double scale = as_double(sbits);
            const double y = 0x1p1009 * __builtin_fma(scale, etmp, scale);
            if (__builtin_isinf(y)) *ovf = 1;
            return y;
        }
        sbits += 1022ULL << 52;
        const double scale = as_double(sbits);
        const double st = etmp * scale;
        double y = scale + st;
        if (__builtin_fabs(y) < 1.0) {
            const double one = y < 0.0 ? -1.0 : 1.0;
            double lo_ = (scale - y) + st;
            const double hi_ = y + one;
            lo_ = ((one - hi_) + y) + lo_;
            y = (lo_ + hi_) - one;
            if (y == 0.0) y = as_double(sbits & 0x8000000000000000ULL);
        }
        return y * 0x1p-1022;
    }
    const double scale = as_double(sbits);
    return __builtin_fma(etmp, scale, scale);
}

/* Python `x ** 2` for a float x (CPython Objects/floatobject.c float_pow). */
PYM_HD double py_pow2(double x, const PowTables& T, int* status) {
    *status = PYM_OK;
    if (__builtin_isnan(x)) return x;
    if (__builtin_isinf(x)) return __builtin_inf();
    if (x == 0.0) return 0.0;
    const double ax = __builtin_fabs(x);
    if (ax == 1.0) return 1.0;
    int ovf = 0;
    const double r = glibc_pow2_pos(ax, T, &ovf);
    if (ovf) *status = PYM_OVERFLOW;
    return r;
}

/* floor(log2(x)) for finite x > 0.  thr[e + 1074] = smallest double in [2^e, 2^(e+1))
 * whose libm log2 is >= e + 1 (2^(e+1) if none), for e in [-1074, 1023]. */
#define PYM_LOG2_THR_N 2098 /* e in [-1074, 1023] */
PYM_HD int py_floor_log2(double x, const double* thr) {
    const uint64_t u = as_u64(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) { /* subnormal: exponent of the leading mantissa bit */
        const uint64_t m = u & 0x000fffffffffffffULL;
        e = -1075 + (64 - __builtin_clzll(m));
    } else {
        e -= 1023;
    }
    /* the index is clamped into the table: a caller outside the contract (inf, NaN, 0) gets a
     * wrong value, never a read past the table */
    const int ti = e + 1074 < 0 ? 0 : e + 1074 > PYM_LOG2_THR_N - 1 ? PYM_LOG2_THR_N - 1 : e + 1074;
    return x >= thr[ti] ? e + 1 : e;
}


}  // namespace pym
