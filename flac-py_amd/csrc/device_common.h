/*
 * device_common.h — shared device code of the CDNA4 (gfx950) kernels for flac-py's per-block analysis.
 *
 * Two kernels per length class (all units of one launch have the same length n):
 *
 *  k_lpc    one LANE per unit.  The reference's autocorrelation is a sequential
 *           left-to-right float sum (encoder.py:447-450); reproducing it bit-exactly
 *           forbids tree reductions, so each lane streams its own unit once and runs all
 *           L+1 lag chains in registers (a ring of the last S windowed samples, fully
 *           unrolled so every ring index is static).  The Tukey window is wave-uniform
 *           (scalar loads).  Levinson-Durbin then runs once at max order with a snapshot
 *           per order (bit-identical to the reference's per-order re-runs,
 *           encoder.py:374-375), each snapshot quantised (encoder.py:482-534) into the
 *           unit's LPC record.
 *
 *  k_resid  one WORKGROUP per unit.  Samples are staged in LDS with 16-byte coalesced
 *           loads; each thread owns 8-sample chunks and computes, from a register
 *           window, the 5 fixed residuals and all L candidate LPC residuals with 24-bit
 *           integer MACs, accumulating sum|r| per candidate (encoder.py:341-352,
 *           386-404).  A workgroup reduction picks fixed vs LPC (encoder.py:135-157);
 *           the chosen residual is zig-zagged (utils.py:91-94), written to HBM
 *           (coalesced) and to LDS in place of the samples; the Rice search
 *           (encoder.py:655-760) then sums partitions at the finest order, builds the
 *           coarser orders as a pyramid, derives every parameter exactly
 *           (floor(log2(S/len)) with a correctly rounded division and the libm-derived
 *           threshold table), and sums (x >> p) over the residual once for all orders.
 *
 * All float code is compiled with -ffp-contract=off; the only FMAs are the explicit
 * ones of the glibc pow emulation (pymath.h).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "flacmi_kernels.h"
#include "pymath.h"

namespace flacmi {

static __constant__ uint64_t c_log_hdr[9] = GLIBC_POW_LOG_HDR;
static __constant__ uint64_t c_log_tab[512] = GLIBC_POW_LOG_TAB;
static __constant__ uint64_t c_exp_hdr[8] = GLIBC_EXP_HDR;
static __constant__ uint64_t c_exp_tab[256] = GLIBC_EXP_TAB;

typedef short short8 __attribute__((ext_vector_type(8)));
typedef int int4v __attribute__((ext_vector_type(4)));

enum {
    ST_OK = FLACMI_STATUS_OK,
    ST_ZERODIV = FLACMI_STATUS_ZERO_DIVISION,
    ST_ASSERT = FLACMI_STATUS_ASSERTION,
    ST_VALUE = FLACMI_STATUS_VALUE_ERROR,
    ST_OVERFLOW = FLACMI_STATUS_OVERFLOW,
};

/* Compile-time loop: f(std::integral_constant<int, I>) for I in [0, N).  Used wherever a
 * register array is indexed by the loop variable, so indexing stays static even when
 * the body is too large for the unroller's heuristics (no scratch spills). */
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_impl(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, N>(f);
    }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl<0, N>(f);
}

static __constant__ int c_fixed_coef[5][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};

__device__ __forceinline__ double pow2_exact(int e) { /* 2^e, 0 <= e <= 62 */
    return pym::as_double((uint64_t)(1023 + e) << 52);
}

/* ====================================================================================
 * k_resid: fixed + LPC candidate residual sums, choice, chosen residual, Rice search
 * ==================================================================================== */

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ uint32_t uabs32(int32_t v) { return v < 0 ? (uint32_t)(-v) : (uint32_t)v; }
__device__ __forceinline__ uint64_t uabs64(int64_t v) { return v < 0 ? (uint64_t)(-v) : (uint64_t)v; }

struct Decision {
    int status, site, kind, order, shift, ncoefs, fixed_order, lpc_order;
    long long fixed_sum, lpc_sum;
    int coef[FLACMI_MAX_LPC_ORDER];
};

constexpr int kCPT = 4; /* max 8-sample chunks per thread */

/* Per-unit result written field by field (no local struct: keeps the kernel scratch-free). */
__device__ __forceinline__ void put_meta(flacmi_unit_meta* m, int status, int site, const Decision* d,
                                         int with_choice) {
    m->status = status;
    m->site = site;
    m->kind = with_choice ? d->kind : 0;
    m->order = with_choice ? d->order : 0;
    m->shift = with_choice ? d->shift : 0;
    m->ncoefs = with_choice ? d->ncoefs : 0;
    m->res_offset = 0;
    m->res_len = 0;
    m->fixed_order = d ? d->fixed_order : 0;
    m->lpc_order = d ? d->lpc_order : 0;
    m->part_order = 0;
    m->n_parts = 0;
    m->coding_method = 0;
    m->reserved0 = 0;
    m->fixed_sum = d ? d->fixed_sum : 0;
    m->lpc_sum = d ? d->lpc_sum : 0;
    m->rice_bits = 0;
    for (int j = 0; j < FLACMI_MAX_LPC_ORDER; ++j) m->coefs[j] = (with_choice && j < d->ncoefs) ? d->coef[j] : 0;
}


template <int LMAX>
struct ResidLayout {
    static constexpr int HP = (LMAX > 4 ? ((LMAX + 7) / 8) * 8 : 8); /* history pad */
    static constexpr int NSUM = 5 + LMAX;
    static constexpr int CPAD = LMAX > 0 ? ((LMAX + 3) / 4) * 4 : 4; /* coefs per order, padded */
};

static inline size_t resid_lds_bytes(int lmax, int n, int nw, int P, int xbytes) {
    const int HP = lmax > 4 ? ((lmax + 7) / 8) * 8 : 8;
    const int nsum = 5 + lmax;
    const int cpad = lmax > 0 ? ((lmax + 3) / 4) * 4 : 4;
    const int npad = ((n + 7) / 8) * 8 + 8;
    size_t b = (size_t)xbytes * (HP + npad);
    b = (b + 15) & ~(size_t)15;
    b += 8 * (size_t)nw * nsum + 8 * (size_t)nsum;
    b += 4 * (size_t)(lmax > 0 ? lmax : 1) * cpad + 4 * 2 * (size_t)(lmax > 0 ? lmax : 1);
    b = (b + 15) & ~(size_t)15;
    b += sizeof(Decision);
    b = (b + 15) & ~(size_t)15;
    b += 8 * 32 + 4 * 4;
    b = (b + 15) & ~(size_t)15;
    b += 8 * (size_t)(2 * P) + 4 * (size_t)(2 * P);
    return b;
}


}  // namespace flacmi
