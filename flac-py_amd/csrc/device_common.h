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

/* ---- wave reductions on DPP (VALU lane moves; no LDS traffic) ------------------------
 * quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror, row_mirror: every lane ends with its
 * 16-lane row's sum; row_bcast15 / row_bcast31 then fold the rows so lane 63 holds the
 * wave total, which readlane broadcasts. */
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_add_u64(uint64_t v) {
    const uint32_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)v);
    const uint32_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)(v >> 32));
    return v + (((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    v = dpp_add_u64<0xB1, 0xf>(v);  /* quad_perm [1,0,3,2] */
    v = dpp_add_u64<0x4E, 0xf>(v);  /* quad_perm [2,3,0,1] */
    v = dpp_add_u64<0x141, 0xf>(v); /* row_half_mirror */
    v = dpp_add_u64<0x140, 0xf>(v); /* row_mirror */
    v = dpp_add_u64<0x142, 0xa>(v); /* row_bcast15 */
    v = dpp_add_u64<0x143, 0xc>(v); /* row_bcast31 */
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

/* u32 wave total (exact while the true total < 2^32); one v_add_u32_dpp per step */
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += dpp_u32<0xB1, 0xf>(v);
    v += dpp_u32<0x4E, 0xf>(v);
    v += dpp_u32<0x141, 0xf>(v);
    v += dpp_u32<0x140, 0xf>(v);
    v += dpp_u32<0x142, 0xa>(v);
    v += dpp_u32<0x143, 0xc>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

/* |a - b| + c on biased (x ^ 0x80000000) operands: one v_sad_u32 (the compiler's own
 * pattern match often misses it and emits min, max, sub and add). */
__device__ __forceinline__ uint32_t sad_acc(uint32_t a, uint32_t b, uint32_t c) {
    return (a > b ? a - b : b - a) + c;
}
/* v_sad_u32 acc + |a - b| as one instruction, forced (the pattern match is lost on a constant b) */
__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t acc) {
    asm("v_sad_u32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    return acc;
}
constexpr uint32_t kBias = 0x80000000u;

__device__ __forceinline__ uint64_t uabs64(int64_t v) { return v < 0 ? (uint64_t)(-v) : (uint64_t)v; }

struct Decision {
    int status, site, kind, order, shift, ncoefs, fixed_order, lpc_order;
    int tiers; /* meta.lpc_tiers: LPC candidate passes made | passes of the path << 8 (0: no pruning) */
    long long fixed_sum, lpc_sum;
    int coef[FLACMI_MAX_LPC_ORDER];
};

constexpr int kCPT = 3; /* max 8-sample chunks per thread */

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
    m->lpc_tiers = d ? d->tiers : 0;
    m->fixed_sum = d ? d->fixed_sum : 0;
    m->lpc_sum = d ? d->lpc_sum : 0;
    m->rice_bits = 0;
    for (int j = 0; j < FLACMI_MAX_LPC_ORDER; ++j) m->coefs[j] = (with_choice && j < d->ncoefs) ? d->coef[j] : 0;
}

/* put_meta(.., with_choice = 1) plus the Rice fields, by one wave: lane i writes dword i of
 * the 52-dword record (one coalesced store instead of ~50 single-lane stores, each behind
 * its own LDS read of the decision) */
__device__ __forceinline__ void put_meta_wave(flacmi_unit_meta* m, int lane, int status, int site, const Decision* d,
                                              int res_offset, int res_len, int part_order, int n_parts, int coding,
                                              long long rice_bits) {
    const int j = lane - 20;
    uint32_t x = (j >= 0 && j < d->ncoefs) ? (uint32_t)d->coef[j < FLACMI_MAX_LPC_ORDER ? j : 0] : 0u;
    const uint32_t f[20] = {(uint32_t)status, (uint32_t)site, (uint32_t)d->kind, (uint32_t)d->order,
                            (uint32_t)d->shift, (uint32_t)d->ncoefs, (uint32_t)res_offset, (uint32_t)res_len,
                            (uint32_t)d->fixed_order, (uint32_t)d->lpc_order, (uint32_t)part_order,
                            (uint32_t)n_parts, (uint32_t)coding, (uint32_t)d->tiers, (uint32_t)d->fixed_sum,
                            (uint32_t)((unsigned long long)d->fixed_sum >> 32), (uint32_t)d->lpc_sum,
                            (uint32_t)((unsigned long long)d->lpc_sum >> 32), (uint32_t)rice_bits,
                            (uint32_t)((unsigned long long)rice_bits >> 32)};
#pragma unroll
    for (int i = 0; i < 20; ++i) x = lane == i ? f[i] : x;
    if (lane < 52) reinterpret_cast<uint32_t*>(m)[lane] = x;
}

/* Workgroup size of k_resid for n samples: 8-sample chunks, up to kCPT per thread while
 * the workgroup stays <= 256 threads (512 for the 64-bit paths: their long blocks fill the
 * LDS with one workgroup per CU, so 8 waves are two per SIMD), more beyond that.  The
 * kernel's launch bound follows the same rule. */
__host__ __device__ inline int resid_threads(int n, bool wide = false) {
    const int nch = (n + 7) / 8;
    int nt = 64 * ((nch + 64 * kCPT - 1) / (64 * kCPT));
    const int cap = wide ? 512 : 256;
    if (nt > cap) nt = cap;
    return nt < 64 ? 64 : nt;
}
/* samples one thread of k_resid accumulates */
__host__ __device__ inline int resid_samples_per_thread(int n) {
    const int nch = (n + 7) / 8;
    const int nt = resid_threads(n);
    return 8 * ((nch + nt - 1) / nt);
}

/* History pad in front of the staged samples (>= LMAX and >= 4, multiple of 8). */
__host__ __device__ constexpr int resid_hp(int lmax) { return lmax > 4 ? ((lmax + 7) / 8) * 8 : 8; }

/* k_resid keeps the chosen zig-zag residual in registers (kCPT chunks of 8 per thread)
 * instead of LDS when it is 32-bit and narrow (< 2^27), every thread owns at most kCPT
 * chunks, and every candidate Rice order has whole-chunk finest partitions, at most 64. */
__host__ __device__ inline bool resid_regz(int n, int rmax_eff, bool narrow32) {
    const int pe = rmax_eff < 0 ? 0 : rmax_eff;
    return narrow32 && n <= 8 * kCPT * 256 && n % (8 << pe) == 0 && (1 << pe) <= 64;
}

/* LDS layout of k_resid: byte offsets (multiples of 16) from the dynamic LDS base.  The
 * host sizes the allocation with the same function the kernel carves it with. */
/* staged samples occupy [-HP, resid_xpad(n)): the 8-sample chunks plus one, and the
 * 64-sample MFMA blocks; zero past n */
__host__ __device__ inline int resid_xpad(int n) {
    const int a = ((n + 7) / 8) * 8 + 8, b = ((n + 63) / 64) * 64 + 8;
    return a > b ? a : b;
}

/* int8-MFMA candidate-sum planes (k_resid, PATH_W64): three byte planes of the samples'
 * balanced base-256 digits, sample i at byte kMf8Pad + i of its plane, zero outside
 * [0, n); the 16-byte tail keeps every 5-dword fragment read inside the plane. */
constexpr int kMf8Pad = 32;
__host__ __device__ inline int mf8_plane_bytes(int n) {
    /* planes 128 B (32 banks) apart modulo 256 B: the slot-1 lanes' windows (another plane)
     * fall on the other half of the banks from the slot-0 lanes' */
    return ((n + kMf8Pad + 16 + 255) & ~255) + 128;
}

struct ResidLds {
    int xs, pl, zz, cs, coef, red, dec, rb, misc, hs, hp, tl, total;
};
/* floor(log2) thresholds staged in LDS for exponents [kTlLo, kTlLo + 64): every Rice
 * mean S/len of a 32-bit residual (S >= 1, len <= 65535, S < 2^48) falls inside. */
constexpr int kTlLo = -16;
__host__ __device__ inline ResidLds resid_lds_layout(int lmax, int n, int nw, int P, int xbytes, int zbytes,
                                                     int coef_bytes, bool regz, bool planes) {
    auto up = [](int b) { return (b + 15) & ~15; };
    const int nsum = 5 + lmax;
    const int npad = ((n + 7) / 8) * 8 + 8;
    ResidLds l;
    int o = 0;
    l.xs = o;   o = up(o + xbytes * (resid_hp(lmax) + resid_xpad(n)));
    /* the MFMA planes are dead after the candidate sums; the residual-side regions reuse them */
    l.pl = o;
    const int pl_end = up(o + (planes ? 3 * mf8_plane_bytes(n) : 0));
    l.zz = o;   o = up(o + (regz ? 0 : zbytes * npad)); /* zig-zag row (LDS-resident mode) */
    l.cs = o;   o = up(o + (regz ? 4 * (npad / 8) : 0)); /* chunk sums (register-resident mode) */
    l.hs = o;   o = up(o + 8 * 2 * P);
    l.hp = o;   o = up(o + 4 * 2 * P);
    o = o > pl_end ? o : pl_end;
    l.coef = o; o = up(o + coef_bytes);
    /* the int8-MFMA path's pruning tiers alternate between two copies (one barrier per test) */
    /* (nsum + 1 per wave: the 16-bit sign bound's fixed sums and K_0 .. K_lmax) */
    l.red = o;  o = up(o + 8 * nw * (nsum + 1 > 16 ? nsum + 1 : 16) * (planes ? 2 : 1));
    l.dec = o;  o = up(o + (int)sizeof(Decision));
    l.rb = o;   o = up(o + 8 * 32);
    l.misc = o; o = up(o + 4 * 8);
    l.tl = o;   o = up(o + 8 * 64);
    l.total = o;
    return l;
}

}  // namespace flacmi
