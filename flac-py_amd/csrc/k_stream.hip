/* k_stream.hip — the residual-side analysis (candidate sums, choice, chosen residual, Rice
 * search) for the common 16-bit shapes: k_resid_stream, one workgroup per unit.
 *
 * Same results as k_resid (k_resid.h) bit for bit; it replaces k_resid's launch where the
 * shape allows (host check: stream_shape_ok):
 *   int16 samples, 32-bit residual rows, reference mode with 1 <= L <= 12 or fixed-only
 *   mode, n % 64 == 0, 64 <= n <= 8 * kSCPT * 256 (10240), at most 32 finest Rice partitions of whole
 *   8-sample chunks.
 *
 * Reference semantics (flac/encoder.py): fixed predictors 331-359, LPC candidate residuals
 * 386-404 with prediction_residual 537-548, the fixed-vs-LPC choice 133-157, encode_residual
 * + rice_partitions + find_rice_parameter + rice_size 632-760.
 *
 * Structure (nw = n/2560 rounded-up waves per workgroup, four workgroup barriers):
 *   - samples sit in LDS biased (x ^ 0x8000: unsigned 16-bit), which makes the MFMA operand
 *     build two byte permutes and two packed subtracts per lane and block;
 *   - candidate sums on v_mfma_f32_16x16x32_f16 with INTEGER taps and the accumulator
 *     initialised to M = 1.5 * 2^23: every partial sum is an integer inside [2^23, 2^24)
 *     (ulp 1) under the per-unit bound (sum|c| + 2^shift) * 33023 < 2^22, so the result is
 *     exactly M + T with T = pred - 2^shift * x[i] whatever the accumulation order.  The
 *     float's bit pattern is then 0x4B400000 + T; 0x4B400000 is a multiple of 2^22, so
 *     (bits >> shift) - (0x4B400000 >> shift) = floor(T / 2^shift) = -r exactly.  Fixed
 *     predictors (shift 0): |r| is one v_sad_u32; LPC: one shift + one v_sad_u32.
 *     MFMA 0 holds fixed orders 1..4 x 4 sample phases, MFMAs 1..NG the LPC orders
 *     4(g-1)+1 .. 4g x 4 phases; each lane builds its B operands from the LDS record (the
 *     fixed group's is a constant).  Units outside the bound are listed for k_resid;
 *   - the choice (a lane-parallel DPP argmin), the Rice parameters (one heap node per lane,
 *     finest partition sums by LDS atomics) and the order choice are
 *     computed redundantly by every wave from LDS data, so no single-wave serial section
 *     sits between barriers;
 *   - the chosen residual is written to HBM from registers and kept as packed 16-bit pairs;
 *     Rice data bits on those pairs (v_pk_lshrrev_b16 + v_dot2_u32_u16) when a chunk's
 *     values are < 2^16;
 *   - the 208-byte meta record is one coalesced store of 52 lanes.
 */
#include <type_traits>

#include "device_common.h"

namespace flacmi {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

#ifndef FLACMI_STREAM_CPT
#define FLACMI_STREAM_CPT 5
#endif
constexpr int kSCPT = FLACMI_STREAM_CPT; /* max 8-sample chunks per thread */
/* workgroup size: 8-sample chunks, up to kSCPT per thread */
__host__ __device__ constexpr int stream_threads(int n) {
    const int nch = n / 8;
    const int nt = 64 * ((nch + 64 * kSCPT - 1) / (64 * kSCPT));
    return nt < 64 ? 64 : nt;
}
constexpr int kSHP = 16;                     /* biased-zero history pad in front of the unit (samples) */
constexpr uint32_t kMagicBits = 0x4B400000u; /* 1.5 * 2^23 */
constexpr int kCoefLimit = 127;              /* (sum|c| + 2^shift) * 33023 < 2^22 */
constexpr int kRiceOrders = 8;               /* orders 0..7 kept per finest partition */

struct SLds {
    int xs, pk, rec, red, red2, red0, pks, total;
};

/* Workgroup LDS (bytes).  Regions whose lifetimes do not overlap share space, which keeps a
 * config-2 unit (n = 4608, two waves) at 10160 B: 16 workgroups per CU.
 *   xs   biased samples behind a 16-sample zero pad             staging .. Rice recompute
 *   pk   u16 [P][RS] Rice parameters per order (entry 0 bit 15: flag) Rice (after B3)
 *   rec  the LPC orders' f16 tap table (aliases pk, tap_table)  staging .. MFMA operands
 *   red  u64 [nw][group][order] MFMA partial sums               MFMA phase .. choice
 *   red2 u64 [nw + 1][order] data bits (aliases red)            Rice (after B3)
 *   red0 u32 [nw] sum|x|                                         staging .. choice
 *        (word 0 then: the Rice table's error flag                 B3 .. B3b)
 *   pks  u32 [P] finest partition sums                          staging (zeroed) .. Rice */
__host__ __device__ inline SLds stream_lds(int n, int nw, int tap_words, int P, int RS) {
    auto up = [](int b) { return (b + 15) & ~15; };
    auto mx = [](int x, int y) { return x > y ? x : y; };
    SLds l;
    int o = 0;
    l.xs = o;   o = up(o + 2 * (kSHP + n));
    l.pk = l.rec = o; o = up(o + mx(2 * P * RS, 4 * mx(tap_words, 1)));
    l.red = l.red2 = o; o = up(o + mx(8 * nw * 16, 8 * (nw + 1) * kRiceOrders));
    l.red0 = o; o = up(o + 4 * nw);
    l.pks = o;  o = up(o + 4 * P);
    l.total = o;
    return l;
}

/* The LPC orders' taps as an f16 table, built in staging straight from the global record
 * (encoder.py:537-548 prediction_residual as taps: T_p[0] = -2^shift_p for x[i] itself,
 * T_p[m] = c_p[m - 1] for x[i - m], 0 elsewhere).  Row p (1 .. 4 NG) holds the halves
 * D_p[k] = T_p[16 - k], k = 0 .. 21, from word 10 (p - 1): descending tap order, so a lane's
 * operand pairs (T[i], T[i-1]) are consecutive halves (one v_alignbit off a dword edge).  Rows
 * overlap by one word (k = 20, 21 of row p = k = 0, 1 of row p + 1: zero in both for p <= 12),
 * rows p > L are zero. */
__host__ __device__ constexpr int tap_table_words(int NG) { return NG > 0 ? 40 * NG + 1 : 0; }
__device__ __forceinline__ uint32_t f16_of_int(int v) {
    return (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)(float)v); /* exact for |v| <= 2048 */
}

/* f16 bit pattern of a small integer (exact) */
constexpr uint32_t f16_bits(int v) {
    if (v == 0) return 0;
    const uint32_t sgn = v < 0 ? 0x8000u : 0u;
    const int m = v < 0 ? -v : v;
    int e = 0;
    while ((m >> (e + 1)) != 0) ++e;
    return sgn | (uint32_t)((e + 15) << 10) | (uint32_t)((m << (10 - e)) & 0x3ff);
}
/* fixed predictor order p (common.py:15-21) as taps: T[0] = -1 (x[i]), T[j] = (-1)^(j-1) C(p, j) */
constexpr int fixed_tap(int p, int j) {
    if (j == 0) return -1;
    if (j < 0 || j > p) return 0;
    int c = 1;
    for (int t = 0; t < j; ++t) c = c * (p - t) / (t + 1);
    return (j & 1) ? c : -c;
}
/* the fixed group's B operand per lane (column = 4 (order - 1) + phase rho, kb = lane / 16):
 * {H(ia), H(ia - 2), L(ia), L(ia - 2)}, ia = 12 + rho - 4 kb, L(i) = (T[i], T[i-1]), H = 256 L */
struct FixB {
    uint32_t w[64 * 4];
};
constexpr FixB make_fixb() {
    FixB t{};
    for (int l = 0; l < 64; ++l) {
        const int col = l & 15, kb = l >> 4, p = (col >> 2) + 1, rho = col & 3, ia = 12 + rho - 4 * kb;
        const int idx[2] = {ia, ia - 2};
        for (int k = 0; k < 2; ++k) {
            const int i = idx[k];
            t.w[4 * l + k] = f16_bits(256 * fixed_tap(p, i)) | f16_bits(256 * fixed_tap(p, i - 1)) << 16;
            t.w[4 * l + 2 + k] = f16_bits(fixed_tap(p, i)) | f16_bits(fixed_tap(p, i - 1)) << 16;
        }
    }
    return t;
}
__constant__ const FixB kFixB = make_fixb();

/* |a - b| + acc: the compiler emits one v_sad_u32 when b is in a VGPR (opaque() keeps a
 * constant b there).  Not inline asm: the hazard recognizer does not see an asm operand
 * read an MFMA result, and such a read without the required wait states returns garbage. */
__device__ __forceinline__ uint32_t sad32(uint32_t a, uint32_t b, uint32_t acc) { return (a > b ? a - b : b - a) + acc; }
/* min with the DPP-moved value of a u64 (all lanes of a row valid for the row patterns used) */
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    return o < v ? o : v;
}
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
/* a wave-uniform constant kept opaque in an SGPR (v_sad_u32 takes it as src1) */
__device__ __forceinline__ uint32_t opaque_s(uint32_t v) {
    asm volatile("" : "+s"(v));
    return v;
}

__device__ __forceinline__ uint32_t h2sub(uint32_t t, float c) {
    const h2 v = __builtin_bit_cast(h2, t) - h2{(_Float16)c, (_Float16)c};
    return __builtin_bit_cast(uint32_t, v);
}

/* Raw A fragment of one lane from 4 biased samples (two dwords): the f16 values 1024 + hb
 * (biased high bytes) then 1024 + l (low bytes), one v_perm per pair.  Raw, it stands for
 * x + 295936 (256 * 1152 + 1024) per sample: the fixed group takes it as it is, because a
 * fixed predictor's taps sum to zero ((1 - z^-1)^o), so the offset cancels, and its partial
 * sums stay exact (|M +- 1279 * 257 * 8| < 2^24 for order 4, whose positive and negative
 * taps each sum to 8). */
__device__ __forceinline__ uint4 a_raw(uint2 q) {
    return uint4{__builtin_amdgcn_perm(0x64646464u, q.x, 0x04030401u), __builtin_amdgcn_perm(0x64646464u, q.y, 0x04030401u),
                 __builtin_amdgcn_perm(0x64646464u, q.x, 0x04020400u), __builtin_amdgcn_perm(0x64646464u, q.y, 0x04020400u)};
}
/* the exact A fragment (the LPC groups' taps do not sum to zero): signed high bytes
 * (1024 + hb) - 1152, low bytes (1024 + l) - 1024, all exact */
__device__ __forceinline__ h8 a_sub(uint4 r) {
    const uint4 v{h2sub(r.x, 1152.0f), h2sub(r.y, 1152.0f), h2sub(r.z, 1024.0f), h2sub(r.w, 1024.0f)};
    return __builtin_bit_cast(h8, v);
}

/* exact floor(log2(s / len)) = max{p : len * 2^p <= s} for s >= 1 (s < 2^46; see
 * k_resid.h rice_params_wave0 for why this equals the reference's float computation) */
__device__ __forceinline__ int rice_param_exact(uint64_t s, int len) {
    const int fs = 63 - __builtin_clzll((unsigned long long)s);
    const int fl = 31 - __builtin_clz((unsigned)len);
    int p = fs - fl;
    if (p >= 0 && ((uint64_t)len << p) > s) --p;
    return p;
}

/* one finest partition's Rice table row (16 bytes: a u16 parameter per order); word o / 2
 * holds orders o (low half) and o + 1 (high half) */
__device__ __forceinline__ void load_ptab(const uint16_t* row, uint32_t (&w)[kRiceOrders / 2]) {
    const uint4 a = *reinterpret_cast<const uint4*>(row);
    w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w;
}
/* both halves of the 16-bit pair d shifted right by the low (HI = 0) or high (HI = 1) half
 * of s: op_sel broadcasts that half to both lanes (no splat instruction) */
template <int HI>
__device__ __forceinline__ uint32_t pk_shr_bcast(uint32_t s, uint32_t d) {
    uint32_t r;
    if constexpr (HI) asm("v_pk_lshrrev_b16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(s), "v"(d));
    else asm("v_pk_lshrrev_b16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(s), "v"(d));
    return r;
}

/* one chunk's eight zig-zag values to the residual row (FLACMI_NT_STORE: non-temporal, A/B) */
__device__ __forceinline__ void store_row(uint32_t* r, const uint32_t (&z)[8]) {
#if FLACMI_NT_STORE
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(v4u{z[0], z[1], z[2], z[3]}, reinterpret_cast<v4u*>(r));
    __builtin_nontemporal_store(v4u{z[4], z[5], z[6], z[7]}, reinterpret_cast<v4u*>(r) + 1);
#else
    reinterpret_cast<uint4*>(r)[0] = uint4{z[0], z[1], z[2], z[3]};
    reinterpret_cast<uint4*>(r)[1] = uint4{z[4], z[5], z[6], z[7]};
#endif
}

/* fixed order K residual of samples i0..i0+7 from biased LDS samples, zig-zagged; the
 * warm-up samples (i < K) give 0 */
template <int K, bool FIRST = true>
__device__ __forceinline__ void fixed_chunk(const uint16_t* xs, int i0, uint32_t (&z)[8]) {
    const uint4 w = *reinterpret_cast<const uint4*>(xs + i0);
    const uint4 v = *reinterpret_cast<const uint4*>(xs + i0 - 8); /* pad >= 8 */
    const uint32_t q[6] = {v.z, v.w, w.x, w.y, w.z, w.w};
    int32_t d[12]; /* biased samples i0-4 .. i0+7 */
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        d[2 * t] = (int32_t)(q[t] & 0xffffu);
        d[2 * t + 1] = (int32_t)(q[t] >> 16);
    }
    if constexpr (K == 0) {
#pragma unroll
        for (int t = 4; t < 12; ++t) d[t] -= 32768;
    }
#pragma unroll
    for (int l = 1; l <= K; ++l)
#pragma unroll
        for (int t = 11; t >= 4 - K + l; --t) d[t] -= d[t - 1];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int32_t r = d[4 + k];
        z[k] = ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
    }
    if (FIRST && i0 == 0) { /* only the first chunk slot can hold chunk 0 */
#pragma unroll
        for (int k = 0; k < K; ++k) z[k] = 0;
    }
}

/* LPC order p (<= 12) residual of samples i0..i0+7 (prediction_residual, encoder.py:537-548):
 * r = x[i] - (sum_j c[j] x[i-1-j] >> shift); |pred| < 2^22 under the MFMA bound.  Samples
 * i < start give 0.  Rare (LPC rarely wins under the reference's sign convention), so it
 * is written for registers, not speed: the 24 samples stay packed, the coefficients are
 * wave-uniform (lane q of coefl holds c[q]; c[q] == 0 for q >= p). */
__device__ __forceinline__ void lpc_chunk(const uint16_t* xs, int i0, int32_t coefl, int sh, int start,
                                          uint32_t (&z)[8]) {
    uint32_t w[12]; /* biased samples i0-16 .. i0+7, two per word */
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const uint4 v = *reinterpret_cast<const uint4*>(xs + i0 - 16 + 8 * g);
        w[4 * g] = v.x;
        w[4 * g + 1] = v.y;
        w[4 * g + 2] = v.z;
        w[4 * g + 3] = v.w;
    }
    auto x = [&](int t) __attribute__((always_inline)) -> int32_t {
        return (int32_t)((t & 1) ? (w[t >> 1] >> 16) : (w[t >> 1] & 0xffffu)) - 32768;
    };
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int32_t pred = 0;
#pragma unroll
        for (int j = 0; j < 12; ++j) pred += __builtin_amdgcn_readlane(coefl, j) * x(16 + k - 1 - j);
        const int32_t r = x(16 + k) - (pred >> sh);
        const uint32_t zz = ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
        z[k] = (i0 + k >= start) ? zz : 0u;
    }
}

/* One wave writes the 52 dwords of a unit's flacmi_unit_meta (include/flacmi.h field order)
 * with one store: lanes 0..19 take the 20 scalar fields (a select chain), lanes 20..51 take
 * coefs[lane - 20] from lane q's `coef`. */
struct MetaVals {
    int status, site, kind, order, shift, ncoefs, res_offset, res_len, fixed_order, lpc_order, part_order,
        n_parts, coding, tiers;
    long long fixed_sum, lpc_sum, rice_bits;
};
__device__ __forceinline__ void store_meta(flacmi_unit_meta* m, int lane, const MetaVals& v, int32_t coef) {
    uint32_t x = (uint32_t)__shfl(coef, (lane - 20) & 63);
    const uint32_t f[20] = {(uint32_t)v.status, (uint32_t)v.site, (uint32_t)v.kind, (uint32_t)v.order,
                            (uint32_t)v.shift, (uint32_t)v.ncoefs, (uint32_t)v.res_offset, (uint32_t)v.res_len,
                            (uint32_t)v.fixed_order, (uint32_t)v.lpc_order, (uint32_t)v.part_order,
                            (uint32_t)v.n_parts, (uint32_t)v.coding, (uint32_t)v.tiers, (uint32_t)v.fixed_sum,
                            (uint32_t)((unsigned long long)v.fixed_sum >> 32), (uint32_t)v.lpc_sum,
                            (uint32_t)((unsigned long long)v.lpc_sum >> 32), (uint32_t)v.rice_bits,
                            (uint32_t)((unsigned long long)v.rice_bits >> 32)};
#pragma unroll
    for (int i = 0; i < 20; ++i) x = lane == i ? f[i] : x;
    if (lane < 52) reinterpret_cast<uint32_t*>(m)[lane] = x;
}

}  // namespace

/* One unit (batch index gid) through the whole analysis.  NG = number of LPC MFMA groups
 * (ceil(L / 4)), 0 in fixed-only mode.  R05: the Rice partition orders are 0..5 for every
 * unit (host-checked: rmin 0, n % 32 == 0 and n / 32 > every predictor order), so the order
 * loops compile without per-order branches.  Every exit is workgroup-uniform (all waves decide
 * from the same LDS data).
 * LIST (k_resid_stream_list, the units the batch kernel listed): the LPC groups' B operands
 * drop the x tap T_p[0] = -2^shift, so the MFMA result is M + pred, exact while sum|c| <= 127
 * whatever the shift; every LPC value is then exact, |r| = |x - floor(pred / 2^shift)| by a
 * shift, a subtract and one v_sad_u32 (no pruning tiers: the units a large shift lists are
 * mostly near-ties no bound decides).  A unit outside even that bound goes to the second list
 * (k_resid's list variant). */
template <int NG, bool R05, int NFIX, bool LIST, typename Args>
__device__ __forceinline__ void stream_unit(const Args& a, const int64_t gid, unsigned char* smem) {
    /* NFIX: the block length (and L = 4 NG, the workgroup size) as compile-time constants, the
     * BASELINE configs' 4608-sample units: loop bounds, chunk guards and partition indices fold */
    /* LIST: the thread id through an opaque register per unit (hoisted out of the unit loop,
     * every value derived from it would stay live across the whole body) */
    const int tid = LIST ? (int)opaque((uint32_t)threadIdx.x) : (int)threadIdx.x, NT = NFIX ? stream_threads(NFIX) : (int)blockDim.x, lane = tid & 63, nw = NT >> 6;
#if FLACMI_STREAM_STAMPS /* diagnostic build only: per-unit phase clock stamps of wave 0 */
    uint64_t stamp[8];
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    stamp[0] = __builtin_amdgcn_s_memtime();
#define STAMP(k) (stamp[k] = __builtin_amdgcn_s_memtime())
#else
#define STAMP(k) ((void)0)
#endif
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = NFIX ? NFIX : a.n, L = NG > 0 ? (NFIX ? 4 * NG : a.L) : 0;
    const int nch = n >> 3, nblk = n >> 6;
    const int rw = NG > 0 ? (NFIX ? 2 + L + (L * (L + 1)) / 2 : a.rec_words) : 0;
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (n % (1 << o) == 0) rmax_eff = o;
    const int Pmax = 1 << rmax_eff; /* host-checked: 0 <= rmax_eff <= 5 */
    constexpr int RS = kRiceOrders; /* Rice table entries per finest partition (16-byte rows: at
                                     * 10160 B a config-2 unit keeps 16 workgroups per CU) */
    const SLds lay = stream_lds(n, nw, tap_table_words(NG), Pmax, RS);
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem + lay.xs) + kSHP;
    int32_t* recl = reinterpret_cast<int32_t*>(smem + lay.rec);
    uint32_t* red0 = reinterpret_cast<uint32_t*>(smem + lay.red0);
    unsigned long long* red2 = reinterpret_cast<unsigned long long*>(smem + lay.red2);
    uint32_t* pks = reinterpret_cast<uint32_t*>(smem + lay.pks); /* finest partition sums */
    uint16_t* pkw = reinterpret_cast<uint16_t*>(smem + lay.pk);
    flacmi_unit_meta* meta = a.meta + gid;
    MetaVals mv{};

    /* ---- stage: biased samples and the record into LDS, sum|x| on the way ---- */
    uint4 fixb; /* the fixed group's MFMA B operand (constant) */
    {
        const uint4* src = reinterpret_cast<const uint4*>((const int16_t*)a.samples + (a.unit0 + gid) * a.stride);
        /* every load is issued before the first wait: clamped indices, no branches (a load
         * inside a guarded block gets its own s_waitcnt there, serialising the HBM trips) */
        uint4 q[kSCPT];
#pragma unroll
        for (int j = 0; j < kSCPT; ++j) {
#if FLACMI_NT_LOAD
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + min(tid + j * NT, nch - 1));
            q[j] = uint4{t.x, t.y, t.z, t.w};
#else
            q[j] = src[min(tid + j * NT, nch - 1)];
#endif
        }
        fixb = reinterpret_cast<const uint4*>(kFixB.w)[lane];
        /* tap table words tid + j NT: word w of row p holds (T_p[16 - 2w], T_p[15 - 2w]); the
         * record values it needs are loaded here, with the samples (clamped, unconditional) */
        constexpr int kTW = tap_table_words(NG), kTJ = NG > 0 ? (kTW + 63) / 64 : 0;
        int32_t tv[kTJ > 0 ? kTJ : 1][2];
        if constexpr (NG > 0) {
            const int32_t* r = a.rec + gid * rw;
#pragma unroll
            for (int j = 0; j < kTJ; ++j) {
                if (j > 0 && j * NT >= kTW) break; /* uniform: a two-wave unit needs j = 0 only */
                const int gw = tid + j * NT, p = gw / 10 + 1, w = gw - 10 * (p - 1);
                const int pc = p < L ? p : L, base = 2 + L + (pc * (pc - 1)) / 2;
                /* T_p[16 - 2w] (the shift for w = 8: T_p[0] = -2^shift) and T_p[15 - 2w] */
                tv[j][0] = r[w == 8 ? 1 + pc : min(max(base + 15 - 2 * w, 0), rw - 1)];
                tv[j][1] = r[min(max(base + 14 - 2 * w, 0), rw - 1)];
            }
        }
        if (tid < kSHP) xs[tid - kSHP] = 0x8000u; /* biased zeros */
        if (tid < Pmax) pks[tid] = a.stop_after == 10 ? (uint32_t)n * 40u : 0u; /* 10: no atomics, sums nonzero */
        const uint32_t k8000 = opaque(0x8000u);
        uint32_t sumx = 0;
#pragma unroll
        for (int j = 0; j < kSCPT; ++j) {
            const int v = tid + j * NT;
            if (v < nch) {
                const uint4 y{q[j].x ^ 0x80008000u, q[j].y ^ 0x80008000u, q[j].z ^ 0x80008000u, q[j].w ^ 0x80008000u};
                *reinterpret_cast<uint4*>(xs + 8 * v) = y;
                const uint32_t yd[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    sumx = sad32(yd[e] & 0xffffu, k8000, sumx);
                    sumx = sad32(yd[e] >> 16, k8000, sumx);
                }
            }
        }
        if constexpr (NG > 0) {
            uint32_t* tt = reinterpret_cast<uint32_t*>(recl);
#pragma unroll
            for (int j = 0; j < kTJ; ++j) {
                if (j > 0 && j * NT >= kTW) break;
                const int gw = tid + j * NT, p = gw / 10 + 1, w = gw - 10 * (p - 1);
                if (gw < kTW) {
                    auto tap = [&](int i, int32_t c) -> uint32_t {
                        if (p > L || i < 0 || i > p) return 0u;
                        return f16_of_int(i == 0 ? -(1 << c) : c);
                    };
                    tt[gw] = tap(16 - 2 * w, tv[j][0]) | tap(15 - 2 * w, tv[j][1]) << 16;
                }
            }
        }
        const uint32_t sx = wave_sum_u32(sumx);
        if (lane == 0) red0[wid] = sx;
    }
    STAMP(1);
    __syncthreads(); /* B1 */
    STAMP(2);
    /* ---- unit status from the LPC record; MFMA exactness bound per order.
     * Every wave reads the same LDS words, so the exits are workgroup-uniform. ---- */
    uint32_t negmask = 0;
    const int32_t* __restrict__ grec = NG > 0 ? a.rec + gid * rw : nullptr; /* wave-uniform: scalar loads */
    if constexpr (NG > 0) {
        const int st = grec[0];
        if (st != 0) { /* the reference raises inside encode_subframe_lpc */
            if (wid == 0) {
                mv.status = st & 0xffff;
                mv.site = st >> 16;
                store_meta(meta, lane, mv, 0);
            }
            return;
        }
        negmask = (uint32_t)grec[1];
    }

    /* ---- candidate sums on MFMA ----
     * Exact mode: every block runs all NG + 1 groups and the LPC values are exact
     * (floor(T / 2^shift), one shift + one sad each).
     * Pruning mode (a.prune): every block runs the fixed group (exact: the fixed choice needs
     * exact sums); every other block of a wave also runs the LPC groups, but accumulates the
     * bound |T| (one sad).  For any subset S of a candidate's values
     *   sum_all |r| >= sum_S |r| >= sum_S (|T| / 2^s - 1) >= sum_lanes floor(acc / 2^s) - n,
     * since |floor(T / 2^s)| >= |T| / 2^s - (1 - 2^-s).  When that bound exceeds the best fixed
     * sum for every order, LPC loses strictly (encoder.py:135-157: no win, no tie) and its
     * exact sums are never needed.  Otherwise the LPC groups run again, exact, over every
     * block (a workgroup-uniform branch: every wave decides from the same LDS words). */
    const bool prune = NG > 0 && a.prune && !LIST;
    unsigned long long* red64 = reinterpret_cast<unsigned long long*>(smem + lay.red); /* [nw][4 groups][4 orders] */
    auto lane_total = [&]() __attribute__((always_inline)) -> uint64_t {
        /* lanes 1..4: fixed orders 1..4, lane 0: order 0 (sum|x|), lanes 16..15+4NG: LPC orders */
        uint64_t t = 0;
        int g = -1, o4l = 0;
        if (lane >= 1 && lane <= 4) {
            g = 0;
            o4l = lane - 1;
        } else if (NG > 0 && lane >= 16 && lane < 16 + 4 * NG) {
            g = 1 + ((lane - 16) >> 2);
            o4l = (lane - 16) & 3;
        }
        if (g >= 0) {
#pragma unroll 1
            for (int w2 = 0; w2 < nw; ++w2) t += red64[(w2 * 4 + g) * 4 + o4l];
        } else if (lane == 0) {
#pragma unroll 1
            for (int w2 = 0; w2 < nw; ++w2) t += red0[w2];
        }
        return t;
    };
    uint64_t tj = 0;
    bool pruned = false;
    {
        const int col = lane & 15, kb = lane >> 4, o4 = col >> 2, rho = col & 3;
        h8 B[NG + 1];
        int shg[NG + 1]; /* (kMagicBits >> shift is recomputed per block in exact mode: one VGPR per group fewer) */
        /* LPC groups: the lane's taps T[ia] .. T[ia-3] (ia = 12 + rho - 4 kb) are the halves
         * D[16 - ia] .. D[19 - ia] of its order's tap-table row: three dwords and two
         * v_alignbit.  The exactness bound (sum|c| + 2^shift) * 33023 < 2^22 is read off the
         * same registers: the lanes with rho = 0 hold disjoint windows [ia - 3, ia] covering
         * taps -3 .. 12, so their |halves| summed over kb give sum_m |T_p[m]|. */
        const uint32_t* tt = reinterpret_cast<const uint32_t*>(recl);
        const int k0 = 4 + 4 * kb - rho; /* 16 - ia */
        const uint32_t alb = 16u * (uint32_t)(k0 & 1);
        bool outside = false;
#pragma unroll
        for (int g = 0; g <= NG; ++g) {
            int sh = 0;
            if (g == 0) {
                B[0] = __builtin_bit_cast(h8, fixb);
            } else {
                const int p = 4 * (g - 1) + o4 + 1, wb = 10 * (p - 1) + (k0 >> 1);
                const uint32_t w0 = tt[wb], w1 = tt[wb + 1], w2 = tt[wb + 2];
                uint32_t l0 = __builtin_amdgcn_alignbit(w1, w0, alb), l2 = __builtin_amdgcn_alignbit(w2, w1, alb);
                if constexpr (LIST) {
                    /* pred-only taps: T_p[0] = -2^shift is half rho of (l0, l2) on the kb = 3 lanes
                     * (their window is T[rho] .. T[rho - 3]); the table keeps it (the shift is read
                     * from it below) */
                    const uint32_t keep = kb == 3 ? ((rho & 1) ? 0x0000ffffu : 0xffff0000u) : 0xffffffffu;
                    l0 &= rho < 2 ? keep : 0xffffffffu;
                    l2 &= rho >= 2 ? keep : 0xffffffffu;
                }
                const h2 k256{(_Float16)256.0f, (_Float16)256.0f};
                const uint32_t h0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(h2, l0) * k256);
                const uint32_t hh = __builtin_bit_cast(uint32_t, __builtin_bit_cast(h2, l2) * k256);
                B[g] = __builtin_bit_cast(h8, uint4{h0, hh, l0, l2});
                /* sum|T| of this window, then over the four kb rows (lanes 16 apart) */
                const h2 one{(_Float16)1.0f, (_Float16)1.0f};
                float sw = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, l0 & 0x7fff7fffu), one, 0.0f, false);
                sw = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, l2 & 0x7fff7fffu), one, sw, false);
                sw += __shfl_xor(sw, 16);
                sw += __shfl_xor(sw, 32);
                outside |= rho == 0 && p <= L && sw > (float)kCoefLimit;
                /* the shift from T_p[0] = -2^shift (half D[16], word 10 (p - 1) + 8) */
                const uint32_t t0 = tt[10 * (p - 1) + 8] & 0xffffu;
                sh = p <= L ? (int)((t0 >> 10) & 31u) - 15 : 0;
            }
            shg[g] = sh;
        }
        if (NG > 0 && __ballot(outside)) {
            /* outside the MFMA exactness bound: the list kernel (pred-only taps) redoes it, and a
             * unit outside that bound too goes to k_resid's list variant */
            if (tid == 0) {
                meta->status = FLACMI_STATUS_RETRY;
                if constexpr (LIST) {
                    const unsigned long long k = atomicAdd(a.retry2_count, 1ull);
                    a.retry2_list[k] = gid;
                } else { /* sub-list gid & 63: 64 counters on their own cache lines */
                    const int r = (int)(gid & 63);
                    const unsigned long long k = atomicAdd(a.retry_sub + 16 * r, 1ull);
                    a.retry_list[r * a.retry_sub_cap + (int64_t)k] = gid;
                }
            }
            return;
        }
        if (a.stop_after == 1) return;
        /* first residual index of group g's order at this lane (block 0 only) */
        auto start_of = [&](int g) __attribute__((always_inline)) -> int {
            const int p = 4 * (g > 0 ? g - 1 : 0) + o4 + 1;
            return (g > 0 && ((negmask >> (p - 1)) & 1)) ? 0 : p;
        };
        const uint32_t mbv = opaque_s(kMagicBits);
        const f4 C{12582912.0f, 12582912.0f, 12582912.0f, 12582912.0f};
        const int eoff = 4 * (lane & 15) - 12 + 4 * kb;
        uint32_t acc[NG + 1];
#pragma unroll
        for (int g = 0; g <= NG; ++g) acc[g] = 0;
        auto ld = [&](int blk) __attribute__((always_inline)) {
            return *reinterpret_cast<const uint2*>(xs + 64 * blk + eoff);
        };
        /* block 0 (masked, once per unit after the loop): its address recomputed from the
         * thread id, so no VGPR holds it across the loop (at 64 VGPRs one would spill) */
        auto ld0 = [&]() __attribute__((always_inline)) {
            const uint32_t t = opaque((uint32_t)tid);
            return *reinterpret_cast<const uint2*>(xs + 4 * (int)(t & 15) - 12 + 4 * (int)((t >> 4) & 3));
        };
        /* LIST: the samples of the lane's four values (block blk, rows 4 kb + r, phase rho), as
         * x - 2^31 (mod 2^32) from the biased x + 2^15 */
        auto ldx = [&](int blk, uint32_t (&xn)[4]) __attribute__((always_inline)) {
            if constexpr (LIST) {
                const uint16_t* xp = xs + 64 * blk + 16 * kb + rho;
#pragma unroll
                for (int r = 0; r < 4; ++r) xn[r] = (uint32_t)xp[4 * r] + 0x7FFF8000u;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) xn[r] = 0u;
            }
        };
        /* an exact LPC value's |r|: floor(T / 2^s) = (bits >> s) - (M >> s) with the x tap in B;
         * LIST: (bits >> s) - (M >> s) = floor(pred / 2^s), and (bits >> s) - (x - 2^31) =
         * (M >> s) - r + 2^31, so |r| is one v_sad_u32 against (M >> s) + 2^31 */
        auto lpc_abs = [&](uint32_t bits, int sh, uint32_t kgv, uint32_t xn, uint32_t acc) __attribute__((always_inline)) {
            return LIST ? sad32((bits >> sh) - xn, kgv + 0x80000000u, acc) : sad32(bits >> sh, kgv, acc);
        };
        /* one 64-sample block through the MFMAs of groups G0..G1; EX: LPC values exact, else
         * the bound |T| */
        auto blockA = [&](auto g0c, auto g1c, auto exc, const uint4 Ar, bool masked, const uint32_t (&xn)[4]) __attribute__((always_inline)) {
            constexpr int G0 = decltype(g0c)::value, G1 = decltype(g1c)::value;
            constexpr bool EX = decltype(exc)::value != 0;
            f4 D[NG + 1];
            h8 A{};
            if constexpr (G1 >= 1) A = a_sub(Ar);
#pragma unroll
            for (int g = G0; g <= G1; ++g)
                D[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(g == 0 ? __builtin_bit_cast(h8, Ar) : A, B[g], C, 0, 0, 0);
#pragma unroll
            for (int g = G0; g <= G1; ++g) {
                const uint32_t kgv = kMagicBits >> shg[g];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    /* (a bit_cast of a vector element reads element 0: clang bug) */
                    const uint32_t bits = __float_as_uint(D[g][r]);
                    if (masked) {
                        const int i = 4 * (4 * kb + r) + rho; /* block 0 */
                        const uint32_t sv =
                            (g == 0 || !EX) ? sad32(bits, mbv, 0u) : lpc_abs(bits, shg[g], kgv, xn[r], 0u);
                        acc[g] += i >= start_of(g) ? sv : 0u;
                    } else if (g == 0 || !EX) { /* opaque: one v_sad_u32 per value, not a reassociated min/max/sub */
                        acc[g] = opaque(sad32(bits, mbv, acc[g]));
                    } else {
                        acc[g] = lpc_abs(bits, shg[g], kgv, xn[r], acc[g]);
                    }
                }
            }
        };
        auto block = [&](auto g0c, auto g1c, auto exc, uint2 q, bool masked, int blk) __attribute__((always_inline)) {
            uint32_t xn[4];
            ldx(blk, xn);
            blockA(g0c, g1c, exc, a_raw(q), masked, xn);
        };
        const uint32_t xnone[4] = {0u, 0u, 0u, 0u};
        /* per (group, order): sum over the 4 phases (quad, < 2^32) then, in 64 bits, over the
         * 4 kb rows; the lanes with rho == 0 and kb == 0 store.  BD: the LPC groups hold the
         * bound sum |T|, stored as floor(acc / 2^shift) per lane (a lower bound of the sum of
         * |T| / 2^shift; acc itself keeps accumulating over later tiers) */
        auto reduce_store = [&](auto g0c, auto bdc) __attribute__((always_inline)) {
            constexpr int G0 = decltype(g0c)::value;
            constexpr bool BD = decltype(bdc)::value != 0;
#pragma unroll
            for (int g = G0; g <= NG; ++g) {
                uint32_t v = (BD && g > 0) ? acc[g] >> shg[g] : acc[g];
                v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
                v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);
                uint64_t w = v;
                w += (uint64_t)(uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F); /* lane ^ 16 */
                w += __shfl_xor((unsigned long long)w, 32);
                if (rho == 0 && kb == 0) red64[(wid * 4 + g) * 4 + o4] = w;
            }
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using ING = std::integral_constant<int, NG>;
        /* this wave's blocks wid + k nw, k = 0 .. kw - 1 (wave 0 takes block 0 masked, last) */
        const int kw = (nblk - wid + nw - 1) / nw;
        if (prune) {
            /* tier 0: the wave's blocks k % 4 == 0 run the LPC groups (bound) beside the fixed
             * group; tiers 1..3 (only while the bound has not decided) add k % 4 == 2, 1, 3 */
            const bool no_lpc = a.stop_after == 12; /* ablation (timing only): no LPC bound at all */
            for (int k = wid == 0 ? 1 : 0; k < kw; ++k) {
                const uint4 A = a_raw(ld(wid + k * nw));
                blockA(I0{}, I0{}, I0{}, A, false, xnone);
                if ((k & 3) == 0 && !no_lpc) blockA(I1{}, ING{}, I0{}, A, false, xnone);
            }
            if (wid == 0) block(I0{}, ING{}, I0{}, ld0(), true, 0);
            reduce_store(I0{}, I1{});
        } else {
            for (int blk = wid == 0 ? nw : wid; blk < nblk; blk += nw) block(I0{}, ING{}, I1{}, ld(blk), false, blk);
            if (wid == 0) block(I0{}, ING{}, I1{}, ld0(), true, 0);
            reduce_store(I0{}, I0{});
            if constexpr (LIST) mv.tiers = 1 | (1 << 8); /* one exact pass (the listed units' marker) */
        }
        __syncthreads(); /* B2 */
        STAMP(3);
        tj = lane_total();
        if constexpr (NG > 0) {
            if (prune) {
                /* best fixed sum (exact) against every LPC order's lower bound */
                uint64_t fk = (lane <= 4) ? (tj << 4) | (uint64_t)lane : ~0ull;
                fk = dpp_min_u64<0xB1>(fk);
                fk = dpp_min_u64<0x4E>(fk);
                fk = dpp_min_u64<0x141>(fk);
                fk = dpp_min_u64<0x140>(fk);
                const uint64_t fmin = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fk >> 32), 0) << 28) |
                                      ((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fk, 0) >> 4);
#pragma unroll 1
                for (int t = 1;; ++t) {
                    const uint64_t lb = tj > (uint64_t)n ? tj - (uint64_t)n : 0ull;
                    const uint64_t open = __ballot(lane >= 16 && lane < 16 + L && lb <= fmin);
                    pruned = open == 0 || a.stop_after >= 11; /* 11, 12: ablation, tier 0 only */
                    mv.tiers = t | (4 << 8);
                    if (pruned || t == 4) break;
                    /* the next quarter of the blocks (k % 4 == 2, 1, 3; block 0 is in tier 0), only
                     * for the groups that hold an undecided order (mostly order 1's) */
                    const uint32_t gneed = (uint32_t)(open >> 16);
                    __syncthreads(); /* every wave has read the bounds */
                    for (int k = t == 1 ? 2 : t == 2 ? 1 : 3; k < kw; k += 4) {
                        const h8 A = a_sub(a_raw(ld(wid + k * nw)));
#pragma unroll
                        for (int g = 1; g <= NG; ++g) {
                            if ((gneed >> (4 * (g - 1))) & 15u) {
                                const f4 D = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B[g], C, 0, 0, 0);
#pragma unroll
                                for (int r = 0; r < 4; ++r) acc[g] = opaque(sad32(__float_as_uint(D[r]), mbv, acc[g]));
                            }
                        }
                    }
                    reduce_store(I1{}, I1{});
                    __syncthreads();
                    tj = lane_total();
                }
                if (!pruned) { /* rare: the exact LPC sums over every block */
                    mv.tiers = 5 | (4 << 8);
                    __syncthreads(); /* every wave has read the bounds */
#pragma unroll
                    for (int g = 1; g <= NG; ++g) acc[g] = 0;
                    for (int blk = wid == 0 ? nw : wid; blk < nblk; blk += nw) block(I1{}, ING{}, I1{}, ld(blk), false, blk);
                    if (wid == 0) block(I1{}, ING{}, I1{}, ld0(), true, 0);
                    reduce_store(I1{}, I0{});
                    __syncthreads();
                    tj = lane_total();
                }
            }
        }
    }
    if (a.stop_after == 2) return;

    /* ---- choice (encoder.py:331-359, 398-404, 135-157), every wave, lane-parallel ----
     * lanes 0..4: fixed orders 0..4; lanes 16..15+L: LPC orders 1..L.  Key = sum * 16 + index,
     * so a row's minimum key is its smallest sum at the lowest order (python min(): the first
     * minimum); four DPP steps reduce each 16-lane row. */
    const bool cand = lane <= 4 || (!pruned && lane >= 16 && lane < 16 + L);
    uint64_t key = cand ? (tj << 4) | (uint64_t)(lane & 15) : ~0ull;
    key = dpp_min_u64<0xB1>(key);  /* quad_perm [1,0,3,2] */
    key = dpp_min_u64<0x4E>(key);  /* quad_perm [2,3,0,1] */
    key = dpp_min_u64<0x141>(key); /* row_half_mirror */
    key = dpp_min_u64<0x140>(key); /* row_mirror */
    auto key_at = [&](int j) __attribute__((always_inline)) -> uint64_t {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), j) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, j);
    };
    const uint64_t fkey = key_at(0);
    const int fo = (int)(fkey & 15);
    const uint64_t fsum = fkey >> 4;
    int lbest = 0;
    uint64_t lsum = 0;
    bool lpc_wins = false, tie = false;
    if constexpr (NG > 0) {
        if (pruned) {
            lbest = FLACMI_LPC_PRUNED;
            lsum = (uint64_t)(int64_t)FLACMI_LPC_PRUNED;
        } else {
            const uint64_t lkey = key_at(16);
            lbest = (int)(lkey & 15) + 1;
            lsum = lkey >> 4;
            /* a coefficient-less candidate sums |x| over all n (= the fixed order-0 sum), so it
             * never wins strictly */
            lpc_wins = lsum < fsum;
            tie = !lpc_wins && !(fsum < lsum);
        }
    }
    if (wid == 0 && a.fixed_sums && lane < 5) a.fixed_sums[gid * 5 + lane] = (long long)tj;
    if (wid == 0 && a.lpc_sums) {
        const uint64_t v = (uint64_t)__shfl((unsigned long long)tj, (lane + 16) & 63);
        if (lane < 32) a.lpc_sums[gid * 32 + lane] = (lane + 1 <= L) ? (long long)v : 0;
    }
    mv.fixed_order = fo;
    mv.lpc_order = lbest;
    mv.fixed_sum = (long long)fsum;
    mv.lpc_sum = (long long)lsum;
    if (tie) {
        if (wid == 0) {
            mv.status = ST_ASSERT;
            mv.site = FLACMI_SITE_CHOICE_TIE;
            store_meta(meta, lane, mv, 0);
        }
        return;
    }
    int32_t coefl = 0; /* lane q: coefficient q of the chosen LPC order */
    mv.kind = lpc_wins ? FLACMI_KIND_LPC : FLACMI_KIND_FIXED;
    mv.order = lpc_wins ? lbest : fo;
    if constexpr (NG > 0) {
        if (lpc_wins) {
            mv.shift = grec[2 + lbest - 1];
            mv.ncoefs = lbest;
            if (lane < lbest) coefl = grec[2 + L + (lbest * (lbest - 1)) / 2 + lane];
        }
    }
    if (a.stop_after == 3) return;
    STAMP(4);

    /* ---- chosen residual: zig-zag (utils.py:91-94) to HBM; kept in registers as 16-bit
     * pairs when every value of the chunk is < 2^16 (else recomputed for the Rice pass);
     * finest partition sums by LDS atomics ---- */
    const int order = mv.order;
    int omax = R05 ? 5 : -1;
    if constexpr (!R05)
        for (int o = a.rmin; o <= a.rmax; ++o)
            if ((n % (1 << o)) == 0 && (n >> o) > order) omax = o;
    const int P = 1 << (omax < 0 ? 0 : omax), cpp = (n >> (omax < 0 ? 0 : omax)) >> 3;
    /* finest partition of chunk c = floor(c / cpp) = mulhi(c, ceil(2^32 / cpp)): exact for c * cpp < 2^32 */
    const uint32_t mcpp = (uint32_t)((0x100000000ull + (uint64_t)cpp - 1) / (uint64_t)cpp);
    auto part_of = [&](int c) __attribute__((always_inline)) -> int { return (int)__umulhi((uint32_t)c, mcpp); };
    uint32_t* __restrict__ rout = reinterpret_cast<uint32_t*>(a.residual) + gid * a.residual_stride;
    const int fixed_k = __builtin_amdgcn_readfirstlane(lpc_wins ? -1 : order);
    const int lsh = mv.shift;
    auto resid = [&](int c, uint32_t (&z)[8]) __attribute__((always_inline)) {
        switch (fixed_k) {
            case 0: fixed_chunk<0>(xs, 8 * c, z); break;
            case 1: fixed_chunk<1>(xs, 8 * c, z); break;
            case 2: fixed_chunk<2>(xs, 8 * c, z); break;
            case 3: fixed_chunk<3>(xs, 8 * c, z); break;
            case 4: fixed_chunk<4>(xs, 8 * c, z); break;
            default:
                if constexpr (NG > 0) lpc_chunk(xs, 8 * c, coefl, lsh, order, z);
                break;
        }
    };
    const bool pairs = (cpp & 1) == 0 && a.stop_after != 9;
    uint32_t zp[kSCPT][4]; /* 16-bit pairs of the chunk's residual */
    uint32_t big = 0;     /* bit j: chunk j holds a value >= 2^16 */
    /* one copy of the chunk loop per predictor (the switch is taken once, not per chunk) */
    auto residual_pass = [&](auto kk) __attribute__((always_inline)) {
        constexpr int KK = decltype(kk)::value;
#pragma unroll
        for (int j = 0; j < kSCPT; ++j) {
            const int c = tid + j * NT;
            zp[j][0] = zp[j][1] = zp[j][2] = zp[j][3] = 0;
            if (c < nch) {
                uint32_t z[8];
                if (j == 0) fixed_chunk<KK, true>(xs, 8 * c, z);
                else fixed_chunk<KK, false>(xs, 8 * c, z);
                store_row(rout + 8 * c, z);
                uint32_t cs = z[0] + z[1] + z[2] + z[3] + z[4] + z[5] + z[6] + z[7];
                /* chunks 2m and 2m + 1 (lanes l and l ^ 1) share a finest partition when it
                 * holds an even number of chunks: one lane adds both, halving the same-address
                 * LDS atomics (stop_after 9: every lane adds, 10: none; timing only) */
                if (pairs) cs += dpp_u32<0xB1, 0xf>(cs);
                if (omax >= 0 && a.stop_after != 10 && (!pairs || (lane & 1) == 0)) atomicAdd(&pks[part_of(c)], cs);
                if ((z[0] | z[1] | z[2] | z[3] | z[4] | z[5] | z[6] | z[7]) >> 16) big |= 1u << j;
#pragma unroll
                for (int i = 0; i < 4; ++i) zp[j][i] = __builtin_amdgcn_perm(z[2 * i + 1], z[2 * i], 0x05040100u);
            }
        }
    };
    /* the LPC predictor (rare: it wins only where the reference's sign convention lets it):
     * one chunk per iteration, not unrolled, every chunk marked for the Rice pass's recompute
     * path (code size: one inlined copy of the 12-tap predictor instead of kSCPT) */
    auto residual_pass_lpc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < kSCPT; ++j) zp[j][0] = zp[j][1] = zp[j][2] = zp[j][3] = 0;
#pragma unroll 1
        for (int j = 0; j < kSCPT; ++j) {
            const int c = tid + j * NT;
            if (c < nch) {
                uint32_t z[8];
                lpc_chunk(xs, 8 * c, coefl, lsh, order, z);
                reinterpret_cast<uint4*>(rout + 8 * c)[0] = uint4{z[0], z[1], z[2], z[3]};
                reinterpret_cast<uint4*>(rout + 8 * c)[1] = uint4{z[4], z[5], z[6], z[7]};
                const uint32_t cs = z[0] + z[1] + z[2] + z[3] + z[4] + z[5] + z[6] + z[7];
                if (omax >= 0) atomicAdd(&pks[part_of(c)], cs);
                big |= 1u << j;
            }
        }
    };
    switch (fixed_k) {
        case 0: residual_pass(std::integral_constant<int, 0>{}); break;
        case 1: residual_pass(std::integral_constant<int, 1>{}); break;
        case 2: residual_pass(std::integral_constant<int, 2>{}); break;
        case 3: residual_pass(std::integral_constant<int, 3>{}); break;
        case 4: residual_pass(std::integral_constant<int, 4>{}); break;
        default:
            if constexpr (NG > 0) residual_pass_lpc();
            break;
    }
    __syncthreads(); /* B3 */
    STAMP(5);
    if (a.stop_after == 4) return;

    /* ---- Rice partition search (encoder.py:655-760) ---- */
    if (omax < 0) {
        if (wid == 0) {
            mv.status = ST_ASSERT;
            mv.site = FLACMI_SITE_RICE_NO_ORDER;
            store_meta(meta, lane, mv, coefl);
        }
        return;
    }
    const int ro = R05 ? 0 : __builtin_amdgcn_readfirstlane(a.rmin), oo = R05 ? 5 : __builtin_amdgcn_readfirstlane(omax);
    /* wave 0 only (the other waves wait at the barrier below, their SIMD slots going to other
     * workgroups): lane j - 1 = heap node j = (order o, partition K), j = 2^o + K < 2P <= 64:
     * node sums from a prefix over the finest sums, one parameter each, the first error in
     * the reference's evaluation order = the lowest node (orders ascending, then partitions) */
    /* 32 bits: the chosen predictor's sum|r| is at most the order-0 sum n * 2^15, so its
     * zig-zag total stays below 2 * 10240 * 2^15 + n < 2^32 */
    const int j = lane + 1;
    const int o = 31 - __builtin_clz((unsigned)j);
    const int K = j - (1 << o), dd = oo - o;
    const bool valid = j < 2 * P && o >= ro;
    const int len = (n >> (o < 16 ? o : 15)) - (K == 0 ? order : 0);
    int prm = 0;
    uint32_t* const eflag = red0; /* free after B2's reads */
    if (wid == 0) {
        uint32_t pre = lane < P ? pks[lane] : 0u;
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)pre, (unsigned)d);
            if (lane >= d) pre += t;
        }
        const int hi_k = ((K + 1) << (dd < 0 ? 0 : dd)) - 1, lo_k = (K << (dd < 0 ? 0 : dd)) - 1;
        const uint32_t ph = (uint32_t)__shfl((int)pre, hi_k & 63);
        const uint32_t pl = (uint32_t)__shfl((int)pre, lo_k & 63);
        const uint32_t snode = ph - (lo_k >= 0 ? pl : 0u);
        const bool zero = snode == 0;
        prm = (zero || !valid) ? 0 : rice_param_exact((uint64_t)snode, len);
        const unsigned long long eb = __ballot(valid && (zero || prm < 0));
        if (lane == 0) eflag[0] = eb != 0;
        if (eb) {
            const int kl = __builtin_ctzll(eb);
            mv.status = ST_VALUE;
            mv.site = __shfl((int)zero, kl) ? FLACMI_SITE_RICE_LOG_DOMAIN : FLACMI_SITE_RICE_NEG_SHIFT;
            store_meta(meta, lane, mv, coefl);
        } else {
            /* the table: finest partition k (lane k) -> the parameter of its ancestor at
             * every order, as p | p << 16 */
            int pmax = 0;
            /* (opaque: lane * 16 bytes would otherwise be shared with the staging's kFixB offset and
             * held, or spilled, across the whole kernel) */
            uint16_t* const prow = pkw + (int)opaque((uint32_t)lane) * RS;
#pragma unroll
            for (int o2 = 0; o2 < kRiceOrders; ++o2) {
                if (o2 >= ro && o2 <= oo) {
                    const int node = (1 << o2) + (lane >> (oo - o2));
                    const int pv = __shfl(prm, (node - 1) & 63);
                    pmax = max(pmax, pv);
                    if (lane < P) prow[o2] = (uint16_t)pv;
                }
            }
            /* bit 15 of a row's entry 0 (order 0's parameter, or unused when rmin > 0): some order's
             * parameter is >= 16, which v_pk_lshrrev_b16 would take mod 16, so the row's chunks take
             * the 32-bit path (possible only where a partition's mean is >= 2^16 while one of its
             * chunks stays below 2^16) */
            if (lane < P) {
                if (ro > 0) prow[0] = pmax >= 16 ? 0x8000u : 0u;
                else if (pmax >= 16) prow[0] |= 0x8000u;
            }
        }
    }
    __syncthreads(); /* B3b: the table and the error flag */
    if (eflag[0]) return; /* workgroup-uniform */
    /* data bits: sum of x >> p over the residual for every candidate order */
    uint32_t tb[kRiceOrders];
#pragma unroll
    for (int o2 = 0; o2 < kRiceOrders; ++o2) tb[o2] = 0;
#pragma unroll
    for (int jc = 0; jc < kSCPT; ++jc) {
        const int c = tid + jc * NT;
        if (c < nch) {
            const int k = part_of(c);
            uint32_t pw[kRiceOrders / 2];
            load_ptab(pkw + k * RS, pw);
            big |= ((pw[0] >> 15) & 1u) << jc; /* a parameter >= 16 in this chunk's row */
            if (!((big >> jc) & 1)) {
#pragma unroll
                for (int o2 = 0; o2 < kRiceOrders; ++o2)
                    if (o2 >= ro && o2 <= oo) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t sh = (o2 & 1) ? pk_shr_bcast<1>(pw[o2 >> 1], zp[jc][i])
                                                         : pk_shr_bcast<0>(pw[o2 >> 1], zp[jc][i]);
                            tb[o2] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, sh), us2{1, 1}, tb[o2], false);
                        }
                    }
            }
        }
    }
    /* rare: chunks holding a value >= 2^16 recompute their residual, in one loop that is not
     * unrolled (one inlined copy of the six predictors instead of one per chunk slot: the
     * kernel's code, and its instruction-cache footprint, shrink by a third) */
    if (big) {
#pragma unroll 1
        for (int jc = 0; jc < kSCPT; ++jc) {
            if (!((big >> jc) & 1)) continue;
            const int c = tid + jc * NT;
            const int k = part_of(c);
            uint32_t pw[kRiceOrders / 2];
            load_ptab(pkw + k * RS, pw);
            uint32_t z[8];
            resid(c, z);
#pragma unroll
            for (int o2 = 0; o2 < kRiceOrders; ++o2)
                if (o2 >= ro && o2 <= oo) {
                    const uint32_t sh = (pw[o2 >> 1] >> (16 * (o2 & 1))) & 0x7fffu;
                    tb[o2] += (z[0] >> sh) + (z[1] >> sh) + (z[2] >> sh) + (z[3] >> sh) + (z[4] >> sh) +
                              (z[5] >> sh) + (z[6] >> sh) + (z[7] >> sh);
                }
        }
    }
    {
        uint32_t any = 0;
#pragma unroll
        for (int o2 = 0; o2 < kRiceOrders; ++o2) any |= (o2 >= ro && o2 <= oo) ? tb[o2] : 0u;
        /* a wave-uniform branch, not a select: the 64-bit reduction (never taken by 16-bit
         * data) would otherwise run beside the 32-bit one for every order */
        if (__ballot(any >= (1u << 26)) == 0) {
            /* DPP row reductions; lane 63 holds the wave total and stores it (no readlane) */
#pragma unroll
            for (int o2 = 0; o2 < kRiceOrders; ++o2)
                if (o2 >= ro && o2 <= oo) {
                    uint32_t v = tb[o2];
                    v += dpp_u32<0xB1, 0xf>(v);
                    v += dpp_u32<0x4E, 0xf>(v);
                    v += dpp_u32<0x141, 0xf>(v);
                    v += dpp_u32<0x140, 0xf>(v);
                    v += dpp_u32<0x142, 0xa>(v);
                    v += dpp_u32<0x143, 0xc>(v);
                    if (lane == 63) red2[wid * kRiceOrders + o2] = v;
                }
        } else {
#pragma unroll 1
            for (int o2 = ro; o2 <= oo; ++o2) {
                uint32_t t = 0;
#pragma unroll
                for (int o3 = 0; o3 < kRiceOrders; ++o3) t = o3 == o2 ? tb[o3] : t;
                const uint64_t w = wave_sum_u64(t);
                if (lane == 0) red2[wid * kRiceOrders + o2] = w;
            }
        }
    }
    __syncthreads(); /* B4 */
    STAMP(6);
#if defined(FLACMI_PAD_VALU) /* diagnostic build only: extra independent VALU per unit (price of issue) */
    {
        uint32_t q0 = lane, q1 = lane ^ 5u, q2 = lane * 3u, q3 = lane + 7u;
#pragma unroll
        for (int i = 0; i < FLACMI_PAD_VALU / 8; ++i)
            asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                         : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(lane));
        if ((q0 ^ q1 ^ q2 ^ q3) == 0xdeadbeefu) meta->lpc_tiers = 1;
    }
#endif
#if defined(FLACMI_PAD_SALU) /* diagnostic build only: extra SALU per unit */
    {
        uint32_t q0 = (uint32_t)gid, q1 = (uint32_t)gid ^ 5u;
#pragma unroll
        for (int i = 0; i < FLACMI_PAD_SALU / 4; ++i)
            asm volatile("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5" : "+s"(q0), "+s"(q1));
        if ((q0 ^ q1) == 0xdeadbeefu) meta->lpc_tiers = 1;
    }
#endif
    if (wid != 0) return;
    /* wave 0: headers per order (lanes of that order's nodes), totals, first minimum */
    const uint32_t hb = valid ? 4u + (prm > 14 ? 5u : 4u) + (uint32_t)len * (uint32_t)(1 + prm) : 0u;
    const unsigned long long m14 = __ballot(valid && prm > 14);
    unsigned long long bb = 0;
    int best = -1;
    uint32_t m5 = 0;
#pragma unroll
    for (int o2 = 0; o2 < kRiceOrders; ++o2)
        if (o2 >= ro && o2 <= oo) {
            const uint32_t ht = wave_sum_u32(o == o2 ? hb : 0u);
            unsigned long long v = ht;
#pragma unroll 1
            for (int w2 = 0; w2 < nw; ++w2) v += red2[w2 * kRiceOrders + o2];
            if (best < 0 || v < bb) {
                bb = v;
                best = o2;
            }
            const unsigned long long om = ((1ull << (1 << o2)) - 1) << ((1 << o2) - 1); /* lanes of order o2 */
            if (m14 & om) m5 |= 1u << o2;
        }
    mv.status = ST_OK;
    mv.res_offset = order;
    mv.res_len = n - order;
    mv.part_order = best;
    mv.n_parts = 1 << best;
    mv.coding = ((m5 >> best) & 1) ? 5 : 4;
    mv.rice_bits = (long long)bb;
    store_meta(meta, lane, mv, coefl);
#if FLACMI_STREAM_STAMPS
    STAMP(7);
    {
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v = lane == k ? stamp[k] : v;
        if (a.lpc_sums && lane < 8) a.lpc_sums[gid * 32 + 24 + lane] = (long long)v;
        if (a.fixed_sums && lane < 2) a.fixed_sums[gid * 5 + 3 + lane] = (long long)(lane ? rt1 : rt0);
    }
#endif
    int32_t* __restrict__ rp = a.rice_params + gid * a.params_stride;
    if (lane < (1 << best)) rp[lane] = (int32_t)(pkw[(lane << (oo - best)) * RS + best] & 0x7fffu);
}

typedef const __attribute__((address_space(4))) ResidArgs* StreamKernarg;

/* one workgroup per unit of the batch */
template <int NG, bool R05, int NFIX = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R05 ? 8 : 7, 8))) void k_resid_stream(ResidArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    stream_unit<NG, R05, NFIX, false>(a, blockIdx.x, smem);
}

/* the units k_resid_stream listed (a.retry_list), pred-only taps: a fixed grid whose
 * workgroups loop over the list (its length is known only on the device); an empty list costs
 * one scalar load per workgroup */
template <int NG, bool R05, int NFIX = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_resid_stream_list(ResidArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    /* the batch kernel's 64 sub-lists: lane r holds the inclusive prefix of their lengths */
    const int lane = threadIdx.x & 63;
    uint32_t incl = (uint32_t)a.retry_sub[16 * lane];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, (unsigned)d);
        if (lane >= d) incl += t;
    }
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        /* the arguments through the kernarg pointer, opaque per unit: hoisted out of the loop,
         * every field would stay live in registers across it */
        StreamKernarg pa = (StreamKernarg)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(pa));
        const int r = __builtin_popcountll(__ballot(incl <= k)); /* incl[r - 1] <= k < incl[r] */
        const uint32_t base = r > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)incl, r - 1) : 0u;
        stream_unit<NG, R05, NFIX, true>(*pa, pa->retry_list[r * pa->retry_sub_cap + (k - base)], smem);
        __syncthreads(); /* every wave is done with this unit's LDS */
    }
}

/* units the list kernel could not take (sum|c| > 127) are handled by k_resid's list variant,
 * see launch_resid_list in k_resid.h */
hipError_t launch_resid_retry_l8(const ResidArgs& a, hipStream_t s);
hipError_t launch_resid_retry_l12(const ResidArgs& a, hipStream_t s);

bool stream_shape_ok(const ResidArgs& a, int path, int residual_bytes) {
    if (!a.stream || path != 0 || residual_bytes != 4 || a.sample_bytes != 2 || !a.mfma || !a.retry_list || !a.retry_count ||
        !a.retry2_list || !a.retry2_count || !a.retry_sub)
        return false;
    const bool ref = a.mode == FLACMI_MODE_REFERENCE && a.L >= 1 && a.L <= 12;
    if (!ref && a.mode != FLACMI_MODE_FIXED_ONLY) return false;
    if (a.n % 64 != 0 || a.n < 64 || a.n > 8 * kSCPT * 256) return false;
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    if (rmax_eff < 0 || (1 << rmax_eff) > 32 || ((a.n >> rmax_eff) & 7) != 0) return false; /* heap nodes < 64 */
    return true;
}

/* the list kernel's grid: 16 workgroups per CU (the batch kernel's residency) */
static unsigned stream_list_grid(int64_t count) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
        ncu = 256;
    const int64_t g = 16 * (int64_t)ncu;
    return (unsigned)(count < g ? count : g);
}

template <int NG, bool R05, int NFIX>
static hipError_t launch_stream_K(const ResidArgs& a, bool list, hipStream_t s) {
    const int nt = NFIX ? stream_threads(NFIX) : stream_threads(a.n);
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const size_t lds = stream_lds(a.n, nt / 64, tap_table_words(NG), 1 << rmax_eff, kRiceOrders).total;
    auto kern = list ? k_resid_stream_list<NG, R05, NFIX> : k_resid_stream<NG, R05, NFIX>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(list ? stream_list_grid(a.count) : (unsigned)a.count), dim3(nt), lds, s, a);
    return hipGetLastError();
}

template <int NG, bool R05>
static hipError_t launch_stream_R(const ResidArgs& a, bool list, hipStream_t s) {
    if constexpr (R05) /* the BASELINE configs' 4608-sample units at L = 4 NG: the constant-shape build */
        if (a.n == 4608 && (NG == 0 || a.L == 4 * NG) && knob(kKnobStreamGeneric) == 0)
            return launch_stream_K<NG, true, 4608>(a, list, s);
    return launch_stream_K<NG, R05, 0>(a, list, s);
}

template <int NG>
static hipError_t launch_stream_T(const ResidArgs& a, bool list, hipStream_t s) {
    /* partition orders 0..5 for every unit: rmin 0, rmax_eff 5 and n / 32 above the largest
     * predictor order (4 fixed, L for LPC) */
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int maxord = NG > 0 && a.L > 4 ? a.L : 4;
    if (a.rmin == 0 && rmax_eff == 5 && (a.n >> 5) > maxord) return launch_stream_R<NG, true>(a, list, s);
    return launch_stream_R<NG, false>(a, list, s);
}

static hipError_t launch_stream_G(const ResidArgs& a, bool list, hipStream_t s) {
    if (a.mode == FLACMI_MODE_FIXED_ONLY) return launch_stream_T<0>(a, list, s);
    if (a.L <= 4) return launch_stream_T<1>(a, list, s);
    if (a.L <= 8) return launch_stream_T<2>(a, list, s);
    return launch_stream_T<3>(a, list, s);
}

/* the batch, then (reference mode) the units it listed through the list kernel (pred-only
 * taps), then the units that one listed through k_resid's list variant */
hipError_t launch_resid_stream(const ResidArgs& a_in, hipStream_t s) {
    ResidArgs a = a_in;
    a.retry_sub_cap = (a.count + 63) / 64; /* sub-list u & 63 holds at most ceil(count / 64) units */
    hipError_t e = hipMemsetAsync(a.retry_sub, 0, 64 * 16 * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if ((e = launch_stream_G(a, false, s)) != hipSuccess) return e;
    if (a.mode == FLACMI_MODE_FIXED_ONLY) return hipSuccess; /* nothing is ever listed */
    if ((e = hipMemsetAsync(a.retry2_count, 0, sizeof(unsigned long long), s)) != hipSuccess) return e;
    if ((e = launch_poison_lds(s)) != hipSuccess) return e;
    if ((e = launch_stream_G(a, true, s)) != hipSuccess) return e;
    if ((e = launch_poison_lds(s)) != hipSuccess) return e;
    ResidArgs b = a;
    b.retry_count = a.retry2_count;
    b.retry_list = a.retry2_list;
    return a.L <= 8 ? launch_resid_retry_l8(b, s) : launch_resid_retry_l12(b, s);
}

}  // namespace flacmi
