/* k_resid.h — fixed + LPC candidate residual sums, choice, chosen residual and Rice
 * search, one workgroup per unit (see device_common.h for the design notes).
 * Instantiated per LPC-order bucket in k_resid_l*.hip so the builds run in parallel.
 *
 * Three arithmetic paths, chosen on the host from exact magnitude bounds:
 *   PATH_S16  int16 samples staged in LDS as packed pairs; every LPC prediction is
 *             ceil(p/2) v_dot2_i32_i16 on (x[i-2-2t], x[i-1-2t]) x (c[2t+1], c[2t]),
 *             coefficient pairs broadcast from LDS.  |r| sums: one v_sad_u32 each on
 *             sign-biased operands.  (16-bit samples, q <= 16, |r| < 2^26.)
 *   PATH_N32  int32 samples, v_mad_i32_i24 predictions (samples and q <= 24 bits).
 *   PATH_W64  int32 samples, int64 predictions and sums (anything else).
 *   PATH_W64S PATH_W64 with the LPC candidate predictions on v_dot2_i32_i16 over two
 *             12-bit sample planes (samples <= 24 bits, q <= 16, host-checked bound);
 *             the recombination, shift and |r| sums stay int64.
 * Samples and the zig-zag residual live in separate LDS regions, so the chosen residual
 * is written to LDS and HBM in the same pass. */
#pragma once
#include "device_common.h"

namespace flacmi {

enum { PATH_S16 = 0, PATH_N32 = 1, PATH_W64 = 2, PATH_W64S = 3 };

typedef short short2v __attribute__((ext_vector_type(2)));
typedef unsigned short us2x __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int32_t sdot2(uint32_t a, uint32_t b, int32_t c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, a), __builtin_bit_cast(short2v, b), c, false);
}
__device__ __forceinline__ int32_t sext24(int32_t v) { return (v << 8) >> 8; }

/* ---------------------------------------------------------------------------------------
 * PATH_S16: a chunk = 8 samples i0..i0+7 with the HP samples before it, as packed pairs
 *   E[m] = (x[i0-HP+2m] lo, x[i0-HP+2m+1] hi),  O[m] = (x[i0-HP+2m+1], x[i0-HP+2m+2]).
 * ------------------------------------------------------------------------------------- */
template <int HP>
struct Win16 {
    static constexpr int NE = (HP + 8) / 2; /* aligned pairs */
    uint32_t E[NE];
    uint32_t O[NE - 1];
    int32_t x[12]; /* samples i0-4 .. i0+7 as int32 */
    __device__ __forceinline__ void load(const int16_t* xs16, int i0) {
        const uint4* src = reinterpret_cast<const uint4*>(xs16 + i0 - HP); /* 16-B aligned */
#pragma unroll
        for (int g = 0; g < NE / 4; ++g) {
            const uint4 v = src[g];
            E[4 * g + 0] = v.x;
            E[4 * g + 1] = v.y;
            E[4 * g + 2] = v.z;
            E[4 * g + 3] = v.w;
        }
#pragma unroll
        for (int m = 0; m < NE - 1; ++m) O[m] = __builtin_amdgcn_alignbit(E[m + 1], E[m], 16);
#pragma unroll
        for (int t = 0; t < 12; ++t) {
            const int pos = HP - 4 + t; /* window position */
            const uint32_t pr = E[pos >> 1];
            x[t] = (pos & 1) ? ((int32_t)pr >> 16) : (int32_t)(int16_t)(pr & 0xffff);
        }
    }
    /* (x[i-1-2t] lo, x[i-2t] hi) for the sample i at window position HP + k.  Position -1
     * only occurs as the lo half of the last pair of an even LMAX = HP, whose coefficient is 0. */
    __device__ __forceinline__ uint32_t pair(int k, int t) const {
        const int lo = HP + k - 1 - 2 * t;
        if (lo < 0) return E[0] << 16;
        return (lo & 1) ? O[(lo - 1) >> 1] : E[lo >> 1];
    }
};

/* fixed orders 0..4 from the 12 samples x[i0-4 .. i0+7] (shared by all paths), with
 * running differences: per sample 4 subtractions, 4 bias xors and 5 v_sad_u32. */
template <bool MASKED, typename A>
__device__ __forceinline__ void fixed_sums32(const int32_t (&x)[12], int i0, int n, A* acc) {
    /* state after sample i-1: x, D1, D2, D3 (plain and biased) */
    int32_t xp = x[3];
    int32_t d1p = x[3] - x[2];
    int32_t d2p = d1p - (x[2] - x[1]);
    int32_t d3p = d2p - ((x[2] - x[1]) - (x[1] - x[0]));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int32_t xc = x[4 + k];
        const int32_t d1 = xc - xp, d2 = d1 - d1p, d3 = d2 - d2p;
        const uint32_t xb = (uint32_t)xc ^ kBias;
        if constexpr (!MASKED && std::is_same<A, uint32_t>::value) {
            /* one v_sad_u32 per order, accumulating in place (32-bit chunk sums) */
            acc[0] = sad_u32(xb, kBias, acc[0]);
            acc[1] = sad_u32(xb, (uint32_t)xp ^ kBias, acc[1]);
            acc[2] = sad_u32((uint32_t)d1 ^ kBias, (uint32_t)d1p ^ kBias, acc[2]);
            acc[3] = sad_u32((uint32_t)d2 ^ kBias, (uint32_t)d2p ^ kBias, acc[3]);
            acc[4] = sad_u32((uint32_t)d3 ^ kBias, (uint32_t)d3p ^ kBias, acc[4]);
            xp = xc;
            d1p = d1;
            d2p = d2;
            d3p = d3;
            continue;
        }
        uint32_t s0 = sad_acc(xb, kBias, 0);                                        /* |x|  */
        uint32_t s1 = sad_acc(xb, (uint32_t)xp ^ kBias, 0);                         /* |D1| */
        uint32_t s2 = sad_acc((uint32_t)d1 ^ kBias, (uint32_t)d1p ^ kBias, 0);      /* |D2| */
        uint32_t s3 = sad_acc((uint32_t)d2 ^ kBias, (uint32_t)d2p ^ kBias, 0);      /* |D3| */
        uint32_t s4 = sad_acc((uint32_t)d3 ^ kBias, (uint32_t)d3p ^ kBias, 0);      /* |D4| */
        if (MASKED) {
            const int i = i0 + k;
            const bool in = i < n;
            s0 = in ? s0 : 0;
            s1 = (in && i >= 1) ? s1 : 0;
            s2 = (in && i >= 2) ? s2 : 0;
            s3 = (in && i >= 3) ? s3 : 0;
            s4 = (in && i >= 4) ? s4 : 0;
        }
        acc[0] += s0;
        acc[1] += s1;
        acc[2] += s2;
        acc[3] += s3;
        acc[4] += s4;
        xp = xc;
        d1p = d1;
        d2p = d2;
        d3p = d3;
    }
}

/* LDS tables of the LPC candidates, filled in phase A */
template <int LMAX>
struct CoefTables {
    static constexpr int NP = (LMAX + 2) / 2; /* pairs per order: taps x[i], x[i-1] .. x[i-LMAX] */
    static constexpr int PPAD = NP > 0 ? ((NP + 3) / 4) * 4 : 4;    /* padded to uint4 */
    static constexpr int CPAD = LMAX > 0 ? ((LMAX + 3) / 4) * 4 : 4;
    /* MFMA tap table (f32): [16 predictor columns][kTapW], tap(jj) at jj + 4, jj in [-4, 16) */
    static constexpr int TAPF_OFF = 16 * ((4 * LMAX * (PPAD + CPAD) + 12 * LMAX + 15) / 16);
    static constexpr int BYTES = TAPF_OFF + 16 * 20 * 4;
};
constexpr int kTapW = 20;

/* The sign-correlation bound's terms over one chunk of 16-bit samples (window at i0 >= HP):
 * K_j += sum_i w_i x_{i-j} for j = 0..LMAX with w_i = sign(x_i) as packed +-1 halves, one
 * v_dot2_i32_i16 per sample pair and lag (exact: no N_- correction inside K_j), and
 * nneg += #{x_i < 0} (the bound's -N_- term). */
template <int LMAX, int HP>
__device__ __forceinline__ void sb16_chunk(const Win16<HP>& W, int32_t (&kk)[LMAX + 1], uint32_t& nneg) {
    static_assert(HP % 2 == 0 && HP >= LMAX, "window pairs start at even positions and cover every lag");
    const uint32_t k15 = 0x000F000Fu;
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        const uint32_t xp = W.E[(HP + k) >> 1]; /* samples i0 + k (lo), i0 + k + 1 (hi) */
        uint32_t sg;
        asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(sg) : "v"(k15), "v"(xp));
        sg |= 0x00010001u; /* +1 or -1 per half */
        nneg += (uint32_t)__builtin_popcount(xp & 0x80008000u);
#pragma unroll
        for (int j = 0; j <= LMAX; ++j) {
            const int lo = HP + k - j; /* window position of x_{i0 + k - j} */
            const uint32_t pr = (lo & 1) ? W.O[(lo - 1) >> 1] : W.E[lo >> 1];
            kk[j] = sdot2(pr, sg, kk[j]);
        }
    }
}

/* PATH_S16 candidate sums.  The dot chain of order p carries one extra tap, x[i] with
 * coefficient -2^sh, and starts from 2^31: t = 2^31 + pred - x[i]*2^sh.  That is exact in
 * [0, 2^32) (|x| <= 2^15, sh <= 15, |pred| < 2^26), so the logical shift t >> sh equals
 * 2^(31-sh) + (pred >> sh) - x[i] and |r| = |(t >> sh) - 2^(31-sh)| is one v_sad_u32
 * accumulate.  Per sample and order: ceil((p+1)/2) v_dot2_i32_i16, a shift and a sad.
 * The eight samples of a chunk run as independent chains, interleaved tap by tap. */
template <int LMAX, int HP, bool MASKED>
__device__ __forceinline__ void chunk_sums_s16(const Win16<HP>& W, int i0, int n, int L, bool do_lpc,
                                               const uint32_t* cpair, const int32_t* lsh,
                                               uint32_t (&acc)[5 + LMAX]) {
    using CT = CoefTables<LMAX>;
    fixed_sums32<MASKED>(W.x, i0, n, acc);
    if (!do_lpc) return;
    static_for<LMAX>([&](auto P_) {
        constexpr int pp = P_ + 1;
        constexpr int np = (pp + 2) / 2;
        __builtin_amdgcn_sched_barrier(0); /* one candidate at a time: bounds register pressure */
        if (pp <= L) {
            uint32_t cq[np];
            const uint4* src = reinterpret_cast<const uint4*>(cpair + (pp - 1) * CT::PPAD);
#pragma unroll
            for (int g = 0; g < (np + 3) / 4; ++g) {
                const uint4 v = src[g];
                if (4 * g + 0 < np) cq[4 * g + 0] = v.x;
                if (4 * g + 1 < np) cq[4 * g + 1] = v.y;
                if (4 * g + 2 < np) cq[4 * g + 2] = v.z;
                if (4 * g + 3 < np) cq[4 * g + 3] = v.w;
            }
            const int sh = lsh[pp - 1];
            const int start = lsh[LMAX + pp - 1];
            const uint32_t kb = (uint32_t)lsh[2 * LMAX + pp - 1]; /* 2^(31-sh) */
            int32_t t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = sdot2(W.pair(k, 0), cq[0], (int32_t)kBias);
#pragma unroll
            for (int j = 1; j < np; ++j)
#pragma unroll
                for (int k = 0; k < 8; ++k) t[k] = sdot2(W.pair(k, j), cq[j], t[k]);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t u = (uint32_t)t[k] >> sh;
                if (MASKED) {
                    const int i = i0 + k;
                    const uint32_t s = sad_acc(u, kb, 0);
                    acc[4 + pp] += (i >= start && i < n) ? s : 0u;
                } else {
                    acc[4 + pp] = sad_acc(u, kb, acc[4 + pp]);
                }
            }
        }
    });
}

/* PATH_W64S: the chunk window split into two int16 planes, x = 4096*h + l with
 * l = sext12(x) in [-2048, 2048) and h = (x - l) >> 12 (|h| <= 2048 for 24-bit samples),
 * each as packed pairs laid out like Win16 (E aligned, O shifted by one sample). */
template <int HP>
struct SplitWin {
    static constexpr int NE = (HP + 8) / 2;
    uint32_t Eh[NE], El[NE], Oh[NE - 1], Ol[NE - 1];
    __device__ __forceinline__ void build(const int32_t (&w)[HP + 8]) {
#pragma unroll
        for (int m = 0; m < NE; ++m) {
            const int32_t a0 = w[2 * m], a1 = w[2 * m + 1];
            const int32_t l0 = (a0 << 20) >> 20, l1 = (a1 << 20) >> 20;
            const int32_t h0 = (a0 - l0) >> 12, h1 = (a1 - l1) >> 12;
            El[m] = __builtin_amdgcn_perm((uint32_t)l1, (uint32_t)l0, 0x05040100u);
            Eh[m] = __builtin_amdgcn_perm((uint32_t)h1, (uint32_t)h0, 0x05040100u);
        }
#pragma unroll
        for (int m = 0; m < NE - 1; ++m) {
            Ol[m] = __builtin_amdgcn_alignbit(El[m + 1], El[m], 16);
            Oh[m] = __builtin_amdgcn_alignbit(Eh[m + 1], Eh[m], 16);
        }
    }
    /* (x[i-1-2t] lo, x[i-2t] hi) of one plane for the sample at window position HP + k */
    __device__ __forceinline__ static uint32_t pick(const uint32_t* E, const uint32_t* O, int k, int t) {
        const int lo = HP + k - 1 - 2 * t;
        if (lo < 0) return E[0] << 16;
        return (lo & 1) ? O[(lo - 1) >> 1] : E[lo >> 1];
    }
};

/* PATH_N32 / PATH_W64 / PATH_W64S: int32 window of HP + 8 samples.  SPLIT (PATH_W64S):
 * every LPC candidate is two v_dot2_i32_i16 chains over the S16 coefficient pairs (extra
 * tap x[i] with -2^sh included), th on the high plane and tl on the low plane.  Both are
 * exact in int32 under the host bound, and T = 4096*th + tl = pred - 2^sh*x[i] exactly,
 * so T >> sh = (pred >> sh) - x[i] = -r: per sample and order ceil((p+1)/2) dots per
 * plane instead of p int64 multiply-adds, then one int64 shift, |.| and add. */
template <int LMAX, int HP, bool MASKED, bool WIDE, bool SPLIT = false>
__device__ __forceinline__ void chunk_sums_32(const int32_t (&w)[HP + 8], int i0, int n, int L, bool do_lpc,
                                              const int32_t* cfl, const int32_t* lsh,
                                              typename std::conditional<WIDE, uint64_t, uint32_t>::type (&acc)[5 + LMAX],
                                              const uint32_t* cpair = nullptr) {
    using CT = CoefTables<LMAX>;
    int32_t x12[12];
#pragma unroll
    for (int t = 0; t < 12; ++t) x12[t] = w[HP - 4 + t];
    if constexpr (!WIDE) {
        fixed_sums32<MASKED>(x12, i0, n, acc);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k;
            const int64_t x0 = w[HP + k], x1 = w[HP + k - 1], x2 = w[HP + k - 2], x3 = w[HP + k - 3],
                          x4 = w[HP + k - 4];
            const int64_t r[5] = {x0, x0 - x1, x0 - 2 * x1 + x2, x0 - 3 * x1 + 3 * x2 - x3,
                                  x0 - 4 * x1 + 6 * x2 - 4 * x3 + x4};
#pragma unroll
            for (int o = 0; o < 5; ++o) acc[o] += (!MASKED || (i >= o && i < n)) ? uabs64(r[o]) : 0;
        }
    }
    if (!do_lpc) return;
    if constexpr (SPLIT) {
        SplitWin<HP> S;
        S.build(w);
        static_for<LMAX>([&](auto P_) {
            constexpr int pp = P_ + 1;
            constexpr int np = (pp + 2) / 2;
            __builtin_amdgcn_sched_barrier(0);
            if (pp <= L) {
                uint32_t cq[np];
                const uint4* src = reinterpret_cast<const uint4*>(cpair + (pp - 1) * CoefTables<LMAX>::PPAD);
#pragma unroll
                for (int g = 0; g < (np + 3) / 4; ++g) {
                    const uint4 v = src[g];
                    if (4 * g + 0 < np) cq[4 * g + 0] = v.x;
                    if (4 * g + 1 < np) cq[4 * g + 1] = v.y;
                    if (4 * g + 2 < np) cq[4 * g + 2] = v.z;
                    if (4 * g + 3 < np) cq[4 * g + 3] = v.w;
                }
                const int sh = lsh[pp - 1];
                const int start = lsh[LMAX + pp - 1];
                int32_t th[8], tl[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    th[k] = sdot2(SplitWin<HP>::pick(S.Eh, S.Oh, k, 0), cq[0], 0);
                    tl[k] = sdot2(SplitWin<HP>::pick(S.El, S.Ol, k, 0), cq[0], 0);
                }
#pragma unroll
                for (int j = 1; j < np; ++j)
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        th[k] = sdot2(SplitWin<HP>::pick(S.Eh, S.Oh, k, j), cq[j], th[k]);
                        tl[k] = sdot2(SplitWin<HP>::pick(S.El, S.Ol, k, j), cq[j], tl[k]);
                    }
                if (lsh[2 * LMAX + pp - 1]) {
                    /* narrow (|r| < 2^28): T >> sh in 32 bits.  sh <= 12: (th << (12-sh)) +
                     * (tl >> sh), exact mod 2^32 hence exact; sh > 12: (th + (tl >> 12)) >>
                     * (sh-12), no wrap.  Eight |r| < 2^31 in one u32, then one 64-bit add. */
                    const int sa = sh < 12 ? 12 - sh : 0, sb = sh < 12 ? sh : 12, sc = sh > 12 ? sh - 12 : 0;
                    uint32_t s32 = 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int i = i0 + k;
                        const int32_t v = (int32_t)(((uint32_t)th[k] << sa) + (uint32_t)(tl[k] >> sb)) >> sc;
                        const uint32_t d = sad_acc((uint32_t)v ^ kBias, kBias, 0);
                        s32 += (!MASKED || (i >= start && i < n)) ? d : 0u;
                    }
                    acc[4 + pp] += s32;
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int i = i0 + k;
                        const int64_t t = ((int64_t)th[k] << 12) + (int64_t)tl[k];
                        const uint64_t v = uabs64(t >> sh);
                        acc[4 + pp] += (!MASKED || (i >= start && i < n)) ? v : 0;
                    }
                }
            }
        });
        return;
    }
    static_for<LMAX>([&](auto P_) {
        constexpr int pp = P_ + 1;
        __builtin_amdgcn_sched_barrier(0); /* one candidate at a time: bounds register pressure */
        if (pp <= L) {
            int32_t c[pp];
            const int4v* src = reinterpret_cast<const int4v*>(cfl + (pp - 1) * CT::CPAD);
#pragma unroll
            for (int g = 0; g < (pp + 3) / 4; ++g) {
                const int4v v = src[g];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * g + e < pp) c[4 * g + e] = v[e];
            }
            const int sh = lsh[pp - 1];
            const int start = lsh[LMAX + pp - 1];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k;
                if constexpr (!WIDE) {
                    int32_t pred = 0;
#pragma unroll
                    for (int j = 0; j < pp; ++j) pred += sext24(c[j]) * sext24(w[HP + k - 1 - j]);
                    uint32_t s = sad_acc((uint32_t)w[HP + k] ^ kBias, (uint32_t)(pred >> sh) ^ kBias, 0);
                    if (MASKED) s = (i >= start && i < n) ? s : 0;
                    acc[4 + pp] += s;
                } else {
                    /* (a 32-bit |r| epilogue under the narrow flag measured slower here:
                     * the duplicated chains spill at the 512-thread register budget) */
                    int64_t pred = 0;
#pragma unroll
                    for (int j = 0; j < pp; ++j) pred += (int64_t)c[j] * (int64_t)w[HP + k - 1 - j];
                    const uint64_t v = uabs64((int64_t)w[HP + k] - (pred >> sh));
                    acc[4 + pp] += (!MASKED || (i >= start && i < n)) ? v : 0;
                }
            }
        }
    });
}

/* ---------------------------------------------------------------------------------------
 * MFMA candidate sums (PATH_S16, L <= 12).  One v_mfma_f32_16x16x32_f16 computes, for 16
 * samples and 16 predictors (LPC orders 1..12, fixed orders 1..4),
 *     f = pred * 2^-sh - x[i] + (2^-(sh+1) - 1/2)          (the C operand is the last term)
 * with every sample split exactly as x = 256*h + l (h signed, l unsigned byte, both exact
 * in f16).  When (sum|c| + 2^sh) * 33023 < 2^22, every product and partial sum is a
 * multiple of 2^-(sh+1) below 2^24 in magnitude, so the f32 accumulation is exact whatever
 * its order; phase A checks that bound per unit (the VALU path takes the rest).  Then
 * w = f + 1.5*2^23 rounds to floor(f) = (pred >> sh) - x[i] = -r, and the bit pattern of w
 * is 0x4B400000 - r: |r| is one v_sad_u32 accumulate.  Per sample and predictor: one
 * v_add_f32 and one v_sad_u32 (the VALU path: ceil((p+1)/2) dots + shift + sad).
 *
 * Block of 64 samples i0..i0+63, MFMAs rho = 0..3: row s of MFMA rho is sample
 * i0 + 4s + rho; its tap window is positions [e, e + 16), e = i0 + 4s - 12, the same for
 * every rho, so the A fragment is built once per block; B_rho puts tap x[i + d] at window
 * slot d + 12 + rho.  A fragment: lane l holds A[row l&15][k = 8(l>>4) + j]; k-block
 * kb = l>>4 is window slots 4kb..4kb+3, j < 4 their h, j >= 4 their l, built from ONE
 * 8-byte LDS read of the int16 samples.  D: lane l holds column l&15, rows 4(l>>4) + r.
 * ------------------------------------------------------------------------------------- */
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float frag_cd __attribute__((ext_vector_type(4)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
constexpr uint32_t kFloorMagicBits = 0x4B400000u; /* 1.5 * 2^23 */
constexpr float kFloorMagic = 12582912.0f;
constexpr int kMfmaCoefLimit = 127; /* sum|c| + 2^sh; 127 * 33023 < 2^22 */


/* two int16 samples (lo, hi) -> f16 pairs of their high bytes (signed) and low bytes:
 * 1024 + v is exact in f16 with the integer in the mantissa, so OR-ing the byte under
 * 0x6400 and subtracting 1024 (1152 for the biased signed byte) converts exactly */
__device__ __forceinline__ uint32_t f16_hi_bytes(uint32_t q) {
    const uint32_t t = ((q >> 8) & 0x00FF00FFu) ^ 0x64806480u;
    const half2v v = __builtin_bit_cast(half2v, t) - half2v{(_Float16)1152.0f, (_Float16)1152.0f};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint32_t f16_lo_bytes(uint32_t q) {
    const uint32_t t = (q & 0x00FF00FFu) | 0x64006400u;
    const half2v v = __builtin_bit_cast(half2v, t) - half2v{(_Float16)1024.0f, (_Float16)1024.0f};
    return __builtin_bit_cast(uint32_t, v);
}

template <bool MASK>
__device__ __forceinline__ uint32_t mfma_block(const int16_t* xs16, int i0, int eoff, const half8 (&B)[4],
                                               const frag_cd& C, int kb, int start, int n, uint32_t mb) {
    const uint2 q = *reinterpret_cast<const uint2*>(xs16 + i0 + eoff);
    const uint4 av{f16_hi_bytes(q.x), f16_hi_bytes(q.y), f16_lo_bytes(q.x), f16_lo_bytes(q.y)};
    const half8 A = __builtin_bit_cast(half8, av);
    frag_cd D[4];
    static_for<4>([&](auto R_) {
        constexpr int rho = R_;
        D[rho] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B[rho], C, 0, 0, 0);
    });
    uint32_t bs[4] = {0, 0, 0, 0};
    static_for<4>([&](auto R_) {
        constexpr int rho = R_;
        static_for<4>([&](auto Q_) {
            constexpr int r = Q_;
            const uint32_t wv = __float_as_uint(D[rho][r] + kFloorMagic);
            if constexpr (MASK) {
                const int i = i0 + 4 * (4 * kb + r) + rho;
                const uint32_t t = sad_u32(wv, mb, 0u);
                bs[r] += (i >= start && i < n) ? t : 0u;
            } else {
                bs[r] = sad_u32(wv, mb, bs[r]);
            }
        });
    });
    return bs[0] + bs[1] + bs[2] + bs[3];
}

/* an unmasked block accumulated into the caller's four running sums (no per-block
 * reduction; the caller bounds how many blocks share them) */
__device__ __forceinline__ void mfma_block_acc(const int16_t* xs16, int i0, int eoff, const half8 (&B)[4],
                                               const frag_cd& C, uint32_t mb, uint32_t (&bs)[4]) {
    const uint2 q = *reinterpret_cast<const uint2*>(xs16 + i0 + eoff);
    const uint4 av{f16_hi_bytes(q.x), f16_hi_bytes(q.y), f16_lo_bytes(q.x), f16_lo_bytes(q.y)};
    const half8 A = __builtin_bit_cast(half8, av);
    frag_cd D[4];
    static_for<4>([&](auto R_) {
        constexpr int rho = R_;
        D[rho] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B[rho], C, 0, 0, 0);
    });
    static_for<4>([&](auto R_) {
        constexpr int rho = R_;
        static_for<4>([&](auto Q_) {
            constexpr int r = Q_;
            bs[r] = sad_u32(__float_as_uint(D[rho][r] + kFloorMagic), mb, bs[r]);
        });
    });
}

/* Sums for the fixed orders 1..4 and LPC orders 1..min(L,12) into red[wid][.] (the order-0
 * sum, sum|x|, comes from the staging pass).  Lane (col, kb) needs the taps
 * tap(jj), jj = 8 - 4kb + m, m = 0..6 of its predictor column (phase A's LDS table):
 * B_rho[j] = (j < 4 ? 256 : 1) * tap(jj) with m = 3 + rho - (j & 3), static per j. */
template <int LMAX>
__device__ __forceinline__ void mfma_candidate_sums(const int16_t* xs16, const float* tapf, const int32_t* lsh,
                                                    int L, int n, int lane, int wid, int nw,
                                                    unsigned long long* red, uint32_t sumx) {
    constexpr int NSUM = 5 + LMAX;
    const int col = lane & 15, kb = lane >> 4;
    const bool lpc_col = col < 12;
    const bool lpc_live = lpc_col && col < L && col < LMAX;
    const int row = (col < LMAX ? col : LMAX - 1);
    float t[7];
    {
        const float* tp = tapf + col * kTapW + (8 - 4 * kb) + 4;
#pragma unroll
        for (int m = 0; m < 7; ++m) t[m] = tp[m];
    }
    half8 B[4];
    static_for<4>([&](auto R_) {
        constexpr int rho = R_;
        uint32_t w[4];
        static_for<4>([&](auto P_) {
            constexpr int pj = P_; /* halves 2pj, 2pj+1 */
            constexpr int j0 = 2 * pj, j1 = 2 * pj + 1;
            const float a0 = t[3 + rho - (j0 & 3)] * (j0 < 4 ? 256.0f : 1.0f);
            const float a1 = t[3 + rho - (j1 & 3)] * (j1 < 4 ? 256.0f : 1.0f);
            w[pj] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a0, a1));
        });
        B[rho] = __builtin_bit_cast(half8, uint4{w[0], w[1], w[2], w[3]});
    });
    const int sh = lpc_live ? lsh[row] : 0;
    const int start = lpc_col ? (lpc_live ? lsh[LMAX + row] : 0) : col - 11;
    const float inv = __uint_as_float((uint32_t)(127 - sh) << 23); /* 2^-sh */
    const float cinit = 0.5f * inv - 0.5f;
    const frag_cd C{cinit, cinit, cinit, cinit};
    const int eoff = 4 * (lane & 15) - 12 + 4 * kb;
    const uint32_t mb = kFloorMagicBits;
    const int nblk = (n + 63) >> 6;
    const int nfull = n >> 6; /* blocks 1 .. nfull-1 need no mask */
    uint64_t acc = 0;
    /* masked blocks: block 0 (warm-up samples) and a partial last block */
    if (wid == 0) acc += mfma_block<true>(xs16, 0, eoff, B, C, kb, start, n, mb);
    if (nblk > nfull && nblk > 1 && (nblk - 1) % nw == wid)
        acc += mfma_block<true>(xs16, (nblk - 1) << 6, eoff, B, C, kb, start, n, mb);
    /* unmasked blocks in groups of up to 16 per wave: every |r| < 2^22 under the exactness
     * bound, so each of the four running sums (64 values) stays below 2^28 */
    int blk = 1 + ((wid - 1 + nw) % nw);
    while (blk < nfull) {
        uint32_t bs[4] = {0u, 0u, 0u, 0u};
#pragma unroll 2
        for (int g = 0; g < 16 && blk < nfull; ++g, blk += nw) mfma_block_acc(xs16, blk << 6, eoff, B, C, mb, bs);
        acc += (uint64_t)((bs[0] + bs[1]) + (bs[2] + bs[3]));
    }
    acc += (uint64_t)__shfl_xor((unsigned long long)acc, 16);
    acc += (uint64_t)__shfl_xor((unsigned long long)acc, 32);
    const uint32_t sx = wave_sum_u32(sumx);
    if (lane < 16) {
        const int si = lpc_col ? 5 + col : col - 11;
        if (si < NSUM) red[wid * NSUM + si] = acc;
    }
    if (lane == 0) red[wid * NSUM] = sx;
}

/* ---------------------------------------------------------------------------------------
 * int8-MFMA candidate sums (PATH_W64, L <= 32, samples <= 24 bits, |c| < 2^15 - 128):
 * the prediction_residual loops of encoder.py:537-548 for all L orders at once, as
 * v_mfma_i32_16x16x64_i8 over Toeplitz windows of byte digits.
 *
 * Digits (balanced base 256): x = b0 + 2^8 b1 + 2^16 b2, c = e0 + 2^8 e1, every digit a
 * signed byte (b2 <= 127 holds for x <= 8355711: checked per unit).  The six digit products
 * are grouped by weight: P_w = sum over d + e = w of sum_j b_d[i-1-j] e_e[c_j], w = 0..3, one
 * MFMA each, |P_w| <= 64 * 2^14 = 2^20.  Then pred = 2^16 (P2 + 2^8 P3) + (P0 + 2^8 P1)
 * with lo = P0 + 2^8 P1 exact in int32, so for any shift s <= 15
 *     floor(pred / 2^s) = ((P2 + 2^8 P3) << (16 - s)) + (lo >> s)      (mod 2^32)
 * exactly, and |r| = |floor(pred / 2^s) - x|.  P2's accumulator starts at 2^(15+s), which
 * adds 2^31 to the result: against x ^ 2^31 one v_sad_u32 gives |r| whenever the true
 * floor(pred/2^s) and x lie in [-2^31, 2^31); the unit's bound B = max|x| + max_p
 * (sum|c_p| max|x| >> s_p) + 1 < 2^30 guarantees it (checked per unit, with the number of
 * tiles G whose 4 values per lane a u32 partial sum can hold).  Per sample and order: 5 VALU
 * (two shift-adds, one shift, one shift-add, one sad) instead of p v_mad_i64_i32.
 *
 * Tile = 16 samples i0..i0+15 (MFMA rows), N-tile nt = orders 16nt+1 .. 16nt+16 (columns).
 * Lane l: row m = l & 15, K quarter qq = l >> 4, slot sg = qq >> 1, half h = qq & 1; its 16
 * K bytes are taps j = 16h + 15 - t (t = 0..15), i.e. the 16 samples from i0 + m - 16 - 16h
 * upward: one unaligned 16-byte window of a digit plane (5 dword reads, 4 v_alignbyte).
 * Slot 0 carries (b0,e0) (b1,e0) (b2,e0) (b2,e1) for P0..P3, slot 1 (b0,e1) (b1,e1) for P1, P2.
 * tools/check_mfma_i8.hip pins the operand layout on gfx950.
 * ------------------------------------------------------------------------------------- */
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int32_t sext8(int32_t v) { return (int32_t)(int8_t)(v & 255); }

/* balanced base-256 digits of an int32 sample (b2 in [-128, 128]: 128 only above 8355711) */
__device__ __forceinline__ void mf8_digits(int32_t x, int32_t& b0, int32_t& b1, int32_t& b2) {
    b0 = sext8(x);
    const int32_t x1 = (x - b0) >> 8;
    b1 = sext8(x1);
    b2 = (x1 - b1) >> 8;
}

/* a 16-byte window of a plane at any byte alignment (tile T of the lane's window starts 16 T
 * bytes after p): the five dwords that cover it and four v_alignbyte by its offset.  With
 * -DFLACMI_MF8_UNALIGNED one unaligned ds_read_b128 instead (gfx950 accepts it, but measured
 * c3 k_resid 55.1 against 39.4 ms: an unaligned 16-byte LDS read is far slower than the five
 * aligned dword reads and four v_alignbyte, profiles/r04c) */
#ifdef FLACMI_MF8_UNALIGNED
struct Mf8Raw {
    v4i v;
};
__device__ __forceinline__ void mf8_load(const unsigned char* p, int T, Mf8Raw& r) {
    __builtin_memcpy(&r.v, p + 16 * T, 16);
}
__device__ __forceinline__ v4i mf8_align(const Mf8Raw& r, uint32_t) { return r.v; }
#else
struct Mf8Raw {
    uint32_t d[5];
};
__device__ __forceinline__ void mf8_load(const unsigned char* p, int T, Mf8Raw& r) {
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p - (reinterpret_cast<uintptr_t>(p) & 3)) + 4 * T;
#pragma unroll
    for (int k = 0; k < 5; ++k) r.d[k] = pw[k];
}
__device__ __forceinline__ v4i mf8_align(const Mf8Raw& r, uint32_t sh) {
    v4i v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (int)__builtin_amdgcn_alignbyte(r.d[k + 1], r.d[k], sh);
    return v;
}
#endif

/* one 16-sample tile for N-tile operands B*, accumulating |r| of the lane's column into s32 */
template <bool MASK>
__device__ __forceinline__ void mf8_tile_epilogue(const v4i (&D)[4], int s, const uint32_t (&xb)[4], int i0r,
                                                  int start, uint32_t& s32) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t lo = (int32_t)((uint32_t)D[0][r] + ((uint32_t)D[1][r] << 8));
        const int32_t hi = (int32_t)((uint32_t)D[2][r] + ((uint32_t)D[3][r] << 8));
        const uint32_t t = ((uint32_t)hi << (16 - s)) + (uint32_t)(lo >> s);
        if constexpr (MASK) {
            const uint32_t v = sad_u32(t, xb[r], 0u);
            s32 += (i0r + r >= start) ? v : 0u;
        } else {
            s32 = sad_u32(t, xb[r], s32);
        }
    }
}

/* (a ^ b) + c in one v_xad_u32 (left to itself the compiler pairs two v_xor_b32 with one
 * v_add3_u32: 1.5 instructions per term) */
__device__ __forceinline__ uint32_t xad_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

/* Sums of |r| for LPC orders 1..L (into red[wid][5 + p - 1]) and fixed orders 0..4 (VALU,
 * 8-sample chunks, into red[wid][0..4]).  pl: the three digit planes, PLB bytes apart;
 * cfl / lsh: phase A's coefficient and shift tables; G: tiles per u32 partial sum.
 *
 * prune (reference mode): the tiles run in eight tiers, the wave's tiles k % 8 == 0, then
 * 4, 2, 6, 1, 5, 3, 7.  After each tier from the second on, every wave reads the workgroup's exact partial LPC sums (a sum
 * over a subset of the values, so a lower bound of each order's full sum) against the best
 * exact fixed sum; once every order's partial sum exceeds it, LPC can neither win nor tie
 * (encoder.py:135-157) and the remaining tiers are skipped (red then holds partial LPC
 * sums).  Otherwise the eight tiers add up to the exact sums.  Returns (workgroup-uniform)
 * the eighths done | 0x100 if pruned, or 0 without pruning. */
template <int LMAX, bool PIPE = true>
__device__ __forceinline__ int mf8_candidate_sums(const int32_t* xs32, const unsigned char* pl, int PLB,
                                                   const int32_t* cfl, const int32_t* lsh, int L, int n, int G,
                                                   int tid, int NT, int lane, int wid, int nw,
                                                   unsigned long long* red, bool prune, int dbg, bool sbound) {
    using CT = CoefTables<LMAX>;
    constexpr int NSUM = 5 + LMAX;
    constexpr int NTMAX = (LMAX + 15) / 16;
    unsigned long long* const red_alt = red + nw * NSUM; /* the second copy of the tier sums */
    /* the sign-correlation bound (below): K_j over R = [LMAX, n), a thread's chunks summed in
     * 32 bits (at most four 8-sample chunks of |x| <= 2^23.01 per thread: |part| < 2^28.01) */
    const bool sb = prune && sbound && dbg < 13 && n <= 32 * NT;
    int32_t kc[LMAX + 1], kneg = 0;
#pragma unroll
    for (int j = 0; j <= LMAX; ++j) kc[j] = 0;
    /* fixed orders on the VALU */
    {
        uint64_t fa[5] = {0, 0, 0, 0, 0};
        const int nch = n >> 3;
#pragma unroll 1
        for (int c = tid; c < nch; c += NT) {
            const int i0 = 8 * c;
            int32_t x12[12];
            const int4v* src = reinterpret_cast<const int4v*>(xs32 + i0 - 4);
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const int4v v = src[g];
#pragma unroll
                for (int e = 0; e < 4; ++e) x12[4 * g + e] = v[e];
            }
            if (sb && i0 >= LMAX) {
                /* w_i = +1 (x_i >= 0) or -1 (x_i < 0) with m_i = x_i >> 31: w_i x = (x ^ m_i) - m_i,
                 * so sum_i w_i x_{i-j} = sum_i (x_{i-j} ^ m_i) + #{m_i = -1}: one v_xad_u32 each */
                int32_t xw[LMAX + 8]; /* samples i0 - LMAX .. i0 + 7 */
                const int4v* wsrc = reinterpret_cast<const int4v*>(xs32 + i0 - LMAX);
#pragma unroll
                for (int g = 0; g < LMAX / 4 - 1; ++g) {
                    const int4v v = wsrc[g];
#pragma unroll
                    for (int e = 0; e < 4; ++e) xw[4 * g + e] = v[e];
                }
#pragma unroll
                for (int e = 0; e < 12; ++e) xw[LMAX - 4 + e] = x12[e];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int32_t m = xw[LMAX + k] >> 31;
                    kneg -= m;
#pragma unroll
                    for (int j = 0; j <= LMAX; ++j) kc[j] = (int32_t)xad_u32((uint32_t)xw[LMAX + k - j], (uint32_t)m, (uint32_t)kc[j]);
                }
            }
            /* a chunk's sums in 32 bits (|x| <= 2^23 on this path: 8 |D4| < 2^30), so each |D|
             * is one v_sad_u32 into its accumulator; 64 bits once per chunk and order */
            uint32_t ca[5] = {0, 0, 0, 0, 0};
            if (i0 >= 8) fixed_sums32<false>(x12, i0, n, ca);
            else fixed_sums32<true>(x12, i0, n, ca);
#pragma unroll
            for (int o = 0; o < 5; ++o) fa[o] += ca[o];
        }
#pragma unroll
        for (int o = 0; o < 5; ++o) {
            const uint64_t v = wave_sum_u64(fa[o]);
            if (lane == 0) red[wid * NSUM + o] = v;
        }
    }
    uint64_t fmin = ~0ull; /* the best exact fixed sum (read at the first test) */
    auto read_fmin = [&]() __attribute__((always_inline)) {
        uint64_t tf = 0;
        if (lane < 5)
            for (int w2 = 0; w2 < nw; ++w2) tf += red[w2 * NSUM + lane];
#pragma unroll
        for (int o = 0; o < 5; ++o) {
            const uint64_t v = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(tf >> 32), o) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tf, o);
            fmin = v < fmin ? v : fmin;
        }
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(tf >> 32), 0) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tf, 0); /* the order-0 sum */
    };
    if (sb) {
        /* The sign-correlation bound.  For any weights |w_i| <= 1 and the residual r of order p
         * (encoder.py:537-548: r_i = x_i - floor(P_i / 2^s), P_i = sum_j c_j x_{i-j}):
         *   sum_{i >= p} |r_i| >= sum_{i in R} w_i r_i >= K_0 - (sum_j c_j K_j) / 2^s - N_-,
         * with R = [LMAX, n) (inside every order's residual range), K_j = sum_{i in R} w_i
         * x_{i-j} and N_- = #{i in R: w_i = -1} (w_i = -1 turns -floor(P/2^s) into at most
         * P/2^s - 1 below).  With w_i = sign(x_i) the bound sits within a few percent of the
         * exact sum whenever the residual follows the signal -- flac-py's negated predictor
         * makes r ~ 2x -- and K_j costs (LMAX + 1) v_xad_u32 per sample instead of
         * the LPC tiles.  When every order's bound exceeds the best fixed sum, LPC can neither
         * win nor tie (encoder.py:135-157); a coefficient-less order ((), 0) has r = x over
         * the whole unit, whose sum is the fixed order-0 sum exactly. */
        /* wave sums in 32-bit steps: quads first (|v| < 2^30.01), then the quad sums split as
         * v = 2^16 hi + lo (lo < 2^16, |hi| < 2^14.01), whose sums over the wave's 16 quads stay
         * below 2^20 and 2^18.01; the slot holds (hi sum, lo sum) as two words, and the
         * evaluating wave forms 2^16 hi + lo in 64 bits */
#pragma unroll
        for (int j = 0; j <= LMAX; ++j) {
            uint32_t v = (uint32_t)kc[j];
            v += dpp_u32<0xB1, 0xf>(v);
            v += dpp_u32<0x4E, 0xf>(v);
            uint32_t lo = v & 0xffffu, hi = (uint32_t)((int32_t)v >> 16);
            lo += dpp_u32<0x141, 0xf>(lo);
            hi += dpp_u32<0x141, 0xf>(hi);
            lo += dpp_u32<0x140, 0xf>(lo);
            hi += dpp_u32<0x140, 0xf>(hi);
            lo += dpp_u32<0x142, 0xa>(lo);
            hi += dpp_u32<0x142, 0xa>(hi);
            lo += dpp_u32<0x143, 0xc>(lo);
            hi += dpp_u32<0x143, 0xc>(hi);
            if (lane == 63) red_alt[wid * NSUM + j] = ((uint64_t)hi << 32) | lo;
        }
        {
            const uint32_t v = wave_sum_u32((uint32_t)kneg);
            if (lane == 0) red_alt[wid * NSUM + LMAX + 1] = v;
        }
        __syncthreads();
        const uint64_t f0 = read_fmin();
        if (wid == 0) { /* one wave evaluates the bounds; the others wait for its verdict */
            int64_t kt = 0; /* lane j <= LMAX: K_j; lane LMAX + 1: N_- */
            if (lane <= LMAX)
                for (int w2 = 0; w2 < nw; ++w2) {
                    const uint64_t v = red_alt[w2 * NSUM + lane];
                    kt += ((int64_t)(int32_t)(uint32_t)(v >> 32) << 16) + (int64_t)(uint32_t)v;
                }
            else if (lane == LMAX + 1)
                for (int w2 = 0; w2 < nw; ++w2) kt += (int64_t)red_alt[w2 * NSUM + lane];
            auto lane64 = [&](int64_t v, int l) __attribute__((always_inline)) -> int64_t {
                return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l));
            };
            const int64_t k0 = lane64(kt, 0) + lane64(kt, LMAX + 1), nneg = lane64(kt, LMAX + 1);
            /* lane p - 1: order p's bound (coefficients c_{p,1..p} = cfl[(p - 1) CPAD + 0 .. p - 1]) */
            int64_t S = 0;
            const int pl = lane + 1;
#pragma unroll 1
            for (int j = 1; j <= L; ++j) {
                const int64_t kj = lane64(kt, j) + nneg;
                const int32_t c = (pl <= L && j <= pl) ? cfl[lane * CT::CPAD + j - 1] : 0;
                S += (int64_t)c * kj;
            }
            bool lose = true; /* this lane's order provably loses */
            if (pl <= L) {
                const int s = lsh[pl - 1], start = lsh[LMAX + pl - 1];
                if (start == 0) lose = f0 > fmin; /* ((), 0): r = x, the fixed order-0 sum */
                else lose = k0 - (S >> s) - 1 - nneg > (int64_t)fmin;
            }
            const bool decided = __ballot(!lose) == 0;
            if (lane == 0) red_alt[LMAX + 2] = decided ? 1ull : 0ull; /* wave 0's unused slot */
        }
        __syncthreads(); /* the verdict; every wave is past its red_alt reads before a tier writes it */
        if (red_alt[LMAX + 2] != 0) return 0x100; /* decided before any LPC tile (meta.lpc_tiers 0/8) */
    }
    const int col = lane & 15, qq = lane >> 4, sg = qq >> 1, h = qq & 1, m = col;
    /* B operands and per-column constants */
    v4i Bw0[NTMAX], Bx[NTMAX], Bw3[NTMAX], C2[NTMAX];
    int sh[NTMAX], st[NTMAX];
#pragma unroll
    for (int nt = 0; nt < NTMAX; ++nt) {
        const int p = 16 * nt + col + 1;
        const bool live = p <= L;
        uint32_t w0[4] = {0, 0, 0, 0}, wx[4] = {0, 0, 0, 0}, w3[4] = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int j = 16 * h + 15 - t;
            const int32_t c = (live && j < p) ? cfl[(p - 1) * CT::CPAD + j] : 0;
            const int32_t e0 = sext8(c), e1 = (c - e0) >> 8;
            const uint32_t bx = (uint32_t)(sg == 0 ? e0 : e1) & 255u;
            const uint32_t b0 = sg == 0 ? (uint32_t)e0 & 255u : 0u;
            const uint32_t b3 = sg == 0 ? (uint32_t)e1 & 255u : 0u;
            wx[t >> 2] |= bx << (8 * (t & 3));
            w0[t >> 2] |= b0 << (8 * (t & 3));
            w3[t >> 2] |= b3 << (8 * (t & 3));
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            Bw0[nt][g] = (int)w0[g];
            Bx[nt][g] = (int)wx[g];
            Bw3[nt][g] = (int)w3[g];
        }
        sh[nt] = live ? lsh[p - 1] : 0;
        st[nt] = live ? lsh[LMAX + p - 1] : 0x7fffffff;
        const int cb = (int)(1u << (15 + sh[nt]));
        C2[nt] = v4i{cb, cb, cb, cb};
    }
    /* the lane's three windows: plane 0; plane 1 (slot 0) or 0 (slot 1); plane 2 or 1.  A
     * tile start is a multiple of 16 samples, so each window's byte alignment is fixed and
     * tile T reads dwords 4T further on. */
    const int off0 = kMf8Pad + m - 16 - 16 * h;
    const int off1 = off0 + (sg == 0 ? PLB : 0);
    const int off2 = off0 + (sg == 0 ? 2 * PLB : PLB);
    const uint32_t al = (uint32_t)(off0 & 3); /* PLB is a multiple of 16 */
    const unsigned char* pw0 = pl + off0;
    const unsigned char* pw1 = pl + off1;
    const unsigned char* pw2 = pl + off2;
    const v4i Z{0, 0, 0, 0};
    uint64_t acc[NTMAX];
    uint32_t s32[NTMAX];
#pragma unroll
    for (int nt = 0; nt < NTMAX; ++nt) acc[nt] = 0, s32[nt] = 0;
    const int ntile = n >> 4;
    /* the MFMAs of one tile with NTL live N-tiles (windows from the raw dwords) */
    auto mm = [&](const Mf8Raw& r0, const Mf8Raw& r1, const Mf8Raw& r2, auto& D) __attribute__((always_inline)) {
        constexpr int NTL = sizeof(D) / sizeof(D[0]);
        const v4i A0 = mf8_align(r0, al), A1 = mf8_align(r1, al), A2 = mf8_align(r2, al);
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) {
            D[nt][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, Bw0[nt], Z, 0, 0, 0);
            D[nt][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, Bx[nt], Z, 0, 0, 0);
            D[nt][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, Bx[nt], C2[nt], 0, 0, 0);
            D[nt][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, Bw3[nt], Z, 0, 0, 0);
        }
    };
    /* |r| of tile T from its MFMA results */
    auto ep = [&](const auto& D, int T, auto MASK_) __attribute__((always_inline)) {
        constexpr int NTL = sizeof(D) / sizeof(D[0]);
        constexpr bool MASK = decltype(MASK_)::value;
        const int i0 = T << 4;
        const int4v xv = *reinterpret_cast<const int4v*>(xs32 + i0 + 4 * qq);
        const uint32_t xb[4] = {(uint32_t)xv[0] ^ kBias, (uint32_t)xv[1] ^ kBias, (uint32_t)xv[2] ^ kBias,
                                (uint32_t)xv[3] ^ kBias};
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) mf8_tile_epilogue<MASK>(D[nt], sh[nt], xb, i0 + 4 * qq, st[nt], s32[nt]);
    };
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < NTMAX; ++nt) acc[nt] += s32[nt], s32[nt] = 0;
    };
    /* tiles T = wid, wid + nw, ...; the first two (samples < 32 >= every start) masked.  The
     * main loop is software-pipelined over two register sets: while the VALU runs the
     * epilogue of tile T, the matrix cores run the MFMAs of the next tile and the LDS
     * delivers the windows of the one after (clamped index: no guarded loads; a clamped
     * tile's MFMAs are never used). */
    auto run = [&](auto NTL_, int T, const int step) __attribute__((always_inline)) {
        constexpr int NTL = decltype(NTL_)::value;
        if constexpr (!PIPE) { /* one register set (kVarMf8: four waves per SIMD hide the latencies) */
            Mf8Raw r0, r1, r2;
            v4i D[NTL][4];
            for (; T < 2 && T < ntile; T += step) { /* masked */
                mf8_load(pw0, T, r0);
                mf8_load(pw1, T, r1);
                mf8_load(pw2, T, r2);
                mm(r0, r1, r2, D);
                ep(D, T, std::true_type{});
            }
            flush();
            int g = 0;
            for (; T < ntile; T += step) {
                mf8_load(pw0, T, r0);
                mf8_load(pw1, T, r1);
                mf8_load(pw2, T, r2);
                mm(r0, r1, r2, D);
                ep(D, T, std::false_type{});
                if (++g == G) flush(), g = 0;
            }
            flush();
            return;
        }
        Mf8Raw a0, a1, a2, b0, b1, b2;
        v4i DA[NTL][4], DB[NTL][4];
        while (T < 2 && T < ntile) {
            mf8_load(pw0, T, a0);
            mf8_load(pw1, T, a1);
            mf8_load(pw2, T, a2);
            mm(a0, a1, a2, DA);
            ep(DA, T, std::true_type{});
            T += step;
        }
        flush();
        if (T >= ntile) return;
        mf8_load(pw0, T, a0);
        mf8_load(pw1, T, a1);
        mf8_load(pw2, T, a2);
        mm(a0, a1, a2, DA);
        int Tn = T + step < ntile ? T + step : T;
        mf8_load(pw0, Tn, b0);
        mf8_load(pw1, Tn, b1);
        mf8_load(pw2, Tn, b2);
        int g = 0;
        for (;;) {
            int Tnn = Tn + step < ntile ? Tn + step : Tn;
            mm(b0, b1, b2, DB);
            mf8_load(pw0, Tnn, a0);
            mf8_load(pw1, Tnn, a1);
            mf8_load(pw2, Tnn, a2);
            ep(DA, T, std::false_type{});
            T += step;
            if (++g == G) flush(), g = 0;
            if (T >= ntile) break;
            Tn = Tnn;
            Tnn = Tn + step < ntile ? Tn + step : Tn;
            mm(a0, a1, a2, DA);
            mf8_load(pw0, Tnn, b0);
            mf8_load(pw1, Tnn, b1);
            mf8_load(pw2, Tnn, b2);
            ep(DB, T, std::false_type{});
            T += step;
            if (++g == G) flush(), g = 0;
            if (T >= ntile) break;
            Tn = Tnn;
        }
        flush();
    };
    /* tiles T0, T0 + step, ... (the first two tiles, samples < 32 >= every start, masked) */
    auto go = [&](int T0, int step) __attribute__((always_inline)) {
        if constexpr (NTMAX >= 2) {
            if (L > 16) run(std::integral_constant<int, 2>{}, T0, step);
            else run(std::integral_constant<int, 1>{}, T0, step);
        } else {
            run(std::integral_constant<int, 1>{}, T0, step);
        }
    };
    /* this wave's running LPC sums (cumulative over tiers) into red */
    auto store = [&](unsigned long long* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < NTMAX; ++nt) {
            uint64_t v = acc[nt];
            v += (uint64_t)__shfl_xor((unsigned long long)v, 16);
            v += (uint64_t)__shfl_xor((unsigned long long)v, 32);
            const int p = 16 * nt + col + 1;
            if (lane < 16 && p <= LMAX) buf[wid * NSUM + 4 + p] = p <= L ? v : 0ull;
        }
    };
    if (!prune) {
        go(wid, nw);
        store(red);
        return 0;
    }
    /* ablation (timing only, FLACMI_DEBUG_STOP): 13 fixed sums alone, 14 the first quarter of
     * the LPC tiles without the tier test, 15 every LPC tile without tier tests; each then
     * reports the unit pruned */
    if (dbg == 13) return 0x100;
    if (dbg == 14 || dbg == 15) {
        go(wid, dbg == 14 ? 4 * nw : nw);
        store(red);
        return 0x100 | (dbg == 14 ? 2 : 8);
    }
    bool pruned = false;
    int done = 0;
    /* tier t stores its running sums into red when 7 - t is even (the last tier's exact sums
     * land where phase D reads them), else into the copy after it: a wave that starts the
     * next tier stores while slower waves may still read this one's, so a test needs one
     * barrier, not two */
    /* eighths of the wave's tiles, spread over the block (residues 0, 4, 2, 6, 1, 5, 3, 7 of
     * the wave's tile index mod 8): a unit stops at the first eighth whose partial LPC sums
     * all exceed the best fixed sum (config 3: LPC sums run ~4x the fixed ones, so most
     * units stop after two or three eighths) */
    constexpr int kTiers = 8;
#pragma unroll 1
    for (int t = 0; t < kTiers; ++t) {
        const int res = (int)((0x73516240u >> (4 * t)) & 15u);
        if (t == 0) { /* the first test after two eighths (few units stop after one): residues 0
                       * and 4 as one quarter, one pipelined run */
            go(wid, 4 * nw);
            ++t;
        } else {
            go(wid + res * nw, kTiers * nw);
        }
        unsigned long long* const buf = ((kTiers - 1 - t) & 1) ? red_alt : red;
        store(buf);
        done = t + 1;
        if (t == kTiers - 1) break; /* every tile done: the sums are exact */
        __syncthreads();
        if (fmin == ~0ull) read_fmin(); /* first test: the fixed sums (exact, stored before the tiers) */
        uint64_t tj = 0;
        if (lane >= 5 && lane < 5 + L)
            for (int w2 = 0; w2 < nw; ++w2) tj += buf[w2 * NSUM + lane];
        pruned = __ballot(lane >= 5 && lane < 5 + L && tj <= fmin) == 0;
        if (pruned) break;
    }
    return done | (pruned ? 0x100 : 0);
}

/* Phase E of the fast kernel for a fixed predictor of order K (encoder.py:331-359,
 * common.py:15-21): the residual of samples i0..i0+7 is their K-th difference, zig-zagged
 * (utils.py:91-94); the warm-up samples i < K give 0.  16-bit samples: |r| < 2^19. */
template <int K>
__device__ __forceinline__ void fixed_resid_chunk(const int16_t* xs16, int i0, uint32_t (&z)[8]) {
    const uint4 w = *reinterpret_cast<const uint4*>(xs16 + i0);
    uint4 v{0, 0, 0, 0};
    if constexpr (K > 0) v = *reinterpret_cast<const uint4*>(xs16 + i0 - 8); /* history pad >= 8 */
    const uint32_t q[6] = {v.z, v.w, w.x, w.y, w.z, w.w};
    int32_t d[12]; /* samples i0-4 .. i0+7 */
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        d[2 * t] = (int32_t)(q[t] << 16) >> 16;
        d[2 * t + 1] = (int32_t)q[t] >> 16;
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
    if (i0 == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) z[k] = 0;
    }
}

/* Phase E for a fixed predictor of order K on 32-bit LDS samples with |x| <= 2^23 (the
 * int8-MFMA path's digit check): the K-th difference (encoder.py:331-359) stays below 2^27,
 * so the chain runs in int32 instead of K 64-bit multiply-adds per value.  Values i < K and
 * i >= n give 0 (only the first and a ragged last chunk test them). */
template <int K, typename ResT>
__device__ __forceinline__ void fixed_resid_chunk32(const int32_t* xs32, int i0, int n, ResT (&zv)[8]) {
    int32_t d[12]; /* samples i0-4 .. i0+7 (history pad >= 4) */
    const int4v* src = reinterpret_cast<const int4v*>(xs32 + i0 - 4);
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const int4v v = src[g];
#pragma unroll
        for (int e = 0; e < 4; ++e) d[4 * g + e] = v[e];
    }
#pragma unroll
    for (int l = 1; l <= K; ++l)
#pragma unroll
        for (int t = 11; t >= 4 - K + l; --t) d[t] -= d[t - 1];
    const bool edge = i0 < 8 || i0 + 8 > n;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int32_t r = d[4 + k];
        const uint32_t z = ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
        zv[k] = (ResT)((!edge || (i0 + k >= K && i0 + k < n)) ? z : 0u);
    }
}

/* floor(log2(x)) for a Rice mean x (normal, > 0): LDS thresholds, global table outside. */
__device__ __forceinline__ int rice_floor_log2(double x, const double* tl, const double* gthr) {
    const int e = (int)((__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
    if (e >= kTlLo && e < kTlLo + 64) return x >= tl[e - kTlLo] ? e + 1 : e;
    return pym::py_floor_log2(x, gthr);
}

/* Rice partition search (encoder.py:655-760) when the residual is 32-bit and narrow, the
 * finest partitions are whole 8-sample chunks and number at most 64:
 *  1. wave 0, lane k = finest partition k, holding its sum S_k: a butterfly (shfl_xor)
 *     gives every lane the sum of its ancestor at each order; the lane computes that
 *     node's parameter floor(log2(S/len)) into pk[k][order]; group leaders add the
 *     partition headers; the first error in the reference's evaluation order (orders, then
 *     partitions, ascending) is kept (rice_params_wave0);
 *  2. every thread, per chunk it owns: sum over the chunk of x >> p for each candidate
 *     order, parameters from pk of the chunk's finest partition (chunk_rice_bits);
 *  3. one wave reduction per order; thread 0 picks the order, first minimum (rice_finish). */
template <bool INTLOG, typename ArgsT>
__device__ __forceinline__ void rice_params_wave0(const ArgsT& a, uint64_t s, const double* tl,
                                                  unsigned long long* rb, int* misc, uint8_t* pk, int n, int order,
                                                  int rmin, int omax, int lane) {
    const int P = 1 << omax, k = lane;
    int ekey = -1, esite = 0;
    uint32_t m5 = 0;
    for (int o = omax; o >= rmin; --o) {
        const int d = omax - o;
        if (d > 0) s += (uint64_t)__shfl_xor((unsigned long long)s, 1 << (d - 1));
        const int K = k >> d;
        const bool lead = k < P && (k & ((1 << d) - 1)) == 0;
        const int len = (n >> o) - (K == 0 ? order : 0);
        int prm = 0;
        const bool zero = s == 0;
        bool neg = false;
        if (!zero) {
            if constexpr (INTLOG) {
                /* exact integer floor(log2(s/len)) = max{p : len * 2^p <= s}.  For s < 2^46 and
                 * len < 2^16 the reference's float division + libm log2 give the same value:
                 * the quotient is at least a relative 2^-46 away from the next power of two,
                 * far outside the rounding of the division and of log2. */
                const int fs = 63 - __builtin_clzll((unsigned long long)s);
                const int fl = 31 - __builtin_clz((unsigned)len);
                int p = fs - fl;
                if (p >= 0 && ((uint64_t)len << p) > s) --p;
                prm = p;
            } else {
                prm = rice_floor_log2((double)s / (double)len, tl, a.log2thr);
            }
            neg = prm < 0;
        }
        if (k < P) pk[16 * k + o] = (uint8_t)prm;
        const unsigned long long eb = __ballot(lead && (zero || neg));
        if (eb) {
            const int kl = __builtin_ctzll(eb);
            ekey = (o << 16) | (kl >> d);
            esite = __shfl((int)zero, kl) ? FLACMI_SITE_RICE_LOG_DOMAIN : FLACMI_SITE_RICE_NEG_SHIFT;
        }
        if (__ballot(lead && prm > 14)) m5 |= 1u << o;
        /* headers: < 2^23 per partition, so the order's total fits 32 bits */
        const uint32_t hb = lead ? 4u + (prm > 14 ? 5u : 4u) + (uint32_t)len * (uint32_t)(1 + prm) : 0u;
        const uint32_t ht = wave_sum_u32(hb);
        if (lane == 0) rb[o] = ht;
    }
    if (lane == 0) {
        misc[0] = ekey;
        misc[1] = esite;
        misc[4] = (int)m5;
    }
}

/* data bits of one chunk for every candidate order (chunk sum < 2^30 for narrow values) */
__device__ __forceinline__ void chunk_rice_bits(const uint32_t (&z)[8], uint4 pv, int ro, int oo,
                                                uint32_t (&tb)[16]) {
    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
    static_for<16>([&](auto O_) {
        constexpr int o = O_;
        if (o >= ro && o <= oo) {
            const uint32_t p = (pw[o >> 2] >> (8 * (o & 3))) & 0xffu;
            tb[o] += (z[0] >> p) + (z[1] >> p) + (z[2] >> p) + (z[3] >> p) + (z[4] >> p) + (z[5] >> p) +
                     (z[6] >> p) + (z[7] >> p);
        }
    });
}

/* reduce the per-thread data bits (each < 2^32), pick the order, write meta and parameters */
template <typename ArgsT> /* ResidArgs, or the kernarg-segment view the looping variants read */
__device__ __forceinline__ void rice_finish(const ArgsT& a, flacmi_unit_meta* meta, const Decision* dec,
                                            const uint32_t (&tb)[16], unsigned long long* rb,
                                            unsigned long long* red, int* misc, const uint8_t* pk, int n,
                                            int start, int rmin, int omax, int tid, int NT, int lane, int wid,
                                            int nw, int64_t gid) {
    const int ro = __builtin_amdgcn_readfirstlane(rmin), oo = __builtin_amdgcn_readfirstlane(omax);
    uint32_t any = 0;
#pragma unroll
    for (int o = 0; o < 16; ++o) any |= (o >= ro && o <= oo) ? tb[o] : 0u;
    if (__ballot(any >= (1u << 26)) == 0) { /* every lane < 2^26: the wave totals fit 32 bits */
#pragma unroll
        for (int o = 0; o < 16; ++o)
            if (o >= ro && o <= oo) {
                const uint32_t w = wave_sum_u32(tb[o]);
                if (lane == 0) red[wid * 16 + o] = w;
            }
    } else {
#pragma unroll
        for (int o = 0; o < 16; ++o)
            if (o >= ro && o <= oo) {
                const uint64_t w = wave_sum_u64(tb[o]);
                if (lane == 0) red[wid * 16 + o] = w;
            }
    }
    __syncthreads();
    if (tid == 0) {
        int best = -1;
        unsigned long long bb = 0;
        for (int o = rmin; o <= omax; ++o) {
            unsigned long long v = rb[o];
            for (int w2 = 0; w2 < nw; ++w2) v += red[w2 * 16 + o];
            if (best < 0 || v < bb) {
                bb = v;
                best = o;
            }
        }
        put_meta(meta, ST_OK, 0, dec, 1);
        meta->res_offset = start;
        meta->res_len = n - start;
        meta->part_order = best;
        meta->n_parts = 1 << best;
        meta->coding_method = ((misc[4] >> best) & 1) ? 5 : 4;
        meta->rice_bits = (long long)bb;
        misc[3] = best;
    }
    __syncthreads();
    const int best = misc[3];
    int32_t* __restrict__ rp = a.rice_params + gid * a.params_stride;
    for (int K = tid; K < (1 << best); K += NT) rp[K] = pk[16 * (K << (omax - best)) + best];
}

/* One unit per workgroup.  VAR selects the variant:
 *   kVarGeneric  unit = blockIdx.x, every path;
 *   kVarFast     unit = blockIdx.x, only the S16 MFMA path with a register-resident
 *                residual (smaller register footprint: more workgroups per CU); a unit
 *                outside the MFMA exactness bound is marked FLACMI_STATUS_RETRY and listed;
 *   kVarList     units retry_list[li], li = blockIdx.x, blockIdx.x + gridDim.x, ... below
 *                *retry_count, every path. */
enum { kVarGeneric = 0, kVarFast = 1, kVarList = 2, kVarMf8 = 3, kVarList1 = 4 };
/* kVarMf8 (PATH_W64, LMAX >= 16): only the int8-MFMA path, fixed-predictor choice and the
 * wide Rice step, as a persistent grid (a.persist: one workgroup per CU loops over the batch;
 * the unit's 140 KB of LDS allows one workgroup per CU anyway) that copies the next unit's
 * samples into LDS during this unit's Rice phase; a unit that needs anything else
 * (outside the int8 bounds, an LPC or order > 4 choice, another Rice shape) is marked
 * FLACMI_STATUS_RETRY and listed for kVarList1: the 512-thread generic body, one workgroup
 * per CU looping over retry_list[li] below *retry_count (its arguments through the kernarg
 * pointer, as kVarMf8's, so the loop does not hold them in registers) */
__host__ __device__ constexpr int resid_launch_bound(int path, int lmax, int var) {
    return path >= PATH_W64 ? 512 : 256;
}
/* the kernel's argument block (k_resid's only argument, at offset 0 of the kernarg segment)
 * through a pointer the compiler cannot follow across the persistent variant's unit loop
 * (else it keeps every field live in registers across it); the kernarg pointer itself, not
 * the address of the parameter, which would copy it to scratch */
typedef const __attribute__((address_space(4))) ResidArgs* KernargArgs;
__device__ __forceinline__ KernargArgs opaque_args() {
    KernargArgs p = (KernargArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

__device__ __forceinline__ uint32_t loop_tid() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

template <int LMAX, int PATH, typename ResT, int VAR>
__global__ __launch_bounds__(resid_launch_bound(PATH, LMAX, VAR)) void k_resid(ResidArgs a_in) {
    constexpr bool FAST = VAR == kVarFast;
    constexpr bool M8V = VAR == kVarMf8;
    static_assert(!M8V || (PATH == PATH_W64 && LMAX >= 16 && sizeof(ResT) == 4), "kVarMf8: int8-MFMA units only");
    /* the list variant (units another kernel handed over) loops over the list with a small
     * grid (kListGrid) instead of a workgroup per unit of the batch: a million near-empty
     * workgroups cost ~0.3 ms of dispatch at config 2.  Every exit of the body is
     * workgroup-uniform, so each one goes to the next listed unit. */
    int64_t li = blockIdx.x, gid = blockIdx.x;
    if constexpr (VAR == kVarList || VAR == kVarList1) {
        if (li >= (int64_t)*a_in.retry_count) return;
    }
    /* kVarMf8 persistent: this unit's samples already sit in LDS (copied during the previous
     * unit's Rice phase) */
    bool pre = false;
    int32_t pre_st = 0, pre_rv0 = 0, pre_rv1 = 0; /* ... and its record's status and words tid, tid + NT */
next_unit:
    auto&& a = [&]() -> decltype(auto) {
        if constexpr (VAR == kVarMf8 || VAR == kVarList || VAR == kVarList1) return *opaque_args();
        else return (a_in);
    }();
    if constexpr (VAR == kVarList || VAR == kVarList1) gid = a.retry_list[li];
    if constexpr (VAR == kVarMf8) gid = li;
    const bool pre_now = pre; /* consumed by this unit's staging */
    pre = false;
    {
    using UX = ResT;
    constexpr bool S16 = PATH == PATH_S16;
    constexpr bool WIDE = PATH == PATH_W64 || PATH == PATH_W64S;
    constexpr bool SPLIT = PATH == PATH_W64S;
    using A = typename std::conditional<WIDE, uint64_t, uint32_t>::type; /* per-thread partial */
    using CT = CoefTables<LMAX>;
    constexpr int HP = resid_hp(LMAX);
    constexpr int NSUM = 5 + LMAX;
    constexpr bool MF = S16 && (LMAX == 8 || LMAX == 12); /* MFMA candidate sums available */
    constexpr bool MF8 = PATH == PATH_W64 && LMAX >= 16 && VAR != kVarFast; /* int8-MFMA sums available */
    static_assert(!FAST || (MF && sizeof(ResT) == 4), "FAST: S16 MFMA path with a 32-bit residual only");

    extern __shared__ __align__(16) unsigned char smem[];
    /* the looping variants re-read the thread id per unit (an asm the compiler cannot hoist):
     * otherwise every value derived from it is hoisted out of the unit loop and held in
     * registers across the whole body */
    const int tid = (VAR == kVarList || VAR == kVarList1) ? (int)loop_tid() : (int)threadIdx.x;
    const int NT = blockDim.x, lane = tid & 63, nw = NT >> 6;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6); /* wave-uniform: scalar loops */
    const int64_t u = a.unit0 + gid;
    const int n = a.n, L = a.L;
    const int nch = (n + 7) >> 3;
    /* LPC records exist in the reference and LPC-only modes */
    const bool ref_mode = FAST || a.mode == FLACMI_MODE_REFERENCE || a.mode == FLACMI_MODE_LPC_ONLY;
    const bool do_lpc = FAST || (LMAX > 0 && ref_mode);
    const bool rice_only = !FAST && a.mode == FLACMI_MODE_RICE_ONLY;
    const bool lpc_only = !FAST && a.mode == FLACMI_MODE_LPC_ONLY;

    /* ---- LDS carve (integer offsets keep every access a ds_* instruction) ---- */
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (n % (1 << o) == 0) rmax_eff = o;
    const bool regz = FAST || resid_regz(n, rmax_eff, !WIDE && sizeof(ResT) == 4);
    const ResidLds lay = resid_lds_layout(LMAX, n, nw, 1 << (rmax_eff < 0 ? 0 : rmax_eff), S16 ? 2 : 4,
                                          (int)sizeof(ResT), CT::BYTES, regz, MF8);
    /* int8-MFMA path: digit planes (alias the residual-side regions), |c| sums and the
     * per-wave max|x| in the (unused) MFMA tap-table region */
    const int PLB = mf8_plane_bytes(n);
    uint32_t* mf8_xmax = reinterpret_cast<uint32_t*>(smem + lay.coef + CT::TAPF_OFF); /* [nw] */
    bool use_mf8 = false, lpc_pruned = false;
    int lpc_tiers = 0; /* meta.lpc_tiers */
    int mf8_G = 0;
    int16_t* xs16 = reinterpret_cast<int16_t*>(smem + lay.xs) + HP; /* [-HP, npad) (S16) */
    int32_t* xs32 = reinterpret_cast<int32_t*>(smem + lay.xs) + HP; /* [-HP, npad) (others) */
    ResT* zz = reinterpret_cast<ResT*>(smem + lay.zz);              /* [npad] (LDS-resident mode) */
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem + lay.cs);       /* [nch] (register-resident mode) */
    uint32_t* cpair = reinterpret_cast<uint32_t*>(smem + lay.coef);  /* [LMAX][PPAD] */
    int32_t* cfl = reinterpret_cast<int32_t*>(smem + lay.coef + 4 * LMAX * CT::PPAD); /* [LMAX][CPAD] */
    int32_t* lsh = cfl + LMAX * CT::CPAD; /* [3*LMAX] shift, start, 2^(31-shift) */
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + lay.red);
    Decision* dec = reinterpret_cast<Decision*>(smem + lay.dec);
    unsigned long long* rb = reinterpret_cast<unsigned long long*>(smem + lay.rb);
    int* misc = reinterpret_cast<int*>(smem + lay.misc);
    unsigned long long* hs = reinterpret_cast<unsigned long long*>(smem + lay.hs);
    int32_t* hp = reinterpret_cast<int32_t*>(smem + lay.hp);
    double* tl = reinterpret_cast<double*>(smem + lay.tl); /* log2 thresholds, e in [kTlLo, kTlLo+64) */
    flacmi_unit_meta* meta = a.meta + gid;
    const int32_t* __restrict__ rec = ref_mode ? a.rec + gid * a.rec_words : nullptr;
    /* kVarMf8: hand the unit to the list variant (workgroup-uniform callers) */
    auto list_unit = [&]() __attribute__((always_inline)) {
        if (tid == 0) {
            meta->status = FLACMI_STATUS_RETRY;
            const unsigned long long k = atomicAdd(a.retry_count, 1ull);
            a.retry_list[k] = gid;
        }
    };

    /* ---- phase A: stage samples and the candidate coefficients ---- */
    uint32_t sumx = 0; /* this thread's sum|x| (MFMA path: the fixed order-0 sum) */
    int mf_ok = 1;     /* this thread's orders pass the MFMA exactness bound */
    /* FAST: one global round trip.  The samples and the LPC record are loaded together;
     * the record is staged in LDS (in the chunk-sum region, free until phase E), and every
     * table is built from there after one barrier. */
    bool use_mfma = false;
    if constexpr (FAST) {
        int32_t* recl = reinterpret_cast<int32_t*>(smem + lay.cs);
        const int16_t* __restrict__ src = (const int16_t*)a.samples + u * a.stride;
        /* the record (<= 92 words at L <= 12) in two loads per thread: a 64-thread
         * workgroup (n <= 2560) needs both */
        static_assert(LMAX <= 12, "FAST stages at most 2 * 64 record words");
        int32_t rw[2] = {0, 0};
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (tid + j * NT < a.rec_words) rw[j] = rec[tid + j * NT];
        for (int i = tid; i < HP; i += NT) xs16[i - HP] = 0;
        for (int i = n + tid; i < resid_xpad(n); i += NT) xs16[i] = 0;
        for (int v = tid; v < (n >> 3); v += NT) { /* n % 8 == 0 */
            const uint4 q = *reinterpret_cast<const uint4*>(src + 8 * v);
            *reinterpret_cast<uint4*>(xs16 + 8 * v) = q;
            const uint32_t qd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int32_t x0 = (int32_t)(qd[e] << 16) >> 16, x1 = (int32_t)qd[e] >> 16;
                sumx += (uint32_t)(x0 < 0 ? -x0 : x0) + (uint32_t)(x1 < 0 ? -x1 : x1);
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (tid + j * NT < a.rec_words) recl[tid + j * NT] = rw[j];
        if (tid == 0) {
            misc[0] = 0x7fffffff;
            misc[1] = 0;
            misc[2] = 0;
        }
        if (tid < 32) rb[tid] = 0;
        __syncthreads();
        const int st = recl[0];
        if (st != 0) { /* the reference raises inside encode_subframe_lpc */
            if (tid == 0) put_meta(meta, st & 0xffff, st >> 16, nullptr, 0);
            goto unit_done;
        }
        const uint32_t negmask = (uint32_t)recl[1];
        for (int i = tid; i < LMAX * CT::CPAD; i += NT) {
            const int pp = i / CT::CPAD + 1, j = i % CT::CPAD;
            cfl[i] = (pp <= L && j < pp) ? recl[2 + L + (pp * (pp - 1)) / 2 + j] : 0;
        }
        for (int i = tid; i < LMAX; i += NT) {
            const int sh = i < L ? recl[2 + i] : 0; /* 0..15 */
            lsh[i] = sh;
            lsh[LMAX + i] = ((negmask >> i) & 1) ? 0 : i + 1; /* first residual index */
            lsh[2 * LMAX + i] = (int32_t)(1u << (31 - sh));
            if (i < L) {
                const int32_t* cp = recl + 2 + L + (i * (i + 1)) / 2;
                int sa = 1 << sh;
#pragma unroll
                for (int j = 0; j < LMAX; ++j)
                    if (j <= i) sa += cp[j] < 0 ? -cp[j] : cp[j];
                mf_ok &= sa <= kMfmaCoefLimit;
            }
        }
        /* MFMA tap table: column col < 12 is LPC order col+1 (c_jj * 2^-shift), 12..15 the
         * fixed orders 1..4; tap(-1) = -1 is x[i] itself */
        float* tapf = reinterpret_cast<float*>(smem + lay.coef + CT::TAPF_OFF);
        for (int i = tid; i < 16 * kTapW; i += NT) {
            const int col = i / kTapW, jj = i % kTapW - 4;
            float v = 0.0f;
            if (jj == -1) {
                v = -1.0f;
            } else if (jj >= 0 && col < 12) {
                if (col < L && col < LMAX && jj <= col) {
                    const int sh = recl[2 + col];
                    v = (float)recl[2 + L + (col * (col + 1)) / 2 + jj] * __uint_as_float((uint32_t)(127 - sh) << 23);
                }
            } else if (jj >= 0) {
                const int k = col - 11; /* fixed order k: c_jj = (-1)^jj C(k, jj+1) */
                const int f[4] = {k, -(k * (k - 1) / 2), k * (k - 1) * (k - 2) / 6, -(k * (k - 1) * (k - 2) * (k - 3) / 24)};
                v = jj < 4 ? (float)f[jj] : 0.0f;
            }
            tapf[i] = v;
        }
        use_mfma = __syncthreads_and(mf_ok) && a.mfma;
    } else {

    /* the unit's LPC status: loaded now, tested after the staging loads are in flight (a
     * test here would put one more HBM round trip in front of them) */
    const int st_rec = (M8V && pre_now) ? pre_st : ref_mode ? rec[0] : 0;
    /* int8-MFMA builds: the record's words tid and tid + NT, loaded beside the samples (the
     * coefficient table is scattered from them after the staging loop instead of gathered
     * from HBM in a second round trip); clamped indices, no guarded loads */
    int32_t rv[2] = {0, 0};
    const bool rec_regs = MF8 && do_lpc && 2 * NT >= a.rec_words;
    if constexpr (MF8) {
        if (M8V && pre_now) {
            rv[0] = pre_rv0;
            rv[1] = pre_rv1;
        } else if (rec_regs) {
#pragma unroll
            for (int j = 0; j < 2; ++j) rv[j] = rec[min(tid + j * NT, a.rec_words - 1)];
        }
    }
    if constexpr (S16) {
        for (int i = tid; i < HP; i += NT) xs16[i - HP] = 0;
        for (int i = n + tid; i < resid_xpad(n); i += NT) xs16[i] = 0;
        const int16_t* __restrict__ src = (const int16_t*)a.samples + u * a.stride;
        const int nv = n >> 3;
        if constexpr (MF) {
            /* also sum|x|: the fixed order-0 sum of the MFMA path */
            for (int v = tid; v < nv; v += NT) {
                const uint4 q = *reinterpret_cast<const uint4*>(src + 8 * v);
                *reinterpret_cast<uint4*>(xs16 + 8 * v) = q;
                const uint32_t qd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int32_t x0 = (int32_t)(qd[e] << 16) >> 16, x1 = (int32_t)qd[e] >> 16;
                    sumx += (uint32_t)(x0 < 0 ? -x0 : x0) + (uint32_t)(x1 < 0 ? -x1 : x1);
                }
            }
            for (int i = nv * 8 + tid; i < n; i += NT) {
                const int32_t x = src[i];
                xs16[i] = (int16_t)x;
                sumx += (uint32_t)(x < 0 ? -x : x);
            }
        } else {
            for (int v = tid; v < nv; v += NT)
                *reinterpret_cast<uint4*>(xs16 + 8 * v) = *reinterpret_cast<const uint4*>(src + 8 * v);
            for (int i = nv * 8 + tid; i < n; i += NT) xs16[i] = src[i];
        }
    } else {
        for (int i = tid; i < HP; i += NT) xs32[i - HP] = 0;
        for (int i = n + tid; i < resid_xpad(n); i += NT) xs32[i] = 0;
        if (a.sample_bytes == 2) {
            const int16_t* __restrict__ src = (const int16_t*)a.samples + u * a.stride;
            const int nv = n >> 3;
            for (int v = tid; v < nv; v += NT) {
                const short8 s = *reinterpret_cast<const short8*>(src + 8 * v);
#pragma unroll
                for (int k = 0; k < 8; ++k) xs32[8 * v + k] = s[k];
            }
            for (int i = nv * 8 + tid; i < n; i += NT) xs32[i] = src[i];
        } else {
            const int32_t* __restrict__ src = (const int32_t*)a.samples + u * a.stride;
            const int nv = n >> 2;
            if (MF8 && a.mfma && do_lpc && L >= 1 && n % 16 == 0 && n >= 32) {
                /* stage and split into the three digit planes in one pass; track max|x| and
                 * whether every top digit fits a signed byte */
                uint32_t* pw = reinterpret_cast<uint32_t*>(smem + lay.pl);
                const int pwd = PLB >> 2;
                int32_t xhi = 0, xlo = 0; /* the thread's largest and smallest samples (0: neutral) */
                /* eight 16-byte loads in flight per thread before any is used (clamped
                 * indices, no guarded loads) */
                constexpr int KB = 8;
                if (M8V && pre_now) { /* every wave's copies of this unit have landed */
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                }
                for (int v0 = tid; v0 < nv; v0 += KB * NT) {
                    int4v qv[KB];
#pragma unroll
                    for (int k = 0; k < KB; ++k) {
                        const int v = v0 + k * NT < nv ? v0 + k * NT : nv - 1;
                        qv[k] = (M8V && pre_now) ? *reinterpret_cast<const int4v*>(xs32 + 4 * v)
                                                 : *reinterpret_cast<const int4v*>(src + 4 * v);
                    }
#pragma unroll
                    for (int k = 0; k < KB; ++k) {
                        const int v = v0 + k * NT;
                        if (v >= nv) break;
                        const int4v q = qv[k];
                        if (!(M8V && pre_now)) *reinterpret_cast<int4v*>(xs32 + 4 * v) = q;
                        /* balanced digits (mf8_digits) by bytes: x + 0x808080 has the unsigned
                         * digits d + 128 of x's balanced ones, so its bytes XOR 0x80 are the
                         * int8 digits b0, b1, b2 (valid while -0x808080 <= x <= 0x7f7f7f) */
                        uint32_t t[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            t[e] = ((uint32_t)q[e] + 0x808080u) ^ 0x808080u;
                            xhi = q[e] > xhi ? q[e] : xhi;
                            xlo = q[e] < xlo ? q[e] : xlo;
                        }
                        /* (b0 t0, b0 t1, b1 t0, b1 t1) and the same for t2, t3, then the planes */
                        const uint32_t p01 = __builtin_amdgcn_perm(t[1], t[0], 0x05010400u);
                        const uint32_t p23 = __builtin_amdgcn_perm(t[3], t[2], 0x05010400u);
                        const uint32_t q01 = __builtin_amdgcn_perm(t[1], t[0], 0x0c0c0602u);
                        const uint32_t q23 = __builtin_amdgcn_perm(t[3], t[2], 0x0c0c0602u);
                        pw[(kMf8Pad >> 2) + v] = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
                        pw[pwd + (kMf8Pad >> 2) + v] = __builtin_amdgcn_perm(p23, p01, 0x07060302u);
                        pw[2 * pwd + (kMf8Pad >> 2) + v] = __builtin_amdgcn_perm(q23, q01, 0x05040100u);
                    }
                }
                /* zero pads: the first kMf8Pad bytes and the tail of each plane (only those
                 * dwords: npad of them per plane) */
                const int tail0 = (kMf8Pad + n) >> 2, head = kMf8Pad >> 2, npad = head + (pwd - tail0);
                for (int i = tid; i < 3 * npad; i += NT) {
                    const int pl = i / npad, k = i - pl * npad;
                    pw[pl * pwd + (k < head ? k : tail0 + (k - head))] = 0u;
                }
                /* every top digit an int8 (both ends: 25-bit and wider samples reach below
                 * -0x808080), else the int64 chains */
                const bool b2ok = xhi <= 0x7f7f7f && xlo >= -0x808080;
                const uint32_t xm = max((uint32_t)xhi, 0u - (uint32_t)xlo);
                uint32_t wm = b2ok ? xm : 0xffffffffu;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    const uint32_t t = (uint32_t)__shfl_xor((int)wm, o);
                    wm = t > wm ? t : wm;
                }
                if (lane == 0) mf8_xmax[wid] = wm;
            } else {
                if (MF8 && tid < nw) mf8_xmax[tid] = 0xffffffffu;
                for (int v = tid; v < nv; v += NT)
                    *reinterpret_cast<int4v*>(xs32 + 4 * v) = *reinterpret_cast<const int4v*>(src + 4 * v);
            }
            for (int i = nv * 4 + tid; i < n; i += NT) xs32[i] = src[i];
        }
    }
    if (st_rec != 0) { /* the reference raises inside encode_subframe_lpc */
        if (tid == 0) put_meta(meta, st_rec & 0xffff, st_rec >> 16, nullptr, 0);
        goto unit_done;
    }
    if (do_lpc) {
        const uint32_t negmask = (uint32_t)rec[1];
        if (MF8 && rec_regs) {
            /* the table's zeros, then every coefficient word w = 2 + L + pp (pp - 1) / 2 + j
             * from the thread that holds it (disjoint entries: no barrier between) */
            for (int i = tid; i < LMAX * CT::CPAD; i += NT) {
                const int pp = i / CT::CPAD + 1, j = i % CT::CPAD;
                if (!(pp <= L && j < pp)) cfl[i] = 0;
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int w = tid + k * NT - 2 - L;
                if (w >= 0 && w < (L * (L + 1)) / 2) {
                    int pp = (int)((1.0f + __builtin_sqrtf(1.0f + 8.0f * (float)w)) * 0.5f);
                    if ((pp * (pp - 1)) / 2 > w) --pp;
                    if ((pp * (pp + 1)) / 2 <= w) ++pp;
                    cfl[(pp - 1) * CT::CPAD + (w - (pp * (pp - 1)) / 2)] = rv[k];
                }
            }
        } else {
            for (int i = tid; i < LMAX * CT::CPAD; i += NT) {
                const int pp = i / CT::CPAD + 1, j = i % CT::CPAD;
                cfl[i] = (pp <= L && j < pp) ? rec[2 + L + (pp * (pp - 1)) / 2 + j] : 0;
            }
        }
        /* pair t of order pp: (lo = c[2t], hi = c[2t-1]) with c[-1] = -2^shift (S16 and
         * W64S paths only) */
        if (S16 || SPLIT)
        for (int i = tid; i < LMAX * CT::PPAD; i += NT) {
            const int pp = i / CT::PPAD + 1, t = i % CT::PPAD;
            const int32_t* cp = rec + 2 + L + (pp * (pp - 1)) / 2;
            const int32_t lo = (pp <= L && 2 * t < pp) ? cp[2 * t] : 0;
            const int32_t hi = (pp <= L && t >= 1 && 2 * t - 1 < pp) ? cp[2 * t - 1]
                               : (pp <= L && t == 0) ? -(1 << rec[2 + pp - 1]) : 0;
            cpair[i] = ((uint32_t)hi << 16) | ((uint32_t)lo & 0xffffu);
        }
        for (int i = tid; i < LMAX; i += NT) {
            const int sh = i < L ? rec[2 + i] : 0; /* 0..15 */
            lsh[i] = sh;
            lsh[LMAX + i] = ((negmask >> i) & 1) ? 0 : i + 1; /* first residual index */
            lsh[2 * LMAX + i] = (int32_t)(1u << (31 - sh));
            if (SPLIT) { /* narrow flag: samples <= 24 bits and sum|c| < 30 * 2^sh, so
                          * |pred >> sh| < 2^28 + 2^23 and |r| < 2^28 */
                int64_t sa = 0;
                if (i < L) {
                    const int32_t* cp = rec + 2 + L + (i * (i + 1)) / 2;
                    for (int j = 0; j <= i; ++j) sa += cp[j] < 0 ? -cp[j] : cp[j];
                }
                lsh[2 * LMAX + i] = (i < L && a.sample_bits <= 24 && sa < 30LL * (1LL << sh)) ? 1 : 0;
            }
            if (MF && i < L) {
                const int32_t* cp = rec + 2 + L + (i * (i + 1)) / 2;
                int sa = 1 << sh;
                for (int j = 0; j <= i; ++j) sa += cp[j] < 0 ? -cp[j] : cp[j];
                mf_ok &= sa <= kMfmaCoefLimit;
            }
        }
    }
    if constexpr (MF) {
        /* MFMA tap table: column col < 12 is LPC order col+1 (c_jj * 2^-shift), 12..15 the
         * fixed orders 1..4; tap(-1) = -1 is x[i] itself */
        float* tapf = reinterpret_cast<float*>(smem + lay.coef + CT::TAPF_OFF);
        if (do_lpc) {
            for (int i = tid; i < 16 * kTapW; i += NT) {
                const int col = i / kTapW, jj = i % kTapW - 4;
                float v = 0.0f;
                if (jj == -1) {
                    v = -1.0f;
                } else if (jj >= 0 && col < 12) {
                    if (col < L && col < LMAX && jj <= col) {
                        const int sh = rec[2 + col];
                        v = (float)rec[2 + L + (col * (col + 1)) / 2 + jj] * __uint_as_float((uint32_t)(127 - sh) << 23);
                    }
                } else if (jj >= 0) {
                    const int k = col - 11; /* fixed order k: c_jj = (-1)^jj C(k, jj+1) */
                    const int f[4] = {k, -(k * (k - 1) / 2), k * (k - 1) * (k - 2) / 6, -(k * (k - 1) * (k - 2) * (k - 3) / 24)};
                    v = jj < 4 ? (float)f[jj] : 0.0f;
                }
                tapf[i] = v;
            }
        }
    }
    if (tid == 0) {
        misc[0] = 0x7fffffff;
        misc[1] = 0;
        misc[2] = 0;
    }
    if (tid < 32) rb[tid] = 0;
    if (tid < 64) tl[tid] = a.log2thr[tid + kTlLo + 1074];
    if constexpr (MF) {
        use_mfma = __syncthreads_and(mf_ok) && do_lpc && a.mfma;
    } else {
        __syncthreads();
    }
    }
    if constexpr (MF8) {
        if (a.sample_bytes == 4 && a.mfma && do_lpc && L >= 1 && n % 16 == 0 && n >= 32) {
            /* the unit's bound B on |r| and |floor(pred / 2^s)|, lane-parallel over the
             * orders (lane p-1) and reduced over wave 0, whose verdict (int8 path or not, tiles
             * per u32 partial sum) the other waves read after one barrier */
            if (wid == 0) {
                uint32_t xm = lane < nw ? mf8_xmax[lane] : 0u;
                uint64_t b = 0;
                if (lane < L) {
                    const int p = lane + 1;
                    uint32_t sa = 0;
                    bool cok = true;
#pragma unroll
                    for (int j = 0; j < LMAX; ++j) {
                        const int32_t c = j < p ? cfl[lane * CT::CPAD + j] : 0;
                        cok &= c <= 32639 && c >= -32640; /* the top coefficient digit fits a byte */
                        sa += (uint32_t)(c < 0 ? -c : c);
                    }
                    b = cok ? ((uint64_t)sa << 32) | (uint32_t)lsh[lane] : ~0ull;
                }
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    const uint32_t t = (uint32_t)__shfl_xor((int)xm, o);
                    xm = t > xm ? t : xm;
                }
                uint64_t bl = 0;
                if (lane < L)
                    bl = b == ~0ull || xm >= (1u << 31) ? ~0ull
                                                        : (uint64_t)xm + (((b >> 32) * (uint64_t)xm) >> (b & 31)) + 1;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    const uint64_t t = (uint64_t)__shfl_xor((unsigned long long)bl, o);
                    bl = t > bl ? t : bl;
                }
                const uint64_t bmax = bl;
                int v = 0;
                if ((bmax >> 29) == 0) {
                    const uint64_t g = 0xffffffffull / (4 * bmax); /* >= 2 under bmax < 2^29 */
                    v = 1 | ((g > 64 ? 64 : (int)g) << 8);
                }
                if (lane == 0) misc[5] = v;
            }
            __syncthreads();
            const int v = __builtin_amdgcn_readfirstlane(misc[5]);
            if (v & 1) {
                use_mf8 = true;
                mf8_G = v >> 8; /* wave-uniform */
            }
        }
    }
    if (a.stop_after == 1) goto unit_done;
    if constexpr (M8V) {
        if (!use_mf8) { /* outside the int8 bounds: the int64 chains of the list variant */
            list_unit();
            goto unit_done;
        }
    }

    /* ---- phase B: sum|r| for fixed orders 0..4 and LPC orders 1..L ---- */
    if (FAST && !use_mfma) { /* outside the MFMA exactness bound: the generic kernel redoes it */
        if (tid == 0) {
            meta->status = FLACMI_STATUS_RETRY;
            const unsigned long long k = atomicAdd(a.retry_count, 1ull);
            a.retry_list[k] = gid;
        }
        goto unit_done;
    }
    if (use_mfma) {
        if constexpr (MF)
            mfma_candidate_sums<LMAX>(xs16, reinterpret_cast<const float*>(smem + lay.coef + CT::TAPF_OFF), lsh, L,
                                      n, lane, wid, nw, red, sumx);
        if (a.stop_after == 2) goto unit_done;
    } else if (MF8 && use_mf8) {
        if constexpr (MF8)
        {
            const int r = mf8_candidate_sums<LMAX>(xs32, smem + lay.pl, PLB, cfl, lsh, L, n, mf8_G, tid, NT, lane, wid,
                                                   nw, red, a.prune != 0 && !lpc_only && !rice_only, a.stop_after,
                                                   a.sign_bound != 0);
            lpc_pruned = (r >> 8) != 0;
            lpc_tiers = r ? (r & 0xff) | (8 << 8) : 0;
        }
        if (a.stop_after == 2) goto unit_done;
    } else if constexpr (!FAST && !M8V) {
    A acc[NSUM];
#pragma unroll
    for (int s = 0; s < NSUM; ++s) acc[s] = 0;
    bool full_pass = true;
    if constexpr (S16) {
        /* Pruning mode, 16-bit samples (e.g. the units k_resid_stream hands over outside its
         * MFMA bound): the exact fixed sums and the sign-correlation bound first (as
         * mf8_candidate_sums does for 24-bit), the LPC chains only for a unit it leaves open */
        if (do_lpc && a.prune && a.sign_bound && a.mode == FLACMI_MODE_REFERENCE && n >= 2 * HP) {
            int32_t kk[LMAX + 1];
#pragma unroll
            for (int j = 0; j <= LMAX; ++j) kk[j] = 0;
            uint32_t nneg = 0;
#pragma unroll 1
            for (int c = tid; c < nch; c += NT) {
                const int i0 = 8 * c;
                Win16<HP> W;
                W.load(xs16, i0);
                if (i0 >= HP && i0 + 8 <= n) {
                    chunk_sums_s16<LMAX, HP, false>(W, i0, n, L, false, cpair, lsh, acc);
                    sb16_chunk<LMAX, HP>(W, kk, nneg); /* R' = the whole chunks inside [HP, n) */
                } else {
                    chunk_sums_s16<LMAX, HP, true>(W, i0, n, L, false, cpair, lsh, acc);
                }
            }
            kk[0] -= (int32_t)nneg; /* K_0 - N_- */
            /* per wave: the five fixed sums, then K_0 - N_-, K_1 .. K_LMAX (|K| per lane < 2^26) */
            constexpr int RS1 = NSUM + 1;
            uint32_t any = 0;
#pragma unroll
            for (int o = 0; o < 5; ++o) any |= acc[o];
            const bool narrow = __ballot(any >= (1u << 26)) == 0;
#pragma unroll
            for (int o = 0; o < 5; ++o) {
                const uint64_t v = narrow ? (uint64_t)wave_sum_u32((uint32_t)acc[o]) : wave_sum_u64((uint64_t)acc[o]);
                if (lane == 0) red[wid * RS1 + o] = v;
            }
#pragma unroll
            for (int j = 0; j <= LMAX; ++j) {
                const uint32_t v = wave_sum_u32((uint32_t)kk[j]);
                if (lane == 0) red[wid * RS1 + 5 + j] = (unsigned long long)(int64_t)(int32_t)v;
            }
            __syncthreads();
            if (wid == 0) {
                uint64_t tf = 0;
                int64_t kt = 0;
                if (lane < 5)
                    for (int w2 = 0; w2 < nw; ++w2) tf += red[w2 * RS1 + lane];
                if (lane <= LMAX)
                    for (int w2 = 0; w2 < nw; ++w2) kt += (int64_t)red[w2 * RS1 + 5 + lane];
                auto l64 = [&](uint64_t v, int l) __attribute__((always_inline)) -> uint64_t {
                    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
                };
                const uint64_t f0 = l64(tf, 0);
                uint64_t fmin = f0;
#pragma unroll
                for (int o = 1; o < 5; ++o) fmin = l64(tf, o) < fmin ? l64(tf, o) : fmin;
                const int64_t k0n = (int64_t)l64((uint64_t)kt, 0);
                const int p = lane + 1;
                int64_t S = 0;
#pragma unroll
                for (int j = 1; j <= LMAX; ++j) {
                    const int64_t kj = (int64_t)l64((uint64_t)kt, j);
                    const int32_t c = (p <= L && j <= p) ? cfl[lane * CT::CPAD + j - 1] : 0;
                    S += (int64_t)c * kj;
                }
                bool lose = true; /* order p provably loses to the best fixed sum */
                if (p <= L) {
                    if (lsh[LMAX + lane] == 0) lose = f0 > fmin; /* coefficient-less: r = x, the order-0 sum */
                    else lose = k0n - (S >> lsh[lane]) - 1 > (int64_t)fmin;
                }
                const bool decided = __ballot(!lose) == 0; /* every lane votes (outside the lane-0 store) */
                if (lane == 0) misc[6] = decided ? 1 : 0;
            }
            __syncthreads();
            if (misc[6]) {
                full_pass = false;
                lpc_pruned = true;
                lpc_tiers = 1 << 8; /* "0/1": decided before the LPC pass */
            } else {
                lpc_tiers = 1 | (1 << 8);
#pragma unroll
                for (int s2 = 0; s2 < NSUM; ++s2) acc[s2] = 0;
            }
        }
    }
#pragma unroll 1
    for (int c = rice_only || !full_pass ? nch : tid; c < nch; c += NT) {
        const int i0 = 8 * c;
        const bool fast = (i0 >= HP) && (i0 + 8 <= n);
        if constexpr (S16) {
            Win16<HP> W;
            W.load(xs16, i0);
            if (fast) chunk_sums_s16<LMAX, HP, false>(W, i0, n, L, do_lpc, cpair, lsh, acc);
            else chunk_sums_s16<LMAX, HP, true>(W, i0, n, L, do_lpc, cpair, lsh, acc);
        } else {
            int32_t w[HP + 8];
            const int4v* src = reinterpret_cast<const int4v*>(xs32 + i0 - HP);
#pragma unroll
            for (int g = 0; g < (HP + 8) / 4; ++g) {
                const int4v v = src[g];
#pragma unroll
                for (int e = 0; e < 4; ++e) w[4 * g + e] = v[e];
            }
            if (fast) chunk_sums_32<LMAX, HP, false, WIDE, SPLIT>(w, i0, n, L, do_lpc, cfl, lsh, acc, cpair);
            else chunk_sums_32<LMAX, HP, true, WIDE, SPLIT>(w, i0, n, L, do_lpc, cfl, lsh, acc, cpair);
        }
    }

    if (a.stop_after == 2) {
        if (tid == 0) meta->rice_bits = (long long)acc[0] + (long long)acc[NSUM - 1];
        goto unit_done;
    }
    /* ---- phase C: workgroup reduction ---- */
    {
        bool narrow = false;
        if constexpr (!WIDE) {
            uint32_t any = 0;
#pragma unroll
            for (int s = 0; s < NSUM; ++s) any |= acc[s];
            narrow = __ballot(any >= (1u << 26)) == 0; /* every partial < 2^26: wave totals fit 32 bits */
        }
        if (narrow) {
#pragma unroll
            for (int s = 0; s < NSUM; ++s) {
                const uint32_t v = wave_sum_u32((uint32_t)acc[s]);
                if (lane == 0) red[wid * NSUM + s] = v;
            }
        } else {
#pragma unroll
            for (int s = 0; s < NSUM; ++s) {
                const uint64_t v = wave_sum_u64((uint64_t)acc[s]);
                if (lane == 0) red[wid * NSUM + s] = v;
            }
        }
    }
    }
    __syncthreads();

    /* ---- phase D: choice (encoder.py:331-359, 398-404, 135-157) by wave 0; lane j holds
     * total j (fixed orders 0..4, then LPC orders 1..L) ---- */
    if (wid == 0) {
        uint64_t tj = 0;
        if (lane < NSUM)
            for (int w2 = 0; w2 < nw; ++w2) tj += red[w2 * NSUM + lane];
        const uint32_t tlo = (uint32_t)tj, thi = (uint32_t)(tj >> 32);
        auto tot_at = [&](int j) __attribute__((always_inline)) -> uint64_t {
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)thi, j) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)tlo, j);
        };
        int fo = 0;
        uint64_t fsum = tot_at(0);
        if (n > 4) {
#pragma unroll
            for (int o = 1; o < 5; ++o) {
                const uint64_t v = tot_at(o);
                if (v < fsum) {
                    fsum = v;
                    fo = o;
                }
            }
        }
        int kind = FLACMI_KIND_FIXED, dorder = fo, dshift = 0, ncoefs = 0, lbest = 0, st = ST_OK, site = 0;
        uint64_t lsum = 0;
        if (rice_only) {
            fo = 0;
            fsum = 0;
            dorder = a.rice_order; /* identity "predictor": the row already is the residual */
        }
        if (do_lpc && lpc_pruned) { /* every LPC candidate provably loses (mf8_candidate_sums) */
            lbest = FLACMI_LPC_PRUNED;
            lsum = (uint64_t)(int64_t)FLACMI_LPC_PRUNED;
        } else if (do_lpc) {
            lbest = 1;
            lsum = tot_at(5);
            static_for<LMAX>([&](auto P_) {
                constexpr int pp = P_ + 1;
                if (pp >= 2 && pp <= L) {
                    const uint64_t v = tot_at(4 + pp);
                    if (v < lsum) {
                        lsum = v;
                        lbest = pp;
                    }
                }
            });
            if (lpc_only) {
                kind = FLACMI_KIND_LPC;
                dorder = lbest;
                dshift = lsh[lbest - 1];
                ncoefs = lsh[LMAX + lbest - 1] == 0 ? 0 : lbest;
            } else if (lsum < fsum) {
                /* A coefficient-less candidate (negative-shift branch) sums |x| over all n
                 * samples, exactly the fixed order-0 sum, so it never gets here. */
                kind = FLACMI_KIND_LPC;
                dorder = lbest;
                dshift = lsh[lbest - 1];
                ncoefs = lbest;
            } else if (!(fsum < lsum)) {
                st = ST_ASSERT;
                site = FLACMI_SITE_CHOICE_TIE;
            }
        }
        if (lane == 0) {
            dec->status = st;
            dec->site = site;
            dec->kind = kind;
            dec->order = dorder;
            dec->shift = dshift;
            dec->ncoefs = ncoefs;
            dec->fixed_order = fo;
            dec->lpc_order = lbest;
            dec->tiers = lpc_tiers;
            dec->fixed_sum = (long long)fsum;
            dec->lpc_sum = (long long)lsum;
        }
        if (lane < FLACMI_MAX_LPC_ORDER) {
            int cv = 0;
            if (kind == FLACMI_KIND_LPC) cv = lane < lbest ? cfl[(lbest - 1) * CT::CPAD + lane] : 0;
            else if (!rice_only && lane < 4) cv = c_fixed_coef[fo][lane];
            dec->coef[lane] = cv;
        }
        if (a.fixed_sums && lane < 5) a.fixed_sums[gid * 5 + lane] = (n > 4 || lane == 0) ? (long long)tj : 0;
        if (a.lpc_sums) {
            const uint64_t v = (uint64_t)__shfl((unsigned long long)tj, (lane + 5) & 63);
            if (lane < 32) a.lpc_sums[gid * 32 + lane] = (do_lpc && lane + 1 <= L) ? (long long)v : 0;
        }
    }
    __syncthreads();
    const int dstatus = dec->status;
    if (dstatus != ST_OK) {
        if (tid == 0) put_meta(meta, dstatus, dec->site, dec, 0);
        goto unit_done;
    }
    if (a.stop_after == 3) goto unit_done;
    const int order = dec->order;
    const int dshift = dec->shift;
    /* the residual starts at index len(warmup); a coefficient-less LPC subframe (only
     * reachable in LPC-only mode) keeps every sample */
    const int start = (dec->kind == FLACMI_KIND_LPC && dec->ncoefs == 0) ? 0 : order;
    constexpr int TAPS = LMAX > 4 ? LMAX : 4;

    /* ---- phase E: chosen residual, zig-zag, to HBM and to registers or LDS ---- */
    int wide_flag = 0;
    ResT* __restrict__ rout = reinterpret_cast<ResT*>(a.residual) + gid * a.residual_stride;
    int32_t cf[TAPS];
#pragma unroll
    for (int j = 0; j < TAPS; ++j) cf[j] = dec->coef[j];
    auto resid_chunk = [&](int c, ResT (&zv)[8]) __attribute__((always_inline)) {
        const int i0 = 8 * c;
        int32_t w[HP + 8];
        if constexpr (S16) {
            const uint4* src = reinterpret_cast<const uint4*>(xs16 + i0 - HP);
#pragma unroll
            for (int g = 0; g < (HP + 8) / 8; ++g) {
                const uint4 v = src[g];
                const uint32_t q4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    w[8 * g + 2 * e] = (int32_t)(int16_t)(q4[e] & 0xffff);
                    w[8 * g + 2 * e + 1] = (int32_t)q4[e] >> 16;
                }
            }
        } else {
            const int4v* src = reinterpret_cast<const int4v*>(xs32 + i0 - HP);
#pragma unroll
            for (int g = 0; g < (HP + 8) / 4; ++g) {
                const int4v v = src[g];
#pragma unroll
                for (int e = 0; e < 4; ++e) w[4 * g + e] = v[e];
            }
        }
        static_for<8>([&](auto K_) {
            constexpr int k = K_;
            int64_t r;
            if constexpr (!WIDE) {
                int32_t pred = 0;
                if (order <= 4) {
                    static_for<4>([&](auto J_) { pred += sext24(cf[J_]) * sext24(w[HP + k - 1 - J_]); });
                } else {
                    static_for<TAPS>([&](auto J_) { pred += sext24(cf[J_]) * sext24(w[HP + k - 1 - J_]); });
                }
                r = (int64_t)(w[HP + k] - (pred >> dshift));
            } else {
                /* only the chosen predictor's taps: coefficients past its order are zero
                 * (a fixed predictor, the common choice, has at most 4) */
                int64_t pred = 0;
                auto taps = [&](auto NT_) __attribute__((always_inline)) {
                    static_for<decltype(NT_)::value>(
                        [&](auto J_) { pred += (int64_t)cf[J_] * (int64_t)w[HP + k - 1 - J_]; });
                };
                if (order <= 4) taps(std::integral_constant<int, (TAPS < 4 ? TAPS : 4)>{});
                else if (sizeof(ResT) == 4 && order <= 16) taps(std::integral_constant<int, (TAPS < 16 ? TAPS : 16)>{});
                else taps(std::integral_constant<int, TAPS>{});
                r = (int64_t)w[HP + k] - (pred >> dshift);
            }
            const int i = i0 + k;
            ResT z;
            if constexpr (sizeof(ResT) == 4) {
                if (WIDE && !(r >= -(1LL << 31) && r < (1LL << 31)) && i >= start && i < n) wide_flag = 1;
                const int32_t r32 = (int32_t)r;
                z = (ResT)(((uint32_t)r32 << 1) ^ (uint32_t)(r32 >> 31));
            } else {
                z = (ResT)(((uint64_t)r << 1) ^ (uint64_t)(r >> 63));
            }
            zv[k] = (i >= start && i < n) ? z : (ResT)0;
        });
    };
    auto store_chunk = [&](int c, const ResT (&zv)[8]) __attribute__((always_inline)) {
        const int i0 = 8 * c;
        if constexpr (sizeof(ResT) == 4) {
            if (i0 + 8 <= n) {
                reinterpret_cast<uint4*>(rout + i0)[0] = uint4{zv[0], zv[1], zv[2], zv[3]};
                reinterpret_cast<uint4*>(rout + i0)[1] = uint4{zv[4], zv[5], zv[6], zv[7]};
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (i0 + k < n) rout[i0 + k] = zv[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (i0 + k < n) rout[i0 + k] = zv[k];
        }
    };
    auto lpc_only_done = [&]() __attribute__((always_inline)) {
        if (tid == 0) {
            put_meta(meta, ST_OK, 0, dec, 1);
            meta->res_offset = start;
            meta->res_len = n - start;
            meta->part_order = -1;
        }
    };
    auto first_order = [&]() __attribute__((always_inline)) {
        int om = -1;
        for (int o = a.rmin; o <= a.rmax; ++o)
            if ((n % (1 << o)) == 0 && (n >> o) > order) om = o;
        return om;
    };

    if constexpr (!WIDE && sizeof(ResT) == 4) {
        if (regz) {
            /* register-resident residual: chunk c = tid + j*NT, j < kCPT */
            uint32_t zr[kCPT][8];
            const int fixed_order = __builtin_amdgcn_readfirstlane(dec->kind == FLACMI_KIND_FIXED ? order : -1);
#pragma unroll
            for (int j = 0; j < kCPT; ++j) {
                const int c = tid + j * NT;
                if (c < nch) {
                    if (FAST && fixed_order >= 0) { /* n % 8 == 0 here: every chunk is whole */
                        switch (fixed_order) {
                            case 0: fixed_resid_chunk<0>(xs16, 8 * c, zr[j]); break;
                            case 1: fixed_resid_chunk<1>(xs16, 8 * c, zr[j]); break;
                            case 2: fixed_resid_chunk<2>(xs16, 8 * c, zr[j]); break;
                            case 3: fixed_resid_chunk<3>(xs16, 8 * c, zr[j]); break;
                            default: fixed_resid_chunk<4>(xs16, 8 * c, zr[j]); break;
                        }
                    } else {
                        resid_chunk(c, zr[j]);
                    }
                    store_chunk(c, zr[j]);
                    cs[c] = zr[j][0] + zr[j][1] + zr[j][2] + zr[j][3] + zr[j][4] + zr[j][5] + zr[j][6] + zr[j][7];
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) zr[j][k] = 0;
                }
            }
            __syncthreads();
            if (a.stop_after == 4) goto unit_done;
            if (lpc_only) {
                lpc_only_done();
                goto unit_done;
            }
            /* ---- phase F (register-resident) ---- */
            const int omax = first_order();
            if (omax < 0) {
                if (tid == 0) put_meta(meta, ST_ASSERT, FLACMI_SITE_RICE_NO_ORDER, dec, 1);
                goto unit_done;
            }
            const int cpp = (n >> omax) >> 3; /* chunks per finest partition */
            uint8_t* pk = reinterpret_cast<uint8_t*>(hs);
            if (wid == 0) {
                uint64_t s = 0;
                if (lane < (1 << omax)) {
#pragma unroll 6
                    for (int c = lane * cpp; c < (lane + 1) * cpp; ++c) s += cs[c];
                }
                /* FAST: residual < 2^27 and n <= 6144, so every partition sum < 2^40 */
                rice_params_wave0<FAST>(a, s, tl, rb, misc, pk, n, order, a.rmin, omax, lane);
            }
            __syncthreads();
            if (misc[0] >= 0) {
                if (tid == 0) put_meta(meta, ST_VALUE, misc[1], dec, 1);
                goto unit_done;
            }
            const int ro = __builtin_amdgcn_readfirstlane(a.rmin), oo = __builtin_amdgcn_readfirstlane(omax);
            uint32_t tb[16];
#pragma unroll
            for (int o = 0; o < 16; ++o) tb[o] = 0;
#pragma unroll
            for (int j = 0; j < kCPT; ++j) {
                const int c = tid + j * NT;
                if (c < nch) chunk_rice_bits(zr[j], *reinterpret_cast<const uint4*>(pk + 16 * (c / cpp)), ro, oo, tb);
            }
            rice_finish(a, meta, dec, tb, rb, red, misc, pk, n, start, a.rmin, omax, tid, NT, lane, wid, nw, gid);
            goto unit_done;
        }
    }
    if constexpr (!FAST) {
    /* WIDE, 32-bit rows, 64..256 finest partitions of at most 64 whole chunks each: the
     * finest partition sums are reduced here across the cpp consecutive lanes that own a
     * partition's chunks, into the heap's finest nodes, for the per-node parameter step */
    int wr_om = -1, wr_cpp = 0;
    if constexpr (WIDE && sizeof(ResT) == 4) {
        const int om = first_order();
        const int cpp = (n >> om) >> 3;
        /* the chunk sums reduce over a partition's lanes by a butterfly: cpp a power of two
         * (n = 4608 at order 6 has 9 chunks per partition: the generic heap path takes it) */
        if (om >= 6 && om <= 8 && ((n >> om) & 7) == 0 && cpp <= 64 && (cpp & (cpp - 1)) == 0 &&
            a.mode != FLACMI_MODE_LPC_ONLY) {
            wr_om = om;
            wr_cpp = (n >> om) >> 3;
        }
    }
    wr_om = __builtin_amdgcn_readfirstlane(wr_om);
    /* int8-MFMA units (|x| <= 2^23) that chose a fixed predictor: int32 difference chains */
    const int wfk = __builtin_amdgcn_readfirstlane(
        (MF8 && use_mf8 && dec->kind == FLACMI_KIND_FIXED && order <= 4) ? order : -1);
    if constexpr (M8V) {
        if (wfk < 0 || wr_om < 0) { /* an LPC (or order > 4) choice, or another Rice shape */
            list_unit();
            goto unit_done;
        }
    }
    auto wide_pass = [&](auto kk) __attribute__((always_inline)) {
    constexpr int KK = decltype(kk)::value;
#pragma unroll 1
    for (int c = tid; c < nch; c += NT) {
        ResT zv[8];
        if constexpr (KK >= 0) fixed_resid_chunk32<KK>(xs32, 8 * c, n, zv);
        else resid_chunk(c, zv);
        store_chunk(c, zv);
        if (WIDE && sizeof(ResT) == 4 && wr_om >= 0) {
            uint64_t cs8 = 0;
            if constexpr (KK >= 0) { /* difference chains: every value < 2^28, eight < 2^31 */
                uint32_t c32 = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) c32 += (uint32_t)zv[k];
                cs8 = c32;
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) cs8 += (uint64_t)zv[k];
            }
            for (int w = 1; w < wr_cpp; w <<= 1) cs8 += (uint64_t)__shfl_xor((unsigned long long)cs8, w);
            if ((c & (wr_cpp - 1)) == 0) hs[(1 << wr_om) + c / wr_cpp] = cs8;
        }
        if constexpr (sizeof(ResT) == 4) {
            reinterpret_cast<uint4*>(zz + 8 * c)[0] = uint4{zv[0], zv[1], zv[2], zv[3]};
            reinterpret_cast<uint4*>(zz + 8 * c)[1] = uint4{zv[4], zv[5], zv[6], zv[7]};
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) zz[8 * c + k] = zv[k];
        }
    }
    };
    if constexpr (MF8) {
        switch (wfk) {
            case 0: wide_pass(std::integral_constant<int, 0>{}); break;
            case 1: wide_pass(std::integral_constant<int, 1>{}); break;
            case 2: wide_pass(std::integral_constant<int, 2>{}); break;
            case 3: wide_pass(std::integral_constant<int, 3>{}); break;
            case 4: wide_pass(std::integral_constant<int, 4>{}); break;
            default:
                if constexpr (!M8V) wide_pass(std::integral_constant<int, -1>{});
                break;
        }
    } else {
        wide_pass(std::integral_constant<int, -1>{});
    }
    if (wide_flag) misc[2] = 1;
    __syncthreads();
    if (a.stop_after == 4) goto unit_done;
    if (misc[2]) {
        if (tid == 0) put_meta(meta, FLACMI_STATUS_RESIDUAL_WIDE, FLACMI_SITE_RESIDUAL_WIDTH, dec, 1);
        goto unit_done;
    }
    if (a.mode == FLACMI_MODE_LPC_ONLY) {
        lpc_only_done();
        goto unit_done;
    }

    /* ---- phase F: Rice partition search (encoder.py:655-760) ---- */
    const int omax = first_order();
    if (omax < 0) {
        if (tid == 0) put_meta(meta, ST_ASSERT, FLACMI_SITE_RICE_NO_ORDER, dec, 1);
        goto unit_done;
    }
    const int rmin = a.rmin;
    const int P = 1 << omax, ps = n >> omax;
    if constexpr (!WIDE && sizeof(ResT) == 4) {
        /* zz < 2^27 here, so a chunk of eight fits 32 bits */
        if ((ps & 7) == 0 && P <= 64 && 8 * kCPT * NT >= n) {
            const int cpp = ps >> 3;
            uint8_t* pk = reinterpret_cast<uint8_t*>(hs);
            if (wid == 0) {
                uint64_t s = 0;
                if (lane < P) {
                    const uint4* z4 = reinterpret_cast<const uint4*>(zz + lane * ps);
                    for (int c = 0; c < cpp; ++c) {
                        const uint4 u = z4[2 * c], v = z4[2 * c + 1];
                        s += (uint64_t)(u.x + u.y + u.z + u.w + v.x + v.y + v.z + v.w);
                    }
                }
                rice_params_wave0<false>(a, s, tl, rb, misc, pk, n, order, rmin, omax, lane);
            }
            __syncthreads();
            if (misc[0] >= 0) {
                if (tid == 0) put_meta(meta, ST_VALUE, misc[1], dec, 1);
                goto unit_done;
            }
            const int ro = __builtin_amdgcn_readfirstlane(rmin), oo = __builtin_amdgcn_readfirstlane(omax);
            uint32_t tb[16];
#pragma unroll
            for (int o = 0; o < 16; ++o) tb[o] = 0;
            for (int c = tid; c < nch; c += NT) {
                const uint4 u = reinterpret_cast<const uint4*>(zz)[2 * c], v = reinterpret_cast<const uint4*>(zz)[2 * c + 1];
                const uint32_t z[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                chunk_rice_bits(z, *reinterpret_cast<const uint4*>(pk + 16 * (c / cpp)), ro, oo, tb);
            }
            rice_finish(a, meta, dec, tb, rb, red, misc, pk, n, start, rmin, omax, tid, NT, lane, wid, nw, gid);
            goto unit_done;
        }
    }
    if constexpr (WIDE && sizeof(ResT) == 4) {
        if (wr_om >= 0) {
            /* kVarMf8 persistent: copy the next unit's samples into the staging region (dead
             * since the chosen-residual pass) while the Rice phase runs; the barriers up to
             * the next unit are raw (lgkmcnt only), or their vmcnt(0) would drain the copies */
            if constexpr (M8V) {
                const int64_t nx = li + gridDim.x;
                pre = a.persist && nx < a.count && (n & 255) == 0 && 2 * NT >= a.rec_words;
                if (pre) {
                    /* the next unit's record status and words (registers: 3 VGPRs across the
                     * unit boundary) */
                    const int32_t* __restrict__ nrec = a.rec + nx * a.rec_words;
                    pre_st = nrec[0];
                    pre_rv0 = nrec[min(tid, a.rec_words - 1)];
                    pre_rv1 = nrec[min(tid + NT, a.rec_words - 1)];
                    /* in inline asm: issued through the builtin, the LDS-DMA makes the compiler
                     * wait for it (vmcnt(0)) before the Rice phase's next LDS access, whatever
                     * address that touches, which drains the copy at once.  This region is not
                     * read before the next unit's staging, which waits for it explicitly. */
                    const int32_t* __restrict__ nsrc = (const int32_t*)a.samples + (a.unit0 + nx) * a.stride;
                    const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>(
                        (const __attribute__((address_space(3))) int32_t*)xs32);
                    for (int b = wid; b < (n >> 8); b += nw) /* 1 KB (256 samples) per wave-instruction */
                        asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off"
                                     :
                                     : "s"(lbase + 1024u * (uint32_t)b), "v"(nsrc + 256 * b + 4 * lane)
                                     : "memory", "m0");
                }
            }
            auto rbar = [&]() __attribute__((always_inline)) {
                if constexpr (M8V) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                } else {
                    __syncthreads();
                }
            };
            /* Every heap node's parameter at once (encoder.py:655-760), one node per thread:
             *  1. wave 0: prefix sums of the finest sums (hs[P..2P), left by phase E) into the
             *     generic path's heap-parameter region (unused here): pre(k), k = 1..P;
             *  2. node j = 2^o + K (orders rmin..omax): S = pre[(K+1) 2^d] - pre[K 2^d], d =
             *     omax - o, its parameter into prmN[j], header bits summed per order (wave sums,
             *     one LDS atomic per wave and order), the first error in the reference's
             *     evaluation order (orders, then partitions: the smallest j) by atomicMin;
             *  3. finest partition k: its ancestors' parameters gathered into its 16-byte row
             *     (byte o = p_o - pm, byte 14 = some delta >= 16, byte 15 = pm), where pk aliases
             *     the finest sums step 1 has consumed.
             * No node waits on another order, and no wave runs the parameters alone. */
            uint8_t* pk = reinterpret_cast<uint8_t*>(hs);
            /* pre(k) = sum of the finest sums below k: preA[k - 1] (8P bytes, the size of hp);
             * node parameters in the coefficient region (>= 1280 bytes, dead since phase E) */
            unsigned long long* preA = reinterpret_cast<unsigned long long*>(hp); /* [P] */
            uint8_t* prmN = reinterpret_cast<uint8_t*>(smem + lay.coef);        /* [2P] */
            const int ro = __builtin_amdgcn_readfirstlane(rmin), oo = __builtin_amdgcn_readfirstlane(omax);
            if (wid == 0) {
                const int J = P >> 6; /* finest partitions per lane: 1, 2 or 4 */
                uint64_t v[4] = {0, 0, 0, 0}, t = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < J) v[j] = hs[P + J * lane + j], t += v[j];
                uint64_t inc = t; /* inclusive scan of the lane totals */
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t u = (uint64_t)__shfl_up((unsigned long long)inc, (unsigned)d);
                    if (lane >= d) inc += u;
                }
                uint64_t e = inc - t;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < J) e += v[j], preA[J * lane + j] = e;
                if (lane < 16) rb[lane] = 0;
                if (lane == 0) misc[0] = 0x7fffffff, misc[4] = 0;
            }
            rbar();
            {
                const bool intlog = n <= 16384; /* S < n 2^32 <= 2^46: exact integer floor(log2(S / len)) */
                for (int j0 = (1 << ro); j0 < 2 * P; j0 += NT) {
                    const int j = j0 + tid;
                    const bool live = j < 2 * P;
                    const int o = live ? 31 - __builtin_clz((unsigned)j) : 0;
                    uint32_t hb = 0;
                    bool big = false;
                    if (live) {
                        const int K = j - (1 << o), d = omax - o;
                        const uint64_t S = preA[((K + 1) << d) - 1] - (K > 0 ? preA[(K << d) - 1] : 0ull);
                        const int len = (n >> o) - (K == 0 ? order : 0);
                        int prm = 0;
                        if (S != 0) {
                            if (intlog) {
                                const int fs = 63 - __builtin_clzll((unsigned long long)S);
                                const int fl = 31 - __builtin_clz((unsigned)len);
                                prm = fs - fl;
                                if (prm >= 0 && ((uint64_t)len << prm) > S) --prm;
                            } else {
                                prm = rice_floor_log2((double)S / (double)len, tl, a.log2thr);
                            }
                        }
                        prmN[j] = (uint8_t)prm;
                        if (S == 0 || prm < 0) atomicMin(&misc[0], (j << 1) | (S == 0 ? 1 : 0));
                        big = prm > 14;
                        hb = 4u + (prm > 14 ? 5u : 4u) + (uint32_t)len * (uint32_t)(1 + prm);
                    }
                    /* header bits: one wave sum per order this wave's nodes span; the orders with a
                     * parameter > 14 (five-bit coding) by ballot, one LDS atomic per wave */
                    const int jw = __builtin_amdgcn_readfirstlane(j);
                    const int ow0 = 31 - __builtin_clz((unsigned)jw);
                    const int jl = min(jw + 63, 2 * P - 1);
                    const int ow1 = 31 - __builtin_clz((unsigned)jl);
                    for (int ow = ow0; ow <= ow1; ++ow) {
                        const uint32_t hs32 = wave_sum_u32(live && o == ow ? hb : 0u);
                        if (lane == 0 && jw < 2 * P) atomicAdd(&rb[ow], (unsigned long long)hs32);
                        if (__ballot(live && o == ow && big) && lane == 0) atomicOr(&misc[4], 1 << ow);
                    }
                }
            }
            rbar();
            if (a.stop_after == 5) goto unit_done; /* ablation: after the parameters */
            if (misc[0] != 0x7fffffff) {
                if (tid == 0)
                    put_meta(meta, ST_VALUE, (misc[0] & 1) ? FLACMI_SITE_RICE_LOG_DOMAIN : FLACMI_SITE_RICE_NEG_SHIFT,
                             dec, 1);
                goto unit_done;
            }
            const int cpp = ps >> 3;
            for (int k = tid; k < P; k += NT) {
                uint32_t w[4] = {0, 0, 0, 0};
                uint32_t pm = 255, dmax = 0;
                uint32_t pv[13];
#pragma unroll
                for (int o = 0; o < 13; ++o) {
                    pv[o] = (o >= ro && o <= oo) ? prmN[(1 << o) + (k >> (omax - o))] : 0u;
                    if (o >= ro && o <= oo) pm = min(pm, pv[o]);
                }
#pragma unroll
                for (int o = 0; o < 13; ++o)
                    if (o >= ro && o <= oo) {
                        const uint32_t dl = pv[o] - pm;
                        dmax = max(dmax, dl);
                        w[o >> 2] |= dl << (8 * (o & 3));
                    }
                /* byte 14: some delta >= 16 (v_pk_lshrrev_b16 shifts by the amount mod 16, so such
                 * a row takes the 32-bit path) */
                w[3] |= ((dmax >= 16 ? 1u : 0u) << 16) | (pm << 24);
                *reinterpret_cast<uint4*>(pk + 16 * k) = uint4{w[0], w[1], w[2], w[3]};
            }
            rbar();
            if (a.stop_after == 6) goto unit_done; /* ablation: after the row transform */
            const uint4* pkv = reinterpret_cast<const uint4*>(hs);
            uint64_t tb[16];
            uint32_t tp[16]; /* packed-path totals: this thread's sum(y >> d) < 4 * 8 * 2^16 per order */
#pragma unroll
            for (int o = 0; o < 16; ++o) tb[o] = 0, tp[o] = 0;
            for (int c = tid; c < nch; c += NT) {
                const uint4 u = reinterpret_cast<const uint4*>(zz)[2 * c], v = reinterpret_cast<const uint4*>(zz)[2 * c + 1];
                const uint32_t z[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                const uint4 pv = pkv[c / cpp];
                const uint32_t pm = pv.w >> 24;
                uint32_t y[8], yo = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) y[k] = z[k] >> pm, yo |= y[k];
                if ((yo >> 16) == 0 && ((pv.w >> 16) & 0xffu) == 0) { /* tp < chunks per thread * 8 * 2^16 < 2^32 */
                    uint32_t yp[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) yp[i] = __builtin_amdgcn_perm(y[2 * i + 1], y[2 * i], 0x05040100u);
                    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                    for (int o = 0; o < 16; ++o)
                        if (o >= ro && o <= oo) {
                            /* d = p_o - pm in both halves */
                            const uint32_t sel = (o & 3) == 0 ? 0x0c000c00u : (o & 3) == 1 ? 0x0c010c01u
                                                 : (o & 3) == 2 ? 0x0c020c02u : 0x0c030c03u;
                            const us2x d = __builtin_bit_cast(us2x, __builtin_amdgcn_perm(0u, pw[o >> 2], sel));
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                tp[o] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2x, yp[i]) >> d, us2x{1, 1}, tp[o], false);
                        }
                } else if (((u.x | u.y | u.z | u.w | v.x | v.y | v.z | v.w) >> 29) == 0) {
                    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w + 0u};
                    (void)pw;
                    uint32_t t32[16];
#pragma unroll
                    for (int o = 0; o < 16; ++o) t32[o] = 0;
                    chunk_rice_bits(y, pv, ro, oo, t32); /* deltas applied to y = z >> pm */
#pragma unroll
                    for (int o = 0; o < 16; ++o)
                        if (o >= ro && o <= oo) tb[o] += t32[o];
                } else {
                    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                    for (int o = 0; o < 16; ++o)
                        if (o >= ro && o <= oo) {
                            const uint32_t d = (pw[o >> 2] >> (8 * (o & 3))) & 0xffu;
#pragma unroll
                            for (int k = 0; k < 8; ++k) tb[o] += (uint64_t)(y[k] >> d);
                        }
                }
            }
#pragma unroll
            for (int o = 0; o < 16; ++o) tb[o] += tp[o];
            if (a.stop_after == 7) { /* ablation: after the data bits (kept live) */
                if (tb[0] == 0x9e3779b9u) meta->lpc_tiers = 1;
                goto unit_done;
            }
            {
                uint64_t any = 0;
#pragma unroll
                for (int o = 0; o < 16; ++o) any |= (o >= ro && o <= oo) ? tb[o] : 0ull;
                /* every lane < 2^26: 32-bit wave sums (a wave-uniform branch) */
                if (__ballot(any >= (1ull << 26)) == 0) {
#pragma unroll
                    for (int o = 0; o < 16; ++o)
                        if (o >= ro && o <= oo) {
                            const uint32_t w = wave_sum_u32((uint32_t)tb[o]);
                            if (lane == 0) red[wid * 16 + o] = w;
                        }
                } else {
#pragma unroll
                    for (int o = 0; o < 16; ++o)
                        if (o >= ro && o <= oo) {
                            const uint64_t w = wave_sum_u64(tb[o]);
                            if (lane == 0) red[wid * 16 + o] = w;
                        }
                }
            }
            rbar();
            {
                /* every wave: lane o holds order o's total (its nw partials loaded side by side);
                 * the first minimum (encoder.py:740-760) by key = total * 16 + order over lanes
                 * 0..15.  Wave 0 writes the meta record; every thread one Rice parameter (was
                 * wave 0 alone, four per lane, with the workgroup's LDS held meanwhile). */
                const bool cand = lane >= ro && lane <= oo;
                unsigned long long v = 0;
                if (cand) {
                    v = rb[lane];
                    for (int w2 = 0; w2 < nw; ++w2) v += red[w2 * 16 + lane];
                }
                unsigned long long key = cand ? (v << 4) | (unsigned long long)lane : ~0ull;
#pragma unroll
                for (int s = 8; s >= 1; s >>= 1) {
                    const unsigned long long t = __shfl_xor(key, s);
                    key = t < key ? t : key;
                }
                const int best = __builtin_amdgcn_readfirstlane((int)(key & 15u));
                const unsigned long long bits = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane(
                                                     (int)(uint32_t)(key >> 36)) << 32) |
                                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(key >> 4));
                if (wid == 0)
                    put_meta_wave(meta, lane, ST_OK, 0, dec, start, n - start, best, 1 << best,
                                  ((misc[4] >> best) & 1) ? 5 : 4, (long long)bits);
                int32_t* __restrict__ rp = a.rice_params + gid * a.params_stride;
                for (int K = tid; K < (1 << best); K += NT) {
                    const int row = 16 * (K << (omax - best));
                    rp[K] = pk[row + 15] + pk[row + best]; /* pm + delta */
                }
            }
            goto unit_done;
        }
    }
    if constexpr (!M8V) {
    /* finest partition sums: heap nodes [P, 2P); zz[i] = 0 for i < start */
    for (int k = wid; k < P; k += nw) {
        const int lo = k * ps, hi = (k + 1) * ps;
        uint64_t s = 0;
        for (int i = lo + lane; i < hi; i += 64) s += (uint64_t)zz[i];
        s = wave_sum_u64(s);
        if (lane == 0) hs[P + k] = s;
    }
    __syncthreads();
    for (int o = omax - 1; o >= rmin; --o) {
        for (int K = tid; K < (1 << o); K += NT) {
            const int j = (1 << o) + K;
            hs[j] = hs[2 * j] + hs[2 * j + 1];
        }
        __syncthreads();
    }
    /* parameters, header bits, first error in the reference's evaluation order */
    for (int j = (1 << rmin) + tid; j < 2 * P; j += NT) {
        const int o = 31 - __builtin_clz(j);
        const int K = j - (1 << o);
        const unsigned long long S = hs[j];
        const int len = (n >> o) - (K == 0 ? order : 0);
        int prm = 0;
        if (S == 0) {
            atomicMin(&misc[0], (o << 16) | K);
        } else {
            const double mean = (double)S / (double)len; /* S < 2^53: correctly rounded */
            prm = pym::py_floor_log2(mean, a.log2thr);
            if (prm < 0) atomicMin(&misc[0], (o << 16) | K);
        }
        hp[j] = prm;
        const unsigned long long hb =
            4ull + (prm > 14 ? 5ull : 4ull) + (unsigned long long)len * (unsigned long long)(1 + prm);
        atomicAdd(&rb[o], hb);
    }
    __syncthreads();
    const int ekey = misc[0];
    if (ekey != 0x7fffffff) {
        if (tid == 0) {
            const int o = ekey >> 16, K = ekey & 0xffff;
            put_meta(meta, ST_VALUE,
                     hs[(1 << o) + K] == 0 ? FLACMI_SITE_RICE_LOG_DOMAIN : FLACMI_SITE_RICE_NEG_SHIFT, dec, 1);
        }
        goto unit_done;
    }
    /* data bits: sum over the residual of (x >> p) for every candidate order at once */
    uint64_t tb[16];
#pragma unroll
    for (int o = 0; o < 16; ++o) tb[o] = 0;
    if (sizeof(ResT) == 4 && (ps & 7) == 0) {
        /* whole 8-sample chunks per partition: the heap sums are dead, so each finest
         * partition's parameters are packed there, one byte per order (16 B x P = the hs
         * region); a chunk reads its residual with two 16-byte loads and its parameters
         * with one.  Chunks whose values are all < 2^29 sum eight shifts in 32 bits. */
        uint4* pkv = reinterpret_cast<uint4*>(hs);
        __syncthreads(); /* the error scan above read hs */
        for (int k = tid; k < P; k += NT) {
            uint32_t pw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int o = 0; o < 16; ++o)
                if (o >= rmin && o <= omax) pw[o >> 2] |= ((uint32_t)hp[(1 << o) + (k >> (omax - o))] & 0xffu) << (8 * (o & 3));
            pkv[k] = uint4{pw[0], pw[1], pw[2], pw[3]};
        }
        __syncthreads();
        const int cpp = ps >> 3;
        const int ro = __builtin_amdgcn_readfirstlane(rmin), oo = __builtin_amdgcn_readfirstlane(omax);
        for (int c = tid; c < nch; c += NT) {
            const uint4 u = reinterpret_cast<const uint4*>(zz)[2 * c], v = reinterpret_cast<const uint4*>(zz)[2 * c + 1];
            const uint32_t z[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            const uint4 pv = pkv[c / cpp];
            if (((u.x | u.y | u.z | u.w | v.x | v.y | v.z | v.w) >> 29) == 0) {
                uint32_t t32[16];
#pragma unroll
                for (int o = 0; o < 16; ++o) t32[o] = 0;
                chunk_rice_bits(z, pv, ro, oo, t32);
#pragma unroll
                for (int o = 0; o < 16; ++o)
                    if (o >= ro && o <= oo) tb[o] += t32[o];
            } else {
                const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                for (int o = 0; o < 16; ++o)
                    if (o >= ro && o <= oo) {
                        const uint32_t p = (pw[o >> 2] >> (8 * (o & 3))) & 0xffu;
#pragma unroll
                        for (int k = 0; k < 8; ++k) tb[o] += (uint64_t)(z[k] >> p);
                    }
            }
        }
    } else
    for (int k = wid; k < P; k += nw) {
        int pk[16];
#pragma unroll
        for (int o = 0; o < 16; ++o) pk[o] = (o >= rmin && o <= omax) ? hp[(1 << o) + (k >> (omax - o))] : 0;
        const int lo = k * ps, hi = (k + 1) * ps;
        for (int i = lo + lane; i < hi; i += 64) {
            const UX xv = zz[i];
#pragma unroll
            for (int o = 0; o < 16; ++o)
                if (o >= rmin && o <= omax) tb[o] += (uint64_t)(xv >> pk[o]);
        }
    }
#pragma unroll
    for (int o = 0; o < 16; ++o) {
        if (o >= rmin && o <= omax) {
            const uint64_t v = wave_sum_u64(tb[o]);
            if (lane == 0) atomicAdd(&rb[16 + o], (unsigned long long)v);
        }
    }
    __syncthreads();
    if (tid == 0) {
        int best = rmin;
        unsigned long long bb = rb[rmin] + rb[16 + rmin];
        for (int o = rmin + 1; o <= omax; ++o) {
            const unsigned long long v = rb[o] + rb[16 + o];
            if (v < bb) {
                bb = v;
                best = o;
            }
        }
        int method = 4;
        for (int K = 0; K < (1 << best); ++K)
            if (hp[(1 << best) + K] > 14) method = 5;
        put_meta(meta, ST_OK, 0, dec, 1);
        meta->res_offset = start;
        meta->res_len = n - start;
        meta->part_order = best;
        meta->n_parts = 1 << best;
        meta->coding_method = method;
        meta->rice_bits = (long long)bb;
        misc[3] = best;
    }
    __syncthreads();
    const int best = misc[3];
    int32_t* __restrict__ rp = a.rice_params + gid * a.params_stride;
    for (int K = tid; K < (1 << best); K += NT) rp[K] = hp[(1 << best) + K];
    } /* !M8V */
    } /* !FAST */
    }
unit_done:
    if constexpr (M8V) {
        if (a.persist) {
            li += gridDim.x;
            if (li < a.count) {
                /* every wave is done with this unit's LDS (raw: the copies stay in flight) */
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                goto next_unit;
            }
        }
    }
    if constexpr (VAR == kVarList || VAR == kVarList1) {
        li += gridDim.x;
        if (li < (int64_t)*a.retry_count) {
            __syncthreads(); /* every wave is done with this unit's LDS */
            goto next_unit;
        }
    }
}

template <int LMAX, int PATH, typename ResT>
static hipError_t launch_resid_T(const ResidArgs& a, hipStream_t s) {
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int nt = resid_threads(a.n, PATH >= PATH_W64);
    const bool regz = resid_regz(a.n, rmax_eff, PATH != PATH_W64 && PATH != PATH_W64S && sizeof(ResT) == 4);
    const size_t lds = resid_lds_layout(LMAX, a.n, nt / 64, 1 << (rmax_eff < 0 ? 0 : rmax_eff),
                                        PATH == PATH_S16 ? 2 : 4, (int)sizeof(ResT), CoefTables<LMAX>::BYTES,
                                        regz, PATH == PATH_W64 && LMAX >= 16).total;
    auto kern = k_resid<LMAX, PATH, ResT, kVarGeneric>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)a.count), dim3(nt), lds, s, a);
    return hipGetLastError();
}

constexpr int kListGrid = 2048; /* workgroups of a list launch (each loops over the list; 8192 and
                                  * 16384 measured no faster on config 2, round 5) */

/* compute units of the current device (the 64-bit list variant's grid: its 140 KB of LDS
 * allows one workgroup per CU, so more workgroups than CUs would only queue) */
static inline int device_cus() {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
        ncu = 256;
    return ncu;
}
/* FLACMI_MF8_GRID=k (test knob, flacmi_set_knob): at most k workgroups in kVarMf8's persistent
 * grid and in the 64-bit list variant's, so each loops over many units (kVarMf8's next-unit
 * prefetch path, kVarList1's unit loop) */
static inline int mf8_grid_cap() { return knob(kKnobMf8Grid); }

/* S16 MFMA fast kernel over the batch, then the generic body over the units it listed */
template <int LMAX>
static hipError_t launch_resid_fast(const ResidArgs& a, hipStream_t s) {
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int nt = resid_threads(a.n);
    const int P = 1 << (rmax_eff < 0 ? 0 : rmax_eff);
    const size_t lds_fast = resid_lds_layout(LMAX, a.n, nt / 64, P, 2, 4, CoefTables<LMAX>::BYTES, true, false).total;
    const size_t lds_gen = resid_lds_layout(LMAX, a.n, nt / 64, P, 2, 4, CoefTables<LMAX>::BYTES,
                                            resid_regz(a.n, rmax_eff, true), false).total;
    hipError_t e = hipMemsetAsync(a.retry_count, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    auto kf = k_resid<LMAX, PATH_S16, uint32_t, kVarFast>;
    e = hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_fast);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kf, dim3((unsigned)a.count), dim3(nt), lds_fast, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_poison_lds(s)) != hipSuccess) return e;
    /* the listed units: a small grid loops over the list */
    auto kl = k_resid<LMAX, PATH_S16, uint32_t, kVarList>;
    e = hipFuncSetAttribute((const void*)kl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_gen);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kl, dim3((unsigned)(a.count < kListGrid ? a.count : kListGrid)), dim3(nt), lds_gen, s, a);
    return hipGetLastError();
}

/* the generic S16 body over the units k_resid_stream listed (k_stream.hip) */
template <int LMAX>
static hipError_t launch_resid_list(const ResidArgs& a, hipStream_t s) {
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int nt = resid_threads(a.n);
    const int P = 1 << (rmax_eff < 0 ? 0 : rmax_eff);
    /* the list variant carves its LDS with resid_regz (k_stream takes n up to 8*kSCPT*256,
     * beyond the register-resident bound 8*kCPT*256): size it the same way */
    const bool regz = resid_regz(a.n, rmax_eff, true);
    const size_t lds = resid_lds_layout(LMAX, a.n, nt / 64, P, 2, 4, CoefTables<LMAX>::BYTES, regz, false).total;
    auto kl = k_resid<LMAX, PATH_S16, uint32_t, kVarList>;
    hipError_t e = hipFuncSetAttribute((const void*)kl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kl, dim3((unsigned)(a.count < kListGrid ? a.count : kListGrid)), dim3(nt), lds, s, a);
    return hipGetLastError();
}

/* the fast kernel's preconditions: reference mode, 32-bit narrow residual kept in
 * registers (resid_regz), MFMA enabled, a retry list to hand exceptions to */
static inline bool resid_fast_ok(const ResidArgs& a) {
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    /* the record is staged in the chunk-sum region during phase A */
    return a.mode == FLACMI_MODE_REFERENCE && a.mfma && a.retry_list && a.retry_count &&
           resid_regz(a.n, rmax_eff, true) && (a.n + 7) / 8 + 1 >= a.rec_words;
}

/* FLACMI_MF8_PERSIST=0: config-3 shapes through the generic k_resid launch instead */
static inline bool mf8_persist_enabled() {
    static const bool on = [] {
        const char* e = getenv("FLACMI_MF8_PERSIST");
        return !(e && e[0] == '0');
    }();
    return on;
}

/* kVarMf8 as a persistent grid (one workgroup per CU), then the list variant over the units
 * it listed */
template <int LMAX>
static hipError_t launch_resid_mf8(const ResidArgs& a_in, hipStream_t s) {
    ResidArgs a = a_in;
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int P = 1 << (rmax_eff < 0 ? 0 : rmax_eff);
    const int nt8 = resid_threads(a.n, true), ntl = nt8; /* 512 */
    const int ncu = device_cus(), cap = mf8_grid_cap();
    a.persist = 1;
    int64_t grid = a.count < ncu ? a.count : ncu;
    if (cap > 0 && grid > cap) grid = cap;
    const size_t lds8 = resid_lds_layout(LMAX, a.n, nt8 / 64, P, 4, 4, CoefTables<LMAX>::BYTES, false, true).total;
    const size_t ldsl = resid_lds_layout(LMAX, a.n, ntl / 64, P, 4, 4, CoefTables<LMAX>::BYTES, false, true).total;
    hipError_t e = hipMemsetAsync(a.retry_count, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    auto k8 = k_resid<LMAX, PATH_W64, uint32_t, kVarMf8>;
    if ((e = hipFuncSetAttribute((const void*)k8, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds8)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k8, dim3((unsigned)grid), dim3(nt8), lds8, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_poison_lds(s)) != hipSuccess) return e;
    auto kl = k_resid<LMAX, PATH_W64, uint32_t, kVarList1>;
    if ((e = hipFuncSetAttribute((const void*)kl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsl)) != hipSuccess)
        return e;
    int64_t lgrid = a.count < ncu ? a.count : ncu;
    if (cap > 0 && lgrid > cap) lgrid = cap;
    hipLaunchKernelGGL(kl, dim3((unsigned)lgrid), dim3(ntl), ldsl, s, a);
    return hipGetLastError();
}

/* k_sb.hip: k_resid_sb<lmax> over the batch (lmax 16 or 32) */
hipError_t launch_resid_sb_kernel(const ResidArgs& a, int lmax, hipStream_t s);

/* FLACMI_SB=0: config-3 shapes through kVarMf8 alone (k_resid_sb off) */
static inline bool sb_enabled() {
    static const bool on = [] {
        const char* e = getenv("FLACMI_SB");
        return !(e && e[0] == '0');
    }();
    return on;
}
/* the finest Rice order of a k_resid_sb launch (the shapes launch_resid_sb admits: 6..8, a
 * power-of-two number of whole chunks per partition, >= 8 samples per partition) */
__host__ __device__ inline int sb_finest_order(int n, int rmin, int rmax) {
    int om = -1;
    for (int o = rmin; o <= rmax; ++o)
        if (n % (1 << o) == 0) om = o;
    return om;
}

/* k_resid_sb's shapes: 8192 <= n <= 16384 (n % 256 == 0: at most four chunks per thread),
 * finest Rice order 6..8 with a power-of-two number of whole chunks per partition.  Samples of
 * at most 24 bits: the kernel lists a unit only when |x| > 2^23, and its 32-bit K_j row sums
 * assume every term in [-2^23, 2^23 - 1] (x = +2^23 needs 25 bits).  k_resid_sb writes no
 * fixed_sums rows, so a caller asking for them takes kVarMf8, which does. */
static inline bool sb_shape_ok(const ResidArgs& a) {
    if (a.n < 8192 || a.n > 16384 || a.n % 256 != 0) return false;
    if (a.sample_bits > 24 || a.fixed_sums) return false;
    const int om = sb_finest_order(a.n, a.rmin, a.rmax);
    if (om < 6 || om > 8) return false;
    const int ps = a.n >> om, cpp = ps >> 3;
    return ps % 8 == 0 && cpp <= 64 && (cpp & (cpp - 1)) == 0;
}

/* k_resid_sb over the batch (k_sb.hip), then the list variant over the units it could not
 * decide */
template <int LMAX>
static hipError_t launch_resid_sb(const ResidArgs& a_in, hipStream_t s) {
    const ResidArgs& a = a_in;
    const int om = sb_finest_order(a.n, a.rmin, a.rmax);
    const size_t ldsl = resid_lds_layout(LMAX, a.n, 512 / 64, 1 << om, 4, 4, CoefTables<LMAX>::BYTES, false, true).total;
    hipError_t e = hipMemsetAsync(a.retry_count, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if ((e = launch_resid_sb_kernel(a, LMAX, s)) != hipSuccess) return e;
    if ((e = launch_poison_lds(s)) != hipSuccess) return e;
    auto kl = k_resid<LMAX, PATH_W64, uint32_t, kVarList1>;
    if ((e = hipFuncSetAttribute((const void*)kl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsl)) != hipSuccess)
        return e;
    const int ncu = device_cus(), cap = mf8_grid_cap();
    int64_t lgrid = a.count < ncu ? a.count : ncu;
    if (cap > 0 && lgrid > cap) lgrid = cap;
    hipLaunchKernelGGL(kl, dim3((unsigned)lgrid), dim3(512), ldsl, s, a);
    return hipGetLastError();
}

template <int LMAX>
static hipError_t launch_resid_bucket(const ResidArgs& a, int path, int rb, hipStream_t s) {
    if (rb == 8) return launch_resid_T<LMAX, PATH_W64, uint64_t>(a, s);
    if constexpr (LMAX >= 16) {
        const bool mf8 = path == PATH_W64 && a.mode == FLACMI_MODE_REFERENCE && a.mfma && a.retry_list &&
                         a.retry_count && a.sample_bytes == 4 && a.L >= 1 && a.n % 256 == 0 && a.n >= 8192;
        if (mf8 && a.prune && a.sign_bound && sb_enabled() && sb_shape_ok(a)) return launch_resid_sb<LMAX>(a, s);
        if (mf8 && mf8_persist_enabled()) return launch_resid_mf8<LMAX>(a, s);
    }
    if constexpr (LMAX == 8 || LMAX == 12)
        if (path == PATH_S16 && resid_fast_ok(a)) return launch_resid_fast<LMAX>(a, s);
    if (path == PATH_S16) return launch_resid_T<LMAX, PATH_S16, uint32_t>(a, s);
    if (path == PATH_N32) return launch_resid_T<LMAX, PATH_N32, uint32_t>(a, s);
    if constexpr (LMAX > 0)
        if (path == PATH_W64S) return launch_resid_T<LMAX, PATH_W64S, uint32_t>(a, s);
    return launch_resid_T<LMAX, PATH_W64, uint32_t>(a, s);
}

}  // namespace flacmi
