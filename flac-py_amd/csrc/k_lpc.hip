/* k_lpc.hip — autocorrelation + Levinson-Durbin + quantisation, one lane per unit
 * (see device_common.h for the design notes). */
#include "device_common.h"

namespace flacmi {

/* ====================================================================================
 * k_lpc: autocorrelation + Levinson-Durbin + quantisation, one lane per unit
 * ==================================================================================== */

template <int LMAX>
__device__ __forceinline__ void write_quant(int32_t* rec, int L, int p, const int32_t* q, int nq,
                                            int shift) {
    rec[2 + p - 1] = shift;
    int32_t* c = rec + 2 + L + (p * (p - 1)) / 2;
#pragma unroll
    for (int j = 0; j < LMAX; ++j)
        if (j < p) c[j] = j < nq ? q[j] : 0;
}

/* ACF_IN: the autocorrelation is read from a.acf ([count][33]) instead of computed from
 * samples -- the entry point flacmi_device_lpc_from_acf uses to drive Levinson-Durbin and
 * the quantiser into the overflow sites integer PCM never reaches. */
template <int LMAX, typename SampleT, bool ACF_IN = false>
__global__ __launch_bounds__(256) void k_lpc(LpcArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.count) return;
    const int64_t u = a.unit0 + gid;
    const SampleT* __restrict__ x = (const SampleT*)a.samples + u * a.stride;
    int32_t* __restrict__ rec = a.rec + gid * a.rec_words;
    const int n = a.n, L = a.L, q = a.q;

    constexpr int S = ((LMAX + 1 + 7) / 8) * 8;
    double acc[LMAX + 1];
    if constexpr (ACF_IN) {
#pragma unroll
        for (int l = 0; l <= LMAX; ++l) acc[l] = l <= L ? a.acf[gid * 33 + l] : 0.0;
    } else {
    if (n >= 4 && n <= 7) { /* tukey: nr == 0 -> pi * 0 / 0 (encoder.py:437) */
        rec[0] = ST_ZERODIV | (FLACMI_SITE_TUKEY << 16);
        rec[1] = 0;
        if (a.acf)
            for (int l = 0; l < 33; ++l) a.acf[gid * 33 + l] = 0.0;
        return;
    }

    /* ---- autocorrelation: acc[l] = sum_{m} a[m-l] * a[m], m = 0 .. n-2 ---- */
    double ring[S];
#pragma unroll
    for (int t = 0; t < S; ++t) ring[t] = 0.0;
#pragma unroll
    for (int l = 0; l <= LMAX; ++l) acc[l] = 0.0;
    const int M = n - 1; /* the last sample never enters a product (encoder.py:449) */
    const double* __restrict__ win = a.window;
    /* Samples arrive in load blocks of SB per lane (64 B: a whole half cache line per row
     * per visit), kept packed (int16 pairs) and prefetched one block ahead; each block is
     * processed as SB / S ring-aligned sub-blocks of S samples. */
    constexpr int PK = sizeof(SampleT) == 2 ? 2 : 1; /* samples per 32-bit word */
    constexpr int SB = sizeof(SampleT) == 2 ? 2 * S : S;
    constexpr int W = SB / PK;
    const int nblk = (M + SB - 1) / SB;
    uint32_t cur[W];
    auto load = [&](int m0, uint32_t (&v)[W]) __attribute__((always_inline)) {
        if (m0 + SB <= M) {
#pragma unroll
            for (int g = 0; g < W / 4; ++g) {
                const uint4 q = *reinterpret_cast<const uint4*>(x + m0 + 4 * PK * g);
                v[4 * g] = q.x;
                v[4 * g + 1] = q.y;
                v[4 * g + 2] = q.z;
                v[4 * g + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if constexpr (PK == 2) {
                    const uint32_t lo = (m0 + 2 * w < M) ? (uint16_t)x[m0 + 2 * w] : 0u;
                    const uint32_t hi = (m0 + 2 * w + 1 < M) ? (uint16_t)x[m0 + 2 * w + 1] : 0u;
                    v[w] = lo | (hi << 16);
                } else {
                    v[w] = (m0 + w < M) ? (uint32_t)x[m0 + w] : 0u;
                }
            }
        }
    };
    auto sample = [&](const uint32_t (&v)[W], int t) __attribute__((always_inline)) -> int32_t {
        if constexpr (PK == 2) return (t & 1) ? (int32_t)v[t >> 1] >> 16 : (int32_t)(v[t >> 1] << 16) >> 16;
        return (int32_t)v[t];
    };
    if constexpr (PK == 1) {
        /* 32-bit samples (L up to 32, S = 40): loading whole S-sample blocks would hold 2 x 40
         * sample registers beside the 33 accumulators and the 40-slot ring (one wave per SIMD,
         * accumulators spilled to AGPRs).  Instead groups of G samples are prefetched one group
         * ahead while the ring cycles through its S slots (static indices throughout). */
        constexpr int G = 8;
        static_assert(S % G == 0, "ring length a multiple of the load group");
        const int ncyc = (M + S - 1) / S;
        uint32_t gc[G], gn[G];
        auto loadg = [&](int m0, uint32_t (&v)[G]) __attribute__((always_inline)) {
            if (m0 + G <= M) {
                const uint4 q0 = *reinterpret_cast<const uint4*>(x + m0);
                const uint4 q1 = *reinterpret_cast<const uint4*>(x + m0 + 4);
                v[0] = q0.x; v[1] = q0.y; v[2] = q0.z; v[3] = q0.w;
                v[4] = q1.x; v[5] = q1.y; v[6] = q1.z; v[7] = q1.w;
            } else {
#pragma unroll
                for (int k = 0; k < G; ++k) v[k] = (m0 + k < M) ? (uint32_t)x[m0 + k] : 0u;
            }
        };
        if (ncyc > 0) loadg(0, gc);
        for (int c = 0; c < ncyc; ++c) {
            const int m0 = c * S;
            const bool rect = m0 - LMAX >= a.fuse_lo && m0 + S <= a.fuse_hi;
#pragma unroll
            for (int g = 0; g < S / G; ++g) {
                const int mg = m0 + g * G;
                loadg(mg + G, gn);
                if (rect) { /* exact integer products: one fused op per term (see below) */
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int t = g * G + k;
                        const double av = (double)(int32_t)gc[k];
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) acc[l] = __builtin_fma(ring[(t - l + S) % S], av, acc[l]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int t = g * G + k;
                        const double av = (double)(int32_t)gc[k] * win[mg + k];
                        ring[t] = av;
#pragma unroll
                        for (int l = 0; l <= LMAX; ++l) {
                            const double prev = ring[(t - l + S) % S];
                            acc[l] = acc[l] + prev * av;
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < G; ++k) gc[k] = gn[k];
            }
        }
    } else {
    if (nblk > 0) load(0, cur);
    for (int b = 0; b < nblk; ++b) {
        const int mb = b * SB;
        uint32_t nxt[W];
        if (b + 1 < nblk) load(mb + SB, nxt);
#pragma unroll
        for (int sb = 0; sb < SB / S; ++sb) {
            const int m0 = mb + sb * S;
            if (m0 - LMAX >= a.fuse_lo && m0 + S <= a.fuse_hi) {
                /* Inside the Tukey window's rectangle (weight exactly 1.0) every windowed
                 * sample and lag partner is the integer sample itself, and the product of two
                 * integers below 2^26 is exact in a double: RN(acc + RN(p * a)) ==
                 * fma(p, a, acc).  One fused op per term instead of a multiply and an add,
                 * bit-identical. */
#pragma unroll
                for (int t = 0; t < S; ++t) {
                    const double av = (double)sample(cur, sb * S + t);
                    ring[t] = av;
#pragma unroll
                    for (int l = 0; l <= LMAX; ++l) acc[l] = __builtin_fma(ring[(t - l + S) % S], av, acc[l]);
                }
            } else {
#pragma unroll
                for (int t = 0; t < S; ++t) {
                    const double av = (double)sample(cur, sb * S + t) * win[m0 + t];
                    ring[t] = av;
#pragma unroll
                    for (int l = 0; l <= LMAX; ++l) {
                        const double prev = ring[(t - l + S) % S];
                        acc[l] = acc[l] + prev * av;
                    }
                }
            }
        }
#pragma unroll
        for (int w = 0; w < W; ++w) cur[w] = nxt[w];
    }
    } /* PK == 2 */
    if (a.acf) {
        double* o = a.acf + gid * 33;
#pragma unroll
        for (int l = 0; l < 33; ++l) o[l] = (l <= LMAX && l <= L) ? acc[l < LMAX ? l : LMAX] : 0.0;
    }
    } /* !ACF_IN */

    /* ---- Levinson-Durbin at max order with a snapshot per order (encoder.py:453-479) ---- */
    const pym::PowTables PT{c_log_hdr, c_log_tab, c_exp_hdr, c_exp_tab};
    double c[LMAX + 1];
    c[0] = 1.0;
#pragma unroll
    for (int j = 1; j <= LMAX; ++j) c[j] = 0.0;
    double err = acc[0];
    int lst = ST_OK, lsite = 0, qst = ST_OK, qsite = 0;
    uint32_t negmask = 0;
    const double qmax = (double)((1LL << (q - 1)) - 1);
    const double qmin = -(double)(1LL << (q - 1));
    static_for<LMAX>([&](auto K_) {
        constexpr int k = K_;
        if (k < L && lst == ST_OK) {
            double lam = 0.0;
#pragma unroll
            for (int j = 0; j <= k; ++j) lam = lam - c[j] * acc[k + 1 - j];
            if (err == 0.0) {
                lst = ST_ZERODIV;
                lsite = FLACMI_SITE_LEVINSON_DIV;
            } else {
                lam = lam / err;
#pragma unroll
                for (int nn = 0; nn <= (k + 1) / 2; ++nn) {
                    const double tmp = c[k + 1 - nn] + lam * c[nn];
                    c[nn] = c[nn] + lam * c[k + 1 - nn];
                    c[k + 1 - nn] = tmp;
                }
                int pst;
                const double l2 = pym::py_pow2(lam, PT, &pst);
                if (pst) {
                    lst = ST_OVERFLOW;
                    lsite = FLACMI_SITE_LEVINSON_POW;
                } else {
                    err = err * (1.0 - l2);
                }
            }
            /* quantise order p = k + 1 (encoder.py:482-534) unless an earlier order failed */
            if (lst == ST_OK && qst == ST_OK) {
                const int p = k + 1;
                double cm = __builtin_fabs(c[1]);
#pragma unroll
                for (int j = 2; j <= LMAX; ++j)
                    if (j <= p && __builtin_fabs(c[j]) > cm) cm = __builtin_fabs(c[j]);
                int32_t qv[LMAX];
                int nq = 0, shift = 0;
                if (!(cm > 0.0)) {
                    qst = ST_ASSERT;
                    qsite = FLACMI_SITE_QUANT_CMAX;
                } else if (__builtin_isinf(cm)) {
                    qst = ST_OVERFLOW;
                    qsite = FLACMI_SITE_QUANT_LOG2;
                } else {
                    shift = q - pym::py_floor_log2(cm, a.log2thr) - 2;
                    if (shift > 15) shift = 15;
                    if (shift < -16) {
                        qst = ST_ASSERT;
                        qsite = FLACMI_SITE_QUANT_SHIFT;
                    } else {
                        const bool neg = shift < 0;
                        const double scale = pow2_exact(neg ? -shift : shift);
                        double e = 0.0;
#pragma unroll
                        for (int j = 1; j <= LMAX; ++j) {
                            if (j <= p && qst == ST_OK) {
                                e = e + c[j] * scale;
                                if (__builtin_isinf(e)) {
                                    qst = ST_OVERFLOW;
                                    qsite = FLACMI_SITE_QUANT_ROUND_INF;
                                } else if (__builtin_isnan(e)) {
                                    qst = ST_VALUE;
                                    qsite = FLACMI_SITE_QUANT_ROUND_NAN;
                                } else {
                                    const double r = __builtin_rint(e);
                                    const double qq = r < qmin ? qmin : (r > qmax ? qmax : r);
                                    e = e - qq;
                                    qv[j - 1] = (int32_t)qq;
                                }
                            }
                        }
                        if (qst == ST_OK) {
                            if (neg) {
                                negmask |= 1u << k;
                                shift = 0;
                                nq = 0;
                            } else {
                                nq = p;
                            }
                            write_quant<LMAX>(rec, L, p, qv, nq, shift);
                        }
                    }
                }
            }
        }
    });
    int st = lst != ST_OK ? lst : qst;
    int site = lst != ST_OK ? lsite : qsite;
    if (st == ST_OK && L == 0) { /* min() over no candidates (encoder.py:404) */
        st = ST_VALUE;
        site = FLACMI_SITE_LPC_EMPTY;
    }
    rec[0] = st | (site << 16);
    rec[1] = (int32_t)negmask;
}

template <int LMAX>
static hipError_t launch_lpc_T(const LpcArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((a.count + 255) / 256));
    if (a.sample_bytes == 2)
        hipLaunchKernelGGL((k_lpc<LMAX, int16_t>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_lpc<LMAX, int32_t>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_lpc_from_acf(const LpcArgs& a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_lpc<32, int32_t, true>), dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_lpc(const LpcArgs& a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    if (a.L <= 4) return launch_lpc_T<4>(a, s);
    if (a.L <= 8) return launch_lpc_T<8>(a, s);
    if (a.L <= 12) return launch_lpc_T<12>(a, s);
    if (a.L <= 16) return launch_lpc_T<16>(a, s);
    return launch_lpc_T<32>(a, s);
}


}  // namespace flacmi
