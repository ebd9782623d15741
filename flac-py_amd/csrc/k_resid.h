/* k_resid.h — fixed + LPC candidate residual sums, choice, chosen residual and Rice
 * search, one workgroup per unit (see device_common.h for the design notes).
 * Instantiated per LPC-order bucket in k_resid_l*.hip so the builds run in parallel. */
#pragma once
#include "device_common.h"

namespace flacmi {

template <int LMAX, bool WIDE, typename ResT>
__global__ __launch_bounds__(LMAX >= 16 ? 512 : 1024) void k_resid(ResidArgs a) {
    using Lay = ResidLayout<LMAX>;
    using X = typename std::conditional<sizeof(ResT) == 8, int64_t, int32_t>::type;
    using Acc = typename std::conditional<WIDE, int64_t, int32_t>::type;
    constexpr int HP = Lay::HP, NSUM = Lay::NSUM, CPAD = Lay::CPAD;

    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x, NT = blockDim.x, lane = tid & 63, wid = tid >> 6, nw = NT >> 6;
    const int64_t gid = blockIdx.x;
    const int64_t u = a.unit0 + gid;
    const int n = a.n, L = a.L;
    const int nch = (n + 7) >> 3;
    const int npad = nch * 8 + 8;

    /* ---- LDS carve ---- */
    X* xs = reinterpret_cast<X*>(smem) + HP;                                   /* [-HP, npad) */
    unsigned char* p = smem + sizeof(X) * (size_t)(HP + npad);
    p = (unsigned char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
    unsigned long long* red = reinterpret_cast<unsigned long long*>(p);       /* [nw][NSUM] */
    p += sizeof(unsigned long long) * nw * NSUM;
    unsigned long long* tot = reinterpret_cast<unsigned long long*>(p);       /* [NSUM] */
    p += sizeof(unsigned long long) * NSUM;
    int32_t* cf = reinterpret_cast<int32_t*>(p);                               /* [LMAX][CPAD] */
    p += sizeof(int32_t) * (LMAX > 0 ? LMAX : 1) * CPAD;
    int32_t* lsh = reinterpret_cast<int32_t*>(p);                              /* [LMAX] shift, start */
    p += sizeof(int32_t) * 2 * (LMAX > 0 ? LMAX : 1);
    p = (unsigned char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
    Decision* dec = reinterpret_cast<Decision*>(p);
    p += sizeof(Decision);
    p = (unsigned char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
    unsigned long long* rb = reinterpret_cast<unsigned long long*>(p);        /* [16] fixed bits, [16] data bits */
    p += sizeof(unsigned long long) * 32;
    int* misc = reinterpret_cast<int*>(p);                                     /* [0] err key, [1] any>14, [2] wide flag */
    p += sizeof(int) * 4;
    p = (unsigned char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
    unsigned long long* hs = reinterpret_cast<unsigned long long*>(p);        /* heap S [2P] */
    /* heap params follow hs: set after P is known */

    flacmi_unit_meta* meta = a.meta + gid;

    /* ---- phase A: stage samples, coefficients ---- */
    for (int i = tid; i < HP; i += NT) xs[i - HP] = 0;
    for (int i = n + tid; i < npad; i += NT) xs[i] = 0;
    if (a.sample_bytes == 2) {
        const int16_t* __restrict__ src = (const int16_t*)a.samples + u * a.stride;
        const int nv = n >> 3;
        for (int v = tid; v < nv; v += NT) {
            const short8 s = *reinterpret_cast<const short8*>(src + 8 * v);
#pragma unroll
            for (int k = 0; k < 8; ++k) xs[8 * v + k] = s[k];
        }
        for (int i = nv * 8 + tid; i < n; i += NT) xs[i] = src[i];
    } else {
        const int32_t* __restrict__ src = (const int32_t*)a.samples + u * a.stride;
        const int nv = n >> 2;
        for (int v = tid; v < nv; v += NT) {
            const int4v s = *reinterpret_cast<const int4v*>(src + 4 * v);
#pragma unroll
            for (int k = 0; k < 4; ++k) xs[4 * v + k] = s[k];
        }
        for (int i = nv * 4 + tid; i < n; i += NT) xs[i] = src[i];
    }
    if (a.mode == FLACMI_MODE_REFERENCE) {
        const int32_t* __restrict__ rec = a.rec + gid * a.rec_words;
        const int st = rec[0];
        if (st != 0) { /* the reference raises inside encode_subframe_lpc */
            if (tid == 0) put_meta(meta, st & 0xffff, st >> 16, nullptr, 0);
            return;
        }
        const uint32_t negmask = (uint32_t)rec[1];
        for (int i = tid; i < LMAX * CPAD; i += NT) {
            const int pp = i / CPAD + 1, j = i % CPAD;
            const bool neg = (negmask >> (pp - 1)) & 1;
            cf[i] = (pp <= L && j < pp && !neg) ? rec[2 + L + (pp * (pp - 1)) / 2 + j] : 0;
        }
        for (int i = tid; i < LMAX; i += NT) {
            const int pp = i + 1;
            const bool neg = (negmask >> i) & 1;
            lsh[i] = pp <= L ? rec[2 + i] : 0;
            lsh[LMAX + i] = neg ? 0 : pp; /* first residual index of this candidate */
        }
    }
    if (tid == 0) {
        misc[0] = 0x7fffffff;
        misc[1] = 0;
        misc[2] = 0;
    }
    if (tid < 32) rb[tid] = 0;
    __syncthreads();

    /* ---- phase B: sum|r| for fixed orders 0..4 and LPC orders 1..L ---- */
    unsigned long long sums[NSUM];
#pragma unroll
    for (int s = 0; s < NSUM; ++s) sums[s] = 0;
    const bool do_lpc = LMAX > 0 && a.mode == FLACMI_MODE_REFERENCE;
#pragma unroll 1
    for (int c = tid; c < nch; c += NT) {
        {
            const int i0 = 8 * c;
            X w[HP + 8];
#pragma unroll
            for (int j = 0; j < HP + 8; ++j) w[j] = xs[i0 - HP + j];
            const bool fast = (i0 >= HP) && (i0 + 8 <= n);
            /* fixed predictors: k-th differences (FIXED_PREDICTOR_COEFFICIENTS) */
            uint32_t fp[5] = {0, 0, 0, 0, 0};
            unsigned long long fpw[5] = {0, 0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k;
                const int64_t x0 = w[HP + k], x1 = w[HP + k - 1], x2 = w[HP + k - 2],
                              x3 = w[HP + k - 3], x4 = w[HP + k - 4];
                const int64_t r[5] = {x0, x0 - x1, x0 - 2 * x1 + x2, x0 - 3 * x1 + 3 * x2 - x3,
                                      x0 - 4 * x1 + 6 * x2 - 4 * x3 + x4};
#pragma unroll
                for (int o = 0; o < 5; ++o) {
                    const bool valid = fast || (i >= o && i < n);
                    if (WIDE) fpw[o] += valid ? uabs64(r[o]) : 0;
                    else fp[o] += valid ? uabs32((int32_t)r[o]) : 0;
                }
            }
#pragma unroll
            for (int o = 0; o < 5; ++o) sums[o] += WIDE ? fpw[o] : fp[o];
            if (do_lpc) {
                static_for<LMAX>([&](auto P_) {
                    constexpr int pp = P_ + 1;
                    if (pp <= L) {
                        Acc coef[LMAX > 0 ? LMAX : 1];
#pragma unroll
                        for (int j = 0; j < LMAX; ++j)
                            if (j < pp) coef[j] = cf[(pp - 1) * CPAD + j];
                        const int sh = lsh[pp - 1];
                        const int start = lsh[LMAX + pp - 1];
                        uint32_t part = 0;
                        unsigned long long partw = 0;
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            Acc pred = 0;
#pragma unroll
                            for (int j = 0; j < LMAX; ++j) {
                                if (j < pp) {
                                    if (WIDE) pred += (Acc)coef[j] * (Acc)w[HP + k - 1 - j];
                                    else pred += __mul24((int)coef[j], (int)w[HP + k - 1 - j]);
                                }
                            }
                            const Acc r = (Acc)w[HP + k] - (pred >> sh);
                            const int i = i0 + k;
                            const bool valid = fast ? (i >= start) : (i >= start && i < n);
                            if (WIDE) partw += valid ? uabs64(r) : 0;
                            else part += valid ? uabs32((int32_t)r) : 0;
                        }
                        sums[4 + pp] += WIDE ? partw : part;
                    }
                });
            }
        }
    }

    /* ---- phase C: workgroup reduction ---- */
#pragma unroll
    for (int s = 0; s < NSUM; ++s) {
        const unsigned long long v = wave_sum(sums[s]);
        if (lane == 0) red[wid * NSUM + s] = v;
    }
    __syncthreads();
    for (int s = tid; s < NSUM; s += NT) {
        unsigned long long v = 0;
        for (int w2 = 0; w2 < nw; ++w2) v += red[w2 * NSUM + s];
        tot[s] = v;
    }
    __syncthreads();

    /* ---- phase D: choice (encoder.py:331-359, 398-404, 135-157) ---- */
    if (tid == 0) {
        Decision& d = *dec;
        d.status = ST_OK;
        d.site = 0;
        int fo = 0;
        if (n > 4)
            for (int o = 1; o < 5; ++o)
                if (tot[o] < tot[fo]) fo = o;
        d.fixed_order = fo;
        d.fixed_sum = (long long)tot[fo];
        d.kind = FLACMI_KIND_FIXED;
        d.order = fo;
        d.shift = 0;
        d.ncoefs = 0;
        d.lpc_order = 0;
        d.lpc_sum = 0;
        for (int j = 0; j < 4; ++j) d.coef[j] = c_fixed_coef[fo][j];
        if (do_lpc) {
            int best = 1;
            for (int pp = 2; pp <= L; ++pp)
                if (tot[4 + pp] < tot[4 + best]) best = pp;
            d.lpc_order = best;
            d.lpc_sum = (long long)tot[4 + best];
            if (tot[4 + best] < tot[fo]) {
                d.kind = FLACMI_KIND_LPC;
                d.order = best;
                d.shift = lsh[best - 1];
                d.ncoefs = lsh[LMAX + best - 1] == 0 ? 0 : best;
                for (int j = 0; j < best; ++j) d.coef[j] = cf[(best - 1) * CPAD + j];
            } else if (!(tot[fo] < tot[4 + best])) {
                d.status = ST_ASSERT;
                d.site = FLACMI_SITE_CHOICE_TIE;
            }
        }
        if (a.fixed_sums) {
            for (int o = 0; o < 5; ++o) a.fixed_sums[gid * 5 + o] = (n > 4 || o == 0) ? (long long)tot[o] : 0;
        }
        if (a.lpc_sums) {
            for (int pp = 1; pp <= 32; ++pp)
                a.lpc_sums[gid * 32 + pp - 1] = (do_lpc && pp <= L) ? (long long)tot[4 + pp] : 0;
        }
    }
    __syncthreads();
    const int dstatus = dec->status;
    if (dstatus != ST_OK) {
        if (tid == 0) put_meta(meta, dstatus, dec->site, dec, 0);
        return;
    }
    /* The chosen LPC candidate always has coefficients: a coefficient-less candidate
     * (negative-shift branch) has sum|x| over all n samples, which is exactly the fixed
     * order-0 sum, so it can never be strictly smaller than the best fixed sum. */
    const int order = dec->order;
    const int dshift = dec->shift;
    const int start = order; /* residual starts at index len(warmup) */

    /* ---- phase E: chosen residual, zig-zag, to HBM and (after a barrier) to LDS ---- */
    ResT zr[kCPT][8];
    bool wide_flag = false;
    ResT* __restrict__ rout = reinterpret_cast<ResT*>(a.residual) + gid * a.residual_stride;
    static_for<kCPT>([&](auto C_) {
        constexpr int cc = C_;
        const int c = tid + cc * NT;
        if (c < nch) {
            const int i0 = 8 * c;
            X w[HP + 8];
#pragma unroll
            for (int j = 0; j < HP + 8; ++j) w[j] = xs[i0 - HP + j];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                int64_t pred = 0;
#pragma unroll
                for (int j = 0; j < (LMAX > 4 ? LMAX : 4); ++j)
                    if (j < order) pred += (int64_t)dec->coef[j] * (int64_t)w[HP + k - 1 - j];
                const int64_t r = (int64_t)w[HP + k] - (pred >> dshift);
                const int i = i0 + k;
                ResT z;
                if (sizeof(ResT) == 4) {
                    const bool fits = r >= -(1LL << 31) && r < (1LL << 31);
                    if (!fits && i >= start && i < n) wide_flag = true;
                    const int32_t r32 = (int32_t)r;
                    z = (ResT)(((uint32_t)r32 << 1) ^ (uint32_t)(r32 >> 31));
                } else {
                    z = (ResT)(((uint64_t)r << 1) ^ (uint64_t)(r >> 63));
                }
                zr[cc][k] = (i >= start && i < n) ? z : (ResT)0;
            }
            if (i0 + 8 <= n) {
                if constexpr (sizeof(ResT) == 4) {
                    int4v* o = reinterpret_cast<int4v*>(rout + i0);
                    o[0] = int4v{(int)zr[cc][0], (int)zr[cc][1], (int)zr[cc][2], (int)zr[cc][3]};
                    o[1] = int4v{(int)zr[cc][4], (int)zr[cc][5], (int)zr[cc][6], (int)zr[cc][7]};
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) rout[i0 + k] = zr[cc][k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (i0 + k < n) rout[i0 + k] = zr[cc][k];
            }
        }
    });
    if (wide_flag) misc[2] = 1;
    __syncthreads();
    static_for<kCPT>([&](auto C_) {
        constexpr int cc = C_;
        const int c = tid + cc * NT;
        if (c < nch) {
#pragma unroll
            for (int k = 0; k < 8; ++k) xs[8 * c + k] = (X)zr[cc][k];
        }
    });
    __syncthreads();
    if (misc[2]) {
        if (tid == 0) put_meta(meta, FLACMI_STATUS_RESIDUAL_WIDE, FLACMI_SITE_RESIDUAL_WIDTH, dec, 1);
        return;
    }

    /* ---- phase F: Rice partition search (encoder.py:655-760) ---- */
    int omax = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if ((n % (1 << o)) == 0 && (n >> o) > order) omax = o;
    if (omax < 0) {
        if (tid == 0) put_meta(meta, ST_ASSERT, FLACMI_SITE_RICE_NO_ORDER, dec, 1);
        return;
    }
    const int rmin = a.rmin;
    const int P = 1 << omax, ps = n >> omax;
    int32_t* hp = reinterpret_cast<int32_t*>(hs + 2 * P); /* heap params [2P] */
    /* finest partition sums: heap nodes [P, 2P) */
    for (int k = wid; k < P; k += nw) {
        const int lo = k == 0 ? start : k * ps, hi = (k + 1) * ps;
        unsigned long long s = 0;
        for (int i = lo + lane; i < hi; i += 64) s += (unsigned long long)(typename std::make_unsigned<X>::type)xs[i];
        s = wave_sum(s);
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
            const double mean = (double)S / (double)len; /* S < 2^53: exact division rounding */
            prm = pym::py_floor_log2(mean, a.log2thr);
            if (prm < 0) atomicMin(&misc[0], (o << 16) | K);
        }
        hp[j] = prm;
        const unsigned long long hb = 4ull + (prm > 14 ? 5ull : 4ull) + (unsigned long long)len * (unsigned long long)(1 + prm);
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
        return;
    }
    /* data bits: sum over the residual of (x >> p) for every candidate order at once */
    unsigned long long tb[16];
#pragma unroll
    for (int o = 0; o < 16; ++o) tb[o] = 0;
    for (int k = wid; k < P; k += nw) {
        int pk[16];
#pragma unroll
        for (int o = 0; o < 16; ++o) pk[o] = (o >= rmin && o <= omax) ? hp[(1 << o) + (k >> (omax - o))] : 0;
        const int lo = k == 0 ? start : k * ps, hi = (k + 1) * ps;
        for (int i = lo + lane; i < hi; i += 64) {
            const auto xv = (typename std::make_unsigned<X>::type)xs[i];
#pragma unroll
            for (int o = 0; o < 16; ++o)
                if (o >= rmin && o <= omax) tb[o] += (unsigned long long)(xv >> pk[o]);
        }
    }
#pragma unroll
    for (int o = 0; o < 16; ++o) {
        if (o >= rmin && o <= omax) {
            const unsigned long long v = wave_sum(tb[o]);
            if (lane == 0) atomicAdd(&rb[16 + o], v);
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
}

template <int LMAX, bool WIDE, typename ResT>
static hipError_t launch_resid_T(const ResidArgs& a, hipStream_t s) {
    int rmax_eff = -1;
    for (int o = a.rmin; o <= a.rmax; ++o)
        if (a.n % (1 << o) == 0) rmax_eff = o;
    const int nch = (a.n + 7) / 8;
    int nt = 64 * ((nch + 64 * kCPT - 1) / (64 * kCPT));
    if (nt < 64) nt = 64;
    const size_t lds = resid_lds_bytes(LMAX, a.n, nt / 64, 1 << (rmax_eff < 0 ? 0 : rmax_eff), (int)sizeof(ResT));
    auto kern = k_resid<LMAX, WIDE, ResT>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)a.count), dim3(nt), lds, s, a);
    return hipGetLastError();
}


template <int LMAX>
static hipError_t launch_resid_bucket(const ResidArgs& a, bool wide, int rb, hipStream_t s) {
    if (rb == 8) return launch_resid_T<LMAX, true, uint64_t>(a, s);
    return wide ? launch_resid_T<LMAX, true, uint32_t>(a, s) : launch_resid_T<LMAX, false, uint32_t>(a, s);
}

}  // namespace flacmi
