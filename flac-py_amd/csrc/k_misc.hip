/* k_misc.hip — small kernels (record expansion, synthetic PCM, stream statistics) and
 * the residual-kernel dispatch. */
#include "device_common.h"

namespace flacmi {

hipError_t launch_resid_l0(const ResidArgs&, int, int, hipStream_t);
hipError_t launch_resid_l8(const ResidArgs&, int, int, hipStream_t);
hipError_t launch_resid_l12(const ResidArgs&, int, int, hipStream_t);
hipError_t launch_resid_l16(const ResidArgs&, int, int, hipStream_t);
hipError_t launch_resid_l32(const ResidArgs&, int, int, hipStream_t);
bool stream_shape_ok(const ResidArgs& a, int path, int residual_bytes);
hipError_t launch_poison_lds(hipStream_t s);
hipError_t launch_resid_stream(const ResidArgs& a, hipStream_t s);

/* ====================================================================================
 * small kernels: record expansion (debug), synthetic PCM, stream statistics
 * ==================================================================================== */
__global__ void k_expand_records(const int32_t* rec, int32_t rec_words, int32_t L, int64_t count,
                                 int32_t* out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= count) return;
    const int32_t* r = rec + gid * rec_words;
    int32_t* o = out + gid * FLACMI_LPC_REC_WORDS(32);
    for (int i = 0; i < FLACMI_LPC_REC_WORDS(32); ++i) o[i] = 0;
    o[0] = r[0];
    o[1] = r[1];
    if ((r[0] & 0xffff) != 0) return;
    for (int pp = 1; pp <= L; ++pp) {
        o[2 + pp - 1] = r[2 + pp - 1];
        for (int j = 0; j < pp; ++j) o[2 + 32 + (pp * (pp - 1)) / 2 + j] = r[2 + L + (pp * (pp - 1)) / 2 + j];
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ int32_t synth_bsum(uint64_t r) { return (int32_t)__builtin_amdgcn_sad_u8((uint32_t)r, 0u, 0u); }

/* a 16-bit value to `bits` bits (low random bits from the sample's hash when widening), clipped */
__device__ __forceinline__ int64_t synth_widen(int64_t v, uint64_t r, int32_t bits) {
    const int64_t lo = -(1LL << (bits - 1)), hi = (1LL << (bits - 1)) - 1;
    if (bits > 16) {
        const int e = bits - 16;
        v = v * (1LL << e) + (int64_t)((r >> 32) & ((1ull << e) - 1)) - (1LL << (e - 1));
    } else if (bits < 16) {
        v >>= (16 - bits);
    }
    return v < lo ? lo : (v > hi ? hi : v);
}

/* SURVEY §8d synthetic signal; identical integer recipe to oracle_synth_unit.  open8 > 0: a
 * unit whose hash byte (h0 >> 56) & 7 is below open8 is the "open" mix's MA(1) near-white
 * noise instead (oracle_synth_unit_mix): LPC candidates the sign bound cannot decide. */
template <typename T>
__global__ __launch_bounds__(256) void k_synth(T* dst, int32_t bits, int64_t stride, int64_t first_unit,
                                               int32_t len, uint64_t seed, const int32_t* __restrict__ sintab,
                                               int32_t open8) {
    const int64_t uu = blockIdx.x;
    const int64_t unit = first_unit + uu;
    const uint64_t h0 = splitmix64(seed ^ ((uint64_t)unit * 0xD1B54A32D192ED03ull));
    if ((int32_t)((h0 >> 56) & 7) < open8) {
        /* |w| <= 510 * 4095 / 128 < 2^14: the products are exact 24-bit multiplies */
        const int32_t sg = 1024 + (int32_t)(splitmix64(h0 + 5) % 3072);
        const int32_t ma = (int32_t)(splitmix64(h0 + 6) % 7) - 3;
        const uint64_t base = seed ^ ((uint64_t)unit << 32);
        for (int i = threadIdx.x; i < len; i += 256) {
            const uint64_t r = splitmix64(base ^ (uint64_t)i);
            const uint64_t rp = splitmix64(base ^ (uint64_t)(int64_t)(i - 1));
            const int32_t w = __mul24(synth_bsum(r) - 510, sg) >> 7;
            const int32_t wp = __mul24(synth_bsum(rp) - 510, sg) >> 7;
            dst[uu * stride + i] = (T)synth_widen((int64_t)(w + ((ma * wp) >> 7)), r, bits);
        }
        return;
    }
    int64_t amp[3];
    uint32_t dphi[3], phi0[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t hk = splitmix64(h0 + (uint64_t)(k + 1));
        amp[k] = 1638 + (int64_t)(hk % 8192);
        const uint64_t f = 20 + ((hk >> 16) % 7981);
        dphi[k] = (uint32_t)((f << 32) / 44100);
        phi0[k] = (uint32_t)(hk >> 32);
    }
    const int64_t sigma = 66 + (int64_t)(splitmix64(h0 + 4) % 590);
    const int64_t lo = -(1LL << (bits - 1)), hi = (1LL << (bits - 1)) - 1;
    /* the 4096-entry sine table in LDS; phases advance by 256 * dphi per iteration.
     * amp < 2^14 and |sintab| <= 2^15, so each product is an exact 24-bit multiply and
     * the sum of three fits 32 bits: the same values as the int64 recipe. */
    __shared__ int32_t tab[4096];
    for (int t = threadIdx.x; t < 4096; t += 256) tab[t] = sintab[t];
    __syncthreads();
    uint32_t ph[3], st[3];
    int32_t a32[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        ph[k] = phi0[k] + (uint32_t)threadIdx.x * dphi[k];
        st[k] = 256u * dphi[k];
        a32[k] = (int32_t)amp[k];
    }
    if (bits <= 24) {
        /* every intermediate fits 32 bits here: |s| < 3 * 2^14, the noise term < 2^12, and
         * (s + noise) * 2^(bits - 16) < 2^25; the byte sum is one v_sad_u8 */
        const int32_t lo32 = (int32_t)lo, hi32 = (int32_t)hi, sg = (int32_t)sigma;
        const int e = bits > 16 ? bits - 16 : 0;
        const uint32_t emask = (1u << e) - 1u;
        const int32_t ehalf = e > 0 ? (1 << (e - 1)) : 0;
        for (int i = threadIdx.x; i < len; i += 256) {
            int32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                acc += __mul24(a32[k], tab[ph[k] >> 20]);
                ph[k] += st[k];
            }
            const uint64_t r = splitmix64(seed ^ ((uint64_t)unit << 32) ^ (uint64_t)i);
            const int32_t bsum = (int32_t)__builtin_amdgcn_sad_u8((uint32_t)r, 0u, 0u);
            int32_t v = (acc >> 15) + (__mul24(bsum - 510, sg) >> 7);
            if (bits > 16) v = v * (1 << e) + (int32_t)((uint32_t)(r >> 32) & emask) - ehalf;
            else if (bits < 16) v >>= (16 - bits);
            dst[uu * stride + i] = (T)(v < lo32 ? lo32 : (v > hi32 ? hi32 : v));
        }
        return;
    }
    for (int i = threadIdx.x; i < len; i += 256) {
        int32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            acc += __mul24(a32[k], tab[ph[k] >> 20]);
            ph[k] += st[k];
        }
        const int64_t s = (int64_t)(acc >> 15);
        const uint64_t r = splitmix64(seed ^ ((uint64_t)unit << 32) ^ (uint64_t)i);
        const int64_t bsum = (int64_t)((r & 0xff) + ((r >> 8) & 0xff) + ((r >> 16) & 0xff) + ((r >> 24) & 0xff));
        int64_t v = s + (int64_t)((__mul24((int32_t)(bsum - 510), (int32_t)sigma)) >> 7);
        if (bits > 16) {
            const int e = bits - 16;
            v = v * (1LL << e) + (int64_t)((r >> 32) & ((1ull << e) - 1)) - (1LL << (e - 1));
        } else if (bits < 16) {
            v >>= (16 - bits);
        }
        dst[uu * stride + i] = (T)(v < lo ? lo : (v > hi ? hi : v));
    }
}

__global__ __launch_bounds__(256) void k_stats(const flacmi_unit_meta* __restrict__ meta, int64_t n_units,
                                               int32_t block_len, int32_t tail_len, int64_t n_tail_units,
                                               unsigned long long* stats) {
    /* the scalar totals accumulate in registers over the grid-stride loop and are reduced once
     * per wave; only the histograms use LDS atomics; one global atomic per nonzero word per
     * workgroup (the grid is a few workgroups per CU: 2048 workgroups adding into the same 128
     * words serialised at L2) */
    __shared__ unsigned long long h[FLACMI_STATS_WORDS];
    for (int i = threadIdx.x; i < FLACMI_STATS_WORDS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    unsigned long long cnt = 0, samples = 0, rice = 0, nfix = 0, nlpc = 0, npruned = 0, hash = 0;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_units; u += (int64_t)gridDim.x * blockDim.x) {
        const flacmi_unit_meta& m = meta[u];
        const int n = u >= n_units - n_tail_units ? tail_len : block_len;
        ++cnt;
        samples += (unsigned long long)n;
        const int st = m.status & 15;
        atomicAdd(&h[64 + (m.status >= 16 ? 15 : st)], 1ull);
        if (m.status != 0) continue;
        rice += (unsigned long long)m.rice_bits;
        if (m.kind == FLACMI_KIND_FIXED) {
            ++nfix;
            atomicAdd(&h[5 + (m.order & 7) % 5], 1ull);
        } else {
            ++nlpc;
            atomicAdd(&h[9 + (m.order >= 1 && m.order <= 32 ? m.order : 32)], 1ull);
        }
        atomicAdd(&h[48 + (m.part_order & 15)], 1ull);
        if (m.lpc_order == FLACMI_LPC_PRUNED) ++npruned;
        /* reference-visible results only (lpc_sum may be FLACMI_LPC_PRUNED) */
        hash += (unsigned long long)m.rice_bits * 0x9E3779B97F4A7C15ull ^ ((unsigned long long)m.fixed_sum << 1) ^
                (unsigned long long)(m.kind * 64 + m.order) * 0xD1B54A32D192ED03ull;
    }
    const unsigned long long v[7] = {cnt, samples, rice, nfix, nlpc, npruned, hash};
    const int slot[7] = {0, 1, 2, 3, 4, 81, 80};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        unsigned long long x = v[k];
        for (int o = 32; o >= 1; o >>= 1) x += (unsigned long long)__shfl_xor(x, o);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&h[slot[k]], x);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < FLACMI_STATS_WORDS; i += blockDim.x)
        if (h[i]) atomicAdd(&stats[i], h[i]);
}

/* ---- pipeline hand-off: a sub-batch's frame offsets and status into page-locked, mapped
 * host memory (flacmi_encode_pipeline), written by the kernel over PCIe so the tiny copy
 * never queues on a DMA engine behind the frame bytes ---- */
__global__ __launch_bounds__(256) void k_export(const int64_t* __restrict__ off, const int32_t* __restrict__ st,
                                                int64_t nf, int64_t* h_off, int32_t* h_st) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= nf; i += (int64_t)gridDim.x * blockDim.x) {
        h_off[i] = off[i];
        if (i < nf) h_st[i] = st[i];
    }
}

hipError_t launch_export(const int64_t* off, const int32_t* st, int64_t nf, int64_t* h_off, int32_t* h_st,
                         hipStream_t s) {
    const int64_t blocks = (nf + 256) / 256;
    hipLaunchKernelGGL(k_export, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, s, off, st, nf, h_off,
                       h_st);
    return hipGetLastError();
}

/* ---- LDS poisoning (test knob FLACMI_POISON_LDS=<hex pattern>, read once per process) ----
 * Before every analysis kernel launch, one 160 KB workgroup per CU slot fills the LDS with a
 * pattern derived from <pattern>, so a kernel that reads LDS words it never wrote sees
 * garbage (and its results change with the pattern) instead of a previous unit's words.
 * Off unless the variable is set. */
__global__ __launch_bounds__(1024) void k_poison_lds(uint32_t pattern, int32_t words) {
    extern __shared__ uint32_t lds_words[];
    for (int i = threadIdx.x; i < words; i += blockDim.x)
        lds_words[i] = pattern ^ ((uint32_t)i * 0x9E3779B1u) ^ (blockIdx.x << 20);
    __syncthreads();
    /* keep the stores: one lane publishes a word nobody reads if the pattern says so */
    if (pattern == 0x5a5a5a5au && threadIdx.x == 0 && blockIdx.x == 0xffffff) lds_words[0] = lds_words[words - 1];
}

static uint32_t poison_pattern(bool* on) {
    static const uint64_t v = [] {
        const char* e = getenv("FLACMI_POISON_LDS");
        return e ? (1ull << 32) | (uint64_t)(uint32_t)strtoul(e, nullptr, 16) : 0ull;
    }();
    *on = (v >> 32) != 0;
    return (uint32_t)v;
}

hipError_t launch_poison_lds(hipStream_t s) {
    bool on = false;
    const uint32_t pat = poison_pattern(&on);
    if (!on) return hipSuccess;
    static uint32_t calls = 0;
    const int bytes = 160 * 1024;
    hipError_t e = hipFuncSetAttribute((const void*)k_poison_lds, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_poison_lds, dim3(1024), dim3(1024), bytes, s, pat ^ (++calls * 0x01000193u), bytes / 4);
    return hipGetLastError();
}

static int lmax_bucket(int L) { return L <= 0 ? 0 : L <= 8 ? 8 : L <= 12 ? 12 : L <= 16 ? 16 : 32; }

ResidLaunch resid_launch_config(int n, int rmax_eff, int residual_bytes) {
    ResidLaunch r;
    r.threads = resid_threads(n, true); /* worst case: the 64-bit paths' workgroup */
    r.lds_bytes = resid_lds_layout(32, n, r.threads / 64, 1 << (rmax_eff < 0 ? 0 : rmax_eff), 4,
                                   residual_bytes == 8 ? 8 : 4, 16 * 1024, false, true).total;
    return r;
}

hipError_t launch_resid(const ResidArgs& a, int path, int residual_bytes, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    if (hipError_t e = launch_poison_lds(s); e != hipSuccess) return e;
    if (stream_shape_ok(a, path, residual_bytes)) return launch_resid_stream(a, s);
    const int lb = (a.mode == FLACMI_MODE_FIXED_ONLY || a.mode == FLACMI_MODE_RICE_ONLY) ? 0 : lmax_bucket(a.L);
    switch (lb) {
        case 0: return launch_resid_l0(a, path, residual_bytes, s);
        case 8: return launch_resid_l8(a, path, residual_bytes, s);
        case 12: return launch_resid_l12(a, path, residual_bytes, s);
        case 16: return launch_resid_l16(a, path, residual_bytes, s);
        default: return launch_resid_l32(a, path, residual_bytes, s);
    }
}

hipError_t launch_expand_records(const int32_t* rec, int32_t rec_words, int32_t L, int64_t count,
                                 int32_t* out, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_expand_records, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, rec,
                       rec_words, L, count, out);
    return hipGetLastError();
}

hipError_t launch_synth(void* dst, int32_t sample_bytes, int32_t bits, int64_t stride, int64_t first_unit,
                        int64_t n_units, int32_t len, uint64_t seed, const int32_t* sintab, int32_t open8,
                        hipStream_t s) {
    if (n_units <= 0) return hipSuccess;
    /* one workgroup per unit: the per-unit recipe (64-bit splitmix, divisions) is scalar
     * work each wave repeats, so every thread loops over len / 256 samples */
    const dim3 grid((unsigned)n_units);
    if (sample_bytes == 2)
        hipLaunchKernelGGL(k_synth<int16_t>, grid, dim3(256), 0, s, (int16_t*)dst, bits, stride, first_unit, len, seed, sintab,
                           open8);
    else
        hipLaunchKernelGGL(k_synth<int32_t>, grid, dim3(256), 0, s, (int32_t*)dst, bits, stride, first_unit, len, seed, sintab,
                           open8);
    return hipGetLastError();
}

hipError_t launch_stats(const flacmi_unit_meta* meta, int64_t n_units, int32_t block_len, int32_t tail_len,
                        int64_t n_tail_units, int64_t* stats, hipStream_t s) {
    if (n_units <= 0) return hipSuccess;
    int64_t blocks = (n_units + 255) / 256;
    if (blocks > 512) blocks = 512; /* two workgroups per CU: fewer global atomics per word */
    hipLaunchKernelGGL(k_stats, dim3((unsigned)blocks), dim3(256), 0, s, meta, n_units, block_len, tail_len,
                       n_tail_units, (unsigned long long*)stats);
    return hipGetLastError();
}

__global__ void k_selftest(int32_t which, const double* __restrict__ x, double* __restrict__ out,
                           int32_t* __restrict__ status, int64_t n, const double* __restrict__ log2thr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (which == 0) {
        const pym::PowTables PT{c_log_hdr, c_log_tab, c_exp_hdr, c_exp_tab};
        int st = 0;
        out[i] = pym::py_pow2(x[i], PT, &st);
        status[i] = st;
    } else {
        out[i] = (double)pym::py_floor_log2(x[i], log2thr);
        status[i] = 0;
    }
}

hipError_t launch_selftest(int32_t which, const double* x, double* out, int32_t* status, int64_t n,
                           const double* log2thr, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, which, x, out, status, n,
                       log2thr);
    return hipGetLastError();
}

}  // namespace flacmi
