/* k_sb.hip — k_resid_sb, the config-3 units the sign-correlation bound decides (its own
 * translation unit: the k_resid_l*.hip instantiations take minutes to build). */
#include "k_resid.h"

namespace flacmi {

/* =======================================================================================
 * k_resid_sb — the int8 path's units that the sign-correlation bound decides (round 5).
 *
 * On config 3 the bound settles every unit before any LPC tile, so the digit
 * planes, the tile loop's register sets and the tier machinery of kVarMf8 are dead weight
 * that holds one 140 KB workgroup per CU.  This kernel keeps only what a decided unit
 * needs -- the int32 samples, the triangle of LPC coefficients, the reduction slots and the
 * Rice tables (77 KB at n = 16384, L = 32) in <= 128 VGPRs -- so two 512-thread workgroups
 * share a CU and one unit's staging overlaps another's arithmetic.  Per unit:
 *   1. stage the samples (16-byte loads, all in flight), the record's status and
 *      coefficient words, max|x|;
 *   2. the exact fixed sums (encoder.py:331-359) over every chunk, and the bound's K_j over
 *      each thread's first kSbSplit chunks, R' = [LMAX, 8 kSbSplit NT) = [LMAX, 8192) (any
 *      subset of R gives a valid bound: every dropped term |r_i| - w_i r_i is >= 0; on
 *      config-3 data R' decides about 3 units in 4);
 *   3. wave 0 tests every LPC order as mf8_candidate_sums does; undecided: the bound over
 *      the rest of R, tested again; still undecided (or |x| > 2^23): the unit is listed for
 *      kVarList1, which redoes it with the planes and the tiers;
 *   4. decided: the first fixed argmin (LPC proven to lose, encoder.py:135-157), its
 *      residual as int32 difference chains to HBM and kept in registers (4 chunks x 8 per
 *      thread), the finest partition sums by DPP steps, the Rice search (encoder.py:655-760)
 *      over those registers (no LDS copy of the residual), the meta record and the
 *      parameters.
 * ======================================================================================= */
constexpr int kSbThreads = 512;
constexpr int kSbChunks = 4; /* 8-sample chunks per thread at n <= 16384 */
constexpr int kSbSplit = 2; /* chunks per thread in the bound's first pass; the second pass takes
                             * the rest (<= 2 at n <= 16384): <= 16 terms per lane and pass */
struct SbLds {
    int xs, cf, red, ks, fs, pre, prm, rb, misc, dec, total;
};
/* per wave: the fixed sums (0..4) and N_- (5); later 16 Rice order totals */
constexpr int kSbRed = 16;
/* K_j row sums: [32 rows (8 waves x 4 DPP rows)][stride] int32, lag j at column j */
__host__ __device__ constexpr int sb_ks_stride(int lmax) { return ((lmax + 1 + 3) / 4) * 4; }
/* LPC coefficients: one padded row per order (c_{p,1..p} at row p - 1, zeros after), rows
 * 16-byte aligned and 36 words apart so wave 0's lanes read four coefficients per ds_read_b128
 * across distinct banks */
__host__ __device__ constexpr int sb_cf_stride(int lmax) { return lmax + 4; }
__host__ __device__ inline SbLds sb_lds_layout(int lmax, int n, int P) {
    auto up = [](int b) { return (b + 15) & ~15; };
    SbLds l;
    int o = 0;
    l.xs = o;   o = up(o + 4 * (resid_hp(lmax) + n));
    l.cf = o;   o = up(o + 4 * lmax * sb_cf_stride(lmax));
    l.red = o;  o = up(o + 8 * (kSbThreads / 64) * kSbRed);
    /* the K_j row sums are dead before the residual pass: they share the Rice region */
    l.ks = o;
    const int ks_end = up(o + 4 * 4 * (kSbThreads / 64) * sb_ks_stride(lmax));
    l.fs = o;   o = up(o + 16 * P); /* finest sums (u64 [P, 2P)), then the Rice rows (16 B x P) */
    l.pre = o;  o = up(o + 8 * P);
    l.prm = o;  o = up(o + 2 * P);
    o = o > ks_end ? o : ks_end;
    l.rb = o;   o = up(o + 8 * 16);
    l.misc = o; o = up(o + 4 * 16);
    l.dec = o;  o = up(o + (int)sizeof(Decision));
    l.total = o;
    return l;
}
/* R08: Rice orders 0..8 (config 3: rmin 0, finest order 8), compile-time order loops;
 * NFIX: the block length as a constant (16384: config 3), 0 = from the arguments */
template <int LMAX, bool R08, int NFIX = 0>
__global__ __launch_bounds__(kSbThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_resid_sb(ResidArgs a) {
    constexpr int HP = resid_hp(LMAX), NT = kSbThreads, nw = NT / 64, NR = kSbRed, KS = sb_ks_stride(LMAX);
    static_assert(HP >= LMAX && LMAX % 4 == 0, "the bound's window reads LMAX samples of history");
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t gid = blockIdx.x;
    const int n = NFIX ? NFIX : a.n, L = NFIX ? LMAX : a.L, nch = n >> 3; /* NFIX variants: L = LMAX */
    const int omax = R08 ? 8 : sb_finest_order(n, a.rmin, a.rmax);
    const int P = 1 << omax, cpp = (n >> omax) >> 3;
    const SbLds lay = sb_lds_layout(LMAX, n, P);
    int32_t* xs = reinterpret_cast<int32_t*>(smem + lay.xs) + HP; /* [-HP, n) */
    int32_t* cf = reinterpret_cast<int32_t*>(smem + lay.cf);      /* order p's c_1..c_p at p(p-1)/2 */
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + lay.red);
    int32_t* ks = reinterpret_cast<int32_t*>(smem + lay.ks);
    unsigned long long* fs = reinterpret_cast<unsigned long long*>(smem + lay.fs);
    unsigned long long* preA = reinterpret_cast<unsigned long long*>(smem + lay.pre);
    uint8_t* prmN = smem + lay.prm;
    unsigned long long* rb = reinterpret_cast<unsigned long long*>(smem + lay.rb);
    int* misc = reinterpret_cast<int*>(smem + lay.misc);
    Decision* dec = reinterpret_cast<Decision*>(smem + lay.dec);
    flacmi_unit_meta* meta = a.meta + gid;
    const int32_t* __restrict__ rec = a.rec + gid * a.rec_words;
    const int32_t* __restrict__ src = (const int32_t*)a.samples + (a.unit0 + gid) * a.stride;
    auto list_unit = [&]() __attribute__((always_inline)) { /* workgroup-uniform callers */
        if (tid == 0) {
            meta->status = FLACMI_STATUS_RETRY;
            const unsigned long long k = atomicAdd(a.retry_count, 1ull);
            a.retry_list[k] = gid;
        }
    };

    /* ---- 1. staging: samples, record status / coefficient words / shifts, max|x| ---- */
    const int st = rec[0];
    const uint32_t negmask = (uint32_t)rec[1];
    constexpr int CFS = sb_cf_stride(LMAX), NCF = LMAX * CFS, KCF = (NCF + NT - 1) / NT;
    int32_t cw[KCF]; /* padded-table entry tid + j NT: order row / CFS + 1, coefficient row % CFS */
#pragma unroll
    for (int j = 0; j < KCF; ++j) {
        const int t = tid + j * NT, row = t / CFS, col = t - row * CFS, pp = row + 1;
        const int32_t v = rec[min(2 + L + (pp * (pp - 1)) / 2 + col, a.rec_words - 1)];
        cw[j] = (pp <= L && col < pp) ? v : 0;
    }
    const int32_t shl = rec[2 + min(lane, L - 1)]; /* order lane + 1's shift (wave 0's test) */
    uint32_t xm = 0;
    {
        const int nv = n >> 2;
        const int4v* s4 = reinterpret_cast<const int4v*>(src);
        int4v* x4 = reinterpret_cast<int4v*>(xs);
        constexpr int KB = 8; /* n <= 16384: every load of the unit in flight at once */
        for (int v0 = tid; v0 < nv; v0 += KB * NT) {
            int4v q[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) q[k] = s4[min(v0 + k * NT, nv - 1)];
#pragma unroll
            for (int k = 0; k < KB; ++k)
                if (v0 + k * NT < nv) {
                    x4[v0 + k * NT] = q[k];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint32_t ax = q[k][e] < 0 ? 0u - (uint32_t)q[k][e] : (uint32_t)q[k][e];
                        xm = ax > xm ? ax : xm;
                    }
                }
        }
    }
    for (int i = tid; i < HP; i += NT) xs[i - HP] = 0;
#pragma unroll
    for (int j = 0; j < KCF; ++j)
        if (tid + j * NT < NCF) cf[tid + j * NT] = cw[j];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t t = (uint32_t)__shfl_xor((int)xm, o);
        xm = t > xm ? t : xm;
    }
    if (lane == 0) misc[8 + wid] = (int)xm;
    __syncthreads();
    if (st != 0) { /* the reference raises inside encode_subframe_lpc */
        if (tid == 0) put_meta(meta, st & 0xffff, st >> 16, nullptr, 0);
        return;
    }
    {
        uint32_t xw = 0;
#pragma unroll
        for (int w2 = 0; w2 < nw; ++w2) xw = max(xw, (uint32_t)misc[8 + w2]);
        if (xw > 0x800000u) { /* |x| > 2^23: the 32-bit partials below do not hold */
            list_unit();
            return;
        }
    }
    if (a.stop_after == 1) return;

    /* ---- 2. fixed sums over every chunk, the bound's K_j over the first split chunks ---- */
    int32_t kc[LMAX + 1];
    int32_t kneg = 0;
#pragma unroll
    for (int j = 0; j <= LMAX; ++j) kc[j] = 0;
    /* w_i = sign(x_i), m_i = x_i >> 31: w_i x = (x ^ m_i) - m_i, so sum_i w_i x_{i-j} =
     * sum_i (x_{i-j} ^ m_i) + #{m_i = -1}, one v_xad_u32 per sample and lag; at most four
     * chunks per thread of |x| <= 2^23: |kc| < 2^28.01 */
    auto bound_chunk = [&](const int32_t (&xw)[LMAX + 8]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int32_t m = xw[LMAX + k] >> 31;
            kneg -= m;
#pragma unroll
            for (int j = 0; j <= LMAX; ++j)
                kc[j] = (int32_t)xad_u32((uint32_t)xw[LMAX + k - j], (uint32_t)m, (uint32_t)kc[j]);
        }
    };
    auto load_window = [&](int i0, int32_t (&xw)[LMAX + 8]) __attribute__((always_inline)) {
        const int4v* w4 = reinterpret_cast<const int4v*>(xs + i0 - LMAX); /* samples i0 - LMAX .. i0 + 7 */
#pragma unroll
        for (int g = 0; g < LMAX / 4 + 2; ++g) {
            const int4v v = w4[g];
#pragma unroll
            for (int e = 0; e < 4; ++e) xw[4 * g + e] = v[e];
        }
    };
    constexpr int split = kSbSplit;
    {
        uint64_t fa[5] = {0, 0, 0, 0, 0};
        auto fixed_chunk_sums = [&](const int32_t (&x12)[12], int i0) __attribute__((always_inline)) {
            uint32_t ca[5] = {0, 0, 0, 0, 0};
            if (i0 >= 8) fixed_sums32<false>(x12, i0, n, ca);
            else fixed_sums32<true>(x12, i0, n, ca);
#pragma unroll
            for (int o = 0; o < 5; ++o) fa[o] += ca[o];
        };
        /* the first split chunks of each thread: the bound's terms beside the fixed sums */
#pragma unroll 1
        for (int k = 0; k < split; ++k) {
            const int c = tid + k * NT;
            if (c >= nch) break;
            const int i0 = 8 * c;
            int32_t xw[LMAX + 8];
            load_window(i0, xw);
            int32_t x12[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) x12[e] = xw[LMAX - 4 + e];
            if (i0 >= LMAX) bound_chunk(xw);
            fixed_chunk_sums(x12, i0);
        }
        /* the rest: fixed sums only */
#pragma unroll 1
        for (int c = tid + split * NT; c < nch; c += NT) {
            const int i0 = 8 * c;
            const int4v* w4 = reinterpret_cast<const int4v*>(xs + i0 - 4);
            int32_t x12[12];
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const int4v v = w4[g];
#pragma unroll
                for (int e = 0; e < 4; ++e) x12[4 * g + e] = v[e];
            }
            fixed_chunk_sums(x12, i0);
        }
        uint64_t any = 0;
#pragma unroll
        for (int o = 0; o < 5; ++o) any |= fa[o];
        if (__ballot(any >= (1ull << 26)) == 0) { /* every lane < 2^26: 32-bit wave sums */
#pragma unroll
            for (int o = 0; o < 5; ++o) {
                const uint32_t v = wave_sum_u32((uint32_t)fa[o]);
                if (lane == 0) red[wid * NR + o] = v;
            }
        } else {
#pragma unroll
            for (int o = 0; o < 5; ++o) {
                const uint64_t v = wave_sum_u64(fa[o]);
                if (lane == 0) red[wid * NR + o] = v;
            }
        }
    }
    /* K_j row sums: quads, then row_half_mirror and row_mirror (4 DPP adds a lag); lane 15
     * of each 16-lane row writes its row's sums.  A pass adds at most 16 terms per lane, each
     * in [-2^23, 2^23 - 1] ((x ^ m) of a sample with |x| <= 2^23), so a row's sum of 256 terms
     * stays inside int32.  N_- as one u32 wave sum. */
    auto reduce_k = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j <= LMAX; ++j) {
            uint32_t v = (uint32_t)kc[j];
            v += dpp_u32<0xB1, 0xf>(v);
            v += dpp_u32<0x4E, 0xf>(v);
            v += dpp_u32<0x141, 0xf>(v);
            v += dpp_u32<0x140, 0xf>(v);
            kc[j] = (int32_t)v;
        }
        if ((lane & 15) == 15) {
            int32_t* dst = ks + (wid * 4 + (lane >> 4)) * KS;
#pragma unroll
            for (int j = 0; j <= LMAX; ++j) dst[j] = kc[j];
        }
        const uint32_t v = wave_sum_u32((uint32_t)kneg);
        if (lane == 0) red[wid * NR + 5] = v;
    };
    auto lane64 = [&](int64_t v, int l) __attribute__((always_inline)) -> int64_t {
        return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l));
    };
    /* wave 0: every order's bound against the best exact fixed sum; misc[0] = decided, and a
     * decided unit's choice into dec (fixed order = the first minimum, LPC pruned) */
    int64_t kt = 0; /* wave 0's K_j totals, kept across the two passes */
    auto evaluate = [&]() __attribute__((always_inline)) {
        uint64_t tf = 0;
        if (lane < 5) {
#pragma unroll
            for (int w2 = 0; w2 < nw; ++w2) tf += red[w2 * NR + lane];
        }
        const uint64_t f0 = (uint64_t)lane64((int64_t)tf, 0);
        uint64_t fmin = f0;
        int fo = 0;
#pragma unroll
        for (int o = 1; o < 5; ++o) {
            const uint64_t v = (uint64_t)lane64((int64_t)tf, o);
            if (v < fmin) fmin = v, fo = o;
        }
        /* lane j <= LMAX: K_j - N_- so far; lane LMAX + 1: N_- (kt accumulates over the passes) */
        if (lane <= LMAX) {
#pragma unroll 8
            for (int r = 0; r < 4 * nw; ++r) kt += (int64_t)ks[r * KS + lane];
        } else if (lane == LMAX + 1) {
#pragma unroll
            for (int w2 = 0; w2 < nw; ++w2) kt += (int64_t)red[w2 * NR + 5];
        }
        const int64_t nneg = lane64(kt, LMAX + 1), k0 = lane64(kt, 0) + nneg;
        const int pl = lane + 1;
        int64_t S = 0;
        /* row pl - 1 holds c_{pl,1..pl} and zeros up to LMAX; lanes past LMAX read row 0 (unused) */
        const int4v* crow = reinterpret_cast<const int4v*>(cf + (lane < LMAX ? lane : 0) * CFS);
#pragma unroll 2
        for (int jb = 0; jb < LMAX / 4; ++jb) {
            const int4v c4 = crow[jb];
#pragma unroll
            for (int e = 0; e < 4; ++e) S += (int64_t)c4[e] * (lane64(kt, 4 * jb + e + 1) + nneg);
        }
        bool lose = true; /* this lane's order provably loses */
        if (pl <= L) {
            if ((negmask >> lane) & 1) lose = f0 > fmin; /* ((), 0): r = x, the fixed order-0 sum */
            else lose = k0 - (S >> shl) - 1 - nneg > (int64_t)fmin;
        }
        const bool decided = __ballot(!lose) == 0;
        if (lane == 0) {
            misc[0] = decided ? 1 : 0;
            misc[1] = fo;
            if (decided) {
                dec->status = ST_OK;
                dec->site = 0;
                dec->kind = FLACMI_KIND_FIXED;
                dec->order = fo;
                dec->shift = 0;
                dec->ncoefs = 0;
                dec->fixed_order = fo;
                dec->lpc_order = FLACMI_LPC_PRUNED;
                dec->tiers = 8 << 8; /* 0 of the eighths (meta.lpc_tiers, as kVarMf8) */
                dec->fixed_sum = (long long)fmin;
                dec->lpc_sum = (long long)FLACMI_LPC_PRUNED;
            }
        }
    };
    reduce_k();
    __syncthreads();
    if (wid == 0) evaluate();
    __syncthreads();
    if (misc[0] == 0 && split < (nch + NT - 1) / NT) {
        /* the rest of R, summed on its own (wave 0 adds its row sums to the first pass's totals) */
#pragma unroll
        for (int j = 0; j <= LMAX; ++j) kc[j] = 0;
        kneg = 0;
#pragma unroll 1
        for (int c = tid + split * NT; c < nch; c += NT) {
            int32_t xw[LMAX + 8];
            load_window(8 * c, xw);
            bound_chunk(xw);
        }
        reduce_k();
        __syncthreads();
        if (wid == 0) evaluate();
        __syncthreads();
    }
    if (misc[0] == 0) { /* an LPC order may win or tie: the list variant's exact tiers */
        list_unit();
        return;
    }
    if (a.stop_after == 2 || a.stop_after == 3) return;
    const int fo = __builtin_amdgcn_readfirstlane(misc[1]);

    /* ---- 4. the chosen fixed residual and the Rice search (the wide path of k_resid) ---- */
    auto tail = [&](auto K_) __attribute__((always_inline)) {
        constexpr int K = decltype(K_)::value;
        uint32_t* __restrict__ rout = reinterpret_cast<uint32_t*>(a.residual) + gid * a.residual_stride;
        /* the residual stays in registers for the data-bits pass (kept, not recomputed): at most
         * kSbChunks chunks per thread (n <= 16384) */
        uint32_t zr[kSbChunks][8];
#pragma unroll
        for (int j = 0; j < kSbChunks; ++j) {
            const int c = tid + j * NT;
            if (c < nch) { /* whole 32-lane groups: nch % 32 == 0 and the partitions' chunk runs divide 32 */
                fixed_resid_chunk32<K>(xs, 8 * c, n, zr[j]);
                reinterpret_cast<uint4*>(rout + 8 * c)[0] = uint4{zr[j][0], zr[j][1], zr[j][2], zr[j][3]};
                reinterpret_cast<uint4*>(rout + 8 * c)[1] = uint4{zr[j][4], zr[j][5], zr[j][6], zr[j][7]};
                uint32_t c32 = 0; /* every value < 2^28: eight < 2^31 */
#pragma unroll
                for (int k = 0; k < 8; ++k) c32 += zr[j][k];
                /* the finest partition's sum over its cpp consecutive lanes: DPP steps in 32 bits
                 * while every chunk sum of the wave is < 2^26 (a partition of <= 32 chunks then
                 * stays < 2^31), else 64-bit shuffles */
                uint64_t cs8;
                if (__ballot(c32 >= (1u << 26)) == 0 && cpp <= 16) {
                    uint32_t v = c32;
                    if (cpp >= 2) v += dpp_u32<0xB1, 0xf>(v);  /* quad_perm [1,0,3,2] */
                    if (cpp >= 4) v += dpp_u32<0x4E, 0xf>(v);  /* quad_perm [2,3,0,1] */
                    if (cpp >= 8) v += dpp_u32<0x141, 0xf>(v); /* row_half_mirror: the other quad */
                    if (cpp >= 16) v += dpp_u32<0x140, 0xf>(v); /* row_mirror: the other half row */
                    cs8 = v;
                } else {
                    cs8 = c32;
                    for (int w = 1; w < cpp; w <<= 1) cs8 += (uint64_t)__shfl_xor((unsigned long long)cs8, w);
                }
                if ((c & (cpp - 1)) == 0) fs[P + c / cpp] = cs8;
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) zr[j][k] = 0;
            }
        }
        __syncthreads();
        if (a.stop_after == 4) return;
        const int ro = R08 ? 0 : __builtin_amdgcn_readfirstlane(a.rmin), oo = R08 ? 8 : __builtin_amdgcn_readfirstlane(omax);
        /* prefix sums of the finest sums (wave 0), then every heap node's parameter, one node
         * per thread, header bits per order, the first error in the reference's evaluation
         * order by atomicMin (see k_resid's wide Rice step) */
        if (wid == 0) {
            const int J = P >> 6; /* 1, 2 or 4 */
            uint64_t v[4] = {0, 0, 0, 0}, t = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < J) v[j] = fs[P + J * lane + j], t += v[j];
            uint64_t inc = t;
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
            if (lane == 0) misc[2] = 0x7fffffff, misc[4] = 0;
        }
        __syncthreads();
        for (int j0 = (1 << ro); j0 < 2 * P; j0 += NT) {
            const int j = j0 + tid;
            const bool live = j < 2 * P;
            const int o = live ? 31 - __builtin_clz((unsigned)j) : 0;
            uint32_t hb = 0;
            bool big = false;
            if (live) {
                const int Kn = j - (1 << o), d = omax - o;
                const uint64_t S = preA[((Kn + 1) << d) - 1] - (Kn > 0 ? preA[(Kn << d) - 1] : 0ull);
                const int len = (n >> o) - (Kn == 0 ? K : 0);
                int prm = 0;
                if (S != 0) { /* S < n 2^32 <= 2^46: exact integer floor(log2(S / len)) */
                    const int fsb = 63 - __builtin_clzll((unsigned long long)S);
                    const int flb = 31 - __builtin_clz((unsigned)len);
                    prm = fsb - flb;
                    if (prm >= 0 && ((uint64_t)len << prm) > S) --prm;
                }
                prmN[j] = (uint8_t)prm;
                if (S == 0 || prm < 0) atomicMin(&misc[2], (j << 1) | (S == 0 ? 1 : 0));
                big = prm > 14;
                hb = 4u + (prm > 14 ? 5u : 4u) + (uint32_t)len * (uint32_t)(1 + prm);
            }
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
        __syncthreads();
        if (a.stop_after == 5) return;
        if (misc[2] != 0x7fffffff) {
            if (tid == 0)
                put_meta(meta, ST_VALUE, (misc[2] & 1) ? FLACMI_SITE_RICE_LOG_DOMAIN : FLACMI_SITE_RICE_NEG_SHIFT, dec, 1);
            return;
        }
        /* finest partition k's row: byte o = p_o - pm, byte 14 = some delta >= 16, byte 15 = pm
         * (over the finest sums, consumed by the prefix step) */
        uint8_t* pk = reinterpret_cast<uint8_t*>(fs);
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
            w[3] |= ((dmax >= 16 ? 1u : 0u) << 16) | (pm << 24);
            *reinterpret_cast<uint4*>(pk + 16 * k) = uint4{w[0], w[1], w[2], w[3]};
        }
        __syncthreads();
        if (a.stop_after == 6) return;
        /* data bits: sum over the residual (the registers of the residual pass) of (z >> p) for
         * every candidate order; y = z >> pm as packed 16-bit pairs where it fits */
        const uint4* pkv = reinterpret_cast<const uint4*>(pk);
        uint64_t tb[16];
        uint32_t tp[16]; /* packed-path totals: < 4 chunks * 8 * 2^16 per order */
#pragma unroll
        for (int o = 0; o < 16; ++o) tb[o] = 0, tp[o] = 0;
#pragma unroll
        for (int j = 0; j < kSbChunks; ++j) {
            const int c = tid + j * NT;
            if (c >= nch) continue;
            const uint32_t(&z)[8] = zr[j];
            const uint4 pv = pkv[c / cpp];
            const uint32_t pm = pv.w >> 24;
            uint32_t y[8], yo = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) y[k] = z[k] >> pm, yo |= y[k];
            if ((yo >> 16) == 0 && ((pv.w >> 16) & 0xffu) == 0) {
                uint32_t yp[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) yp[i] = __builtin_amdgcn_perm(y[2 * i + 1], y[2 * i], 0x05040100u);
                const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                for (int o = 0; o < 16; ++o)
                    if (o >= ro && o <= oo) {
                        const uint32_t sel = (o & 3) == 0 ? 0x0c000c00u : (o & 3) == 1 ? 0x0c010c01u
                                             : (o & 3) == 2 ? 0x0c020c02u : 0x0c030c03u;
                        const us2x d = __builtin_bit_cast(us2x, __builtin_amdgcn_perm(0u, pw[o >> 2], sel));
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            tp[o] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2x, yp[i]) >> d, us2x{1, 1}, tp[o], false);
                    }
            } else {
                /* z < 2^28 on this path: a chunk's eight shifted values sum in 32 bits */
                uint32_t t32[16];
#pragma unroll
                for (int o = 0; o < 16; ++o) t32[o] = 0;
                chunk_rice_bits(y, pv, ro, oo, t32);
#pragma unroll
                for (int o = 0; o < 16; ++o)
                    if (o >= ro && o <= oo) tb[o] += t32[o];
            }
        }
#pragma unroll
        for (int o = 0; o < 16; ++o) tb[o] += tp[o];
        if (a.stop_after == 7) {
            if (tb[0] == 0x9e3779b9u) meta->lpc_tiers = 1;
            return;
        }
        {
            uint64_t any = 0;
#pragma unroll
            for (int o = 0; o < 16; ++o) any |= (o >= ro && o <= oo) ? tb[o] : 0ull;
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
        __syncthreads();
        {
            /* lane o: order o's total; the first minimum by key = total * 16 + order */
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
                put_meta_wave(meta, lane, ST_OK, 0, dec, K, n - K, best, 1 << best, ((misc[4] >> best) & 1) ? 5 : 4,
                              (long long)bits);
            int32_t* __restrict__ rp = a.rice_params + gid * a.params_stride;
            for (int Kp = tid; Kp < (1 << best); Kp += NT) {
                const int row = 16 * (Kp << (omax - best));
                rp[Kp] = pk[row + 15] + pk[row + best]; /* pm + delta */
            }
        }
    };
    switch (fo) {
        case 0: tail(std::integral_constant<int, 0>{}); break;
        case 1: tail(std::integral_constant<int, 1>{}); break;
        case 2: tail(std::integral_constant<int, 2>{}); break;
        case 3: tail(std::integral_constant<int, 3>{}); break;
        default: tail(std::integral_constant<int, 4>{}); break;
    }
}


hipError_t launch_resid_sb_kernel(const ResidArgs& a, int lmax, hipStream_t s) {
    const int om = sb_finest_order(a.n, a.rmin, a.rmax);
    const size_t lds = sb_lds_layout(lmax, a.n, 1 << om).total;
    const bool r08 = a.rmin == 0 && om == 8;
    auto ks = lmax == 16 ? (r08 ? k_resid_sb<16, true> : k_resid_sb<16, false>)
                         : (r08 ? (a.n == 16384 && a.L == 32 ? k_resid_sb<32, true, 16384> : k_resid_sb<32, true>)
                                : k_resid_sb<32, false>);
    hipError_t e = hipFuncSetAttribute((const void*)ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ks, dim3((unsigned)a.count), dim3(kSbThreads), lds, s, a);
    return hipGetLastError();
}

}  // namespace flacmi
