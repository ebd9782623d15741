/*
 * flacmi_host.cpp — the C-ABI of libflacmi.so (include/flacmi.h): contexts, argument
 * validation, per-length launch planning, tables computed from the host libm, and
 * device-memory helpers.  All compute is in the HIP kernels (k_*.hip).
 *
 * Host-side tables (built with the same libm CPython uses, so the device sees exactly
 * the values the reference computes):
 *   - Tukey(0.5) window per block length (flac/encoder.py:423-440, libm cos);
 *   - floor(log2(x)) thresholds per binary exponent (libm log2), for
 *     quantize_lpc_coefficients (encoder.py:503) and find_rice_parameter (:753);
 *   - the int16 sine table of the synthetic generator (libm sin).
 * This file is compiled with -ffp-contract=off like the kernels.
 */
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/flacmi.h"
#include "flacmi_kernels.h"
#include "pymath.h"
#include "device_common.h"

using namespace flacmi;

static double (*volatile libm_cos)(double) = cos;
static double (*volatile libm_log2)(double) = log2;
static double (*volatile libm_sin)(double) = sin;

/* ------------------------------------------------------------------------------------
 * errors
 * ---------------------------------------------------------------------------------- */
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(FLACMI_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                            \
    } while (0)

/* ------------------------------------------------------------------------------------
 * process-wide host tables
 * ---------------------------------------------------------------------------------- */
static std::once_flag g_tables_once;
static std::vector<double> g_log2thr;   /* PYM_LOG2_THR_N */
static std::vector<int32_t> g_sintab;   /* 4096 */
static std::string g_tables_error;

static void build_tables() {
    g_log2thr.assign(PYM_LOG2_THR_N, 0.0);
    for (int e = -1074; e <= 1023; ++e) {
        const double hi = ldexp(1.0, e + 1); /* inf for e = 1023 */
        double thr = hi;
        {
            double x = nextafter(hi, 0.0); /* DBL_MAX for e = 1023 */
            while (x >= ldexp(1.0, e) && libm_log2(x) >= (double)(e + 1)) {
                thr = x;
                x = nextafter(x, 0.0);
            }
            /* monotonicity guard: nothing further below may reach e + 1 */
            for (int k = 0; k < 64 && x >= ldexp(1.0, e); ++k, x = nextafter(x, 0.0))
                if (libm_log2(x) >= (double)(e + 1)) g_tables_error = "libm log2 not monotonic near a power of two";
        }
        /* and nothing just above 2^e may fall below e */
        double y = ldexp(1.0, e);
        for (int k = 0; k < 64; ++k, y = nextafter(y, INFINITY))
            if (libm_log2(y) < (double)e) g_tables_error = "libm log2 below the exponent just above 2^e";
        g_log2thr[e + 1074] = thr;
    }
    g_sintab.resize(4096);
    for (int k = 0; k < 4096; ++k)
        g_sintab[k] = (int32_t)nearbyint(32767.0 * libm_sin(6.283185307179586 * (double)k / 4096.0));
}

static void ensure_tables() { std::call_once(g_tables_once, build_tables); }

/* CRC-16 tables of the frame writer (poly x^16 + x^15 + x^2 + 1, MSB first, init 0;
 * crc.py:25-31): [4][256] slice-by-4 tables T_k[v] = v * x^(16+8k) mod P, then for
 * b = 0..27 the linear map c -> c * x^(8*2^b) mod P as two 256-entry tables (low byte,
 * high byte of c), built by repeated squaring of the map. */
static std::vector<uint16_t> crc16_tables() {
    std::vector<uint16_t> t(4 * 256 + 28 * 512);
    auto mul8 = [&](uint32_t r) -> uint32_t { return ((r << 8) & 0xFFFF) ^ t[r >> 8]; };
    for (uint32_t v = 0; v < 256; ++v) {
        uint32_t r = v << 8;
        for (int i = 0; i < 8; ++i) r = (r & 0x8000) ? ((r << 1) ^ 0x8005) & 0xFFFF : (r << 1) & 0xFFFF;
        t[v] = (uint16_t)r;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t v = 0; v < 256; ++v) t[k * 256 + v] = (uint16_t)mul8(t[(k - 1) * 256 + v]);
    uint32_t M[16], M2[16];
    for (int i = 0; i < 16; ++i) M[i] = mul8(1u << i);
    auto apply = [](const uint32_t* m, uint32_t c) {
        uint32_t r = 0;
        for (int i = 0; i < 16; ++i)
            if (c >> i & 1) r ^= m[i];
        return r;
    };
    for (int b = 0; b < 28; ++b) {
        uint16_t* o = t.data() + 4 * 256 + b * 512;
        for (uint32_t v = 0; v < 256; ++v) {
            o[v] = (uint16_t)apply(M, v);
            o[256 + v] = (uint16_t)apply(M, v << 8);
        }
        for (int i = 0; i < 16; ++i) M2[i] = apply(M, apply(M, 1u << i));
        memcpy(M, M2, sizeof M);
    }
    return t;
}

/* Tukey(0.5) window exactly as encoder.py:423-440 computes it; padded with zeros. */
static std::vector<double> tukey_window(int n, int pad) {
    std::vector<double> w((size_t)n + pad, 0.0);
    for (int i = 0; i < n; ++i) w[i] = 1.0;
    const int nr = (int)floor(0.25 * (double)n) - 1;
    if (nr > 0) {
        for (int i = 0; i < nr + 1; ++i) {
            w[i] = 0.5 - 0.5 * libm_cos(3.141592653589793 * (double)i / (double)nr);
            w[n - nr - 1 + i] = 0.5 - 0.5 * libm_cos(3.141592653589793 * (double)(i + nr) / (double)nr);
        }
    }
    return w;
}

/* ------------------------------------------------------------------------------------
 * context
 * ---------------------------------------------------------------------------------- */
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct flacmi_ctx {
    int device = 0;
    hipStream_t stream = nullptr; /* used by the host entry points */
    double* d_log2thr = nullptr;
    int32_t* d_sintab = nullptr;
    std::map<int, double*> windows;
    std::map<int, std::pair<int, int>> window_one; /* per n: [lo, hi) where the weight is 1.0 */
    DevBuf rec, retry, h_samples, h_meta, h_params, h_residual, h_acf, h_fs, h_ls, h_recs;
    uint16_t* d_crc = nullptr;  /* CRC-16 slice tables [4][256] + power tables [28][512] */
    DevBuf scan, h_offsets, h_status, h_frames, dec, slow;
    int64_t frames_bytes = 0;   /* bytes of the last flacmi_encode_host call */
    static constexpr int kRing = 64;
    static constexpr int kMaxChunks = 8;
    /* per call: start, LPC done, residual done, then (overlap) per chunk the k_resid start/end */
    hipEvent_t ev[kRing][3 + 2 * kMaxChunks] = {};
    int nchunks[kRing] = {};
    hipEvent_t lpc_done[kMaxChunks] = {}; /* k_lpc of chunk i finished (no timing) */
    int ncalls = 0; /* calls since the last timing reset */
    struct EncState* enc = nullptr; /* flacmi_encode_pipeline's streams, slots and pinned arrays */
};
static void enc_free(struct EncState* es);
static int enc_streams(flacmi_ctx* ctx);
static hipStream_t enc_side(flacmi_ctx* ctx);

static int ensure_buf(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return 0;
    if (b.p) HIP_TRY(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    size_t want = bytes + bytes / 8 + 4096;
    HIP_TRY(hipMalloc(&b.p, want));
    b.bytes = want;
    return 0;
}

/* device row pitch in samples (flacmi_unit_stride) */
static int64_t row_pitch(int64_t n, int64_t sample_bytes) {
    int64_t bytes = ((n * sample_bytes + 15) / 16) * 16;
    if (bytes % 4096 == 0) bytes += 128;
    return bytes / sample_bytes;
}

static int set_device(flacmi_ctx* ctx) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    HIP_TRY(hipSetDevice(ctx->device));
    return 0;
}

/* flacmi_set_knob: environment read once, then atomics (no getenv on launch paths) */
namespace {
struct KnobDef {
    const char* name;
    int dflt;
};
constexpr KnobDef kKnobs[kKnobCount] = {{"FLACMI_OVERLAP", -1}, {"FLACMI_MF8_GRID", 0}, {"FLACMI_STREAM_GENERIC", 0}, {"FLACMI_DECODE_GENERIC", 0},
                                        {"FLACMI_PACK_GENERIC", 0}};
std::atomic<int> g_knob[kKnobCount];
std::once_flag g_knob_once;
void knobs_init() {
    std::call_once(g_knob_once, [] {
        for (int i = 0; i < kKnobCount; ++i) {
            const char* e = getenv(kKnobs[i].name);
            g_knob[i].store(e && e[0] ? atoi(e) : kKnobs[i].dflt);
        }
    });
}
int knob_index(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < kKnobCount; ++i)
        if (strcmp(name, kKnobs[i].name) == 0) return i;
    return -1;
}
}  // namespace

int flacmi::knob(Knob k) {
    knobs_init();
    return g_knob[k].load(std::memory_order_relaxed);
}

extern "C" {

int flacmi_set_knob(const char* name, int32_t value) {
    const int i = knob_index(name);
    if (i < 0) return fail(FLACMI_E_INVALID, "unknown knob %s", name ? name : "(null)");
    knobs_init();
    g_knob[i].store(value);
    return 0;
}

int flacmi_get_knob(const char* name, int32_t* value) {
    const int i = knob_index(name);
    if (i < 0 || !value) return fail(FLACMI_E_INVALID, "unknown knob %s", name ? name : "(null)");
    *value = knob((Knob)i);
    return 0;
}

int flacmi_abi_version(void) { return FLACMI_ABI_VERSION; }

const char* flacmi_last_error(void) { return g_err.c_str(); }

int flacmi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

flacmi_ctx* flacmi_create(int device) {
    ensure_tables();
    if (!g_tables_error.empty()) {
        fail(FLACMI_E_UNSUPPORTED, "%s", g_tables_error.c_str());
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail(FLACMI_E_HIP, "no HIP device available");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        fail(FLACMI_E_INVALID, "device %d out of range (0..%d)", device, ndev - 1);
        return nullptr;
    }
    flacmi_ctx* ctx = new flacmi_ctx();
    ctx->device = device;
    auto bad = [&](hipError_t e, const char* what) {
        fail(FLACMI_E_HIP, "%s: %s", what, hipGetErrorString(e));
        flacmi_destroy(ctx);
        return (flacmi_ctx*)nullptr;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bad(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    for (auto& slot : ctx->ev)
        for (auto& ev : slot)
            if ((e = hipEventCreate(&ev)) != hipSuccess) return bad(e, "hipEventCreate");
    for (auto& ev : ctx->lpc_done)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipMalloc(&ctx->d_log2thr, sizeof(double) * PYM_LOG2_THR_N)) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemcpy(ctx->d_log2thr, g_log2thr.data(), sizeof(double) * PYM_LOG2_THR_N, hipMemcpyHostToDevice)) != hipSuccess)
        return bad(e, "hipMemcpy");
    if ((e = hipMalloc(&ctx->d_sintab, sizeof(int32_t) * 4096)) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemcpy(ctx->d_sintab, g_sintab.data(), sizeof(int32_t) * 4096, hipMemcpyHostToDevice)) != hipSuccess)
        return bad(e, "hipMemcpy");
    const std::vector<uint16_t> crc = crc16_tables();
    if ((e = hipMalloc(&ctx->d_crc, sizeof(uint16_t) * crc.size())) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemcpy(ctx->d_crc, crc.data(), sizeof(uint16_t) * crc.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return bad(e, "hipMemcpy");
    return ctx;
}

void flacmi_destroy(flacmi_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    enc_free(ctx->enc);
    for (auto& kv : ctx->windows) (void)hipFree(kv.second);
    for (DevBuf* b : {&ctx->slow, &ctx->dec, &ctx->rec, &ctx->retry, &ctx->h_samples, &ctx->h_meta, &ctx->h_params, &ctx->h_residual, &ctx->h_acf,
                      &ctx->h_fs, &ctx->h_ls, &ctx->h_recs, &ctx->scan, &ctx->h_offsets, &ctx->h_status,
                      &ctx->h_frames})
        if (b->p) (void)hipFree(b->p);
    if (ctx->d_log2thr) (void)hipFree(ctx->d_log2thr);
    if (ctx->d_sintab) (void)hipFree(ctx->d_sintab);
    if (ctx->d_crc) (void)hipFree(ctx->d_crc);
    for (auto& slot : ctx->ev)
        for (auto& ev : slot)
            if (ev) (void)hipEventDestroy(ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    for (auto& ev : ctx->lpc_done)
        if (ev) (void)hipEventDestroy(ev);
    delete ctx;
}

}  // extern "C"

static int get_window(flacmi_ctx* ctx, int n, double** out, int* one_lo = nullptr, int* one_hi = nullptr) {
    auto it = ctx->windows.find(n);
    if (it == ctx->windows.end()) {
        std::vector<double> w = tukey_window(n, 64);
        double* d = nullptr;
        HIP_TRY(hipMalloc(&d, sizeof(double) * w.size()));
        HIP_TRY(hipMemcpy(d, w.data(), sizeof(double) * w.size(), hipMemcpyHostToDevice));
        ctx->windows[n] = d;
        /* the longest run of weights exactly 1.0 (the rectangle of encoder.py:433) */
        int best_lo = 0, best_hi = 0;
        for (int i = 0; i < n;) {
            if (w[i] != 1.0) {
                ++i;
                continue;
            }
            int j = i;
            while (j < n && w[j] == 1.0) ++j;
            if (j - i > best_hi - best_lo) {
                best_lo = i;
                best_hi = j;
            }
            i = j;
        }
        ctx->window_one[n] = {best_lo, best_hi};
        it = ctx->windows.find(n);
    }
    *out = it->second;
    if (one_lo) *one_lo = ctx->window_one[n].first;
    if (one_hi) *one_hi = ctx->window_one[n].second;
    return 0;
}

/* Largest candidate partition order for a block of n samples (predictor order 0). */
static int rice_max_eff(int n, int rmin, int rmax) {
    int r = -1;
    for (int o = rmin; o <= rmax; ++o)
        if (n % (1 << o) == 0) r = o;
    return r;
}

static int validate(const flacmi_batch* b, const flacmi_params* p, const flacmi_outputs* o) {
    if (!b || !p || !o) return fail(FLACMI_E_INVALID, "null argument");
    if (b->sample_bytes != 2 && b->sample_bytes != 4) return fail(FLACMI_E_INVALID, "sample_bytes must be 2 or 4");
    if (b->sample_bits < 2 || b->sample_bits > 8 * b->sample_bytes)
        return fail(FLACMI_E_INVALID, "sample_bits %d invalid for %d-byte samples", b->sample_bits, b->sample_bytes);
    if (b->n_units < 0 || b->n_tail_units < 0 || b->n_tail_units > b->n_units)
        return fail(FLACMI_E_INVALID, "bad unit counts");
    if (b->block_len < 1 || b->block_len > FLACMI_MAX_BLOCK) return fail(FLACMI_E_INVALID, "block_len out of range");
    if (b->n_tail_units > 0 && (b->tail_len < 1 || b->tail_len > b->block_len))
        return fail(FLACMI_E_INVALID, "tail_len out of range");
    if (b->unit_stride < b->block_len) return fail(FLACMI_E_INVALID, "unit_stride < block_len");
    if ((b->unit_stride * b->sample_bytes) % 16 != 0 || ((uintptr_t)b->samples % 16) != 0)
        return fail(FLACMI_E_INVALID, "sample rows must be 16-byte aligned");
    if (p->max_lpc_order < 0 || p->max_lpc_order > FLACMI_MAX_LPC_ORDER)
        return fail(FLACMI_E_INVALID, "max_lpc_order must be 0..32");
    if (p->qlp_precision < 5 || p->qlp_precision > 31) return fail(FLACMI_E_INVALID, "qlp_precision must be 5..31");
    if (p->rice_min < 0 || p->rice_max > FLACMI_MAX_RICE_ORDER)
        return fail(FLACMI_E_INVALID, "rice partition orders must be within 0..15");
    if (p->mode < FLACMI_MODE_REFERENCE || p->mode > FLACMI_MODE_RICE_ONLY) return fail(FLACMI_E_INVALID, "bad mode");
    if (p->mode == FLACMI_MODE_RICE_ONLY && (p->reserved[0] < 0 || p->reserved[0] > FLACMI_MAX_LPC_ORDER))
        return fail(FLACMI_E_INVALID, "RICE_ONLY predictor order (reserved[0]) must be 0..32");
    if (p->mode == FLACMI_MODE_LPC_ONLY && p->max_lpc_order < 1)
        return fail(FLACMI_E_INVALID, "LPC_ONLY needs max_lpc_order >= 1");
    if (p->mode != FLACMI_MODE_FIXED_ONLY && p->mode != FLACMI_MODE_RICE_ONLY && b->sample_bits + p->qlp_precision > 44)
        return fail(FLACMI_E_UNSUPPORTED,
                    "sample_bits + qlp_precision > 44: candidate residual sums may exceed int64 (see DESIGN.md)");
    if (o->residual_bytes != 4 && o->residual_bytes != 8) return fail(FLACMI_E_INVALID, "residual_bytes must be 4 or 8");
    if (o->residual_stride < b->block_len || (o->residual_stride * o->residual_bytes) % 16 != 0 ||
        ((uintptr_t)o->residual % 16) != 0)
        return fail(FLACMI_E_INVALID, "residual rows must hold block_len elements and be 16-byte aligned");
    if (!o->meta || !o->rice_params || !o->residual) return fail(FLACMI_E_INVALID, "null output buffer");
    const int lens[2] = {b->block_len, b->n_tail_units ? b->tail_len : b->block_len};
    for (int n : lens) {
        const int re = rice_max_eff(n, p->rice_min, p->rice_max);
        if (re >= 0 && (1 << re) > kMaxFinestParts)
            return fail(FLACMI_E_UNSUPPORTED, "2^%d Rice partitions exceed the %d this build stages in LDS", re,
                        kMaxFinestParts);
        if (re >= 0 && o->params_stride < (1 << re)) return fail(FLACMI_E_INVALID, "params_stride < 2^%d", re);
        const ResidLaunch rl = resid_launch_config(n, re, o->residual_bytes);
        if (rl.lds_bytes > 160 * 1024)
            return fail(FLACMI_E_UNSUPPORTED, "block of %d samples needs %zu bytes of LDS", n, rl.lds_bytes);
    }
    return 0;
}

/* int32 arithmetic is exact when every |prediction| and |residual| < 2^26 and a thread's
 * partial sum of |r| over the samples it owns still fits 32 bits.  Otherwise int64. */
static bool needs_wide(int n, int bits, int L, int q, int mode) {
    if (bits > 24 || q > 24) return true;
    const double xmax = ldexp(1.0, bits - 1);
    const double rmax = (mode == FLACMI_MODE_FIXED_ONLY || mode == FLACMI_MODE_RICE_ONLY) ? 16.0 * xmax : xmax * (1.0 + (double)L * ldexp(1.0, q - 1)) + 16.0 * xmax;
    return rmax >= ldexp(1.0, 26) || rmax * resid_samples_per_thread(n) >= ldexp(1.0, 32);
}

/* PATH_W64S preconditions: samples <= 24 bits and q <= 16 (every sample plane, coefficient
 * and -2^shift fits int16), and each plane's dot chain stays inside int32:
 * max|plane| * (L * 2^(q-1) + 2^15) < 2^31.  Opt-in (FLACMI_SPLIT=1): on MI355X it
 * measured slower than PATH_W64's v_mad_i64_i32 chains (c3: 71.0 vs 67.1 ms), the plane
 * build costing more than the dot2 pairing saves. */
static bool split_ok(int bits, int L, int q) {
    static const int off = [] {
        const char* e = getenv("FLACMI_SPLIT");
        return (e && atoi(e) != 0) ? 0 : 1;
    }();
    if (off || bits > 24 || q > 16 || L < 1) return false;
    const double plane = bits > 24 - 12 ? ldexp(1.0, bits - 13) : 0.0;
    const double pmax = plane > 2048.0 ? plane : 2048.0;
    return pmax * ((double)L * ldexp(1.0, q - 1) + 32768.0) < ldexp(1.0, 31);
}

/* FLACMI_DEBUG_STOP=k truncates k_resid after phase k (profiling ablation only: the
 * outputs are then incomplete). */
static int debug_stop() {
    static const int v = [] {
        const char* e = getenv("FLACMI_DEBUG_STOP");
        return e ? atoi(e) : 0;
    }();
    return v;
}

/* FLACMI_NO_MFMA=1 keeps the candidate sums on the VALU path (comparison runs). */
static int use_mfma() {
    static const int v = [] {
        const char* e = getenv("FLACMI_NO_MFMA");
        return (e && atoi(e) != 0) ? 0 : 1;
    }();
    return v;
}

/* FLACMI_NO_STREAM=1 keeps k_resid's one-workgroup-per-unit kernels (comparison runs). */
static int use_stream() {
    static const int v = [] {
        const char* e = getenv("FLACMI_NO_STREAM");
        return (e && atoi(e) != 0) ? 0 : 1;
    }();
    return v;
}

/* FLACMI_NO_SIGNBOUND=1 prunes the int8-MFMA path with the partial-sum tiers alone, as
 * FLACMI_FLAG_TIERS_ONLY does per call (A/B runs). */
static int sign_bound_allowed() {
    static const int v = [] {
        const char* e = getenv("FLACMI_NO_SIGNBOUND");
        return (e && atoi(e) != 0) ? 0 : 1;
    }();
    return v;
}

/* FLACMI_NO_PRUNE=1 computes every LPC candidate's exact sum in reference mode, as
 * FLACMI_FLAG_ALL_CANDIDATES does per call (comparison runs). */
static int prune_allowed() {
    static const int v = [] {
        const char* e = getenv("FLACMI_NO_PRUNE");
        return (e && atoi(e) != 0) ? 0 : 1;
    }();
    return v;
}

/* k_lpc and k_resid of consecutive chunks overlap on two streams (see analyze_device_impl).
 * FLACMI_OVERLAP (flacmi_set_knob; the environment's value at first use): unset or -1 = round-aligned (the default): the units of
 * k_lpc's whole rounds, then the remainder (a partly filled last round), whose k_lpc runs
 * beside k_resid of the first chunk, when the remainder holds at least kOverlapMinUnits;
 * 0 = no overlap; k > 1 = up to k equal chunks of at least kOverlapMinUnits; -R (R > 1) =
 * round-aligned with R units per round and no minimum (tests). */
constexpr int64_t kOverlapMinUnits = 16384;
static int overlap_mode() { return knob(kKnobOverlap); }

static int analyze_device_impl(flacmi_ctx* ctx, const flacmi_batch* b, const flacmi_params* p,
                               const flacmi_outputs* o, hipStream_t s, bool allow_overlap = true) {
    if (int rc = set_device(ctx)) return rc;
    const bool lpc = p->mode == FLACMI_MODE_REFERENCE || p->mode == FLACMI_MODE_LPC_ONLY;
    const int L = lpc ? p->max_lpc_order : 0;
    const int rec_words = FLACMI_LPC_REC_WORDS(L);
    if (lpc) {
        if (int rc = ensure_buf(ctx->rec, sizeof(int32_t) * (size_t)rec_words * (size_t)(b->n_units > 0 ? b->n_units : 1)))
            return rc;
    }
    /* fast-kernel retry lists: 64 sub-list counters (k_resid_stream's batch kernel, 128 B apart),
     * a counter and one batch index per unit (plus 64 for the sub-lists' rounding), then the
     * second list through which k_resid_stream's list kernel hands units on */
    constexpr int64_t kSubWords = 64 * 16;
    if (int rc = ensure_buf(ctx->retry, sizeof(int64_t) * (size_t)(kSubWords + 2 * b->n_units + 68))) return rc;
    struct Cls {
        int64_t unit0, count;
        int n;
    } cls[2];
    int ncls = 0;
    const int64_t nfull = b->n_units - b->n_tail_units;
    if (b->n_tail_units == 0 || b->tail_len == b->block_len) {
        cls[ncls++] = {0, b->n_units, b->block_len};
    } else {
        if (nfull > 0) cls[ncls++] = {0, nfull, b->block_len};
        cls[ncls++] = {nfull, b->n_tail_units, b->tail_len};
    }
    if (o->acf && !lpc)
        HIP_TRY(hipMemsetAsync(o->acf, 0, sizeof(double) * 33 * b->n_units, s));
    /* Units in chunks of one class each.  Without overlap: one chunk per class, the LPC
     * pass over all of them, then the residual pass, in order on s.  With overlap
     * (FLACMI_OVERLAP=k > 1): each class in up to k chunks; k_lpc runs the chunks in order
     * on the side stream and k_resid of chunk i (on s) waits only for k_lpc of chunk i, so
     * the f64 autocorrelation of chunk i+1 shares the GPU with the integer/MFMA work of
     * chunk i. */
    struct Chunk {
        int64_t unit0, count;
        int n;
    } ch[flacmi_ctx::kMaxChunks];
    auto lpc_params_for = [&](int n) {
        LpcArgs a{};
        a.stride = b->unit_stride;
        a.sample_bytes = b->sample_bytes;
        a.n = n;
        a.L = L;
        return a;
    };
    int nch = 0;
    const int ov = lpc ? overlap_mode() : 0;
    const int want = ov > 1 ? ov : 1;
    bool overlap = want > 1 && b->n_units >= 2 * kOverlapMinUnits;
    for (int c = 0; c < ncls; ++c) {
        if (ov < -1 || (ov == -1 && cls[c].count >= 2 * kOverlapMinUnits)) {
            /* round-aligned: the units of k_lpc's whole rounds, then the remainder, whose
             * k_lpc fills the last round's idle slots beside k_resid of the first chunk */
            const int64_t R = ov < -1 ? -(int64_t)ov : lpc_units_per_round(lpc_params_for(cls[c].n));
            const int64_t whole = R > 0 ? cls[c].count / R * R : 0, rest = cls[c].count - whole;
            if (whole > 0 && rest > 0 && (ov < -1 || rest >= kOverlapMinUnits) &&
                nch + 2 + (ncls - 1 - c) <= flacmi_ctx::kMaxChunks) {
                ch[nch++] = {cls[c].unit0, whole, cls[c].n};
                ch[nch++] = {cls[c].unit0 + whole, rest, cls[c].n};
                overlap = true;
                continue;
            }
        }
        int64_t k = overlap && ov > 1 ? cls[c].count / kOverlapMinUnits : 1;
        const int left = flacmi_ctx::kMaxChunks - nch - (ncls - 1 - c);
        k = k < 1 ? 1 : k > want ? want : k;
        k = k > left ? left : k;
        for (int64_t i = 0; i < k; ++i) {
            const int64_t u0 = cls[c].count * i / k, u1 = cls[c].count * (i + 1) / k;
            ch[nch++] = {cls[c].unit0 + u0, u1 - u0, cls[c].n};
        }
    }
    auto lpc_args = [&](const Chunk& k, LpcArgs& a) -> int {
        a = LpcArgs{};
        a.samples = b->samples;
        a.stride = b->unit_stride;
        a.unit0 = k.unit0;
        a.count = k.count;
        a.sample_bytes = b->sample_bytes;
        a.n = k.n;
        a.L = L;
        a.q = p->qlp_precision;
        if (int rc = get_window(ctx, k.n, (double**)&a.window, &a.fuse_lo, &a.fuse_hi)) return rc;
        if (b->sample_bits > 26) a.fuse_lo = a.fuse_hi = 0; /* products must stay below 2^52 */
        a.log2thr = ctx->d_log2thr;
        a.rec = (int32_t*)ctx->rec.p + k.unit0 * rec_words;
        a.rec_words = rec_words;
        a.acf = o->acf ? o->acf + k.unit0 * 33 : nullptr;
        return 0;
    };
    auto launch_resid_chunk = [&](const Chunk& k, hipStream_t st) -> hipError_t {
        ResidArgs a{};
        a.samples = b->samples;
        a.stride = b->unit_stride;
        a.unit0 = k.unit0;
        a.count = k.count;
        a.sample_bytes = b->sample_bytes;
        a.n = k.n;
        a.L = L;
        a.mode = p->mode;
        a.rmin = p->rice_min;
        a.rmax = p->rice_max;
        a.rec = lpc ? (const int32_t*)ctx->rec.p + k.unit0 * rec_words : nullptr;
        a.rice_order = p->mode == FLACMI_MODE_RICE_ONLY ? p->reserved[0] : 0;
        a.rec_words = rec_words;
        a.log2thr = ctx->d_log2thr;
        a.meta = o->meta + k.unit0;
        a.rice_params = o->rice_params + k.unit0 * o->params_stride;
        a.params_stride = o->params_stride;
        a.residual = (char*)o->residual + (size_t)k.unit0 * o->residual_stride * o->residual_bytes;
        a.residual_stride = o->residual_stride;
        a.fixed_sums = o->fixed_sums ? o->fixed_sums + k.unit0 * 5 : nullptr;
        a.lpc_sums = o->lpc_sums ? o->lpc_sums + k.unit0 * 32 : nullptr;
        a.stop_after = debug_stop();
        a.mfma = use_mfma();
        int64_t* const rb = (int64_t*)ctx->retry.p;
        a.retry_sub = (unsigned long long*)rb;
        a.retry_count = (unsigned long long*)(rb + kSubWords);
        a.retry_list = rb + kSubWords + 2;
        a.retry2_count = (unsigned long long*)(rb + kSubWords + 2 + b->n_units + 64);
        a.retry2_list = rb + kSubWords + 4 + b->n_units + 64;
        a.sample_bits = b->sample_bits;
        a.stream = use_stream();
        a.prune = p->mode == FLACMI_MODE_REFERENCE && !o->lpc_sums && !(p->reserved[1] & FLACMI_FLAG_ALL_CANDIDATES) &&
                  prune_allowed();
        a.sign_bound = !(p->reserved[1] & FLACMI_FLAG_TIERS_ONLY) && sign_bound_allowed();
        const bool wide = needs_wide(k.n, b->sample_bits, L, p->qlp_precision, p->mode);
        int path = (wide || o->residual_bytes == 8) ? 2 : (b->sample_bytes == 2 && p->qlp_precision <= 16) ? 0 : 1;
        if (path == 2 && o->residual_bytes == 4 && split_ok(b->sample_bits, L, p->qlp_precision)) path = 3;
        return launch_resid(a, path, o->residual_bytes, st);
    };
    const int slot = ctx->ncalls % flacmi_ctx::kRing;
    hipEvent_t* ev = ctx->ev[slot];
    hipStream_t side = nullptr;
    if (overlap && !allow_overlap) overlap = false;
    if (overlap) {
        /* k_lpc runs on the pipeline's H2D stream, which lives as long as the context: a
         * stream created here would have to be destroyed before returning, and destroying a
         * stream with queued work waits for it (the call would block the host).  A stream
         * left open instead takes a hardware queue that the pipeline's copies then share
         * (measured: the 1e5-unit host-to-host encode 20.4 -> 38.5 ms wall). */
        if (int rc = enc_streams(ctx)) return rc;
        side = enc_side(ctx);
        if (side == s) overlap = false;
    }
    ctx->nchunks[slot] = overlap ? nch : 0;
    HIP_TRY(hipEventRecord(ev[0], s));
    if (overlap) {
        HIP_TRY(hipStreamWaitEvent(side, ev[0], 0));
        for (int i = 0; i < nch; ++i) {
            LpcArgs a;
            if (int rc = lpc_args(ch[i], a)) return rc;
            HIP_TRY(launch_lpc(a, side));
            HIP_TRY(hipEventRecord(ctx->lpc_done[i], side));
        }
        HIP_TRY(hipEventRecord(ev[1], side));
        for (int i = 0; i < nch; ++i) {
            HIP_TRY(hipStreamWaitEvent(s, ctx->lpc_done[i], 0));
            HIP_TRY(hipEventRecord(ev[3 + 2 * i], s));
            HIP_TRY(launch_resid_chunk(ch[i], s));
            HIP_TRY(hipEventRecord(ev[4 + 2 * i], s));
        }
    } else {
        for (int i = 0; i < nch && lpc; ++i) {
            LpcArgs a;
            if (int rc = lpc_args(ch[i], a)) return rc;
            HIP_TRY(launch_lpc(a, s));
        }
        HIP_TRY(hipEventRecord(ev[1], s));
        for (int i = 0; i < nch; ++i) HIP_TRY(launch_resid_chunk(ch[i], s));
    }
    HIP_TRY(hipEventRecord(ev[2], s));
    ctx->ncalls++;
    if (o->lpc_records) {
        if (lpc) {
            HIP_TRY(launch_expand_records((const int32_t*)ctx->rec.p, rec_words, L, b->n_units, o->lpc_records, s));
        } else {
            HIP_TRY(hipMemsetAsync(o->lpc_records, 0, sizeof(int32_t) * FLACMI_LPC_REC_WORDS(32) * b->n_units, s));
        }
    }
    return 0;
}

extern "C" {

int flacmi_analyze_device(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                          const flacmi_outputs* out, void* stream) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    if (int rc = validate(batch, params, out)) return rc;
    if (batch->n_units == 0) return 0;
    return analyze_device_impl(ctx, batch, params, out, (hipStream_t)stream);
}

int flacmi_analyze_host(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                        const flacmi_outputs* out) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    if (!batch || !params || !out) return fail(FLACMI_E_INVALID, "null argument");
    if (batch->n_units == 0) return 0;
    if (int rc = set_device(ctx)) return rc;
    const size_t nu = (size_t)batch->n_units;
    /* device mirrors with 16-byte aligned rows */
    const int64_t sstride = row_pitch(batch->block_len, batch->sample_bytes);
    const int64_t rstride = ((batch->block_len * out->residual_bytes + 15) / 16) * 16 / out->residual_bytes;
    if (int rc = ensure_buf(ctx->h_samples, nu * sstride * batch->sample_bytes)) return rc;
    if (int rc = ensure_buf(ctx->h_meta, nu * sizeof(flacmi_unit_meta))) return rc;
    if (int rc = ensure_buf(ctx->h_params, nu * out->params_stride * sizeof(int32_t))) return rc;
    if (int rc = ensure_buf(ctx->h_residual, nu * rstride * out->residual_bytes)) return rc;
    flacmi_batch db = *batch;
    db.samples = ctx->h_samples.p;
    db.unit_stride = sstride;
    HIP_TRY(hipMemcpy2DAsync(ctx->h_samples.p, sstride * batch->sample_bytes, batch->samples,
                             batch->unit_stride * batch->sample_bytes, batch->block_len * batch->sample_bytes, nu,
                             hipMemcpyHostToDevice, ctx->stream));
    flacmi_outputs dout = *out;
    dout.meta = (flacmi_unit_meta*)ctx->h_meta.p;
    dout.rice_params = (int32_t*)ctx->h_params.p;
    dout.residual = ctx->h_residual.p;
    dout.residual_stride = rstride;
    if (out->acf) {
        if (int rc = ensure_buf(ctx->h_acf, nu * 33 * sizeof(double))) return rc;
        dout.acf = (double*)ctx->h_acf.p;
    }
    if (out->fixed_sums) {
        if (int rc = ensure_buf(ctx->h_fs, nu * 5 * sizeof(int64_t))) return rc;
        dout.fixed_sums = (int64_t*)ctx->h_fs.p;
    }
    if (out->lpc_sums) {
        if (int rc = ensure_buf(ctx->h_ls, nu * 32 * sizeof(int64_t))) return rc;
        dout.lpc_sums = (int64_t*)ctx->h_ls.p;
    }
    if (out->lpc_records) {
        if (int rc = ensure_buf(ctx->h_recs, nu * FLACMI_LPC_REC_WORDS(32) * sizeof(int32_t))) return rc;
        dout.lpc_records = (int32_t*)ctx->h_recs.p;
    }
    if (int rc = validate(&db, params, &dout)) return rc;
    if (int rc = analyze_device_impl(ctx, &db, params, &dout, ctx->stream)) return rc;
    HIP_TRY(hipMemcpyAsync(out->meta, dout.meta, nu * sizeof(flacmi_unit_meta), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(out->rice_params, dout.rice_params, nu * out->params_stride * sizeof(int32_t),
                           hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpy2DAsync(out->residual, out->residual_stride * out->residual_bytes, dout.residual,
                             rstride * out->residual_bytes, batch->block_len * out->residual_bytes, nu,
                             hipMemcpyDeviceToHost, ctx->stream));
    if (out->acf)
        HIP_TRY(hipMemcpyAsync(out->acf, dout.acf, nu * 33 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (out->fixed_sums)
        HIP_TRY(hipMemcpyAsync(out->fixed_sums, dout.fixed_sums, nu * 5 * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    if (out->lpc_sums)
        HIP_TRY(hipMemcpyAsync(out->lpc_sums, dout.lpc_sums, nu * 32 * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    if (out->lpc_records)
        HIP_TRY(hipMemcpyAsync(out->lpc_records, dout.lpc_records, nu * FLACMI_LPC_REC_WORDS(32) * sizeof(int32_t),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"

/* ---- frame writer ---------------------------------------------------------------- */
static int validate_frames(const flacmi_batch* b, const flacmi_frame_params* fp, int64_t* n_frames) {
    if (!b || !fp) return fail(FLACMI_E_INVALID, "null argument");
    if (fp->channels < 1 || fp->channels > 8) return fail(FLACMI_E_INVALID, "channels must be 1..8");
    if (fp->sample_size < 1 || fp->sample_size > 32) return fail(FLACMI_E_INVALID, "sample_size must be 1..32");
    if (fp->qlp_precision < 5 || fp->qlp_precision > 31) return fail(FLACMI_E_INVALID, "qlp_precision must be 5..31");
    if (fp->first_frame < 0) return fail(FLACMI_E_INVALID, "first_frame must be >= 0");
    if (b->n_units % fp->channels != 0) return fail(FLACMI_E_INVALID, "n_units must be a multiple of channels");
    if (b->n_tail_units != 0 && b->n_tail_units != fp->channels)
        return fail(FLACMI_E_INVALID, "the short last frame must hold exactly `channels` tail units");
    if (b->block_len < 1 || b->block_len > FLACMI_MAX_BLOCK) return fail(FLACMI_E_INVALID, "block_len out of range");
    *n_frames = b->n_units / fp->channels;
    return 0;
}

static FrameArgs frame_args(flacmi_ctx* ctx, const flacmi_batch* b, const flacmi_frame_params* fp,
                            const flacmi_unit_meta* meta, const int32_t* rice_params, int64_t params_stride,
                            int64_t n_frames) {
    FrameArgs a{};
    a.samples = b->samples;
    a.stride = b->unit_stride;
    a.sample_bytes = b->sample_bytes;
    a.block_len = b->block_len;
    a.tail_len = b->n_tail_units ? b->tail_len : b->block_len;
    a.n_units = b->n_units;
    a.n_tail_units = b->n_tail_units;
    a.channels = fp->channels;
    a.sample_size = fp->sample_size;
    a.q = fp->qlp_precision;
    a.first_frame = fp->first_frame;
    a.n_frames = n_frames;
    a.meta = meta;
    a.rice_params = rice_params;
    a.params_stride = params_stride;
    a.crc_slice = ctx->d_crc;
    a.crc_pow = ctx->d_crc + 4 * 256;
    return a;
}

/* the k_pack32 -> k_pack hand-off list (count word + one index per frame) */
static int pack_lists(flacmi_ctx* ctx, FrameArgs& a) {
    if (int rc = ensure_buf(ctx->slow, sizeof(int64_t) * (size_t)(a.n_frames + 2))) return rc;
    a.slow_count = (unsigned long long*)ctx->slow.p;
    a.slow_list = (int64_t*)ctx->slow.p + 2;
    return 0;
}

static int frame_sizes_impl(flacmi_ctx* ctx, FrameArgs& a, int64_t* offsets, int32_t* status, hipStream_t s) {
    a.offsets = offsets;
    a.status = status;
    if (int rc = ensure_buf(ctx->scan, sizeof(int64_t) * (size_t)(frame_scan_blocks(a.n_frames) + 1))) return rc;
    HIP_TRY(launch_frame_sizes(a, (int64_t*)ctx->scan.p, s));
    return 0;
}

extern "C" {

int flacmi_frame_sizes_device(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_frame_params* fp,
                              const flacmi_unit_meta* meta, const int32_t* rice_params, int64_t params_stride,
                              int64_t* frame_offsets, int32_t* frame_status, void* stream) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    int64_t nf = 0;
    if (int rc = validate_frames(batch, fp, &nf)) return rc;
    if (!meta || !rice_params || !frame_offsets || !frame_status) return fail(FLACMI_E_INVALID, "null buffer");
    if (int rc = set_device(ctx)) return rc;
    if (nf == 0) {
        HIP_TRY(hipMemsetAsync(frame_offsets, 0, sizeof(int64_t), (hipStream_t)stream));
        return 0;
    }
    FrameArgs a = frame_args(ctx, batch, fp, meta, rice_params, params_stride, nf);
    return frame_sizes_impl(ctx, a, frame_offsets, frame_status, (hipStream_t)stream);
}

int flacmi_pack_frames_device(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_frame_params* fp,
                              const flacmi_unit_meta* meta, const int32_t* rice_params, int64_t params_stride,
                              const void* residual, int32_t residual_bytes, int64_t residual_stride,
                              const int64_t* frame_offsets, int32_t* frame_status, uint8_t* out,
                              int64_t out_capacity, void* stream) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    int64_t nf = 0;
    if (int rc = validate_frames(batch, fp, &nf)) return rc;
    if (!meta || !rice_params || !residual || !frame_offsets || !frame_status || (!out && out_capacity > 0))
        return fail(FLACMI_E_INVALID, "null buffer");
    if (residual_bytes != 4 && residual_bytes != 8) return fail(FLACMI_E_INVALID, "residual_bytes must be 4 or 8");
    if (residual_stride < batch->block_len) return fail(FLACMI_E_INVALID, "residual_stride < block_len");
    if (((uintptr_t)out & 3) != 0) return fail(FLACMI_E_INVALID, "out must be 4-byte aligned");
    if (nf == 0) return 0;
    if (int rc = set_device(ctx)) return rc;
    FrameArgs a = frame_args(ctx, batch, fp, meta, rice_params, params_stride, nf);
    a.residual = residual;
    a.residual_bytes = residual_bytes;
    a.residual_stride = residual_stride;
    a.offsets = const_cast<int64_t*>(frame_offsets);
    a.status = frame_status;
    a.out = out;
    a.capacity = out_capacity;
    if (int rc = pack_lists(ctx, a)) return rc;
    HIP_TRY(launch_pack(a, (hipStream_t)stream));
    return 0;
}

int flacmi_decode_frames_device(flacmi_ctx* ctx, const uint8_t* stream_data, int64_t stream_bytes,
                                const int64_t* frame_offsets, int64_t n_frames,
                                const flacmi_decode_params* dp, const flacmi_batch* expect,
                                int32_t* samples_out, int64_t out_stride, int32_t* frame_status,
                                int64_t* frame_mismatch, void* stream) {
    if (!ctx || !dp) return fail(FLACMI_E_INVALID, "null argument");
    if (n_frames < 0 || stream_bytes < 0) return fail(FLACMI_E_INVALID, "negative size");
    if (n_frames == 0) return 0;
    if (!stream_data || !frame_offsets || !frame_status || !frame_mismatch) return fail(FLACMI_E_INVALID, "null buffer");
    if (((uintptr_t)stream_data & 3) != 0) return fail(FLACMI_E_INVALID, "stream_data must be 4-byte aligned");
    if (dp->channels < 1 || dp->channels > 8) return fail(FLACMI_E_INVALID, "channels must be 1..8");
    if (dp->sample_size < 4 || dp->sample_size > 32) return fail(FLACMI_E_INVALID, "sample_size must be 4..32");
    if (samples_out && (out_stride < 1 || (out_stride & 3) != 0 || ((uintptr_t)samples_out & 15) != 0))
        return fail(FLACMI_E_INVALID, "samples_out rows must be 16-byte aligned (out_stride a multiple of 4)");
    if (expect) {
        if (expect->sample_bytes != 2 && expect->sample_bytes != 4) return fail(FLACMI_E_INVALID, "expect: sample_bytes 2 or 4");
        if (expect->n_units != n_frames * dp->channels) return fail(FLACMI_E_INVALID, "expect: n_units != n_frames * channels");
        if (expect->unit_stride < expect->block_len) return fail(FLACMI_E_INVALID, "expect: unit_stride < block_len");
        if (expect->n_tail_units && expect->tail_len > expect->block_len) return fail(FLACMI_E_INVALID, "expect: tail_len > block_len");
    }
    if (int rc = set_device(ctx)) return rc;
    /* workspace: decorr codes [n_frames] i32, then two deferred-frame lists (an 8 B count and
     * [n_frames] i64 each) */
    const size_t dlist = (sizeof(int32_t) * (size_t)n_frames + 15) & ~(size_t)15;
    const size_t dl2 = dlist + 16 + sizeof(int64_t) * (size_t)n_frames; /* the second list */
    if (int rc = ensure_buf(ctx->dec, dl2 + 16 + sizeof(int64_t) * (size_t)n_frames)) return rc;
    DecodeArgs a{};
    a.words = reinterpret_cast<const uint32_t*>(stream_data);
    a.stream_bytes = stream_bytes;
    a.n_words = (stream_bytes + 3) / 4;
    a.offsets = frame_offsets;
    a.n_frames = n_frames;
    a.channels = dp->channels;
    a.sample_size = dp->sample_size;
    a.first_frame = dp->first_frame;
    a.check_crc = dp->check_crc;
    if (expect) {
        a.expect = expect->samples;
        a.expect_stride = expect->unit_stride;
        a.expect_bytes = expect->sample_bytes;
        a.expect_vec = ((uintptr_t)expect->samples & 15) == 0 && ((expect->unit_stride * expect->sample_bytes) & 15) == 0;
        a.block_len = expect->block_len;
        a.tail_len = expect->n_tail_units ? expect->tail_len : expect->block_len;
        a.n_units = expect->n_units;
        a.n_tail_units = expect->n_tail_units;
    }
    a.out = samples_out;
    a.out_stride = out_stride;
    a.status = frame_status;
    a.mismatch = frame_mismatch;
    a.decorr = (int32_t*)ctx->dec.p;
    a.defer_count = (unsigned long long*)((char*)ctx->dec.p + dlist);
    a.defer_list = (int64_t*)((char*)ctx->dec.p + dlist + 16);
    a.defer2_count = (unsigned long long*)((char*)ctx->dec.p + dl2);
    a.defer2_list = (int64_t*)((char*)ctx->dec.p + dl2 + 16);
    a.defer_all = knob(kKnobDecodeGeneric) != 0;
    a.crc_slice = ctx->d_crc;
    HIP_TRY(launch_decode(a, (hipStream_t)stream));
    return 0;
}

int flacmi_encode_host(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                       const flacmi_frame_params* fp, int64_t* frame_offsets, int32_t* frame_status) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    int64_t nf = 0;
    if (int rc = validate_frames(batch, fp, &nf)) return rc;
    if (!params || !frame_offsets || !frame_status) return fail(FLACMI_E_INVALID, "null argument");
    ctx->frames_bytes = 0;
    if (nf == 0) {
        frame_offsets[0] = 0;
        return 0;
    }
    if (int rc = set_device(ctx)) return rc;
    const size_t nu = (size_t)batch->n_units;
    const int64_t sstride = row_pitch(batch->block_len, batch->sample_bytes);
    const int64_t pstride = (1LL << (params->rice_max > 0 ? params->rice_max : 0)) + 1;
    if (int rc = ensure_buf(ctx->h_samples, nu * sstride * batch->sample_bytes)) return rc;
    if (int rc = ensure_buf(ctx->h_meta, nu * sizeof(flacmi_unit_meta))) return rc;
    if (int rc = ensure_buf(ctx->h_params, nu * pstride * sizeof(int32_t))) return rc;
    if (int rc = ensure_buf(ctx->h_offsets, sizeof(int64_t) * (size_t)(nf + 1))) return rc;
    if (int rc = ensure_buf(ctx->h_status, sizeof(int32_t) * (size_t)nf)) return rc;
    flacmi_batch db = *batch;
    db.samples = ctx->h_samples.p;
    db.unit_stride = sstride;
    HIP_TRY(hipMemcpy2DAsync(ctx->h_samples.p, sstride * batch->sample_bytes, batch->samples,
                             batch->unit_stride * batch->sample_bytes, batch->block_len * batch->sample_bytes, nu,
                             hipMemcpyHostToDevice, ctx->stream));
    for (int rbytes = 4;; rbytes = 8) {
        const int64_t rstride = ((batch->block_len * rbytes + 15) / 16) * 16 / rbytes;
        if (int rc = ensure_buf(ctx->h_residual, nu * rstride * rbytes)) return rc;
        flacmi_outputs o{};
        o.meta = (flacmi_unit_meta*)ctx->h_meta.p;
        o.rice_params = (int32_t*)ctx->h_params.p;
        o.params_stride = pstride;
        o.residual = ctx->h_residual.p;
        o.residual_bytes = rbytes;
        o.residual_stride = rstride;
        if (int rc = validate(&db, params, &o)) return rc;
        if (int rc = analyze_device_impl(ctx, &db, params, &o, ctx->stream)) return rc;
        FrameArgs a = frame_args(ctx, &db, fp, o.meta, o.rice_params, pstride, nf);
        if (int rc = frame_sizes_impl(ctx, a, (int64_t*)ctx->h_offsets.p, (int32_t*)ctx->h_status.p, ctx->stream))
            return rc;
        HIP_TRY(hipMemcpyAsync(frame_offsets, ctx->h_offsets.p, sizeof(int64_t) * (nf + 1), hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipMemcpyAsync(frame_status, ctx->h_status.p, sizeof(int32_t) * nf, hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        bool wide = false;
        for (int64_t f = 0; f < nf && rbytes == 4; ++f)
            if ((frame_status[f] & 0xffff) == FLACMI_STATUS_RESIDUAL_WIDE) wide = true;
        if (wide) continue; /* a chosen residual needs 64 bits: redo with 8-byte rows */
        const int64_t total = frame_offsets[nf];
        if (int rc = ensure_buf(ctx->h_frames, (size_t)total + 16)) return rc;
        a.residual = ctx->h_residual.p;
        a.residual_bytes = rbytes;
        a.residual_stride = rstride;
        a.offsets = (int64_t*)ctx->h_offsets.p;
        a.status = (int32_t*)ctx->h_status.p;
        a.out = (uint8_t*)ctx->h_frames.p;
        a.capacity = total;
        if (int rc = pack_lists(ctx, a)) return rc;
        HIP_TRY(launch_pack(a, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->frames_bytes = total;
        return 0;
    }
}

/* ---- pipelined host encode ---------------------------------------------------------
 * Streams: `cs` = the context's stream (compute: analysis, sizes, k_export of the offsets /
 * status into mapped host memory, pack, in order, so the context's shared scratch is never used by two launches
 * at once), `is`
 * (host -> device samples) and `os` (device -> host frame bytes).  Per sub-batch k (slot
 * k % kEncSlots):
 *   front(k): is: H2D rows -> cs: analyze, frame sizes, k_export (offsets/status to host)
 *   back(k):  host waits for those offsets, then cs: pack -> os: frame bytes D2H into out
 * issued as front(0), front(1), back(0), front(2), back(1), ... so the copies of one
 * sub-batch run under the kernels of the others.  The offsets of k are written by a kernel
 * into mapped host memory: as a DMA copy they queued behind the frame bytes of k - 1 and
 * the host waited for that copy before issuing the next H2D (the two copy directions then
 * ran back to back).
 * Streams, events, slot buffers and the pinned offset arrays live in the context and grow
 * as needed (ensure_buf), so streaming many calls pays no setup. */
namespace {
constexpr int kEncSlots = 4; /* with 3 the host waited for the D2H of sub-batch k - 3 before issuing the H2D of k */
struct EncSlot {
    DevBuf samples, meta, params, residual, offsets, status, frames;
    int64_t* h_off = nullptr;   /* pinned, mapped: frame offsets of the sub-batch */
    int32_t* h_st = nullptr;    /* pinned, mapped: frame status */
    int64_t* d_off = nullptr;   /* their device-side addresses (k_export writes them) */
    int32_t* d_st = nullptr;
    hipEvent_t e[9] = {};       /* h2d start/end, analyze end, sizes end, pack start/end, d2h start/end, offsets copied */
    flacmi_batch b{};
    int64_t first_unit = 0, nf = 0, total = 0, dstride = 0;
    int rbytes = 4;
};
float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.0f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.0f;
}
}  // namespace

struct EncState {
    hipStream_t is = nullptr, os = nullptr; /* compute runs on the context's stream */
    EncSlot slot[kEncSlots];
    int64_t cap_nf = 0; /* frames the pinned arrays of each slot hold */
};

static hipStream_t enc_side(flacmi_ctx* ctx) { return ctx->enc ? ctx->enc->is : nullptr; }

static void enc_free(EncState* es) {
    if (!es) return;
    for (hipStream_t st : {es->is, es->os})
        if (st) (void)hipStreamSynchronize(st);
    for (auto& sl : es->slot) {
        for (DevBuf* d : {&sl.samples, &sl.meta, &sl.params, &sl.residual, &sl.offsets, &sl.status, &sl.frames})
            if (d->p) (void)hipFree(d->p);
        if (sl.h_off) (void)hipHostFree(sl.h_off);
        if (sl.h_st) (void)hipHostFree(sl.h_st);
        for (auto& e : sl.e)
            if (e) (void)hipEventDestroy(e);
    }
    for (hipStream_t st : {es->is, es->os})
        if (st) (void)hipStreamDestroy(st);
    delete es;
}

/* The pipeline's streams, created on first use and kept for the context's lifetime.  The
 * overlap mode of analyze_device_impl borrows `is` for its k_lpc launches, so no call creates
 * or destroys a stream of its own (a process holds GPU_MAX_HW_QUEUES hardware queues). */
static int enc_streams(flacmi_ctx* ctx) {
    if (!ctx->enc) {
        /* built whole before it is published: a failed create leaves no half state behind */
        EncState* es = new EncState();
        hipError_t e = hipStreamCreateWithFlags(&es->is, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&es->os, hipStreamNonBlocking);
        for (auto& sl : es->slot)
            for (auto& ev : sl.e)
                if (e == hipSuccess) e = hipEventCreate(&ev);
        if (e != hipSuccess) {
            enc_free(es);
            return fail(FLACMI_E_HIP, "encode pipeline state: %s", hipGetErrorString(e));
        }
        ctx->enc = es;
    }
    return 0;
}

static int enc_state(flacmi_ctx* ctx, int64_t per_nf, EncState** out) {
    if (int rc = enc_streams(ctx)) return rc;
    EncState* es = ctx->enc;
    if (es->cap_nf < per_nf) {
        for (auto& sl : es->slot) {
            if (sl.h_off) HIP_TRY(hipHostFree(sl.h_off));
            if (sl.h_st) HIP_TRY(hipHostFree(sl.h_st));
            sl.h_off = nullptr;
            sl.h_st = nullptr;
        }
        es->cap_nf = 0;
        for (auto& sl : es->slot) {
            HIP_TRY(hipHostMalloc((void**)&sl.h_off, sizeof(int64_t) * (per_nf + 1), hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostMalloc((void**)&sl.h_st, sizeof(int32_t) * per_nf, hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void**)&sl.d_off, sl.h_off, 0));
            HIP_TRY(hipHostGetDevicePointer((void**)&sl.d_st, sl.h_st, 0));
        }
        es->cap_nf = per_nf;
    }
    *out = es;
    return 0;
}

static int enc_front(flacmi_ctx* ctx, EncSlot& sl, const flacmi_batch* whole, const flacmi_params* params,
                     const flacmi_frame_params* fp, hipStream_t cs, hipStream_t is) {
    const flacmi_batch& b = sl.b;
    const size_t nu = (size_t)b.n_units;
    /* rows already at the padded device stride go as one linear copy; any other stride (a
       row view of a wider array) is packed to padded device rows by a 2-D copy */
    const int64_t padded = row_pitch(b.block_len, b.sample_bytes);
    const bool linear = whole->unit_stride == padded;
    sl.dstride = padded;
    const int64_t sstride = sl.dstride;
    const int64_t pstride = (1LL << (params->rice_max > 0 ? params->rice_max : 0)) + 1;
    const int64_t rstride = ((b.block_len * sl.rbytes + 15) / 16) * 16 / sl.rbytes;
    if (int rc = ensure_buf(sl.samples, nu * sstride * b.sample_bytes)) return rc;
    if (int rc = ensure_buf(sl.meta, nu * sizeof(flacmi_unit_meta))) return rc;
    if (int rc = ensure_buf(sl.params, nu * pstride * sizeof(int32_t))) return rc;
    if (int rc = ensure_buf(sl.residual, nu * rstride * sl.rbytes)) return rc;
    if (int rc = ensure_buf(sl.offsets, sizeof(int64_t) * (size_t)(sl.nf + 1))) return rc;
    if (int rc = ensure_buf(sl.status, sizeof(int32_t) * (size_t)sl.nf)) return rc;
    const uint8_t* src = (const uint8_t*)whole->samples + sl.first_unit * whole->unit_stride * b.sample_bytes;
    HIP_TRY(hipEventRecord(sl.e[0], is));
    if (linear)
        HIP_TRY(hipMemcpyAsync(sl.samples.p, src, ((nu - 1) * sstride + b.block_len) * b.sample_bytes,
                               hipMemcpyHostToDevice, is));
    else
        HIP_TRY(hipMemcpy2DAsync(sl.samples.p, sstride * b.sample_bytes, src, whole->unit_stride * b.sample_bytes,
                                 b.block_len * b.sample_bytes, nu, hipMemcpyHostToDevice, is));
    HIP_TRY(hipEventRecord(sl.e[1], is));
    HIP_TRY(hipStreamWaitEvent(cs, sl.e[1], 0));
    flacmi_batch db = b;
    db.samples = sl.samples.p;
    db.unit_stride = sstride;
    flacmi_outputs o{};
    o.meta = (flacmi_unit_meta*)sl.meta.p;
    o.rice_params = (int32_t*)sl.params.p;
    o.params_stride = pstride;
    o.residual = sl.residual.p;
    o.residual_bytes = sl.rbytes;
    o.residual_stride = rstride;
    if (int rc = validate(&db, params, &o)) return rc;
    /* no chunk overlap inside the pipeline: its side stream is this pipeline's H2D stream,
       and the next sub-batch's copy would queue behind this one's k_lpc */
    if (int rc = analyze_device_impl(ctx, &db, params, &o, cs, false)) return rc;
    HIP_TRY(hipEventRecord(sl.e[2], cs));
    flacmi_frame_params f = *fp;
    f.first_frame = fp->first_frame + sl.first_unit / fp->channels;
    FrameArgs a = frame_args(ctx, &db, &f, o.meta, o.rice_params, pstride, sl.nf);
    if (int rc = frame_sizes_impl(ctx, a, (int64_t*)sl.offsets.p, (int32_t*)sl.status.p, cs)) return rc;
    HIP_TRY(hipEventRecord(sl.e[3], cs));
    HIP_TRY(launch_export((const int64_t*)sl.offsets.p, (const int32_t*)sl.status.p, sl.nf, sl.d_off, sl.d_st, cs));
    HIP_TRY(hipEventRecord(sl.e[8], cs));
    return 0;
}

extern "C" int flacmi_host_register(flacmi_ctx* ctx, void* ptr, size_t bytes) {
    if (!ctx || !ptr || bytes == 0) return fail(FLACMI_E_INVALID, "null context, pointer or empty range");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return 0;
}

extern "C" int flacmi_host_unregister(flacmi_ctx* ctx, void* ptr) {
    if (!ctx || !ptr) return fail(FLACMI_E_INVALID, "null context or pointer");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipHostUnregister(ptr));
    return 0;
}

extern "C" void* flacmi_host_alloc(flacmi_ctx* ctx, size_t bytes) {
    if (!ctx || bytes == 0) {
        fail(FLACMI_E_INVALID, "null context or empty range");
        return nullptr;
    }
    if (set_device(ctx)) return nullptr;
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        fail(FLACMI_E_NOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

extern "C" int flacmi_host_free(flacmi_ctx* ctx, void* ptr) {
    if (!ptr) return 0;
    if (ctx)
        if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipHostFree(ptr));
    return 0;
}

extern "C" int flacmi_encode_pipeline(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                                      const flacmi_frame_params* fp, int64_t units_per_batch, uint8_t* out,
                                      int64_t out_capacity, int64_t* frame_offsets, int32_t* frame_status,
                                      flacmi_encode_timing* timing) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    int64_t nf = 0;
    if (int rc = validate_frames(batch, fp, &nf)) return rc;
    if (!params || !frame_offsets || !frame_status || (!out && out_capacity > 0))
        return fail(FLACMI_E_INVALID, "null argument");
    const int C = fp->channels;
    if (units_per_batch < C || units_per_batch % C) return fail(FLACMI_E_INVALID, "units_per_batch must be a positive multiple of channels");
    if (batch->unit_stride < batch->block_len) return fail(FLACMI_E_INVALID, "unit_stride < block_len");
    flacmi_encode_timing t{};
    const auto w0 = std::chrono::steady_clock::now();
    frame_offsets[0] = 0;
    if (nf == 0) {
        if (timing) *timing = t;
        return 0;
    }
    if (int rc = set_device(ctx)) return rc;
    units_per_batch = std::min(units_per_batch, ((batch->n_units + C - 1) / C) * C);
    EncState* es = nullptr;
    if (int rc = enc_state(ctx, units_per_batch / C, &es)) return rc;
    /* the caller's rows and output, page-locked in place for the call */
    const auto r0 = std::chrono::steady_clock::now();
    const size_t in_bytes = (size_t)((batch->n_units - 1) * batch->unit_stride + batch->block_len) * batch->sample_bytes;
    /* a buffer already page-locked (flacmi_host_register, flacmi_host_alloc) is used as it is */
    auto locked = [](const void* q) {
        hipPointerAttribute_t at{};
        const bool y = hipPointerGetAttributes(&at, q) == hipSuccess && at.type == hipMemoryTypeHost;
        (void)hipGetLastError();
        return y;
    };
    const bool reg_in = !locked(batch->samples) &&
                        hipHostRegister(const_cast<void*>(batch->samples), in_bytes, hipHostRegisterDefault) == hipSuccess;
    const bool reg_out = out_capacity > 0 && !locked(out) &&
                         hipHostRegister(out, (size_t)out_capacity, hipHostRegisterDefault) == hipSuccess;
    (void)hipGetLastError();
    t.register_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count();
    /* three streams in all (with the null stream four: GPU_MAX_HW_QUEUES' default).  With a
     * fifth the runtime maps two streams onto one hardware queue, and the copies of the two
     * directions then wait for each other in submission order (measured: H2D of sub-batch
     * k + 2 started only when the D2H of k had finished). */
    hipStream_t cs = ctx->stream, is = es->is, os = es->os;
    EncSlot* slot = es->slot;
    int rc = 0;
    {
        const int64_t nsub = (batch->n_units + units_per_batch - 1) / units_per_batch;
        auto setup = [&](int64_t k) {
            EncSlot& sl = slot[k % kEncSlots];
            sl.first_unit = k * units_per_batch;
            const int64_t nu = std::min(units_per_batch, batch->n_units - sl.first_unit);
            sl.b = *batch;
            sl.b.n_units = nu;
            sl.b.n_tail_units = (sl.first_unit + nu == batch->n_units) ? batch->n_tail_units : 0;
            sl.nf = nu / C;
            sl.rbytes = 4;
        };
        int64_t written = 0; /* frame bytes of the sub-batches already placed */
        auto back = [&](int64_t k) -> int {
            EncSlot& sl = slot[k % kEncSlots];
            HIP_TRY(hipEventSynchronize(sl.e[8])); /* the offsets / status of sub-batch k */
            bool wide = false;
            for (int64_t f = 0; f < sl.nf && sl.rbytes == 4; ++f)
                if ((sl.h_st[f] & 0xffff) == FLACMI_STATUS_RESIDUAL_WIDE) wide = true;
            if (wide) { /* a chosen residual needs 64 bits: redo this sub-batch with 8-byte rows */
                sl.rbytes = 8;
                if (int r = enc_front(ctx, sl, batch, params, fp, cs, is)) return r;
                HIP_TRY(hipEventSynchronize(sl.e[8]));
            }
            sl.total = sl.h_off[sl.nf];
            const int64_t f0 = sl.first_unit / C;
            for (int64_t f = 0; f < sl.nf; ++f) {
                frame_offsets[f0 + f + 1] = written + sl.h_off[f + 1];
                frame_status[f0 + f] = sl.h_st[f];
            }
            if (written + sl.total > out_capacity)
                return fail(FLACMI_E_NOMEM, "frames need %lld bytes, out holds %lld", (long long)(written + sl.total),
                            (long long)out_capacity);
            if (int r = ensure_buf(sl.frames, (size_t)sl.total + 16)) return r;
            const int64_t pstride = (1LL << (params->rice_max > 0 ? params->rice_max : 0)) + 1;
            const int64_t rstride = ((sl.b.block_len * sl.rbytes + 15) / 16) * 16 / sl.rbytes;
            flacmi_batch db = sl.b;
            db.samples = sl.samples.p;
            db.unit_stride = sl.dstride;
            flacmi_frame_params f = *fp;
            f.first_frame = fp->first_frame + f0;
            FrameArgs a = frame_args(ctx, &db, &f, (const flacmi_unit_meta*)sl.meta.p, (const int32_t*)sl.params.p,
                                     pstride, sl.nf);
            a.residual = sl.residual.p;
            a.residual_bytes = sl.rbytes;
            a.residual_stride = rstride;
            a.offsets = (int64_t*)sl.offsets.p;
            a.status = (int32_t*)sl.status.p;
            a.out = (uint8_t*)sl.frames.p;
            a.capacity = sl.total;
            if (int r = pack_lists(ctx, a)) return r;
            HIP_TRY(hipEventRecord(sl.e[4], cs));
            HIP_TRY(launch_pack(a, cs));
            HIP_TRY(hipEventRecord(sl.e[5], cs));
            HIP_TRY(hipStreamWaitEvent(os, sl.e[5], 0));
            HIP_TRY(hipEventRecord(sl.e[6], os));
            if (sl.total > 0)
                HIP_TRY(hipMemcpyAsync(out + written, sl.frames.p, (size_t)sl.total, hipMemcpyDeviceToHost, os));
            HIP_TRY(hipEventRecord(sl.e[7], os));
            written += sl.total;
            t.bytes_out += sl.total;
            return 0;
        };
        /* diagnostic (FLACMI_ENC_TRACE): per-sub-batch timeline in ms from the call's start */
        hipEvent_t tb = nullptr;
        static const bool trace = std::getenv("FLACMI_ENC_TRACE") != nullptr; /* read once */
        if (trace && hipEventCreate(&tb) == hipSuccess) (void)hipEventRecord(tb, is);
        auto account = [&](int64_t k) {
            EncSlot& sl = slot[k % kEncSlots];
            (void)hipEventSynchronize(sl.e[7]);
            if (tb)
                std::fprintf(stderr, "enc %lld: h2d %.2f-%.2f an-end %.2f sz-end %.2f off %.2f pack %.2f-%.2f d2h %.2f-%.2f\n",
                             (long long)k, ev_ms(tb, sl.e[0]), ev_ms(tb, sl.e[1]), ev_ms(tb, sl.e[2]), ev_ms(tb, sl.e[3]),
                             ev_ms(tb, sl.e[8]), ev_ms(tb, sl.e[4]), ev_ms(tb, sl.e[5]), ev_ms(tb, sl.e[6]), ev_ms(tb, sl.e[7]));
            t.h2d_ms += ev_ms(sl.e[0], sl.e[1]);
            t.analyze_ms += ev_ms(sl.e[1], sl.e[2]);
            t.sizes_ms += ev_ms(sl.e[2], sl.e[3]);
            t.pack_ms += ev_ms(sl.e[4], sl.e[5]);
            t.d2h_ms += ev_ms(sl.e[6], sl.e[7]);
            t.bytes_in += (int64_t)sl.b.n_units * sl.b.block_len * sl.b.sample_bytes;
        };
        for (int64_t k = 0; k < nsub; ++k) {
            if (k >= kEncSlots) account(k - kEncSlots); /* the slot is free once those frames are copied */
            setup(k);
            if ((rc = enc_front(ctx, slot[k % kEncSlots], batch, params, fp, cs, is))) break;
            if (k >= 1 && (rc = back(k - 1))) break;
        }
        if (!rc && (rc = back(nsub - 1)) == 0)
            for (int64_t k = (nsub >= kEncSlots ? nsub - kEncSlots : 0); k < nsub; ++k) account(k);
        t.sub_batches = nsub;
        if (tb) (void)hipEventDestroy(tb);
    }
    /* nothing may still read the caller's rows or write its buffer once this returns */
    for (hipStream_t st : {cs, is, os}) {
        hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess && !rc) rc = fail(FLACMI_E_HIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
    }
    {
        const auto u0 = std::chrono::steady_clock::now();
        if (reg_in) (void)hipHostUnregister(const_cast<void*>(batch->samples));
        if (reg_out) (void)hipHostUnregister(out);
        t.register_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - u0).count();
    }
    t.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    if (timing) *timing = t;
    return rc;
}

int flacmi_encode_fetch(flacmi_ctx* ctx, uint8_t* out, int64_t bytes) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    if (bytes < 0 || bytes > ctx->frames_bytes) return fail(FLACMI_E_INVALID, "at most %lld bytes are held",
                                                            (long long)ctx->frames_bytes);
    if (bytes == 0) return 0;
    if (!out) return fail(FLACMI_E_INVALID, "null output");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipMemcpy(out, ctx->h_frames.p, (size_t)bytes, hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"

extern "C" {

int flacmi_stream_stats(flacmi_ctx* ctx, const flacmi_unit_meta* d_meta, int64_t n_units, int32_t block_len,
                        int32_t tail_len, int64_t n_tail_units, int64_t* d_stats, void* stream) {
    if (!ctx || !d_stats) return fail(FLACMI_E_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipMemsetAsync(d_stats, 0, sizeof(int64_t) * FLACMI_STATS_WORDS, (hipStream_t)stream));
    HIP_TRY(launch_stats(d_meta, n_units, block_len, tail_len, n_tail_units, d_stats, (hipStream_t)stream));
    return 0;
}

/* ---- RCCL stats reduce: librccl.so.1 is opened on first use (no link-time dependency, so
 * the product library loads where RCCL is absent; a process that already loaded RCCL, e.g.
 * through torch, gets the same library back from dlopen) ---- */
namespace {
struct Rccl {
    void* h = nullptr;
    int (*get_id)(void* id) = nullptr;
    int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*destroy)(void*) = nullptr;
    const char* (*err)(int) = nullptr;
};
struct RcclId {
    char b[FLACMI_COMM_ID_BYTES];
};
/* ncclCommInitRank takes the 128-byte ncclUniqueId by value */
typedef int (*rccl_init_rank_t)(void** comm, int nranks, RcclId id, int rank);
Rccl g_rccl;
rccl_init_rank_t g_rccl_init = nullptr;
std::mutex g_rccl_mu;
constexpr int kNcclInt64 = 4, kNcclSum = 0; /* ncclDataType_t ncclInt64, ncclRedOp_t ncclSum */

int rccl_load() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.h) return 0;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return fail(FLACMI_E_UNSUPPORTED, "librccl.so.1 not found: %s", dlerror());
    Rccl r;
    r.h = h;
    r.get_id = (int (*)(void*))dlsym(h, "ncclGetUniqueId");
    g_rccl_init = (rccl_init_rank_t)dlsym(h, "ncclCommInitRank");
    r.all_reduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclAllReduce");
    r.destroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
    r.err = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
    if (!r.get_id || !g_rccl_init || !r.all_reduce || !r.destroy || !r.err)
        return fail(FLACMI_E_UNSUPPORTED, "librccl.so.1 lacks an entry point");
    g_rccl = r;
    return 0;
}
int rccl_fail(const char* what, int rc) {
    return fail(FLACMI_E_HIP, "%s: RCCL error %d (%s)", what, rc, g_rccl.err ? g_rccl.err(rc) : "?");
}
}  // namespace

struct flacmi_comm {
    flacmi_ctx* ctx;
    void* comm; /* ncclComm_t */
    int nranks, rank;
};

int flacmi_comm_available(void) { return rccl_load(); }

int64_t flacmi_unit_stride(int32_t block_len, int32_t sample_bytes) {
    if (block_len < 1 || (sample_bytes != 2 && sample_bytes != 4)) return fail(FLACMI_E_INVALID, "block_len < 1 or sample_bytes not 2/4");
    return row_pitch(block_len, sample_bytes);
}

int flacmi_comm_id(void* id_out) {
    if (!id_out) return fail(FLACMI_E_INVALID, "null argument");
    if (int rc = rccl_load()) return rc;
    if (int rc = g_rccl.get_id(id_out)) return rccl_fail("ncclGetUniqueId", rc);
    return 0;
}

int flacmi_comm_init(flacmi_ctx* ctx, int nranks, int rank, const void* id, flacmi_comm** out) {
    if (!ctx || !id || !out) return fail(FLACMI_E_INVALID, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(FLACMI_E_INVALID, "rank %d of %d", rank, nranks);
    if (int rc = rccl_load()) return rc;
    if (int rc = set_device(ctx)) return rc;
    RcclId cid;
    memcpy(cid.b, id, FLACMI_COMM_ID_BYTES);
    void* c = nullptr;
    if (int rc = g_rccl_init(&c, nranks, cid, rank)) return rccl_fail("ncclCommInitRank", rc);
    *out = new flacmi_comm{ctx, c, nranks, rank};
    return 0;
}

int flacmi_allreduce_stats(flacmi_comm* comm, int64_t* d_stats, void* stream) {
    if (!comm || !d_stats) return fail(FLACMI_E_INVALID, "null argument");
    if (int rc = set_device(comm->ctx)) return rc;
    if (int rc = g_rccl.all_reduce(d_stats, d_stats, FLACMI_STATS_WORDS, kNcclInt64, kNcclSum, comm->comm,
                                   (hipStream_t)stream))
        return rccl_fail("ncclAllReduce", rc);
    return 0;
}

int flacmi_comm_destroy(flacmi_comm* comm) {
    if (!comm) return 0;
    int rc = 0;
    if (comm->comm && g_rccl.destroy) {
        if (int e = set_device(comm->ctx)) rc = e;
        if (int e = g_rccl.destroy(comm->comm)) rc = rccl_fail("ncclCommDestroy", e);
    }
    delete comm;
    return rc;
}

int flacmi_synth_mix_device(flacmi_ctx* ctx, void* dst, int32_t sample_bytes, int32_t sample_bits,
                            int64_t unit_stride, int64_t first_unit, int64_t n_units, int32_t len, uint64_t seed,
                            int32_t open_eighths, void* stream) {
    if (!ctx || !dst) return fail(FLACMI_E_INVALID, "null argument");
    if (sample_bytes != 2 && sample_bytes != 4) return fail(FLACMI_E_INVALID, "sample_bytes must be 2 or 4");
    if (sample_bits < 8 || sample_bits > 8 * sample_bytes || (sample_bits > 16 && sample_bits - 16 > 15))
        return fail(FLACMI_E_INVALID, "sample_bits out of range");
    if (len < 1 || unit_stride < len) return fail(FLACMI_E_INVALID, "bad length/stride");
    if (n_units > 0x7fffffff) return fail(FLACMI_E_INVALID, "at most 2^31-1 units per synth call");
    if (open_eighths < 0 || open_eighths > 8) return fail(FLACMI_E_INVALID, "open_eighths must be 0..8");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(launch_synth(dst, sample_bytes, sample_bits, unit_stride, first_unit, n_units, len, seed, ctx->d_sintab,
                         open_eighths, (hipStream_t)stream));
    return 0;
}

int flacmi_synth_device(flacmi_ctx* ctx, void* dst, int32_t sample_bytes, int32_t sample_bits, int64_t unit_stride,
                        int64_t first_unit, int64_t n_units, int32_t len, uint64_t seed, void* stream) {
    return flacmi_synth_mix_device(ctx, dst, sample_bytes, sample_bits, unit_stride, first_unit, n_units, len, seed, 0,
                                   stream);
}

void* flacmi_device_alloc(flacmi_ctx* ctx, size_t bytes) {
    if (!ctx) return nullptr;
    if (set_device(ctx)) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        fail(FLACMI_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

int flacmi_device_free(flacmi_ctx* ctx, void* ptr) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipFree(ptr));
    return 0;
}

int flacmi_memcpy_h2d(flacmi_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return 0;
}

int flacmi_memcpy_d2h(flacmi_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}

int flacmi_synchronize(flacmi_ctx* ctx) {
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipDeviceSynchronize());
    return 0;
}

int flacmi_last_timing(flacmi_ctx* ctx, float* ms, int n) {
    if (!ctx || ctx->ncalls == 0) return fail(FLACMI_E_INVALID, "no timed call");
    if (int rc = set_device(ctx)) return rc;
    const int k = ctx->ncalls < flacmi_ctx::kRing ? ctx->ncalls : flacmi_ctx::kRing;
    double acc[3] = {0, 0, 0};
    for (int c = ctx->ncalls - k; c < ctx->ncalls; ++c) {
        hipEvent_t* ev = ctx->ev[c % flacmi_ctx::kRing];
        HIP_TRY(hipEventSynchronize(ev[2]));
        float t;
        HIP_TRY(hipEventElapsedTime(&t, ev[0], ev[1]));
        acc[0] += t;
        const int nk = ctx->nchunks[c % flacmi_ctx::kRing];
        if (nk == 0) {
            HIP_TRY(hipEventElapsedTime(&t, ev[1], ev[2]));
            acc[1] += t;
        } else { /* overlap: the k_resid launches' own spans */
            for (int i = 0; i < nk; ++i) {
                HIP_TRY(hipEventElapsedTime(&t, ev[3 + 2 * i], ev[4 + 2 * i]));
                acc[1] += t;
            }
        }
        HIP_TRY(hipEventElapsedTime(&t, ev[0], ev[2]));
        acc[2] += t;
    }
    const float vals[4] = {(float)(acc[0] / k), (float)(acc[1] / k), (float)(acc[2] / k), (float)k};
    const int m = n < 4 ? n : 4;
    for (int i = 0; i < m; ++i) ms[i] = vals[i];
    return m;
}

int flacmi_timing_reset(flacmi_ctx* ctx) {
    if (!ctx) return fail(FLACMI_E_INVALID, "null context");
    ctx->ncalls = 0;
    return 0;
}

double flacmi_host_pypow2(double x, int32_t* status) {
    static const uint64_t lh[] = GLIBC_POW_LOG_HDR, lt[] = GLIBC_POW_LOG_TAB, eh[] = GLIBC_EXP_HDR,
                          et[] = GLIBC_EXP_TAB;
    const pym::PowTables T{lh, lt, eh, et};
    int st = 0;
    const double r = pym::py_pow2(x, T, &st);
    if (status) *status = st;
    return r;
}

int32_t flacmi_host_floor_log2(double x) {
    ensure_tables();
    if (!(x > 0.0) || std::isinf(x)) return INT32_MIN; /* outside the domain (the table covers finite x > 0) */
    return pym::py_floor_log2(x, g_log2thr.data());
}

int flacmi_device_selftest(flacmi_ctx* ctx, int32_t which, const double* x, double* out, int32_t* status,
                           int64_t n) {
    if (!ctx || !x || !out || !status) return fail(FLACMI_E_INVALID, "null argument");
    if (which != 0 && which != 1) return fail(FLACMI_E_INVALID, "which must be 0 or 1");
    if (n <= 0) return 0;
    if (int rc = set_device(ctx)) return rc;
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)n * (8 + 8 + 4)));
    double* dx = (double*)d;
    double* dout = dx + n;
    int32_t* dst = (int32_t*)(dout + n);
    int rc = 0;
    hipError_t e = hipMemcpyAsync(dx, x, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = launch_selftest(which, dx, dout, dst, n, ctx->d_log2thr, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(status, dst, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = fail(FLACMI_E_HIP, "selftest: %s", hipGetErrorString(e));
    (void)hipFree(d);
    return rc;
}

int flacmi_device_lpc_from_acf(flacmi_ctx* ctx, const double* acf, int64_t n, int32_t L, int32_t q, int32_t* rec) {
    if (!ctx || !acf || !rec) return fail(FLACMI_E_INVALID, "null argument");
    if (L < 1 || L > FLACMI_MAX_LPC_ORDER) return fail(FLACMI_E_INVALID, "L must be in 1..%d", FLACMI_MAX_LPC_ORDER);
    if (q < 5 || q > 15) return fail(FLACMI_E_INVALID, "q must be in 5..15");
    if (n <= 0) return 0;
    if (int rc = set_device(ctx)) return rc;
    const int rw = FLACMI_LPC_REC_WORDS(L);
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)n * (33 * 8 + (size_t)rw * 4)));
    LpcArgs a{};
    a.acf = (double*)d;
    a.rec = (int32_t*)(a.acf + n * 33);
    a.count = n;
    a.n = 1 << 12;
    a.L = L;
    a.q = q;
    a.rec_words = rw;
    a.log2thr = ctx->d_log2thr;
    int rc = 0;
    hipError_t e = hipMemcpyAsync(a.acf, acf, (size_t)n * 33 * 8, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = launch_lpc_from_acf(a, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(rec, a.rec, (size_t)n * rw * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = fail(FLACMI_E_HIP, "lpc_from_acf: %s", hipGetErrorString(e));
    (void)hipFree(d);
    return rc;
}

}  // extern "C"
