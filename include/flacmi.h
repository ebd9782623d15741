/*
 * flacmi.h — C-ABI of the MI355X FLAC encode-analysis library (libflacmi.so).
 *
 * This is the drop-in boundary for turlando/flac-py's per-block analysis hot path.
 * flac-py has no FFI layer of its own; the interface this library replaces is the
 * Python function triple called once per (block, channel) from encode():
 *
 *   encode_subframe_fixed(samples)                       flac/encoder.py:331-359
 *   encode_subframe_lpc(samples, lpc_order, precision)   flac/encoder.py:362-420
 *     (tukey 423-440, autocorrelation 443-450, levinson_durbin 453-479,
 *      quantize_lpc_coefficients 482-534, prediction_residual 537-548)
 *   the fixed-vs-LPC choice on sum(|residual|)           flac/encoder.py:133-157
 *   encode_residual(residual, block_size, sample_size,
 *                   predictor_order, partition_order_range)  flac/encoder.py:632-760
 *     (called by the writer at flac/encoder.py:588 and :608)
 *
 * One call analyses a whole batch of independent "units" (one unit = one channel of
 * one block) and returns, per unit, exactly the fields of the reference's
 * SubframeHeader / SubframeFixed / SubframeLPC / Residual / RicePartition values
 * (flac/common.py:286-309, 334-361, 378-420), bit-identical.  Where the reference
 * would raise a Python exception the unit's `status` names the exception class and
 * `site` names the raising statement (see flacmi_status / flacmi_site).
 *
 * Conventions: plain C types, caller-owned buffers, return 0 on success or a
 * negative flacmi_error; flacmi_last_error() describes the last failure of the
 * calling thread.  A context is bound to one HIP device and is not thread-safe;
 * use one context per host thread.  The *_device entry points take device pointers
 * and enqueue on the given hipStream_t (passed as void*), returning without a host
 * synchronisation; the *_host entry points take host pointers and are synchronous.
 * The *_device calls of one context share its scratch buffers (LPC records, retry and
 * pack lists, decoder state): issue them on one stream, or make each call's stream
 * wait for the previous call's work, never concurrently on two streams.
 */
#ifndef FLACMI_H
#define FLACMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: in the default (pruning) mode meta.lpc_order / meta.lpc_sum of a unit whose LPC
      candidates provably lose read FLACMI_LPC_PRUNED, and stats word 80 no longer folds
      lpc_sum (round 3); version 1 callers read exact LPC fields there */
#define FLACMI_ABI_VERSION 2
#define FLACMI_MAX_LPC_ORDER 32      /* EncoderParameters: lpc_order.stop <= 33 (encoder.py:42) */
#define FLACMI_MAX_BLOCK 65535       /* largest block the reference writes (encoder.py:249-253, 16-bit uncommon
                                        code); analysis returns FLACMI_E_UNSUPPORTED where a block's
                                        workgroup staging exceeds LDS (above ~16K samples) */
#define FLACMI_MAX_RICE_ORDER 15     /* 4-bit partition-order field (encoder.py:767) */
#define FLACMI_LPC_REC_WORDS(L) (2 + (L) + ((L) * ((L) + 1)) / 2)

/* ---- return codes (API level) ------------------------------------------------ */
enum flacmi_error {
    FLACMI_OK = 0,
    FLACMI_E_INVALID = -1,       /* bad argument (shape, range, alignment) */
    FLACMI_E_HIP = -2,           /* HIP runtime error */
    FLACMI_E_UNSUPPORTED = -3,   /* shape this build does not handle (see flacmi_last_error) */
    FLACMI_E_NOMEM = -4,
};

/* ---- per-unit status: the Python exception the reference would raise ---------- */
enum flacmi_status {
    FLACMI_STATUS_OK = 0,
    FLACMI_STATUS_ZERO_DIVISION = 1,  /* ZeroDivisionError */
    FLACMI_STATUS_ASSERTION = 2,      /* AssertionError */
    FLACMI_STATUS_VALUE_ERROR = 3,    /* ValueError */
    FLACMI_STATUS_OVERFLOW = 4,       /* OverflowError */
    FLACMI_STATUS_RESIDUAL_WIDE = 16, /* not a reference exception: chosen residual does not fit
                                         the requested residual element width; re-run with 8 bytes */
};

/* ---- per-unit site: which reference statement raises ------------------------------ */
enum flacmi_site {
    FLACMI_SITE_NONE = 0,
    FLACMI_SITE_TUKEY = 1,           /* encoder.py:437  pi*i/nr with nr == 0 (4 <= n <= 7) */
    FLACMI_SITE_LEVINSON_DIV = 2,    /* encoder.py:469  lambda_ /= error, error == 0 */
    FLACMI_SITE_LEVINSON_POW = 3,    /* encoder.py:476  lambda_ ** 2 overflows */
    FLACMI_SITE_QUANT_CMAX = 4,      /* encoder.py:496  assert coef_max > 0.0 */
    FLACMI_SITE_QUANT_LOG2 = 5,      /* encoder.py:503  floor(log2(inf)) */
    FLACMI_SITE_QUANT_SHIFT = 6,     /* encoder.py:508  shift < shift_min */
    FLACMI_SITE_QUANT_ROUND_INF = 7, /* encoder.py:520/530 round(inf) */
    FLACMI_SITE_QUANT_ROUND_NAN = 8, /* encoder.py:520/530 round(nan) */
    FLACMI_SITE_LPC_EMPTY = 9,       /* encoder.py:404  min() of no candidate orders (-l 0) */
    FLACMI_SITE_CHOICE_TIE = 10,     /* encoder.py:157  fixed_size == lpc_size */
    FLACMI_SITE_RICE_NO_ORDER = 11,  /* encoder.py:669  no valid partition order */
    FLACMI_SITE_RICE_LOG_DOMAIN = 12,/* encoder.py:753  log2(0): partition sum is 0 */
    FLACMI_SITE_RICE_NEG_SHIFT = 13, /* encoder.py:758  1 << parameter, parameter < 0 */
    FLACMI_SITE_RESIDUAL_WIDTH = 14, /* not a reference site: see FLACMI_STATUS_RESIDUAL_WIDE */
    /* frame writer (flacmi_frame_sizes_device): statements of the reference's writer */
    FLACMI_SITE_CODED_NUMBER = 15,   /* coded_number.py:38  frame number needs more than 31 bits (ValueError) */
    FLACMI_SITE_LPC_PRECISION = 16,  /* encoder.py:619  assert precision - 1 != 0b1111 (AssertionError) */
    FLACMI_SITE_FRAME_SIZE = 17,     /* not a reference site: see FLACMI_STATUS_FRAME_TOO_LARGE */
};

/* frame writer status beyond the reference's exceptions */
#define FLACMI_STATUS_FRAME_TOO_LARGE 17 /* a frame of >= 2^28 bytes: this build does not pack it */

/* ---- analysis modes -------------------------------------------------------------- */
enum flacmi_mode {
    FLACMI_MODE_REFERENCE = 0,   /* fixed + LPC + choice + Rice, exactly as encode() does */
    FLACMI_MODE_FIXED_ONLY = 1,  /* fixed predictor + Rice only (BASELINE config 5; the
                                    reference's own -l 0 raises ValueError instead) */
    FLACMI_MODE_LPC_ONLY = 2,    /* encode_subframe_lpc alone (encoder.py:362-420): the best LPC
                                    candidate is the result, no fixed comparison, no Rice search
                                    (part_order = -1); its residual row is returned */
    FLACMI_MODE_RICE_ONLY = 3,   /* encode_residual alone (encoder.py:632-652): each row holds a
                                    residual at [reserved[0], len) for predictor order
                                    params.reserved[0]; only the Rice search runs */
};

enum flacmi_kind { FLACMI_KIND_FIXED = 0, FLACMI_KIND_LPC = 1 };

typedef struct flacmi_params {
    int32_t max_lpc_order;   /* L = lpc_order.stop - 1, 0..32 (lpc_order.start must be 0) */
    int32_t qlp_precision;   /* EncoderParameters.qlp_precision, 5..31 */
    int32_t rice_min;        /* rice_partition_order.start */
    int32_t rice_max;        /* rice_partition_order.stop - 1 (rice_max < rice_min: empty range) */
    int32_t mode;            /* flacmi_mode */
    int32_t reserved[3];     /* reserved[0]: predictor order in FLACMI_MODE_RICE_ONLY, else 0;
                                reserved[1]: flacmi_flags; reserved[2]: 0 */
} flacmi_params;

/* params.reserved[1] bits */
enum flacmi_flags {
    /* compute every LPC candidate's exact sum(|r|) in FLACMI_MODE_REFERENCE (meta.lpc_order /
     * lpc_sum always exact).  Without it the analysis may prune: see FLACMI_LPC_PRUNED. */
    FLACMI_FLAG_ALL_CANDIDATES = 1,
    /* diagnostic: prune with the partial-sum tiers alone (no sign-correlation bound), so a
     * test reaches the tier decisions on data the bound already settles */
    FLACMI_FLAG_TIERS_ONLY = 2,
};

/* meta.lpc_order and meta.lpc_sum of a unit whose LPC candidates were pruned: exact lower
 * bounds proved every candidate's sum(|r|) strictly above the best fixed sum, so the
 * reference's choice (encoder.py:135-157) is the fixed subframe and no tie is possible.
 * Everything the reference writes (kind, order, residual, Rice fields) is unaffected.  Runs
 * with outputs.lpc_sums or FLACMI_FLAG_ALL_CANDIDATES never prune. */
#define FLACMI_LPC_PRUNED (-1)

/* One batch of units.  Samples are planar: unit u occupies
 * samples[u*unit_stride .. u*unit_stride + len(u)).  Every unit has `block_len`
 * samples except the last `n_tail_units`, which have `tail_len` (the short last
 * block of a stream, one unit per channel).  Rows must be 16-byte aligned. */
typedef struct flacmi_batch {
    const void* samples;     /* int16 (sample_bytes 2) or int32 (sample_bytes 4) */
    int32_t sample_bytes;    /* 2 or 4 */
    int32_t sample_bits;     /* every sample fits a signed integer of this many bits (<= 8*sample_bytes) */
    int64_t unit_stride;     /* elements between consecutive units (flacmi_unit_stride: the pitch
                                the library itself lays rows out at) */
    int64_t n_units;
    int32_t block_len;       /* 1..FLACMI_MAX_BLOCK */
    int32_t tail_len;        /* length of the trailing units, 1..block_len (ignored if n_tail_units == 0) */
    int64_t n_tail_units;    /* 0..n_units */
} flacmi_batch;

/* Per-unit result.  Field names follow flac/common.py:
 *   kind/order        -> SubframeHeader.type_ = SubframeTypeFixed(order) | SubframeTypeLPC(order)
 *   warmup            -> samples[:order]  (not copied: the caller has the samples)
 *   shift/coefs/ncoefs-> SubframeLPC.shift / .coefficients (qlp precision is the parameter)
 *   residual          -> residual row [res_offset, res_offset + res_len), zig-zag encoded,
 *                        i.e. the concatenation of RicePartition.residual
 *   part_order/n_parts/coding_method/rice params -> Residual  */
typedef struct flacmi_unit_meta {
    int32_t status;          /* flacmi_status */
    int32_t site;            /* flacmi_site */
    int32_t kind;            /* flacmi_kind of the chosen subframe */
    int32_t order;           /* predictor order of the chosen subframe = len(warmup) */
    int32_t shift;           /* SubframeLPC.shift (0 for fixed) */
    int32_t ncoefs;          /* len(SubframeLPC.coefficients): order, or 0 in the negative-shift branch */
    int32_t res_offset;      /* first valid element of the residual row */
    int32_t res_len;         /* len(residual) */
    int32_t fixed_order;     /* best fixed order 0..4 */
    int32_t lpc_order;       /* best LPC order 1..L (0 in fixed-only mode, FLACMI_LPC_PRUNED if pruned) */
    int32_t part_order;      /* Residual.partition_order as chosen by rice_partitions */
    int32_t n_parts;         /* len(Residual.partitions) */
    int32_t coding_method;   /* RiceCodingMethod value: 4 or 5 */
    int32_t lpc_tiers;       /* diagnostic, the pruning decision: LPC candidate passes made | passes of the
                                path << 8.  16-bit stream kernel: quarter-block bound passes 1..4, then 5 =
                                the exact pass; int8-MFMA path: eighths 2..8 of exact partial sums (8 = every
                                tile), 0/8 when the sign-correlation bound decides (k_resid_sb included);
                                16-bit k_resid: 0/1 (sign bound decides) or 1/1 (the exact LPC pass).  0 where
                                no pruning runs (fixed-only, all-candidates, the 64-bit chains) */
    int64_t fixed_sum;       /* sum(|r|) of the best fixed residual */
    int64_t lpc_sum;         /* sum(|r|) of the best LPC residual (0 in fixed-only mode, FLACMI_LPC_PRUNED if pruned) */
    int64_t rice_bits;       /* size estimate of the chosen partitioning (encoder.py:714-727) */
    int32_t coefs[FLACMI_MAX_LPC_ORDER];
} flacmi_unit_meta;

typedef struct flacmi_outputs {
    flacmi_unit_meta* meta;  /* [n_units] */
    int32_t* rice_params;    /* [n_units][params_stride], RicePartition.parameter per partition */
    int64_t params_stride;   /* >= 2^rice_max + 1 */
    void* residual;          /* [n_units][residual_stride] uint32 or uint64 zig-zag residuals */
    int32_t residual_bytes;  /* 4 or 8 */
    int32_t reserved0;
    int64_t residual_stride; /* elements, >= block_len */
    /* optional intermediates (NULL to skip), used by parity tests */
    double* acf;             /* [n_units][33]  autocorrelation lags 0..L */
    int64_t* fixed_sums;     /* [n_units][5]   sum(|r|) for fixed orders 0..4 */
    int64_t* lpc_sums;       /* [n_units][32]  sum(|r|) for LPC orders 1..L */
    int32_t* lpc_records;    /* [n_units][FLACMI_LPC_REC_WORDS(32)] status/site, negmask, shifts, coefs */
} flacmi_outputs;

typedef struct flacmi_ctx flacmi_ctx;

/* ---- library / context ------------------------------------------------------------ */
int flacmi_abi_version(void);
const char* flacmi_last_error(void);
int flacmi_device_count(void);
flacmi_ctx* flacmi_create(int device);
void flacmi_destroy(flacmi_ctx* ctx);

/* ---- the hot path ---------------------------------------------------------------- */
/* Device pointers, enqueued on `stream` (hipStream_t). */
int flacmi_analyze_device(flacmi_ctx* ctx, const flacmi_batch* batch,
                          const flacmi_params* params, const flacmi_outputs* out,
                          void* stream);
/* Host pointers; copies in and out, synchronous. */
int flacmi_analyze_host(flacmi_ctx* ctx, const flacmi_batch* batch,
                        const flacmi_params* params, const flacmi_outputs* out);

/* ---- frame writer: FLAC frames from the analysis results -------------------------- */
/* The reference writes each frame on the host, bit by bit (encoder.py:87-165 frame loop;
 * put_frame_header :194-234 with coded_number.py:7-39 and crc.py:18-31; _put_subframe_header
 * :553-569; _put_subframe_fixed/_lpc :581-627; put_residual / put_rice_partition /
 * put_rice_int :765-806; padding + CRC-16 footer :159-163).  These entry points produce
 * the same bytes on the device: frame f of a batch holds the units
 * [f*channels, (f+1)*channels) (one subframe per channel, in channel order); the last
 * frame may be short (the batch's tail units).  Frames are byte-aligned and packed back
 * to back in `out` at frame_offsets[f] .. frame_offsets[f+1]. */
typedef struct flacmi_frame_params {
    int32_t channels;        /* units per frame, 1..8 (encode()'s channels) */
    int32_t sample_size;     /* bits per warm-up sample in the stream (encode()'s sample_size), 1..32 */
    int32_t qlp_precision;   /* SubframeLPC.precision (EncoderParameters.qlp_precision) */
    int32_t reserved0;
    int64_t first_frame;     /* coded number of the batch's first frame (block index, encoder.py:97) */
    int64_t reserved[2];
} flacmi_frame_params;

/* Frame sizes and their exclusive prefix sums (device pointers, enqueued on `stream`).
 * frame_offsets[n_frames + 1] receives byte offsets (frame_offsets[n_frames] = total);
 * frame_status[n_frames] receives 0, or (site << 16) | status of the first subframe (in
 * channel order) the reference would fail on while analysing or writing the frame; such
 * a frame gets size 0 and is not written.  meta / rice_params are analyze outputs for the
 * same batch; n_frames = ceil(n_units / channels). */
int flacmi_frame_sizes_device(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_frame_params* fp,
                              const flacmi_unit_meta* meta, const int32_t* rice_params, int64_t params_stride,
                              int64_t* frame_offsets, int32_t* frame_status, void* stream);
/* Write every frame with status 0 into out[frame_offsets[f] ..) (device pointers).  The
 * residual rows are the analyze outputs (zig-zag u32 or u64 rows, residual_bytes 4 or 8).
 * out must hold frame_offsets[n_frames] bytes (checked on the device against out_capacity;
 * on overflow nothing is written and frame_status[0] is set to FLACMI_STATUS_FRAME_TOO_LARGE). */
int flacmi_pack_frames_device(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_frame_params* fp,
                              const flacmi_unit_meta* meta, const int32_t* rice_params, int64_t params_stride,
                              const void* residual, int32_t residual_bytes, int64_t residual_stride,
                              const int64_t* frame_offsets, int32_t* frame_status, uint8_t* out,
                              int64_t out_capacity, void* stream);
/* Host form of analyze + frame sizes + pack (synchronous): host samples in; frame_offsets
 * [n_frames + 1] and frame_status [n_frames] out.  The frame bytes stay in a context
 * buffer until flacmi_encode_fetch copies them (frame_offsets[n_frames] bytes) to the host. */
int flacmi_encode_host(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                       const flacmi_frame_params* fp, int64_t* frame_offsets, int32_t* frame_status);
int flacmi_encode_fetch(flacmi_ctx* ctx, uint8_t* out, int64_t bytes);

/* Pipelined host encode (SURVEY §8d end-to-end; the reference's encode() loop plus its
 * writer, encoder.py:87-165, 765-806): host sample rows in, FLAC frame bytes out, the batch
 * cut into sub-batches of units_per_batch units (a multiple of channels) with two in
 * flight: the copy of sub-batch k+1 to the device and its analysis overlap the frame
 * writing and the copy back of sub-batch k.  The caller's sample rows and `out` are
 * page-locked in place for the call (hipHostRegister) so both copies are DMA at PCIe rate.
 * Buffers the caller already page-locked with flacmi_host_register are used as they are
 * (no per-call register / unregister: the way to stream many calls through the same
 * buffers).
 * out receives the frames back to back; frame_offsets[n_frames + 1] their byte offsets and
 * frame_status[n_frames] as flacmi_frame_sizes_device (a failing frame has no bytes).
 * FLACMI_E_NOMEM if the frames exceed out_capacity (frame_offsets then hold the sizes of
 * the sub-batches written so far).  timing (optional) receives per-step times. */
typedef struct flacmi_encode_timing {
    double wall_ms;        /* the whole call */
    double h2d_ms;         /* sum over sub-batches of each step's own duration (HIP events): */
    double analyze_ms;     /*   host -> device sample copy, analysis (k_lpc + k_resid), */
    double sizes_ms;       /*   frame sizes + scan, frame writing (k_pack32 / k_pack), */
    double pack_ms;        /*   device -> host frame copy; the steps of different */
    double d2h_ms;         /*   sub-batches overlap in wall time */
    double register_ms;    /* hipHostRegister / Unregister of the caller's buffers */
    int64_t sub_batches;
    int64_t bytes_in;      /* sample bytes copied to the device */
    int64_t bytes_out;     /* frame bytes copied back */
} flacmi_encode_timing;
int flacmi_encode_pipeline(flacmi_ctx* ctx, const flacmi_batch* batch, const flacmi_params* params,
                           const flacmi_frame_params* fp, int64_t units_per_batch, uint8_t* out,
                           int64_t out_capacity, int64_t* frame_offsets, int32_t* frame_status,
                           flacmi_encode_timing* timing);

/* Page-lock a host range for the lifetime the caller chooses (hipHostRegister on the
 * context's device), so repeated flacmi_encode_pipeline / flacmi_analyze_host calls over
 * the same buffers copy at PCIe rate without paying the page-locking each call.  Replaces
 * nothing in the reference (its encode() has no device copies); the host-side analogue of
 * keeping a reused buffer (__main__.py:94-109 writes one output file per run).
 * FLACMI_E_HIP if the range cannot be locked (e.g. it overlaps a locked range). */
int flacmi_host_register(flacmi_ctx* ctx, void* ptr, size_t bytes);
int flacmi_host_unregister(flacmi_ctx* ctx, void* ptr);

/* Page-locked host memory owned by the caller until flacmi_host_free (hipHostMalloc on the
 * context's device): the staging rows and frame buffer a streaming caller fills and drains
 * batch after batch (flac_amd.encoder's encode paths), with no per-call page-locking.
 * NULL (flacmi_last_error) if it cannot be allocated.  flacmi_host_free takes a NULL ctx too
 * (memory that outlives its context). */
void* flacmi_host_alloc(flacmi_ctx* ctx, size_t bytes);
int flacmi_host_free(flacmi_ctx* ctx, void* ptr);

/* ---- decoder verifier (BASELINE config 5 round trip) ------------- */
/* Replaces the reference's frame decoder: decoder.py:111-130 get_frame, :133-190
 * get_frame_header (+ coded_number.py:45-70 decode), :192-245 field decoders, :267-344
 * get_subframe / get_subframe_header / get_subframe_type, :346-355 get_wasted_bits, :358-421
 * get_residual / get_rice_partition / get_rice_int, :431-498 decode_frame / decode_*_subframe
 * / _decode_prediction.  Frame f is the bytes stream[frame_offsets[f] .. frame_offsets[f+1]).
 * Per frame the device parses the header, every subframe and the footer, restores the
 * samples and (optionally) compares them with the batch they were encoded from.
 *
 * frame_status[f] = (site << 16) | status: the exception the reference decoder raises
 * (AssertionError / ValueError / EOFError, flacmi_decode_site names the statement), or a
 * verifier finding the reference does not check (FLACMI_STATUS_VERIFY: CRC-8 / CRC-16,
 * frame end, frame number, block size, sample mismatch).  frame_mismatch[f] counts the
 * samples that differ from `expect` (0 when expect is NULL).  Decoding is byte-exact to
 * the reference on every valid frame, with two documented choices: an L_R frame holds
 * dp->channels subframes (encoder.py:95 writes L_R whatever the channel count, so the
 * reference decoder cannot read back its own mono or 3+ channel streams), and, as in
 * decode_subframe, wasted bits are parsed but not shifted back in. */
#define FLACMI_STATUS_EOF 5        /* EOFError: the frame runs past the end of the stream */
#define FLACMI_STATUS_VERIFY 18    /* verifier finding (not a reference exception) */
enum flacmi_decode_site {
    FLACMI_DSITE_SYNC = 32,          /* decoder.py:134  assert sync code */
    FLACMI_DSITE_BLOCK_SIZE_CODE,    /* :194  assert 0 < block-size code < 15 */
    FLACMI_DSITE_SAMPLE_RATE_CODE,   /* :213  assert sample-rate code < 15 */
    FLACMI_DSITE_CHANNELS_CODE,      /* :232  assert channel code <= 10 */
    FLACMI_DSITE_SAMPLE_SIZE_CODE,   /* :239  assert sample-size code != 3 */
    FLACMI_DSITE_RESERVED,           /* :141  assert reserved bit == 0 */
    FLACMI_DSITE_SUBFRAME_PAD,       /* :319  assert subframe padding bit == 0 */
    FLACMI_DSITE_SUBFRAME_TYPE,      /* :329-331  assert reserved subframe type */
    FLACMI_DSITE_LPC_PRECISION,      /* :302  assert precision != 0b1111 */
    FLACMI_DSITE_CODING_METHOD,      /* :394  ValueError: cannot read coding method */
    FLACMI_DSITE_PARTITIONS,         /* :363-364  assert block size / partition order */
    FLACMI_DSITE_ESCAPE_ZERO,        /* binary.py:131 sint(0): ValueError negative shift count */
    FLACMI_DSITE_NEG_SHIFT,          /* :496-497  ValueError: negative LPC shift in _decode_prediction */
    FLACMI_DSITE_PADDING,            /* :126  assert frame padding == 0 */
    FLACMI_DSITE_EOF,                /* binary.py:40  EOFError: the stream ends inside the frame */
    FLACMI_DSITE_CRC8,               /* verifier: header CRC-8 mismatch (crc.py:18-22) */
    FLACMI_DSITE_CRC16,              /* verifier: frame CRC-16 mismatch (crc.py:25-31) */
    FLACMI_DSITE_FRAME_END,          /* verifier: the frame does not end at frame_offsets[f+1] */
    FLACMI_DSITE_FRAME_NUMBER,       /* verifier: coded number != first_frame + f */
    FLACMI_DSITE_BLOCK_SIZE,         /* verifier: block size != the expected unit length / out_stride */
    FLACMI_DSITE_CHANNELS,           /* verifier: header channel count != dp->channels */
    FLACMI_DSITE_SAMPLES,            /* verifier: decoded samples differ from `expect` */
};
typedef struct flacmi_decode_params {
    int32_t channels;        /* subframes per frame (STREAMINFO channels), 1..8 */
    int32_t sample_size;     /* STREAMINFO sample size, used when the header defers to it, 4..32 */
    int64_t first_frame;     /* coded number expected for frame 0, or -1: not checked */
    int32_t check_crc;       /* 1: verify CRC-8 and CRC-16 (the reference reads them unchecked) */
    int32_t reserved0;
    int64_t reserved[2];
} flacmi_decode_params;
/* All pointers are device pointers; the work is enqueued on `stream`.  stream_bytes is the
 * readable size of `stream` (4-byte aligned base).  expect: NULL, or the batch whose unit
 * f*channels + c the subframe c of frame f must reproduce (block_len / tail_len /
 * n_tail_units give the expected block sizes).  samples_out: NULL, or int32 rows
 * [n_frames*channels][out_stride] (out_stride a multiple of 4, 16-byte aligned rows) that
 * receive the decoded samples; required when a frame uses L_S / S_R / M_S stereo. */
int flacmi_decode_frames_device(flacmi_ctx* ctx, const uint8_t* stream_data, int64_t stream_bytes,
                                const int64_t* frame_offsets, int64_t n_frames,
                                const flacmi_decode_params* dp, const flacmi_batch* expect,
                                int32_t* samples_out, int64_t out_stride, int32_t* frame_status,
                                int64_t* frame_mismatch, void* stream);

/* ---- stream statistics (reduced across GPUs with one RCCL all-reduce) ------------- */
#define FLACMI_STATS_WORDS 128
/* stats[0] units, [1] samples, [2] rice bits, [3] fixed units, [4] lpc units,
 * [5..9] fixed order histogram, [10..42] lpc order histogram (index 10+order-1... 41),
 * [48..63] partition order histogram, [64..79] status histogram, [80] checksum of the units'
 * (rice_bits, fixed_sum, kind, order): results that do not depend on LPC pruning; [81] units whose
 * LPC candidates were pruned (FLACMI_LPC_PRUNED) */
int flacmi_stream_stats(flacmi_ctx* ctx, const flacmi_unit_meta* d_meta, int64_t n_units,
                        int32_t block_len, int32_t tail_len, int64_t n_tail_units,
                        int64_t* d_stats, void* stream);

/* ---- the cross-GPU stats reduce without torch (SURVEY §8b flacmi_allreduce_stats) ----- */
/* One process (or host thread) per GPU.  Rank 0 makes an id with flacmi_comm_id and hands
 * its FLACMI_COMM_ID_BYTES to every rank over any out-of-band channel (a file, a socket,
 * MPI); each rank then calls flacmi_comm_init with the same id, the world size and its rank
 * (collective: every rank must call it).  RCCL (librccl.so.1, loaded on first use) runs
 * the all-reduce over xGMI.  Replaces the reference's nothing: flac-py is single-process;
 * the streams' statistics are the only cross-GPU exchange (encoder.py:81 writes no MD5). */
#define FLACMI_COMM_ID_BYTES 128
typedef struct flacmi_comm flacmi_comm;
/* 0 when RCCL loads here with every entry point the communicator uses (a local check, no id
 * or socket made): every rank runs it before rank 0 makes the id and all ranks enter the
 * collective flacmi_comm_init.  A failure inside ncclCommInitRank itself is not covered. */
int flacmi_comm_available(void);
int flacmi_comm_id(void* id_out);
int flacmi_comm_init(flacmi_ctx* ctx, int nranks, int rank, const void* id, flacmi_comm** out);
/* Sum of every rank's FLACMI_STATS_WORDS int64 words, in place (device pointer), enqueued
 * on `stream` (a stream of the communicator's context device). */
int flacmi_allreduce_stats(flacmi_comm* comm, int64_t* d_stats, void* stream);
int flacmi_comm_destroy(flacmi_comm* comm);

/* ---- row layout ------------------------------------------------------------------------ */
/* The unit pitch, in samples, at which this library lays out device rows (the *_host entry
 * points' mirrors, the encode pipeline's sub-batches) and which it recommends to callers of
 * the *_device entry points: the row rounded up to 16 bytes, plus 128 bytes when that is a
 * multiple of 4 KB.  k_lpc reads 64 rows at one offset per load instruction; at a 4 KB-multiple
 * pitch those lines fall into the same L2 sets and are fetched again.  A host
 * batch already at this pitch goes to the device as one linear copy.  No device needed. */
int64_t flacmi_unit_stride(int32_t block_len, int32_t sample_bytes);

/* ---- synthetic PCM (BASELINE configs 2-5) --------------------------------- */
/* Writes units [first_unit, first_unit + n_units) of the integer synthetic signal into
 * dst[(u - first_unit) * unit_stride ...]: sum of 3 DDS sinusoids + splitmix64 noise,
 * clipped to sample_bits; bit-identical to oracle/flac_oracle.c:oracle_synth_unit. */
int flacmi_synth_device(flacmi_ctx* ctx, void* dst, int32_t sample_bytes, int32_t sample_bits,
                        int64_t unit_stride, int64_t first_unit, int64_t n_units, int32_t len,
                        uint64_t seed, void* stream);
/* The same with open_eighths / 8 of the units (those whose hash byte is below open_eighths)
 * replaced by MA(1) near-white noise, whose LPC candidates tie the fixed order-0 sum within a
 * fraction of a percent: no bound decides them, so every candidate's exact sum is computed
 * (bench.py --open, the "undecided" workload).  Bit-identical to oracle_synth_unit_mix;
 * open_eighths = 0 is flacmi_synth_device. */
int flacmi_synth_mix_device(flacmi_ctx* ctx, void* dst, int32_t sample_bytes, int32_t sample_bits,
                            int64_t unit_stride, int64_t first_unit, int64_t n_units, int32_t len,
                            uint64_t seed, int32_t open_eighths, void* stream);

/* ---- device memory helpers (so hosts without a HIP binding can drive the device path) --- */
void* flacmi_device_alloc(flacmi_ctx* ctx, size_t bytes);
int flacmi_device_free(flacmi_ctx* ctx, void* ptr);
int flacmi_memcpy_h2d(flacmi_ctx* ctx, void* dst, const void* src, size_t bytes);
int flacmi_memcpy_d2h(flacmi_ctx* ctx, void* dst, const void* src, size_t bytes);
int flacmi_synchronize(flacmi_ctx* ctx);

/* ---- kernel timing (HIP events recorded on the stream each analyze call runs on) ----- */
/* Averages over the analyze calls since the last flacmi_timing_reset (up to 256 calls):
 * ms[0] k_lpc phase (autocorrelation + Levinson + quantisation), ms[1] k_resid phase
 * (residual sums + choice + Rice), ms[2] whole call, ms[3] number of calls averaged.
 * Synchronises on the recorded events; returns the number of values written. */
int flacmi_last_timing(flacmi_ctx* ctx, float* ms, int n);
int flacmi_timing_reset(flacmi_ctx* ctx);

/* ---- test and diagnostic knobs ---------------------------------------------------------- */
/* Process-wide knobs for A/B runs and tests, read from the environment once (the first time
 * any is used) and changed afterwards only through flacmi_set_knob, so no launch calls getenv
 * while another thread may change the environment.  Names: "FLACMI_OVERLAP" (analyze chunk
 * overlap: -1 round-aligned (default), 0 off, k > 1 equal chunks, -R R units per round),
 * "FLACMI_MF8_GRID" (cap on the int8-MFMA persistent grid, 0 = none), "FLACMI_STREAM_GENERIC"
 * (1 = the runtime-shape stream kernel for 4608-sample units), "FLACMI_DECODE_GENERIC" (1 =
 * every frame of flacmi_decode_frames_device through the general decoder kernel),
 * "FLACMI_PACK_GENERIC" (frame writer: 1 = every frame through the general writer kernel,
 * 2 = no ring-window writer (the one-window writer where a frame fits, else the general one),
 * 3 = the ring writer with 2048-value tiles, 6 / 8 = the ring writer built for 256 / 128
 * threads, 7 = as 2 with the one-window writer on its 16 KB window only).
 * FLACMI_E_INVALID for any other name.  No device needed. */
int flacmi_set_knob(const char* name, int32_t value);
int flacmi_get_knob(const char* name, int32_t* value);

/* ---- host-side views of the device arithmetic (for CPU verification of the helpers) ---- */
/* Python float `x ** 2` as CPython 3.10 + glibc 2.35 pow (FMA variant) computes it;
 * *status receives FLACMI_STATUS_OVERFLOW where Python raises OverflowError. */
double flacmi_host_pypow2(double x, int32_t* status);
/* floor(math.log2(x)) for finite x > 0, via the threshold table the device uses
 * (built once per process from libm log2); INT32_MIN for any other x. */
int32_t flacmi_host_floor_log2(double x);

/* The same helpers executed by the device kernels, over n host inputs (synchronous):
 * which = 0: out[i] = x[i] ** 2 (status[i] as flacmi_host_pypow2);
 * which = 1: out[i] = floor(log2(x[i])) for finite x[i] > 0. */
int flacmi_device_selftest(flacmi_ctx* ctx, int32_t which, const double* x, double* out,
                           int32_t* status, int64_t n);
/* k_lpc's Levinson-Durbin + quantiser (encoder.py:453-534) driven from n autocorrelation
 * rows acf[n][33] (lags 0..L used) instead of samples: rec[n][FLACMI_LPC_REC_WORDS(L)]
 * receives the LPC record k_lpc writes (word 0 = status | site << 16, word 1 = negative-shift
 * mask, then L shifts and the triangular coefficient table).  Reaches the overflow sites
 * (FLACMI_SITE_LEVINSON_POW, FLACMI_SITE_QUANT_LOG2) that no integer PCM block reaches
 * (DESIGN §4).  Synchronous; L in 1..32, q in 5..15. */
int flacmi_device_lpc_from_acf(flacmi_ctx* ctx, const double* acf, int64_t n, int32_t L, int32_t q,
                               int32_t* rec);

#ifdef __cplusplus
}
#endif
#endif /* FLACMI_H */
