/*
 * flacmi_kernels.h — internal interface between the host driver (flacmi_host.cpp) and
 * the HIP kernels (flacmi_kernels.hip).  Not part of the public C-ABI.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flacmi.h"

namespace flacmi {

/* One launch = one "length class": units [unit0, unit0 + count) that all have length n. */
struct LpcArgs {
    const void* samples;     /* batch base pointer */
    int64_t stride;          /* elements between units */
    int64_t unit0, count;
    int32_t sample_bytes;
    int32_t n, L, q;
    const double* window;    /* [n] Tukey(0.5) window for this n (host libm cos) */
    const double* log2thr;   /* [PYM_LOG2_THR_N] floor(log2) thresholds */
    int32_t* rec;            /* [count][rec_words] LPC records (workspace) */
    int32_t rec_words;
    double* acf;             /* optional [count][33] */
    int32_t fuse_lo, fuse_hi; /* window[i] == 1.0 exactly for i in [fuse_lo, fuse_hi) and
                                 |x| < 2^26 (0, 0: no fused blocks), see k_lpc */
};

struct ResidArgs {
    const void* samples;
    int64_t stride;
    int64_t unit0, count;
    int32_t sample_bytes;
    int32_t n, L, mode;
    int32_t rmin, rmax;      /* rice range; rmax < rmin => empty */
    int32_t rice_order;      /* predictor order in FLACMI_MODE_RICE_ONLY */
    const int32_t* rec;      /* [count][rec_words] (NULL in fixed-only mode) */
    int32_t rec_words;
    const double* log2thr;
    flacmi_unit_meta* meta;  /* [count] */
    int32_t* rice_params;    /* [count][params_stride] */
    int64_t params_stride;
    void* residual;          /* [count][residual_stride] u32 or u64 */
    int64_t residual_stride;
    int64_t* fixed_sums;     /* optional [count][5] */
    int64_t* lpc_sums;       /* optional [count][32] */
    int32_t stop_after;      /* profiling ablation (env FLACMI_DEBUG_STOP): 0 = full kernel,
                                1 = after staging, 2 = after candidate sums, 3 = after the
                                choice, 4 = after the chosen residual (k_resid config-3
                                Rice phase: 5 = after the parameters, 6 = after the row
                                transform, 7 = after the data bits); k_resid_stream prune
                                mode: 11 = bound tier 0 only, 12 = no LPC bound (wrong
                                results, timing only) */
    int32_t mfma;            /* 1 = MFMA candidate sums where exact (env FLACMI_NO_MFMA=1 -> 0) */
    unsigned long long* retry_count; /* fast-path units handed to the generic kernel: count, */
    int64_t* retry_list;             /* and their batch indices (NULL: no fast path) */
    unsigned long long* retry2_count; /* k_resid_stream: the units its list kernel hands on to k_resid's */
    int64_t* retry2_list;             /* list variant (a second list of at most count entries) */
    unsigned long long* retry_sub;    /* k_resid_stream's batch kernel lists unit u in sub-list u & 63: its
                                         counter retry_sub[16 (u & 63)] (128 B apart), its entries
                                         retry_list[(u & 63) retry_sub_cap ..] (one counter for every
                                         workgroup serialised ~13 ns per listed unit at L2) */
    int64_t retry_sub_cap;
    int32_t sample_bits;             /* declared sample width (bounds the 64-bit paths' narrow sums) */
    int32_t stream;                  /* 1 = k_resid_stream where the shape allows (env FLACMI_NO_STREAM=1 -> 0) */
    int32_t prune;                   /* 1 = reference mode may skip the exact LPC candidate sums of a unit
                                        whose lower bounds already lose to the best fixed sum
                                        (meta lpc_order = lpc_sum = FLACMI_LPC_PRUNED) */
    int32_t persist;                 /* k_resid kVarMf8: the grid loops over the batch and copies the next
                                        unit's samples into LDS (LDS-DMA) during this unit's Rice phase */
    int32_t sign_bound;              /* int8-MFMA pruning: try the sign-correlation bound before the tiers */
};
/* internal unit status between the fast and the generic k_resid (never returned) */
#define FLACMI_STATUS_RETRY 0x7e

/* Frame writer (k_frame.hip): frame f = units [f*channels, (f+1)*channels). */
struct FrameArgs {
    const void* samples;     /* warm-up samples come from the batch rows */
    int64_t stride;
    int32_t sample_bytes;
    int32_t block_len, tail_len;
    int64_t n_units, n_tail_units;
    int32_t channels, sample_size, q;
    int64_t first_frame, n_frames;
    const flacmi_unit_meta* meta;
    const int32_t* rice_params;
    int64_t params_stride;
    const void* residual;
    int32_t residual_bytes;
    int64_t residual_stride;
    int64_t* offsets;        /* [n_frames + 1] */
    int32_t* status;         /* [n_frames] */
    uint8_t* out;
    int64_t capacity;
    const uint16_t* crc_slice; /* [4][256] CRC-16 slice-by-4 tables */
    const uint16_t* crc_pow;   /* [28][512] multiply-by-x^(8*2^b) tables */
    int32_t pack_split;        /* 1: k_pack32 writes the frames it can hold, k_pack the rest */
    unsigned long long* slow_count; /* pack_split: frames k_pack32 hands to k_pack: count, */
    int64_t* slow_list;              /* and their indices ([n_frames]) */
    int32_t ablate;            /* profiling only (env FLACMI_PACK_ABLATE): 1 no CRC shift, 2 no residual codes,
                                  3 neither (output invalid) */
};

/* Decoder verifier (k_decode.hip): frame f = bytes [offsets[f], offsets[f+1]) of words. */
struct DecodeArgs {
    const uint32_t* words;   /* the stream as dwords (4-byte aligned base) */
    int64_t stream_bytes, n_words;
    const int64_t* offsets;  /* [n_frames + 1] */
    int64_t n_frames;
    int32_t channels, sample_size;
    int64_t first_frame;
    int32_t check_crc;
    const void* expect;      /* optional source rows [n_frames*channels][expect_stride] */
    int64_t expect_stride;
    int32_t expect_bytes;
    int32_t expect_vec;      /* rows 16-byte aligned: the comparison uses 16-byte loads */
    int32_t block_len, tail_len;
    int64_t n_units, n_tail_units;
    int32_t* out;            /* optional [n_frames*channels][out_stride] */
    int64_t out_stride;
    int32_t* status;         /* [n_frames] */
    int64_t* mismatch;       /* [n_frames] */
    int32_t* decorr;         /* [n_frames] scratch: (bs << 8) | channel code for k_decorr, else 0 */
    const uint16_t* crc_slice; /* [4][256] CRC-16 slice-by-4 tables */
    unsigned long long* defer_count; /* frames k_decode_fx hands to k_decode: count, */
    int64_t* defer_list;             /* and their indices ([n_frames]) */
    int32_t defer_all;               /* knob FLACMI_DECODE_GENERIC: every frame through k_decode */
    unsigned long long* defer2_count; /* the frames k_decode_fx's LPC pass hands on: count, */
    int64_t* defer2_list;             /* and their indices ([n_frames]) */
    int32_t lpc_pass;                 /* k_decode_fx's LPC pass runs (env FLACMI_DECODE_LPC=0: off) */
};

struct ResidLaunch {
    int threads;             /* workgroup size (multiple of 64) */
    size_t lds_bytes;        /* dynamic LDS */
};

/* Launch configuration the residual kernel needs for (n, L, rice range, residual width). */
ResidLaunch resid_launch_config(int n, int rmax_eff, int residual_bytes);
/* Largest partition order the LDS tables support. */
constexpr int kMaxFinestParts = 4096;

/* flacmi_set_knob's knobs: the environment's value (read once) or the last value set */
enum Knob { kKnobOverlap = 0, kKnobMf8Grid, kKnobStreamGeneric, kKnobDecodeGeneric, kKnobPackGeneric, kKnobCount };
int knob(Knob k);

hipError_t launch_lpc(const LpcArgs& a, hipStream_t s);
/* units one full round of launch_lpc's kernel covers on the current device (resident
 * workgroups per CU x 256 units x CUs); 0 when the occupancy query fails */
int64_t lpc_units_per_round(const LpcArgs& a);
/* test knob: fill every CU's LDS with a pattern (env FLACMI_POISON_LDS), else nothing */
hipError_t launch_poison_lds(hipStream_t s);
/* copy nf + 1 frame offsets and nf statuses to mapped host memory (k_misc.hip) */
hipError_t launch_export(const int64_t* off, const int32_t* st, int64_t nf, int64_t* h_off, int32_t* h_st,
                         hipStream_t s);
/* k_lpc<32> with the autocorrelation read from a.acf (flacmi_device_lpc_from_acf) */
hipError_t launch_lpc_from_acf(const LpcArgs& a, hipStream_t s);
/* path: 0 = int16 samples / sdot2, 1 = int32 samples / mad24, 2 = int64 arithmetic */
hipError_t launch_resid(const ResidArgs& a, int path, int residual_bytes, hipStream_t s);
hipError_t launch_expand_records(const int32_t* rec, int32_t rec_words, int32_t L, int64_t count,
                                 int32_t* out, hipStream_t s);
hipError_t launch_synth(void* dst, int32_t sample_bytes, int32_t bits, int64_t stride,
                        int64_t first_unit, int64_t n_units, int32_t len, uint64_t seed,
                        const int32_t* sintab, int32_t open8, hipStream_t s);
hipError_t launch_stats(const flacmi_unit_meta* meta, int64_t n_units, int32_t block_len,
                        int32_t tail_len, int64_t n_tail_units, int64_t* stats, hipStream_t s);

/* frame sizes + exclusive scan into a.offsets; bsum: frame_scan_blocks(n_frames) words */
hipError_t launch_frame_sizes(const FrameArgs& a, int64_t* bsum, hipStream_t s);
int64_t frame_scan_blocks(int64_t n_frames);
hipError_t launch_pack(const FrameArgs& a, hipStream_t s);
hipError_t launch_decode(DecodeArgs a, hipStream_t s);

hipError_t launch_selftest(int32_t which, const double* x, double* out, int32_t* status, int64_t n,
                           const double* log2thr, hipStream_t s);

}  // namespace flacmi
