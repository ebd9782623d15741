/*
 * flac_oracle.h — CPU restatement of turlando/flac-py's encode-analysis hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this code, and only as the checker / the timed CPU
 * baseline.  The product (flac-py_amd/, libflacmi.so) never links or calls it.
 *
 * Parity is pinned by golden vectors produced by importing the reference itself
 * (tests/golden/make_golden.py writes the JSON fixtures); see tests/test_oracle_golden.py.
 */
#ifndef FLAC_ORACLE_H
#define FLAC_ORACLE_H
#include <stdint.h>
#include "../include/flacmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Analyse one unit exactly as encode() does for one channel of one block
 * (encoder.py:127-157 plus encode_residual from the writer at :588/:608).
 * samples: n ints.  Outputs mirror flacmi_outputs for a single unit.
 * residual: n uint64 zig-zag values (row layout as in flacmi: [res_offset, res_offset+res_len)).
 * rice_params: >= 2^rice_max + 1 ints.  acf: 33 doubles, fixed_sums: 5, lpc_sums: 32,
 * lpc_record: FLACMI_LPC_REC_WORDS(32) ints.  Any debug pointer may be NULL. */
int oracle_analyze_unit(const int64_t* samples, int32_t n, const flacmi_params* p,
                        flacmi_unit_meta* meta, int32_t* rice_params, uint64_t* residual,
                        double* acf, int64_t* fixed_sums, int64_t* lpc_sums, int32_t* lpc_record);

/* Batch over planar int16/int32 units with the flacmi_batch layout, using `threads` pthreads.
 * Output layouts as flacmi_outputs (residual element width 8 bytes). */
int oracle_analyze_batch(const flacmi_batch* b, const flacmi_params* p, flacmi_unit_meta* meta,
                         int32_t* rice_params, int64_t params_stride, uint64_t* residual,
                         int64_t residual_stride, double* acf, int64_t* fixed_sums,
                         int64_t* lpc_sums, int32_t* lpc_records, int threads);

/* Individual reference functions, for localising mismatches. */
int oracle_tukey(int32_t n, double* w);                               /* encoder.py:423-440 */
double oracle_autocorrelation(const double* x, int32_t n, int32_t lag); /* encoder.py:443-450 */
int oracle_levinson(const double* r, int32_t order, double* coefs, int32_t* site); /* :453-479 */
int oracle_quantize(const double* c, int32_t n, int32_t precision, int32_t* q,
                    int32_t* nq, int32_t* shift, int32_t* site);        /* encoder.py:482-534 */
double oracle_pypow2(double x, int32_t* status);                       /* float ** 2 */
int32_t oracle_floor_log2(double x, int32_t* status);                   /* floor(math.log2(x)) */

/* Synthetic signal, bit-identical to flacmi_synth_device. */
void oracle_synth_unit(int64_t unit, int32_t len, int32_t bits, uint64_t seed, int32_t* out);
/* ... with open_eighths / 8 of the units MA(1) near-white noise (flacmi_synth_mix_device) */
void oracle_synth_unit_mix(int64_t unit, int32_t len, int32_t bits, uint64_t seed, int32_t open_eighths,
                           int32_t* out);

#ifdef __cplusplus
}
#endif
#endif
