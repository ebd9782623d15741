"""ctypes mirror of ``include/flacmi.h`` (the C-ABI of libflacmi.so).

Kept in one place so the product loader (``_lib.py``) and the test harness agree on
struct layouts.  Pure data definitions: importing this module loads no library.
"""
import ctypes as C

import numpy as np

ABI_VERSION = 2  # include/flacmi.h FLACMI_ABI_VERSION
MAX_LPC_ORDER = 32
MAX_BLOCK = 65535
MAX_RICE_ORDER = 15
STATS_WORDS = 128
# flacmi_error
E_INVALID, E_HIP, E_UNSUPPORTED, E_NOMEM = -1, -2, -3, -4


def lpc_rec_words(L: int) -> int:
    return 2 + L + (L * (L + 1)) // 2


# flacmi_status
STATUS_OK = 0
STATUS_ZERO_DIVISION = 1
STATUS_ASSERTION = 2
STATUS_VALUE_ERROR = 3
STATUS_OVERFLOW = 4
STATUS_RESIDUAL_WIDE = 16
STATUS_FRAME_TOO_LARGE = 17
STATUS_EOF = 5          # EOFError (decoder)
STATUS_VERIFY = 18      # decoder verifier finding, not a reference exception

STATUS_EXCEPTION = {
    STATUS_ZERO_DIVISION: ZeroDivisionError,
    STATUS_ASSERTION: AssertionError,
    STATUS_VALUE_ERROR: ValueError,
    STATUS_OVERFLOW: OverflowError,
    STATUS_EOF: EOFError,
}

# flacmi_site
SITE_NAMES = {
    0: "none",
    1: "tukey: float division by zero (encoder.py:437)",
    2: "levinson_durbin: float division by zero (encoder.py:469)",
    3: "levinson_durbin: lambda_ ** 2 overflow (encoder.py:476)",
    4: "quantize_lpc_coefficients: assert coef_max > 0.0 (encoder.py:496)",
    5: "quantize_lpc_coefficients: floor(log2(inf)) (encoder.py:503)",
    6: "quantize_lpc_coefficients: shift < shift_min (encoder.py:508)",
    7: "quantize_lpc_coefficients: round(inf) (encoder.py:520)",
    8: "quantize_lpc_coefficients: round(nan) (encoder.py:520)",
    9: "encode_subframe_lpc: min() arg is an empty sequence (encoder.py:404)",
    10: "encode: fixed and LPC residual sums tie (encoder.py:157)",
    11: "rice_partitions: no valid partition order (encoder.py:669)",
    12: "find_rice_parameter: math domain error (encoder.py:753)",
    13: "rice_size: negative shift count (encoder.py:758)",
    14: "residual does not fit the requested element width",
    15: "coded_number.encode: frame number needs more than 31 bits (coded_number.py:38)",
    16: "_put_subframe_lpc: assert precision - 1 != 0b1111 (encoder.py:619)",
    17: "frame of 2^28 bytes or more (not packed by this build)",
}

SITE_CHOICE_TIE = 10  # FLACMI_SITE_CHOICE_TIE

MODE_REFERENCE = 0
MODE_FIXED_ONLY = 1
MODE_LPC_ONLY = 2
MODE_RICE_ONLY = 3
KIND_FIXED = 0
KIND_LPC = 1
FLAG_ALL_CANDIDATES = 1  # params.reserved[1]: exact sums for every LPC candidate (no pruning)
FLAG_TIERS_ONLY = 2  # params.reserved[1]: prune with the partial-sum tiers alone (diagnostic)
LPC_PRUNED = -1          # meta.lpc_order / lpc_sum of a unit whose LPC candidates were pruned


class Params(C.Structure):
    _fields_ = [
        ("max_lpc_order", C.c_int32),
        ("qlp_precision", C.c_int32),
        ("rice_min", C.c_int32),
        ("rice_max", C.c_int32),
        ("mode", C.c_int32),
        ("reserved", C.c_int32 * 3),
    ]


class Batch(C.Structure):
    _fields_ = [
        ("samples", C.c_void_p),
        ("sample_bytes", C.c_int32),
        ("sample_bits", C.c_int32),
        ("unit_stride", C.c_int64),
        ("n_units", C.c_int64),
        ("block_len", C.c_int32),
        ("tail_len", C.c_int32),
        ("n_tail_units", C.c_int64),
    ]


class UnitMeta(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("site", C.c_int32),
        ("kind", C.c_int32),
        ("order", C.c_int32),
        ("shift", C.c_int32),
        ("ncoefs", C.c_int32),
        ("res_offset", C.c_int32),
        ("res_len", C.c_int32),
        ("fixed_order", C.c_int32),
        ("lpc_order", C.c_int32),
        ("part_order", C.c_int32),
        ("n_parts", C.c_int32),
        ("coding_method", C.c_int32),
        ("lpc_tiers", C.c_int32),
        ("fixed_sum", C.c_int64),
        ("lpc_sum", C.c_int64),
        ("rice_bits", C.c_int64),
        ("coefs", C.c_int32 * MAX_LPC_ORDER),
    ]


# numpy view of flacmi_unit_meta, for zero-copy access to a meta array
META_DTYPE = np.dtype([
    ("status", "<i4"), ("site", "<i4"), ("kind", "<i4"), ("order", "<i4"),
    ("shift", "<i4"), ("ncoefs", "<i4"), ("res_offset", "<i4"), ("res_len", "<i4"),
    ("fixed_order", "<i4"), ("lpc_order", "<i4"), ("part_order", "<i4"), ("n_parts", "<i4"),
    ("coding_method", "<i4"), ("lpc_tiers", "<i4"),
    ("fixed_sum", "<i8"), ("lpc_sum", "<i8"), ("rice_bits", "<i8"),
    ("coefs", "<i4", (MAX_LPC_ORDER,)),
])
assert META_DTYPE.itemsize == C.sizeof(UnitMeta) == 208


class Outputs(C.Structure):
    _fields_ = [
        ("meta", C.c_void_p),
        ("rice_params", C.c_void_p),
        ("params_stride", C.c_int64),
        ("residual", C.c_void_p),
        ("residual_bytes", C.c_int32),
        ("reserved0", C.c_int32),
        ("residual_stride", C.c_int64),
        ("acf", C.c_void_p),
        ("fixed_sums", C.c_void_p),
        ("lpc_sums", C.c_void_p),
        ("lpc_records", C.c_void_p),
    ]


class FrameParams(C.Structure):
    _fields_ = [
        ("channels", C.c_int32),
        ("sample_size", C.c_int32),
        ("qlp_precision", C.c_int32),
        ("reserved0", C.c_int32),
        ("first_frame", C.c_int64),
        ("reserved", C.c_int64 * 2),
    ]


class EncodeTiming(C.Structure):
    _fields_ = [
        ("wall_ms", C.c_double),
        ("h2d_ms", C.c_double),
        ("analyze_ms", C.c_double),
        ("sizes_ms", C.c_double),
        ("pack_ms", C.c_double),
        ("d2h_ms", C.c_double),
        ("register_ms", C.c_double),
        ("sub_batches", C.c_int64),
        ("bytes_in", C.c_int64),
        ("bytes_out", C.c_int64),
    ]


class DecodeParams(C.Structure):
    _fields_ = [
        ("channels", C.c_int32),
        ("sample_size", C.c_int32),
        ("first_frame", C.c_int64),
        ("check_crc", C.c_int32),
        ("reserved0", C.c_int32),
        ("reserved", C.c_int64 * 2),
    ]


# flacmi_decode_site (frame_status >> 16 of flacmi_decode_frames_device)
DSITE = {name: 32 + i for i, name in enumerate((
    "sync", "block_size_code", "sample_rate_code", "channels_code", "sample_size_code", "reserved",
    "subframe_pad", "subframe_type", "lpc_precision", "coding_method", "partitions", "escape_zero",
    "neg_shift", "padding", "eof", "crc8", "crc16", "frame_end", "frame_number", "block_size", "channels",
    "samples"))}


COMM_ID_BYTES = 128  # FLACMI_COMM_ID_BYTES

# Every symbol include/flacmi.h declares, with its ctypes signature.
SIGNATURES = {
    "flacmi_abi_version": (C.c_int, []),
    "flacmi_last_error": (C.c_char_p, []),
    "flacmi_device_count": (C.c_int, []),
    "flacmi_create": (C.c_void_p, [C.c_int]),
    "flacmi_destroy": (None, [C.c_void_p]),
    "flacmi_analyze_device": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Params),
                                        C.POINTER(Outputs), C.c_void_p]),
    "flacmi_analyze_host": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Params),
                                      C.POINTER(Outputs)]),
    "flacmi_frame_sizes_device": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(FrameParams), C.c_void_p,
                                            C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "flacmi_pack_frames_device": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(FrameParams), C.c_void_p,
                                            C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_int64, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "flacmi_encode_host": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Params), C.POINTER(FrameParams),
                                     C.c_void_p, C.c_void_p]),
    "flacmi_encode_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    "flacmi_encode_pipeline": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Params), C.POINTER(FrameParams),
                                         C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                         C.POINTER(EncodeTiming)]),
    "flacmi_host_register": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "flacmi_host_unregister": (C.c_int, [C.c_void_p, C.c_void_p]),
    "flacmi_host_alloc": (C.c_void_p, [C.c_void_p, C.c_size_t]),
    "flacmi_host_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "flacmi_decode_frames_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                              C.POINTER(DecodeParams), C.POINTER(Batch), C.c_void_p, C.c_int64,
                                              C.c_void_p, C.c_void_p, C.c_void_p]),
    "flacmi_stream_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                      C.c_int64, C.c_void_p, C.c_void_p]),
    "flacmi_comm_available": (C.c_int, []),
    "flacmi_unit_stride": (C.c_int64, [C.c_int32, C.c_int32]),
    "flacmi_comm_id": (C.c_int, [C.c_void_p]),
    "flacmi_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    "flacmi_allreduce_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "flacmi_comm_destroy": (C.c_int, [C.c_void_p]),
    "flacmi_synth_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64,
                                      C.c_int64, C.c_int64, C.c_int32, C.c_uint64, C.c_void_p]),
    "flacmi_synth_mix_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64,
                                          C.c_int64, C.c_int64, C.c_int32, C.c_uint64, C.c_int32, C.c_void_p]),
    "flacmi_device_alloc": (C.c_void_p, [C.c_void_p, C.c_size_t]),
    "flacmi_device_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "flacmi_memcpy_h2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "flacmi_memcpy_d2h": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "flacmi_synchronize": (C.c_int, [C.c_void_p]),
    "flacmi_last_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int]),
    "flacmi_timing_reset": (C.c_int, [C.c_void_p]),
    "flacmi_set_knob": (C.c_int, [C.c_char_p, C.c_int32]),
    "flacmi_get_knob": (C.c_int, [C.c_char_p, C.POINTER(C.c_int32)]),
    "flacmi_host_pypow2": (C.c_double, [C.c_double, C.POINTER(C.c_int32)]),
    "flacmi_host_floor_log2": (C.c_int32, [C.c_double]),
    "flacmi_device_selftest": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_int64]),
    "flacmi_device_lpc_from_acf": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                             C.c_void_p]),
}
