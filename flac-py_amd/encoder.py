"""flac-py's encoder interface (flac/encoder.py) on the MI355X analysis path.

`encode()` keeps the reference's signature and output bytes: it consumes the PCM
iterator in batches of blocks, analyses every (block, channel) unit on the GPU through
libflacmi.so (fixed predictors, Tukey/autocorrelation/Levinson/quantisation, all LPC
candidates, the subframe choice and the Rice partition search) and writes each frame on
the host.  Frames are yielded in block order; a unit the reference would fail on raises
the reference's exception at the same point of the stream.

`encode_subframe_fixed`, `encode_subframe_lpc` and `encode_residual` are the
single-unit forms of the same device analysis, returning the reference's dataclasses.
"""
from dataclasses import dataclass
from typing import Iterator, Optional

import numpy as np

from . import abi
from . import coded_number
from ._lib import FlacmiError
from .analysis import Analyzer, make_params, params_stride_for
from .binary import Put
from .common import (
    CHANNELS_ENCODING, CRC8_POLYNOMIAL, FRAME_SYNC_CODE, MAGIC,
    BLOCK_SIZE_ENCODING, BlockingStrategy, Channels, FrameHeader, MetadataBlockHeader,
    MetadataBlockType, Residual, RiceCodingMethod, RicePartition, Streaminfo, SubframeFixed,
    SubframeHeader, SubframeLPC, SubframeTypeFixed, SubframeTypeLPC,
)
from .crc import crc8
from .utils import batch

__all__ = ["EncoderParameters", "encode", "encode_planar", "encode_wav", "encode_subframe_fixed", "encode_subframe_lpc",
           "encode_residual", "put_frame_header", "put_metadata_block_header",
           "put_metadata_block_streaminfo"]


@dataclass
class EncoderParameters:
    """Same contract as flac/encoder.py:33-43."""
    block_size: int
    rice_partition_order: range
    lpc_order: range
    qlp_precision: int

    def __post_init__(self):
        assert self.lpc_order.start == 0
        assert self.lpc_order.stop <= 33
        assert self.qlp_precision >= 5


_ANALYZERS = {}


def _analyzer(device: int) -> Analyzer:
    if device not in _ANALYZERS:
        _ANALYZERS[device] = Analyzer(device)
    return _ANALYZERS[device]


# ---------------------------------------------------------------------------------
# the reference's exceptions, by flacmi_site
# ---------------------------------------------------------------------------------
_SITE_EXCEPTION = {
    1: (ZeroDivisionError, "float division by zero"),
    2: (ZeroDivisionError, "float division by zero"),
    3: (OverflowError, "(34, 'Numerical result out of range')"),
    4: (AssertionError, ""),
    5: (OverflowError, "cannot convert float infinity to integer"),
    6: (AssertionError, ""),
    7: (OverflowError, "cannot convert float infinity to integer"),
    8: (ValueError, "cannot convert float NaN to integer"),
    9: (ValueError, "min() arg is an empty sequence"),
    10: (AssertionError, ""),
    11: (AssertionError, ""),
    12: (ValueError, "math domain error"),
    13: (ValueError, "negative shift count"),
    15: (ValueError, "Cannot encode coded number"),
    16: (AssertionError, ""),
}


def _raise_status(st: int, site: int) -> None:
    if st == abi.STATUS_OK:
        return
    if st == abi.STATUS_FRAME_TOO_LARGE:
        raise FlacmiError(abi.SITE_NAMES[17])
    exc, msg = _SITE_EXCEPTION.get(site, (abi.STATUS_EXCEPTION.get(st, RuntimeError), ""))
    raise exc(msg) if msg else exc()


def _raise_for(meta_row) -> None:
    _raise_status(int(meta_row["status"]), int(meta_row["site"]))


def _rice_range(r: range):
    if r.step != 1:
        raise ValueError("rice_partition_order must be a contiguous range")
    return r.start, r.stop - 1


def _sample_bits(a: np.ndarray) -> int:
    if a.size == 0:
        return 2
    m = int(max(-int(a.min()), int(a.max()), 1))
    return max(2, m.bit_length() + 1)


def _planar(blocks, channels: int, block_len: int):
    """List of blocks (lists of frames) -> int16/int32 [n_blocks*channels][stride] rows."""
    nb = len(blocks)
    tail_len = len(blocks[-1])
    rows = np.zeros((nb * channels, block_len), dtype=np.int64)
    for b, xs in enumerate(blocks):
        a = np.asarray([x[:channels] for x in xs], dtype=np.int64).reshape(len(xs), channels)
        rows[b * channels:(b + 1) * channels, :len(xs)] = a.T
    bits = _sample_bits(rows)
    dt = np.int16 if bits <= 16 else np.int32
    stride = ((block_len * np.dtype(dt).itemsize + 15) // 16) * 16 // np.dtype(dt).itemsize
    out = np.zeros((nb * channels, stride), dtype=dt)
    out[:, :block_len] = rows
    n_tail = channels if tail_len != block_len else 0
    return out, bits, tail_len, n_tail


# ---------------------------------------------------------------------------------
# stream and frame writers (flac/encoder.py:170-320, 553-628, 765-806)
# ---------------------------------------------------------------------------------
def put_metadata_block_header(header: MetadataBlockHeader) -> Put:
    put = Put()
    put.bool(header.last)
    put.uint(header.type.value, 7)
    put.uint(header.length, 24)
    return put


def put_metadata_block_streaminfo(si: Streaminfo) -> Put:
    put = Put()
    for value, width in ((si.min_block_size, 16), (si.max_block_size, 16), (si.min_frame_size, 24),
                         (si.max_frame_size, 24), (si.sample_rate, 20), (si.channels - 1, 3),
                         (si.sample_size - 1, 5), (si.samples, 36)):
        put.uint(value, width)
    put.bytes(si.md5)
    return put


def put_frame_header(header: FrameHeader) -> Put:
    """Frame header as the reference writes it from encode(): sample rate and sample size
    'from STREAMINFO' (None), 8/16-bit explicit block size when it has no code."""
    put = Put()
    put.uint(FRAME_SYNC_CODE, 15)
    put.uint(header.blocking_strategy.value, 1)
    bs = header.block_size
    code = BLOCK_SIZE_ENCODING.get(bs)
    if code is None:
        if 0 < bs.bit_length() <= 8:
            code = 0b0110
        elif 8 < bs.bit_length() <= 16:
            code = 0b0111
        else:
            raise ValueError(f"Cannot encode block size: {bs}")
    put.uint(code, 4)
    if header.sample_rate is not None or header.sample_size is not None:
        raise NotImplementedError("explicit frame sample rate/size (encode() never writes them)")
    put.uint(0b0000, 4)
    put.uint(CHANNELS_ENCODING[header.channels], 4)
    put.uint(0b000, 3)
    put.uint(0, 1)
    put.bytes(coded_number.encode(header.coded_number))
    if code == 0b0110:
        put.uint(bs - 1, 8)
    elif code == 0b0111:
        put.uint(bs - 1, 16)
    put.uint(crc8(put.buffer, CRC8_POLYNOMIAL), 8)
    return put


def encode(sample_rate: int, sample_size: int, channels: int, frames: int,
           samples: Iterator[list], parameters: EncoderParameters, *, device: int = 0,
           blocks_per_batch: int = 2048, fixed_only: bool = False) -> Iterator[bytes]:
    """flac/encoder.py:48-165 on the GPU: the per-channel analysis (k_lpc, k_resid) and
    the frame writer (k_frame.hip: Rice packing, headers, CRC-8/16).  Only the stream
    header (magic + STREAMINFO) is written here.

    fixed_only=True selects fixed predictors only (BASELINE config 5); the reference
    has no such mode (its -l 0 raises ValueError, which the default mode reproduces)."""
    if sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(sample_rate, sample_size, channels, frames, parameters)
    rmin, rmax = _rice_range(parameters.rice_partition_order)
    L = parameters.lpc_order.stop - 1
    mode = abi.MODE_FIXED_ONLY if fixed_only else abi.MODE_REFERENCE
    params = make_params(L, parameters.qlp_precision, rmin, rmax, mode)
    az = _analyzer(device)
    index = 0
    blocks_iter = batch(samples, parameters.block_size)
    pending = []
    for blk in blocks_iter:
        pending.append(blk)
        if len(pending) < blocks_per_batch:
            continue
        yield from _encode_batch(az, pending, index, channels, sample_size, parameters, params)
        index += len(pending)
        pending = []
    if pending:
        yield from _encode_batch(az, pending, index, channels, sample_size, parameters, params)


def encode_planar(sample_rate: int, sample_size: int, pcm: np.ndarray, parameters: EncoderParameters, *,
                  frames: Optional[int] = None, device: int = 0, blocks_per_batch: int = 8192,
                  fixed_only: bool = False) -> Iterator[bytes]:
    """encode() over planar PCM (int [channels][frames], e.g. from ingest.read_wav): the
    same bytes as encode(sample_rate, sample_size, channels, frames, <the frames of pcm>,
    parameters), without building a Python list per frame.  Blocks go to the device in
    batches of blocks_per_batch (ingest.planar_blocks)."""
    from .ingest import planar_blocks
    channels, total = pcm.shape
    if sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(sample_rate, sample_size, channels, total if frames is None else frames,
                              parameters)
    rmin, rmax = _rice_range(parameters.rice_partition_order)
    mode = abi.MODE_FIXED_ONLY if fixed_only else abi.MODE_REFERENCE
    params = make_params(parameters.lpc_order.stop - 1, parameters.qlp_precision, rmin, rmax, mode)
    az = _analyzer(device)
    n = parameters.block_size
    nb = (total + n - 1) // n
    for b0 in range(0, nb, blocks_per_batch):
        rows, bits, tail_len, n_tail = planar_blocks(pcm, n, b0, blocks_per_batch)
        data, offsets, status = az.encode_frames(rows, params, n, tail_len, n_tail, sample_bits=bits,
                                                 channels=channels, sample_size=sample_size, first_frame=b0)
        buf = data.tobytes()
        for b in range(rows.shape[0] // channels):
            st = int(status[b])
            _raise_status(st & 0xFFFF, st >> 16)
            yield buf[int(offsets[b]):int(offsets[b + 1])]


def encode_wav(path, parameters: EncoderParameters, *, quirk: bool = True, device: int = 0,
               blocks_per_batch: int = 8192, fixed_only: bool = False) -> Iterator[bytes]:
    """The reference CLI's encode action (flac/__main__.py:58-109) on a WAV file, streamed:
    the stream header first, then frames batch by batch (ingest.iter_wav_batches), so the
    host holds one batch of PCM at a time.  A reader failure (the reference's IndexError on
    its byte grouping, encoder.py:102) is raised after the stream header, as the reference
    CLI has written it by then."""
    from .ingest import iter_wav_batches, wav_info
    info = wav_info(path)
    if info.sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(info.sample_rate, info.sample_width * 8, info.channels, info.frames, parameters)
    rmin, rmax = _rice_range(parameters.rice_partition_order)
    mode = abi.MODE_FIXED_ONLY if fixed_only else abi.MODE_REFERENCE
    params = make_params(parameters.lpc_order.stop - 1, parameters.qlp_precision, rmin, rmax, mode)
    n, C = parameters.block_size, info.channels
    for b0, rows, bits, tail_len, n_tail in iter_wav_batches(path, n, blocks_per_batch, quirk):
        az = _analyzer(device)  # after the first batch is read: a reader failure needs no device
        data, offsets, status = az.encode_frames(rows, params, n, tail_len, n_tail, sample_bits=bits,
                                                 channels=C, sample_size=info.sample_width * 8, first_frame=b0)
        buf = data.tobytes()
        for b in range(rows.shape[0] // C):
            st = int(status[b])
            _raise_status(st & 0xFFFF, st >> 16)
            yield buf[int(offsets[b]):int(offsets[b + 1])]


def _stream_header(sample_rate, sample_size, channels, frames, parameters):
    yield MAGIC
    yield put_metadata_block_header(
        MetadataBlockHeader(last=True, type=MetadataBlockType.Streaminfo, length=34)).buffer
    yield put_metadata_block_streaminfo(Streaminfo(
        min_block_size=parameters.block_size, max_block_size=parameters.block_size,
        min_frame_size=0, max_frame_size=0, sample_rate=sample_rate, channels=channels,
        sample_size=sample_size, samples=frames, md5=bytes(16))).buffer


def _encode_batch(az, blocks, index0, channels, sample_size, parameters, params):
    n = parameters.block_size
    rows, bits, tail_len, n_tail = _planar(blocks, channels, n)
    data, offsets, status = az.encode_frames(rows, params, n, tail_len, n_tail, sample_bits=bits,
                                             channels=channels, sample_size=sample_size, first_frame=index0)
    buf = data.tobytes()
    for b in range(len(blocks)):
        st = int(status[b])
        _raise_status(st & 0xFFFF, st >> 16)  # the reference raises after the frames before it
        yield buf[int(offsets[b]):int(offsets[b + 1])]


# ---------------------------------------------------------------------------------
# single-unit forms (the reference's function-level interface)
# ---------------------------------------------------------------------------------
def _one(samples, params, bits=None):
    xs = np.asarray(samples, dtype=np.int64)
    n = len(xs)
    bits = bits or _sample_bits(xs)
    dt = np.int16 if bits <= 16 else np.int32
    stride = max(8, ((n * np.dtype(dt).itemsize + 15) // 16) * 16 // np.dtype(dt).itemsize)
    row = np.zeros((1, stride), dtype=dt)
    row[0, :n] = xs
    out = _analyzer(0).analyze(row, params, n, sample_bits=bits)
    return out, out["meta"][0]


def encode_subframe_fixed(samples: list):
    """flac/encoder.py:331-359 -> (SubframeHeader, SubframeFixed)."""
    out, m = _one(samples, make_params(0, 5, 0, -1, abi.MODE_FIXED_ONLY))
    if int(m["status"]) not in (abi.STATUS_OK, abi.STATUS_ASSERTION):
        _raise_for(m)
    order = int(m["fixed_order"])
    off = 0 if len(samples) <= 4 else order
    # the fixed residual is the chosen row; the empty Rice range only skips the search
    zz = out["residual"][0][off:len(samples)].astype(np.int64)
    residual = [int(v) for v in (zz >> 1) ^ -(zz & 1)]
    return (SubframeHeader(SubframeTypeFixed(order=order), 0),
            SubframeFixed(list(samples[:order]), residual))


def encode_subframe_lpc(samples: list, lpc_order: range, precision: int):
    """flac/encoder.py:362-420 -> (SubframeHeader, SubframeLPC)."""
    L = lpc_order.stop - 1
    if L < 1:
        raise ValueError("min() arg is an empty sequence")
    out, m = _one(samples, make_params(L, precision, 0, -1, abi.MODE_LPC_ONLY))
    _raise_for(m)
    order = int(m["order"])
    off, ln = int(m["res_offset"]), int(m["res_len"])
    zz = out["residual"][0][off:off + ln].astype(np.int64)
    residual = [int(v) for v in (zz >> 1) ^ -(zz & 1)]
    return (SubframeHeader(SubframeTypeLPC(order=order), 0),
            SubframeLPC(warmup=list(samples[:order]), precision=precision, shift=int(m["shift"]),
                        coefficients=[int(c) for c in m["coefs"][: int(m["ncoefs"])]],
                        residual=residual))


def encode_residual(samples: list, block_size: int, sample_size: int, predictor_order: int,
                    partition_order_range: range) -> Residual:
    """flac/encoder.py:632-652 on a residual list of block_size - predictor_order values."""
    if len(samples) != block_size - predictor_order:
        raise NotImplementedError("residual length must be block_size - predictor_order")
    rmin, rmax = _rice_range(partition_order_range)
    row = [0] * predictor_order + list(samples)
    p = make_params(0, 5, rmin, rmax, abi.MODE_RICE_ONLY)
    p.reserved[0] = predictor_order
    out, m = _one(row, p)
    _raise_for(m)
    off, ln = int(m["res_offset"]), int(m["res_len"])
    zz = out["residual"][0][off:off + ln]
    po, n_parts = int(m["part_order"]), int(m["n_parts"])
    ps = block_size >> po
    lens = [ps - predictor_order] + [ps] * (n_parts - 1)
    parts, pos = [], 0
    for prm, l_ in zip(out["rice_params"][0][:n_parts], lens):
        parts.append(RicePartition(int(prm), [int(v) for v in zz[pos:pos + l_]]))
        pos += l_
    method = RiceCodingMethod.Rice5Bit if int(m["coding_method"]) == 5 else RiceCodingMethod.Rice4Bit
    return Residual(method, parts)
