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
import collections
import concurrent.futures
import functools
import threading
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence

import numpy as np

from . import abi
from . import coded_number
from ._lib import FlacmiError
from .analysis import Analyzer, make_params, params_stride_for, unit_stride
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


def _planar(blocks, channels: int, block_len: int, alloc=None):
    """List of blocks (lists of frames) -> int16/int32 [n_blocks*channels][stride] rows
    (in alloc(shape, dtype)'s memory when given)."""
    nb = len(blocks)
    tail_len = len(blocks[-1])
    rows = np.zeros((nb * channels, block_len), dtype=np.int64)
    for b, xs in enumerate(blocks):
        a = np.asarray([x[:channels] for x in xs], dtype=np.int64).reshape(len(xs), channels)
        rows[b * channels:(b + 1) * channels, :len(xs)] = a.T
    bits = _sample_bits(rows)
    dt = np.int16 if bits <= 16 else np.int32
    stride = unit_stride(block_len, np.dtype(dt).itemsize)
    if alloc is None:
        out = np.zeros((nb * channels, stride), dtype=dt)
    else:
        out = alloc((nb * channels, stride), dt)
        out[:, block_len:] = 0
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
           devices: Optional[Sequence[int]] = None, blocks_per_batch: int = 2048,
           fixed_only: bool = False) -> Iterator[bytes]:
    """flac/encoder.py:48-165 on the GPU: the per-channel analysis (k_lpc, k_resid) and
    the frame writer (k_frame.hip: Rice packing, headers, CRC-8/16), streamed through
    flacmi_encode_pipeline.  Only the stream header (magic + STREAMINFO) is written here.

    devices: encode on several devices (or several contexts of one device: [0, 0]); the
    batches go round-robin to one worker per entry and the frames come back in block
    order, byte-identical to one device.  fixed_only=True selects fixed predictors only
    (BASELINE config 5); the reference has no such mode (its -l 0 raises ValueError, which
    the default mode reproduces)."""
    if sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(sample_rate, sample_size, channels, frames, parameters)
    params = _params(parameters, fixed_only)
    n = parameters.block_size

    def batches():
        index = 0
        pending = []
        for blk in batch(samples, n):
            pending.append(blk)
            if len(pending) == blocks_per_batch:
                yield index, functools.partial(_planar, pending, channels, n)
                index += len(pending)
                pending = []
        if pending:
            yield index, functools.partial(_planar, pending, channels, n)

    yield from _drive(batches(), lambda: _sessions(device, devices), params, n, channels, sample_size)


def encode_planar(sample_rate: int, sample_size: int, pcm: np.ndarray, parameters: EncoderParameters, *,
                  frames: Optional[int] = None, device: int = 0, devices: Optional[Sequence[int]] = None,
                  blocks_per_batch: int = 0, fixed_only: bool = False) -> Iterator[bytes]:
    """encode() over planar PCM (int [channels][frames], e.g. from ingest.read_wav): the
    same bytes as encode(sample_rate, sample_size, channels, frames, <the frames of pcm>,
    parameters), without building a Python list per frame.  Blocks are cut straight into
    page-locked staging rows (ingest.planar_blocks) in batches of blocks_per_batch (0: about
    256 MB of samples) and streamed through flacmi_encode_pipeline; devices as encode()."""
    from .ingest import planar_blocks
    channels, total = pcm.shape
    if sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(sample_rate, sample_size, channels, total if frames is None else frames,
                              parameters)
    params = _params(parameters, fixed_only)
    n = parameters.block_size
    nb = (total + n - 1) // n
    bpb = blocks_per_batch or _default_blocks(n, channels)

    def batches():
        for b0 in range(0, nb, bpb):
            yield b0, functools.partial(planar_blocks, pcm, n, b0, bpb)

    yield from _drive(batches(), lambda: _sessions(device, devices), params, n, channels, sample_size)


def encode_wav(path, parameters: EncoderParameters, *, quirk: bool = True, device: int = 0,
               devices: Optional[Sequence[int]] = None, blocks_per_batch: int = 0,
               fixed_only: bool = False) -> Iterator[bytes]:
    """The reference CLI's encode action (flac/__main__.py:58-109) on a WAV file, streamed:
    the stream header first, then frames batch by batch (ingest.iter_wav_pcm), so the host
    holds a bounded number of batches of PCM.  A reader failure (the reference's IndexError
    on its byte grouping, encoder.py:102) is raised after the stream header and the frames
    of the batches before it, as the reference CLI has written them by then."""
    from .ingest import iter_wav_pcm, planar_blocks, wav_info
    info = wav_info(path)
    if info.sample_rate <= 48_000:
        assert parameters.lpc_order.stop <= 13
    yield from _stream_header(info.sample_rate, info.sample_width * 8, info.channels, info.frames, parameters)
    params = _params(parameters, fixed_only)
    n, C = parameters.block_size, info.channels
    bpb = blocks_per_batch or _default_blocks(n, C)

    def batches():
        for b0, pcm in iter_wav_pcm(path, n, bpb, quirk):
            yield b0, functools.partial(planar_blocks, pcm, n)

    # sessions are opened after the first batch is read: a reader failure needs no device
    yield from _drive(batches(), lambda: _sessions(device, devices), params, n, C, info.sample_width * 8)


def _stream_header(sample_rate, sample_size, channels, frames, parameters):
    yield MAGIC
    yield put_metadata_block_header(
        MetadataBlockHeader(last=True, type=MetadataBlockType.Streaminfo, length=34)).buffer
    yield put_metadata_block_streaminfo(Streaminfo(
        min_block_size=parameters.block_size, max_block_size=parameters.block_size,
        min_frame_size=0, max_frame_size=0, sample_rate=sample_rate, channels=channels,
        sample_size=sample_size, samples=frames, md5=bytes(16))).buffer


def _params(parameters: EncoderParameters, fixed_only: bool) -> abi.Params:
    rmin, rmax = _rice_range(parameters.rice_partition_order)
    mode = abi.MODE_FIXED_ONLY if fixed_only else abi.MODE_REFERENCE
    return make_params(parameters.lpc_order.stop - 1, parameters.qlp_precision, rmin, rmax, mode)


# ---------------------------------------------------------------------------------
# streaming driver: page-locked staging, flacmi_encode_pipeline, one worker per device
# ---------------------------------------------------------------------------------
_BATCH_BYTES = 256 << 20   # samples per batch (about): one pipeline call's worth of PCM
_SUB_UNITS = 8192          # units per pipeline sub-batch (the copies of one overlap the others' kernels)


def _default_blocks(block_size: int, channels: int) -> int:
    return max(1, _BATCH_BYTES // (4 * max(block_size, 1) * max(channels, 1)))


class _Session:
    """One encode context (one flacmi_ctx on `device`): two page-locked staging buffers
    for sample rows (the host cuts batch k + 1 into one while the device encodes batch k
    from the other), a page-locked frame buffer and one worker thread, all reused batch
    after batch."""

    def __init__(self, device: int):
        self.az = Analyzer(device)
        self.stage = [None, None]
        self.out = None
        self.pool = concurrent.futures.ThreadPoolExecutor(1)

    def staging(self, slot: int, shape, dtype) -> np.ndarray:
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        buf = self.stage[slot]
        if buf is None or buf.size < nbytes:
            buf = self.stage[slot] = self.az.host_array((max(nbytes, 1),), np.uint8)
        return buf[:nbytes].view(dtype).reshape(shape)

    def encode(self, rows, bits, tail_len, n_tail, params, n, channels, sample_size, first_frame):
        """-> (frame bytes, offsets, status) of one batch (host copies: the buffers are reused)."""
        cap = int(rows.shape[0] * (n * rows.itemsize * 1.25 + 256)) + (1 << 20)
        while True:
            if self.out is None or self.out.size < cap:
                self.out = None
                self.out = self.az.host_array((cap,), np.uint8)
            try:
                data, offsets, status, _ = self.az.encode_pipeline(
                    rows, params, n, tail_len, n_tail, sample_bits=bits, channels=channels,
                    sample_size=sample_size, first_frame=first_frame, units_per_batch=_SUB_UNITS,
                    out=self.out)
            except FlacmiError as e:
                if e.code == abi.E_NOMEM:
                    cap = 2 * max(cap, self.out.size)
                    continue
                raise
            return data.tobytes(), offsets, status

    def close(self) -> None:
        self.pool.shutdown(wait=True)
        self.stage = [None, None]
        self.out = None
        self.az.close()


_IDLE = collections.defaultdict(list)   # device -> sessions no running encode holds
_IDLE_LOCK = threading.Lock()
# idle sessions kept per device: a burst of concurrent or interleaved generators creates one
# session each, and each holds a context, pinned staging and frame buffers and a worker
# thread, so the sessions beyond this many are closed when they come back
_IDLE_MAX = 2


def _sessions(device: int, devices: Optional[Sequence[int]]):
    """Check out one session per entry of devices (an entry repeated: another context on
    that device).  A session belongs to one _drive call at a time: its staging slots are
    written by the generator while its worker copies the previous batch from them, so two
    generators on one device (interleaved, or on two threads) get two sessions.  _drive
    returns them when it finishes or is closed."""
    ds = [int(d) for d in (list(devices) if devices else [device])]
    if not ds:
        raise ValueError("devices is empty")
    with _IDLE_LOCK:
        out = [_IDLE[d].pop() if _IDLE[d] else None for d in ds]
    try:
        for k, d in enumerate(ds):
            if out[k] is None:
                out[k] = _Session(d)
    except BaseException:
        _release([s for s in out if s is not None])
        raise
    return out


def _release(sessions) -> None:
    extra = []
    with _IDLE_LOCK:
        for s in sessions:
            pool = _IDLE[s.az.device]
            (pool if len(pool) < _IDLE_MAX else extra).append(s)
    for s in extra:
        s.close()


def _drive(batches, sessions, params, n, channels, sample_size) -> Iterator[bytes]:
    """batches yields (first_block, cut) with cut(alloc=...) -> (rows, bits, tail_len,
    n_tail_units); batch i goes to sessions[i % D].  Frames are yielded in block order; a
    frame the reference would fail on raises its exception after the frames before it, and
    an exception from `batches` itself (the WAV reader) after every earlier batch's frames.
    sessions (a list from _sessions, or a callable returning one) are held until the
    generator ends or is closed, after every queued batch has finished with them."""
    queue = collections.deque()
    failure = None
    it = iter(batches)
    held = None
    i = 0
    try:
        while True:
            try:
                item = next(it)
            except StopIteration:
                break
            except Exception as e:  # the reader's failure surfaces in stream order
                failure = e
                break
            if held is None:
                held = sessions() if callable(sessions) else sessions
            D = len(held)
            while len(queue) >= 2 * D:  # batch i reuses the staging slot of batch i - 2D
                yield from _frames(*queue.popleft().result())
            first_block, cut = item
            s, slot = held[i % D], (i // D) % 2
            try:
                rows, bits, tail_len, n_tail = cut(alloc=functools.partial(s.staging, slot))
            except Exception as e:
                failure = e
                break
            queue.append(s.pool.submit(s.encode, rows, bits, tail_len, n_tail, params, n, channels, sample_size,
                                       first_block))
            i += 1
        while queue:
            yield from _frames(*queue.popleft().result())
        if failure is not None:
            raise failure
    finally:
        for f in queue:  # closed early: the workers may still read the staging slots
            concurrent.futures.wait([f])
        if held is not None:
            _release(held)
        elif not callable(sessions):
            _release(sessions)


def _frames(buf: bytes, offsets: np.ndarray, status: np.ndarray) -> Iterator[bytes]:
    for b in range(len(status)):
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
    stride = max(8, unit_stride(n, np.dtype(dt).itemsize))
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
