"""PCM ingest: WAV file -> planar device-ready unit rows, vectorised.

The reference reads a WAV one frame at a time (flac/__main__.py:82-92): `readframes(1)`,
then `group(xs, channels)` (utils.py:61-66) splits the frame's bytes into chunks of
`channels` bytes, each read as a little-endian signed int, and encode() takes
`x[c] for c in range(channels)` (encoder.py:102) — chunks of `channels` bytes, not of
`sampwidth` bytes.  For 16-bit stereo the two coincide; for mono 16-bit every sample
becomes the int8 of its low byte; with sampwidth < channels the reference raises
IndexError.  `quirk=True` (the default, as the reference CLI does) reproduces exactly
that; `quirk=False` reads each channel's sampwidth-byte little-endian signed sample (8-bit
WAV samples are unsigned with a 128 offset).

Blocks are then cut as utils.batch (utils.py:31-40) does — `block_size` frames each, the
last one short — and laid out as the C-ABI's planar units: row b*channels + c holds
channel c of block b (flacmi_batch in include/flacmi.h).  iter_wav_batches reads a file
batch by batch through the stdlib wave reader, so memory stays bounded by one batch.
"""
import wave
from dataclasses import dataclass

import numpy as np

from .analysis import unit_stride


@dataclass
class PcmInfo:
    sample_rate: int
    sample_width: int      # bytes per sample in the file
    channels: int
    frames: int


def _le_signed(cols: np.ndarray) -> np.ndarray:
    """[n][k] uint8 little-endian byte groups -> int64 signed values (int.from_bytes)."""
    k = cols.shape[1]
    v = np.zeros(cols.shape[0], dtype=np.int64)
    for j in range(k):
        v |= cols[:, j].astype(np.int64) << (8 * j)
    sign = np.int64(1) << (8 * k - 1)
    return (v ^ sign) - sign


def frames_to_channels(raw: bytes, channels: int, width: int, quirk: bool = True) -> np.ndarray:
    """Raw interleaved frame bytes -> int64 [channels][n_frames] as encode() sees them."""
    fb = channels * width
    a = np.frombuffer(raw, dtype=np.uint8)
    if a.size % fb:
        raise AssertionError("len(xs) == channels * sample_size_bytes")  # __main__.py:89
    a = a.reshape(-1, fb)
    if quirk:
        chunk = channels  # group(xs, channels): chunks of `channels` bytes
        n_chunks = (fb + chunk - 1) // chunk
        if n_chunks < channels:
            raise IndexError("list index out of range")  # encoder.py:102 x[c]
        return np.stack([_le_signed(a[:, c * chunk:min((c + 1) * chunk, fb)]) for c in range(channels)])
    if width == 1:  # WAV 8-bit PCM is unsigned with a 128 offset
        return np.stack([a[:, c].astype(np.int64) - 128 for c in range(channels)])
    return np.stack([_le_signed(a[:, c * width:(c + 1) * width]) for c in range(channels)])


def wav_info(path) -> PcmInfo:
    with wave.open(str(path), "rb") as w:
        return PcmInfo(w.getframerate(), w.getsampwidth(), w.getnchannels(), w.getnframes())


def iter_wav_pcm(path, block_size: int, blocks_per_batch: int, quirk: bool = True):
    """Stream a WAV file as int64 [channels][frames] pieces of blocks_per_batch * block_size
    frames: yields (first_block, pcm), so memory is bounded by one batch whatever the file
    size.  planar_blocks(pcm, block_size) cuts a piece into device rows."""
    with wave.open(str(path), "rb") as w:
        channels, width = w.getnchannels(), w.getsampwidth()
        first = 0
        while True:
            raw = w.readframes(blocks_per_batch * block_size)
            if not raw:
                return
            pcm = frames_to_channels(raw, channels, width, quirk)
            yield first, pcm
            first += (pcm.shape[1] + block_size - 1) // block_size


def iter_wav_batches(path, block_size: int, blocks_per_batch: int, quirk: bool = True):
    """Stream a WAV file as device-ready batches: yields (first_block, rows, bits, tail_len,
    n_tail_units) exactly as planar_blocks() cuts them, reading blocks_per_batch *
    block_size frames at a time, so memory is bounded by one batch whatever the file size."""
    with wave.open(str(path), "rb") as w:
        channels, width = w.getnchannels(), w.getsampwidth()
        first = 0
        while True:
            raw = w.readframes(blocks_per_batch * block_size)
            if not raw:
                return
            pcm = frames_to_channels(raw, channels, width, quirk)
            rows, bits, tail_len, n_tail = planar_blocks(pcm, block_size)
            yield first, rows, bits, tail_len, n_tail
            first += rows.shape[0] // channels


def read_wav(path, quirk: bool = True, chunk_frames: int = 1 << 20):
    """-> (PcmInfo, int64 [channels][frames]): the whole file in memory (tests and small
    files; the CLI streams through iter_wav_batches)."""
    with wave.open(str(path), "rb") as w:
        info = PcmInfo(w.getframerate(), w.getsampwidth(), w.getnchannels(), w.getnframes())
        parts = []
        while True:
            raw = w.readframes(chunk_frames)
            if not raw:
                break
            parts.append(frames_to_channels(raw, info.channels, info.sample_width, quirk))
    pcm = np.concatenate(parts, axis=1) if parts else np.zeros((info.channels, 0), dtype=np.int64)
    return info, pcm


def sample_bits(pcm: np.ndarray) -> int:
    """Bits the device arithmetic needs for these values (>= 2)."""
    if pcm.size == 0:
        return 2
    m = int(max(-int(pcm.min()), int(pcm.max()), 1))
    return max(2, m.bit_length() + 1)


def planar_blocks(pcm: np.ndarray, block_size: int, first_block: int = 0, n_blocks: int = -1, alloc=None):
    """int64 [channels][frames] -> (rows [n_blocks*channels][stride] int16/int32, bits,
    tail_len, n_tail_units) for blocks [first_block, first_block + n_blocks) of
    utils.batch(frames, block_size).  Rows are at the library's device pitch
    (flacmi_unit_stride), so a batch goes to the device as one linear copy; samples past a short
    block's end are zero.  alloc(shape, dtype) (optional) supplies the rows' memory, e.g.
    a page-locked staging buffer reused batch after batch."""
    C, frames = pcm.shape
    total = (frames + block_size - 1) // block_size
    if n_blocks < 0:
        n_blocks = total - first_block
    n_blocks = max(0, min(n_blocks, total - first_block))
    lo = first_block * block_size
    hi = min(frames, (first_block + n_blocks) * block_size)
    seg = pcm[:, lo:hi]
    bits = sample_bits(seg)
    dt = np.int16 if bits <= 16 else np.int32
    isz = np.dtype(dt).itemsize
    stride = unit_stride(block_size, isz)
    if alloc is None:
        rows = np.zeros((n_blocks, C, stride), dtype=dt)
    else:
        rows = alloc((n_blocks, C, stride), dt)
        rows[:, :, block_size:] = 0
    full = seg.shape[1] // block_size
    if full:
        rows[:full, :, :block_size] = seg[:, :full * block_size].reshape(C, full, block_size).transpose(1, 0, 2)
    tail_len = seg.shape[1] - full * block_size
    if tail_len:
        rows[full, :, :tail_len] = seg[:, full * block_size:]
        rows[full, :, tail_len:] = 0
    n_tail = C if tail_len else 0
    return rows.reshape(n_blocks * C, stride), bits, (tail_len if tail_len else block_size), n_tail
