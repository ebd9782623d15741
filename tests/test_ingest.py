"""PCM ingest (flac-py_amd/ingest.py) against the reference reader's
semantics, restated here as the per-frame loop of flac/__main__.py:82-92 (readframes(1),
group(xs, channels) from utils.py:61-66, int.from_bytes(..., 'little', signed=True)) and
the x[c] selection of encoder.py:102 — the checker, in pure Python on small inputs — and
against the golden config-1 sample hashes (tests/golden/streams.json, made by the
reference itself).  CPU only."""
import io
import math
import wave

import numpy as np
import pytest

import golden_util as G
from flac_amd import ingest
from flac_amd.utils import batch, group


def ref_reader(raw: bytes, channels: int, width: int, n_frames: int):
    """__main__.py:82-92 + encoder.py:102, frame by frame (the checker)."""
    out = [[] for _ in range(channels)]
    fb = channels * width
    for f in range(n_frames):
        xs = raw[f * fb:(f + 1) * fb]
        vals = [int.from_bytes(x, byteorder="little", signed=True) for x in group(xs, channels)]
        for c in range(channels):
            out[c].append(vals[c])  # IndexError when there are fewer groups than channels
    return out


def _wav_bytes(channels, width, rate, raw):
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(rate)
        w.writeframes(raw)
    return buf.getvalue()


@pytest.mark.parametrize("channels,width", [(1, 1), (1, 2), (1, 3), (1, 4), (2, 2), (2, 3), (2, 4),
                                            (3, 4), (4, 4), (6, 6)])
def test_quirk_reader_matches_reference_loop(channels, width):
    rng = np.random.default_rng(channels * 10 + width)
    n = 257
    raw = rng.integers(0, 256, size=n * channels * width, dtype=np.uint8).tobytes()
    got = ingest.frames_to_channels(raw, channels, width, quirk=True)
    assert got.tolist() == ref_reader(raw, channels, width, n)


@pytest.mark.parametrize("channels,width", [(2, 1), (3, 2), (4, 3), (8, 2), (5, 4), (8, 4)])
def test_quirk_reader_raises_like_reference(channels, width):
    raw = bytes(range(channels * width)) * 3
    with pytest.raises(IndexError):
        ref_reader(raw, channels, width, 3)
    with pytest.raises(IndexError):
        ingest.frames_to_channels(raw, channels, width, quirk=True)


@pytest.mark.parametrize("channels,width", [(1, 2), (2, 3), (6, 4), (1, 1)])
def test_correct_reader(channels, width):
    rng = np.random.default_rng(99 + channels)
    n = 100
    raw = rng.integers(0, 256, size=n * channels * width, dtype=np.uint8).tobytes()
    got = ingest.frames_to_channels(raw, channels, width, quirk=False)
    fb = channels * width
    if width == 1:  # 8-bit WAV samples are unsigned, offset 128
        want = [[raw[f * fb + c] - 128 for f in range(n)] for c in range(channels)]
    else:
        want = [[int.from_bytes(raw[f * fb + c * width:f * fb + (c + 1) * width], "little", signed=True)
                 for f in range(n)] for c in range(channels)]
    assert got.tolist() == want


@pytest.mark.parametrize("frames,block,channels,width,per", [(100000, 4608, 1, 2, 3), (30001, 1000, 2, 3, 4),
                                                              (4608 * 4, 4608, 2, 2, 2), (5, 4608, 1, 2, 8)])
@pytest.mark.parametrize("quirk", [True, False])
def test_streamed_batches_equal_whole_file(tmp_path, frames, block, channels, width, per, quirk):
    """iter_wav_batches (the CLI's bounded-memory reader) cuts the same rows as
    planar_blocks over the whole file."""
    if quirk and width < channels:
        pytest.skip("the reference reader raises for this shape")
    rng = np.random.default_rng(frames + width)
    raw = rng.integers(0, 256, size=frames * channels * width, dtype=np.uint8).tobytes()
    path = tmp_path / "x.wav"
    path.write_bytes(_wav_bytes(channels, width, 44100, raw))
    _, pcm = ingest.read_wav(path, quirk=quirk)
    nb = (frames + block - 1) // block
    seen = 0
    for first, rows, bits, tail_len, n_tail in ingest.iter_wav_batches(path, block, per, quirk):
        assert first == seen
        want_rows, _, want_tail, want_nt = ingest.planar_blocks(pcm, block, first, per)
        assert np.array_equal(rows.astype(np.int64), want_rows.astype(np.int64))
        assert (tail_len, n_tail) == (want_tail, want_nt)
        seen += rows.shape[0] // channels
    assert seen == nb


def test_cli_reader_error_after_stream_header(tmp_path):
    """The reference CLI raises its reader's IndexError (encoder.py:102) after writing the
    42-byte stream header; so does ours (before touching a device)."""
    from flac_amd import cli
    path = tmp_path / "x.wav"
    path.write_bytes(_wav_bytes(3, 2, 44100, bytes(range(60)) * 10))
    out = tmp_path / "x.flac"
    with pytest.raises(IndexError):
        cli.main(["encode", str(path), str(out)])
    data = out.read_bytes()
    assert len(data) == 42 and data[:4] == b"fLaC"


def _sine(n):
    return [round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n)]


def test_c1_wav_ingest_matches_golden_sample_hashes(tmp_path):
    """The config-1 WAV read back gives the reference's quirk samples (its CLI) and, with
    the correct reader, the true samples (golden hashes from the reference run)."""
    S = G.load("streams.json")
    pcm = np.array(_sine(441000), dtype="<i2")
    path = tmp_path / "c1.wav"
    path.write_bytes(_wav_bytes(1, 2, 44100, pcm.tobytes()))
    info, q = ingest.read_wav(path, quirk=True, chunk_frames=100_000)
    assert (info.sample_rate, info.sample_width, info.channels, info.frames) == (44100, 2, 1, 441000)
    assert G.samples_sha([int(v) for v in q[0]]) == S["c1_quirk"]["samples_sha256"]
    _, c = ingest.read_wav(path, quirk=False)
    assert G.samples_sha([int(v) for v in c[0]]) == S["c1_correct"]["samples_sha256"]


@pytest.mark.parametrize("frames,block,channels", [(441000, 4608, 1), (10000, 1000, 3), (4608 * 3, 4608, 2),
                                                    (5, 4608, 2), (70000, 16384, 2)])
def test_planar_blocks_follow_utils_batch(frames, block, channels):
    rng = np.random.default_rng(frames)
    pcm = rng.integers(-30000, 30000, size=(channels, frames)).astype(np.int64)
    blocks = list(batch(iter(list(map(list, zip(*pcm.tolist())))), block))
    for first, count in ((0, -1), (1, 2), (len(blocks) - 1, 5)):
        if first >= len(blocks):
            continue
        rows, bits, tail_len, n_tail = ingest.planar_blocks(pcm, block, first, count)
        sel = blocks[first:] if count < 0 else blocks[first:first + count]
        assert rows.shape[0] == len(sel) * channels and rows.shape[1] * rows.itemsize % 16 == 0
        assert rows.dtype == (np.int16 if bits <= 16 else np.int32)
        for b, blk in enumerate(sel):
            for c in range(channels):
                assert rows[b * channels + c, :len(blk)].tolist() == [x[c] for x in blk]
                assert not rows[b * channels + c, len(blk):block].any()
        short = len(sel[-1]) != block
        assert n_tail == (channels if short else 0) and tail_len == (len(sel[-1]) if short else block)
