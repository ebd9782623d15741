"""The drop-in encoder interface on the device: whole streams byte-identical to the
reference's encode() (tests/golden/streams.json, made by tests/golden/make_golden.py)
and the single-unit forms (encode_subframe_fixed / encode_subframe_lpc /
encode_residual) against the golden per-unit fixtures."""
import hashlib
import math

import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

EXC = {"ZeroDivisionError": ZeroDivisionError, "AssertionError": AssertionError,
       "ValueError": ValueError, "OverflowError": OverflowError}


@pytest.fixture(scope="module")
def enc():
    from flac_amd import encoder
    return encoder


@pytest.fixture(scope="module")
def synth():
    import oracle
    return oracle.synth_unit


def _sine(n):
    return [round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n)]


def _stream(enc, rate, size, ch, frames, chans, p, **kw):
    it = iter(list(t) for t in zip(*chans))
    data = b"".join(enc.encode(rate, size, ch, frames, it, p, **kw))
    return len(data), hashlib.sha256(data).hexdigest()


@pytest.mark.parametrize("name", ["c1_correct", "c1_quirk"])
def test_stream_c1_matches_reference(enc, name):
    S = G.load("streams.json")
    pcm = _sine(441000)
    if name == "c1_quirk":  # flac/__main__.py's reader hands encode() the low byte as int8
        pcm = [((v & 0xFF) ^ 0x80) - 0x80 for v in pcm]
    assert G.samples_sha(pcm) == S[name]["samples_sha256"]
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 9), qlp_precision=5)
    got = _stream(enc, 44100, 16, 1, len(pcm), [pcm], p, blocks_per_batch=32)
    assert got == (S[name]["len"], S[name]["sha256"])


def test_stream_c1_batching_invariant(enc):
    S = G.load("streams.json")
    pcm = _sine(441000)
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 9), qlp_precision=5)
    for bpb in (1, 7, 4096):
        assert _stream(enc, 44100, 16, 1, len(pcm), [pcm], p, blocks_per_batch=bpb) == \
            (S["c1_correct"]["len"], S["c1_correct"]["sha256"])


def test_stream_c3_stereo_24bit_matches_reference(enc, synth):
    e = G.load("streams.json")["c3_stereo"]
    n = e["frames"]
    chans = [[int(v) for v in synth(c["unit"], n, e["sample_size"], c["seed"])] for c in e["channels"]]
    p = enc.EncoderParameters(block_size=e["block_size"],
                              rice_partition_order=range(e["rice"][0], e["rice"][1] + 1),
                              lpc_order=range(0, e["max_lpc_order"] + 1),
                              qlp_precision=e["qlp_precision"])
    assert _stream(enc, e["sample_rate"], e["sample_size"], 2, n, chans, p) == (e["len"], e["sha256"])


def _units(names=("c1.json", "c2.json", "c3.json", "edge.json")):
    for nm in names:
        for i, e in enumerate(G.load(nm)["units"]):
            yield pytest.param(nm, i, id=f"{nm[:-5]}-{i}")


def _entry(nm, i, synth):
    e = G.load(nm)["units"][i]
    return e, G.samples_for(e, synth)


def _fixed_residual(xs, order):
    a = np.asarray(xs, dtype=np.int64)
    for _ in range(order):
        a = np.diff(a)
    return a


@pytest.mark.parametrize("nm,i", list(_units()))
def test_encode_subframe_fixed(enc, synth, nm, i):
    e, xs = _entry(nm, i, synth)
    exp = e["expect"]
    if "fixed_order" not in exp:
        pytest.skip("fixture has no fixed analysis (failed earlier)")
    hdr, sf = enc.encode_subframe_fixed(xs)
    assert hdr.type_.order == exp["fixed_order"] == sf.order
    assert sf.warmup == xs[:sf.order]
    want = _fixed_residual(xs, sf.order) if len(xs) > 4 else np.asarray(xs[sf.order:])
    assert sf.residual == [int(v) for v in want]
    assert sum(abs(r) for r in sf.residual) == exp["fixed_sums"][sf.order]


@pytest.mark.parametrize("nm,i", list(_units()))
def test_encode_subframe_lpc(enc, synth, nm, i):
    e, xs = _entry(nm, i, synth)
    exp, p = e["expect"], e["params"]
    if p["fixed_only"]:
        pytest.skip("fixed-only fixture")
    lpc_exc = exp.get("exception") if exp.get("exception_stage") == "lpc" else None
    if lpc_exc is not None:
        with pytest.raises(EXC[lpc_exc["type"]]):
            enc.encode_subframe_lpc(xs, range(0, p["L"] + 1), p["q"])
        return
    if "lpc" not in exp:
        pytest.skip("fixture has no LPC analysis")
    hdr, sf = enc.encode_subframe_lpc(xs, range(0, p["L"] + 1), p["q"])
    want = exp["lpc"]
    assert (hdr.type_.order, sf.shift, sf.coefficients, sf.precision, len(sf.residual)) == \
        (want["order"], want["shift"], want["coefs"], want["precision"], want["res_len"])
    assert sf.warmup == xs[:sf.order]
    assert sum(abs(r) for r in sf.residual) == exp["lpc_size"]


@pytest.mark.parametrize("nm,i", list(_units()))
def test_encode_residual(enc, synth, nm, i):
    e, xs = _entry(nm, i, synth)
    exp, p = e["expect"], e["params"]
    if "exception" in exp or exp.get("kind") != "fixed" or len(xs) <= 4:
        pytest.skip("needs a successful fixed-predictor unit")
    order = exp["order"]
    res = [int(v) for v in _fixed_residual(xs, order)]
    r = enc.encode_residual(res, len(xs), p["sample_size"], order, range(p["rmin"], p["rmax"] + 1))
    assert r.partition_order == exp["partition_order"]
    assert r.coding_method.value == exp["coding_method"]
    assert [q.parameter for q in r.partitions] == exp["params"]
    assert [len(q.residual) for q in r.partitions] == exp["part_lens"]
    h = hashlib.sha256()
    for q in r.partitions:
        h.update(b"".join(int(x).to_bytes(8, "little") for x in q.residual))
    assert h.hexdigest() == exp["zz_sha256"]


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_stream_c1_multi_context_matches_reference(enc, devices):
    """encode(devices=[...]): batches round-robin over several contexts (two or three on
    one GPU here), frames merged in block order: byte-identical to the reference."""
    S = G.load("streams.json")
    pcm = _sine(441000)
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 9), qlp_precision=5)
    for bpb in (1, 5):
        assert _stream(enc, 44100, 16, 1, len(pcm), [pcm], p, blocks_per_batch=bpb, devices=devices) == \
            (S["c1_correct"]["len"], S["c1_correct"]["sha256"])


def test_stream_c1_two_devices_matches_reference(enc):
    """encode(devices=[0, 1]): one context per GPU (skipped with fewer than two visible),
    batches round-robin, frames merged in block order: byte-identical to the reference."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("fewer than two GPUs visible")
    S = G.load("streams.json")
    pcm = _sine(441000)
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 9), qlp_precision=5)
    for bpb in (1, 5):
        assert _stream(enc, 44100, 16, 1, len(pcm), [pcm], p, blocks_per_batch=bpb, devices=[0, 1]) == \
            (S["c1_correct"]["len"], S["c1_correct"]["sha256"])


def test_encode_planar_multi_context_and_frame_error_order(enc):
    """encode_planar over two contexts equals one context; a unit the reference fails on
    (an all-zero block: ZeroDivisionError in levinson_durbin) raises after exactly the
    frames before it, whichever context encoded its batch."""
    pcm = np.array([_sine(4608 * 9)], dtype=np.int64)
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 13), qlp_precision=5)
    one = list(enc.encode_planar(44100, 16, pcm, p, blocks_per_batch=2))
    two = list(enc.encode_planar(44100, 16, pcm, p, blocks_per_batch=2, devices=[0, 0]))
    assert one == two and len(one) == 3 + 9
    bad = pcm.copy()
    bad[0, 4608 * 5:4608 * 6] = 0
    got = []
    with pytest.raises(ZeroDivisionError):
        for f in enc.encode_planar(44100, 16, bad, p, blocks_per_batch=2, devices=[0, 0]):
            got.append(f)
    assert got == one[:3 + 5]


def test_interleaved_generators_do_not_share_staging(enc):
    """Two encode_planar generators on one device consumed in turn (zip), and two threads
    encoding at once: each stream equals its own sequential run byte for byte (each _drive
    call checks out its own session and staging slots)."""
    import concurrent.futures
    p = enc.EncoderParameters(block_size=4608, rice_partition_order=range(0, 6),
                              lpc_order=range(0, 13), qlp_precision=5)
    a = np.array([_sine(4608 * 12)], dtype=np.int64)
    b = np.random.default_rng(7).integers(-9000, 9000, (1, 4608 * 12)).astype(np.int64)
    seq_a = list(enc.encode_planar(44100, 16, a, p, blocks_per_batch=1))
    seq_b = list(enc.encode_planar(44100, 16, b, p, blocks_per_batch=1))
    assert seq_a != seq_b
    za, zb = [], []
    for fa, fb in zip(enc.encode_planar(44100, 16, a, p, blocks_per_batch=1),
                      enc.encode_planar(44100, 16, b, p, blocks_per_batch=1)):
        za.append(fa)
        zb.append(fb)
    assert za == seq_a and zb == seq_b
    with concurrent.futures.ThreadPoolExecutor(2) as ex:
        fa = ex.submit(lambda: list(enc.encode_planar(44100, 16, a, p, blocks_per_batch=1)))
        fb = ex.submit(lambda: list(enc.encode_planar(44100, 16, b, p, blocks_per_batch=1)))
        assert fa.result() == seq_a and fb.result() == seq_b
    # a generator closed early hands its session back
    g = enc.encode_planar(44100, 16, a, p, blocks_per_batch=1)
    next(g), next(g), next(g), next(g)
    g.close()
    assert list(enc.encode_planar(44100, 16, a, p, blocks_per_batch=1)) == seq_a
    # a burst of four concurrent generators: the sessions beyond _IDLE_MAX per device are
    # closed when they come back (each holds a context, pinned buffers and a worker thread)
    with concurrent.futures.ThreadPoolExecutor(4) as ex:
        fs = [ex.submit(lambda: list(enc.encode_planar(44100, 16, a, p, blocks_per_batch=1))) for _ in range(4)]
        assert all(f.result() == seq_a for f in fs)
    assert len(enc._IDLE[0]) <= enc._IDLE_MAX
    assert list(enc.encode_planar(44100, 16, b, p, blocks_per_batch=1)) == seq_b
