"""PCM ingest + device encode end to end: the CLI (flac-py_amd/cli.py,
flac/__main__.py's encode action) on the config-1 WAV writes the reference CLI's exact
output file (golden hash recorded from `python -m flac encode` by make_golden.py), and
encode_planar writes encode()'s bytes for every golden stream."""
import hashlib
import io
import math
import wave

import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu


def _sine(n):
    return [round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n)]


@pytest.fixture(scope="module")
def c1_wav(tmp_path_factory):
    path = tmp_path_factory.mktemp("c1") / "sine.wav"
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(44100)
        w.writeframes(np.array(_sine(441000), dtype="<i2").tobytes())
    return path


@pytest.mark.parametrize("name,extra", [("c1_cli", []), ("c1_correct", ["--correct-reader"])])
def test_cli_encode_matches_reference_cli(c1_wav, tmp_path, name, extra):
    from flac_amd import cli
    S = G.load("streams.json")
    out = tmp_path / "out.flac"
    assert cli.main(["encode", str(c1_wav), str(out), "-b", "4608", "-l", "8", "-r", "5", *extra]) == 0
    data = out.read_bytes()
    assert (len(data), hashlib.sha256(data).hexdigest()) == (int(S[name]["len"]), S[name]["sha256"])


def test_encode_planar_c3_stereo_matches_reference():
    import oracle
    from flac_amd import encoder as enc
    e = G.load("streams.json")["c3_stereo"]
    n = int(e["frames"])
    pcm = np.stack([oracle.synth_unit(c["unit"], n, int(e["sample_size"]), c["seed"]).astype(np.int64)
                    for c in e["channels"]])
    p = enc.EncoderParameters(block_size=int(e["block_size"]),
                              rice_partition_order=range(e["rice"][0], e["rice"][1] + 1),
                              lpc_order=range(0, int(e["max_lpc_order"]) + 1), qlp_precision=int(e["qlp_precision"]))
    for bpb in (1, 3):
        data = b"".join(enc.encode_planar(int(e["sample_rate"]), int(e["sample_size"]), pcm, p, blocks_per_batch=bpb))
        assert (len(data), hashlib.sha256(data).hexdigest()) == (int(e["len"]), e["sha256"])
