"""Generate golden fixtures by running the reference (turlando/flac-py) itself.

Run ONLY in the build container, where the reference is readable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports flac.encoder from /root/reference (read-only, nothing is copied) and
records, per unit, what the reference computes at every step of the hot path:
window/autocorrelation/Levinson intermediates (float.hex), every LPC candidate
(quantised coefficients, shift, sum|r|), the fixed sums, the chosen subframe, the
Rice partitioning and a SHA-256 of the zig-zag residual -- or the exception the
reference raises.  Inputs are either literal sample lists or recipes for the
integer synthetic generator, restated here in Python so the oracle's
and the device's generators are pinned too (samples_sha256).

The GPU box never runs this script and never needs /root/reference.
"""
import hashlib
import json
import math
import os
import random
import subprocess
import sys
import tempfile
import wave

REF = os.environ.get("FLAC_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from flac import encoder as E  # noqa: E402  (the reference, imported read-only)
from flac.common import FIXED_PREDICTOR_COEFFICIENTS  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


# ---------------------------------------------------------------------------------
# Synthetic generator (same integer recipe as oracle_synth_unit / flacmi_synth_device)
# ---------------------------------------------------------------------------------
def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


SINTAB = [round(32767.0 * math.sin(6.283185307179586 * k / 4096.0)) for k in range(4096)]


def synth_unit(unit, length, bits, seed):
    h0 = splitmix64(seed ^ ((unit * 0xD1B54A32D192ED03) & M64))
    amp, dphi, phi0 = [], [], []
    for k in range(3):
        hk = splitmix64((h0 + k + 1) & M64)
        amp.append(1638 + hk % 8192)
        f = 20 + ((hk >> 16) % 7981)
        dphi.append(((f << 32) // 44100) & M32)
        phi0.append((hk >> 32) & M32)
    sigma = 66 + splitmix64((h0 + 4) & M64) % 590
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    out = []
    for i in range(length):
        acc = sum(amp[k] * SINTAB[((phi0[k] + ((i * dphi[k]) & M32)) & M32) >> 20] for k in range(3))
        s = acc >> 15
        r = splitmix64(seed ^ ((unit << 32) & M64) ^ i)
        bsum = (r & 0xff) + ((r >> 8) & 0xff) + ((r >> 16) & 0xff) + ((r >> 24) & 0xff)
        v = s + (((bsum - 510) * sigma) >> 7)
        if bits > 16:
            e = bits - 16
            v = v * (1 << e) + ((r >> 32) & ((1 << e) - 1)) - (1 << (e - 1))
        elif bits < 16:
            v >>= (16 - bits)
        out.append(min(max(v, lo), hi))
    return out


def sine_pcm(n_samples, freq=440.0, rate=44100, amp=0.6):
    return [round(amp * 32767 * math.sin(2 * math.pi * freq * i / rate)) for i in range(n_samples)]


def cli_quirk(values):
    """flac/__main__.py:91-92 splits a mono 16-bit frame into 1-byte groups; encode()
    then sees only the low byte, as a signed int8."""
    return [((v & 0xff) ^ 0x80) - 0x80 for v in values]


def samples_sha(xs):
    h = hashlib.sha256()
    h.update(b"".join(int(x).to_bytes(8, "little", signed=True) for x in xs))
    return h.hexdigest()


def zz_sha(partitions):
    h = hashlib.sha256()
    for p in partitions:
        h.update(b"".join(int(x).to_bytes(8, "little", signed=False) for x in p.residual))
    return h.hexdigest()


# ---------------------------------------------------------------------------------
# The reference's per-channel body of encode() (encoder.py:127-157) + the writer's
# encode_residual call (encoder.py:588/608), with intermediates recorded.
# ---------------------------------------------------------------------------------
def exc(e):
    return {"type": type(e).__name__, "msg": str(e)}


def ref_unit(samples, L, q, rrange, fixed_only=False, sample_size=16, intermediates=True):
    n = len(samples)
    rec = {"n": n}
    fh, fs = E.encode_subframe_fixed(samples)
    rec["fixed_order"] = fh.type_.order
    if n > 4:
        rec["fixed_sums"] = [sum(abs(r) for r in E.prediction_residual(samples, c))
                             for c in FIXED_PREDICTOR_COEFFICIENTS]
    else:
        rec["fixed_sums"] = [sum(abs(x) for x in samples)]
    chosen_h, chosen = fh, fs
    if not fixed_only:
        if intermediates:
            rec["inter"] = ref_intermediates(samples, L, q)
        try:
            lh, ls = E.encode_subframe_lpc(samples, range(L + 1), q)
        except Exception as e:  # the reference raises: the unit's result is the exception
            rec["exception"] = exc(e)
            rec["exception_stage"] = "lpc"
            return rec
        rec["lpc"] = {"order": lh.type_.order, "shift": ls.shift, "coefs": list(ls.coefficients),
                      "precision": ls.precision, "res_len": len(ls.residual)}
        fixed_size = sum(abs(x) for x in fs.residual)
        lpc_size = sum(abs(x) for x in ls.residual)
        rec["fixed_size"], rec["lpc_size"] = fixed_size, lpc_size
        if fixed_size < lpc_size:
            chosen_h, chosen = fh, fs
        elif lpc_size < fixed_size:
            chosen_h, chosen = lh, ls
        else:
            rec["exception"] = {"type": "AssertionError", "msg": ""}
            rec["exception_stage"] = "choice"
            return rec
    rec["kind"] = "lpc" if chosen is not fs else "fixed"
    rec["order"] = chosen.order
    try:
        res = E.encode_residual(chosen.residual, n, sample_size, chosen.order, rrange)
    except Exception as e:
        rec["exception"] = exc(e)
        rec["exception_stage"] = "rice"
        return rec
    rec["res_len"] = len(chosen.residual)
    rec["coding_method"] = res.coding_method.value
    rec["partition_order"] = res.partition_order
    rec["n_parts"] = len(res.partitions)
    rec["params"] = [p.parameter for p in res.partitions]
    rec["part_lens"] = [len(p.residual) for p in res.partitions]
    rec["rice_bits"] = sum(E.estimate_rice_partition_size_and_parameter(p.residual)[0]
                           for p in res.partitions)
    rec["zz_sha256"] = zz_sha(res.partitions)
    return rec


def ref_intermediates(samples, L, q):
    """tukey -> autocorrelation -> levinson per order -> quantise per order, as
    encode_subframe_lpc computes them (encoder.py:367-390), each step guarded."""
    n = len(samples)
    out = {}
    try:
        w = E.tukey(n, 0.5)
    except Exception as e:
        out["tukey_exception"] = exc(e)
        return out
    out["window_sha256"] = hashlib.sha256("".join(x.hex() for x in w).encode()).hexdigest()
    windowed = [x * v for x, v in zip(samples, w)]
    ac = [E.autocorrelation(windowed, i) for i in range(L + 1)]
    out["acf"] = [float(a).hex() for a in ac]
    levs, quants, sums = [], [], []
    for i in range(2, L + 2):
        try:
            c = E.levinson_durbin(ac[:i])
        except Exception as e:
            levs.append(exc(e))
            continue
        levs.append([x.hex() for x in c])
    out["levinson"] = levs
    if any(isinstance(x, dict) for x in levs):
        return out
    for c in levs:
        try:
            qc, sh = E.quantize_lpc_coefficients([float.fromhex(x) for x in c], q)
        except Exception as e:
            quants.append(exc(e))
            continue
        quants.append({"coefs": qc, "shift": sh})
        r = E.prediction_residual(samples, qc, sh)
        sums.append(sum(abs(x) for x in r))
    out["quant"] = quants
    out["lpc_sums"] = sums
    return out


# ---------------------------------------------------------------------------------
# Fixture sets
# ---------------------------------------------------------------------------------
def unit_entry(source, samples, L, q, rrange, fixed_only=False, sample_size=16, intermediates=True):
    e = {"source": source, "samples_sha256": samples_sha(samples),
         "params": {"L": L, "q": q, "rmin": rrange.start, "rmax": rrange.stop - 1,
                    "fixed_only": fixed_only, "sample_size": sample_size}}
    if source["kind"] == "literal":
        pass
    e["expect"] = ref_unit(samples, L, q, rrange, fixed_only, sample_size, intermediates)
    return e


def synth_set(name, units, length, bits, seed, L, q, rrange, fixed_only=False):
    entries = []
    for u in units:
        s = synth_unit(u, length, bits, seed)
        src = {"kind": "synth", "unit": u, "len": length, "bits": bits, "seed": seed}
        entries.append(unit_entry(src, s, L, q, rrange, fixed_only, sample_size=bits))
        print(name, u, entries[-1]["expect"].get("kind"), entries[-1]["expect"].get("order"),
              entries[-1]["expect"].get("exception"), flush=True)
    return entries


def literal(samples, L, q, rrange, fixed_only=False, tag="", src=None):
    src = dict(src or {"kind": "literal", "samples": list(samples)}, tag=tag)
    return unit_entry(src, list(samples), L, q, rrange, fixed_only)


def multitone(freqs, amp, n):
    """Recipe source: round(amp * sum(sin(2*pi*f*i/44100 + 0.5*k)) / K)."""
    K = len(freqs)
    xs = [round(amp * sum(math.sin(2 * math.pi * f * i / 44100 + 0.5 * k)
                          for k, f in enumerate(freqs)) / K) for i in range(n)]
    return xs, {"kind": "multitone", "freqs": list(freqs), "amp": amp, "n": n}


def tone(f, n=4608, amp=12000):
    """Recipe source: round(amp*sin(2*pi*f*i/44100))."""
    return ([round(amp * math.sin(2 * math.pi * f * i / 44100)) for i in range(n)],
            {"kind": "tone", "f": f, "n": n, "amp": amp})


def edge_set():
    rnd = random.Random(12345)
    E_ = []
    # tiny blocks, every length 1..12, default-ish params
    for n in range(1, 13):
        xs = [rnd.randint(-300, 300) for _ in range(n)]
        E_.append(literal(xs, 8, 5, range(0, 6), tag=f"tiny{n}"))
        E_.append(literal(xs, 8, 5, range(0, 6), fixed_only=True, tag=f"tiny{n}-fixed"))
    # silence / constant / ramp / impulse
    E_.append(literal([0] * 64, 8, 5, range(0, 6), tag="silence64"))
    E_.append(literal([0] * 4608, 12, 5, range(0, 6), tag="silence4608",
                      src={"kind": "const", "value": 0, "n": 4608}))
    E_.append(literal([7] * 256, 8, 5, range(0, 6), tag="const256"))
    E_.append(literal([7] * 256, 8, 5, range(0, 6), fixed_only=True, tag="const256-fixed"))
    E_.append(literal(list(range(-128, 128)), 8, 5, range(0, 6), tag="ramp256"))
    E_.append(literal([0] * 100 + [1000] + [0] * 155, 8, 5, range(0, 6), tag="impulse256"))
    # -l 0 (ValueError in the reference), -l 1, empty rice range, high orders
    xs = synth_unit(7, 1024, 16, 99)
    syn = {"kind": "synth", "unit": 7, "len": 1024, "bits": 16, "seed": 99}
    E_.append(literal(xs, 0, 5, range(0, 6), tag="l0", src=syn))
    E_.append(literal(xs, 1, 5, range(0, 6), tag="l1", src=syn))
    E_.append(literal(xs, 12, 5, range(3, 3), tag="rice-empty", src=syn))
    E_.append(literal(xs, 12, 5, range(4, 9), tag="rice-4-8", src=syn))
    E_.append(literal(xs, 32, 15, range(0, 9), tag="l32q15", src=syn))
    E_.append(literal(xs, 12, 12, range(0, 6), tag="q12", src=syn))
    E_.append(literal(xs, 12, 15, range(0, 16), tag="q15r15", src=syn))
    # small residuals: 0 < sum < len in a partition (negative Rice parameter)
    E_.append(literal([rnd.choice([0, 0, 0, 1]) for _ in range(512)], 4, 5, range(0, 6), tag="sparse512"))
    # odd lengths (short last blocks)
    for n in (3240, 1000, 999, 577):
        E_.append(literal(synth_unit(n, n, 16, 5), 8, 5, range(0, 6), tag=f"short{n}",
                          src={"kind": "synth", "unit": n, "len": n, "bits": 16, "seed": 5}))
    # low-frequency pure tones: large Levinson coefficients (negative-shift branch)
    for f, L, q in ((20.0, 12, 5), (40.0, 12, 5), (30.0, 32, 5), (60.0, 8, 5), (25.0, 12, 7)):
        xs, src = tone(f)
        E_.append(literal(xs, L, q, range(0, 6), tag=f"tone{f}-L{L}-q{q}", src=src))
    # high-frequency multi-tones: |Levinson coefficient| >= 2^(q-1), i.e. the negative-shift
    # branch of quantize_lpc_coefficients (encoder.py:523-532) returns ([], 0)
    for fs_, amp, n, L in (((19401.4, 17113.6, 10839.5), 30000, 512, 24),
                           ((12316.6, 18965.5, 17232.8, 8024.8), 30000, 512, 32),
                           ((3086.0, 10848.9, 4042.3, 4591.7, 16951.9, 892.2), 30000, 1024, 24),
                           ((8209.8, 3016.2), 30000, 512, 32),
                           ((628.5, 3948.5, 8159.3, 12209.7, 3124.8, 849.7), 30000, 1024, 24),
                           ((5426.7, 12686.2, 14312.7, 18728.8, 8749.5, 5165.4), 30000, 1024, 24),
                           ((1436.4, 7716.6, 7793.3, 6083.1), 30000, 256, 16)):
        xs, src = multitone(fs_, amp, n)
        E_.append(literal(xs, L, 5, range(0, 6), tag=f"multitone{len(fs_)}-L{L}", src=src))
    # white noise, full scale: Rice parameters > 14 (Rice5Bit) and shift capping at 15
    xs = [rnd.randint(-32768, 32767) for _ in range(4608)]
    E_.append(literal(xs, 12, 15, range(0, 6), tag="noise-fs-q15"))
    E_.append(literal(xs, 12, 5, range(0, 6), fixed_only=True, tag="noise-fs-fixed"))
    # random search for reference exceptions at each stage (small blocks, cheap)
    found = {}
    for trial in range(4000):
        n = rnd.choice([8, 9, 10, 12, 16, 20, 24, 32])
        amp = rnd.choice([1, 2, 3, 5, 50])
        xs = [rnd.randint(-amp, amp) for _ in range(n)]
        L = rnd.choice([1, 2, 4, 8])
        r = ref_unit(xs, L, 5, range(0, 3), intermediates=False)
        key = (r.get("exception", {}).get("type"), r.get("exception_stage"),
               r.get("exception", {}).get("msg", "")[:24])
        if key not in found:
            found[key] = literal(xs, L, 5, range(0, 3), tag=f"search-{key}")
    E_.extend(found.values())
    print("edge exception kinds:", sorted(str(k) for k in found), flush=True)
    return E_


def stream_set():
    """Whole-stream fixtures: reference encode() bytes (and its CLI) for config 1."""
    from flac.encoder import EncoderParameters, encode
    pcm = sine_pcm(441000)
    params = dict(block_size=4608, rice_partition_order=range(0, 6), lpc_order=range(0, 9),
                  qlp_precision=5)
    out = {}
    for name, vals in (("c1_quirk", cli_quirk(pcm)), ("c1_correct", pcm)):
        data = b"".join(encode(44100, 16, 1, len(vals), iter([[v] for v in vals]),
                               EncoderParameters(**params)))
        out[name] = {"len": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                     "samples_sha256": samples_sha(vals)}
        print(name, out[name], flush=True)
    # the reference CLI on a WAV file must give the c1_quirk bytes
    with tempfile.TemporaryDirectory() as d:
        wav = os.path.join(d, "sine.wav")
        with wave.open(wav, "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(44100)
            w.writeframes(b"".join(v.to_bytes(2, "little", signed=True) for v in pcm))
        flac = os.path.join(d, "sine.flac")
        env = dict(os.environ, PYTHONPATH=REF, PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, "-m", "flac", "encode", "-b", "4608", "-l", "8", "-r", "5",
                        wav, flac], check=True, env=env, cwd=d)
        data = open(flac, "rb").read()
        out["c1_cli"] = {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()}
        print("c1_cli", out["c1_cli"], flush=True)
    out["c1_params"] = {"block_size": 4608, "rice": [0, 5], "max_lpc_order": 8, "qlp_precision": 5,
                        "sample_rate": 44100, "sample_size": 16, "channels": 1,
                        "signal": "round(0.6*32767*sin(2*pi*440*i/44100)), i < 441000"}
    # a small stereo 24-bit stream (exercises channels, 24-bit sample size, 96 kHz)
    n = 16384 * 2 + 1000
    left = synth_unit(1, n, 24, 3)
    right = synth_unit(2, n, 24, 3)
    p3 = EncoderParameters(block_size=16384, rice_partition_order=range(0, 9),
                           lpc_order=range(0, 33), qlp_precision=15)
    data = b"".join(encode(96000, 24, 2, n, iter([[a, b] for a, b in zip(left, right)]), p3))
    out["c3_stereo"] = {"len": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                        "frames": n, "block_size": 16384, "rice": [0, 8], "max_lpc_order": 32,
                        "qlp_precision": 15, "sample_rate": 96000, "sample_size": 24,
                        "channels": [{"unit": 1, "seed": 3}, {"unit": 2, "seed": 3}]}
    print("c3_stereo", out["c3_stereo"], flush=True)
    return out


# ---------------------------------------------------------------------------------
# ACF-driven rows: the Levinson-Durbin / quantiser exception sites that integer PCM
# never reaches (encoder.py:476 OverflowError of lambda_ ** 2, encoder.py:503
# floor(log2(inf))), reached from autocorrelation vectors directly.  Each row runs the
# reference's steps 3-4 of encode_subframe_lpc (encoder.py:376-384) on the row: every
# order's levinson_durbin first, then every order's quantize_lpc_coefficients.
# ---------------------------------------------------------------------------------
def _raise_line(e):
    import traceback
    tb = [f for f in traceback.extract_tb(e.__traceback__) if f.filename.endswith("encoder.py")]
    return tb[-1].lineno if tb else None


def ref_from_acf(ac, L, q):
    out = {"acf": [float(a).hex() for a in ac], "L": L, "q": q}
    try:
        coefs = [E.levinson_durbin(ac[:i]) for i in range(2, L + 2)]
    except Exception as e:
        out["exception"] = dict(exc(e), stage="levinson", line=_raise_line(e))
        return out
    out["levinson"] = [[x.hex() for x in c] for c in coefs]
    quants = []
    for c in coefs:
        try:
            qc, sh = E.quantize_lpc_coefficients(c, q)
        except Exception as e:
            out["exception"] = dict(exc(e), stage="quant", line=_raise_line(e), order=len(c))
            break
        quants.append({"coefs": qc, "shift": sh})
    out["quant"] = quants
    return out


def acf_set():
    rows = []
    tiny = 5e-324
    # lambda_ ** 2 overflows at the first / a later step (encoder.py:476)
    for L, q, ac in ((1, 5, [1e-200, 1.0]), (4, 12, [1e-160, -3.0, 2.0, 1.0, 0.5]),
                     (8, 15, [1.0, 0.5, 0.25, 0.125, 1e200, 0.0, 0.0, 0.0, 0.0]),
                     (32, 5, [1e-300] + [1e10 / (k + 1) for k in range(32)])):
        rows.append(ref_from_acf(ac, L, q))
    # lambda_ overflows to inf in the division (no exception), coefficient inf -> floor(log2(inf))
    for L, q, ac in ((1, 5, [tiny, 1.0]), (2, 5, [1e-310, 1.0, 1.0]), (12, 15, [tiny] + [1.0] * 12)):
        rows.append(ref_from_acf(ac, L, q))
    # zero error, assertion sites, NaN coefficients
    for L, q, ac in ((3, 5, [0.0, 1.0, 1.0, 1.0]), (2, 5, [1.0, 0.0, 0.0]), (2, 5, [1e-30, 1.0, 0.3]),
                     (2, 5, [1.0, float("nan"), 0.0]), (2, 5, [1.0, 0.5, float("nan")]),
                     (3, 5, [float("inf"), 1.0, 1.0, 1.0]), (2, 5, [1.0, float("inf"), 0.0])):
        rows.append(ref_from_acf(ac, L, q))
    # random rows over a wide exponent range: one row per distinct outcome
    rnd = random.Random(4711)
    found = {}
    for trial in range(20000):
        L = rnd.choice([1, 2, 3, 4, 8, 12, 32])
        q = rnd.choice([5, 12, 15])
        ac = [rnd.choice([-1, 1]) * 10.0 ** rnd.uniform(-320, 300) if rnd.random() < 0.3 else
              rnd.uniform(-1, 1) * 10.0 ** rnd.uniform(-5, 5) for _ in range(L + 1)]
        ac[0] = abs(ac[0])
        r = ref_from_acf(ac, L, q)
        ex = r.get("exception")
        key = (ex["type"], ex["stage"], ex["line"]) if ex else ("ok", min(L, 4))
        if found.get(key, 0) < 3:
            found[key] = found.get(key, 0) + 1
            rows.append(r)
    print("acf outcomes:", sorted(str(k) for k in found), flush=True)
    return rows


def dump(name, obj):
    path = os.path.join(OUT, name)
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes", flush=True)


def main(which):
    if "c2" in which:
        dump("c2.json", {"config": "BASELINE config 2: 4608 x int16, -l 12 -q 5 -r 0,5",
                         "units": synth_set("c2", range(6), 4608, 16, 2024, 12, 5, range(0, 6))})
    if "c1" in which:
        dump("c1.json", {"config": "BASELINE config 1 params: -b 4608 -l 8 -q 5 -r 5",
                         "units": synth_set("c1", range(4), 4608, 16, 7, 8, 5, range(0, 6))})
    if "c3" in which:
        dump("c3.json", {"config": "BASELINE config 3: 16384 x 24-bit, -l 32 -q 15 -r 0,8",
                         "units": synth_set("c3", range(2), 16384, 24, 96, 32, 15, range(0, 9))})
    if "c5" in which:
        dump("c5.json", {"config": "BASELINE config 5: fixed-only, 4608 x int16, -r 0,5",
                         "units": synth_set("c5", range(8), 4608, 16, 55, 0, 5, range(0, 6),
                                            fixed_only=True)})
    if "edge" in which:
        dump("edge.json", {"config": "edge cases and reference exceptions", "units": edge_set()})
    if "stream" in which:
        dump("streams.json", stream_set())
    if "acf" in which:
        dump("acf_sites.json", {"config": "Levinson-Durbin / quantiser sites driven from ACF rows",
                                "rows": acf_set()})


if __name__ == "__main__":
    main(sys.argv[1:] or ["c2", "c1", "c3", "c5", "edge", "stream", "acf"])
