"""Device (libflacmi.so HIP kernels) vs the reference's golden vectors and vs the CPU
oracle, bit-exact: autocorrelation (float.hex), every LPC candidate, sums, choice,
residuals, Rice parameters — and the same Python exceptions."""
import math
import random

import numpy as np
import pytest

import golden_util as G
import oracle
import sign_bound
from flac_amd import abi
from flac_amd.analysis import Analyzer, knob, make_params, unit_result

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def az():
    a = Analyzer(0)
    yield a
    a.close()


def run_units(az, units, n, params, bits=16, tail=None, debug=True, residual_bytes=4):
    """units: list of int lists, all of length n except the optional trailing `tail` ones."""
    dt = np.int16 if bits <= 16 else np.int32
    stride = ((n * np.dtype(dt).itemsize + 15) // 16) * 16 // np.dtype(dt).itemsize
    a = np.zeros((len(units), stride), dtype=dt)
    for i, u in enumerate(units):
        a[i, :len(u)] = u
    ntail = 0 if tail is None else tail[1]
    tlen = 0 if tail is None else tail[0]
    return az.analyze(a, params, n, tlen, ntail, sample_bits=bits, residual_bytes=residual_bytes, debug=debug)


# ---------------------------------------------------------------------------------------
# golden fixtures (produced by the reference itself)
# ---------------------------------------------------------------------------------------
def _golden_cases():
    for s in ["c1.json", "c2.json", "c3.json", "c5.json", "edge.json"]:
        d = G.load(s)
        for i, e in enumerate(d["units"]):
            tag = e["source"].get("tag") or f"u{e['source'].get('unit', i)}"
            yield pytest.param(e, id=f"{s[:-5]}-{i}-{tag}"[:60])


@pytest.mark.parametrize("entry", list(_golden_cases()))
def test_device_matches_reference_golden(az, entry):
    xs = G.samples_for(entry, oracle.synth_unit)
    bits = entry["params"]["sample_size"] if entry["source"]["kind"] == "synth" else 16
    bits = max(bits, max((abs(v) for v in xs), default=0).bit_length() + 1)
    out = run_units(az, [xs], len(xs), make_params(**G.params_of(entry)), bits=bits)
    res = unit_result(out, 0)
    bad = G.check(res, entry)
    assert not bad, "\n".join(bad)


# ---------------------------------------------------------------------------------------
# batches vs the oracle
# ---------------------------------------------------------------------------------------
def compare_with_oracle(out, ora, lens):
    gm, om = out["meta"], ora["meta"]
    for u, n in enumerate(lens):
        st = int(om["status"][u])
        assert int(gm["status"][u]) == st, (u, "status", int(gm["status"][u]), st)
        assert int(gm["site"][u]) == int(om["site"][u]), (u, "site")
        if st != 0:
            continue
        bad = oracle.meta_mismatches(gm[u], om[u])
        assert not bad, (u, bad)
        if "lpc_sums" in out:  # debug runs never prune
            assert int(gm["lpc_order"][u]) != abi.LPC_PRUNED, (u, "pruned in a debug run")
        npart = int(om["n_parts"][u])
        assert np.array_equal(out["rice_params"][u][:npart], ora["rice_params"][u][:npart]), (u, "params")
        off, ln = int(om["res_offset"][u]), int(om["res_len"][u])
        assert np.array_equal(out["residual"][u][off:off + ln].astype(np.uint64),
                              ora["residual"][u][off:off + ln]), (u, "residual")
        if "acf" in out:
            assert np.array_equal(out["acf"][u].view(np.uint64), ora["acf"][u].view(np.uint64)), (u, "acf")
            assert np.array_equal(out["fixed_sums"][u], ora["fixed_sums"][u]), (u, "fixed_sums")
            assert np.array_equal(out["lpc_sums"][u], ora["lpc_sums"][u]), (u, "lpc_sums")
            assert np.array_equal(out["lpc_records"][u], ora["lpc_records"][u]), (u, "lpc_records")


def batch_case(az, n_units, n, bits, seed, L, q, rmin, rmax, mode=abi.MODE_REFERENCE, tail=None, threads=16):
    dt = np.int16 if bits <= 16 else np.int32
    a = oracle.synth_batch(0, n_units, n, bits, seed, dtype=dt)
    if tail:
        tl, tn = tail
        a[n_units - tn:, tl:] = 0
    p = make_params(L, q, rmin, rmax, mode)
    out = az.analyze(a, p, n, tail[0] if tail else 0, tail[1] if tail else 0, sample_bits=bits, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, rmin, rmax, mode), n, tail[0] if tail else 0,
                               tail[1] if tail else 0, sample_bits=bits, threads=threads)
    lens = [n] * n_units
    if tail:
        for i in range(n_units - tail[1], n_units):
            lens[i] = tail[0]
    compare_with_oracle(out, ora, lens)
    return out


def test_c2_shape_batch(az):
    """BASELINE config 2 shape: 4608 x int16, -l 12 -q 5 -r 0,5."""
    batch_case(az, 192, 4608, 16, 2024, 12, 5, 0, 5)


@pytest.mark.parametrize("L,mode", [(12, abi.MODE_REFERENCE), (8, abi.MODE_REFERENCE), (0, abi.MODE_FIXED_ONLY)])
def test_stream_constant_and_runtime_shape_builds_agree(az, monkeypatch, L, mode):
    """4608-sample units take k_resid_stream's constant-shape build; the FLACMI_STREAM_GENERIC knob
    takes the runtime-shape build.  Both against the oracle, in production (pruning) mode and
    with every candidate exact, and field for field against each other."""
    n = 4608
    a = oracle.synth_batch(700, 96, n, 16, 31 + L, dtype=np.int16)
    ora = oracle.analyze_batch(a, oracle.make_params(L, 5, 0, 5, mode), n, sample_bits=16, threads=16)
    runs = {}
    for generic in (False, True):
        with knob("FLACMI_STREAM_GENERIC", int(generic)):
            for debug in (False, True):
                out = az.analyze(a, make_params(L, 5, 0, 5, mode), n, sample_bits=16, debug=debug)
                compare_with_oracle(out, ora, [n] * len(a))
                runs[(generic, debug)] = out
    for debug in (False, True):
        x, y = runs[(False, debug)], runs[(True, debug)]
        assert np.array_equal(x["meta"], y["meta"]) and np.array_equal(x["rice_params"], y["rice_params"])
        assert np.array_equal(x["residual"], y["residual"])


@pytest.mark.parametrize("shape", ["c2q6", "c3"])
def test_round_aligned_overlap_chunks(az, monkeypatch, shape):
    """The default chunking (flacmi_host.cpp overlap_mode): k_lpc's whole rounds, then the
    remainder, whose k_lpc runs on the side stream beside k_resid of the first chunk.
    FLACMI_OVERLAP=-R forces R units per round, so a small batch splits: against the oracle
    and field for field against FLACMI_OVERLAP=0 (one chunk), production and debug calls.
    q 6 at config 2 sends about a third of the units of both chunks through the stream kernel's
    retry list."""
    if shape == "c3":
        n, bits, L, q, rmax, units, R, dt = 16384, 24, 32, 15, 8, 40, 24, np.int32
    else:
        n, bits, L, q, rmax, units, R, dt = 4608, 16, 12, 6, 5, 200, 128, np.int16
    a = oracle.synth_batch(1300, units, n, bits, 77, dtype=dt)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, rmax), n, sample_bits=bits, threads=16)
    runs = {}
    for ov in ("0", "-%d" % R):
        with knob("FLACMI_OVERLAP", int(ov)):
            for debug in (False, True):
                out = az.analyze(a, make_params(L, q, 0, rmax), n, sample_bits=bits, debug=debug)
                compare_with_oracle(out, ora, [n] * units)
                runs[(ov, debug)] = out
    for debug in (False, True):
        x, y = runs[("0", debug)], runs[("-%d" % R, debug)]
        assert np.array_equal(x["meta"], y["meta"]) and np.array_equal(x["rice_params"], y["rice_params"])
        assert np.array_equal(x["residual"], y["residual"])
    if shape == "c2q6":
        st = runs[("0", False)]["meta"]["lpc_tiers"].astype(np.int64)
        listed = np.nonzero(st >> 8 == 1)[0]
        assert (listed < R).any() and (listed >= R).any(), listed


@pytest.mark.parametrize("q", [6, 7, 9, 15])
def test_c2_shape_fast_kernel_and_retry_list(az, q):
    """config 2 shape at higher precisions: the fast S16 MFMA kernel takes the units inside
    its exactness bound (sum|c| + 2^shift <= 127) and hands the rest to the generic kernel
    through the retry list; q = 15 sends every LPC unit there."""
    batch_case(az, 96, 4608, 16, 300 + q, 12, q, 0, 5)
    batch_case(az, 64, 4608, 16, 400 + q, 8, q, 0, 5)


def test_c1_params_with_short_tail(az):
    """config 1 parameters with a stream's short last block (3240 samples)."""
    batch_case(az, 40, 4608, 16, 7, 8, 5, 0, 5, tail=(3240, 1))


def test_c3_shape_batch(az):
    """BASELINE config 3 shape: 16384 x 24-bit, -l 32 -q 15 -r 0,8."""
    batch_case(az, 12, 16384, 24, 96, 32, 15, 0, 8)


def test_c5_fixed_only_batch(az):
    batch_case(az, 256, 4608, 16, 55, 0, 5, 0, 5, mode=abi.MODE_FIXED_ONLY)


@pytest.mark.parametrize("L", [1, 2, 3, 5, 8, 11, 13, 16, 20, 24, 31, 32])
def test_every_order_bucket(az, L):
    batch_case(az, 24, 1152, 16, 100 + L, L, 5 + (L % 9), 0, 6)


def test_random_edge_units(az):
    """Small random blocks of every length 1..64 and odd params: statuses, sites and
    results all equal the oracle's (which the golden tests pin to the reference)."""
    rnd = random.Random(7)
    for trial in range(40):
        n = rnd.randint(1, 64)
        L = rnd.choice([0, 1, 2, 4, 8, 12])
        q = rnd.choice([5, 6, 9, 15])
        rmin = rnd.choice([0, 0, 1, 2])
        rmax = rnd.choice([rmin - 1, rmin, rmin + 2, 6])
        mode = rnd.choice([abi.MODE_REFERENCE, abi.MODE_REFERENCE, abi.MODE_FIXED_ONLY])
        amp = rnd.choice([0, 1, 3, 100, 30000])
        units = [[rnd.randint(-amp, amp) for _ in range(n)] for _ in range(8)]
        a = np.zeros((8, ((n + 7) // 8) * 8), dtype=np.int16)
        for i, u in enumerate(units):
            a[i, :n] = u
        if rmax < rmin:
            rmax_c = rmin - 1
        else:
            rmax_c = rmax
        p = make_params(L, q, rmin, rmax_c, mode)
        out = az.analyze(a, p, n, sample_bits=16, debug=True)
        ora = oracle.analyze_batch(a, oracle.make_params(L, q, rmin, rmax_c, mode), n, sample_bits=16)
        compare_with_oracle(out, ora, [n] * 8)


def test_device_pypow2_and_floor_log2_match_libm(az):
    import ctypes as C
    rnd = random.Random(3)
    xs = [rnd.uniform(-1, 1) for _ in range(200000)]
    xs += [math.ldexp(rnd.uniform(0.5, 1), rnd.randint(-1074, 1023)) for _ in range(100000)]
    xs += [0.0, -0.0, 1.0, -1.0, math.inf, 5e-324, 1e154, 1.3407807929942596e154, 1e200, 2.0 ** -600]
    x = np.array(xs, dtype=np.float64)
    got = np.zeros_like(x)
    st = np.zeros(len(x), dtype=np.int32)
    lib = az.lib
    rc = lib.flacmi_device_selftest(az.ctx, 0, x.ctypes.data, got.ctypes.data, st.ctypes.data, len(x))
    assert rc == 0
    for i in range(0, len(x), 97):
        want, wst = oracle.pypow2(float(x[i]))
        assert got[i] == want or (math.isnan(got[i]) and math.isnan(want)), (x[i].hex(), got[i], want)
        assert st[i] == wst
    # full corpus against the host emulation (itself checked against libm in test_pymath)
    hst = C.c_int32()
    host = np.array([lib.flacmi_host_pypow2(float(v), hst) for v in x])
    assert np.array_equal(host.view(np.uint64), got.view(np.uint64))
    pos = np.abs(x[np.isfinite(x) & (x != 0)])
    got2 = np.zeros_like(pos)
    st2 = np.zeros(len(pos), dtype=np.int32)
    assert lib.flacmi_device_selftest(az.ctx, 1, pos.ctypes.data, got2.ctypes.data, st2.ctypes.data, len(pos)) == 0
    for i in range(0, len(pos), 53):
        assert int(got2[i]) == oracle.floor_log2(float(pos[i]))[0]


def test_device_lpc_sites_from_acf_rows(az):
    """k_lpc's Levinson-Durbin + quantiser driven from ACF rows (flacmi_device_lpc_from_acf)
    against the reference's outcome on the same rows (tests/golden/acf_sites.json): the
    OverflowError sites encoder.py:476 (lambda_ ** 2) and :503 (floor(log2(inf))) that no
    integer PCM block reaches, plus the other Levinson/quantiser outcomes."""
    from collections import defaultdict
    groups = defaultdict(list)
    for row in G.acf_rows():
        groups[(row["L"], row["q"])].append(row)
    sites, bad = set(), []
    for (L, q), rows in groups.items():
        acf = np.zeros((len(rows), 33), dtype=np.float64)
        for i, r in enumerate(rows):
            acf[i, : L + 1] = r["acf_values"]
        rec = np.zeros((len(rows), abi.lpc_rec_words(L)), dtype=np.int32)
        assert az.lib.flacmi_device_lpc_from_acf(az.ctx, acf.ctypes.data, len(rows), L, q, rec.ctypes.data) == 0
        for i, r in enumerate(rows):
            bad += [f"L={L} q={q} row {i}: {m}" for m in G.check_acf_record(rec[i], r)]
            if r.get("exception"):
                sites.add(int(rec[i, 0]) >> 16)
    assert not bad, "\n".join(bad[:20])
    assert {3, 5} <= sites, sites


@pytest.mark.parametrize("open_eighths", [0, 5, 8])
def test_synth_device_matches_oracle(az, open_eighths):
    """k_synth vs oracle_synth_unit(_mix): the tone recipe and (open_eighths > 0) the open
    mix's MA(1) noise units, every width."""
    n_units, n = 9 if open_eighths == 0 else 24, 4608
    # bits <= 24: the 32-bit path of k_synth; 28 and 31 (the widest it takes): its int64 path
    for bits, dt in ((8, np.int16), (12, np.int16), (16, np.int16), (20, np.int32), (24, np.int32),
                     (28, np.int32), (31, np.int32)):
        nbytes = np.dtype(dt).itemsize
        d = az.lib.flacmi_device_alloc(az.ctx, n_units * n * nbytes)
        az.synth_device(d, nbytes, bits, n, 5, n_units, n, 42, open_eighths=open_eighths)
        host = np.zeros((n_units, n), dtype=dt)
        assert az.lib.flacmi_memcpy_d2h(az.ctx, host.ctypes.data, d, host.nbytes) == 0
        az.lib.flacmi_device_free(az.ctx, d)
        want = oracle.synth_batch(5, n_units, n, bits, 42, dtype=dt, open_eighths=open_eighths)
        assert np.array_equal(host, want), bits


# ---------------------------------------------------------------------------------------
# 24-bit wide paths: the narrow (32-bit |r|) sums and the int64 ones
# ---------------------------------------------------------------------------------------
def _tones24(n_units, n, seed, noise):
    """Near-full-scale 24-bit tone sums; without noise, high-order LPC candidates get
    sum|c| >= 30 * 2^shift (outside the narrow bound), with it they stay inside."""
    r = np.random.default_rng(seed)
    t = np.arange(n)
    a = np.zeros((n_units, n), np.int32)
    for u in range(n_units):
        x = np.zeros(n)
        for _ in range(r.integers(1, 4)):
            x += r.uniform(0.1, 0.3) * np.sin(2 * np.pi * r.uniform(5, 2000) / 96000 * t + r.uniform(0, 6.28))
        x = x * (2 ** 23 - 1) + r.normal(0, noise, n)
        a[u] = np.clip(np.round(x), -2 ** 23, 2 ** 23 - 1)
    return a


def _outside_narrow(ora, L):
    cnt = 0
    for rec in ora["lpc_records"]:
        if rec[0] != 0:
            continue
        for p in range(1, L + 1):
            sh = int(rec[2 + p - 1])
            c = rec[2 + L + p * (p - 1) // 2: 2 + L + p * (p - 1) // 2 + p].astype(np.int64)
            cnt += int(np.abs(c).sum() >= 30 * 2 ** sh)
    return cnt


@pytest.mark.parametrize("q", [15, 12])
@pytest.mark.parametrize("noise", [0.0, 0.5, 4.0])
def test_24bit_tones_narrow_and_wide_candidate_sums(az, q, noise):
    n, L = 4096, 32
    a = _tones24(16, n, 11, noise)
    out = az.analyze(a, make_params(L, q, 0, 8), n, sample_bits=24, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 8), n, sample_bits=24, threads=16)
    if noise == 0.0:
        assert _outside_narrow(ora, L) > 0  # the int64 sums are exercised
    compare_with_oracle(out, ora, [n] * 16)


@pytest.mark.parametrize("L", [16, 17, 24, 32])
@pytest.mark.parametrize("bits", [20, 24])
def test_int8_mfma_candidate_sums_orders(az, L, bits):
    """PATH_W64 int8-MFMA candidate sums (k_resid.h mf8_*): both N-tiles, partial second
    N-tile, masked warm-up tiles, 20/24-bit synthetic units and tones, against the oracle."""
    n = 2048
    a = oracle.synth_batch(0, 24, n, bits, 500 + L + bits, dtype=np.int32)
    t = _tones24(8, n, L + bits, 2.0) >> (24 - bits)
    a = np.concatenate([a, t])
    for q in (15, 11):
        out = az.analyze(a, make_params(L, q, 0, 6), n, sample_bits=bits, debug=True)
        ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 6), n, sample_bits=bits, threads=16)
        compare_with_oracle(out, ora, [n] * len(a))


def test_int8_mfma_fallbacks(az):
    """Units the int8 path must hand to the int64 chains: a top digit of 128 (a sample above
    8355711) or of -129 (a 25-bit sample below -8421504), n not a multiple of 16; next to
    ordinary units, the most negative 24-bit sample and both ends of the int8 digit range."""
    n = 2048
    a = oracle.synth_batch(0, 12, n, 24, 77, dtype=np.int32)
    a[1, 700] = 8355712
    a[2, 5] = 2 ** 23 - 1
    a[3, 1000:1100] = -2 ** 23
    a[4, :] = a[4, :] // 2 + 8355711 // 2
    out = az.analyze(a, make_params(32, 15, 0, 6), n, sample_bits=24, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(32, 15, 0, 6), n, sample_bits=24, threads=16)
    compare_with_oracle(out, ora, [n] * len(a))
    # 25-bit samples: the top digit leaves int8 below -0x808080 as well as above 0x7f7f7f
    c = oracle.synth_batch(100, 8, n, 25, 78, dtype=np.int32) // 4
    c[1, 300] = -0x808081  # one past the lower end: the int64 chains
    c[2, 301] = -0x808080  # the lower end itself: still int8 digits
    c[3, 302] = 0x7f7f7f
    c[4, 303:310] = -0x900000
    for bits in (25, 24):
        cc = c if bits == 25 else np.clip(c, -2 ** 23, 2 ** 23 - 1)
        out = az.analyze(cc, make_params(32, 15, 0, 6), n, sample_bits=bits, debug=True)
        ora = oracle.analyze_batch(cc, oracle.make_params(32, 15, 0, 6), n, sample_bits=bits, threads=16)
        compare_with_oracle(out, ora, [n] * len(cc))
    m = 2040  # n % 16 != 0
    b = np.ascontiguousarray(a[:, :m])
    out = az.analyze(b, make_params(32, 15, 0, 3), m, sample_bits=24, debug=True)
    ora = oracle.analyze_batch(b, oracle.make_params(32, 15, 0, 3), m, sample_bits=24, threads=16)
    compare_with_oracle(out, ora, [m] * len(b))


def test_split_plane_path_opt_in():
    """PATH_W64S (opt-in, FLACMI_SPLIT=1, read once per process): config 3 shape and
    full-scale tones, in a child process, bit-exact against the oracle."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path[:0] = ['tests', 'oracle', '.']\n"
            "import test_gpu_parity as T\n"
            "from flac_amd.analysis import Analyzer, make_params\n"
            "az = Analyzer(0)\n"
            "T.batch_case(az, 12, 16384, 24, 97, 32, 15, 0, 8)\n"
            "a = T._tones24(16, 4096, 12, 0.0)\n"
            "out = az.analyze(a, make_params(32, 15, 0, 8), 4096, sample_bits=24, debug=True)\n"
            "ora = T.oracle.analyze_batch(a, T.oracle.make_params(32, 15, 0, 8), 4096, sample_bits=24, threads=16)\n"
            "T.compare_with_oracle(out, ora, [4096] * 16)\n"
            "az.close()\n"
            "print('split ok')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, env={**os.environ, "FLACMI_SPLIT": "1"},
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "split ok" in r.stdout, r.stdout[-1000:] + r.stderr[-3000:]


@pytest.mark.parametrize("mode", [abi.MODE_FIXED_ONLY, abi.MODE_REFERENCE])
def test_large_residuals_chunked_rice_bits(az, mode):
    """32-bit samples near +-2^30 in long blocks (LDS-resident residual, 256 finest
    partitions): zig-zag values >= 2^29 take the chunked data-bits pass's 64-bit branch,
    quiet units its 32-bit one."""
    n, nu = 16384, 8
    r = np.random.default_rng(5)
    a = np.zeros((nu, n), np.int32)
    for u in range(nu):
        amp = [2 ** 30, 2 ** 12][u % 2]
        a[u] = r.integers(-amp, amp, n, dtype=np.int64).astype(np.int32)
    L = 0 if mode == abi.MODE_FIXED_ONLY else 8
    out = az.analyze(a, make_params(L, 12, 0, 8, mode), n, sample_bits=32, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(L, 12, 0, 8, mode), n, sample_bits=32, threads=16)
    assert int((ora["meta"]["status"] == 0).sum()) >= nu // 2
    compare_with_oracle(out, ora, [n] * nu)


def test_long_blocks_are_declared_unsupported(az):
    """The reference writes blocks up to 65535 samples (16-bit uncommon block-size code,
    encoder.py:249-253); the API accepts them, and a block whose workgroup staging exceeds
    the 160 KB LDS is refused with FLACMI_E_UNSUPPORTED naming the LDS need,
    never with E_INVALID and never by a failed launch."""
    from flac_amd._lib import FlacmiError
    params = make_params(8, 5, 0, 5)
    for n in (40000, 65535):
        rows = np.zeros((1, ((n * 2 + 15) // 16) * 8), dtype=np.int16)
        with pytest.raises(FlacmiError) as ei:
            az.analyze(rows, params, n)
        assert f"({abi.E_UNSUPPORTED})" in str(ei.value) and "LDS" in str(ei.value)


def test_wide_chosen_residual_redoes_only_those_units(az):
    """32-bit samples where the chosen residual needs more than 32 bits (a near-full-scale block
    with one opposite spike: order 1 wins with |r| ~ 2^32) next to ordinary units and a short
    tail unit: the analyzer redoes only the wide units with 64-bit rows; every unit equals
    the oracle."""
    n, nu = 1024, 8
    a = oracle.synth_batch(0, nu, n, 32, 9, dtype=np.int32)
    r = np.random.default_rng(5)
    for u in (1, 4, 7):
        a[u, :] = (2 ** 31 - 1000) + r.integers(-100, 100, n)
        a[u, 300 + u] = -2 ** 31
    a[7, 700:] = 0  # the tail unit (700 samples)
    p = make_params(8, 12, 0, 4)  # sample_bits + q <= 44
    out = az.analyze(a, p, n, 700, 1, sample_bits=32, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(8, 12, 0, 4), n, 700, 1, sample_bits=32, threads=8)
    assert out["residual"].dtype == np.uint64
    assert int(np.max(ora["residual"][1])) >= 2 ** 32
    compare_with_oracle(out, ora, [n] * (nu - 1) + [700])


@pytest.mark.parametrize("n,rmax", [(4096, 8), (2048, 6), (8192, 7), (4608, 6), (12288, 7), (6144, 8)])
def test_wide_rice_wave0_parameters_and_errors(az, n, rmax):
    """PATH_W64 with 64..256 finest partitions: the heap nodes' parameters come from the
    finest sums phase E reduced across the lanes that own a partition's chunks (4608/6,
    12288/7, 6144/8: 9, 12 and 3 chunks per finest partition, not a power of two).  Silent stretches give a zero
    partition sum (log of 0: ValueError), sparse +-1 stretches a mean below 1 (negative
    parameter); loud units exercise Rice5Bit parameters (> 14) at every level."""
    r = np.random.default_rng(n + rmax)
    a = oracle.synth_batch(0, 16, n, 24, n + rmax, dtype=np.int32)
    a[1, n // 2:] = 0                                    # zero partitions (coarse orders still fine)
    a[2, :] = 0
    a[2, ::97] = r.integers(-1, 2, len(a[2, ::97]))      # sums below the partition length
    a[3, 3 * n // 4:] = 0
    a[3, 3 * n // 4::5] = 1
    a[4, :] = r.integers(-2 ** 23, 2 ** 23, n)           # white full-scale noise: parameters > 14
    a[5, : n // 8] = 0                                   # silent start (first partition shorter)
    a[6, :] = (r.integers(-3, 4, n) * (np.arange(n) % 512 < 64)).astype(np.int32)
    out = az.analyze(a, make_params(32, 15, 0, rmax), n, sample_bits=24, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(32, 15, 0, rmax), n, sample_bits=24, threads=16)
    sts = set(int(v) for v in ora["meta"]["status"])
    compare_with_oracle(out, ora, [n] * len(a))
    assert len(sts) >= 2, sts


def test_stream_rice_parameters_of_16_and_more(az):
    """k_resid_stream's packed Rice pass shifts 16-bit pairs by the parameter, which
    v_pk_lshrrev_b16 takes mod 16: a finest partition whose mean is >= 2^16 (parameter >= 16)
    while some of its chunks stay below 2^16 must take the 32-bit path.  Loud smooth sines
    (fixed order 1 wins) with full-scale alternation in 10..14 chunks of one finest partition:
    that partition's parameter is 16, and the oracle picks the 32 finest partitions."""
    n, units = 4608, 8
    r = np.random.default_rng(7)
    a = np.zeros((units, n), np.int16)
    t = np.arange(n)
    for u in range(units):
        x = (20000 + 1000 * u) * np.sin(2 * np.pi * t / (900 + 37 * u) + u) + r.normal(0, 3, n)
        k = 5 + 3 * u
        for c in range(10 + u % 5):
            x[144 * k + 8 * c: 144 * k + 8 * c + 8] = 32767 * np.array([1, -1] * 4)
        a[u] = np.clip(np.round(x), -32768, 32767)
    out = az.analyze(a, make_params(12, 5, 0, 5), n, sample_bits=16, debug=True)
    ora = oracle.analyze_batch(a, oracle.make_params(12, 5, 0, 5), n, sample_bits=16, threads=16)
    assert set(int(v) for v in ora["meta"]["part_order"]) == {5}
    compare_with_oracle(out, ora, [n] * units)


@pytest.mark.parametrize("rmin,rmax", [(0, 6), (3, 2)])
def test_fast_kernel_stages_the_whole_record(az, rmin, rmax):
    """The S16 fast kernel with a 64-thread workgroup (n = 1024) and L = 12: the LPC record
    (92 words) is longer than the workgroup, so each thread stages two words.  Many units per
    launch, so a word left unstaged would read another unit's record from LDS.  r 0..6 and
    the empty Rice range keep k_resid_stream out (more than 32 finest partitions / none)."""
    batch_case(az, 256, 1024, 16, 31 + rmin, 12, 5, rmin, rmax)


def _meta_params_residual_equal(a, b, u):
    """a: production run (may prune), b: a run with every LPC candidate's exact sum."""
    am, bm = a["meta"], b["meta"]
    pruned = int(am["lpc_order"][u]) == abi.LPC_PRUNED
    for f in abi.META_DTYPE.names:
        if f == "lpc_tiers" or (pruned and f in ("lpc_order", "lpc_sum")):
            continue
        assert np.array_equal(am[f][u], bm[f][u]), (u, f, am[f][u], bm[f][u])
    if pruned:
        assert int(am["lpc_sum"][u]) == abi.LPC_PRUNED
        assert int(bm["kind"][u]) == abi.KIND_FIXED and int(bm["lpc_sum"][u]) > int(bm["fixed_sum"][u]), u
    if int(am["status"][u]) == 0:
        k = int(am["n_parts"][u])
        assert np.array_equal(a["rice_params"][u][:k], b["rice_params"][u][:k]), (u, "params")
        off, ln = int(am["res_offset"][u]), int(am["res_len"][u])
        assert np.array_equal(a["residual"][u][off:off + ln], b["residual"][u][off:off + ln]), (u, "residual")


@pytest.mark.parametrize("entry", list(_golden_cases()))
def test_golden_without_debug_outputs(az, entry):
    """The production call (no debug outputs) against the debug run that
    test_device_matches_reference_golden pins to the reference: every golden unit, fixed/LPC
    winner, tie assertion and exception included, gives the same meta, parameters and
    residual."""
    xs = G.samples_for(entry, oracle.synth_unit)
    bits = entry["params"]["sample_size"] if entry["source"]["kind"] == "synth" else 16
    bits = max(bits, max((abs(v) for v in xs), default=0).bit_length() + 1)
    p = make_params(**G.params_of(entry))
    full = run_units(az, [xs], len(xs), p, bits=bits, debug=True)
    pruned = run_units(az, [xs], len(xs), p, bits=bits, debug=False)
    _meta_params_residual_equal(pruned, full, 0)


@pytest.mark.parametrize("q", [5, 7, 9])
def test_production_call_near_tied_orders_vs_oracle(az, q):
    """Config-2 shape batches through the production call (no debug outputs) against the
    oracle, plus units whose LPC orders nearly tie: pure tones (several orders predict them
    equally well) and quantisation-limited noise."""
    n = 4608
    a = oracle.synth_batch(0, 160, n, 16, 900 + q, dtype=np.int16)
    t = np.arange(n)
    for u in range(8):
        a[u] = np.round(8000 * np.sin(2 * np.pi * (u + 1) * 37.0 / 4608 * t)).astype(np.int16)
    r = np.random.default_rng(q)
    a[8:16] = r.integers(-3, 4, (8, n)).astype(np.int16)
    out = az.analyze(a, make_params(12, q, 0, 5), n, sample_bits=16, debug=False)
    ora = oracle.analyze_batch(a, oracle.make_params(12, q, 0, 5), n, sample_bits=16, threads=16)
    compare_with_oracle(out, ora, [n] * len(a))


def _outside_stream_bound(ora, L, limit=127):
    """Units with an LPC order outside k_resid_stream's MFMA exactness bound
    (sum|c| + 2^shift > 127): the stream kernel lists them for k_resid's list variant."""
    cnt = 0
    for rec in ora["lpc_records"]:
        if rec[0] != 0:
            continue
        for p in range(1, L + 1):
            base = 2 + 32 + p * (p - 1) // 2
            if int(np.abs(rec[base: base + p].astype(np.int64)).sum()) + (1 << int(rec[2 + p - 1])) > limit:
                cnt += 1
                break
    return cnt


@pytest.mark.parametrize("q", [7, 8, 9])
@pytest.mark.parametrize("debug", [True, False])
def test_stream_retry_list_above_6144(az, q, debug):
    """n = 8192 takes k_resid_stream (n <= 10240) while the retry list's k_resid variant keeps
    its residual in LDS (n > 8 * kCPT * 256): the list launch must size its LDS the way that
    variant carves it (it used the register-resident layout).  Some units must
    actually be retried."""
    n, nu = 8192, 48
    a = oracle.synth_batch(0, nu, n, 16, 8000 + q, dtype=np.int16)
    ora = oracle.analyze_batch(a, oracle.make_params(12, q, 0, 5), n, sample_bits=16, threads=16)
    assert _outside_stream_bound(ora, 12) > 0
    out = az.analyze(a, make_params(12, q, 0, 5), n, sample_bits=16, debug=debug)
    compare_with_oracle(out, ora, [n] * nu)


def _prune_signals(n, seed):
    """Units on every side of the LPC lower bound: config-2 synthetic units (pruned), AR(1)
    noise (LPC within 1.3x of fixed: the half-block bound fails, the exact pass runs and
    fixed wins), white noise (LPC wins or loses by a few units) and tones."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    rows = [oracle.synth_batch(0, 24, n, 16, seed, dtype=np.int16)]
    x = []
    for u in range(8):
        w = rng.normal(0, 2000, n)
        ar = w.copy()
        ar[1:] += (0.9 if u % 2 else -0.7) * w[:-1]
        x += [ar, rng.integers(-3000, 3000, n), 8000 * np.sin(2 * np.pi * (u + 1) * 37 / n * t) + rng.normal(0, 40, n)]
    rows.append(np.clip(np.round(np.array(x)), -32768, 32767).astype(np.int16))
    return np.concatenate(rows)


@pytest.mark.parametrize("q", [5, 9, 15])
def test_lpc_pruning_paths_vs_oracle(az, q):
    """Production calls prune LPC candidates whose lower bound already loses (include/flacmi.h
    FLACMI_LPC_PRUNED): every reference-visible field equals the oracle on pruned units, on
    units where the bound fails and the exact pass decides for fixed, and on LPC-chosen units;
    FLACMI_FLAG_ALL_CANDIDATES gives the exact LPC sums with the same results."""
    n = 4608
    a = _prune_signals(n, 50 + q)
    ora = oracle.analyze_batch(a, oracle.make_params(12, q, 0, 5), n, sample_bits=16, threads=16)
    prod = az.analyze(a, make_params(12, q, 0, 5), n, sample_bits=16)
    full = az.analyze(a, make_params(12, q, 0, 5, all_candidates=True), n, sample_bits=16)
    compare_with_oracle(prod, ora, [n] * len(a))
    compare_with_oracle(full, ora, [n] * len(a))
    pm, om = prod["meta"], ora["meta"]
    assert not (full["meta"]["lpc_order"] == abi.LPC_PRUNED).any()
    for u in range(len(a)):
        _meta_params_residual_equal(prod, full, u)
    ok = om["status"] == 0
    pruned = pm["lpc_order"] == abi.LPC_PRUNED
    if q == 5:  # (q >= 9 at L 12 takes the 64-bit path: no pruning there)
        assert pruned[:24].sum() >= 12, "config-2 units should mostly prune"
    # meta.lpc_tiers: k_resid_stream's quarter bound passes 1..4 (pruned) or 5 (the exact
    # pass), x/4; for the units its retry list redid on k_resid, the 16-bit sign-correlation
    # bound: 0/1 (pruned before the LPC pass) or 1/1 (the exact pass)
    tiers = pm["lpc_tiers"].astype(np.int64)
    st = tiers != 0
    s4, s1 = st & (tiers >> 8 == 4), st & (tiers >> 8 == 1)
    assert (s4 | s1 | ~st).all(), np.unique(tiers)
    assert (pruned[s4] == ((tiers[s4] & 0xff) <= 4)).all()
    assert ((tiers[s4] & 0xff) <= 5).all() and ((tiers[s4] & 0xff) >= 1).all()
    assert (pruned[s1] == ((tiers[s1] & 0xff) == 0)).all() and ((tiers[s1] & 0xff) <= 1).all()
    assert not pruned[~st].any()
    if q == 5:  # the LPC-winning units the stream kernel lists take the 16-bit bound's exact pass
        assert (tiers == (1 | 1 << 8)).any(), np.unique(tiers)
    if q == 5:  # pruned after the first quarter, and after later ones
        assert (tiers == (1 | 4 << 8)).any() and ((tiers[st] & 0xff) >= 2).any(), np.unique(tiers)
    assert (ok & ~pruned & (om["kind"] == abi.KIND_FIXED)).any(), "no unit took the exact pass and chose fixed"
    assert (ok & (om["kind"] == abi.KIND_LPC)).any(), "no LPC-chosen unit"


def _stream_tap_sums(rec, L):
    """Per LPC order p <= L of the oracle's record: (sum|c_p|, 2^shift_p), the two terms of
    k_resid_stream's f16-MFMA exactness bounds (coefficient-less orders: (0, 1))."""
    out = []
    for p in range(1, L + 1):
        if (int(rec[1]) >> (p - 1)) & 1:
            out.append((0, 1))
            continue
        base = 2 + 32 + p * (p - 1) // 2
        out.append((int(np.abs(rec[base:base + p].astype(np.int64)).sum()), 1 << int(rec[2 + p - 1])))
    return out


@pytest.mark.parametrize("cfg", ["c2", "c2open", "c2q6", "c3", "c3open"])
def test_production_batches_vs_oracle(az, cfg):
    """Production calls (no debug outputs: LPC pruning on, every kernel variant the dispatch
    picks) over larger batches of the bench's own synthetic units against the oracle: 2048
    config-2 units (k_resid_stream, its list kernel, k_resid's list variant) and 192 config-3
    units (k_resid_sb, kVarList1's int8-MFMA tiers, the packed Rice pass); the "open" batches
    are bench.py --open 5 (5/8 of the units MA(1) near-white noise: LPC near-ties no bound
    decides, LPC wins some).  A unit reporting FLACMI_LPC_PRUNED must lose to fixed in the
    oracle; every other field is compared bit for bit."""
    open8 = 5 if cfg.endswith("open") else 0
    if cfg == "c2q6":  # q 6: 2^shift lists a third of the units, sum|c| > 127 an eighth
        n, bits, L, q, rmax, units, dt = 4608, 16, 12, 6, 5, 512, np.int16
    elif cfg.startswith("c2"):
        n, bits, L, q, rmax, units, dt = 4608, 16, 12, 5, 5, 2048, np.int16
    else:
        n, bits, L, q, rmax, units, dt = 16384, 24, 32, 15, 8, 192, np.int32
    a = oracle.synth_batch(5000, units, n, bits, 11, dtype=dt, open_eighths=open8)
    out = az.analyze(a, make_params(L, q, 0, rmax), n, sample_bits=bits)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, rmax), n, sample_bits=bits, threads=16)
    compare_with_oracle(out, ora, [n] * units)
    pruned = out["meta"]["lpc_order"] == abi.LPC_PRUNED
    assert pruned.mean() > (0.2 if open8 else 0.5 if q > 5 else 0.9), pruned.mean()
    assert (ora["meta"]["kind"][pruned] == abi.KIND_FIXED).all()
    if open8:
        ok = ora["meta"]["status"] == 0
        assert (ora["meta"]["kind"][ok] == abi.KIND_LPC).sum() > 0.05 * units  # LPC winners
    if cfg.startswith("c2"):
        # k_resid_stream lists the units outside its f16 bound (sum|c| + 2^shift) * 33023 < 2^22.
        # Its list kernel redoes them with pred-only taps (exact while sum|c| <= 127): one exact
        # pass, lpc_tiers 1/1.  A unit outside that too takes k_resid's 16-bit sign-correlation
        # bound over R' = [16, n): 0/1 exactly when the bound restated on the oracle's record
        # decides, 1/1 (the exact LPC pass) otherwise.
        t = out["meta"]["lpc_tiers"].astype(np.int64)
        seen = set()
        for u in range(units):
            if int(ora["meta"]["status"][u]) != 0 and int(ora["meta"]["site"][u]) != abi.SITE_CHOICE_TIE:
                continue
            sums = _stream_tap_sums(ora["lpc_records"][u], L)
            if all((c + sh) * 33023 < 2 ** 22 for c, sh in sums):
                assert int(t[u]) >> 8 == 4, (u, int(t[u]))  # the batch kernel's quarter tiers
                seen.add("batch")
            elif all(c <= 127 for c, _ in sums):
                assert int(t[u]) == 1 | 1 << 8, (u, int(t[u]))
                seen.add("list")
            else:
                want = sign_bound.decides(a[u], ora["lpc_records"][u], L, ora["fixed_sums"][u], lmax=16)
                assert int(t[u]) == ((1 << 8) if want else (1 | 1 << 8)), (u, int(t[u]), want)
                seen.add("list2")
        assert seen >= {"c2": {"batch"}, "c2open": {"batch", "list"}, "c2q6": {"batch", "list", "list2"}}[cfg], seen


# ---------------------------------------------------------------------------------------
# config-3 production mode: the int8-MFMA path's LPC pruning tiers (k_resid.h
# mf8_candidate_sums) against the oracle, with the tier that decided each unit
# ---------------------------------------------------------------------------------------
def _resid_threads_wide(n):
    """device_common.h resid_threads(n, wide=true): k_resid's workgroup on the 64-bit paths."""
    nch = (n + 7) // 8
    nt = 64 * ((nch + 64 * 3 - 1) // (64 * 3))
    return max(64, min(nt, 512))


def _lpc_abs_tiles(x, rec, p):
    """|r| of LPC order p (encoder.py:537-548) from the oracle's record, summed per 16-sample
    tile, zero below the candidate's first residual (p, or 0 in the negative-shift branch)."""
    n = len(x)
    x64 = x.astype(np.int64)
    r = np.zeros(n, np.int64)
    if (int(rec[1]) >> (p - 1)) & 1:  # ([], 0): the residual is the samples
        r = np.abs(x64)
    else:
        sh = int(rec[2 + p - 1])
        c = rec[2 + 32 + p * (p - 1) // 2: 2 + 32 + p * (p - 1) // 2 + p].astype(np.int64)
        pred = np.zeros(n - p, np.int64)
        for j in range(p):
            pred += c[j] * x64[p - 1 - j: n - 1 - j]
        r[p:] = np.abs(x64[p:] - (pred >> sh))
    return r.reshape(-1, 16).sum(1)


def _int8_path(x, rec, L):
    """Whether k_resid runs the unit's candidate sums on int8 MFMA (k_resid.h, phase A's
    bound): every sample's top balanced digit fits a byte (x <= 8355711), every coefficient's
    top digit too (c in [-32640, 32639]), and B = max|x| + max_p (sum|c_p| max|x| >> s_p) + 1 <
    2^29.  Otherwise the exact int64 chains run, without pruning."""
    xa = x.astype(np.int64)
    if int(xa.max()) > 8355711:
        return False
    xm = int(np.abs(xa).max())
    b = 0
    for p in range(1, L + 1):
        c = rec[2 + 32 + p * (p - 1) // 2: 2 + 32 + p * (p - 1) // 2 + p].astype(np.int64)
        if (c > 32639).any() or (c < -32640).any():
            return False
        sa = int(np.abs(c).sum()) & 0xFFFFFFFF
        b = max(b, xm + ((sa * xm) >> int(rec[2 + p - 1])) + 1)
    return b < (1 << 29)


def _emulate_eighths(x, rec, L, fixed_sums):
    """The pruning decision of mf8_candidate_sums restated on the oracle's record: wave w
    of nw owns tiles w + k nw; the eighths run residues {0, 4}, 2, 6, 1, 5, 3, 7 of k mod 8;
    after each, the unit is pruned when every order's exact partial sum exceeds the best
    fixed sum (encoder.py:135-157: LPC can then neither win nor tie).  -> (eighths, pruned)."""
    ntile = len(x) // 16
    k = np.arange(ntile) // (_resid_threads_wide(len(x)) // 64)
    per = np.array([_lpc_abs_tiles(x, rec, p) for p in range(1, L + 1)])
    fmin = int(np.min(fixed_sums))
    mask = np.zeros(ntile, bool)
    done = 0
    for res in ((0, 4), (2,), (6,), (1,), (5,), (3,), (7,)):
        for r_ in res:
            mask |= (k % 8) == r_
        done += len(res)
        if done < 8 and (per[:, mask].sum(1) > fmin).all():
            return done, True
    return 8, False


def _sb_lean(n, rmax=8):
    """k_resid.h launch_resid_sb's shapes (k_resid_sb, which tests the bound first over each
    thread's first two chunks: R' = [lmax, 8192) with 512 threads)."""
    om = max(o for o in range(0, rmax + 1) if n % (1 << o) == 0)
    cpp = (n >> om) // 8
    return 8192 <= n <= 16384 and n % 256 == 0 and 6 <= om <= 8 and (n >> om) % 8 == 0 and cpp & (cpp - 1) == 0


@pytest.mark.parametrize("n,L,rmax", [(16384, 32, 8), (8192, 32, 8), (8192, 32, 7), (8192, 32, 6),
                                     (16384, 16, 8), (16384, 20, 7)])
def test_sb_builds_vs_oracle(az, n, L, rmax):
    """k_resid_sb's builds through production calls against the oracle: the config-3 constant
    build (16384 samples, L 32, Rice orders 0..8), the orders-0..8 build at runtime n and L,
    and the generic build (finest order 6 or 7).  A unit the bound decides reports 0/8 tiers
    and must lose to fixed in the oracle; every unit matches the oracle field for field."""
    assert _sb_lean(n, rmax)
    a = oracle.synth_batch(3000, 40, n, 24, 7 + n // 1024 + L + rmax, dtype=np.int32)
    ora = oracle.analyze_batch(a, oracle.make_params(L, 15, 0, rmax), n, sample_bits=24, threads=16)
    out = az.analyze(a, make_params(L, 15, 0, rmax), n, sample_bits=24)
    compare_with_oracle(out, ora, [n] * len(a))
    pm = out["meta"]
    pruned = pm["lpc_order"] == abi.LPC_PRUNED
    assert pruned.mean() > 0.5, pruned.mean()
    assert (pm["lpc_tiers"][pruned] == 8 << 8).all()
    assert (ora["meta"]["kind"][pruned] == abi.KIND_FIXED).all()
    for u in np.nonzero(pruned)[0]:
        assert _emulate_sign_bound(a[u], ora["lpc_records"][u], L, ora["fixed_sums"][u], lean=True), u


def _emulate_sign_bound(x, rec, L, fixed_sums, lmax=32, lean=False):
    """The sign-correlation bound of mf8_candidate_sums / k_resid_sb restated on the oracle's
    record (tests/sign_bound.py) -> True when every order loses to the best fixed sum."""
    return sign_bound.decides(x, rec, L, fixed_sums, lmax, split_end=8 * 2 * 512 if lean else None)


def _c3_tier_units(n, q):
    """24-bit units on every side of the eighth-tier decision (explored with
    _emulate_eighths): full-scale tones at noise 0 / 0.5 / 4 and config-3 synthetic units
    (pruned after two eighths, some after three to six), AR(1) noise (LPC ~1.3x fixed:
    pruned after six or seven), weak AR(1) and white noise (every eighth, then fixed or LPC
    wins), small white noise (LPC within a few units of fixed: near ties) and, at n = 4096,
    units whose best LPC and fixed sums are equal (the tie AssertionError, encoder.py:157)."""
    rng = np.random.default_rng(n + q)
    rows = [_tones24(3, n, 1, 0.0), _tones24(3, n, 2, 0.5), _tones24(3, n, 3, 4.0),
            oracle.synth_batch(0, 6, n, 24, 11, dtype=np.int32)]
    x = []
    for u in range(4):
        w = rng.normal(0, 2e5, n)
        a = w.copy()
        a[1:] += (0.9 if u % 2 else -0.7) * w[:-1]
        x.append(a)
    for u in range(4):
        w = rng.normal(0, 2e5, n)
        a = w.copy()
        a[1:] += (0.4 + 0.05 * u) * w[:-1]
        x.append(a)
    for u in range(6):
        w = rng.normal(0, 2e5, n)
        a = w.copy()
        a[1:] += 0.02 * (u - 3) * w[:-1]
        x.append(a)
    rows.append(np.clip(np.round(np.array(x)), -2 ** 23, 2 ** 23 - 1).astype(np.int32))
    rows.append(rng.integers(-2 ** 22, 2 ** 22, (4, n)).astype(np.int32))
    rows.append(rng.integers(-300, 300, (8, n)).astype(np.int32))
    if n == 4096:  # searched with the oracle: an exact tie of the best fixed and LPC sums
        for seed, u in ({15: ((15002, 440), (15003, 1)), 12: ((12003, 138), (12003, 461))}[q]):
            rows.append(np.random.default_rng(seed).integers(-300, 300, (512, n)).astype(np.int32)[u:u + 1])
    return np.ascontiguousarray(np.concatenate(rows))


@pytest.mark.parametrize("n,q,L", [(16384, 15, 32), (16384, 12, 32), (4096, 15, 32), (4096, 12, 32),
                                   (16384, 15, 16), (16384, 15, 20), (4096, 15, 16)])
def test_c3_int8_pruning_tiers_vs_oracle(az, n, q, L):
    """Config-3 production mode (LPC pruning on) on the int8-MFMA path, 24-bit, L = 32,
    r 0..8: every reference-visible field equals the oracle and the all-candidates run, and
    meta.lpc_tiers equals the decision restated on the oracle's exact candidates: 0/8 when
    the sign-correlation bound settles the unit before any LPC tile (_emulate_sign_bound),
    else the eighths computed before the decision; the tiers-only run (FLACMI_FLAG_TIERS_ONLY)
    takes the eighths for every unit.  Each outcome occurs: pruned by the sign bound, pruned
    after two eighths, pruned later, every eighth then fixed, LPC chosen, a near tie, and
    (n = 4096) the tie AssertionError (encoder.py:133-157).  At n = 16384 production runs
    k_resid_sb (the bound first over the block's first half, then over all of it; decided units
    never reach the int8 path, so units outside it can prune too); L = 16 / 20 pin the bound's
    indexing for the LMAX = 16 and 32 template buckets below L = 32."""
    lmax = 16 if L <= 16 else 32
    lean = _sb_lean(n)
    a = _c3_tier_units(n, q)
    nu = len(a)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 8), n, sample_bits=24, threads=16)
    prod = az.analyze(a, make_params(L, q, 0, 8), n, sample_bits=24)
    tier = az.analyze(a, make_params(L, q, 0, 8, tiers_only=True), n, sample_bits=24)
    full = az.analyze(a, make_params(L, q, 0, 8, all_candidates=True), n, sample_bits=24)
    compare_with_oracle(prod, ora, [n] * nu)
    compare_with_oracle(tier, ora, [n] * nu)
    compare_with_oracle(full, ora, [n] * nu)
    assert (full["meta"]["lpc_tiers"] == 0).all()
    pm, tm, om = prod["meta"], tier["meta"], ora["meta"]
    seen = set()
    for u in range(nu):
        _meta_params_residual_equal(prod, full, u)
        _meta_params_residual_equal(tier, full, u)
        st = int(om["status"][u])
        if st != 0 and int(om["site"][u]) != abi.SITE_CHOICE_TIE:
            continue
        tiers = int(tm["lpc_tiers"][u])
        sbp = _emulate_sign_bound(a[u], ora["lpc_records"][u], L, ora["fixed_sums"][u], lmax, lean)
        if not _int8_path(a[u], ora["lpc_records"][u], L):  # the int64 chains: exact, no pruning
            assert tiers == 0 and int(tm["lpc_order"][u]) != abi.LPC_PRUNED, (u, "int64 path", tiers)
            want_p = lean and sbp  # k_resid_sb decides before any int8 check
            assert int(pm["lpc_tiers"][u]) == ((8 << 8) if want_p else 0), (u, "int64 path", int(pm["lpc_tiers"][u]))
            assert (int(pm["lpc_order"][u]) == abi.LPC_PRUNED) == want_p, (u, "int64 path")
            seen.add("int64")
            continue
        done, pr = _emulate_eighths(a[u], ora["lpc_records"][u], L, ora["fixed_sums"][u])
        assert tiers == done | (8 << 8), (u, "lpc_tiers", tiers & 0xff, tiers >> 8, "want", done)
        assert (int(tm["lpc_order"][u]) == abi.LPC_PRUNED) == pr, (u, "pruned")
        want_prod = (8 << 8) if sbp else done | (8 << 8)
        assert int(pm["lpc_tiers"][u]) == want_prod, (u, "production lpc_tiers", int(pm["lpc_tiers"][u]), want_prod)
        assert (int(pm["lpc_order"][u]) == abi.LPC_PRUNED) == (sbp or pr), (u, "pruned (production)")
        if sbp:
            assert pr or st == 0 and int(om["lpc_sum"][u]) > int(om["fixed_sum"][u]), (u, "sign bound vs exact sums")
            seen.add("sign-bound")
        if st != 0:
            seen.add("tie")
        elif pr:
            seen.add("pruned@2" if done == 2 else "pruned-later")
        elif int(om["kind"][u]) == abi.KIND_LPC:
            seen.add("lpc")
        else:
            seen.add("exact-fixed")
        if st == 0 and not pr and abs(int(om["lpc_sum"][u]) - int(om["fixed_sum"][u])) <= 1e-3 * int(om["fixed_sum"][u]):
            seen.add("near-tie")
    if L == 32:
        want = {"sign-bound", "pruned@2", "pruned-later", "exact-fixed", "lpc", "near-tie"} | ({"tie"} if n == 4096 else set())
    else:
        want = {"sign-bound", "pruned@2", "exact-fixed"}
    assert want <= seen, want - seen


def test_c3_fixed_sums_only_and_25bit_samples(az):
    """k_resid_sb writes no fixed_sums rows, so a caller that asks for fixed_sums
    alone (LPC pruning stays on) must take kVarMf8, which does; and k_resid_sb lists a unit
    only when |x| > 2^23, so 25-bit input (x = +2^23 possible, its 32-bit K_j row sums assume
    every term below 2^23) must not reach it.  Both against the oracle, every field."""
    n, L, q = 16384, 32, 15
    a = oracle.synth_batch(3100, 24, n, 24, 21, dtype=np.int32)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 8), n, sample_bits=24, threads=16)
    out = az.analyze(a, make_params(L, q, 0, 8), n, sample_bits=24, extras=("fixed_sums",))
    compare_with_oracle(out, ora, [n] * len(a))
    assert np.array_equal(out["fixed_sums"], ora["fixed_sums"])
    assert (out["meta"]["lpc_order"] == abi.LPC_PRUNED).all()  # pruning stayed on
    b = a.copy()
    b[:, 5000] = 2 ** 23          # +2^23: 25 bits
    b[::2, 9000] = -(2 ** 23)
    orb = oracle.analyze_batch(b, oracle.make_params(L, 14, 0, 8), n, sample_bits=25, threads=16)
    out = az.analyze(b, make_params(L, 14, 0, 8), n, sample_bits=25)
    compare_with_oracle(out, orb, [n] * len(b))


def test_mf8_persistent_grid_loops_over_units(az, monkeypatch):
    """kVarMf8's persistent grid (k_resid.h) with every workgroup looping over many units:
    FLACMI_MF8_GRID=4 caps it (and the 64-bit list variant's grid) at four workgroups, so the
    next unit's LDS-DMA copy, the raw barriers and the next unit's record status and words
    carried in registers all run (the uncapped grid has a workgroup per unit for test-sized
    batches).  The batch mixes pruned units, units that run every eighth, LPC
    winners, a unit whose LPC record carries an exception (a silent block), units outside the
    int8 path (a top digit of 128: listed for kVarList1), and a short run of each kind between
    them.  Tiers-only runs (kVarMf8), then production runs (k_resid_sb + kVarList1), capped vs
    uncapped vs the oracle, every meta field (lpc_tiers included), parameter and residual."""
    n, L, q = 16384, 32, 15
    base = _c3_tier_units(n, q)
    odd = oracle.synth_batch(900, 6, n, 24, 5, dtype=np.int32)
    odd[0, 4000] = 8355712   # top digit 128: the int64 chains (listed)
    odd[1, :] = 0            # a silent block: the LPC record's exception
    odd[2, 100:] = 0
    odd[3, 77] = 2 ** 23 - 1  # above 8355711 too
    a = np.ascontiguousarray(np.concatenate([base[:20], odd, base[20:], odd[[0, 3]], base[:10]]))
    nu = len(a)
    ora = oracle.analyze_batch(a, oracle.make_params(L, q, 0, 8), n, sample_bits=24, threads=16)
    runs = {}
    for cap in ("", "4", "3"):
        with knob("FLACMI_MF8_GRID", int(cap or 0)):
            for kind in ("tier", "prod"):
                p = make_params(L, q, 0, 8, tiers_only=(kind == "tier"))
                runs[(cap, kind)] = az.analyze(a, p, n, sample_bits=24)
    for (cap, kind), out in runs.items():
        compare_with_oracle(out, ora, [n] * nu)
        ref = runs[("", kind)]
        for f in abi.META_DTYPE.names:
            assert np.array_equal(out["meta"][f], ref["meta"][f]), (cap, kind, f)
        assert np.array_equal(out["residual"], ref["residual"]), (cap, kind)
        assert np.array_equal(out["rice_params"], ref["rice_params"]), (cap, kind)
    tm, om = runs[("4", "tier")]["meta"], ora["meta"]
    assert (om["status"] != 0).any() and (om["kind"] == abi.KIND_LPC).any()
    assert (tm["lpc_order"] == abi.LPC_PRUNED).any() and ((tm["lpc_tiers"] & 0xff) == 8).any()
