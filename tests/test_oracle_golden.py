"""The CPU oracle (oracle/flac_oracle.c) against golden vectors produced by the reference.

This pins the oracle: every fixture in tests/golden/ was produced by importing
turlando/flac-py itself (tests/golden/make_golden.py).  The device path is then
checked against this oracle and against the same fixtures (tests/test_gpu_parity.py).
"""
import pytest

import golden_util as G
import oracle

SETS = ["c1.json", "c2.json", "c3.json", "c5.json", "edge.json"]


def _cases():
    for s in SETS:
        d = G.load(s)
        for i, e in enumerate(d["units"]):
            tag = e["source"].get("tag") or f"u{e['source'].get('unit', i)}"
            yield pytest.param(e, id=f"{s[:-5]}-{i}-{tag}"[:60])


@pytest.mark.parametrize("entry", list(_cases()))
def test_oracle_matches_reference(entry):
    xs = G.samples_for(entry, oracle.synth_unit)
    res = oracle.analyze_unit(xs, oracle.make_params(**G.params_of(entry)))
    bad = G.check(res, entry)
    assert not bad, "\n".join(bad)


def test_synth_matches_python_restatement():
    # the golden script's Python generator produced samples_sha256 for these
    d = G.load("c2.json")
    for e in d["units"][:2]:
        G.samples_for(e, oracle.synth_unit)


def test_levinson_snapshots_equal_per_order_runs():
    """A single max-order Levinson run snapshotted after iteration k equals the
    reference's from-scratch call on r[:k+2] (what the device kernel relies on)."""
    d = G.load("c3.json")
    for e in d["units"]:
        acf = [float.fromhex(h) for h in e["expect"]["inter"]["acf"]]
        st, site, full = oracle.levinson(acf, 32)
        assert st == 0
        for o, want in enumerate(e["expect"]["inter"]["levinson"], start=1):
            st, site, c = oracle.levinson(acf, o)
            assert [v.hex() for v in c] == want


def test_oracle_levinson_quantize_on_acf_rows():
    """The overflow sites integer PCM never reaches: the oracle's Levinson and
    quantiser, run as encode_subframe_lpc runs them (every order's Levinson, then every
    order's quantisation, encoder.py:376-384), against the reference on ACF rows
    (tests/golden/acf_sites.json)."""
    sites = set()
    for row in G.acf_rows():
        L, q, ac = row["L"], row["q"], row["acf_values"]
        exc = row.get("exception")
        got = None
        coefs = []
        for o in range(1, L + 1):
            st, site, c = oracle.levinson(ac[: o + 1], o)
            if st:
                got = (st, site)
                break
            coefs.append(c)
        quant = []
        if got is None:
            for c in coefs:
                st, site, qc, sh = oracle.quantize(c, q)
                if st:
                    got = (st, site)
                    break
                quant.append({"coefs": [int(v) for v in qc], "shift": sh})
            if exc is None:
                assert [[v.hex() for v in c] for c in coefs] == row["levinson"]
        if exc:
            assert got == (G.EXC_STATUS[exc["type"]], G.acf_expected_site(exc)), (row, got)
            sites.add(got[1])
        else:
            assert got is None, (row, got)
        assert quant == row.get("quant", []), row
    assert {3, 5} <= sites, sites
