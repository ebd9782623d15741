"""Helpers shared by the parity tests: golden fixture loading, input reconstruction and
a field-by-field checker that works on any per-unit result dict (oracle or device).

Result dict keys (as produced by oracle.analyze_unit and flac_amd.analysis.unit_result):
status, site, kind, order, shift, ncoefs, coefs, res_offset, res_len, fixed_order,
lpc_order, part_order, n_parts, coding_method, rice_bits, rice_params, residual (zig-zag
uint64), optionally acf, fixed_sums, lpc_sums, lpc_record.
"""
import hashlib
import json
import math
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EXC_STATUS = {"ZeroDivisionError": 1, "AssertionError": 2, "ValueError": 3, "OverflowError": 4}


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def samples_sha(xs):
    a = np.asarray(xs, dtype="<i8")
    return hashlib.sha256(a.tobytes()).hexdigest()


def samples_for(entry, synth):
    """Rebuild a unit's input from its fixture source; synth(unit, len, bits, seed)."""
    src = entry["source"]
    k = src["kind"]
    if k == "literal":
        xs = list(src["samples"])
    elif k == "synth":
        xs = [int(v) for v in synth(src["unit"], src["len"], src["bits"], src["seed"])]
    elif k == "const":
        xs = [src["value"]] * src["n"]
    elif k == "tone":
        xs = [round(src["amp"] * math.sin(2 * math.pi * src["f"] * i / 44100)) for i in range(src["n"])]
    elif k == "multitone":
        fs, K = src["freqs"], len(src["freqs"])
        xs = [round(src["amp"] * sum(math.sin(2 * math.pi * f * i / 44100 + 0.5 * j)
                                     for j, f in enumerate(fs)) / K) for i in range(src["n"])]
    else:
        raise ValueError(k)
    assert samples_sha(xs) == entry["samples_sha256"], f"input reconstruction differs for {src}"
    return xs


def params_of(entry):
    p = entry["params"]
    return dict(max_lpc_order=p["L"], qlp_precision=p["q"], rice_min=p["rmin"], rice_max=p["rmax"],
                mode=1 if p["fixed_only"] else 0)


def zz_sha(residual):
    return hashlib.sha256(np.asarray(residual, dtype="<u8").tobytes()).hexdigest()


def check(res, entry, intermediates=True):
    """Return a list of human-readable mismatches between `res` and the golden entry."""
    exp = entry["expect"]
    bad = []

    def eq(name, got, want):
        if got != want:
            bad.append(f"{name}: got {got!r} want {want!r}")

    if "exception" in exp:
        eq("status", int(res["status"]), EXC_STATUS[exp["exception"]["type"]])
        msg = exp["exception"]["msg"]
        site = int(res["site"])
        if msg == "math domain error":
            eq("site", site, 12)
        elif msg == "negative shift count":
            eq("site", site, 13)
        elif msg.startswith("min() arg"):
            eq("site", site, 9)
        elif exp.get("exception_stage") == "choice":
            eq("site", site, 10)
    else:
        eq("status", int(res["status"]), 0)
    n = exp["n"]
    if exp.get("exception_stage") in ("choice", "rice", None) or "exception" not in exp:
        eq("fixed_order", int(res["fixed_order"]), exp["fixed_order"])
        if "fixed_sums" in res and res["fixed_sums"] is not None:
            k = 5 if n > 4 else 1
            eq("fixed_sums", [int(v) for v in res["fixed_sums"][:k]], exp["fixed_sums"])
    inter = exp.get("inter", {})
    if intermediates and "acf" in inter and res.get("acf") is not None:
        L = entry["params"]["L"]
        eq("acf", [float(v).hex() for v in res["acf"][: L + 1]], inter["acf"])
    if intermediates and "quant" in inter and res.get("lpc_record") is not None and \
            all(isinstance(q, dict) and "coefs" in q for q in inter["quant"]):
        rec = res["lpc_record"]
        for o, q in enumerate(inter["quant"], start=1):
            neg = (int(rec[1]) >> (o - 1)) & 1
            ncoef = 0 if neg else o
            eq(f"quant[{o}].ncoef", ncoef, len(q["coefs"]))
            eq(f"quant[{o}].shift", int(rec[2 + o - 1]), q["shift"])
            base = 2 + 32 + (o * (o - 1)) // 2
            eq(f"quant[{o}].coefs", [int(v) for v in rec[base: base + ncoef]], q["coefs"])
        if res.get("lpc_sums") is not None and "lpc_sums" in inter:
            eq("lpc_sums", [int(v) for v in res["lpc_sums"][: len(inter["lpc_sums"])]], inter["lpc_sums"])
    if "exception" in exp:
        return bad
    eq("kind", "lpc" if int(res["kind"]) == 1 else "fixed", exp["kind"])
    eq("order", int(res["order"]), exp["order"])
    if exp["kind"] == "lpc":
        eq("shift", int(res["shift"]), exp["lpc"]["shift"])
        eq("coefs", [int(c) for c in res["coefs"][: int(res["ncoefs"])]], exp["lpc"]["coefs"])
    eq("res_len", int(res["res_len"]), exp["res_len"])
    eq("coding_method", int(res["coding_method"]), exp["coding_method"])
    eq("part_order", int(res["part_order"]), exp["partition_order"])
    eq("n_parts", int(res["n_parts"]), exp["n_parts"])
    eq("rice_params", [int(v) for v in res["rice_params"][: int(res["n_parts"])]], exp["params"])
    eq("rice_bits", int(res["rice_bits"]), exp["rice_bits"])
    eq("zz_sha256", zz_sha(res["residual"]), exp["zz_sha256"])
    return bad


# reference raise line (encoder.py) -> flacmi_site, for the ACF-driven rows (acf_sites.json)
ACF_LINE_SITE = {469: 2, 476: 3, 496: 4, 503: 5, 508: 6}


def acf_expected_site(exc):
    """flacmi_site of a reference exception recorded by make_golden.ref_from_acf."""
    if exc["line"] in (520, 530):
        return 7 if exc["type"] == "OverflowError" else 8
    return ACF_LINE_SITE[exc["line"]]


def acf_rows():
    d = load("acf_sites.json")
    for r in d["rows"]:
        r = dict(r)
        r["acf_values"] = [float.fromhex(h) for h in r["acf"]]
        yield r


def check_acf_record(rec, row):
    """Mismatches between an LPC record (k_lpc layout for L = row['L']: word 0 status|site<<16,
    word 1 negative-shift mask, L shifts, triangular coefficients) and a reference row."""
    L, bad = row["L"], []
    exc = row.get("exception")
    st, site = int(rec[0]) & 0xFFFF, int(rec[0]) >> 16
    if exc:
        if (st, site) != (EXC_STATUS[exc["type"]], acf_expected_site(exc)):
            bad.append(f"status/site {(st, site)} want {(EXC_STATUS[exc['type']], acf_expected_site(exc))} {exc}")
    elif (st, site) != (0, 0):
        bad.append(f"status/site {(st, site)} want ok")
    for o, q in enumerate(row.get("quant", []), start=1):
        neg = (int(rec[1]) >> (o - 1)) & 1
        ncoef = 0 if neg else o
        base = 2 + L + (o * (o - 1)) // 2
        got = ([int(v) for v in rec[base: base + ncoef]], int(rec[2 + o - 1]))
        if got != (q["coefs"], q["shift"]):
            bad.append(f"order {o}: got {got} want {(q['coefs'], q['shift'])}")
    return bad
