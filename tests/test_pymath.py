"""The device's Python-float helpers, run on the host: glibc pow(x, 2.0) emulation and
floor(log2(x)) thresholds, against the live libm (through the oracle)."""
import math
import random

import numpy as np

import oracle
from flac_amd._lib import load


def test_pypow2_matches_libm_random():
    lib = load()
    st = __import__("ctypes").c_int32()
    rnd = random.Random(1)
    diffs = 0
    xs = [rnd.uniform(-1, 1) for _ in range(60000)]
    xs += [math.ldexp(rnd.uniform(0.5, 1), rnd.randint(-1074, 1023)) for _ in range(20000)]
    xs += [rnd.uniform(-1e-3, 1e-3) for _ in range(10000)]
    xs += [0.0, -0.0, 1.0, -1.0, math.inf, -math.inf, 5e-324, 1e154, 1.3407807929942596e154, 1e200, 2.0 ** -600]
    for x in xs:
        got = lib.flacmi_host_pypow2(x, st)
        want, wst = oracle.pypow2(x)
        assert (got == want or (math.isnan(got) and math.isnan(want))) and \
            math.copysign(1, got) == math.copysign(1, want), (x.hex(), got, want)
        assert st.value == wst, x
        if got != abs(x) * abs(x):
            diffs += 1
    assert diffs > 0  # the corpus does exercise pow(x,2) != x*x


def test_pypow2_bulk_native():
    """20M-input sweep compiled from the same header (tools/check_pymath.cpp)."""
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    exe = os.path.join("/tmp", "flacmi_check_pymath")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-I", os.path.join(repo, "flac-py_amd", "csrc"),
                    os.path.join(repo, "tools", "check_pymath.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe, "4000000"], check=True, capture_output=True, text=True).stdout
    assert "bad=0" in out, out


def test_floor_log2_thresholds():
    lib = load()
    rnd = random.Random(2)
    xs = []
    for e in list(range(-1074, 1024, 7)) + list(range(-40, 40)):
        p = math.ldexp(1.0, e)
        x = p
        for _ in range(80):  # walk below 2^e, where log2 rounds up to e
            xs.append(x)
            x = math.nextafter(x, 0.0)
        x = p
        for _ in range(20):
            xs.append(x)
            x = math.nextafter(x, math.inf)
    xs += [rnd.uniform(1e-300, 1e300) for _ in range(20000)] + [5e-324, 1e-310, 1.7976931348623157e308]
    for x in xs:
        if x <= 0 or not math.isfinite(x):
            continue
        want, st = oracle.floor_log2(x)
        assert st == 0
        assert lib.flacmi_host_floor_log2(x) == want, x.hex()
