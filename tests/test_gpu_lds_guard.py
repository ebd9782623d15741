"""Guard against the LDS-aliasing bug class (a kernel reading LDS words it never wrote: round
2 hit one in the fast S16 kernel, `gpurun_out/mf8e/pytest_gpu.log`, fixed in 807d6dc) and a
determinism check (run twice, compare).

Each child process (tests/lds_guard_child.py) analyses the same unit sets in four batch
arrangements (natural order, reversed, shuffled inside a larger batch, one unit per call)
under one kernel variant: the default dispatch (k_resid_stream, its retry list, k_resid's
fast / generic / int8-MFMA paths by shape), FLACMI_NO_STREAM, FLACMI_NO_MFMA and
FLACMI_NO_PRUNE, each with FLACMI_POISON_LDS filling every CU's LDS with a different
pattern before every analysis kernel.  Every unit must give the same meta, Rice parameters
and residual in every arrangement, variant and pattern as in the plain default run."""
import os
import subprocess
import sys

import numpy as np
import pytest

from flac_amd import abi

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VARIANTS = [
    ("plain", {}),
    ("plain-again", {}),
    ("poison-a5", {"FLACMI_POISON_LDS": "a5a5a5a5"}),
    ("poison-ff", {"FLACMI_POISON_LDS": "ffffffff"}),
    ("no-stream", {"FLACMI_NO_STREAM": "1", "FLACMI_POISON_LDS": "0"}),
    ("no-mfma", {"FLACMI_NO_MFMA": "1", "FLACMI_POISON_LDS": "3c3c3c3c"}),
    ("no-prune", {"FLACMI_NO_PRUNE": "1", "FLACMI_POISON_LDS": "12345678"}),
]


def _run(tmp_path, name, env):
    out = os.path.join(str(tmp_path), f"{name}.npz")
    e = {k: v for k, v in os.environ.items() if not k.startswith("FLACMI_")}
    e.update(env)
    r = subprocess.run([sys.executable, os.path.join(HERE, "lds_guard_child.py"), out], env=e,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-1000:] + r.stderr[-3000:]
    return dict(np.load(out))


def _equal(a, b, key, k):
    ma, mb = a[key + "|meta"][:k], b[key + "|meta"][:k]
    for u in range(k):
        pruned = int(ma[u]["lpc_order"]) == abi.LPC_PRUNED or int(mb[u]["lpc_order"]) == abi.LPC_PRUNED
        for f in abi.META_DTYPE.names:
            if f == "lpc_tiers" or (pruned and f in ("lpc_order", "lpc_sum")):
                continue
            assert np.array_equal(ma[u][f], mb[u][f]), (key, u, f, ma[u][f], mb[u][f])
        if int(ma[u]["status"]) != 0:
            continue
        off, ln, npart = int(ma[u]["res_offset"]), int(ma[u]["res_len"]), int(ma[u]["n_parts"])
        assert np.array_equal(a[key + "|residual"][u][off:off + ln], b[key + "|residual"][u][off:off + ln]), (key, u)
        assert np.array_equal(a[key + "|params"][u][:npart], b[key + "|params"][u][:npart]), (key, u)


def test_lds_poison_arrangements_and_variants(tmp_path):
    runs = {name: _run(tmp_path, name, env) for name, env in VARIANTS}
    ref = runs["plain"]
    keys = sorted({k.rsplit("|", 1)[0] for k in ref})
    naturals = [k for k in keys if k.endswith("|natural")]
    assert len(naturals) >= 9
    n_checked = 0
    for name, got in runs.items():
        for key in keys:
            base = key.rsplit("|", 1)[0] + "|natural"
            k = len(got[key + "|meta"])
            # every arrangement against the plain natural-order run of the same unit set
            a = {s: got[key + s] for s in ("|meta", "|residual", "|params")}
            b = {s: ref[base + s][:k] for s in ("|meta", "|residual", "|params")}
            _equal({key + s: v for s, v in a.items()}, {key + s: v for s, v in b.items()}, key, k)
            n_checked += k
    assert n_checked > 5000
    # the unit sets exercise every outcome class: pruned, exact-pass fixed, LPC-chosen, errors
    m = ref["s16|12,5,0,5|natural|meta"]
    assert (m["lpc_order"] == abi.LPC_PRUNED).any() and (m["kind"] == abi.KIND_LPC).any()
    assert (m["status"] != 0).any()
