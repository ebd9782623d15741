"""Debug probe (experiments): one golden unit through the production and all-candidates calls."""
import os, sys
import numpy as np
sys.path[:0] = ['.', 'oracle', 'tests']
import golden_util as G, oracle
from flac_amd.analysis import Analyzer, make_params
from flac_amd import abi
f, i = sys.argv[1], int(sys.argv[2])
e = G.load(f)["units"][i]
xs = G.samples_for(e, oracle.synth_unit)
n = len(xs)
a = np.zeros((1, ((n * 2 + 15) // 16) * 8), dtype=np.int16); a[0, :n] = xs
az = Analyzer(0)
p = make_params(**G.params_of(e))
for dbg in (False, True):
    out = az.analyze(a, p, n, sample_bits=16, debug=dbg)
    m = out["meta"][0]
    print("debug" if dbg else "prod ", {k: int(m[k]) for k in ("status", "site", "kind", "order", "fixed_order", "lpc_order", "fixed_sum", "lpc_sum", "lpc_tiers")})
    if dbg:
        print(" fixed", list(out["fixed_sums"][0]) if "fixed_sums" in out else None)
