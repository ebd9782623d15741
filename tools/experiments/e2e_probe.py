"""Run only bench.py's end_to_end leg (host PCM -> frame bytes through flacmi_encode_pipeline)
and print its JSON.  Usage: python tools/experiments/e2e_probe.py [units] [units_per_sub_batch] [alloc]
alloc: copy the rows into flacmi_host_alloc memory (instead of host_register'ing them)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from flac_amd.analysis import Analyzer  # noqa: E402

units = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
per = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
args = argparse.Namespace(e2e_units=units, e2e_batch=per, seed=2024)
az = Analyzer(0)
if len(sys.argv) > 3 and sys.argv[3] == "alloc":
    real_reg, real_unreg = az.host_register, az.host_unregister
    az.host_register = lambda a: None
    az.host_unregister = lambda a: None
    orig = az.encode_pipeline

    def enc(host, params, n, out=None, **kw):
        if out is None:
            return orig(host, params, n, **kw)
        h = az.host_array(host.shape, host.dtype)
        h[...] = host
        o = az.host_array(out.shape, out.dtype)
        r = orig(h, params, n, out=o, **kw)
        return r
    az.encode_pipeline = enc
r = bench.end_to_end_leg(args, dict(bench.CONFIGS["c2"]), az)
print(json.dumps(r))
