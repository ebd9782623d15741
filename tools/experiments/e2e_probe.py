"""Run only bench.py's end_to_end leg (host PCM -> frame bytes through flacmi_encode_pipeline)
and print its JSON.  Usage: python tools/experiments/e2e_probe.py [units] [units_per_sub_batch]"""
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
r = bench.end_to_end_leg(args, dict(bench.CONFIGS["c2"]), az)
print(json.dumps(r))
