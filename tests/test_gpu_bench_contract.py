"""bench.py's one-line JSON contract on the GPU (the driver parses this line every round):
a short config-2 run in a child process must print exactly one JSON line carrying the
BASELINE metric, the whole-job value, the roofline object (HIP-event kernel time against
SURVEY §8d bytes) and the cpu_baseline object, with the sampled parity clean."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line_contract():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--units", "20000", "--steps", "2", "--warmup", "1",
           "--cpu-seconds", "0.5", "--parity-units", "16", "--no-frames", "--e2e-units", "0"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert "workload" in d["config"]
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s"
    assert 0 < roof["frac"] < 1 and abs(roof["achieved"] / roof["peak"] - roof["frac"]) < 1e-6
    cpu = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    assert cpu["kind"] in ("port", "reference") and cpu["value"] > 0 and cpu["cores"] >= 1
    assert d["parity"]["mismatches"] == 0 and d["parity"]["units_checked"] > 0
