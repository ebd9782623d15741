# Quick iteration: GPU suite, c2 bench line, one SQ instruction-count pass of k_resid_stream
# (VALU / SALU / LDS / MFMA per unit).  Usage: bash tools/gpu_quick.sh <tag> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e-units 0 --no-frames "$@" > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python tools/show_bench.py $OUT/bench_c2.json | head -3
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/pmc -o run -- python3 bench.py --units 200000 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 "$@" > $OUT/pmc.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
python3 - $OUT/pmc <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_resid_stream" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("per unit:", " ".join(f"{k[9:]}={sum(v)/len(v)/2e5:.0f}" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
PY
