# VALU / SALU / MFMA / LDS instruction counts of k_resid_stream per ablation stop (1 = staging,
# 2 = candidate sums, 3 = choice, 4 = chosen residual, 0 = whole), for c2 and c5, 200k units.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmcphase}; mkdir -p $OUT
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
for c in ${CFGS:-c2 c5}; do
  for k in 1 2 3 4 0; do
    FLACMI_DEBUG_STOP=$k timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$c.s$k -o run -- python3 bench.py --config $c --units 200000 --steps 1 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 > $OUT/$c.s$k.json 2> $OUT/$c.s$k.err || { echo "$c stop $k failed"; tail -5 $OUT/$c.s$k.err; exit 1; }
    python3 - $OUT/$c.s$k $c $k <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_resid_stream" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
u = 2e5
print(sys.argv[2], "stop", sys.argv[3], " ".join(f"{k[9:]}={sum(v)/len(v)/u:.0f}" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
PY
  done
done
