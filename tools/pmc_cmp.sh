# SQ instruction counts of the whole analysis for two configs / knobs (one --pmc pass each).
# Usage: bash tools/pmc_cmp.sh <tag> ; env FLACMI_DEBUG_STOP etc. pass through
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmccmp}
mkdir -p $OUT
I="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
W="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for c in c2 c5; do
  for set in I W; do
    eval CTRS=\$$set
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$c$set -o run -- python3 bench.py --config $c --units 200000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0 > $OUT/$c$set.json 2> $OUT/$c$set.err || { echo "$c $set failed"; tail -5 $OUT/$c$set.err; exit 1; }
    echo "== $c $set"; python3 tools/pmc_summary.py $OUT/$c$set | grep -A9 "k_resid_stream"
  done
done
