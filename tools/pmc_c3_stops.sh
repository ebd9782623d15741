# SQ counters of the c3 k_resid per ablation stop (1 staging, 13 fixed sums only, 2 candidate
# sums incl. the sign-correlation bound, 0 whole kernel), 40k units, one --pmc pass per stop
# and counter set.  Usage: bash tools/pmc_c3_stops.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_c3_stops}
mkdir -p $OUT
ARGS="--config c3 --units 40000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0"
I="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
W="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
for k in 1 13 2 0; do
  for set in I W; do
    eval CT=\$$set
    FLACMI_DEBUG_STOP=$k timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d $OUT/s${k}_$set -o run -- python3 bench.py $ARGS > $OUT/s${k}_$set.json 2> $OUT/s${k}_$set.err || { echo "stop $k $set failed"; tail -5 $OUT/s${k}_$set.err; exit 1; }
    echo "== stop $k $set"; python3 tools/pmc_summary.py $OUT/s${k}_$set | grep -A9 "k_resid<32, 2, unsigned int, 3>"
  done
done
