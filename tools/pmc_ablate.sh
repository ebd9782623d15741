# k_resid per-phase instruction / wait counts: one SQ pass per FLACMI_DEBUG_STOP value.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmcabl
mkdir -p $OUT
P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for k in 1 2 3 4 0; do
  FLACMI_DEBUG_STOP=$k timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/s$k -o run -- python3 bench.py --units 200000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames > $OUT/s$k.json 2> $OUT/s$k.err || { echo "stop $k failed"; tail -5 $OUT/s$k.err; exit 1; }
  echo "== stop=$k"; python3 tools/pmc_summary.py $OUT/s$k 2>/dev/null | sed -n '/k_resid/,/SQ_WAVE_CYCLES/p' | tail -8
done
