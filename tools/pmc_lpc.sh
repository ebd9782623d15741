# k_lpc issue evidence on config 2 (200k units): SQ issue counters, then the f64 VALU mix.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_lpc}
mkdir -p $OUT
ARGS="--units 200000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && grep -A20 "k_lpc" $OUT/summary.txt | head -24
