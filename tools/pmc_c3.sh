# SQ counters of the c3 kernels (k_resid_sb, the int8-MFMA k_resid variants, k_lpc<32>) at 40k units
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_c3}
mkdir -p $OUT
ARGS="--config c3 --units 40000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames --e2e-units 0"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && grep -A18 "k_resid" $OUT/summary.txt | head -60
