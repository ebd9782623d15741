# SQ counters per k_resid_stream phase: one rocprofv3 --pmc pass per ablation stop
# (FLACMI_DEBUG_STOP=k ends each unit after phase k; 0 = whole kernel).
# Usage: [STOPS="1 2 3 4 0"] [KPAT=k_resid_stream] bash tools/pmc_stops.sh <tag> <counter set: insts|lds> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmcstops}; SET=${2:-insts}; shift 2
case $SET in
  insts) CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_MFMA";;
  lds) CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY";;
  *) echo "unknown set $SET"; exit 2;;
esac
mkdir -p $OUT
ARGS="--units ${UNITS:-200000} --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-frames $*"
for k in ${STOPS:-1 2 3 4 0}; do
  FLACMI_DEBUG_STOP=$k timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/s$k -o run -- python3 bench.py $ARGS > $OUT/s$k.json 2> $OUT/s$k.err || { echo "stop $k failed"; tail -5 $OUT/s$k.err; exit 1; }
  echo "== stop $k"; python3 tools/pmc_summary.py $OUT/s$k | grep -A9 ${KPAT:-k_resid_stream}
done
