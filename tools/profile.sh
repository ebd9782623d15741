# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command (per-kernel average durations);
#   2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass);
#   3. tools/traffic.py -> per-launch HBM bytes (gfx950 FETCH_SIZE x 2 correction).
# Usage: bash tools/profile.sh <tag> [bench args...]
# FLACMI_OVERLAP=0: one k_lpc and one k_resid launch per call, the launches bench.py's
# roofline times (its timed steps overlap two chunks; bench.py then times one-chunk calls).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --cpu-seconds 0 --no-parity $*"
FLACMI_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
FLACMI_OVERLAP=0 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity $* > /dev/null 2> $OUT/fetch.err || { tail $OUT/fetch.err; exit 1; }
FLACMI_OVERLAP=0 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity $* > /dev/null 2> $OUT/write.err || { tail $OUT/write.err; exit 1; }
python3 tools/traffic.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
