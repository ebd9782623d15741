# c3 k_resid split at HEAD (persistent kVarMf8 default): ablation stops + SQ counters; c5 line.
set -o pipefail
TAG=${1:-r04e}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
STOPS="0 1 2 13 14 3 4 5 7" bash tools/gpu_c3_split.sh $TAG/c3 || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0 > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || { tail gpurun_out/$TAG/c5.err; exit 1; }
python tools/show_bench.py gpurun_out/$TAG/c5.json | head -2
