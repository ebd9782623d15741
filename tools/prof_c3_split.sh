set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b -o prof -- python3 bench.py --config c3 --steps 5 --warmup 2 --cpu-seconds 0 --no-frames --e2e-units 0 > gpurun_out/r05b/b.json 2> gpurun_out/r05b/b.err
