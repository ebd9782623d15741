# c3 library A/B on one box: GPU suite with the working-tree library, then alternating c3
# bench lines of libflacmi_<base>.so and the working tree.  bash tools/gpu_c3ab.sh <tag> <base>
set -o pipefail
TAG=${1:-c3ab}; BASE=${2:-base}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh $TAG "$BASE default $BASE default" c3
