# run one pytest selection against several library builds (FLACMI_LIB)
# Usage: bash tools/gpu_bisect.sh "<pytest -k expr>" "<lib names: default a b ...>"
K=$1; LIBS=$2
mkdir -p gpurun_out/bisect
for v in $LIBS; do
  if [ "$v" = default ]; then L=$PWD/flac-py_amd/libflacmi.so; else L=$PWD/flac-py_amd/libflacmi_$v.so; fi
  FLACMI_LIB=$L timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/bisect/$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/bisect/$v.log)"
done
