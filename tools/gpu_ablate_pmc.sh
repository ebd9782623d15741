set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --units 200000 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bdec.json 2> gpurun_out/bdec.err || { tail -20 gpurun_out/bdec.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bdec.json')); print(json.dumps(d['frame_writer']))"
bash tools/ablate.sh --no-frames || exit 1
bash tools/pmc.sh pmc_r01d --no-frames
