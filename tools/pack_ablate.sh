# k_pack32 ablation: frame-writer leg timing with parts of the kernel switched off
# (FLACMI_PACK_ABLATE: 1 no CRC shift, 2 no residual codes, 3 neither; outputs invalid)
set -o pipefail
mkdir -p gpurun_out
for k in 0 1 2 3; do
  FLACMI_PACK_ABLATE=$k timeout -k 10 300 python bench.py --units 200000 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > gpurun_out/pab_$k.json 2>gpurun_out/pab_$k.err || { tail gpurun_out/pab_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pab_$k.json')); print('ablate=$k', 'frame_ms %.3f' % d['frame_writer']['ms_per_call'])"
done
