"""Print VGPRs / scratch / occupancy per kernel from the hipcc -Rpass-analysis reports
(flac-py_amd/csrc/build/*.res).  Usage: python tools/resusage.py [substring]"""
import glob, re, sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
for f in sorted(glob.glob("flac-py_amd/csrc/build/*.res")):
    cur = None
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            continue
        if cur is None:
            continue
        for key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill"):
            m = re.search(re.escape(key) + r": (\d+)", line)
            if m:
                cur[key] = int(m.group(1))
        if "LDS Size" in line:
            if pat in cur["name"]:
                print(f"{cur['name'][:70]:70s} vgpr {cur.get('VGPRs')} agpr {cur.get('AGPRs')} scratch {cur.get('ScratchSize [bytes/lane]')} "
                      f"occ {cur.get('Occupancy [waves/SIMD]')} spill s/v {cur.get('SGPRs Spill')}/{cur.get('VGPRs Spill')}")
            cur = None
