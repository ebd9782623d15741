"""Summarise tools/profile.sh output: per-kernel average duration (kernel trace) and
per-launch HBM traffic from the separate FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per 128-B
request of a wide coalesced read, i.e. half the bytes, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  Both are reported by rocprofv3 in KiB."""
import csv
import glob
import json
import os
import re
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


STAGES = ("k_resid", "k_lpc", "k_stats", "k_synth", "k_pack32", "k_pack", "k_frame_sizes", "k_decode", "k_decorr")


def short(name):
    """Full kernel name without the argument list, e.g. 'k_resid<12, 0, unsigned int, 1>'."""
    name = name.split("(")[0]
    name = name[5:] if name.startswith("void ") else name
    return name.replace("flacmi::", "")[:60]


def stage(name):
    if short(name).startswith(("k_resid_stream", "k_resid_sb")):  # k_resid's one-workgroup-per-unit variants
        return "k_resid"
    for k in STAGES:
        if re.match(k + r"\b", short(name)):
            return k
    return None


def lib_sha16(path=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flac-py_amd",
                                  "libflacmi.so")):
    """sha256[:16] of the library the profile timed (bench.py flags a traffic file whose
    library differs from the one it runs)."""
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def main(d):
    res = {"kernels": {}, "library_sha16": lib_sha16()}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        res["kernels"].setdefault(short(r["Name"]), {})["avg_ms"] = float(r["AverageNs"]) / 1e6
    for counter, scale in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        acc = {}
        for r in rows(os.path.join(d, counter.split("_")[0].lower(), "**", "*counter_collection.csv")):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            acc.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0 * scale)
        for k, v in acc.items():
            res["kernels"].setdefault(k, {})[counter.lower() + "_bytes"] = sum(v) / len(v)
    for k, v in res["kernels"].items():
        if "fetch_size_bytes" in v and "write_size_bytes" in v:
            v["hbm_bytes_per_launch"] = v["fetch_size_bytes"] + v["write_size_bytes"]
    # A stage (e.g. k_resid: the MFMA variant plus its retry launch) is timed as one HIP
    # event interval by the library, so its traffic is the sum over its variants.
    for k, v in res["kernels"].items():
        st = stage(k)
        if st and "hbm_bytes_per_launch" in v:
            res[st] = res.get(st, 0.0) + v["hbm_bytes_per_launch"]
            res.setdefault("stage_avg_ms", {})
            res["stage_avg_ms"][st] = res["stage_avg_ms"].get(st, 0.0) + v.get("avg_ms", 0.0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
