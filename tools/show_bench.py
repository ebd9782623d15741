"""Print the headline fields of a bench.py JSON line: python tools/show_bench.py <file>"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4e  frac %.3f  kernels %s" % (d["value"], d["roofline"]["frac"], d["kernels"]))
for k in ("end_to_end", "cpu_baseline", "parity", "stream_stats"):
    if d.get(k) is not None:
        print(k, json.dumps(d[k]))
