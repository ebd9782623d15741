import math, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
from flac_amd.analysis import Analyzer, make_params
n = 4608
sine = np.array([round(0.6 * 32767 * math.sin(2 * math.pi * 440.0 * i / 44100)) for i in range(n * 2)], dtype=np.int16).reshape(2, n)
print("host x[0..3]", sine[0, :4], "sum|x|", np.abs(sine[0].astype(np.int64)).sum())
az = Analyzer(0)
g = az.analyze(sine, make_params(8, 5, 0, 5, 0), n, sample_bits=16, debug=True)
print("fixed_sums", g["fixed_sums"][0])
