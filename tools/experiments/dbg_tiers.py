"""Debug probe (experiments): lpc_tiers histogram of the pruning-path test batch."""
import sys
import numpy as np
sys.path[:0] = ['.', 'oracle', 'tests']
import test_gpu_parity as T
from flac_amd.analysis import Analyzer, make_params
from flac_amd import abi
az = Analyzer(0)
for q in (5, 9, 15):
    a = T._prune_signals(4608, 50 + q)
    prod = az.analyze(a, make_params(12, q, 0, 5), 4608, sample_bits=16)
    t = prod["meta"]["lpc_tiers"]
    u, c = np.unique(t, return_counts=True)
    print(q, len(a), dict(zip([hex(int(x)) for x in u], c.tolist())), "pruned", int((prod["meta"]["lpc_order"] == abi.LPC_PRUNED).sum()),
          "status", np.unique(prod["meta"]["status"]).tolist())
