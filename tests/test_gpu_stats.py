"""Device stream statistics (flacmi_stream_stats, the vector bench.py all-reduces) against
the numpy restatement in tests/stats_mirror.py, on oracle-checked meta including error
units and a tail class."""
import numpy as np
import pytest

import oracle
from stats_mirror import stream_stats

pytestmark = pytest.mark.gpu


def test_device_stream_stats_match_mirror():
    import torch
    from flac_amd import abi
    from flac_amd.analysis import Analyzer, make_params

    az = Analyzer(0)
    n, units, tail = 4608, 96, 1000
    a = oracle.synth_batch(0, units, n, 16, 77, dtype=np.int16)
    a[5, :] = 0      # zero block -> the reference's ValueError path
    a[9, 10:] = 3    # near-constant block
    out = az.analyze(a, make_params(12, 5, 0, 5, abi.MODE_REFERENCE), n, tail, 2, sample_bits=16)
    meta = out["meta"]
    want = stream_stats(meta, n, tail, 2)
    dev = torch.device("cuda", 0)
    m_dev = torch.from_numpy(meta.view(np.uint8).reshape(units, -1).copy()).to(dev)
    st = torch.zeros(abi.STATS_WORDS, dtype=torch.int64, device=dev)
    az.stream_stats(m_dev.data_ptr(), units, n, st.data_ptr(), 0, tail, 2)
    torch.cuda.synchronize()
    assert st.cpu().numpy().tolist() == want.tolist()
    assert want[0] == units and want[64:80].sum() == units
