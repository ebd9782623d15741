"""flacmi_analyze_device returns without a host synchronisation (include/flacmi.h), also when
the call splits its units into chunks whose k_lpc runs on a second stream (the round-aligned
overlap, flacmi_host.cpp analyze_device_impl).  Round 5 created that stream per call and
destroyed it before returning; destroying a stream with queued work waits for the work, so the
call blocked until k_lpc had finished.  The side stream is now the context's own
pipeline H2D stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_analyze_device_returns_while_the_stream_is_busy():
    import torch

    from flac_amd import abi
    from flac_amd.analysis import Analyzer, knob, make_params, params_stride_for, unit_stride

    n, units = 4608, 131072
    stride = unit_stride(n, 2)
    dev = torch.device("cuda", 0)
    az = Analyzer(0)
    try:
        x = torch.empty(units * stride, dtype=torch.int16, device=dev)
        meta = torch.empty(units * abi.META_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        ps = params_stride_for(5)
        prm = torch.empty(units * ps, dtype=torch.int32, device=dev)
        res = torch.empty(units * n, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        az.synth_device(x.data_ptr(), 2, 16, stride, 0, units, n, 2024, stream=s.cuda_stream)
        s.synchronize()
        p = make_params(12, 5, 0, 5)
        runs = []
        for ov in (-(units // 2), 0):
            with knob("FLACMI_OVERLAP", ov):
                for _ in range(2):  # the second call reuses the context's side stream
                    az.analyze_device(x.data_ptr(), 2, 16, stride, units, n, p, meta.data_ptr(), prm.data_ptr(),
                                      ps, res.data_ptr(), n, stream=s.cuda_stream)
                    busy = not s.query()
                    s.synchronize()
                    assert busy, f"analyze_device (overlap {ov}) returned after its work had finished"
            runs.append((meta.cpu(), prm.cpu(), res.cpu()))
        for a, b in zip(*runs):
            assert torch.equal(a, b)
        m = runs[0][0].numpy().view(abi.META_DTYPE)
        assert np.all(m["status"] == 0)
    finally:
        az.close()
