"""The C-ABI's cross-GPU stats reduce (flacmi_comm_* / flacmi_allreduce_stats, RCCL), the
collective a caller without torch.distributed uses.  One GPU on the test box, so
the communicator has one rank: the all-reduce must leave the stats vector unchanged, and the
argument checks must refuse bad ranks.  The N-rank path is the same RCCL call bench.py makes
through torch.distributed (tests/test_multirank.py covers the rank logic on gloo)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_comm_world_one_allreduce_is_identity():
    import torch

    from flac_amd import abi
    from flac_amd._lib import FlacmiError
    from flac_amd.analysis import Analyzer, StatsComm

    az = Analyzer(0)
    StatsComm.available(az.lib)  # RCCL loads (the check every rank runs before the id)
    cid = StatsComm.comm_id(az.lib)
    assert len(cid) == abi.COMM_ID_BYTES
    with pytest.raises(FlacmiError):
        StatsComm(az, 1, 1, cid)  # rank outside the world
    comm = StatsComm(az, 1, 0, cid)
    try:
        v = torch.arange(abi.STATS_WORDS, dtype=torch.int64,
                         device="cuda:0") * 7 - 300
        want = v.clone()
        comm.allreduce_stats(v.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(v, want)
    finally:
        comm.close()


def test_comm_two_devices_allreduce_sums_ranks(tmp_path):
    """Two processes on devices 0 and 1 (skipped with fewer than two GPUs visible): rank 0's
    flacmi_comm_id reaches rank 1 through a rendezvous directory, both build the communicator
    with flacmi_comm_init and sum distinct stats vectors with flacmi_allreduce_stats; each rank
    checks the sum of every rank's vector (tests/comm_child.py).  The CPU analogue with the same
    hand-off and vectors over gloo is tests/test_multirank.py::test_comm_child_gloo_two_ranks."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("fewer than two GPUs visible")
    import comm_child
    comm_child.launch(2, "rccl", str(tmp_path), timeout=180)
