"""N > 1 path on CPU: world_size-2 gloo ranks, each analysing its own contiguous shard of
synthetic units (bench.shard_first_unit) through the oracle, then bench.reduce_stats /
bench.reduce_elapsed over torch.distributed.  The all-reduced stream statistics must equal
the single-process statistics of the whole unit range: the shards are disjoint, cover the
range, and every statistic is a sum (no data-path collective)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
N, BITS, L, Q, RMIN, RMAX, SEED, U = 4608, 16, 12, 5, 0, 5, 2024, 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_stats(rank):
    for p in (REPO, os.path.join(REPO, "oracle"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import bench
    import oracle
    from stats_mirror import stream_stats
    first = bench.shard_first_unit(rank, U)
    a = oracle.synth_batch(first, U, N, BITS, SEED, dtype=np.int16)
    r = oracle.analyze_batch(a, oracle.make_params(L, Q, RMIN, RMAX, 0), N, threads=2)
    return stream_stats(r["meta"], N)


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        st = torch.from_numpy(_shard_stats(rank))
        bench.reduce_stats(st, dist)
        el = bench.reduce_elapsed(0.5 + rank, dist)
        out.put((rank, st.numpy().tolist(), el))
    finally:
        dist.destroy_process_group()


def test_two_rank_stats_equal_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process over the whole range [0, world*U)
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), HERE]
    import oracle
    from stats_mirror import stream_stats
    a = oracle.synth_batch(0, world * U, N, BITS, SEED, dtype=np.int16)
    r = oracle.analyze_batch(a, oracle.make_params(L, Q, RMIN, RMAX, 0), N, threads=4)
    want = stream_stats(r["meta"], N).tolist()
    for rank, st, el in res:
        assert st == want, f"rank {rank}: all-reduced stats differ from the single-process stats"
        assert el == 1.5  # max over ranks of 0.5 and 1.5
    assert want[0] == world * U and want[1] == world * U * N


def test_shards_disjoint_and_covering():
    sys.path.insert(0, REPO)
    import bench
    for world in (1, 2, 4, 8):
        spans = [(bench.shard_first_unit(r, 1000), bench.shard_first_unit(r, 1000) + 1000) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == world * 1000
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def _bench(args, env_extra=None, timeout=300):
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def _json_line(out):
    import json
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("gpus,config", [(2, "c2"), (4, "c4")])
def test_bench_self_launches_n_ranks(gpus, config):
    """`bench.py --gpus N` (no torch.distributed environment) starts N ranks itself; every
    rank sees world size N; the all-reduced shard vector covers the job exactly once."""
    extra = ["--total-units", "1000003", "--units", "100000"] if config == "c4" else []
    r = _bench(["--gpus", str(gpus), "--config", config, "--launch-check"] + extra)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["world_size"] == gpus and d["gpus_arg"] == gpus
    assert d["rank_mask"] == (1 << gpus) - 1
    assert d["units_total"] == d["expected_units"]
    assert d["elapsed_max"] == pytest.approx(0.001 * gpus)
    assert d["comm_id_broadcast_ok"] is True  # rank 0's comm id reached every rank


def test_bench_rejects_world_size_mismatch():
    """A rank whose process group does not hold --gpus ranks stops with an error."""
    r = _bench(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0
    assert "process group has 1 rank" in r.stderr


def test_shard_plan_round_robin_chunks():
    sys.path.insert(0, REPO)
    import bench
    cfg = bench.CONFIGS["c4"]
    for world in (1, 2, 4, 8):
        seen = []
        for r in range(world):
            first, chunks, total = bench.shard_plan(cfg, r, world, 1000, 10_500)
            assert total == 10_500 and all(c % world == r for c in chunks)
            seen += chunks
        assert sorted(seen) == list(range(11))


def test_reduce_stats_routes_through_the_c_abi_comm():
    """With a C-ABI communicator bench.reduce_stats calls its allreduce_stats on the stats
    buffer and the launch stream (flacmi_allreduce_stats), not torch.distributed."""
    import torch
    sys.path.insert(0, REPO)
    import bench

    class Comm:
        calls = []

        def allreduce_stats(self, ptr, stream):
            self.calls.append((ptr, stream))

    st = torch.zeros(128, dtype=torch.int64)
    c = Comm()
    assert bench.reduce_stats(st, None, c, 1234) is st
    assert c.calls == [(st.data_ptr(), 1234)]


def _comm_worker(rank, world, port, out):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench

    class _NoRccl:  # an analyzer whose library cannot load RCCL on rank 1
        class lib:  # noqa: N801
            @staticmethod
            def flacmi_comm_available():
                return -5 if rank == 1 else 0

            @staticmethod
            def flacmi_comm_id(buf):
                assert rank == 0, "only rank 0 makes the id"
                return 0

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        comm, why = bench.open_stats_comm(_NoRccl(), dist, rank, world, None)
        out.put((rank, comm is None, why))
    finally:
        dist.destroy_process_group()


def test_open_stats_comm_falls_back_together():
    """When one rank cannot load RCCL (flacmi_comm_available fails there), every rank learns it
    before the collective flacmi_comm_init and returns no communicator, so the N-rank bench
    reduces through torch.distributed instead of hanging or failing (the reason goes into
    the bench line's config.stats_collective)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(none for _, none, _ in res)
    assert "rank 1" in res[1][2] and "flacmi_comm_available" in res[1][2]
    assert res[0][2]  # rank 0 reports why too


def test_comm_child_gloo_two_ranks(tmp_path):
    """CPU analogue of tests/test_gpu_comm.py::test_comm_two_devices_allreduce_sums_ranks: the
    same rank script, id hand-off through the rendezvous directory and per-rank vectors,
    summed over gloo."""
    import comm_child
    comm_child.launch(2, "gloo", str(tmp_path), timeout=180)
