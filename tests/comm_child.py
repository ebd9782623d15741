"""One rank of the two-process stats all-reduce test (tests/test_gpu_comm.py,
tests/test_multirank.py).

usage: comm_child.py RANK NRANKS RENDEZVOUS_DIR {rccl|gloo}

rccl: rank r opens a context on device r, rank 0 writes the C-ABI's communicator id
      (flacmi_comm_id) into RENDEZVOUS_DIR, every rank builds the communicator with
      flacmi_comm_init and sums its stats vector with flacmi_allreduce_stats.
gloo: the CPU analogue: the same id hand-off through the directory and the same per-rank
      vectors, summed with torch.distributed over gloo (no device).
Each rank checks the sum against every rank's vector and prints "ok RANK".
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

STATS_WORDS = 128


def rank_vector(r: int):
    import numpy as np
    return (np.arange(STATS_WORDS, dtype=np.int64) * (r + 3) - 1000 * r) ^ (r << 20)


def expected(nranks: int):
    return sum(rank_vector(r) for r in range(nranks))


def wait_for(path: str, seconds: float = 60.0) -> bytes:
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > seconds:
            raise TimeoutError(f"no communicator id at {path} after {seconds} s")
        time.sleep(0.05)
    return open(path, "rb").read()


def publish(path: str, data: bytes) -> None:
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def launch(nranks: int, backend: str, rdv: str, timeout: float = 120.0) -> None:
    """Run nranks child processes (this file) and require every one to report ok."""
    import subprocess
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), str(r), str(nranks), rdv, backend],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(nranks)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"ok {r}" in out, f"rank {r} (rc {p.returncode}):\n{out[-3000:]}"


def main() -> int:
    import numpy as np
    rank, nranks, rdv, backend = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    id_path = os.path.join(rdv, "comm_id")
    import torch
    if backend == "gloo":
        if rank == 0:
            publish(id_path, os.urandom(128))
        cid = wait_for(id_path)
        assert len(cid) == 128
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="file://" + os.path.join(rdv, "pg"),
                                rank=rank, world_size=nranks)
        ids = [None] * nranks
        dist.all_gather_object(ids, cid)
        assert all(i == cid for i in ids), "ranks hold different ids"
        v = torch.from_numpy(rank_vector(rank).copy())
        dist.all_reduce(v)
        dist.destroy_process_group()
        got = v.numpy()
    else:
        from flac_amd import abi
        from flac_amd.analysis import Analyzer, StatsComm
        az = Analyzer(rank)
        StatsComm.available(az.lib)
        if rank == 0:
            publish(id_path, StatsComm.comm_id(az.lib))
        cid = wait_for(id_path)
        assert len(cid) == abi.COMM_ID_BYTES
        comm = StatsComm(az, nranks, rank, cid)
        try:
            dev = torch.device("cuda", rank)
            v = torch.from_numpy(rank_vector(rank).copy()).to(dev)
            comm.allreduce_stats(v.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev)
            got = v.cpu().numpy()
        finally:
            comm.close()
            az.close()
    want = expected(nranks)
    assert np.array_equal(got, want), f"rank {rank}: sum differs in {int((got != want).sum())} words"
    print(f"ok {rank}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
