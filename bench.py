"""Encode-analysis throughput on MI355X (BASELINE.json metric, config 2 workload).

One step = the whole analysis hot path (fixed predictors, Tukey-windowed
autocorrelation, Levinson-Durbin, LPC quantisation, all candidate residuals, subframe
choice, Rice partition search; residuals written back zig-zagged for the host packer)
over one resident batch of --units synthetic 4608-sample int16 blocks per GPU, plus the
per-step stream statistics that are all-reduced over RCCL when N > 1.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--units U] [--config c2|c3|c4|c5]

For N > 1 one process runs per GPU.  Either the driver starts them with
torch.distributed.run (WORLD_SIZE set), or `bench.py --gpus N` starts them itself: it
spawns torch.distributed.run with N ranks as a child process before any GPU call and
exits with its status.  Every rank checks that the process group holds exactly N ranks;
each analyses its own shard (weak scaling: --units per GPU; c4: round-robin chunks of one
fixed job, strong scaling).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    # BASELINE.json configs[1] — the metric's workload
    "c2": dict(workload="1e6 synthetic mono 4608-sample int16 blocks, -l 12 -q 5 -r 0,5",
               n=4608, bits=16, L=12, q=5, rmin=0, rmax=5, mode=0, units=1_000_000, channels=1),
    # configs[2]: stereo 24-bit/96 kHz, -b 16384 -l 32 -q 15 -r 0,8 (each channel one unit;
    # 1e5 stereo blocks = 2e5 units = 3.3e9 samples)
    "c3": dict(workload="stereo 24-bit 16384-sample blocks, -l 32 -q 15 -r 0,8",
               n=16384, bits=24, L=32, q=15, rmin=0, rmax=8, mode=0, units=200_000, channels=2),
    # configs[3]: 1e8 blocks of config 2's shape, generated on the device chunk by chunk
    # (9.2e11 bytes of PCM cannot be materialised); chunks go round-robin to the ranks and
    # one step is the whole 1e8 blocks: strong scaling, generation inside the timed region
    "c4": dict(workload="1e8 synthetic mono 4608-sample int16 blocks generated on device in 1e6-block chunks "
                        "(double-buffered: the next chunk generated while this one is analysed), -l 12 -q 5 -r 0,5", n=4608, bits=16, L=12, q=5, rmin=0, rmax=5, mode=0,
               units=1_000_000, channels=1, total_units=100_000_000),
    # configs[4]: fixed-only (-l 0 mode of this build) + Rice search
    "c5": dict(workload="fixed-only 4608-sample int16 blocks, -r 0,5",
               n=4608, bits=16, L=0, q=5, rmin=0, rmax=5, mode=1, units=1_000_000, channels=1),
    # not a BASELINE config: FLAC's common 4096-sample block at -l 8 -r 0,4, which runs the
    # runtime-shape kernel builds (the BASELINE shapes have constant-shape builds)
    "b4096": dict(workload="1e6 synthetic mono 4096-sample int16 blocks, -l 8 -q 5 -r 0,4 (non-BASELINE shape)",
                  n=4096, bits=16, L=8, q=5, rmin=0, rmax=4, mode=0, units=1_000_000, channels=1),
}
# --open K: K/8 of the units are MA(1) near-white noise (flacmi_synth_mix_device), whose LPC
# candidates tie the fixed order-0 sum within a fraction of a percent, so neither the sign
# bound nor the partial-sum tiers decide them and every candidate's exact sum is computed
# (the reference's full candidate work, encoder.py:387-404, 537-548)
OPEN_NOTE = ("open mix: {k}/8 of the units MA(1) near-white noise (LPC near-ties that no bound decides: every "
             "candidate's exact sum), the rest the SURVEY §8d tones")
METRIC = "PCM samples/sec encode-analysis, 4608-blk/16-bit mono, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--units", type=int, default=0, help="units per GPU (default: the config's); c4: chunk size")
    ap.add_argument("--total-units", type=int, default=0, help="c4: blocks in the whole job (default 1e8)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--open", type=int, default=0, choices=range(9), metavar="K",
                    help="K/8 of the units MA(1) near-white noise: the undecided-LPC workload (0 = the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--parity-units", type=int, default=64)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-frames", action="store_true", help="skip the frame-writer measurement")
    ap.add_argument("--e2e-units", type=int, default=100_000,
                    help="end-to-end leg: host PCM blocks through flacmi_encode_pipeline (0 = skip)")
    ap.add_argument("--e2e-batch", type=int, default=8192, help="end-to-end leg: units per sub-batch")
    ap.add_argument("--launch-check", action="store_true",
                    help="multi-rank plumbing only (CPU, gloo): self-launch, world-size check, shard "
                         "coverage and the stats all-reduce; prints a launch_check JSON line, no metric")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv):
    """`--gpus N > 1` outside a torch.distributed job: run N ranks of this script under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a CHILD process
    and return its exit status.  Called before anything touches the GPU (this process never
    initialises HIP), so nothing is exec'ed over a GPU-initialised process.  Returns None
    when no launch is needed (N == 1, or already a rank of a launched job)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL on this host: dmabuf IPC only
    return subprocess.call(cmd, env=env)


def check_world(args, world):
    """The process group must hold exactly the ranks --gpus asked for."""
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s); run "
                         f"`python bench.py --gpus {args.gpus}` (self-launch) or torch.distributed.run with "
                         f"--nproc-per-node {args.gpus}")


def algorithmic_bytes(cfg, meta_np, n_units):
    """SURVEY §8d algorithmic bytes per batch, B = n*s_in + 4*(n - order) + M per unit with
    M = 16 + 4*2^rmax + 4*L (samples in, the chosen zig-zag residual and the metadata out),
    per kernel:
      k_lpc  : n*s_in (it reads the samples; its LPC record is workspace)
      k_resid: B (samples in, residual + metadata out)
      step   : B (the whole analysis call)
    and, labelled separately, the same with the k_lpc -> k_resid LPC record (4 * rec_words:
    intermediate workspace, not SURVEY bytes) and this build's real metadata (208 B meta +
    4 B per Rice parameter)."""
    s_in = 2 if cfg["bits"] <= 16 else 4
    n = cfg["n"]
    rec = 4 * (2 + cfg["L"] + cfg["L"] * (cfg["L"] + 1) // 2) if cfg["mode"] == 0 else 0
    res = 4.0 * float(meta_np["res_len"].mean())
    parts = 4.0 * float(meta_np["n_parts"].mean())
    m_survey = 16 + 4 * (1 << cfg["rmax"]) + 4 * cfg["L"]
    survey = {"k_lpc": n_units * n * s_in, "k_resid": n_units * (n * s_in + res + m_survey),
              "step": n_units * (n * s_in + res + m_survey)}
    workspace = {"k_lpc": n_units * (n * s_in + rec), "k_resid": n_units * (n * s_in + rec + res + 208 + parts),
                 "step": n_units * (n * s_in + res + 208 + parts)}
    return survey, workspace


def _host_cpus():
    """(CPU model, nproc, CPUs this process may use): the affinity mask, capped by a cgroup
    v2 CPU quota when one is set (a GPU box shares its host between jobs)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return model, nproc, usable


def cpu_baseline(cfg, seconds, seed, open_eighths=0):
    """Oracle (oracle/flac_oracle.c, a C port of the reference's hot path) on host cores,
    on a bounded sample of the same workload (chunks of distinct synthetic units): every
    CPU this process may use, and one thread."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np

    import oracle  # test infrastructure: the CPU baseline leg only

    model, nproc, threads = _host_cpus()
    dt = np.int16 if cfg["bits"] <= 16 else np.int32
    p = oracle.make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])

    def run(nthreads, budget, chunk, first):
        done, t_an = 0, 0.0
        while t_an < budget:
            a = oracle.synth_batch(first + done, chunk, cfg["n"], cfg["bits"], seed, dtype=dt, open_eighths=open_eighths)
            t0 = time.perf_counter()
            oracle.analyze_batch(a, p, cfg["n"], sample_bits=cfg["bits"], threads=nthreads)
            t_an += time.perf_counter() - t0
            done += chunk
        return done, t_an

    chunk = (1024 if cfg["n"] <= 8192 else 128) * max(1, threads // 16)
    done, t_an = run(threads, seconds, chunk, 0)
    one, t_one = run(1, max(1.0, seconds / 4), 32 if cfg["n"] <= 8192 else 4, done)
    return {"value": done * cfg["n"] / t_an, "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": model, "nproc": nproc,
            "one_thread": {"value": one * cfg["n"] / t_one, "unit": "samples/s",
                           "sample": f"{one} units, {t_one:.1f} s"},
            "sample": f"{done} units x {cfg['n']} samples (synthetic units 0..{done - 1}), "
                      f"oracle/flac_oracle.c on {threads} host threads (the CPUs this process may use of "
                      f"{nproc}), {t_an:.1f} s; the reference Python itself measured 56.8k samples/s/core "
                      f"here (BASELINE.md)"}


def end_to_end_leg(args, cfg, az):
    """Host PCM rows -> FLAC frame bytes in host memory (end-to-end with the
    copies reported separately): flacmi_encode_pipeline over e2e_units synthetic blocks
    in sub-batches, the caller's buffers page-locked in place, H2D / analysis / sizes /
    pack / D2H each timed with HIP events (they overlap across sub-batches; wall is the
    whole call, page-locking included).  The first frames are compared with the one-shot
    flacmi_encode_host path."""
    import numpy as np
    import torch

    from flac_amd.analysis import make_params, unit_stride
    n, bits, C = cfg["n"], cfg["bits"], cfg["channels"]
    units = (args.e2e_units // C) * C
    dt = torch.int16 if bits <= 16 else torch.int32
    stride = unit_stride(n, 2 if bits <= 16 else 4)
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.empty((units, stride), dtype=dt, device=dev)
    az.synth_device(g.data_ptr(), g.element_size(), bits, stride, 10_000_000, units, n, args.seed,
                    open_eighths=args.open)
    torch.cuda.synchronize(dev)
    host = g.cpu().numpy()
    del g
    params = make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])
    kw = dict(sample_bits=bits, channels=C, sample_size=bits, units_per_batch=args.e2e_batch)
    az.encode_pipeline(host[: 4 * C], params, n, **kw)  # warm-up: contexts, windows, tables
    # cold: the call page-locks the caller's rows and its frame buffer itself
    data, offsets, status, tc = az.encode_pipeline(host, params, n, **kw)
    # streaming: page-locked staging rows and frame buffer allocated once and reused
    # (flacmi_host_alloc), as flac_amd.encoder's encode paths run batch after batch
    p0 = time.perf_counter()
    rows = az.host_array(host.shape, host.dtype)
    out = az.host_array((int(offsets[-1] * 1.05) + (1 << 20),), np.uint8)
    pin_ms = (time.perf_counter() - p0) * 1e3
    rows[...] = host
    data, offsets, status, t = az.encode_pipeline(rows, params, n, out=out, **kw)
    data = data.copy()
    k = min(256, units // C)
    ref = az.encode_frames(host[: k * C], params, n, sample_bits=bits, channels=C, sample_size=bits)
    same = bool(np.array_equal(offsets[: k + 1], ref[1]) and
                data[: int(offsets[k])].tobytes() == ref[0][: int(ref[1][k])].tobytes())
    wall = t["wall_ms"]
    cold = {"samples_per_s": units * n / (tc["wall_ms"] * 1e-3), "wall_ms": tc["wall_ms"],
            "register_ms": tc["register_ms"]}
    return {"units": units, "samples_per_s": units * n / (wall * 1e-3), "wall_ms": wall,
            "pinned_once_ms": pin_ms, "cold_call": cold,
            "units_per_sub_batch": args.e2e_batch, "sub_batches": t["sub_batches"],
            "step_ms": {k2: t[k2] for k2 in ("h2d_ms", "analyze_ms", "sizes_ms", "pack_ms", "d2h_ms", "register_ms")},
            "h2d_GBs": t["bytes_in"] / (t["h2d_ms"] * 1e-3) / 1e9 if t["h2d_ms"] else None,
            "d2h_GBs": t["bytes_out"] / (t["d2h_ms"] * 1e-3) / 1e9 if t["d2h_ms"] else None,
            "bytes_in": t["bytes_in"], "bytes_out": t["bytes_out"],
            "frames_with_status": int((status != 0).sum()),
            "first_frames_equal_one_shot_path": same,
            "note": "host int16 rows -> frame bytes in host memory through flacmi_encode_pipeline from "
                    "page-locked staging rows and frame buffer allocated once (flacmi_host_alloc, "
                    "pinned_once_ms, outside wall_ms), as the product's encode paths reuse them; cold_call: "
                    "ordinary numpy buffers the call page-locks itself; step times are per-step sums over "
                    "sub-batches (HIP events) and overlap in wall time"}


def frame_writer_leg(args, cfg, az, samples, meta, rparams, residual, pstride, units, sptr, check):
    """FLAC frames from the timed batch's analysis (not part of the
    metric, which is encode-analysis): k_frame_sizes + scan + k_pack, timed with HIP
    events on the launch stream over a few calls; a sample of frames is checked against
    the frame-writer oracle (oracle/frame_writer.py) on the device's own analysis."""
    import numpy as np
    import torch

    from flac_amd import abi
    from flac_amd.analysis import device_batch, frame_params

    dev = samples.device
    n, bits = cfg["n"], cfg["bits"]
    C = cfg["channels"]
    nf = units // C
    sbytes = samples.element_size()
    b = device_batch(samples.data_ptr(), sbytes, bits, samples.shape[1], nf * C, n)
    fp = frame_params(C, bits, cfg["q"], 0)
    off = torch.empty(nf + 1, dtype=torch.int64, device=dev)
    st = torch.empty(nf, dtype=torch.int32, device=dev)
    az.frame_sizes_device(b, fp, meta.data_ptr(), rparams.data_ptr(), pstride, off.data_ptr(), st.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    total = int(off[-1].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)

    def call():
        az.frame_sizes_device(b, fp, meta.data_ptr(), rparams.data_ptr(), pstride, off.data_ptr(), st.data_ptr(),
                              sptr)
        az.pack_frames_device(b, fp, meta.data_ptr(), rparams.data_ptr(), pstride, residual.data_ptr(), 4,
                              residual.shape[1], off.data_ptr(), st.data_ptr(), out.data_ptr(), out.numel(), sptr)

    call()
    torch.cuda.synchronize(dev)
    reps = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    bad_status = int((st != 0).sum().item())
    meta_np = meta[:, :].cpu().numpy().view(abi.META_DTYPE).reshape(units)
    res_read = 4.0 * float(meta_np["res_len"].sum())
    algo = res_read + total + units * 208 + 4.0 * float(meta_np["n_parts"].sum()) + 16.0 * nf
    res = {"ms_per_call": ms, "frames": nf, "bytes_out": total, "bytes_per_sample": total / (nf * C * n),
           "samples_per_s": nf * C * n / (ms * 1e-3), "algorithmic_GBs": algo / (ms * 1e-3) / 1e9,
           "frames_with_status": bad_status,
           "note": "k_frame_sizes + 3-kernel scan + k_pack per call; reads the zig-zag residual rows, writes "
                   "byte-exact FLAC frames (headers, Rice codes, CRC-8/16)"}
    # decoder round trip (BASELINE config 5): every frame decoded on the
    # device and compared in-kernel with the source units (CRC-8/16, frame numbers and
    # frame ends verified too)
    dst = torch.empty(nf, dtype=torch.int32, device=dev)
    dmm = torch.empty(nf, dtype=torch.int64, device=dev)
    dp = abi.DecodeParams()
    dp.channels, dp.sample_size, dp.first_frame, dp.check_crc = C, bits, 0, 1
    eb = device_batch(samples.data_ptr(), sbytes, bits, samples.shape[1], nf * C, n)

    def dcall():
        az.decode_frames_device(out.data_ptr(), total, off.data_ptr(), nf, dp, eb, 0, 0, dst.data_ptr(),
                                dmm.data_ptr(), sptr)

    dcall()
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(2):
        dcall()
    e1.record()
    torch.cuda.synchronize(dev)
    dms = e0.elapsed_time(e1) / 2
    res["decoder_round_trip"] = {
        "ms_per_call": dms, "samples_per_s": nf * C * n / (dms * 1e-3),
        "algorithmic_GBs": (total + nf * C * n * sbytes) / (dms * 1e-3) / 1e9,
        "frames_with_status": int((dst != 0).sum().item()), "samples_mismatched": int(dmm.sum().item()),
        "note": "k_decode_fx (one lane per frame: CONSTANT/VERBATIM/FIXED subframes, every check passing) "
                "then k_decode (the general decoder) over the frames it lists, decoded samples compared "
                "in-kernel with the source units; CRC-8/16, frame numbers and frame ends verified; "
                "algorithmic bytes = the stream read + the source rows compared"}
    if check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import frame_writer as FW  # checker only
        rng = np.random.default_rng(args.seed + 1)
        pick = np.sort(rng.choice(nf, size=min(32, nf), replace=False))
        offs = off.cpu().numpy()
        rp_np = rparams.cpu().numpy() if units <= 65536 else None
        bad = 0
        for f in pick:
            us = list(range(f * C, (f + 1) * C))
            rows = samples[torch.as_tensor(us, device=dev)].cpu().numpy()[:, :n]
            ms_ = [meta_np[u] for u in us]
            zz = [residual[u].cpu().numpy().view(np.uint32)[int(m["res_offset"]):int(m["res_offset"]) + int(m["res_len"])]
                  for u, m in zip(us, ms_)]
            prm = [(rp_np[u] if rp_np is not None else rparams[u].cpu().numpy())[: int(m["n_parts"])]
                   for u, m in zip(us, ms_)]
            want = FW.frame(int(f), n, list(rows), ms_, zz, prm, bits, cfg["q"])
            got = out[int(offs[f]):int(offs[f + 1])].cpu().numpy().tobytes()
            bad += 0 if got == want else 1
        res["parity"] = {"frames_checked": int(len(pick)), "mismatches": bad,
                         "check": "bytes vs oracle/frame_writer.py on the device analysis"}
    return res


def library_sha16():
    """sha256[:16] of the libflacmi.so this process loads (flac_amd._lib.LIB_PATH)."""
    import hashlib
    from flac_amd import _lib
    try:
        return hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def shard_first_unit(rank, units_per_rank):
    """First global unit of a rank's shard: contiguous, disjoint block ranges (units are
    independent), so the stream statistics are a plain sum over ranks."""
    return rank * units_per_rank


def reduce_stats(stats, dist=None, comm=None, stream=0):
    """Stream totals over ranks: the one collective of the multi-GPU path.  On the GPU it is
    the C-ABI's flacmi_allreduce_stats (RCCL over xGMI, `comm` a flac_amd StatsComm, on the
    launch stream); without a comm (the gloo CPU tests) the same sum over torch.distributed."""
    if comm is not None:
        comm.allreduce_stats(stats.data_ptr(), stream)
    elif dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats)
    return stats


def broadcast_comm_id(cid, dist, nbytes, device=None):
    """Rank 0's flacmi_comm_id bytes (ncclUniqueId) to every rank over the existing process
    group, so each rank can build the C-ABI communicator (flacmi_comm_init)."""
    import torch
    t = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    if dist.get_rank() == 0:
        if cid is None or len(cid) != nbytes:
            raise ValueError(f"rank 0 needs a {nbytes}-byte comm id")
        t.copy_(torch.frombuffer(bytearray(cid), dtype=torch.uint8))
    dist.broadcast(t, 0)
    return bytes(t.cpu().numpy().tobytes())


def all_ranks_ok(ok, dist, device=None):
    """True when `ok` holds on every rank (a MIN all-reduce over the process group)."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def open_stats_comm(az, dist, rank, world, device):
    """The C-ABI stats communicator of an N-rank job: rank 0's id broadcast over the process
    group, then flacmi_comm_init on every rank (a collective call).  -> (comm, reason): comm
    None, with the reason, when some rank cannot load RCCL or build the communicator, so the
    job reduces through torch.distributed instead of failing.  Every rank's local
    preconditions run first and all ranks agree on them before the collective init: the
    device is set when the Analyzer opens its context, flacmi_comm_available loads RCCL and
    its entry points (no id, no listener), and only rank 0 calls flacmi_comm_id (an id makes a
    bootstrap listener).  Not covered: a rank failing inside ncclCommInitRank itself, after
    the others have entered it (they then block in RCCL's bootstrap)."""
    from flac_amd import abi
    from flac_amd.analysis import StatsComm
    why, cid = "", None
    try:
        StatsComm.available(az.lib)
        if rank == 0:
            cid = StatsComm.comm_id(az.lib)
        ok = True
    except Exception as e:  # noqa: BLE001 (recorded in the bench line)
        ok, why = False, f"rank {rank}: {'flacmi_comm_id' if 'comm_id' in str(e) else 'flacmi_comm_available'}: {e}"
    if not all_ranks_ok(ok, dist, device):
        return None, why or "a rank could not load RCCL (flacmi_comm_available / flacmi_comm_id)"
    cid = broadcast_comm_id(cid if rank == 0 else None, dist, abi.COMM_ID_BYTES, device)
    comm = None
    try:
        comm = StatsComm(az, world, rank, cid)
    except Exception as e:  # noqa: BLE001
        why = f"rank {rank}: flacmi_comm_init: {e}"
    if not all_ranks_ok(comm is not None, dist, device):
        if comm is not None:
            comm.close()
        return None, why or "a rank could not build the communicator (flacmi_comm_init)"
    return comm, ""


def reduce_elapsed(elapsed, dist=None, device=None):
    """Max over ranks of the timed region (the contract's whole-job time)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return elapsed


def shard_plan(cfg, rank, world, units, total_units_arg=0):
    """(first_unit, chunks) of one rank.  Non-chunked configs: the contiguous shard
    [rank*U, (rank+1)*U) (weak scaling).  c4: chunk ci of the fixed job goes to rank
    ci % world (round-robin, BASELINE config 4), chunks of `units` blocks."""
    if "total_units" not in cfg:
        return shard_first_unit(rank, units), [], world * units
    total = total_units_arg or cfg["total_units"]
    n_chunks = (total + units - 1) // units
    return 0, list(range(rank, n_chunks, world)), total


def run_chunks(az, cfg, params, bufs, chunk_ids, units, total_units, seed, stream=0, on_chunk=None, open_eighths=0):
    """One rank's share of a chunked job (config 4): for each of its round-robin chunks,
    generate the chunk's blocks on the device (global block index = chunk * units + i, the
    frame number of the reference's block loop, encoder.py:87-97), analyse them and add the
    chunk's stream statistics into bufs["stats_acc"] (zeroed first).  on_chunk(ci, cu), if
    given, runs after each chunk's analysis (tests sample the chunk's units there)."""
    n, bits = cfg["n"], cfg["bits"]
    samples, meta, rparams, residual = bufs["samples"], bufs["meta"], bufs["rparams"], bufs["residual"]
    sbytes = samples.element_size()
    sstride, pstride, rstride = samples.shape[1], rparams.shape[1], residual.shape[1]
    bufs["stats_acc"].zero_()

    def analyse(ci, cu, rows):
        az.analyze_device(rows.data_ptr(), sbytes, bits, sstride, cu, n, params, meta.data_ptr(),
                          rparams.data_ptr(), pstride, residual.data_ptr(), rstride, 4, stream)
        az.stream_stats(meta.data_ptr(), cu, n, bufs["stats"].data_ptr(), stream)
        bufs["stats_acc"].add_(bufs["stats"])
        bufs["cur_samples"] = rows
        if on_chunk is not None:
            on_chunk(ci, cu)

    def size(ci):
        return min(units, total_units - ci * units)

    if "samples_b" not in bufs or len(chunk_ids) < 2:
        for ci in chunk_ids:
            az.synth_device(samples.data_ptr(), sbytes, bits, sstride, ci * units, size(ci), n, seed, stream, open_eighths)
            analyse(ci, size(ci), samples)
        return bufs["stats_acc"]
    # double-buffered (the input of a streaming encoder): chunk k + 1 is generated into the
    # other buffer on bufs["synth_stream"] while chunk k is analysed; events order each buffer's
    # generation after the analysis that last read it, and each analysis after its generation
    import torch
    main = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
    side = bufs["synth_stream"]
    rows = (samples, bufs["samples_b"])
    ready = (torch.cuda.Event(), torch.cuda.Event())
    freed = (torch.cuda.Event(), torch.cuda.Event())
    start = torch.cuda.Event()
    start.record(main)
    side.wait_event(start)  # the previous step's last reads of buffer 0

    def gen(k):
        ci = chunk_ids[k]
        az.synth_device(rows[k & 1].data_ptr(), sbytes, bits, sstride, ci * units, size(ci), n, seed,
                        side.cuda_stream, open_eighths)
        ready[k & 1].record(side)

    gen(0)
    for k, ci in enumerate(chunk_ids):
        main.wait_event(ready[k & 1])
        analyse(ci, size(ci), rows[k & 1])
        freed[k & 1].record(main)
        if k + 1 < len(chunk_ids):
            if k >= 1:
                side.wait_event(freed[(k + 1) & 1])  # chunk k - 1's analysis read that buffer
            gen(k + 1)
    return bufs["stats_acc"]


def launch_check(args, cfg, units):
    """Multi-rank plumbing without a GPU (gloo): each rank reports its shard as a stats
    vector [units, samples, first, last+1, rank bit]; the all-reduced vector must cover
    the job exactly once.  Rank 0 prints one launch_check JSON line."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    check_world(args, world)
    first, chunks, total = shard_plan(cfg, rank, world, units, args.total_units)
    if chunks:
        mine = sum(min(units, total - ci * units) for ci in chunks)
        lo, hi = chunks[0] * units, min(total, chunks[-1] * units + units)
    else:
        mine, lo, hi = units, first, first + units
    st = torch.tensor([mine, mine * cfg["n"], lo, hi, 1 << rank], dtype=torch.int64)
    reduce_stats(st, dist)
    el = reduce_elapsed(0.001 * (rank + 1), dist)
    id_ok = None
    if world > 1:
        # the comm-id hand-off the GPU path makes before flacmi_comm_init (a fixed 128-byte
        # pattern stands in for rank 0's ncclUniqueId); every rank must hold rank 0's bytes
        pattern = bytes((i * 37 + 11) % 256 for i in range(128))
        got = broadcast_comm_id(pattern if rank == 0 else None, dist, 128)
        ok = torch.tensor([int(got == pattern)], dtype=torch.int64)
        dist.all_reduce(ok)
        id_ok = int(ok.item()) == world
    if rank == 0:
        print(json.dumps({"launch_check": True, "world_size": world, "gpus_arg": args.gpus, "config": args.config,
                          "units_total": int(st[0]), "samples_total": int(st[1]), "expected_units": total,
                          "rank_mask": int(st[4]), "elapsed_max": el, "comm_id_broadcast_ok": id_ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        return rc
    cfg = dict(CONFIGS[args.config])
    if args.open:
        cfg["workload"] += "; " + OPEN_NOTE.format(k=args.open)
    units = args.units or cfg["units"]
    if args.launch_check:
        launch_check(args, cfg, units)
        return 0

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
    check_world(args, world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from flac_amd import abi
    from flac_amd.analysis import Analyzer, get_knob, knob, make_params, params_stride_for, unit_stride

    az = Analyzer(local)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    n, bits = cfg["n"], cfg["bits"]
    sdt = torch.int16 if bits <= 16 else torch.int32
    sbytes = 2 if bits <= 16 else 4
    sstride = unit_stride(n, sbytes)
    rstride = ((n * 4 + 15) // 16) * 16 // 4
    pstride = params_stride_for(cfg["rmax"])
    first_unit, my_chunks, total_units = shard_plan(cfg, rank, world, units, args.total_units)
    chunked = "total_units" in cfg

    samples = torch.empty((units, sstride), dtype=sdt, device=dev)
    meta = torch.empty((units, abi.META_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    rparams = torch.empty((units, pstride), dtype=torch.int32, device=dev)
    residual = torch.empty((units, rstride), dtype=torch.int32, device=dev)
    stats = torch.zeros(abi.STATS_WORDS, dtype=torch.int64, device=dev)
    az.synth_device(samples.data_ptr(), sbytes, bits, sstride, first_unit, units, n, args.seed, sptr, args.open)
    params = make_params(cfg["L"], cfg["q"], cfg["rmin"], cfg["rmax"], cfg["mode"])

    stats_acc = torch.zeros_like(stats)
    bufs = dict(samples=samples, meta=meta, rparams=rparams, residual=residual, stats=stats, stats_acc=stats_acc)
    if chunked and len(my_chunks) > 1:  # c4: the next chunk is generated while this one is analysed
        bufs["samples_b"] = torch.empty_like(samples)
        bufs["synth_stream"] = torch.cuda.Stream(dev)
    # N > 1: the stream totals go through the C-ABI collective (flacmi_allreduce_stats)
    comm, comm_note = open_stats_comm(az, dist, rank, world, dev) if distributed else (None, "")

    def step():
        if not chunked:
            az.analyze_device(samples.data_ptr(), sbytes, bits, sstride, units, n, params, meta.data_ptr(),
                              rparams.data_ptr(), pstride, residual.data_ptr(), rstride, 4, sptr)
            az.stream_stats(meta.data_ptr(), units, n, stats.data_ptr(), sptr)
            reduce_stats(stats, dist, comm, sptr)
            return
        run_chunks(az, cfg, params, bufs, my_chunks, units, total_units, args.seed, sptr, open_eighths=args.open)
        reduce_stats(stats_acc, dist, comm, sptr)
        stats.copy_(stats_acc)

    for _ in range(args.warmup):
        step()
    if comm is not None:
        # the C-ABI reduce must equal torch.distributed's sum of the same per-rank vectors
        # (outside the timed region: one more step's local stats, reduced both ways)
        local_stats = (stats_acc if chunked else stats).clone()
        if not chunked:
            az.stream_stats(meta.data_ptr(), units, n, local_stats.data_ptr(), sptr)
        via_torch = local_stats.clone()
        torch.cuda.synchronize(dev)
        dist.all_reduce(via_torch)
        reduce_stats(local_stats, dist, comm, sptr)
        torch.cuda.synchronize(dev)
        if not all_ranks_ok(torch.equal(local_stats, via_torch), dist, dev):
            # recorded in the bench line; the timed steps then reduce through torch.distributed
            comm.close()
            comm, comm_note = None, "flacmi_allreduce_stats differed from torch.distributed's all_reduce"
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    az.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kt = az.timing()
    elapsed = reduce_elapsed(elapsed, dist, dev)
    kt_steps, isolated_calls = kt, 0
    if cfg["L"] > 0 and not cfg["mode"] and get_knob("FLACMI_OVERLAP") != 0:
        # The library's default chunking overlaps k_lpc's last, partly filled round with
        # k_resid of the first chunk (flacmi_host.cpp overlap_mode), so the timed
        # steps' stage spans include the other kernel's waves.  The roofline prices each kernel
        # on launches of its own: a few more calls with one chunk (the FLACMI_OVERLAP knob at 0),
        # after the timed region.
        with knob("FLACMI_OVERLAP", 0):
            step()
            torch.cuda.synchronize(dev)
            az.timing_reset()
            isolated_calls = max(1, min(args.steps, 5))
            for _ in range(isolated_calls):
                step()
            torch.cuda.synchronize(dev)
            kt = az.timing()

    meta_np = meta.cpu().numpy().view(abi.META_DTYPE).reshape(units)
    st = stats.cpu().numpy()
    total_samples = total_units * n * args.steps
    value = total_samples / elapsed

    # ---- parity: sampled units vs the CPU oracle (outside the timed region) ----
    parity = None
    if rank == 0 and not args.no_parity and args.parity_units > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # checker only
        rng = np.random.default_rng(args.seed)
        pick = rng.choice(units, size=min(args.parity_units, units), replace=False)
        # plus up to 8 units of every pruning path the batch took (meta.lpc_tiers: quarter or
        # eighth tiers, the sign bound's passes, the retry list's 0/1 and 1/1, exact passes)
        tiers_all = meta_np["lpc_tiers"].astype(np.int64)
        extra = [rng.choice(np.nonzero(tiers_all == t)[0], size=min(8, int((tiers_all == t).sum())), replace=False)
                 for t in np.unique(tiers_all)]
        pick = np.unique(np.concatenate([pick] + extra))
        rows = bufs.get("cur_samples", samples)  # c4: the buffer the last analysed chunk was generated in
        s_host = rows[torch.as_tensor(pick, device=dev)].cpu().numpy()[:, :n]
        ora = oracle.analyze_batch(np.ascontiguousarray(s_host), oracle.make_params(cfg["L"], cfg["q"], cfg["rmin"],
                                   cfg["rmax"], cfg["mode"]), n, sample_bits=bits, threads=16)
        res_host = residual[torch.as_tensor(pick, device=dev)].cpu().numpy().view(np.uint32)
        par_host = rparams[torch.as_tensor(pick, device=dev)].cpu().numpy()
        bad = pruned = 0
        for j, u in enumerate(pick):
            g, o = meta_np[u], ora["meta"][j]
            same = not oracle.meta_mismatches(g, o)
            pruned += int(g["lpc_order"]) == abi.LPC_PRUNED
            off, ln = int(o["res_offset"]), int(o["res_len"])
            same = same and np.array_equal(res_host[j][off:off + ln].astype(np.uint64), ora["residual"][j][off:off + ln])
            k = int(o["n_parts"])
            same = same and np.array_equal(par_host[j][:k], ora["rice_params"][j][:k])
            bad += 0 if same else 1
        covered = {f"{t & 0xff}/{t >> 8}": int((tiers_all[pick] == t).sum()) for t in np.unique(tiers_all)}
        parity = {"units_checked": int(len(pick)), "mismatches": bad, "lpc_pruned": pruned, "lpc_tiers_checked": covered,
                  "check": "meta, coefficients, zig-zag residual and Rice parameters bit-exact vs oracle "
                           "(a unit reporting FLACMI_LPC_PRUNED must lose to fixed in the oracle too)"}

    frames = None
    if not args.no_frames and not chunked:
        frames = frame_writer_leg(args, cfg, az, samples, meta, rparams, residual, pstride, units, sptr,
                                  rank == 0 and not args.no_parity)

    e2e = None
    # (FLACMI_DEBUG_STOP truncates k_resid: its metadata must never reach the frame writer)
    if rank == 0 and world == 1 and args.e2e_units > 0 and not chunked and not os.environ.get("FLACMI_DEBUG_STOP"):
        e2e = end_to_end_leg(args, cfg, az)

    ab, ab_ws = algorithmic_bytes(cfg, meta_np, units)
    lpc_b, resid_b, pipe_b = ab["k_lpc"], ab["k_resid"], ab["step"]
    lpc_gbs = lpc_b / (kt["lpc_ms"] * 1e-3) / 1e9 if kt["lpc_ms"] > 0 else 0.0
    resid_gbs = resid_b / (kt["resid_ms"] * 1e-3) / 1e9 if kt["resid_ms"] > 0 else 0.0
    dominant = "k_resid" if kt["resid_ms"] >= kt["lpc_ms"] else "k_lpc"
    dom_gbs = resid_gbs if dominant == "k_resid" else lpc_gbs
    dom_bytes = resid_b if dominant == "k_resid" else lpc_b
    dom_ms = kt["resid_ms"] if dominant == "k_resid" else kt["lpc_ms"]
    traffic, traffic_lib = None, None
    tfile = os.path.join(REPO, "profiles", f"traffic_{args.config}" + (f"_open{args.open}" if args.open else "") +
                         ("_noprune" if os.environ.get("FLACMI_NO_PRUNE", "0") not in ("", "0") else "") + ".json")
    if os.path.exists(tfile):  # HBM bytes per launch from the separate rocprofv3 --pmc passes
        try:
            tj = json.load(open(tfile))
            traffic, traffic_lib = tj.get(dominant), tj.get("library_sha16")
        except Exception:
            traffic = None
    # counters cannot be collected inside the timed run: the committed figure is current only
    # while it was measured on this very library
    lib_now = library_sha16()
    traffic_current = traffic is not None and traffic_lib is not None and traffic_lib == lib_now
    if traffic is not None and not traffic_current and rank == 0:
        print(f"bench.py: {os.path.relpath(tfile, REPO)} was profiled on library {traffic_lib}, this run uses "
              f"{lib_now}: re-run tools/profile.sh for a current traffic figure", file=sys.stderr)

    if rank == 0:
        # rank 0 only, after the timed region (the other ranks are idle by then)
        cpu = cpu_baseline(cfg, args.cpu_seconds, args.seed, args.open) if args.cpu_seconds > 0 else None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if chunked else "weak",
            "vs_baseline": None,
            "dtype": "i16 in; f64 autocorrelation/Levinson; i32 predictors",
            "data": "synthetic: on-device integer generator (3 DDS tones + splitmix64 noise, SURVEY §8d)" +
                    (f"; {args.open}/8 of the units MA(1) near-white noise (--open)" if args.open else ""),
            "config": {"workload": cfg["workload"], "units_per_gpu": total_units // world,
                       "units_total": total_units, "chunk_units": units if chunked else None, "block": n, "sample_bits": bits,
                       "max_lpc_order": cfg["L"], "qlp_precision": cfg["q"], "rice": [cfg["rmin"], cfg["rmax"]],
                       "mode": "fixed-only" if cfg["mode"] else "reference", "parallelism": f"dp{world} (block shards)",
                       "open_eighths": args.open,
                       "lpc_pruning": ("off: every LPC candidate's exact sum (FLACMI_NO_PRUNE=1)"
                                       if os.environ.get("FLACMI_NO_PRUNE", "0") not in ("", "0") else
                                       "on: candidates proven to lose skipped (sign bound, partial-sum tiers)"),
                       "stats_collective": ("flacmi_allreduce_stats (C-ABI, RCCL)" if comm is not None else
                                            f"torch.distributed all_reduce ({comm_note})" if distributed else None)},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": dom_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": dom_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": (os.path.relpath(tfile, REPO) + ": rocprofv3 FETCH_SIZE/WRITE_SIZE passes "
                                            "of this config (tools/profile.sh, tools/traffic.py)") if traffic else None,
                         "traffic_current": traffic_current,  # profiled on the library this run timed
                         "traffic_library_sha16": traffic_lib, "library_sha16": lib_now,
                         "algorithmic_bytes_per_launch": dom_bytes,
                         "algorithmic_bytes_source": "SURVEY §8d: n*s_in + 4*(n - order) + 16 + 4*2^rmax + 4*L per unit",
                         "kernel_ms": dom_ms,
                         # labelled separately: with the k_lpc -> k_resid LPC record (workspace)
                         # and this build's 208-byte meta + Rice parameters
                         "with_workspace": {"bytes_per_launch": ab_ws[dominant],
                                            "frac": ab_ws[dominant] / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                            if dom_ms else None},
                         # the whole analysis step (k_lpc + k_resid + retries): SURVEY 8d bytes / call time
                         "pipeline_frac": (pipe_b / (kt_steps["call_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS)
                         if kt_steps["call_ms"] else None,
                         "pipeline_algorithmic_bytes": pipe_b},
            "kernels": {"k_lpc_ms": kt["lpc_ms"], "k_resid_ms": kt["resid_ms"], "call_ms": kt["call_ms"],
                        "k_lpc_GBs": lpc_gbs, "k_resid_GBs": resid_gbs,
                        "pipeline_GBs": pipe_b / (kt_steps["call_ms"] * 1e-3) / 1e9 if kt_steps["call_ms"] else 0.0,
                        "timed_calls": kt["calls"],
                        "launches": ("one chunk per call (FLACMI_OVERLAP=0): %d calls after the timed steps, "
                                     "whose calls overlap k_lpc's last round with k_resid" % isolated_calls)
                        if isolated_calls else "the timed steps' calls",
                        "timed_steps": {"call_ms": kt_steps["call_ms"], "k_lpc_span_ms": kt_steps["lpc_ms"],
                                        "k_resid_span_ms": kt_steps["resid_ms"]} if isolated_calls else None},
            "cpu_baseline": cpu,
            "frame_writer": frames,
            "end_to_end": e2e,
            "parity": parity,
            "stream_stats": {"units": int(st[0]), "samples": int(st[1]), "rice_bits": int(st[2]),
                             "fixed": int(st[3]), "lpc": int(st[4]), "lpc_pruned": int(st[81]),
                             "errors": int(st[65:80].sum()),
                             # meta.lpc_tiers of this rank's last batch: LPC candidate passes made
                             # before the decision, as "passes/passes of the path": units
                             "lpc_tiers": {f"{t & 0xff}/{t >> 8}": int(c) for t, c in
                                           zip(*np.unique(meta_np["lpc_tiers"], return_counts=True))}},
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    az.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
