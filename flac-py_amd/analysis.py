"""Batched encode-analysis on the GPU through libflacmi.so.

`Analyzer` owns one flacmi context (one HIP device).  `analyze()` takes a 2-D array of
planar units (one row per (block, channel)), runs fixed + LPC + choice + Rice search
on the device and returns numpy views of the per-unit results (the fields of
flac/common.py's SubframeHeader / SubframeFixed / SubframeLPC / Residual, see
include/flacmi.h).  `analyze_device()` is the zero-copy form on device pointers used by
bench.py.
"""
import ctypes as C
import weakref

import numpy as np

from . import abi
from ._lib import FlacmiError, check, load


def make_params(max_lpc_order: int, qlp_precision: int, rice_min: int, rice_max: int,
                mode: int = abi.MODE_REFERENCE, all_candidates: bool = False,
                tiers_only: bool = False) -> abi.Params:
    """all_candidates: exact sum(|r|) for every LPC candidate (meta.lpc_order / lpc_sum always
    exact); by default a unit whose LPC candidates provably lose reports abi.LPC_PRUNED there.
    tiers_only (diagnostic): the int8-MFMA path prunes with its partial-sum tiers alone."""
    p = abi.Params()
    p.max_lpc_order = max_lpc_order
    p.qlp_precision = qlp_precision
    p.rice_min = rice_min
    p.rice_max = rice_max
    p.mode = mode
    p.reserved[1] = (abi.FLAG_ALL_CANDIDATES if all_candidates else 0) | (abi.FLAG_TIERS_ONLY if tiers_only else 0)
    return p


def frame_params(channels: int, sample_size: int, qlp_precision: int, first_frame: int = 0) -> abi.FrameParams:
    fp = abi.FrameParams()
    fp.channels = channels
    fp.sample_size = sample_size
    fp.qlp_precision = qlp_precision
    fp.first_frame = first_frame
    return fp


def device_batch(samples_ptr: int, sample_bytes: int, sample_bits: int, unit_stride: int, n_units: int,
                 block_len: int, tail_len: int = 0, n_tail_units: int = 0) -> abi.Batch:
    b = abi.Batch()
    b.samples = samples_ptr
    b.sample_bytes = sample_bytes
    b.sample_bits = sample_bits
    b.unit_stride = unit_stride
    b.n_units = n_units
    b.block_len = block_len
    b.tail_len = tail_len
    b.n_tail_units = n_tail_units
    return b


def unit_stride(block_len: int, sample_bytes: int) -> int:
    """The row pitch (samples) the library lays device rows out at (flacmi_unit_stride): 16-byte
    rows, plus 128 bytes when the pitch is a multiple of 4 KB."""
    v = load().flacmi_unit_stride(block_len, sample_bytes)
    check(v if v < 0 else 0, "flacmi_unit_stride")
    return v


def get_knob(name: str) -> int:
    """A test/diagnostic knob of the library (flacmi_get_knob)."""
    v = C.c_int32(0)
    check(load().flacmi_get_knob(name.encode(), C.byref(v)), "flacmi_get_knob")
    return v.value


def set_knob(name: str, value: int) -> None:
    """Set a test/diagnostic knob (flacmi_set_knob): FLACMI_OVERLAP, FLACMI_MF8_GRID,
    FLACMI_STREAM_GENERIC, FLACMI_DECODE_GENERIC.  The library reads their environment variables once; this is the
    thread-safe way to change them afterwards."""
    check(load().flacmi_set_knob(name.encode(), int(value)), "flacmi_set_knob")


class knob:
    """`with knob("FLACMI_OVERLAP", 0): ...` sets a knob and restores its previous value."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, value

    def __enter__(self):
        self.prev = get_knob(self.name)
        set_knob(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_knob(self.name, self.prev)
        return False


def params_stride_for(rice_max: int) -> int:
    return (1 << max(rice_max, 0)) + 1


class Analyzer:
    def __init__(self, device: int = 0):
        self.lib = load()
        self.device = device
        self.ctx = self.lib.flacmi_create(device)
        if not self.ctx:
            raise FlacmiError(f"flacmi_create({device}) failed: "
                              f"{self.lib.flacmi_last_error().decode(errors='replace')}")

    def close(self):
        if self.ctx:
            self.lib.flacmi_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------------
    def analyze(self, samples: np.ndarray, params: abi.Params, block_len: int, tail_len: int = 0,
                n_tail_units: int = 0, sample_bits: int = 16, residual_bytes: int = 4,
                debug: bool = False, extras=()) -> dict:
        """Host arrays in, host arrays out (synchronous).  debug: every optional output (acf,
        fixed_sums, lpc_sums, lpc_records); extras: a subset of those names instead (lpc_sums
        turns LPC pruning off, the others do not)."""
        s = np.ascontiguousarray(samples)
        if s.dtype not in (np.int16, np.int32) or s.ndim != 2:
            raise ValueError("samples must be a 2-D int16 or int32 array")
        n_units, stride = s.shape
        b = abi.Batch()
        b.samples = s.ctypes.data
        b.sample_bytes = s.dtype.itemsize
        b.sample_bits = sample_bits
        b.unit_stride = stride
        b.n_units = n_units
        b.block_len = block_len
        b.tail_len = tail_len
        b.n_tail_units = n_tail_units
        pstride = params_stride_for(params.rice_max)
        rdt = np.uint32 if residual_bytes == 4 else np.uint64
        rstride = ((block_len * residual_bytes + 15) // 16) * 16 // residual_bytes
        out = {
            "meta": np.zeros(n_units, dtype=abi.META_DTYPE),
            "rice_params": np.zeros((n_units, pstride), dtype=np.int32),
            "residual": np.zeros((n_units, rstride), dtype=rdt),
        }
        o = abi.Outputs()
        o.meta = out["meta"].ctypes.data
        o.rice_params = out["rice_params"].ctypes.data
        o.params_stride = pstride
        o.residual = out["residual"].ctypes.data
        o.residual_bytes = residual_bytes
        o.residual_stride = rstride
        want = ("acf", "fixed_sums", "lpc_sums", "lpc_records") if debug else tuple(extras)
        shapes = {"acf": (33, np.float64), "fixed_sums": (5, np.int64), "lpc_sums": (32, np.int64),
                  "lpc_records": (abi.lpc_rec_words(32), np.int32)}
        for k in want:
            w, dt = shapes[k]
            out[k] = np.zeros((n_units, w), dtype=dt)
            setattr(o, k, out[k].ctypes.data)
        check(self.lib.flacmi_analyze_host(self.ctx, C.byref(b), C.byref(params), C.byref(o)),
              "flacmi_analyze_host")
        wide = np.flatnonzero(out["meta"]["status"] == abi.STATUS_RESIDUAL_WIDE) if residual_bytes == 4 else []
        if len(wide):
            # a chosen residual needs more than 32 bits: redo only those units with 64-bit
            # rows and widen the batch's rows (the other units' results stand)
            first_tail = n_units - n_tail_units
            sub = self.analyze(np.ascontiguousarray(s[wide]), params, block_len, tail_len,
                               int(np.count_nonzero(wide >= first_tail)), sample_bits, 8, debug, extras)
            w = max(out["residual"].shape[1], sub["residual"].shape[1])
            res = np.zeros((n_units, w), dtype=np.uint64)
            res[:, :out["residual"].shape[1]] = out["residual"]
            res[wide] = 0
            res[wide, :sub["residual"].shape[1]] = sub["residual"]
            out["residual"] = res
            for k, v in sub.items():
                if k != "residual":
                    out[k][wide] = v
        return out

    def analyze_device(self, samples_ptr: int, sample_bytes: int, sample_bits: int, unit_stride: int,
                       n_units: int, block_len: int, params: abi.Params, meta_ptr: int,
                       params_ptr: int, params_stride: int, residual_ptr: int, residual_stride: int,
                       residual_bytes: int = 4, stream: int = 0, tail_len: int = 0,
                       n_tail_units: int = 0) -> None:
        """Device pointers in/out; enqueued on `stream`, returns without synchronising."""
        b = abi.Batch()
        b.samples = samples_ptr
        b.sample_bytes = sample_bytes
        b.sample_bits = sample_bits
        b.unit_stride = unit_stride
        b.n_units = n_units
        b.block_len = block_len
        b.tail_len = tail_len
        b.n_tail_units = n_tail_units
        o = abi.Outputs()
        o.meta = meta_ptr
        o.rice_params = params_ptr
        o.params_stride = params_stride
        o.residual = residual_ptr
        o.residual_bytes = residual_bytes
        o.residual_stride = residual_stride
        check(self.lib.flacmi_analyze_device(self.ctx, C.byref(b), C.byref(params), C.byref(o), stream),
              "flacmi_analyze_device")

    # ------------------------------------------------------------------------------
    # frame writer (include/flacmi.h flacmi_frame_sizes_device / flacmi_pack_frames_device)
    # ------------------------------------------------------------------------------
    def encode_frames(self, samples: np.ndarray, params: abi.Params, block_len: int, tail_len: int = 0,
                      n_tail_units: int = 0, sample_bits: int = 16, channels: int = 1,
                      sample_size: int = 16, first_frame: int = 0):
        """Host rows in -> (frame bytes, frame offsets [n_frames + 1], frame status [n_frames]).

        Row f*channels + c is channel c of frame f.  A frame whose status is non-zero
        (the reference's exception, (site << 16) | status) has no bytes."""
        s = np.ascontiguousarray(samples)
        if s.dtype not in (np.int16, np.int32) or s.ndim != 2:
            raise ValueError("samples must be a 2-D int16 or int32 array")
        n_units, stride = s.shape
        b = abi.Batch()
        b.samples = s.ctypes.data
        b.sample_bytes = s.dtype.itemsize
        b.sample_bits = sample_bits
        b.unit_stride = stride
        b.n_units = n_units
        b.block_len = block_len
        b.tail_len = tail_len
        b.n_tail_units = n_tail_units
        fp = frame_params(channels, sample_size, params.qlp_precision, first_frame)
        n_frames = n_units // channels if channels else 0
        offsets = np.zeros(n_frames + 1, dtype=np.int64)
        status = np.zeros(max(n_frames, 1), dtype=np.int32)
        check(self.lib.flacmi_encode_host(self.ctx, C.byref(b), C.byref(params), C.byref(fp),
                                          offsets.ctypes.data, status.ctypes.data), "flacmi_encode_host")
        total = int(offsets[-1])
        out = np.empty(total, dtype=np.uint8)
        check(self.lib.flacmi_encode_fetch(self.ctx, out.ctypes.data, total), "flacmi_encode_fetch")
        return out, offsets, status[:n_frames]

    def encode_pipeline(self, samples: np.ndarray, params: abi.Params, block_len: int, tail_len: int = 0,
                        n_tail_units: int = 0, sample_bits: int = 16, channels: int = 1, sample_size: int = 16,
                        first_frame: int = 0, units_per_batch: int = 8192, capacity: int = 0,
                        out: np.ndarray = None):
        """encode_frames through flacmi_encode_pipeline: host rows in (any row stride), the
        batch streamed through the device in sub-batches of units_per_batch units with the
        PCIe copies overlapping the kernels.  `out` (optional, uint8): the caller's frame
        buffer, reused across calls (with host_register it stays page-locked).  Returns
        (frame bytes, frame offsets [n_frames + 1], frame status [n_frames], timing dict)."""
        s = samples
        if s.dtype not in (np.int16, np.int32) or s.ndim != 2 or s.strides[1] != s.itemsize:
            raise ValueError("samples must be a 2-D int16 or int32 array with contiguous rows")
        if s.strides[0] % s.itemsize:
            raise ValueError("the row stride must be a whole number of samples")
        if s.shape[1] < max(block_len, tail_len if n_tail_units else 0):
            raise ValueError(f"rows hold {s.shape[1]} samples, fewer than the block length")
        n_units = s.shape[0]
        b = abi.Batch()
        b.samples = s.ctypes.data
        b.sample_bytes = s.itemsize
        b.sample_bits = sample_bits
        b.unit_stride = s.strides[0] // s.itemsize
        b.n_units = n_units
        b.block_len = block_len
        b.tail_len = tail_len
        b.n_tail_units = n_tail_units
        fp = frame_params(channels, sample_size, params.qlp_precision, first_frame)
        n_frames = n_units // channels if channels else 0
        offsets = np.zeros(n_frames + 1, dtype=np.int64)
        status = np.zeros(max(n_frames, 1), dtype=np.int32)
        upb = max(channels, (units_per_batch // channels) * channels)
        if out is not None:
            if out.dtype != np.uint8 or out.ndim != 1 or not out.flags.c_contiguous:
                raise ValueError("out must be a contiguous 1-D uint8 array")
            capacity = out.size
        cap = capacity or int(n_units * (block_len * s.itemsize * 1.25 + 256)) + (1 << 20)
        given = out
        while True:
            out = given if given is not None else np.empty(cap, dtype=np.uint8)
            t = abi.EncodeTiming()
            rc = self.lib.flacmi_encode_pipeline(self.ctx, C.byref(b), C.byref(params), C.byref(fp), upb,
                                                 out.ctypes.data, cap, offsets.ctypes.data, status.ctypes.data,
                                                 C.byref(t))
            if rc == abi.E_NOMEM and not capacity:
                cap *= 2
                continue
            check(rc, "flacmi_encode_pipeline")
            break
        timing = {f: getattr(t, f) for f, _ in abi.EncodeTiming._fields_}
        return out[:int(offsets[-1])], offsets, status[:n_frames], timing

    def host_register(self, a: np.ndarray) -> None:
        """Page-lock a host array until host_unregister (flacmi_host_register)."""
        check(self.lib.flacmi_host_register(self.ctx, a.ctypes.data, a.nbytes), "flacmi_host_register")

    def host_unregister(self, a: np.ndarray) -> None:
        check(self.lib.flacmi_host_unregister(self.ctx, a.ctypes.data), "flacmi_host_unregister")

    def host_array(self, shape, dtype) -> np.ndarray:
        """A numpy array over page-locked host memory (flacmi_host_alloc), freed with the
        array: staging rows and frame buffers reused call after call without page-locking."""
        dt = np.dtype(dtype)
        count = int(np.prod(shape)) if len(shape) else 1
        nbytes = max(count * dt.itemsize, 1)
        p = self.lib.flacmi_host_alloc(self.ctx, nbytes)
        if not p:
            raise FlacmiError(f"flacmi_host_alloc({nbytes}): {self.lib.flacmi_last_error().decode(errors='replace')}")
        raw = (C.c_uint8 * nbytes).from_address(p)
        # every numpy view of the memory keeps `raw` alive: free with the last view (valid
        # after close() too)
        weakref.finalize(raw, self.lib.flacmi_host_free, None, p)
        return np.frombuffer(raw, dtype=dt, count=count).reshape(shape)

    def frame_sizes_device(self, batch: abi.Batch, fp: abi.FrameParams, meta_ptr: int, params_ptr: int,
                           params_stride: int, offsets_ptr: int, status_ptr: int, stream: int = 0) -> None:
        check(self.lib.flacmi_frame_sizes_device(self.ctx, C.byref(batch), C.byref(fp), meta_ptr, params_ptr,
                                                 params_stride, offsets_ptr, status_ptr, stream),
              "flacmi_frame_sizes_device")

    def pack_frames_device(self, batch: abi.Batch, fp: abi.FrameParams, meta_ptr: int, params_ptr: int,
                           params_stride: int, residual_ptr: int, residual_bytes: int, residual_stride: int,
                           offsets_ptr: int, status_ptr: int, out_ptr: int, capacity: int,
                           stream: int = 0) -> None:
        check(self.lib.flacmi_pack_frames_device(self.ctx, C.byref(batch), C.byref(fp), meta_ptr, params_ptr,
                                                 params_stride, residual_ptr, residual_bytes, residual_stride,
                                                 offsets_ptr, status_ptr, out_ptr, capacity, stream),
              "flacmi_pack_frames_device")

    # ------------------------------------------------------------------------------
    # decoder verifier (include/flacmi.h flacmi_decode_frames_device)
    # ------------------------------------------------------------------------------
    def decode_frames_device(self, data_ptr: int, data_bytes: int, offsets_ptr: int, n_frames: int,
                             dp: abi.DecodeParams, expect: abi.Batch = None, out_ptr: int = 0,
                             out_stride: int = 0, status_ptr: int = 0, mismatch_ptr: int = 0,
                             stream: int = 0) -> None:
        check(self.lib.flacmi_decode_frames_device(self.ctx, data_ptr, data_bytes, offsets_ptr, n_frames,
                                                   C.byref(dp), C.byref(expect) if expect is not None else None,
                                                   out_ptr or None, out_stride, status_ptr, mismatch_ptr, stream),
              "flacmi_decode_frames_device")

    def decode_frames(self, data: np.ndarray, offsets: np.ndarray, channels: int, sample_size: int,
                      first_frame: int = -1, expect: np.ndarray = None, block_len: int = 0, tail_len: int = 0,
                      n_tail_units: int = 0, out_stride: int = 0, check_crc: bool = True):
        """Host bytes in -> (decoded int32 rows [n_frames*channels][out_stride], frame status,
        mismatches per frame), decoded on the device.  `expect` (int16/int32 rows of the
        source units) turns on the in-kernel comparison."""
        import torch
        dev = torch.device("cuda", self.device)
        n_frames = len(offsets) - 1
        nb = int(len(data))
        buf = torch.zeros(((nb + 3) // 4) * 4 + 16, dtype=torch.uint8, device=dev)
        if nb:
            buf[:nb] = torch.from_numpy(np.array(data, dtype=np.uint8, copy=True)).to(dev)
        off = torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int64)).to(dev)
        if out_stride <= 0:
            out_stride = ((max(block_len, 1) + 3) // 4) * 4
        out = torch.zeros((max(n_frames * channels, 1), out_stride), dtype=torch.int32, device=dev)
        st = torch.zeros(max(n_frames, 1), dtype=torch.int32, device=dev)
        mm = torch.zeros(max(n_frames, 1), dtype=torch.int64, device=dev)
        dp = abi.DecodeParams()
        dp.channels, dp.sample_size, dp.first_frame, dp.check_crc = channels, sample_size, first_frame, int(check_crc)
        eb = None
        if expect is not None:
            e = torch.from_numpy(np.ascontiguousarray(expect)).to(dev)
            eb = device_batch(e.data_ptr(), e.element_size(), 16 if e.element_size() == 2 else 32, e.shape[1],
                              e.shape[0], block_len, tail_len, n_tail_units)
        stream = torch.cuda.current_stream(dev).cuda_stream
        self.decode_frames_device(buf.data_ptr(), nb, off.data_ptr(), n_frames, dp, eb, out.data_ptr(), out_stride,
                                  st.data_ptr(), mm.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy(), st.cpu().numpy()[:n_frames], mm.cpu().numpy()[:n_frames]

    def timing(self) -> dict:
        """Average k_lpc / k_resid / whole-call milliseconds over the analyze calls since
        the last timing_reset() (HIP events recorded on each call's stream)."""
        ms = (C.c_float * 4)()
        k = self.lib.flacmi_last_timing(self.ctx, ms, 4)
        if k < 0:
            check(k, "flacmi_last_timing")
        return {"lpc_ms": ms[0], "resid_ms": ms[1], "call_ms": ms[2], "calls": int(ms[3])}

    def timing_reset(self) -> None:
        check(self.lib.flacmi_timing_reset(self.ctx), "flacmi_timing_reset")

    def synth_device(self, dst_ptr: int, sample_bytes: int, sample_bits: int, unit_stride: int,
                     first_unit: int, n_units: int, length: int, seed: int, stream: int = 0,
                     open_eighths: int = 0) -> None:
        """Synthetic units on the device (flacmi_synth_mix_device; open_eighths / 8 of them the
        "open" mix's near-white noise)."""
        done = 0
        while done < n_units:
            k = min(1 << 30, n_units - done)
            check(self.lib.flacmi_synth_mix_device(self.ctx, dst_ptr + done * unit_stride * sample_bytes,
                                                   sample_bytes, sample_bits, unit_stride, first_unit + done,
                                                   k, length, seed, open_eighths, stream), "flacmi_synth_mix_device")
            done += k

    def stream_stats(self, meta_ptr: int, n_units: int, block_len: int, stats_ptr: int,
                     stream: int = 0, tail_len: int = 0, n_tail_units: int = 0) -> None:
        check(self.lib.flacmi_stream_stats(self.ctx, meta_ptr, n_units, block_len, tail_len,
                                           n_tail_units, stats_ptr, stream), "flacmi_stream_stats")


class StatsComm:
    """The cross-GPU stream-statistics reduce of the C-ABI (flacmi_comm_* /
    flacmi_allreduce_stats: RCCL over xGMI), for callers without torch.distributed.  Rank 0
    calls comm_id() and hands the bytes to every rank; every rank builds StatsComm(az,
    nranks, rank, id) (a collective call)."""

    def __init__(self, az: "Analyzer", nranks: int, rank: int, comm_id: bytes):
        if len(comm_id) != abi.COMM_ID_BYTES:
            raise ValueError(f"comm id must be {abi.COMM_ID_BYTES} bytes")
        self.lib = az.lib
        buf = C.create_string_buffer(bytes(comm_id), abi.COMM_ID_BYTES)
        h = C.c_void_p()
        check(self.lib.flacmi_comm_init(az.ctx, nranks, rank, buf, C.byref(h)), "flacmi_comm_init")
        self.comm = h.value

    @staticmethod
    def available(lib) -> None:
        """Raises FlacmiError unless RCCL loads here (no id made: the check every rank runs
        before rank 0's comm_id and the collective init)."""
        check(lib.flacmi_comm_available(), "flacmi_comm_available")

    @staticmethod
    def comm_id(lib) -> bytes:
        buf = C.create_string_buffer(abi.COMM_ID_BYTES)
        check(lib.flacmi_comm_id(buf), "flacmi_comm_id")
        return buf.raw

    def allreduce_stats(self, stats_ptr: int, stream: int = 0) -> None:
        check(self.lib.flacmi_allreduce_stats(self.comm, stats_ptr, stream), "flacmi_allreduce_stats")

    def close(self) -> None:
        if self.comm:
            check(self.lib.flacmi_comm_destroy(self.comm), "flacmi_comm_destroy")
            self.comm = None


def unit_result(out: dict, i: int) -> dict:
    """Per-unit dict view of analyze() results (the keys tests/golden_util.check reads)."""
    m = out["meta"][i]
    r = {name: int(m[name]) for name in abi.META_DTYPE.names if name != "coefs"}
    r["coefs"] = [int(c) for c in m["coefs"][: int(m["ncoefs"])]]
    r["rice_params"] = out["rice_params"][i][: int(m["n_parts"])]
    off, ln = int(m["res_offset"]), int(m["res_len"])
    r["residual"] = out["residual"][i][off: off + ln].astype(np.uint64)
    for k in ("acf", "fixed_sums", "lpc_sums"):
        r[k] = out[k][i] if k in out else None
    r["lpc_record"] = out["lpc_records"][i] if "lpc_records" in out else None
    return r
