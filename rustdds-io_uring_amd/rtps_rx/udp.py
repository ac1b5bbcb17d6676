"""UDP batch receive into a datagram arena (rtps_udp_* in include/rtps_rx.h).

Host side of the path's input: the reference's UDPListener + io_uring
RecvMulti on a provided-buffer ring (io_uring/network/udp_listener.rs:101-209)
feeding Domain::handle_event one datagram at a time
(io_uring/rtps/dp_event_loop.rs:190-211).  Here the kernel writes every
datagram into a slot of an arena the caller owns (pinned host memory, so the
GPU parses it in place), and a batch is (offset, length) arrays ready for
MessageReceiver.parse_batch_device.
"""
import ctypes

import numpy as np

from . import lib, _check, ABI_VERSION, _Out, _IngestOut, INGEST_BEST_EFFORT, RtpsRxError

UDP_REUSE = 0x1
UDP_FORCE_RECVMMSG = 0x2
UDP_SQPOLL = 0x4
IO_URING, RECVMMSG, IO_URING_SQPOLL = 1, 2, 3


class _UdpConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("ipv4_addr", ctypes.c_uint32), ("port", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("multicast_group", ctypes.c_uint32), ("arena", ctypes.c_void_p),
                ("slot_bytes", ctypes.c_uint32), ("n_slots", ctypes.c_uint32), ("rcvbuf_bytes", ctypes.c_uint32)]


PUMP_INGEST = 0x1
PUMP_CDR = 0x2


class _PumpBuffers(ctypes.Structure):
    _fields_ = [("out", _Out), ("ingest", _IngestOut), ("rows", ctypes.c_void_p), ("row_status", ctypes.c_void_p)]


class _PumpBatch(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_uint64), ("buffer", ctypes.c_uint32), ("n_datagrams", ctypes.c_uint32),
                ("dgram_off", ctypes.POINTER(ctypes.c_uint64)), ("dgram_len", ctypes.POINTER(ctypes.c_uint32)),
                ("n_records", ctypes.c_uint64), ("n_accepted", ctypes.c_uint64)]


_PUMP_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(_PumpBatch))


class _PumpConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("max_batch", ctypes.c_uint32),
                ("wait_ms", ctypes.c_int32), ("stop_after", ctypes.c_uint64), ("idle_stop_ms", ctypes.c_uint32),
                ("ingest_flags", ctypes.c_uint32), ("cdr_prog", ctypes.c_void_p), ("cdr_n_ops", ctypes.c_uint32),
                ("cdr_row_bytes", ctypes.c_uint32), ("buffers", ctypes.POINTER(_PumpBuffers)),
                ("on_batch", _PUMP_FN), ("user", ctypes.c_void_p), ("stop", ctypes.POINTER(ctypes.c_uint32))]


class PumpStats(ctypes.Structure):
    """rtps_pump_stats: live counters of a running pump (readable from other threads)."""
    _fields_ = [("datagrams", ctypes.c_uint64), ("completed", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("records", ctypes.c_uint64), ("accepted", ctypes.c_uint64), ("truncated", ctypes.c_uint64),
                ("first_ns", ctypes.c_uint64), ("last_ns", ctypes.c_uint64)]


def _bind():
    L = lib()
    if getattr(L, "_udp_bound", False):
        return L
    P, U32, U64, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.rtps_udp_open.argtypes = [ctypes.POINTER(_UdpConfig), ctypes.POINTER(P)]
    L.rtps_udp_open.restype = I
    L.rtps_udp_close.argtypes = [P]
    L.rtps_udp_close.restype = I
    L.rtps_udp_port.argtypes = [P]
    L.rtps_udp_port.restype = I
    L.rtps_udp_backend.argtypes = [P]
    L.rtps_udp_backend.restype = I
    L.rtps_udp_recv_batch.argtypes = [P, P, P, U32, I, P]
    L.rtps_udp_recv_batch.restype = I
    L.rtps_udp_release.argtypes = [P, P, U32]
    L.rtps_udp_release.restype = I
    L.rtps_udp_send_batch.argtypes = [U32, ctypes.c_uint16, P, P, P, U32]
    L.rtps_udp_send_batch.restype = I
    L.rtps_rx_pump.argtypes = [P, P, P, U64, ctypes.POINTER(_PumpConfig), ctypes.POINTER(PumpStats)]
    L.rtps_rx_pump.restype = I
    L._udp_bound = True
    return L


def ipv4(addr):
    a = [int(x) for x in addr.split(".")]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


class UdpReceiver:
    """One bound UDP socket whose datagrams land in the slots of `arena`
    (n_slots x slot_bytes).  arena: a numpy uint8 array or a (pinned) torch
    uint8 tensor on the host; it must outlive the receiver."""

    def __init__(self, arena, slot_bytes=2048, addr="127.0.0.1", port=0, multicast=None, reuse=False,
                 force_recvmmsg=False, sqpoll=True, rcvbuf_bytes=0):
        L = _bind()
        nbytes = arena.nbytes if isinstance(arena, np.ndarray) else arena.numel()
        self.arena = arena
        self.arena_np = arena if isinstance(arena, np.ndarray) else arena.numpy()
        self.slot_bytes = slot_bytes
        self.n_slots = nbytes // slot_bytes
        cfg = _UdpConfig()
        cfg.abi_version = ABI_VERSION
        cfg.ipv4_addr = ipv4(addr)
        cfg.port = port
        cfg.flags = ((UDP_REUSE if reuse else 0) | (UDP_FORCE_RECVMMSG if force_recvmmsg else 0) |
                     (UDP_SQPOLL if sqpoll else 0))
        cfg.multicast_group = ipv4(multicast) if multicast else 0
        cfg.arena = self.arena_np.ctypes.data
        cfg.slot_bytes = slot_bytes
        cfg.n_slots = self.n_slots
        cfg.rcvbuf_bytes = rcvbuf_bytes
        h = ctypes.c_void_p()
        _check(L.rtps_udp_open(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.port = L.rtps_udp_port(h)
        self.backend = L.rtps_udp_backend(h)
        self.truncated = ctypes.c_uint64(0)

    def close(self):
        if getattr(self, "_h", None):
            _bind().rtps_udp_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def recv_batch(self, max_n, timeout_ms=0):
        """-> (off uint64[n], len uint32[n]) of up to max_n datagrams, in arrival order."""
        off = np.empty(max(max_n, 1), dtype=np.uint64)
        ln = np.empty(max(max_n, 1), dtype=np.uint32)
        n = _bind().rtps_udp_recv_batch(self._h, off.ctypes.data, ln.ctypes.data, max_n, timeout_ms,
                                       ctypes.byref(self.truncated))
        _check(min(n, 0))
        return off[:n], ln[:n]

    def release(self, off):
        off = np.ascontiguousarray(off, dtype=np.uint64)
        _check(_bind().rtps_udp_release(self._h, off.ctypes.data if len(off) else None, len(off)))


def send_batch(addr, port, arena, off, ln):
    """sendmmsg of datagrams arena[off[i]:off[i]+len[i]] (the loopback publisher side)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    n = _bind().rtps_udp_send_batch(ipv4(addr), port, arena.ctypes.data, off.ctypes.data, ln.ctypes.data, len(off))
    _check(min(n, 0))
    return n


class PumpBatch:
    """One finished batch handed to a pump callback.  off / len are copies;
    outs / iouts / rows / row_status are the device outputs of the batch (the
    buffer set it was parsed into), valid until the callback returns."""

    def __init__(self, b, bufs):
        self.seq = b.seq
        self.buffer = b.buffer
        self.n_datagrams = b.n_datagrams
        n = b.n_datagrams
        self.off = np.ctypeslib.as_array(b.dgram_off, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
        self.len = np.ctypeslib.as_array(b.dgram_len, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
        self.n_records = b.n_records
        self.n_accepted = b.n_accepted
        self.outs, self.iouts, self.rows, self.row_status = bufs


class Pump:
    """Native receive loop (rtps_rx_pump): UDP arena -> GPU parse -> ingest ->
    CDR decode, two batches in flight, on the calling thread.  The batch form of
    Domain::handle_event's DataRecv arm (io_uring/rtps/dp_event_loop.rs:162-211).

    rx: a MessageReceiver (its match table is used for the ingest);
    rxu: a UdpReceiver whose arena is device-visible (pinned torch tensor)."""

    def __init__(self, rx, rxu, max_batch=16384, ingest=False, sample_type=None, best_effort=False,
                 max_recs=None, n_entries=1):
        if isinstance(rxu.arena, np.ndarray) or not getattr(rxu.arena, "is_pinned", lambda: False)():
            raise RtpsRxError("Pump: the receiver's arena must be a pinned torch tensor (the GPU parses it in place)")
        self.rx, self.rxu = rx, rxu
        cap = max_recs if max_recs is not None else max_batch * max(1, (rxu.slot_bytes - 20) // 4)
        self.cap = cap
        self.sets = []
        arr = (_PumpBuffers * 2)()
        for b in range(2):
            outs = rx.alloc_outputs(max_batch, cap)
            iouts = rx.alloc_ingest_outputs(cap, n_entries) if ingest else None
            rows = rx.alloc_rows(sample_type, cap) if sample_type is not None else (None, None)
            o = arr[b].out
            o.status, o.records, o.max_records = outs["status"].data_ptr(), outs["records"].data_ptr(), cap
            o.target, o.rec_begin, o.n_records = (outs["target"].data_ptr(), outs["rec_begin"].data_ptr(),
                                                  outs["n_records"].data_ptr())
            if ingest:
                g = arr[b].ingest
                g.accept, g.accepted, g.n_accepted = (iouts["accept"].data_ptr(), iouts["accepted"].data_ptr(),
                                                      iouts["n_accepted"].data_ptr())
                g.max_accepted = iouts["max_accepted"]
                g.ack_base, g.n_window_overflow = iouts["ack_base"].data_ptr(), iouts["n_window_overflow"].data_ptr()
            if sample_type is not None:
                arr[b].rows, arr[b].row_status = rows[0].data_ptr(), rows[1].data_ptr()
            self.sets.append((outs, iouts, rows[0], rows[1]))
        self._bufs = arr
        self._ops = sample_type.ops if sample_type is not None else None
        cfg = _PumpConfig()
        cfg.abi_version = ABI_VERSION
        cfg.flags = (PUMP_INGEST if ingest else 0) | (PUMP_CDR if sample_type is not None else 0)
        cfg.max_batch = max_batch
        cfg.ingest_flags = INGEST_BEST_EFFORT if best_effort else 0
        if sample_type is not None:
            cfg.cdr_prog = self._ops.ctypes.data
            cfg.cdr_n_ops = len(self._ops)
            cfg.cdr_row_bytes = sample_type.row_bytes
        cfg.buffers = ctypes.cast(arr, ctypes.POINTER(_PumpBuffers))
        self._cfg = cfg
        self._stop = ctypes.c_uint32(0)
        cfg.stop = ctypes.pointer(self._stop)
        self.stats = PumpStats()
        self._error = None

    def stop(self):
        """Ask a running pump (on another thread) to return after its current batch."""
        self._stop.value = 1

    def run(self, wait_ms=5, stop_after=0, idle_stop_ms=0, on_batch=None):
        """Run until stop_after datagrams, idle_stop_ms without traffic, stop(), or
        on_batch returning True.  on_batch(PumpBatch) runs on this thread after the
        batch's GPU work finished.  Returns a copy of the final PumpStats
        (self.stats is the live one, for other threads)."""
        self._stop.value = 0
        cfg = self._cfg
        cfg.wait_ms, cfg.stop_after, cfg.idle_stop_ms = wait_ms, stop_after, idle_stop_ms

        def tramp(_user, bp):
            try:
                return 1 if on_batch(PumpBatch(bp.contents, self.sets[bp.contents.buffer])) else 0
            except BaseException as e:  # surfaced after the loop returns
                self._error = e
                return 1

        cfg.on_batch = _PUMP_FN(tramp) if on_batch is not None else _PUMP_FN()
        self._tramp = cfg.on_batch
        self._error = None
        arena = self.rxu.arena
        rc = _bind().rtps_rx_pump(self.rx._h, self.rxu._h, arena.data_ptr(), arena.numel(), ctypes.byref(cfg),
                                  ctypes.byref(self.stats))
        if self._error is not None:
            raise self._error
        _check(rc)
        return PumpStats.from_buffer_copy(self.stats)
