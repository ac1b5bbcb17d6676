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

from . import lib, _check, ABI_VERSION

UDP_REUSE = 0x1
UDP_FORCE_RECVMMSG = 0x2
UDP_SQPOLL = 0x4
IO_URING, RECVMMSG, IO_URING_SQPOLL = 1, 2, 3


class _UdpConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("ipv4_addr", ctypes.c_uint32), ("port", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("multicast_group", ctypes.c_uint32), ("arena", ctypes.c_void_p),
                ("slot_bytes", ctypes.c_uint32), ("n_slots", ctypes.c_uint32), ("rcvbuf_bytes", ctypes.c_uint32)]


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
