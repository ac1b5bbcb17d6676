"""Variants of the read-head + write-record ceiling on the T arena: head bytes,
non-temporal loads/stores, datagrams per lane (memory-level parallelism)."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
D = ctypes.CDLL(os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so"))
D.diag_ceiling_var.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
D.diag_ceiling.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
dev = torch.device("cuda", 0)
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_T, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_T, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, n)
rec = torch.empty((n, 64), dtype=torch.uint8, device=dev)
status = torch.empty(n, dtype=torch.uint8, device=dev); rb = torch.empty(n, dtype=torch.int32, device=dev)
variants = [(64, 0, 0, 1), (48, 0, 0, 1), (32, 0, 0, 1), (64, 1, 0, 1), (64, 0, 1, 1), (64, 1, 1, 1), (48, 1, 1, 1),
            (64, 0, 0, 2), (64, 0, 0, 4), (48, 0, 1, 2), (64, 1, 1, 2)]


def run(v):
    if v == "parse":
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
    else:
        rc = D.diag_ceiling_var(*v, arena.data_ptr(), off_t.data_ptr(), ln_t.data_ptr(), n, rec.data_ptr(),
                                status.data_ptr(), rb.data_ptr(), ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, (v, rc)


res = {}
for rep in range(3):
    for v in ["parse"] + variants:
        for _ in range(3): run(v)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20): run(v)
        e1.record(st); e1.synchronize()
        res.setdefault(v, []).append(e0.elapsed_time(e1) / 20 * 1e3)
for v, t in res.items():
    name = v if v == "parse" else "head %dB ntl=%d nts=%d per_lane=%d" % v
    print(f"T {name:36s} {min(t):7.1f} us")
rx.close()
