"""Copy ceilings for the CDR decode's traffic shape (T: 976 B per datagram -> 976-B rows)
next to the decode kernel itself and a plain device-to-device memcpy of the same bytes."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
from rtps_rx import cdr
D = ctypes.CDLL(os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so"))
D.diag_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
dev = torch.device("cuda", 0)
n = 1 << 20
wl = rtps_rx.WL_T
off, ln, size = rtps_rx.gen_layout(wl, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, n)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
t = cdr.TSample
rows, rst = rx.alloc_rows(t, n)
dst = torch.empty(n * 976, dtype=torch.uint8, device=dev)
def timeit(fn, reps=20):
    for _ in range(3): fn()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps): fn()
    e1.record(st); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
res = {"decode": timeit(lambda: rx.cdr_decode(t, arena, off_t, outs, rows, rst)),
       "memcpy_d2d_976MB": timeit(lambda: dst.copy_(arena[:n * 976]))}
for blocks in (1024, 2048, 4096, 8192):
    for mode, name in ((0, "wave"), (1, "flat")):
        res[f"copy_{name}_b{blocks}"] = timeit(lambda: D.diag_copy(mode, arena.data_ptr(), off_t.data_ptr(), n,
                                                                    rows.data_ptr(), 976, 48, blocks,
                                                                    ctypes.c_void_p(st.cuda_stream)))
for k, v in res.items():
    print(f"{k:24s} {v:8.1f} us  {2 * n * 976 / (v * 1e-6) / 1e9:7.0f} GB/s (2 x 976 B per datagram)")
