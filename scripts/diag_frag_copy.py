"""Copy ceilings for the DataFrag reassembly's traffic shape (C4: 1M datagrams, 1344 payload
bytes at datagram offset 56 -> contiguous heap rows), by element width, loads in flight and
store policy, at source offsets 48 (16-B aligned), 52 (4-B) and 56 (8-B: the real one)."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
D = ctypes.CDLL(os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so"))
D.diag_copy_w.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
dev = torch.device("cuda", 0)
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C4, n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st)
arena = torch.zeros(size + 4096, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
rows = torch.empty(n * 1344, dtype=torch.uint8, device=dev)
def timeit(fn, reps=20):
    for _ in range(3): fn()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps): fn()
    e1.record(st); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
res = {"memcpy_d2d": timeit(lambda: rows.copy_(arena[:n * 1344]))}
for skip in (48, 52, 56):
    for w, u, nt in ((16, 1, 0), (16, 2, 0), (16, 1, 1), (16, 2, 1), (8, 1, 1), (8, 2, 1), (8, 3, 1), (4, 3, 1), (4, 6, 1)):
        for blocks in (4096, 8192):
            rc = []
            t = timeit(lambda: rc.append(D.diag_copy_w(w, u, nt, arena.data_ptr(), off_t.data_ptr(), n, rows.data_ptr(),
                                                       1344, skip, blocks, ctypes.c_void_p(st.cuda_stream))))
            assert set(rc) == {0}, rc
            res[f"s{skip}_w{w}_u{u}_nt{nt}_b{blocks}"] = t
for k, v in res.items():
    print(f"{k:28s} {v:8.1f} us  {2 * n * 1344 / (v * 1e-6) / 1e9:7.0f} GB/s (2 x 1344 B per datagram)", flush=True)
