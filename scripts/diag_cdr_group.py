"""Copy ceilings for the T CDR decode's traffic shape (1M x 976 value bytes at datagram offset 48 ->
976-B rows): one wave per row (the decode's segment copy) against R rows per wave as one flat chunk
list (diag copy_group), beside the decode itself (bench.py's cdr leg)."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
D = ctypes.CDLL(os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so"))
D.diag_copy_w.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                          ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
D.diag_copy_group.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
dev = torch.device("cuda", 0)
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_T, n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st)
arena = torch.randint(0, 255, (size + 4096,), dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
rows = torch.empty(n * 976, dtype=torch.uint8, device=dev)


def timeit(fn, reps=20):
    for _ in range(3): fn()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps): fn()
    e1.record(st); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


s = st.cuda_stream
res = {}
for blocks in (4096, 8192):
    for nt in (0, 1):
        rc = []
        res[f"wave_w16_u1_nt{nt}_b{blocks}"] = timeit(lambda: rc.append(D.diag_copy_w(
            16, 1, nt, arena.data_ptr(), off_t.data_ptr(), n, rows.data_ptr(), 976, 48, blocks, ctypes.c_void_p(s))))
        assert set(rc) == {0}, rc
    for r, nt in ((2, 1), (3, 1), (4, 1), (3, 0)):
        rc = []
        res[f"group_r{r}_nt{nt}_b{blocks}"] = timeit(lambda: rc.append(D.diag_copy_group(
            r, nt, arena.data_ptr(), off_t.data_ptr(), n, rows.data_ptr(), 976, 48, blocks, ctypes.c_void_p(s))))
        assert set(rc) == {0}, rc
for k, v in res.items():
    print(f"{k:28s} {v:8.1f} us  {2 * n * 976 / (v * 1e-6) / 1e9:7.0f} GB/s (2 x 976 B per row)", flush=True)
