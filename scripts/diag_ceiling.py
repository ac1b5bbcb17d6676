"""Time the traffic-shape ceiling kernels vs the real parse on the same T / C2 arena."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
D = ctypes.CDLL(os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so"))
D.diag_ceiling.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
dev = torch.device("cuda", 0)
for wlname in (sys.argv[1:] or ["T", "C2"]):
    wl = rtps_rx.WORKLOADS[wlname]
    n = 1 << 20
    off, ln, size = rtps_rx.gen_layout(wl, n)
    rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
    st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
    arena = torch.empty(size, dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.generate(wl, arena, off_t, ln_t, n)
    outs = rx.alloc_outputs(n, n)
    rec = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev); rb = torch.empty(n, dtype=torch.int32, device=dev)
    def run(mode):
        if mode < 0:
            rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        else:
            D.diag_ceiling(mode, arena.data_ptr(), off_t.data_ptr(), ln_t.data_ptr(), n, rec.data_ptr(),
                           status.data_ptr(), rb.data_ptr(), ctypes.c_void_p(st.cuda_stream))
    res = {}
    for rep in range(3):
        for mode in (-1, 0, 1, 2, 3):
            for _ in range(3): run(mode)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20): run(mode)
            e1.record(st); e1.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 20 * 1e3)
    names = {-1: "parse(A+S+B)", 0: "read+write", 1: "read only", 2: "write only", 3: "read+write(LDS transpose)"}
    for mode, v in res.items():
        print(f"{wlname} {names[mode]:28s} {min(v):7.1f} us")
    rx.close()
