"""Zero-copy parse (the kernel reads datagram heads from pinned host memory and writes status /
records to pinned host memory) with the host buffers allocated three ways: torch pin_memory (what
bench.py's e2e leg uses), hipHostMalloc default (coherent) and hipHostMalloc NonCoherent (the GPU
may cache the lines in L2, so the four 16-B head loads of a datagram share one PCIe read)."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
FLAGS = {"hip_default": 0x0, "hip_coherent": 0x40000000, "hip_noncoherent": 0x80000000}
dev = torch.device("cuda", 0)
wl_name = sys.argv[1] if len(sys.argv) > 1 else "T"
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(rtps_rx.WORKLOADS[wl_name], n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WORKLOADS[wl_name], arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, 4 * n)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
torch.cuda.synchronize()
m = int(outs["n_records"].item())
ref_s, ref_r = outs["status"][:n].cpu(), outs["records"][:m].cpu()


def host_tensor(nbytes, how, dtype=torch.uint8):
    if how == "torch_pinned":
        return torch.empty(nbytes // torch.tensor([], dtype=dtype).element_size(), dtype=dtype, pin_memory=True), None
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), nbytes, FLAGS[how]) == 0
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    return torch.frombuffer(buf, dtype=dtype), p


for how in ("torch_pinned", "hip_default", "hip_coherent", "hip_noncoherent"):
    keep = []
    ha, p = host_tensor(size, how); keep.append(p)
    ha.copy_(arena.cpu())
    ho, p = host_tensor(n * 8, how, torch.int64); keep.append(p); ho.copy_(off_t.cpu())
    hl, p = host_tensor(n * 4, how, torch.int32); keep.append(p); hl.copy_(ln_t.cpu())
    hs, p = host_tensor(n, how); keep.append(p)
    hr, p = host_tensor(m * 64, how); keep.append(p)
    ht, p = host_tensor(m * 4, how, torch.int32); keep.append(p)
    hb, p = host_tensor(n * 4, how, torch.int32); keep.append(p)
    hn, p = host_tensor(8, how, torch.int64); keep.append(p)
    h_outs = {"status": hs, "records": hr.view(m, 64), "target": ht, "rec_begin": hb, "n_records": hn,
              "max_records": m}
    ts = []
    for _ in range(6):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        rx.parse_batch_device(ha, ho, hl, n, h_outs)
        e1.record(st); e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ok = torch.equal(hs, ref_s) and torch.equal(hr.view(m, 64), ref_r)
    print(f"{wl_name} {how:16s} best {min(ts[1:]):7.3f} ms  {n / (min(ts[1:]) * 1e-3) / 1e6:7.1f} M datagrams/s  "
          f"parity {ok}", flush=True)
    del ha, ho, hl, hs, hr, ht, hb, hn, h_outs
    torch.cuda.synchronize()
    for p in keep:
        if p is not None: hip.hipHostFree(p)
rx.close()
