"""End-to-end variants for host-resident datagrams (T, 1M x 1 KiB):
 (i)   pinned H2D of the whole arena + parse + D2H of status/records
 (ii)  zero-copy: kernel reads datagram heads from pinned host memory; outputs in HBM + D2H
 (iii) zero-copy in and out: outputs written straight to pinned host memory
Every variant's outputs are checked against the device-resident parse."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
wlname = sys.argv[1] if len(sys.argv) > 1 else "T"
wl = rtps_rx.WORKLOADS[wlname]
n = 1 << 20
dev = torch.device("cuda", 0)
off, ln, size = rtps_rx.gen_layout(wl, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n)
probe = rx.alloc_outputs(n, 1); rx.parse_batch_device(arena, off_t, ln_t, n, probe); torch.cuda.synchronize()
nrec = int(probe["n_records"].item())
ref = rx.alloc_outputs(n, nrec); rx.parse_batch_device(arena, off_t, ln_t, n, ref); torch.cuda.synchronize()
ref_recs = ref["records"][:nrec].cpu(); ref_status = ref["status"][:n].cpu()
h_arena = torch.empty(size, dtype=torch.uint8, pin_memory=True); h_arena.copy_(arena)
h_off = torch.empty(n, dtype=torch.int64, pin_memory=True); h_off.copy_(off_t)
h_ln = torch.empty(n, dtype=torch.int32, pin_memory=True); h_ln.copy_(ln_t)
h_status = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h_recs = torch.empty((nrec, 64), dtype=torch.uint8, pin_memory=True)
outs = rx.alloc_outputs(n, nrec)
h_outs = {"status": h_status, "records": h_recs, "match": torch.empty(nrec, dtype=torch.int16, pin_memory=True),
          "rec_begin": torch.empty(n, dtype=torch.int32, pin_memory=True),
          "n_records": torch.zeros(1, dtype=torch.int64, pin_memory=True), "max_records": nrec}
torch.cuda.synchronize()

def v1():
    arena.copy_(h_arena, non_blocking=True)
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
    h_status.copy_(outs["status"][:n], non_blocking=True); h_recs.copy_(outs["records"][:nrec], non_blocking=True)
def v2():
    rx.parse_batch_device(h_arena, h_off, h_ln, n, outs)
    h_status.copy_(outs["status"][:n], non_blocking=True); h_recs.copy_(outs["records"][:nrec], non_blocking=True)
def v3():
    rx.parse_batch_device(h_arena, h_off, h_ln, n, h_outs)
def v4():  # parse only (device resident) for reference
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
for name, fn in (("full H2D+parse+D2H", v1), ("zero-copy in, D2H out", v2), ("zero-copy in+out", v3),
                 ("device-resident parse", v4)):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st); fn(); e1.record(st); e1.synchronize(); ts.append(e0.elapsed_time(e1))
    ok = torch.equal(h_status if fn is not v4 else outs["status"][:n].cpu(), ref_status) and \
        torch.equal(h_recs if fn is not v4 else outs["records"][:nrec].cpu(), ref_recs)
    print(f"{wlname} {name:24s} {min(ts):8.3f} ms  {n / min(ts) * 1e3 / 1e6:9.1f} M datagrams/s  {'OK' if ok else 'MISMATCH'}")
