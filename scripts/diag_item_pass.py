"""Diagnostic (needs the itemdiag variant: `make variant NAME=itemdiag VDEFS=-DRTPS_ITEM_DIAG`):
on C3 (1M datagrams, every writer subscribed as bench.py does), the chained parse's time against a
record-parallel write pass that already knows every record's (datagram, submessage offset), i.e.
the second half of a chained kernel whose count walk left those items behind.  Checks that the
pass rebuilds the parse's records and target sets bit-exactly, then times both store forms."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
from rtps_rx import lib, _check
from rtps_rx.records import RECORD_DTYPE, MATCH_DTYPE

n = 1 << 20
wl = rtps_rx.WORKLOADS["C3"]
dev = torch.device("cuda", 0)
off, ln, size = rtps_rx.gen_layout(wl, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, 4 * n)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
torch.cuda.synchronize()
m = int(outs["n_records"].item())
r = outs["records"][:m].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
wk = np.isin(r["kind"], [0x15, 0x16, 0x07, 0x13, 0x08])  # writer kinds, as bench.py subscribes
g = np.concatenate([r["prefix"][wk], r["writer_id"][wk]], axis=1)
guids = np.unique(g.view(np.dtype((np.void, 16))).reshape(-1))
tbl = np.zeros(len(guids), dtype=MATCH_DTYPE)
tbl["writer_guid"] = np.frombuffer(guids.tobytes(), dtype=np.uint8).reshape(-1, 16)
rx.set_match_table(tbl)
for _ in range(3):
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
torch.cuda.synchronize()
m = int(outs["n_records"].item())
print("records", m, "writers", len(guids), flush=True)

fn = lib().rtps_rx_debug_item_pass
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
               ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(rtps_rx._Out), ctypes.c_uint32]
fn.restype = ctypes.c_int
outs2 = rx.alloc_outputs(n, 4 * n)
o2 = rtps_rx._Out()
o2.status = outs2["status"].data_ptr(); o2.records = outs2["records"].data_ptr(); o2.max_records = outs2["max_records"]
o2.target = outs2["target"].data_ptr(); o2.rec_begin = None; o2.n_records = outs2["n_records"].data_ptr()


def item(mode):
    _check(fn(rx._h, arena.data_ptr(), arena.numel(), off_t.data_ptr(), ln_t.data_ptr(), n,
              outs["records"].data_ptr(), m, ctypes.byref(o2), mode))


def timeit(f, reps=20):
    for _ in range(3): f()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps): f()
    e1.record(st); e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for mode in (0, 1):
    outs2["records"].zero_()
    item(mode)
    torch.cuda.synchronize()
    same = torch.equal(outs2["records"][:m], outs["records"][:m])
    same_t = torch.equal(outs2["target"][:m], outs["target"][:m])
    bad = int((outs2["records"][:m] != outs["records"][:m]).any(dim=1).sum().item())
    print(f"mode {mode}: records equal {same} ({bad} differ), targets equal {same_t}", flush=True)
for rep in range(2):
    tp = timeit(lambda: rx.parse_batch_device(arena, off_t, ln_t, n, outs))
    t0 = timeit(lambda: item(0))
    t1 = timeit(lambda: item(1))
    print(f"parse step {tp:7.1f} us   item pass: per-lane stores {t0:7.1f} us, LDS-transposed stores {t1:7.1f} us",
          flush=True)
# ablations (wrong output, timing only): 2 no per-kind reader, 4 no classification, 8 no record stores
for mode, what in ((1 | 2, "no per-kind reader"), (1 | 4, "no classification"), (8, "no record stores"),
                   (2 | 4 | 8, "window + interpreter loads only")):
    print(f"ablation {what:32s} {timeit(lambda: item(mode)):7.1f} us", flush=True)
rx.close()
