"""Debug: the 70-reader frag + ingest case alone, with memory and count diagnostics."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "rustdds-io_uring_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import oracle, frag_ref, rtps_rx
from rtps_rx.records import Readers, max_records
dev = torch.device("cuda", 0)
rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 21)
print("mem before", torch.cuda.mem_get_info(), flush=True)
n_r = 70
slots = [100 + k for k in range(n_r)]
readers = [(bytes([0, 0, 1 + k, 0x07]), slots[k], 0) for k in range(n_r)]
g1 = frag_ref.RS_PREFIX[0] + frag_ref.RS_WRITER[0]
g2 = frag_ref.RS_PREFIX[1] + frag_ref.RS_WRITER[1]
rd = Readers(readers, [(g1, k) for k in range(n_r)] + [(g2, k) for k in range(0, n_r, 3)])
rx.set_readers(rd)
dgrams = frag_ref.reader_scenario(300, 5, 1, 64)
arena, off, ln = oracle.pack(dgrams, align=4)
A = torch.from_numpy(arena).to(dev); O = torch.from_numpy(off.view(np.int64)).to(dev); L = torch.from_numpy(ln.view(np.int32)).to(dev)
cap = max_records(ln)
print("cap", cap, "arena", len(arena), "proxies", rd.n_proxies, flush=True)
outs = rx.alloc_outputs(len(ln), cap)
fouts = rx.alloc_frag_outputs(80 * cap, 80 * len(arena) + (1 << 20))
iouts = rx.alloc_ingest_outputs(cap, rd.n_proxies)
rx.parse_batch_device(A, O, L, len(ln), outs)
rx.frag_assemble(A, O, outs, fouts)
rx.sync()
print("n_records", int(outs["n_records"].item()), "n_samples", int(fouts["n_samples"].item()), flush=True)
print("mem mid", torch.cuda.mem_get_info(), flush=True)
for path in (0, 1, 2):
    rx.debug_ingest_path(path)
    try:
        rx.ingest(A, O, outs, iouts, fouts)
        rx.sync()
        print("path", path, "ok: accepted", int(iouts["n_accepted"].item()), flush=True)
    except Exception as ex:
        print("path", path, "FAILED", ex, flush=True)
    rx.ingest_reset()
try:
    rx.debug_ingest_path(0)
    rx.ingest(A, O, outs, iouts)  # without the frag samples
    rx.sync()
    print("no-frag ok", int(iouts["n_accepted"].item()), flush=True)
except Exception as ex:
    print("no-frag FAILED", ex, flush=True)
