"""Composite-program CDR decode timing (lane-per-row kernel, cdr_nested_kernel):
clean little-endian samples of tests/cdr_ref.py's POLYGON and NESTED types, 8 copies
of 65,536 distinct datagrams, parsed once on the GPU, then rtps_rx_cdr_decode timed
with HIP events on the receiver's stream.  Checks a sample of rows against the oracle.
--ascii: strings of ASCII characters only.
Algorithmic bytes per decoded row: 40 B of the record + the value bytes + row_bytes
+ 1 status byte."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import cdr_ref  # noqa: E402
import oracle  # noqa: E402
import rtps_rx  # noqa: E402

dev = torch.device("cuda", 0)
if "--ascii" in sys.argv:  # ASCII-only strings (the default alphabet has 2-4-byte UTF-8 characters)
    cdr_ref.random_values.__defaults__ = (("a", "Z", "0", " ", "q"),)
for name, t in (("polygon", cdr_ref.POLYGON), ("nested", cdr_ref.NESTED)):
    base = cdr_ref.corpus(t, 65536, seed=11, le_only=True, clean=True)
    dgrams = base * 8
    arena, off, ln = oracle.pack(dgrams)
    n = len(dgrams)
    rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=n)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    rx.set_stream(st)
    a_t = torch.from_numpy(arena).to(dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    outs = rx.alloc_outputs(n, n)
    rx.parse_batch_device(a_t, off_t, ln_t, n, outs)
    torch.cuda.synchronize()
    nrec = int(outs["n_records"].item())
    rows, rst = rx.alloc_rows(t, nrec)
    rx.cdr_decode(t, a_t, off_t, outs, rows, rst)
    torch.cuda.synchronize()
    # oracle check on the first 65,536 records (the distinct ones)
    _, o_recs, _, _ = oracle.parse(arena, off, ln, threads=8)
    m = 65536
    o_rows, o_status = oracle.cdr_decode(t, arena, off, o_recs[:m])
    g_rows = rows[:m].cpu().numpy()
    g_st = rst[:m].cpu().numpy()
    assert np.array_equal(g_st, o_status) and np.array_equal(g_rows, o_rows), name
    ok = int((rst[:nrec] == 0).sum().item())
    vbytes = sum(int.from_bytes(r["u"].tobytes()[2:4], "little") - 4 for r in o_recs[:m])
    vbytes *= nrec // m
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        rx.cdr_decode(t, a_t, off_t, outs, rows, rst)
    e0.record(st)
    for _ in range(reps):
        rx.cdr_decode(t, a_t, off_t, outs, rows, rst)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    algo = nrec * (40 + t.row_bytes + 1) + vbytes
    print(f"{name}: {nrec} rows ({ok} OK), row_bytes {t.row_bytes}, value bytes {vbytes / nrec:.1f}/row, "
          f"{ms * 1e3:.1f} us per decode, {nrec / ms / 1e6:.2f} G rows/s, {algo / ms / 1e9:.3f} TB/s algorithmic "
          f"({algo / ms / 1e9 / 8.0:.3f} of 8 TB/s)", flush=True)
    rx.close()
