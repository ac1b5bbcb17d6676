"""Diagnostic: where the gap between bench.py's wall time per step and the
parse's event time goes (T, 1M datagrams).

Measures, on the parse stream:
  host   - host time per rtps_rx_parse_batch call, queue kept full (no sync)
  ev     - wall per step with two events recorded around every step (bench.py's loop)
  noev   - wall per step with no events inside the loop
  ev2    - wall per step with events around the whole loop only (total / K)
"""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx

n = 1 << 20
wl = rtps_rx.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "T"]
K = 200
dev = torch.device("cuda", 0)
off, ln, size = rtps_rx.gen_layout(wl, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
rx.set_stream(stream)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, 4 * n)
if "match" in sys.argv[2:]:  # subscribe to every writer of the batch, as bench.py does
    from rtps_rx.records import RECORD_DTYPE, MATCH_DTYPE
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
    torch.cuda.synchronize()
    r = outs["records"][:n].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
    g = np.concatenate([r["prefix"], r["writer_id"]], axis=1)
    guids = np.unique(g.view(np.dtype((np.void, 16))).reshape(-1))
    tbl = np.zeros(len(guids), dtype=MATCH_DTYPE)
    tbl["writer_guid"] = np.frombuffer(guids.tobytes(), dtype=np.uint8).reshape(-1, 16)
    rx.set_match_table(tbl)
    print("match table:", len(guids), "writers")
for _ in range(20):
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
torch.cuda.synchronize()


def run(mode):
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    ends = [torch.cuda.Event(enable_timing=(mode != "evnt")) for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == "ev2":
        starts[0].record(stream)
    for k in range(K):
        if mode == "ev":
            starts[k].record(stream)
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        if mode in ("ev", "evnt"):
            ends[k].record(stream)
    th = time.perf_counter() - t0
    if mode == "ev2":
        ends[0].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev = None
    if mode == "ev":
        ev = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)])) * 1e3
    elif mode == "ev2":
        ev = starts[0].elapsed_time(ends[0]) / K * 1e3
    return th / K * 1e6, wall / K * 1e6, ev


for rep in range(2):
    for mode in ("ev", "noev", "ev2", "evnt"):
        h, w, e = run(mode)
        print(f"{mode:5s} host/call {h:6.1f} us  wall/step {w:6.1f} us  event/step {e if e is None else round(e, 1)} us",
              flush=True)
rx.close()
