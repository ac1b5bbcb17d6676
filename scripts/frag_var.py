"""Run-to-run spread of the C4 reassembly step (1M fragments): several fresh heap
allocations in one process, 10 timed steps each (mean / min / max, ms), and the
span copy's share from a second pass of the same shape (diag copy ceiling)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
dev = torch.device("cuda", 0)
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C4, n)
rx = rtps_rx.MessageReceiver(bytes(range(1, 13)), max_datagrams=n)
st = torch.cuda.Stream(dev); torch.cuda.set_stream(st); rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_C4, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, n)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
keep = []
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    if trial % 2:  # shift the next heap's placement
        keep.append(torch.empty(int(np.random.default_rng(trial).integers(1, 64)) << 21, dtype=torch.uint8, device=dev))
    fouts = rx.alloc_frag_outputs(n, size + 16 * n + (1 << 24))
    for _ in range(2):
        rx.frag_reset(); rx.frag_assemble(arena, off_t, outs, fouts)
    ts = []
    for _ in range(10):
        rx.frag_reset()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(st); rx.frag_assemble(arena, off_t, outs, fouts); b.record(st); b.synchronize()
        ts.append(a.elapsed_time(b))
    print(f"trial {trial}: heap at {fouts['heap'].data_ptr() & ((1 << 30) - 1):#x}  mean {np.mean(ts):.3f}  "
          f"min {np.min(ts):.3f}  max {np.max(ts):.3f} ms", flush=True)
    del fouts
rx.close()
