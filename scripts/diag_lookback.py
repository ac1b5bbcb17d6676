"""Diagnostic: look-back polls/spins per tile for a T batch (needs the RTPS_DIAG build)."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch, rtps_rx
wl = rtps_rx.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "T"]
n = 1 << 20
off, ln, size = rtps_rx.gen_layout(wl, n)
rx = rtps_rx.MessageReceiver(bytes.fromhex("0103000c292d31a228200208"), max_datagrams=n)
dev = torch.device("cuda", 0)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev); ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n); rx.sync()
outs = rx.alloc_outputs(n, 4 * n)
L = rtps_rx.lib(); L.rtps_rx_debug_scratch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
for rep in range(3):
    rx.parse_batch_device(arena, off_t, ln_t, n, outs); rx.sync()
    h = np.zeros(4, dtype=np.uint64); L.rtps_rx_debug_scratch(rx._h, h.ctypes.data, 4)
    tiles = (n + 255) // 256
    print(f"tickets={h[0]} timeouts={h[1]} polls={h[2]} ({h[2]/tiles:.2f}/tile) spins={h[3]} ({h[3]/tiles:.2f}/tile)")
