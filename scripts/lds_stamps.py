"""Per-phase timing of the LDS-tile parse kernel (D) from its in-kernel stamps.
Needs a tuning build with RTPS_LDS_STAMPS (make variant NAME=stamps VDEFS=-DRTPS_LDS_STAMPS)
selected with RTPS_RX_LIB.  Runs the C3 workload (1M datagrams unless argv[1]) on cuda:0,
the first kernel alone (as bench.py times it), and prints the median / p90 duration of
each phase over the tiles plus the launch's span.

python scripts/lds_stamps.py [n]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch

import rtps_rx
from rtps_rx import lib, _check

OWN = bytes(range(1, 13))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = torch.device("cuda", 0)
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C3, n)
rx = rtps_rx.MessageReceiver(OWN, max_datagrams=n)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_C3, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, rtps_rx.max_records(ln))
rx.set_spec_hint(0)
rx.debug_set_mixed_pass(True)
for _ in range(3):
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.sync()
which = rx.debug_parse_phases(arena, off_t, ln_t, n, outs, 1)
rx.sync()
assert which == 3, f"first kernel {which}, not the LDS tiles"
NS = 24  # STAMP_N of the tuning builds
fn = lib().rtps_rx_debug_lds_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
tiles = min((n + 31) // 32, 1 << 16)
buf = np.zeros(tiles * NS * 4, dtype=np.uint64)  # room for LT >= 8
_check(fn(rx._h, buf.ctypes.data, buf.size))
lt = int(os.environ.get("LT", "32"))
tiles = min((n + lt - 1) // lt, 1 << 16)
st = buf[:tiles * NS].reshape(tiles, NS).astype(np.int64)
ok = (st[:, 7] > 0) & (st[:, 0] > 0)
st = st[ok]
names = ["stage tables", "stage bytes", "count walk", "item walk", "item pass", "look-back", "copy-out"]
print(f"C3 n={n} LT={lt}: {ok.sum()} tiles with stamps (10 ns ticks)")
for k, nm in enumerate(names):
    d = (st[:, k + 1] - st[:, k]) * 10
    d = d[st[:, k + 1] > 0]
    print(f"  {nm:13s} median {np.median(d):8.0f} ns  p90 {np.percentile(d, 90):8.0f} ns  mean {d.mean():8.0f} ns")
tot = (st[:, 7] - st[:, 0]) * 10
print(f"  tile total    median {np.median(tot):8.0f} ns  p90 {np.percentile(tot, 90):8.0f} ns")
span = (st[:, 7].max() - st[:, 0].min()) * 10
print(f"  launch span {span / 1e3:.1f} us; tile starts spread {(st[:, 0].max() - st[:, 0].min()) * 10 / 1e3:.1f} us")
rx.close()
