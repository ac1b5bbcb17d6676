"""Phase timing of the item pass's record pass W (rtps_parse_emit_kernel) on C3 (1M datagrams,
the bench's reader table), from a tuning build with RTPS_EM_STAMPS selected by RTPS_RX_LIB:
  make variant NAME=emst VDEFS=-DRTPS_EM_STAMPS      (rustdds-io_uring_amd/csrc)
Per tile: thread 0's phase ends (its own item's marks wait for their loads) and every wave's end.
Prints mean phase times, the tile's life (start to its last wave's end), the launch's span and the
mean number of tiles in flight."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch

import rtps_rx
from rtps_rx import lib, _check
from rtps_rx.records import RECORD_DTYPE, MATCH_DTYPE, DATA, DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = torch.device("cuda", 0)
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C3, n)
rx = rtps_rx.MessageReceiver(bytes(range(1, 13)), max_datagrams=n)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_C3, arena, off_t, ln_t, n)
outs = rx.alloc_outputs(n, rtps_rx.max_records(ln))
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.sync()
n_rec = int(outs["n_records"].item())
r = outs["records"][:n_rec].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
wk = np.isin(r["kind"], [DATA, DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP])
g = np.concatenate([r["prefix"][wk], r["writer_id"][wk]], axis=1)
guids = np.unique(g.view(np.dtype((np.void, 16))).reshape(-1))
tbl = np.zeros(len(guids), dtype=MATCH_DTYPE)
tbl["writer_guid"] = np.frombuffer(guids.tobytes(), dtype=np.uint8).reshape(-1, 16)
rx.set_match_table(tbl)
for _ in range(3):
    rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.sync()
NS = 24
tiles = (n + 255) // 256
buf = np.zeros(tiles * NS, dtype=np.uint64)
fn = lib().rtps_rx_debug_lds_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
_check(fn(rx._h, buf.ctypes.data, buf.size))
st = buf.reshape(-1, NS).astype(np.float64) * 0.01  # 100 MHz ticks -> us
t0 = st[:, 0].min()
st -= t0
names = ["stage + loads", "barrier 1", "scan, barriers", "item + window", "src prefix",
         "sub_body", "rec_finish"]
print(f"C3 n={n}: {n_rec} records, {tiles} tiles, {len(guids)} writer GUIDs")
for k, nm in enumerate(names):
    d = st[:, k + 1] - st[:, k]
    print(f"  {nm:15s} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")
wend = st[:, 8:24]
last = wend.max(1)
print(f"  thread 0's item to its wave's end: mean {(wend[:, 0] - st[:, 7]).mean():.2f} us")
print(f"  waves' ends after the loop start: mean {(wend - st[:, 3:4]).mean():.2f}, "
      f"last wave {(last - st[:, 3]).mean():.2f} us")
life = last - st[:, 0]
span = last.max()
print(f"  tile life mean {life.mean():.2f} us; launch span {span:.1f} us; mean tiles in flight {life.sum() / span:.0f}")
rx.close()
