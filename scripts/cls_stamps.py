"""Phase timing of the ingest's bucketing classify (k_classify, BUCKET) on C3 (1M datagrams),
from a tuning build with RTPS_CLS_STAMPS selected by RTPS_RX_LIB:
  make variant NAME=cstamps VDEFS="-DRTPS_CLS_STAMPS [-DRTPS_PB_CHR=...]"   (rustdds-io_uring_amd/csrc)
Wave 0 of every workgroup stamps the end of each phase (absolute 100 MHz ticks).  Prints the mean
per-workgroup phase times, the kernel's span and the mean number of workgroups in flight.
env CHR: the build's record slots per workgroup (default 1024)."""
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
chr_ = int(os.environ.get("CHR", "1024"))
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
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
outs["max_records"] = n_rec  # as bench.py sizes the ingest: the batch's records
iouts = rx.alloc_ingest_outputs(n_rec, len(guids))
for _ in range(3):
    rx.ingest_reset()
    rx.ingest(arena, off_t, outs, iouts)
rx.sync()
nblk = (n_rec + chr_ - 1) // chr_
buf = np.zeros(nblk * 16, dtype=np.uint64)
fn = lib().rtps_rx_debug_proxy_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
_check(fn(rx._h, buf.ctypes.data, buf.size))
allst = buf.reshape(-1, 16).astype(np.float64) * 0.01  # 100 MHz ticks -> us
st = allst[:, :7].copy()
ss = allst[:, 8:12]  # in-step phase sums (builds whose steps wait at each mark)
t0 = st[:, 0].min()
st -= t0
names = ["stage tables", "record steps", "step barrier", "count scan", "scatter", "tail counts"]
print(f"C3 n={n}: {n_rec} records, {nblk} workgroups of {chr_} slots, {len(guids)} proxies")
for k, nm in enumerate(names):
    d = st[:, k + 1] - st[:, k]
    print(f"  {nm:13s} mean {d.mean():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")
for k, nm in enumerate(["record load", "hash lookup", "set entries", "event + count"]):
    print(f"  step sum {nm:14s} mean {ss[:, k].mean():7.2f} us per workgroup")
life = st[:, 6] - st[:, 0]
span = st[:, 6].max()
print(f"  workgroup life mean {life.mean():.2f} us; kernel span {span:.1f} us; "
      f"mean workgroups in flight {life.sum() / span:.0f}")
for q in (0.0, 0.25, 0.5, 0.75, 1.0):
    print(f"  start quantile {q:.2f}: {np.quantile(st[:, 0], q):7.1f} us")
rx.close()
