"""Per-phase timing of the ingest's per-proxy kernel (k_proxy) on C3 (1M datagrams),
from a tuning build with RTPS_PROXY_STAMPS selected by RTPS_RX_LIB:
  make variant NAME=pstamps VDEFS=-DRTPS_PROXY_STAMPS  (in rustdds-io_uring_amd/csrc; the
  define must reach rtps_ingest.hip: see the Makefile's variant target)
Prints the mean over proxies of each phase's summed time (us) and the mean events per proxy."""
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
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.debug_ingest_path(int(os.environ.get("INGEST_PATH", "0")))  # 0: the library's choice; 4: the radix-sort layout
outs["max_records"] = n_rec  # as bench.py sizes the ingest (the proxy bucketing's workgroup bound)
iouts = rx.alloc_ingest_outputs(n_rec, len(guids))
for _ in range(3):
    rx.ingest_reset()
    rx.ingest(arena, off_t, outs, iouts)
rx.sync()
NS = 8
buf = np.zeros(16384 * 8 + 2 * len(guids), dtype=np.uint64)  # the sums, then (start, end) per proxy
fn = lib().rtps_rx_debug_proxy_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
_check(fn(rx._h, buf.ctypes.data, buf.size))
st = buf[:len(guids) * NS].reshape(-1, NS).astype(np.float64) * 0.01  # 100 MHz ticks -> us
se = buf[16384 * 8:].reshape(-1, 2).astype(np.float64) * 0.01
se -= se[:, 0].min()
names = ["setup", "load chunk", "HB scans", "hash insert", "GAP marks", "decide", "merge", "state"]
print(f"C3 n={n}: {len(guids)} proxies; per-proxy phase sums, mean / max over proxies (us)")
for k, nm in enumerate(names):
    print(f"  {nm:12s} {st[:, k].mean():8.1f} {st[:, k].max():8.1f}")
print(f"  total        {st.sum(1).mean():8.1f} {st.sum(1).max():8.1f}")
print(f"  workgroup starts: min 0, p50 {np.median(se[:, 0]):.1f}, p90 {np.quantile(se[:, 0], 0.9):.1f}, "
      f"max {se[:, 0].max():.1f} us; last end {se[:, 1].max():.1f} us")
rx.close()
