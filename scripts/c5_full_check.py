"""C5's per-rank size on one GPU (8M C3 datagrams = 64M / 8 ranks), through both
multi-GPU exchanges with a one-rank RCCL communicator (every bucket goes to
itself), checked on the device without host copies of the 2-GB record arrays:

  * owner-side exchange: rtps_rx_shard_pack -> rtps_rx_shard_exchange / _finish
    (library RCCL rounds) -> rtps_rx_shard_unpack, slots sized from the batch: no
    spill, and the owner batch holds every writer-kind PASS record in order
    (all 64 bytes but dgram_idx, which becomes the record index, for the kinds that
    cross whole; kind, flags, writer GUID, route, payload kind and SN of a DATA, which
    crosses as its 16-B item; origin = the record's index in the parse output), with
    every GAP bitmap at arena + dgram_off + bitmap_off;
  * record exchange: rtps_rx_bucket_by_writer_padded -> rtps_rx_exchange: no
    overflow, received == bucketed.
Launch: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 scripts/c5_full_check.py"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch
import torch.distributed as dist

import rtps_rx
from rtps_rx.shard import OwnerShard, Exchange, destroy_comms, dev_copy

OWN = bytes.fromhex("0103000c292d31a228200208")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
t0 = time.time()
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C3, n, first_idx=0)
rx = rtps_rx.MessageReceiver(OWN, device=0, max_datagrams=n)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
rx.set_stream(st)
arena = torch.empty(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_C3, arena, off_t, ln_t, n)
probe = rx.alloc_outputs(n, 1)
rx.parse_batch_device(arena, off_t, ln_t, n, probe)
rx.sync()
n_rec = int(probe["n_records"].item())
del probe
outs = rx.alloc_outputs(n, n_rec)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.sync()
# the reader subscribed to every writer of the stream (as bench.py's owner exchange): the shard's
# owner table lists them, so their DATA cross as compact 16-B items
r0 = outs["records"][:n_rec]
wk = (r0[:, 6] == 0x15) | (r0[:, 6] == 0x16) | (r0[:, 6] == 0x07) | (r0[:, 6] == 0x08) | (r0[:, 6] == 0x13)
guids = torch.unique(r0[wk][:, 8:24], dim=0).cpu().numpy()
from rtps_rx.records import MATCH_DTYPE
tbl = np.zeros(len(guids), dtype=MATCH_DTYPE)
tbl["writer_guid"] = guids
rx.set_match_table(tbl)
del r0, wk
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
rx.sync()
print(f"parsed {n} datagrams ({size / 2**30:.2f} GiB), {n_rec} records, {time.time() - t0:.0f} s", flush=True)

recs = outs["records"][:n_rec]
kind, route = recs[:, 6], recs[:, 30]
writer = (kind == 0x15) | (kind == 0x16) | (kind == 0x07) | (kind == 0x08) | (kind == 0x13)
items = writer & ((route & 1) != 0)
n_items = int(items.sum().item())
gap = items & (kind == 0x08)
nb = recs[:, 48:52].contiguous().view(torch.int32).reshape(-1).to(torch.int64)
gap_bytes = torch.where(gap & (nb > 0), ((4 * ((nb + 31) // 32)) + 15) // 16 * 16, torch.zeros_like(nb))
# blob bytes: every item that is not a DATA sends its 64-B record (C3 has no DATA_FRAG; every DATA's
# writer is listed: compact)
blob_total = int(gap_bytes.sum().item()) + 64 * int((items & (kind != 0x15)).sum().item())
ok = True

# ---- owner-side exchange, one rank, slots sized to the batch ----
sh = OwnerShard(rx, 1, dist, dev, n_items, blob_total)
sh.pack(arena, off_t, outs)
sh.exchange()
sh.finish()
ob = sh.unpack()
sc = sh.counts("send")
spill = int(sc["n"][0] - sc["cut"][0])
got = torch.empty((max(ob.n_records, 1), 64), dtype=torch.uint8, device=dev)
dev_copy(got.data_ptr(), ob.outs["records"].ptr, 64 * ob.n_records)
exp = recs[items]
idx_ok = torch.equal(got[:, 0:4].contiguous().view(torch.int32).reshape(-1),
                     torch.arange(ob.n_records, dtype=torch.int32, device=dev))
# a DATA crosses as its item: kind, flags, writer GUID, route, payload kind, sn (the rest zero)
is_data = exp[:, 6] == 0x15
keep = torch.zeros(64, dtype=torch.bool, device=dev)
keep[[6, 7] + list(range(8, 24)) + [30, 31] + list(range(32, 40))] = True
exp_d = torch.where(is_data[:, None] & ~keep[None, :], torch.zeros_like(exp), exp)
body_ok = torch.equal(got[:, 4:], exp_d[:, 4:])
origin = torch.empty(ob.n_records, dtype=torch.int64, device=dev)
dev_copy(origin.data_ptr(), ob.origin_ptr, 8 * ob.n_records)
org_ok = torch.equal(origin & 0xFFFFFFFF, torch.nonzero(items).reshape(-1)) and int((origin >> 32).max().item()) == 0
# every GAP bitmap word where the owner's consumers read it
goff = torch.empty(ob.n_records, dtype=torch.int64, device=dev)
dev_copy(goff.data_ptr(), ob.off.ptr, 8 * ob.n_records)
oarena = torch.empty(ob.arena.nbytes, dtype=torch.uint8, device=dev)
dev_copy(oarena.data_ptr(), ob.arena.ptr, ob.arena.nbytes)
g = gap[items]
gi = torch.nonzero(g & (nb[items] > 0)).reshape(-1)
bmo = exp[gi, 52:54].contiguous().view(torch.int16).reshape(-1).to(torch.int64) & 0xFFFF
src = off_t[exp[gi, 0:4].contiguous().view(torch.int32).reshape(-1).to(torch.int64)] + bmo
dst = goff[gi] + bmo
bm_ok = torch.equal(arena[src], oarena[dst]) and torch.equal(arena[src + 3], oarena[dst + 3])
if not org_ok:
    want = torch.nonzero(items).reshape(-1)
    bad = torch.nonzero((origin & 0xFFFFFFFF) != want).reshape(-1)
    i = int(bad[0].item()) if len(bad) else -1
    print(f"  {len(bad)} origins differ, first {i}: got {int(origin[i].item()):#x} want {int(want[i].item())}; "
          f"{len(origin)} vs {len(want)}", flush=True)
if not body_ok:
    bad = torch.nonzero((got[:, 4:] != exp_d[:, 4:]).any(dim=1)).reshape(-1)
    i = int(bad[0].item())
    print(f"  {len(bad)} rows differ, first {i}: got {got[i].cpu().numpy().tobytes().hex()} "
          f"exp {exp_d[i].cpu().numpy().tobytes().hex()}", flush=True)
ok &= ob.n_records == n_items and spill == 0 and idx_ok and body_ok and org_ok and bm_ok
print(f"owner exchange (library RCCL rounds): {n_items} items, {blob_total} blob bytes, spill {spill}, "
      f"records {'ok' if body_ok and idx_ok else 'BAD'}, origin {'ok' if org_ok else 'BAD'}, "
      f"GAP bitmaps ({len(gi)}) {'ok' if bm_ok else 'BAD'}, {time.time() - t0:.0f} s", flush=True)
sh.close()
del got, origin, goff, oarena

# ---- record exchange: padded buckets + rtps_rx_exchange, one rank ----
exch_kind = writer | (kind == 0x06) | (kind == 0x12)
n_exch = int(exch_kind.sum().item())
ex = Exchange(rx, n_rec, 1, dist, dev, cap=n_exch)
ex.bucket(outs)
rx.sync()
over = ex.overflowed()
got, split = ex.exchange()
torch.cuda.synchronize()
rec_ok = got.shape[0] == n_exch and torch.equal(got, recs[exch_kind])
if not rec_ok and got.shape[0] == n_exch:
    bad = torch.nonzero((got != recs[exch_kind]).any(dim=1)).reshape(-1)
    i = int(bad[0].item())
    print(f"  {len(bad)} rows differ, first {i}: got {got[i].cpu().numpy().tobytes().hex()} "
          f"exp {recs[exch_kind][i].cpu().numpy().tobytes().hex()}", flush=True)
ok &= rec_ok and not over
print(f"record exchange (rtps_rx_exchange): {n_exch} records, overflow {over}, "
      f"received {'== bucketed' if rec_ok else 'MISMATCH'}, {time.time() - t0:.0f} s", flush=True)
print("C5 full OK" if ok else "C5 full MISMATCH", flush=True)
destroy_comms()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
