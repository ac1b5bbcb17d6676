"""World-size-N check of the owner-side exchange on GPU(s) (rtps_rx_shard_*): each
rank generates its chunk on the device, parses it, packs its writer records (with
GAP bitmaps / DATA_FRAG payloads) for their owners, exchanges them (gloo on a
1-GPU box, the library's RCCL rounds with nccl), unpacks what it owns and runs
the reassembly and the history ingest on it.  Every rank then checks its
deliveries (mapped to the whole stream through `origin`) and its proxies'
all_ackable_before against ONE oracle run over the whole stream, restricted to
the writers it owns.  Launch with
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/owner_check.py \
    [gloo|nccl] [c3|c4] [small]
c3: chunks at C5's generator indices (rank * 8M); c4: consecutive chunks (DataFrag
samples straddle them).  small: slots of 200 records / 4 KiB, most items spill."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd"), os.path.join(REPO, "tests")]
import torch
import torch.distributed as dist

import oracle
import rtps_rx
from rtps_rx.records import DELIVERY_DTYPE, WRITER_KINDS, pack_match_table, max_records
from rtps_rx.shard import OwnerShard, destroy_comms

backend = sys.argv[1] if len(sys.argv) > 1 else "gloo"
c4 = "c4" in sys.argv[2:]
small = "small" in sys.argv[2:]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group(backend)
wl = oracle.WL_C4 if c4 else oracle.WL_C3
n = 6000 if c4 else 20000
stride = n if c4 else (8 << 20)


def chunk(r):
    return oracle.gen(wl, n, first_idx=r * stride)


# the whole stream on the host (every rank builds the same): chunks back to back
arenas, offs, lens, base = [], [], [], 0
for r in range(world):
    a, o, l = chunk(r)
    arenas.append(a)
    offs.append(o + np.uint64(base))
    lens.append(l)
    base += len(a)
wa, wo, wlen = np.concatenate(arenas), np.concatenate(offs), np.concatenate(lens)
_, r0, _, _ = oracle.parse(wa, wo, wlen, threads=8)
guids = sorted({bytes(x["prefix"]) + bytes(x["writer_id"]) for x in r0[np.isin(r0["kind"], WRITER_KINDS)]})
tbl = pack_match_table([(g, 100) for g in guids] + [(g, 101) for g in guids[::2]])

# ---- this rank: device chunk -> parse -> owner exchange -> reassembly + ingest ----
rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, device=dev.index, max_datagrams=n)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
rx.set_stream(st)
off, ln, size = rtps_rx.gen_layout(wl, n, first_idx=rank * stride)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(wl, arena, off_t, ln_t, n, first_idx=rank * stride)
rx.set_match_table(tbl)
outs = rx.alloc_outputs(n, max_records(ln))
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
cap, bcap = (200, 4096) if small else (8 * n, 64 << 20)
sh = OwnerShard(rx, world, dist, dev, cap, bcap)
sh.pack(arena, off_t, outs)
sh.exchange()
sh.finish()
ob = sh.unpack()
m = ob.n_records
fouts = rx.alloc_frag_outputs(max(m, 1), ob.arena.nbytes + 16 * m + (1 << 20))
iouts = rx.alloc_ingest_outputs(max(m, 1), len(tbl))
rx.frag_assemble(ob.arena, ob.off, ob.outs, fouts)
rx.ingest(ob.arena, ob.off, ob.outs, iouts, fouts)
rx.sync()
na = int(iouts["n_accepted"].item())
dels = iouts["accepted"][:na].cpu().numpy().reshape(-1).view(DELIVERY_DTYPE)
ack = iouts["ack_base"][:len(tbl)].cpu().numpy()
orecs = ob.records()
orank, osrc = ob.origin()
spilled = int(sum(int(c["n"] - c["cut"]) for c in sh.counts("recv")))

# ---- the single-rank oracle over the whole stream, restricted to this rank's writers ----
_, recs, _, _ = oracle.parse(wa, wo, wlen, match_table=tbl, threads=8)
samples = oracle.FragAssembler().batch_readers(wa, wo, recs, tbl)[0]
_, odels, oack = oracle.HistoryIngest(tbl).batch(wa, wo, recs, samples)
# the shard's owner of each writer (its owner table: the default RTPS_OWNER_BALANCED deal)
own = {}


def owner(g):
    g = bytes(g)
    if g not in own:
        own[g] = sh.owner_of(g)
    return own[g]


mine = np.array([owner(r[8:24]) == rank for r in recs.view(np.uint8).reshape(-1, 64)])
# origin names (source rank, record index in that rank's parse); rank r parsed datagrams [r n, (r+1) n)
first_rec = np.searchsorted(recs["dgram_idx"], np.arange(world) * n)
got = [(int(first_rec[int(orank[j])]) + int(osrc[j]), int(d["reader_slot"])) for d in dels for j in [int(d["rec_idx"])]]
exp = [(int(d["rec_idx"]), int(d["reader_slot"])) for d in odels if mine[int(d["rec_idx"])]]
owned_proxy = np.array([owner(t["writer_guid"]) == rank for t in tbl])
ok = got == exp and len(exp) > 0 and np.array_equal(ack[owned_proxy], oack[owned_proxy]) and \
    (ack[~owned_proxy] == 1).all() and (spilled > 0) == (small and world > 0)
via = "library RCCL rounds" if sh.comm is not None else "torch.distributed " + backend
print(f"rank {rank}/{world} ({via}, {'C4' if c4 else 'C3 at C5 indices'}{', small slots' if small else ''}): "
      f"{m} records owned, {spilled} via the spill, {len(got)} deliveries (expected {len(exp)}), "
      f"{'OK' if ok else 'MISMATCH'}", flush=True)
sh.close()
dist.barrier()
destroy_comms()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
