"""World-size-N check of the full sharded path on GPU(s): each rank generates
its chunk on the device, parses it, buckets by writer GUID on the device and
exchanges records (gloo on a 1-GPU box, nccl=RCCL across GPUs); every rank
verifies what it received against the CPU oracle.  Launch with
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/shard_check.py [backend] [padded|desc] [c5]

c5: each rank's chunk starts at generator index rank * 8M, as BASELINE config C5
(64M datagrams over 8 GPUs) lays the stream out (reduced n per rank).  With the
nccl backend and padded buckets the records move through the library's own RCCL
exchange (rtps_rx_exchange); one rank exchanges with itself."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd"), os.path.join(REPO, "tests")]
import torch
import torch.distributed as dist

import oracle
import rtps_rx
from rtps_rx.records import RECORD_DTYPE
from rtps_rx.shard import Exchange
from shard_ref import owner_np

backend = sys.argv[1] if len(sys.argv) > 1 else "gloo"
padded = len(sys.argv) > 2 and sys.argv[2] in ("padded", "desc")
desc = len(sys.argv) > 2 and sys.argv[2] == "desc"
c5 = "c5" in sys.argv[2:]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ngpu = torch.cuda.device_count()
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % ngpu)
torch.cuda.set_device(dev)
dist.init_process_group(backend)
n = 20000
stride = (8 << 20) if c5 else n  # generator index of rank r's first datagram: r * stride
off, ln, size = rtps_rx.gen_layout(rtps_rx.WL_C3, n, first_idx=rank * stride)
rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, device=dev.index, max_datagrams=n)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
rx.set_stream(st)
arena = torch.zeros(size, dtype=torch.uint8, device=dev)
off_t = torch.from_numpy(off.view(np.int64)).to(dev)
ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
rx.generate(rtps_rx.WL_C3, arena, off_t, ln_t, n, first_idx=rank * stride)
cap = rtps_rx.max_records(ln)
outs = rx.alloc_outputs(n, cap)
table = None
if desc:  # every rank matches the same writers, listed in the same (sorted) order
    from rtps_rx.records import MATCH_DTYPE
    a0, o0, l0 = oracle.gen(oracle.WL_C3, 4000)
    _, r0, _, _ = oracle.parse(a0, o0, l0)
    guids = sorted({bytes(r["prefix"]) + bytes(r["writer_id"]) for r in r0 if r["kind"] in (0x15, 0x07, 0x08)})
    table = np.zeros(len(guids), dtype=MATCH_DTYPE)
    for k, g in enumerate(guids):
        table[k]["writer_guid"] = np.frombuffer(g, dtype=np.uint8)
    rx.set_match_table(table)
rx.parse_batch_device(arena, off_t, ln_t, n, outs)
if padded:  # fixed bucket capacity agreed over ranks from a first bucketing
    probe = Exchange(rx, cap, world, dist, dev, cap=cap, item="descriptors") if desc else Exchange(rx, cap, world, dist, dev)
    probe.bucket(outs)
    t = probe.counts.max().reshape(1)
    t = t.cpu() if backend == "gloo" else t
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ex = Exchange(rx, cap, world, dist, dev, cap=int(t.item()), item="descriptors" if desc else "records")
else:
    ex = Exchange(rx, cap, world, dist, dev)
ex.bucket(outs)
torch.cuda.synchronize(dev)
assert not (padded and ex.overflowed())
got, split = ex.exchange()
torch.cuda.synchronize(dev)
if desc:
    from rtps_rx.records import XDESC_DTYPE
    from shard_ref import desc_bucket_np
    got = got.cpu().numpy().reshape(-1).view(XDESC_DTYPE)
    exp = []
    for r in range(world):
        a, o, l = oracle.gen(oracle.WL_C3, n, first_idx=r * stride)
        _, recs, _, _ = oracle.parse(a, o, l, match_table=table)
        # the target set numbers of rank r's records (TARGETED-only records go to their entity
        # set's owner): rank r's chunk parsed again here with the same table
        off_r, ln_r, size_r = rtps_rx.gen_layout(rtps_rx.WL_C3, n, first_idx=r * stride)
        arena_r = torch.zeros(size_r, dtype=torch.uint8, device=dev)
        off_rt = torch.from_numpy(off_r.view(np.int64)).to(dev)
        ln_rt = torch.from_numpy(ln_r.view(np.int32)).to(dev)
        outs_r = rx.alloc_outputs(n, rtps_rx.max_records(ln_r))
        rx.generate(rtps_rx.WL_C3, arena_r, off_rt, ln_rt, n, first_idx=r * stride)
        rx.parse_batch_device(arena_r, off_rt, ln_rt, n, outs_r)
        torch.cuda.synchronize(dev)
        sets = outs_r["target"][:len(recs)].cpu().numpy().view(np.uint32)
        exp.append(desc_bucket_np(recs, [bytes(t["writer_guid"]) for t in table], world, entity_sets=sets)[rank])
    exp = np.concatenate(exp)
else:
    got = got.cpu().numpy().reshape(-1).view(RECORD_DTYPE)
    exp = []
    for r in range(world):
        a, o, l = oracle.gen(oracle.WL_C3, n, first_idx=r * stride)
        _, recs, _, _ = oracle.parse(a, o, l)
        exp.append(recs[owner_np(recs, world) == rank])
    exp = np.concatenate(exp)
ok = got.tobytes() == exp.tobytes()
via = "library RCCL exchange" if getattr(ex, "comm", None) is not None else "torch.distributed " + backend
print(f"rank {rank}/{world} ({via}{', desc' if desc else ', padded' if padded else ''}{', C5 indices' if c5 else ''}): "
      f"received {len(got)} records, expected {len(exp)}, "
      f"{'OK' if ok else 'MISMATCH'}", flush=True)
dist.barrier()
from rtps_rx.shard import destroy_comms
destroy_comms()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
