"""One diagnostic run: which single, unchunked RCCL point-to-point message
sizes arrive whole on this image's RCCL.  One rank sends to itself (the only pair a 1-GPU box
has; round 4 saw a 1.2-GB self-send deliver only its first half): for each size, a pattern-
filled send buffer, one ncclSend + ncclRecv in one group (rtps_rx_debug_rccl_p2p), then the
first wrong byte offset of the receive buffer (or none).  Prints one JSON line.
Launch: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
            scripts/rccl_size_probe.py"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rustdds-io_uring_amd")]
import torch
import torch.distributed as dist

import rtps_rx
from rtps_rx.shard import rccl_comm, destroy_comms

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
rx = rtps_rx.MessageReceiver(bytes(12), device=0, max_datagrams=16)
comm = rccl_comm(rx, dist, dev)
L = rtps_rx.lib()
fn = L.rtps_rx_debug_rccl_p2p
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
fn.restype = ctypes.c_int
MiB = 1 << 20
sizes = [64 * MiB, 256 * MiB, 512 * MiB, 768 * MiB, 1024 * MiB - 4, 1024 * MiB, 1024 * MiB + 4, 1152 * MiB,
         1280 * MiB, 1536 * MiB, 2048 * MiB - 4, 2048 * MiB, 2304 * MiB]
top = max(sizes)
st = torch.cuda.Stream(dev)
send = (torch.arange(top // 4, dtype=torch.int32, device=dev) * -1640531535).view(torch.uint8)
recv = torch.empty(top, dtype=torch.uint8, device=dev)
res = []
for n in sizes:
    recv.fill_(0xA5)
    torch.cuda.synchronize()
    rc = fn(comm, ctypes.c_void_p(st.cuda_stream), send.data_ptr(), recv.data_ptr(), n, 0)
    torch.cuda.synchronize()
    if rc != 0:
        res.append({"bytes": n, "rc": rc})
        print(json.dumps(res[-1]), flush=True)
        break
    m = recv[:n] != send[:n]
    cnt = int(m.sum().item())
    first = int(m.to(torch.uint8).argmax().item()) if cnt else None
    del m
    res.append({"bytes": n, "whole": first is None, "first_wrong_byte": first,
                "wrong_bytes": cnt, "first_wrong_frac": None if first is None else first / n})
    print(json.dumps(res[-1]), flush=True)
print(json.dumps({"rccl_p2p_size_probe": res, "rccl_version": torch.cuda.nccl.version()}), flush=True)
destroy_comms()
dist.destroy_process_group()
