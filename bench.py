#!/usr/bin/env python3
"""Benchmark: device-resident RTPS receive-path parse on MI355X.

One step = parse one batch of synthetic datagrams already resident in HBM
(the whole receive-path parse: header + submessage walk + interpreter +
classification + ordered 64-B records).  The default workload is T at every N
(1M x 1 KiB datagrams per GPU: weak scaling).  At N >= 2 GPUs (one process per
GPU, torch.distributed over RCCL) the step adds the owner-side exchange
(SURVEY.md §8e): every writer record that passes goes to its writer's owner
(writer-GUID hash) with its GAP bitmap / DATA_FRAG payload bytes, in fixed
slots over one grouped RCCL send/recv per peer (pipelined with the next parse)
plus an exact spill round when a slot overflows, and is unpacked there as one
batch; the same steps are then timed again with every owner's history-cache
ingest added (`pipeline_with_ingest`).  N >= 2 then measures BASELINE's 8-GPU
config C5 (64M datagrams of the C3 mix in total, rank r parses the r-th chunk:
strong scaling) the same way, reported as `c5`.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload T|C2|C3|C4]

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "rustdds-io_uring_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import rtps_rx  # noqa: E402
from rtps_rx.records import (RECORD_DTYPE, DATA, DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP, ACKNACK,  # noqa: E402
                             NACK_FRAG, INFO_TS, INFO_SRC, INFO_DST, INFO_REPLY, PK_DATA, PK_KEY, MATCH_DTYPE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
OWN_PREFIX = bytes.fromhex("0103000c292d31a228200208")
WORKLOAD_DESC = {
    "T": "1M x 1024 B RTPS datagrams, one DATA each (980 B payload incl. CDR_LE encapsulation), 16 writers",
    "C2": "1M x 300 B RTPS datagrams, one DATA each (256 B CDR payload), 16 writers",
    "C3": "1M mixed datagrams 128-1500 B: DATA/HEARTBEAT/ACKNACK/GAP/INFO_TS/INFO_DST/INFO_SRC, 16 writers",
    "C4": "1M x 1400 B DATA_FRAG datagrams (64 KiB samples, 1344 B fragments), 16 writers",
    "C5": "64M datagrams of the C3 mix in total (64M / N per GPU, rank r's chunk at generator index r * 64M / N), "
          "16 writers, records hash-sharded by writer GUID with one RCCL all-to-all over xGMI",
}
C5_TOTAL = 64 << 20


def algorithmic_bytes(status, recs, n, record_bytes=64):
    """Bytes the parse must move (zero-copy: payload bytes are never read).

    reads : 12 B of (offset, length) per datagram, the 20-B RTPS header of every
            parsed datagram, per materialised submessage its 4-B header plus the
            fixed fields the reference reader consumes (+ inline QoS, + the 4-B
            encapsulation of a DATA payload);
    writes: 1 B status + 4 B rec_begin per datagram, 64 B record + 4 B target set
            per record.
    """
    k = recs["kind"]
    fixed = np.zeros(len(recs), dtype=np.int64)
    fixed[k == DATA] = 20
    fixed[k == DATA_FRAG] = 32
    fixed[k == HEARTBEAT] = 28
    fixed[k == HEARTBEAT_FRAG] = 24
    fixed[k == GAP] = 28
    fixed[k == ACKNACK] = 24
    fixed[k == NACK_FRAG] = 28
    fixed[k == INFO_SRC] = 20
    fixed[k == INFO_DST] = 12
    fixed[k == INFO_REPLY] = 5
    fixed[(k == INFO_TS) & ((recs["flags"] & 2) == 0)] = 8
    qos = np.where((k == DATA) | (k == DATA_FRAG), recs["aux16"].astype(np.int64), 0)
    enc = np.where((k == DATA) & np.isin(recs["payload_kind"], (PK_DATA, PK_KEY)), 4, 0)
    reads = 12 * n + 20 * int((status == 0).sum()) + int((4 + fixed + qos + enc).sum())
    writes = 5 * n + (record_bytes + 4) * len(recs)
    return reads + writes, reads, writes


def pmc_profile(workload):
    """Calibrated per-launch HBM bytes of the parse kernels from the newest committed
    rocprofv3 PMC summary (profiles/r<NN>_pmc_<workload>.json, scripts/gpu_pmc.sh):
    FETCH_SIZE (reads, scaled by the fetch calibration of MI355X_MICROARCH.md) and
    WRITE_SIZE, in separate --pmc passes."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{workload}.json")),
                   key=lambda f: int(re.search(r"r(\d+)_pmc", f).group(1)))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    d["_source"] = os.path.relpath(files[-1], REPO)
    return d


PMC_KEYS = {"rtps_parse_spec_kernel": "parse_spec", "rtps_parse_chain_kernel": "parse_chain",
            "rtps_parse_lds_kernel": "parse_lds", "rtps_parse_item_kernel": "parse_item",
            "rtps_parse_rslab_kernel": "parse_rslab", "rtps_parse_scan_kernel": "parse_scan",
            "rtps_parse_emit_kernel": "parse_emit", "rtps_parse_emit2_kernel": "parse_emit2"}
KERNEL_NAMES = {1: "rtps_parse_spec_kernel", 2: "rtps_parse_chain_kernel", 3: "rtps_parse_lds_kernel",
                4: "rtps_parse_item_kernel", 5: "rtps_parse_rslab_kernel"}


def _time_phases(rx, arena, off_t, ln_t, n, outs, stream, steps, phases):
    which = 0
    for _ in range(3):
        which = rx.debug_parse_phases(arena, off_t, ln_t, n, outs, phases)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for _ in range(steps):
        rx.debug_parse_phases(arena, off_t, ln_t, n, outs, phases)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps, which


def time_dominant_kernel(rx, arena, off_t, ln_t, n, outs, stream, steps):
    """Live HIP-event timing of the parse's dominant kernel alone, K back-to-back launches on
    the parse stream, one event pair.  The first kernel of rtps_rx_parse_batch
    (rtps_parse_spec_kernel; for mixed traffic the item pass's walk rtps_parse_item_kernel E,
    or the chained kernels) is timed; for the item pass also the record pass W alone
    (rtps_parse_emit2_kernel, or rtps_parse_emit_kernel) and the scan + record pass.  The
    dominant kernel is the slower of E and W: its name and time are returned."""
    ms, which = _time_phases(rx, arena, off_t, ln_t, n, outs, stream, steps, 1)
    kname, extra = KERNEL_NAMES[which], {}
    if which in (4, 5):
        ms2, _ = _time_phases(rx, arena, off_t, ln_t, n, outs, stream, steps, 2)
        extra = {"item_kernel_ms": ms, "scan_plus_emit_ms": ms2}
        if which == 4:
            w_ms, _ = _time_phases(rx, arena, off_t, ln_t, n, outs, stream, steps, 2 | 4)
            wname = "rtps_parse_emit_kernel" if rx.debug_emit() == 1 else "rtps_parse_emit2_kernel"
            extra.update({"emit_kernel": wname, "emit_kernel_ms": w_ms, "scan_ms": max(0.0, ms2 - w_ms)})
            if w_ms > ms:
                kname, ms = wname, w_ms
    for _ in range(2):  # full launches restore the per-launch bookkeeping
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
    torch.cuda.synchronize()
    return ms, kname, extra


def time_ceilings(arena, off_t, ln_t, n, stream, steps):
    """Live timing of the same-shape ceiling kernels (csrc/diag/ceiling.hip: no parse,
    only the parse's memory traffic: 12 B (offset, length) + the 64-B head of every
    datagram at its stride; 'read+write' adds the 64-B record through an LDS transpose
    and the status / rec_begin stores).  None if the diagnostic library is absent."""
    import ctypes
    path = os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so")
    if not os.path.exists(path):
        return None
    D = ctypes.CDLL(path)
    D.diag_ceiling.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    rec = torch.empty((n, 64), dtype=torch.uint8, device=arena.device)
    status = torch.empty(n, dtype=torch.uint8, device=arena.device)
    rb = torch.empty(n, dtype=torch.int32, device=arena.device)
    res = {}
    for name, mode in (("read_only", 1), ("read_write", 3)):
        def run():
            D.diag_ceiling(mode, arena.data_ptr(), off_t.data_ptr(), ln_t.data_ptr(), n, rec.data_ptr(),
                           status.data_ptr(), rb.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
        for _ in range(3):
            run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(steps):
            run()
        b.record(stream)
        torch.cuda.synchronize()
        res[name] = a.elapsed_time(b) / steps
    return res


def time_hops_ceilings(arena, off_t, ln_t, n, outs, n_rec, stream, steps):
    """Live timing of the mixed-traffic floor (csrc/diag/ceiling.hip ceil_hops_kernel): the
    parse's dependent header hops (one 16-B window per submessage) and a 64-B record store per
    materialised submessage at the parse's own positions (its status / rec_begin), no field
    decode, no validation, no classification; one walk, and two walks (count, then write) as the
    chained kernel does.  None if the diagnostic library is absent."""
    import ctypes
    path = os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so")
    if not os.path.exists(path):
        return None
    D = ctypes.CDLL(path)
    D.diag_ceiling_hops.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 2 + \
        [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    rec = torch.empty((max(n_rec, 1), 64), dtype=torch.uint8, device=arena.device)
    res = {}
    for walks in (1, 2):
        def run():
            D.diag_ceiling_hops(walks, arena.data_ptr(), arena.numel(), off_t.data_ptr(), ln_t.data_ptr(), n,
                                outs["status"].data_ptr(), outs["rec_begin"].data_ptr(), rec.data_ptr(),
                                ctypes.c_void_p(stream.cuda_stream))
        for _ in range(3):
            run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(steps):
            run()
        b.record(stream)
        torch.cuda.synchronize()
        res[walks] = a.elapsed_time(b) / steps
    return res


def end_to_end(rx, arena, off_t, ln_t, n, outs, n_rec, stream, reps=5):
    """Host-memory-in / host-memory-out rate (the path starts in io_uring receive
    buffers and ends in the history cache).  Two modes, both checked against the
    device-resident result; never the headline value:
      copy      : pinned H2D of the whole arena + parse + D2H of status and records
      zero_copy : the kernel reads datagram heads straight from pinned host memory
                  and writes status/records straight to pinned host memory."""
    host_arena = torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True)
    host_arena.copy_(arena)
    h_off = torch.empty(n, dtype=torch.int64, pin_memory=True)
    h_off.copy_(off_t)
    h_ln = torch.empty(n, dtype=torch.int32, pin_memory=True)
    h_ln.copy_(ln_t)
    h_outs = {"status": torch.empty(n, dtype=torch.uint8, pin_memory=True),
              "records": torch.empty((max(n_rec, 1), 64), dtype=torch.uint8, pin_memory=True),
              "target": torch.empty(max(n_rec, 1), dtype=torch.int32, pin_memory=True),
              "rec_begin": torch.empty(n, dtype=torch.int32, pin_memory=True),
              "n_records": torch.zeros(1, dtype=torch.int64, pin_memory=True), "max_records": n_rec}
    torch.cuda.synchronize()
    ref_status = outs["status"][:n].cpu()
    ref_recs = outs["records"][:n_rec].cpu()

    def copy_mode():
        arena.copy_(host_arena, non_blocking=True)
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        h_outs["status"].copy_(outs["status"][:n], non_blocking=True)
        h_outs["records"][:n_rec].copy_(outs["records"][:n_rec], non_blocking=True)

    def zero_copy_mode():
        rx.parse_batch_device(host_arena, h_off, h_ln, n, h_outs)

    res = {}
    for name, fn in (("copy", copy_mode), ("zero_copy", zero_copy_mode)):
        times = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) * 1e-3)
        ok = torch.equal(h_outs["status"], ref_status) and torch.equal(h_outs["records"][:n_rec], ref_recs)
        t = min(times)
        res[name] = {"datagrams_per_s": n / t, "ms": t * 1e3, "parity_ok": bool(ok)}
    res["copy"]["pcie_bytes"] = arena.numel() + n + n_rec * 64
    res["best"] = max(("copy", "zero_copy"), key=lambda k: res[k]["datagrams_per_s"])
    return res


def full_chain(rx, workload, arena, off_t, ln_t, n, n_rec, n_entries, reps=5):
    """The receive path from host memory to host memory, as north_star names it (io_uring
    receive buffers in, parsed samples back to the DDS history cache): the datagrams in pinned
    host memory -> parse -> history-cache ingest with the topic caches (TopicCache::add_change,
    reader.rs:693-758 -> make_cache_change :1185-1205 -> dds_cache.rs:210-276) -> CDR decode of
    the deliveries (compact rows: the samples the cache takes) -> D2H of the deliveries and
    their rows.  Input two ways: 'zero_copy' (the kernels read the datagram heads and the
    delivered payloads straight from pinned host memory) and 'copy' (one H2D of the arena
    first).  Fresh writer proxies and empty topic caches before each run (outside the clock);
    the host waits for the delivery count, then copies exactly the deliveries and rows.  Wall
    clock per run, best of `reps`; checked against the same chain on the HBM-resident batch."""
    from rtps_rx import cdr
    t = getattr(cdr, CDR_TYPES[workload])
    dev = arena.device
    host_arena = torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True)
    host_arena.copy_(arena)
    h_off = torch.empty(n, dtype=torch.int64, pin_memory=True)
    h_off.copy_(off_t)
    h_ln = torch.empty(n, dtype=torch.int32, pin_memory=True)
    h_ln.copy_(ln_t)
    rx.set_topics([(1, 64)], [(0, 1)])
    outs = rx.alloc_outputs(n, n_rec)
    iouts = rx.alloc_ingest_outputs(n_rec, n_entries)
    max_del = iouts["max_accepted"]
    rows, rst = rx.alloc_rows(t, max_del)
    h_na = torch.zeros(1, dtype=torch.int64, pin_memory=True)
    h_dels = torch.empty((max(max_del, 1), 8), dtype=torch.uint8, pin_memory=True)
    h_rows = torch.empty((max(max_del, 1), t.row_bytes), dtype=torch.uint8, pin_memory=True)
    h_rst = torch.empty(max(max_del, 1), dtype=torch.uint8, pin_memory=True)
    dev_arena = torch.empty_like(arena)

    def chain(src, o, l, copy_in):
        if copy_in:
            dev_arena.copy_(host_arena, non_blocking=True)
            src, o, l = dev_arena, off_t, ln_t
        rx.parse_batch_device(src, o, l, n, outs)
        rx.ingest(src, o, outs, iouts, topic_cache=True)
        rx.cdr_decode_list(t, src, o, outs, iouts["accepted"], 8, iouts["n_accepted"], max_del, rows, rst)
        h_na.copy_(iouts["n_accepted"], non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        na = min(int(h_na.item()), max_del)
        h_dels[:na].copy_(iouts["accepted"][:na], non_blocking=True)
        h_rows[:na].copy_(rows[:na], non_blocking=True)
        h_rst[:na].copy_(rst[:na], non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        return na

    _reset_caches(rx, True)
    na_ref = chain(arena, off_t, ln_t, False)  # the HBM-resident reference
    ref = (h_dels[:na_ref].clone(), h_rows[:na_ref].clone(), h_rst[:na_ref].clone())
    res = {}
    for name, args in (("zero_copy", (host_arena, h_off, h_ln, False)), ("copy", (None, None, None, True))):
        times = []
        for _ in range(reps):
            _reset_caches(rx, True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            na = chain(*args)
            times.append(time.perf_counter() - t0)
        ok = na == na_ref and torch.equal(h_dels[:na], ref[0]) and torch.equal(h_rows[:na], ref[1]) and \
            torch.equal(h_rst[:na], ref[2])
        tm = min(times)
        res[name] = {"ms": tm * 1e3, "datagrams_per_s": n / tm, "deliveries": na, "deliveries_per_s": na / tm,
                     "d2h_bytes": na * (8 + t.row_bytes + 1), "parity_ok": bool(ok)}
    res["copy"]["h2d_bytes"] = int(arena.numel())
    res["best"] = max(("copy", "zero_copy"), key=lambda k: res[k]["datagrams_per_s"])
    res["what"] = ("host-memory datagrams -> parse -> ingest + topic caches -> CDR rows of the deliveries -> "
                   "deliveries and rows in host memory; wall clock incl. the H2D / D2H copies and one host wait "
                   f"for the delivery count; sample type {CDR_TYPES[workload]}")
    rx.set_topics([], [])
    return res


def pcie_probe(h2d_bytes, d2h_bytes, dev, reps=3, chunk=128 << 20):
    """Pinned-memory PCIe rates of this box: h2d_bytes host -> device alone, d2h_bytes device ->
    host alone, and both at once (full duplex: the H2D chunks on one stream, the D2H chunks on
    another, issued interleaved as a receive pipeline issues them): the bound of a host-to-host
    chain that moves those bytes.  Copies of `chunk` bytes; best of `reps` wall-clock runs."""
    hs = torch.empty(h2d_bytes, dtype=torch.uint8, pin_memory=True)
    hd = torch.empty(d2h_bytes, dtype=torch.uint8, pin_memory=True)
    ds = torch.empty(h2d_bytes, dtype=torch.uint8, device=dev)
    dd = torch.empty(d2h_bytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run(h2d, d2h):
        best = float("inf")
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for c in range(0, max(h2d_bytes, d2h_bytes), chunk):
                if h2d and c < h2d_bytes:
                    with torch.cuda.stream(s1):
                        ds[c:c + chunk].copy_(hs[c:c + chunk], non_blocking=True)
                if d2h and c < d2h_bytes:
                    with torch.cuda.stream(s2):
                        hd[c:c + chunk].copy_(dd[c:c + chunk], non_blocking=True)
            s1.synchronize()
            s2.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best
    t_h, t_d, t_b = run(True, False), run(False, True), run(True, True)
    # the duplex rate: 1 GiB each way in interleaved chunks (short transfers do not overlap on this
    # box's copy engines, so the rate is taken where they do)
    sym = 1 << 30
    hb, db = h2d_bytes, d2h_bytes
    hs = torch.empty(sym, dtype=torch.uint8, pin_memory=True)
    hd = torch.empty(sym, dtype=torch.uint8, pin_memory=True)
    ds = torch.empty(sym, dtype=torch.uint8, device=dev)
    dd = torch.empty(sym, dtype=torch.uint8, device=dev)
    h2d_bytes = d2h_bytes = sym
    t_s = run(True, True)
    h2d_bytes, d2h_bytes = hb, db
    duplex = 2 * sym / t_s / 1e9
    bound = max(t_h, t_d, (hb + db) / (duplex * 1e9))
    return {"h2d_gbs": hb / t_h / 1e9, "d2h_gbs": db / t_d / 1e9, "h2d_ms": t_h * 1e3,
            "d2h_ms": t_d * 1e3, "both_ms": t_b * 1e3, "duplex_gbs": duplex, "duplex_probe_bytes_each_way": sym,
            "serial_ms": (t_h + t_d) * 1e3, "h2d_bytes": hb, "d2h_bytes": db, "chunk_bytes": chunk,
            "bound_ms": bound * 1e3,
            "bound": "max(H2D alone, D2H alone, both volumes at the measured duplex rate)"}


def full_chain_pipelined(rx, workload, arena, off_t, ln_t, n, n_entries, batch=1 << 17, slots=3, reps=3,
                         rows_to_host=False):
    """the host-to-host chain as a receive loop runs it (Domain::handle_event
    per CQE, io_uring/rtps/dp_event_loop.rs:164-211, batched): the 1M-datagram stream in pinned
    host memory cut into batches of `batch` datagrams; batch k+1's H2D (arena piece + offsets +
    lengths) on a copy stream, batch k's parse -> ingest + topic caches -> CDR decode of the
    deliveries on the compute stream, batch k-1's D2H of exactly its deliveries and rows on a
    third stream, ordered by events (the host waits only for a finished batch's delivery count,
    which it needs to size that batch's D2H).  The writer proxies and topic caches carry across
    the batches (one stream, as the reference's reader sees it).  Every batch is checked against
    the same chain run batch by batch on the HBM-resident stream (parity_ok).
    rows_to_host: the CDR decode writes each batch's rows and row statuses straight into the
    batch's pinned host buffers (the device -> host direction carried by the kernel's own PCIe
    writes, beside the copy engine's host -> device traffic); only the deliveries are copied."""
    from rtps_rx import cdr
    t = getattr(cdr, CDR_TYPES[workload])
    dev = arena.device
    comp = torch.cuda.current_stream(dev)
    off = off_t.cpu().numpy().astype(np.int64)
    ln = ln_t.cpu().numpy().astype(np.int64)
    nb = (n + batch - 1) // batch
    cuts = [(k * batch, min(n, (k + 1) * batch)) for k in range(nb)]
    spans = [(int(off[a]), int(off[b - 1] + ln[b - 1])) for a, b in cuts]
    host_arena = torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True)
    host_arena.copy_(arena)
    h_off = [torch.from_numpy(off[a:b] - off[a]).pin_memory() for a, b in cuts]
    h_ln = [torch.from_numpy(ln[a:b].astype(np.int32)).pin_memory() for a, b in cuts]
    piece = max(e - a for a, e in spans)
    rx.set_topics([(1, 64)], [(0, 1)])
    # per-slot device buffers, sized from a probe parse of every batch (records per batch)
    n_rec_b = []
    probe = rx.alloc_outputs(batch, 1)
    for (a, b), (s0, s1) in zip(cuts, spans):
        o = (off_t[a:b] - int(off[a])).contiguous()
        rx.parse_batch_device(arena[s0:s1], o, ln_t[a:b].contiguous(), b - a, probe)
        torch.cuda.synchronize(dev)
        n_rec_b.append(int(probe["n_records"].item()))
    del probe
    mrec = max(n_rec_b)
    S = [{"arena": torch.empty(piece, dtype=torch.uint8, device=dev),
          "off": torch.empty(batch, dtype=torch.int64, device=dev),
          "ln": torch.empty(batch, dtype=torch.int32, device=dev),
          "outs": rx.alloc_outputs(batch, mrec),
          "iouts": rx.alloc_ingest_outputs(mrec, n_entries)} for _ in range(slots)]
    max_del = S[0]["iouts"]["max_accepted"]
    for x in S:
        x["rows"], x["rst"] = rx.alloc_rows(t, max_del)
    h_na = [torch.zeros(1, dtype=torch.int64, pin_memory=True) for _ in range(nb)]
    h_dels = [torch.empty((max(n_rec_b[k], 1), 8), dtype=torch.uint8, pin_memory=True) for k in range(nb)]
    h_rows = [torch.empty((max(n_rec_b[k], 1), t.row_bytes), dtype=torch.uint8, pin_memory=True) for k in range(nb)]
    h_rst = [torch.empty(max(n_rec_b[k], 1), dtype=torch.uint8, pin_memory=True) for k in range(nb)]
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def compute(k, x, src, o, l, to_host=False):
        m = cuts[k][1] - cuts[k][0]
        rx.parse_batch_device(src, o, l, m, x["outs"])
        rx.ingest(src, o, x["outs"], x["iouts"], topic_cache=True)
        rows, rst, cap = (h_rows[k], h_rst[k], h_rst[k].shape[0]) if to_host else (x["rows"], x["rst"], max_del)
        rx.cdr_decode_list(t, src, o, x["outs"], x["iouts"]["accepted"], 8, x["iouts"]["n_accepted"], cap, rows, rst)
        h_na[k].copy_(x["iouts"]["n_accepted"], non_blocking=True)

    def copy_out(k, x, stream, to_host=False):
        na = min(int(h_na[k].item()), max_del, h_dels[k].shape[0])
        with torch.cuda.stream(stream):
            h_dels[k][:na].copy_(x["iouts"]["accepted"][:na], non_blocking=True)
            if not to_host:
                h_rows[k][:na].copy_(x["rows"][:na], non_blocking=True)
                h_rst[k][:na].copy_(x["rst"][:na], non_blocking=True)
        return na

    # the reference: batch by batch on the HBM-resident stream, synchronised
    _reset_caches(rx, True)
    ref = []
    for k, ((a, b), (s0, s1)) in enumerate(zip(cuts, spans)):
        x = S[0]
        compute(k, x, arena[s0:s1], (off_t[a:b] - int(off[a])).contiguous(), ln_t[a:b].contiguous())
        torch.cuda.synchronize(dev)
        na = copy_out(k, x, comp)
        torch.cuda.synchronize(dev)
        ref.append((na, h_dels[k][:na].clone(), h_rows[k][:na].clone(), h_rst[k][:na].clone()))

    def pipelined():
        ev_h2d = [torch.cuda.Event() for _ in range(nb)]
        ev_comp = [torch.cuda.Event() for _ in range(nb)]
        ev_d2h = [torch.cuda.Event() for _ in range(nb)]
        t1 = torch.cuda.Event(enable_timing=True)
        nas = [0] * nb

        def load(k):
            x = S[k % slots]
            (a, b), (s0, s1) = cuts[k], spans[k]
            with torch.cuda.stream(h2d):
                if k >= slots:
                    h2d.wait_event(ev_comp[k - slots])  # the slot's last compute has read its inputs
                x["arena"][:s1 - s0].copy_(host_arena[s0:s1], non_blocking=True)
                x["off"][:b - a].copy_(h_off[k], non_blocking=True)
                x["ln"][:b - a].copy_(h_ln[k], non_blocking=True)
                ev_h2d[k].record(h2d)

        def drain(k):
            ev_comp[k].synchronize()  # (host: this batch's delivery count is in h_na[k])
            x = S[k % slots]
            d2h.wait_event(ev_comp[k])
            nas[k] = copy_out(k, x, d2h, rows_to_host)
            ev_d2h[k].record(d2h)

        load(0)
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record(h2d)  # batch 0 is in: the steady window starts
        for k in range(nb):
            if k + 1 < nb:
                load(k + 1)
            x = S[k % slots]
            (a, b), (s0, s1) = cuts[k], spans[k]
            comp.wait_event(ev_h2d[k])
            if k >= slots:
                comp.wait_event(ev_d2h[k - slots])  # the slot's outputs have left for the host
            compute(k, x, x["arena"][:s1 - s0], x["off"][:b - a], x["ln"][:b - a], rows_to_host)
            ev_comp[k].record(comp)
            if k >= 1:
                drain(k - 1)
                if k == nb - 1:
                    t1.record(d2h)  # batch nb-2 is out: the steady window ends
        drain(nb - 1)
        d2h.synchronize()
        if nb > 1:
            steady.append(t0.elapsed_time(t1) * 1e-3)
        return nas

    times = []
    steady = []  # seconds from batch 0's arrival to batch nb-2's departure: nb-1 batches each way
    ok = True
    nas = []
    for _ in range(reps):
        _reset_caches(rx, True)
        for k in range(nb):  # (the reference's copies stay in ref; every output is rewritten)
            h_rows[k].zero_()
            h_rst[k].fill_(0xff)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        nas = pipelined()
        times.append(time.perf_counter() - t0)
        for k in range(nb):
            na = nas[k]
            r = ref[k]
            ok = ok and na == r[0] and torch.equal(h_dels[k][:na], r[1]) and torch.equal(h_rows[k][:na], r[2]) and \
                torch.equal(h_rst[k][:na], r[3])
    tm = min(times)
    dels = int(sum(nas))
    h2d_bytes = int(sum(e - a for a, e in spans)) + 12 * n
    d2h_bytes = dels * (8 + t.row_bytes + 1) + 8 * nb
    probe = pcie_probe(h2d_bytes, max(d2h_bytes, 1), dev)
    rx.set_topics([], [])
    bound_ms = probe["bound_ms"]
    return {"what": f"{nb} batches of {batch} datagrams streamed host -> device -> host: batch k+1's H2D, batch "
                    "k's parse + ingest + topic caches + CDR rows, batch k-1's D2H on three streams ordered by "
                    "events; proxies and topic caches carry across batches; wall clock, best of "
                    f"{reps}; sample type {CDR_TYPES[workload]}" + (
                        "; rows written by the decode kernel straight into pinned host memory" if rows_to_host else
                        "; deliveries, rows and statuses copied by the copy engine"),
            "rows_to_host": rows_to_host,
            "batches": nb, "batch_datagrams": batch, "slots": slots, "ms": tm * 1e3, "datagrams_per_s": n / tm,
            "steady_state_datagrams_per_s": (n - (cuts[0][1] - cuts[0][0])) / min(steady) if nb > 1 else None,
            "steady_state": "batches 1..nb-1 in and 0..nb-2 out, from batch 0's arrival to batch nb-2's departure "
                            "(HIP events on the copy streams): the pipeline without its fill and drain",
            "deliveries": dels, "deliveries_per_s": dels / tm, "h2d_bytes": h2d_bytes, "d2h_bytes": d2h_bytes,
            "parity_ok": bool(ok), "pcie": probe,
            "pcie_bound_ms": bound_ms, "pcie_bound_datagrams_per_s": n / (bound_ms * 1e-3),
            "frac_of_pcie_bound": bound_ms / (tm * 1e3),
            "steady_frac_of_pcie_bound": ((n - (cuts[0][1] - cuts[0][0])) / min(steady)) /
                                         (n / (bound_ms * 1e-3)) if nb > 1 else None}


def roofline(rx, args, arena, off_t, ln_t, n, outs, stream, total_bytes, alg_reads, alg_writes):
    """SURVEY §8(d) roofline of the dominant parse kernel.  The algorithmic unit is the
    datagram's bytes (Σ lengths) only if every byte streams (FETCH_SIZE >= Σ lengths);
    the parse is zero-copy (payload bytes are never read, like the reference's
    Bytes::split_off), so the fraction is on the FETCH_SIZE basis: calibrated HBM read
    bytes of the kernel per launch (committed PMC summary) / its live launch time /
    8 TB/s.  Writes (the 64-B records) are reported beside it, not in the numerator."""
    ms, kname, extra = time_dominant_kernel(rx, arena, off_t, ln_t, n, outs, stream, args.steps)
    pmc = pmc_profile(args.workload)
    key = PMC_KEYS[kname]
    k = (pmc or {}).get(key) or {}
    scale = (pmc or {}).get("fetch_scale") or 1.0
    if pmc and pmc.get("datagrams_per_launch") == n and "FETCH_SIZE" in k:
        read_b, write_b = k["FETCH_SIZE"] * scale, k.get("WRITE_SIZE")
        basis = f"FETCH_SIZE x fetch_scale of {kname} ({pmc['_source']})"
    else:
        read_b, write_b = float(alg_reads), float(alg_writes)
        basis = "algorithmic head/field reads (no PMC summary for this workload and size)"
    achieved = read_b / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": (read_b + write_b) if write_b is not None else None,
         "read_bytes": read_b, "write_bytes": write_b, "basis": basis,
         "kernel": kname, "kernel_ms": ms,
         "kernel_ms_source": "HIP events on the parse stream around K back-to-back launches of the kernel alone, / K",
         "sum_datagram_bytes": total_bytes,
         "alg_read_bytes": alg_reads, "alg_write_bytes": alg_writes,
         "note": "zero-copy parse: FETCH_SIZE << sum of datagram bytes, so the fraction is on the FETCH basis; "
                 ">= 70 % of HBM read bandwidth is structurally out of reach for a head-only parse (the read-only "
                 "ceiling of this access shape is read_ceiling_frac)"}
    if pmc:
        r["pmc_source"] = pmc["_source"]
    r.update(extra)
    item_pass = "item_kernel_ms" in extra
    if item_pass:
        # the whole item pass E + S + W: calibrated reads of the three launches / their time / peak
        e_ms, sw_ms = extra["item_kernel_ms"], extra["scan_plus_emit_ms"]
        ks = [(pmc or {}).get(PMC_KEYS[x]) or {} for x in ("rtps_parse_item_kernel", "rtps_parse_scan_kernel",
                                                            extra.get("emit_kernel", "rtps_parse_emit_kernel"))]
        if pmc and pmc.get("datagrams_per_launch") == n and all("FETCH_SIZE" in x for x in ks):
            fetch = sum(x["FETCH_SIZE"] for x in ks) * scale
            r["item_pass"] = {"ms": e_ms + sw_ms, "read_bytes": fetch,
                              "write_bytes": sum(x.get("WRITE_SIZE", 0.0) for x in ks),
                              "frac": fetch / ((e_ms + sw_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS,
                              "kernels": "rtps_parse_item_kernel + rtps_parse_scan_kernel + " + extra["emit_kernel"]}
            r["item_pass_frac"] = r["item_pass"]["frac"]
    if kname == "rtps_parse_chain_kernel" or item_pass:
        torch.cuda.synchronize()
        n_rec = int(outs["n_records"].item())
        c = time_hops_ceilings(arena, off_t, ln_t, n, outs, n_rec, stream, args.steps)
        if c:
            r["ceiling"] = {"kernel": "diag ceil_hops_kernel (csrc/diag/ceiling.hip): the same dependent header "
                                      "hops per datagram + a 64-B record store per materialised submessage at the "
                                      "parse's positions, no field decode",
                            "one_walk_ms": c[1], "two_walk_ms": c[2]}
            # same-shape one-walk floor / the parse's kernel time (the item pass: all three launches)
            pm = extra["item_kernel_ms"] + extra["scan_plus_emit_ms"] if item_pass else ms
            r["attainable_frac"] = c[1] / pm
            r["attainable_frac_two_walk"] = c[2] / pm
    if kname == "rtps_parse_spec_kernel":
        c = time_ceilings(arena, off_t, ln_t, n, stream, args.steps)
        if c:
            ceil_read = n * (12 + 64)  # the read-only ceiling's bytes: exact, its own shape
            r["ceiling"] = {"kernel": "diag ceil_kernel (csrc/diag/ceiling.hip)", "read_only_ms": c["read_only"],
                            "read_write_ms": c["read_write"],
                            "read_only_gbs": ceil_read / (c["read_only"] * 1e-3) / 1e9}
            r["read_ceiling_frac"] = r["ceiling"]["read_only_gbs"] / HBM_PEAK_GBS
            r["attainable_frac"] = c["read_write"] / ms  # same-shape read+write ceiling time / kernel time
    return r


CDR_TYPES = {"T": "TSample", "C2": "C2Sample", "C3": "ShapeType", "C4": "C2Sample"}


def _time_launches(fn, stream, steps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)  # back-to-back launches, one event pair (see main's timed loop)
    for _ in range(steps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def cdr_decode_leg(rx, workload, arena, off_t, outs, n_rec, stream, steps, iouts=None):
    """a18: batch CDR decode of this batch's samples into fixed-layout rows, timed separately
    from the parse step (HIP events on the launch stream).  With the ingest's deliveries
    (iouts) the rows are COMPACT: one per sample that entered a history cache
    (rtps_rx_cdr_decode_list over the delivery list), as the reference decodes only the
    samples a DataReader takes; the per-record layout (a row per record, zero rows for the
    records that are not samples) is timed beside it."""
    from rtps_rx import cdr
    t = getattr(cdr, CDR_TYPES[workload])
    rows, row_status = rx.alloc_rows(t, n_rec)
    ms_rec = _time_launches(lambda: rx.cdr_decode(t, arena, off_t, outs, rows, row_status), stream, steps)
    st = row_status[:n_rec].cpu().numpy()
    ok = int((st == cdr.CDR_OK).sum())
    # algorithmic bytes: 40 B of each record read, 1 status byte + one row written per record,
    # and for decoded rows the value bytes consumed (= row_bytes for these all-primitive types)
    alg_rec = n_rec * (40 + 1 + t.row_bytes) + ok * t.row_bytes
    if ok == 0:  # nothing decoded (e.g. C4: its samples are DATA_FRAG, decoded after reassembly): no rate
        return {"sample_type": CDR_TYPES[workload], "records": n_rec, "decoded_ok": 0,
                "status_hist": np.bincount(st, minlength=7).tolist(),
                "note": "no DATA record of this batch decodes as this type, so no rate is reported"}
    per_record = {"layout": "a row per record (rtps_rx_cdr_decode)", "kernel_ms": ms_rec, "rows": n_rec,
                  "alg_bytes_per_launch": alg_rec, "achieved_gbs": alg_rec / (ms_rec * 1e-3) / 1e9,
                  "frac": alg_rec / (ms_rec * 1e-3) / 1e9 / HBM_PEAK_GBS}
    r = {"sample_type": CDR_TYPES[workload], "row_bytes": t.row_bytes, "records": n_rec, "decoded_ok": ok,
         "status_hist": np.bincount(st, minlength=7).tolist(), "kernel": "cdr_decode_kernel"}
    if iouts is None:
        r.update({"layout": per_record["layout"], "kernel_ms": ms_rec, "rows_per_s": ok / (ms_rec * 1e-3),
                  "alg_bytes_per_launch": alg_rec, "achieved_gbs": per_record["achieved_gbs"],
                  "frac": per_record["frac"]})
        return r
    na = int(iouts["n_accepted"].item())
    lrows, lst = rx.alloc_rows(t, max(na, 1))
    ms = _time_launches(lambda: rx.cdr_decode_list(t, arena, off_t, outs, iouts["accepted"], 8, iouts["n_accepted"],
                                                   na, lrows, lst), stream, steps)
    lsv = lst[:na].cpu().numpy()
    lok = int((lsv == cdr.CDR_OK).sum())
    # compact rows: 8 B of delivery + 40 B of its record read, the value bytes consumed, one row
    # + 1 status byte written per delivery
    alg = na * (8 + 40 + 1 + t.row_bytes) + lok * t.row_bytes
    r.update({"layout": "compact: a row per delivery (rtps_rx_cdr_decode_list over the ingest's deliveries)",
              "rows": na, "rows_ok": lok, "kernel_ms": ms, "rows_per_s": lok / (ms * 1e-3),
              "alg_bytes_per_launch": alg, "achieved_gbs": alg / (ms * 1e-3) / 1e9,
              "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "per_record_layout": per_record})
    return r


def frag_leg(rx, arena, off_t, outs, n_rec, recs, stream, steps):
    """DataFrag reassembly of this batch's DATA_FRAG records (§8f rank 1), timed
    separately (HIP events on the launch stream).  Each step re-assembles the same
    batch from a reset state, so every step does the same work."""
    u = recs["u"].view(np.uint8).reshape(-1, 16)
    frag = recs["kind"] == DATA_FRAG
    payload = int(u[frag][:, 2:4].copy().view("<u2").astype(np.int64).sum())
    heap_bytes = int(arena.numel()) + 16 * n_rec + (1 << 24)
    fouts = rx.alloc_frag_outputs(n_rec, heap_bytes)
    for _ in range(2):
        rx.frag_reset()
        rx.frag_assemble(arena, off_t, outs, fouts)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        rx.frag_reset()
        a.record(stream)
        rx.frag_assemble(arena, off_t, outs, fouts)
        b.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ns = int(fouts["n_samples"].item())
    # algorithmic bytes: each fragment's payload read once and written once + its 64-B record read
    alg = 2 * payload + 64 * int(frag.sum())
    return fouts, {"kernel": "rtps_frag_assemble (sort + walk + place + copy launches)", "ms": ms,
            "samples": ns, "pending": int(fouts["n_pending"].item()), "fragments": int(frag.sum()),
            "samples_per_s": ns / (ms * 1e-3), "gib_per_s_assembled": int(fouts["heap_used"].item()) / (ms * 1e-3) / 2**30,
            "alg_bytes_per_launch": alg, "achieved_gbs": alg / (ms * 1e-3) / 1e9,
            "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


XGMI_LINK_GBS = 153.0  # one xGMI link, one direction (8-GPU node: one link per peer pair, 7 per GPU)


def exchange_prediction(rx, arena, off_t, outs, dev, worlds=(2, 4, 8)):
    """What the owner-side exchange of THIS batch would move at N ranks (weak scaling: every
    rank parses a batch like this one): the library's pack with n_ranks = N, its per-destination
    counts (16-B items + blob bytes), the bytes each rank sends to its peers per step and the
    xGMI time they take at the link rate (every peer on its own link, all in parallel: the
    largest per-peer volume bounds the round)."""
    from rtps_rx.shard import OwnerShard, ITEM_BYTES_OWNER
    out = {}
    for w in worlds:
        sh = OwnerShard(rx, w, None, dev, 1, 0)
        try:
            sh.pack(arena, off_t, outs)
            c = sh.counts("send")
        finally:
            sh.close()
        n, b = c["n"].astype(np.int64), c["bytes"].astype(np.int64)
        # rank 0's view: destination 0 stays local; the others cross a link each
        peer = ITEM_BYTES_OWNER * n[1:] + b[1:] + 32  # items, blobs, the 32-B counts
        out[str(w)] = {"items_per_dest": [int(v) for v in n], "blob_bytes_per_dest": [int(v) for v in b],
                       "bytes_sent_per_rank_per_step": int(peer.sum()),
                       "max_bytes_per_peer": int(peer.max()),
                       "predicted_xgmi_ms": float(peer.max()) / (XGMI_LINK_GBS * 1e9) * 1e3}
    return {"what": "owner-side exchange volume of this batch at N ranks (rank 0's sends; library pack with "
                    "n_ranks = N on this GPU), predicted round time at one xGMI link per peer",
            "link_gbs": XGMI_LINK_GBS, "item_bytes": ITEM_BYTES_OWNER, **out}


def time_ingest_ceiling(outs, n_rec, n_sets, stream, steps):
    """Live timing of the ingest's same-shape floor (csrc/diag/ceiling.hip ceil_ingest_kernel):
    every 64-B record read, 1 accept byte written; per event (a matched DATA / HEARTBEAT / GAP)
    its proxy's 8-B state read and a 4-B change-set word OR-ed at its SN's bit; per delivery
    (a matched DATA) 8 B appended.  None if the diagnostic library is absent."""
    import ctypes
    path = os.path.join(REPO, "rustdds-io_uring_amd", "libdiag_ceiling.so")
    if not os.path.exists(path):
        return None
    D = ctypes.CDLL(path)
    D.diag_ceiling_ingest.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 5 + \
        [ctypes.c_uint32, ctypes.c_void_p]
    dev = outs["records"].device
    n_sets = max(n_sets, 1)
    state = torch.zeros(n_sets, dtype=torch.int64, device=dev)
    bits = torch.zeros(n_sets * (1 << 17) // 32, dtype=torch.int32, device=dev)
    accept = torch.empty(max(n_rec, 1), dtype=torch.uint8, device=dev)
    dels = torch.empty(max(n_rec, 1), dtype=torch.int64, device=dev)
    n_del = torch.zeros(1, dtype=torch.int64, device=dev)

    def run():
        D.diag_ceiling_ingest(outs["records"].data_ptr(), outs["target"].data_ptr(), n_rec, state.data_ptr(),
                              bits.data_ptr(), accept.data_ptr(), dels.data_ptr(), n_del.data_ptr(), n_sets,
                              ctypes.c_void_p(stream.cuda_stream))
    return _time_launches(run, stream, steps)


def _reset_caches(rx, topic_cache):
    rx.ingest_reset()
    if topic_cache:
        rx.topic_reset()


def _time_ingest(rx, arena, off_t, outs, iouts, fa, stream, steps, topic_cache):
    """Mean HIP-event time of one ingest launch sequence; every step starts from fresh writer
    proxies (and, with the topic caches, empty caches): the resets are outside the events."""
    for _ in range(2):
        _reset_caches(rx, topic_cache)
        rx.ingest(arena, off_t, outs, iouts, *fa, topic_cache=topic_cache)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        _reset_caches(rx, topic_cache)
        a.record(stream)
        rx.ingest(arena, off_t, outs, iouts, *fa, topic_cache=topic_cache)
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def ingest_leg(rx, arena, off_t, outs, n_rec, recs, n_entries, stream, steps, fouts=None):
    """History-cache ingest (§8f rank 2) of this batch's samples / HEARTBEATs / GAPs,
    timed separately (HIP events on the launch stream).  Every step starts from
    fresh writer proxies (the reset is outside the timed region), so every step
    does the same work: all first copies accepted.  fouts: the batch's reassembled
    DataFrag samples (C4), ingested at their completing records.  Timed again with the
    topic caches (RTPS_INGEST_TOPIC_CACHE: TopicCache::add_change of every delivery, the
    subscribed reader's topic with max_keep 64, emptied before each step): topic_cache_ms."""
    iouts = rx.alloc_ingest_outputs(n_rec, n_entries)
    fa = (fouts,) if fouts is not None else ()
    rx.set_topics([(1, 64)], [(0, 1)])  # the bench's reader (slot 0) on one topic
    ms_tc = _time_ingest(rx, arena, off_t, outs, iouts, fa, stream, steps, True)
    torch.cuda.synchronize()
    cached = int(((iouts["accepted"][:int(iouts["n_accepted"].item())].reshape(-1, 8)[:, 6] & 1) != 0).sum().item())
    ms = _time_ingest(rx, arena, off_t, outs, iouts, fa, stream, steps, False)
    rx.set_topics([], [])  # (no topic configured: the owner tables of the legs below deal writers, not topics)
    na = int(iouts["n_accepted"].item())
    k = recs["kind"]
    events = int((((recs["route"] & 0x21) == 0x21) & np.isin(k, (DATA, HEARTBEAT, GAP))).sum())
    if fouts is not None:  # + the completed DataFrag samples
        events += int(fouts["n_samples"].item())
    # algorithmic bytes: every record read once (64 B), 1 accept byte written per record, 8 B per
    # delivery, per event 8 B of proxy state read and 4 B of change-set bits touched
    alg = n_rec * (64 + 1) + 8 * na + 12 * events
    ceil_ms = time_ingest_ceiling(outs, n_rec, n_entries, stream, steps)
    ceil = None if ceil_ms is None else {
        "kernel": "diag ceil_ingest_kernel (csrc/diag/ceiling.hip): each 64-B record read, 1 accept byte; per event "
                  "8 B of proxy state + a 4-B change-set word at its SN; per delivery 8 B appended",
        "ms": ceil_ms, "attainable_frac": ceil_ms / ms}
    return iouts, {"kernel": "rtps_ingest (classify + heartbeat sort/scans + marks + decide + select + merge + state)",
            "ms": ms, "topic_cache_ms": ms_tc, "topic_cache_extra_ms": ms_tc - ms,
            "ceiling": ceil, "attainable_frac": None if ceil is None else ceil["attainable_frac"],
            "topic_cache_stored": cached,
            "records": n_rec, "events": events, "accepted": na,
            "samples_per_s": na / (ms * 1e-3), "records_per_s": n_rec / (ms * 1e-3),
            "window_overflow": int(iouts["n_window_overflow"].item()),
            "alg_bytes_per_launch": alg, "achieved_gbs": alg / (ms * 1e-3) / 1e9,
            "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


SPDP_READER = bytes([0x00, 0x01, 0x00, 0xC7])  # EntityId::SPDP_BUILTIN_PARTICIPANT_READER (DUPLICATES_OK)


def spdp_repeat_batch(n, pattern):
    """n datagrams of one DATA each (52 B in 64-B slots) from one user writer to the SPDP
    participant reader, SNs with >= 50 % repeats: 'pairs' = every SN twice in a row (i // 2 + 1),
    'halves' = the second half repeats the first (i % (n / 2) + 1)."""
    import struct
    prefix = bytes([0xB0] * 12)
    writer = bytes([0, 0, 1, 0x02])
    body = struct.pack("<HH", 0, 16) + bytes(4) + writer + bytes(8) + b"\x00\x01\x00\x00abcd"
    dg = b"RTPS\x02\x04\x01\x0f" + prefix + bytes([0x15, 0x05]) + struct.pack("<H", len(body)) + body
    slot = 64
    tmpl = np.frombuffer(dg.ljust(slot, b"\0"), dtype=np.uint8)
    arena = np.tile(tmpl, n)
    i = np.arange(n, dtype=np.int64)
    sn = (i // 2 + 1) if pattern == "pairs" else (i % (n // 2) + 1)
    a = arena.reshape(n, slot)
    a[:, 36:40] = (sn >> 32).astype("<i4").view(np.uint8).reshape(n, 4)   # SN high (i32), then low (u32)
    a[:, 40:44] = (sn & 0xFFFFFFFF).astype("<u4").view(np.uint8).reshape(n, 4)
    off = (i * slot).astype(np.uint64)
    ln = np.full(n, len(dg), dtype=np.uint32)
    return arena, off, ln, prefix + writer


def spdp_repeats_leg(dev, stream, steps, n=1 << 20):
    """The topic caches' adversarial case: the SPDP participant reader
    accepts duplicates (reader.rs:712-722), so every delivery of its topic is a candidate and
    the repeats of a key stored earlier in the batch are decided in order by one thread per
    topic (tc_resolve).  1M datagrams, one topic (max_keep 64), >= 50 % repeated SNs; the
    ingest timed with and without RTPS_INGEST_TOPIC_CACHE (fresh proxies and caches each
    step), and the CACHED decisions checked against the reference's add_change restated: a
    change is stored iff its (writer, SN) is not held at that moment."""
    from rtps_rx.records import Readers
    out = {}
    rx = rtps_rx.MessageReceiver(OWN_PREFIX, device=dev.index, max_datagrams=n)
    rx.set_stream(stream)
    try:
        for pattern in ("pairs", "halves"):
            arena_np, off, ln, guid = spdp_repeat_batch(n, pattern)
            arena = torch.from_numpy(arena_np).to(dev)
            off_t = torch.from_numpy(off.view(np.int64)).to(dev)
            ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
            rx.set_readers(Readers([(SPDP_READER, 14, 0)], [(guid, 0)]))
            rx.set_topics([(9, 64)], [(14, 9)])
            outs = rx.alloc_outputs(n, n)
            rx.parse_batch_device(arena, off_t, ln_t, n, outs)
            iouts = rx.alloc_ingest_outputs(n, 1)
            ms_tc = _time_ingest(rx, arena, off_t, outs, iouts, (), stream, steps, True)
            torch.cuda.synchronize()
            na = int(iouts["n_accepted"].item())
            flags = iouts["accepted"][:na].reshape(-1, 8)[:, 6].cpu().numpy() & 1
            ms = _time_ingest(rx, arena, off_t, outs, iouts, (), stream, steps, False)
            # add_change restated (dds_cache.rs:221-276): GC at SN % 64 == 0 keeps the 64 newest,
            # then store iff not held (insertion order = receive order)
            sn = ((np.arange(n) // 2 + 1) if pattern == "pairs" else (np.arange(n) % (n // 2) + 1)).tolist()
            held, order, exp = set(), [], np.zeros(n, np.uint8)
            from collections import deque
            order = deque()
            for k, x in enumerate(sn):
                if x % 64 == 0:
                    while len(order) > 64:
                        held.discard(order.popleft())
                if x not in held:
                    held.add(x)
                    order.append(x)
                    exp[k] = 1
            out[pattern] = {"datagrams": n, "deliveries": na, "repeats": int(n - len(set(sn))),
                            "stored": int(flags.sum()), "parity_ok": bool(na == n and np.array_equal(flags, exp)),
                            "ingest_ms": ms, "ingest_topic_cache_ms": ms_tc, "topic_cache_extra_ms": ms_tc - ms}
    finally:
        rx.close()
    return {"what": "SPDP participant reader (DUPLICATES_OK), one topic, max_keep 64: every delivery a candidate, "
                    ">= 50 % of them repeats of keys stored earlier in the batch (tc_resolve, one thread per topic)",
            **out}


HELLO_PREFIX = bytes([0x01, 0x0f, 0x99, 0x06, 0x78, 0x34, 0x00, 0x00, 0x01, 0x00, 0x00, 0x00])
HELLO_WRITER = bytes([0x00, 0x00, 0x01, 0x02])


def hello_world_datagrams(n):
    """C1 traffic: what examples/io_uring_hello_world_publisher.rs writes (HelloWorldData
    {user_id: i32, message: String}, :13-16, written at :162), as 64-byte serialized samples:
    RTPS header + INFO_TS + one DATA per datagram (120 B), one writer, SN 1..n."""
    L = 120
    t = bytearray(L)
    t[0:20] = b"RTPS\x02\x04\x01\x0f" + HELLO_PREFIX
    t[20:24] = bytes([0x09, 0x01, 8, 0])                       # INFO_TS, LE, 8 bytes
    t[32:36] = bytes([0x15, 0x05, 84, 0])                      # DATA, LE + D, 20 + 64 bytes
    t[36:40] = bytes([0, 0, 16, 0])                            # extraFlags, octetsToInlineQos
    t[44:48] = HELLO_WRITER                                    # readerId UNKNOWN (40:44), writerId
    t[56:60] = bytes([0x00, 0x01, 0x00, 0x00])                 # CDR_LE encapsulation
    t[64:68] = (52).to_bytes(4, "little")                      # string length incl. NUL
    t[68:119] = b"Hello World! ".ljust(51, b".")
    a = np.tile(np.frombuffer(bytes(t), dtype=np.uint8), (n, 1))
    i = np.arange(n, dtype=np.int64)
    a[:, 24:28] = (1_700_000_000 + i // 1000).astype("<u4").view(np.uint8).reshape(n, 4)
    a[:, 28:32] = ((i % 1000) * 4294967).astype("<u4").view(np.uint8).reshape(n, 4)
    sn = i + 1
    a[:, 48:52] = (sn >> 32).astype("<i4").view(np.uint8).reshape(n, 4)
    a[:, 52:56] = (sn & 0xFFFFFFFF).astype("<u4").view(np.uint8).reshape(n, 4)
    a[:, 60:64] = (i % 1000).astype("<i4").view(np.uint8).reshape(n, 4)   # user_id
    digits = np.char.zfill((i % 10**8).astype(str), 8).astype("S8")
    a[:, 81:89] = np.frombuffer(digits.tobytes(), dtype=np.uint8).reshape(n, 8)
    return a.reshape(-1), (np.arange(n, dtype=np.uint64) * L), np.full(n, L, dtype=np.uint32)


def c1_loopback(dev, stream, n=200_000, batch=16384, publishers=1):
    """Config C1 (BASELINE.json configs[0]): hello-world publisher -> subscriber over UDP
    loopback, 64-B samples.  Publisher: sendmmsg on a thread, flow-controlled to two batches
    ahead of the subscriber (an unthrottled loopback sender outruns any receiver: what gets
    through is then set by the socket buffer, not by the pipeline).  Subscriber: the native
    receive loop (rtps_rx_pump): io_uring lands datagrams in slots of a pinned arena, and each
    batch is parsed in place by the GPU (zero-copy), ingested into the history cache and
    CDR-decoded, two batches in flight.  Loopback and the kernel bound the rate; dropped
    datagrams (socket buffer overruns) are reported, never hidden."""
    import threading
    from rtps_rx import udp, cdr
    hello_t = cdr.CdrType([("user_id", "i32"), ("message", cdr.String(60))])
    data, off, ln = hello_world_datagrams(n)
    slot, nslot = 256, 32768
    arena = torch.zeros(slot * nslot, dtype=torch.uint8, pin_memory=True)
    rxu = udp.UdpReceiver(arena, slot_bytes=slot, rcvbuf_bytes=64 << 20)
    rx = rtps_rx.MessageReceiver(OWN_PREFIX, device=dev.index, max_datagrams=batch)
    rx.set_stream(stream)
    tbl = np.zeros(1, dtype=MATCH_DTYPE)
    tbl["writer_guid"][0] = np.frombuffer(HELLO_PREFIX + HELLO_WRITER, dtype=np.uint8)
    rx.set_match_table(tbl)
    pump = udp.Pump(rx, rxu, max_batch=batch, ingest=True, sample_type=hello_t, max_recs=2 * batch, n_entries=1)
    live = pump.stats
    sent = [0]
    window = 2 * batch

    send_s = [0.0, 0.0]  # time inside sendmmsg, time waiting on flow control (summed over publishers)
    lock = threading.Lock()

    def sender(p):
        # publisher p of `publishers` sends chunks p, p+publishers, ... (one writer: with several
        # publishers its SNs arrive out of order, none twice, so every sample is still accepted)
        chunk = 4096
        for a in range(p * chunk, n, chunk * publishers):
            w0 = time.perf_counter()
            while sent[0] - live.datagrams > window:
                time.sleep(0.0002)
            b = min(n, a + chunk)
            s0 = time.perf_counter()
            k = udp.send_batch("127.0.0.1", rxu.port, data, off[a:b], ln[a:b])
            s1 = time.perf_counter()
            with lock:
                sent[0] += k
                send_s[0] += s1 - s0
                send_s[1] += s0 - w0

    decoded = [0]

    def on_batch(b):
        m = min(b.n_records, pump.cap)
        decoded[0] += int((b.row_status[:m] == cdr.CDR_OK).sum().item())
        return False

    ths = [threading.Thread(target=sender, args=(p,), daemon=True) for p in range(publishers)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    st = pump.run(wait_ms=5, stop_after=n, idle_stop_ms=2000, on_batch=on_batch)
    wall = time.perf_counter() - t0
    for t in ths:
        t.join(timeout=5)
    received = st.datagrams
    busy = (st.last_ns - st.first_ns) / 1e9 if st.batches else float("nan")  # first batch .. last finished
    rxu.close()
    rx.close()
    # the CPU reference parse of the same datagrams (oracle, one thread), for scale
    import oracle
    c0 = time.perf_counter()
    oracle.parse(data, off, ln, threads=1)
    cpu_s = time.perf_counter() - c0
    return {"config": "C1: hello-world publisher -> subscriber over UDP loopback, 64-B HelloWorldData samples",
            "receive_backend": {udp.IO_URING: "io_uring", udp.IO_URING_SQPOLL: "io_uring+sqpoll",
                                udp.RECVMMSG: "recvmmsg"}[rxu.backend],
            "loop": "native rtps_rx_pump, 2 batches in flight", "publishers": publishers,
            "datagrams_built": n, "datagrams_sent": sent[0], "datagrams_received": received,
            "dropped": sent[0] - received, "batches": st.batches,
            "samples_accepted": st.accepted, "samples_decoded": decoded[0], "wall_s": wall, "stream_s": busy,
            "datagrams_per_s": received / busy, "publisher_sendmmsg_s": send_s[0],
            "publisher_flow_wait_s": send_s[1], "cpu_reference_parse_per_s_1_thread": n / cpu_s}


def host_cpus():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota
    (a GPU box grants each GPU a share of the host: os.cpu_count() is the machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota}


def cpu_baseline(workload, n, match_table=None, samples=5, min_sample_s=0.25):
    """The oracle (C restatement of the reference parse) on this host's cores, with the
    same readers as the device run: all usable cores (contiguous slices, one thread
    each) and one thread; median of `samples` timed samples each.
    A sample repeats the full batch until it has run `min_sample_s`."""
    import oracle
    threads, cpus = host_cpus()
    arena, off, ln = oracle.gen(rtps_rx.WORKLOADS[workload], n)

    def rate(th, k):
        o, l = off[:k], ln[:k]
        oracle.parse(arena, o, l, threads=th, want_targets=False, match_table=match_table)  # warm
        rates = []
        for _ in range(samples):
            t0 = time.perf_counter()
            reps = 0
            while True:
                oracle.parse(arena, o, l, threads=th, want_targets=False, match_table=match_table)
                reps += 1
                if time.perf_counter() - t0 >= min_sample_s:
                    break
            rates.append(reps * k / (time.perf_counter() - t0))
        return float(np.median(rates)), rates

    v_all, r_all = rate(threads, n)
    v_one, r_one = rate(1, n)
    return {"value": v_all, "unit": "datagrams/s", "cores": threads, "kind": "port",
            "host": cpus,
            "sample": f"full {workload} batch ({n} datagrams, generated on host), oracle/rtps_oracle.c on "
                      f"{threads} threads (contiguous slices), median of {samples} samples of >= {min_sample_s} s",
            "samples": r_all,
            "single_thread": {"value": v_one, "unit": "datagrams/s", "cores": 1,
                              "sample": f"the same batch on 1 thread, median of {samples}", "samples": r_one}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default=None, choices=sorted(rtps_rx.WORKLOADS) + ["C5"],
                    help="default: T at every N (the headline config; N>1 adds the owner exchange and a C5 "
                         "measurement, BASELINE config 8xMI355X, as `c5`)")
    ap.add_argument("--datagrams", type=int, default=None, help="datagrams per GPU (default 1M; C5: 64M / N)")
    ap.add_argument("--writers", type=int, default=16)
    ap.add_argument("--spec-hint", type=int, default=None,
                    help="rtps_rx_set_spec_hint (records per datagram; 0 = mixed traffic, chained launch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-cdr", action="store_true", help="skip the CDR decode (a18) measurement")
    ap.add_argument("--no-frag", action="store_true", help="skip the DataFrag reassembly measurement (C4)")
    ap.add_argument("--no-ingest", action="store_true", help="skip the history-cache ingest measurement")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 UDP-loopback pipeline measurement")
    ap.add_argument("--match", default="writers", choices=["writers", "none"],
                    help="match table: every writer of the workload (a reader subscribed to all of them) or none")
    ap.add_argument("--exchange", default="owner", choices=["owner", "records", "descriptors"],
                    help="N>1: what crosses xGMI: 'owner' (default) = every writer record that passes, with its "
                         "GAP bitmap / DATA_FRAG payload, to its writer's owner (writer-GUID hash % N), unpacked "
                         "there for reassembly and ingest; 'records' = the 64-B records of every writer / reader "
                         "submessage; 'descriptors' = 16-B descriptors of MATCHED records")
    ap.add_argument("--no-owner-ingest", action="store_true",
                    help="N>1 / C5: skip the second timed loop that adds the owners' history-cache ingest")
    ap.add_argument("--no-c5", action="store_true",
                    help="N>1: skip the C5 measurement (64M datagrams in total) that follows the T line")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (gloo only to rehearse several ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)

    def allreduce_sum(x):
        if dist is None:
            return x
        if args.backend == "gloo":
            y = x.cpu()
            dist.all_reduce(y)
            return y.to(x.device)
        dist.all_reduce(x)
        return x

    def allreduce_max(x):
        if dist is None:
            return x
        if args.backend == "gloo":
            y = x.cpu()
            dist.all_reduce(y, op=dist.ReduceOp.MAX)
            return y.to(x.device)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return x

    # the headline config at every N (weak scaling: 1M T datagrams per GPU, plus the owner-side
    # exchange at N >= 2), so that the 1/2/4/8-GPU lines measure one workload; BASELINE's
    # 8-GPU config C5 (64M datagrams in total: strong scaling) rides along at N >= 2 as `c5`
    explicit = args.workload is not None
    args.workload = args.workload or "T"
    result = measure(args, world, rank, dist, dev, allreduce_sum, allreduce_max)
    if world > 1 and not explicit and not args.no_c5:
        a5 = argparse.Namespace(**vars(args))
        a5.workload = "C5"  # (--datagrams, when given, sizes both: tests)
        a5.steps, a5.warmup = min(args.steps, 20), min(args.warmup, 5)
        try:  # the T line above is the measurement; a C5 failure is reported inside it, not instead of it
            r5 = measure(a5, world, rank, dist, dev, allreduce_sum, allreduce_max)
            result["c5"] = {k: r5[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "scaling",
                                              "gib_per_s_covered", "config", "pipeline_with_ingest") if k in r5}
        except (RuntimeError, ValueError, MemoryError) as ex:
            result["c5"] = {"error": f"{type(ex).__name__}: {str(ex)[:300]}"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        from rtps_rx.shard import destroy_comms
        destroy_comms()  # the library's RCCL communicators, before the process group goes
        dist.destroy_process_group()


def measure(args, world, rank, dist, dev, allreduce_sum, allreduce_max):
    """One workload at this N: the timed steps and (N = 1) the downstream legs; returns the line."""
    c5 = args.workload == "C5"
    wl = rtps_rx.WL_C3 if c5 else rtps_rx.WORKLOADS[args.workload]
    n = args.datagrams or ((C5_TOTAL // world) if c5 else 1 << 20)
    if c5:  # the C5 batch is the C3 mix; what is not a parse / exchange measurement is skipped
        args.no_cdr = args.no_frag = args.no_ingest = args.no_c1 = args.no_e2e = True

    # ---- input: this rank's chunk of the synthetic stream, generated in HBM ----
    off, ln, size = rtps_rx.gen_layout(wl, n, first_idx=rank * n, n_writers=args.writers)
    rx = rtps_rx.MessageReceiver(OWN_PREFIX, device=dev.index, max_datagrams=n)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    rx.set_stream(stream)
    if args.spec_hint is not None:
        rx.set_spec_hint(args.spec_hint)
    arena = torch.empty(size, dtype=torch.uint8, device=dev)
    off_t = torch.from_numpy(off.view(np.int64)).to(dev)
    ln_t = torch.from_numpy(ln.view(np.int32)).to(dev)
    rx.generate(wl, arena, off_t, ln_t, n, first_idx=rank * n, n_writers=args.writers)

    # size the record buffer from a first parse of this batch (the count is a
    # property of the input; the kernel never writes past max_records)
    probe = rx.alloc_outputs(n, 1)
    rx.parse_batch_device(arena, off_t, ln_t, n, probe)
    torch.cuda.synchronize(dev)
    n_rec = int(probe["n_records"].item())
    outs = rx.alloc_outputs(n, n_rec)
    del probe
    n_matched_writers = 0
    tbl = None
    if args.match == "writers" or (world > 1 and args.exchange in ("descriptors", "owner")):
        # the reader is subscribed to every writer of the stream: match table = the writer
        # GUIDs found in this batch, sorted (the same table, in the same order, on every rank)
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        torch.cuda.synchronize(dev)
        r = outs["records"][:min(n_rec, 1 << 22)].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        wk = np.isin(r["kind"], [DATA, DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP])
        g = np.concatenate([r["prefix"][wk], r["writer_id"][wk]], axis=1)
        guids = np.unique(g.view(np.dtype((np.void, 16))).reshape(-1))
        tbl = np.zeros(len(guids), dtype=MATCH_DTYPE)
        tbl["writer_guid"] = np.frombuffer(guids.tobytes(), dtype=np.uint8).reshape(-1, 16)
        rx.set_match_table(tbl)
        n_matched_writers = len(guids)
    exch = None
    shards = None
    works = [[], []]
    bcap = 0
    owner = world > 1 and args.exchange == "owner"
    if world > 1 and not owner:
        # Record / descriptor exchange (round 2's path): two buffer sets; the equal-split
        # all-to-all of batch k (padded buckets, counts alongside, no host round trip) runs
        # on the RCCL stream while batch k+1 is parsed.  Bucket capacity = the largest bucket
        # of this batch over all ranks (the batch repeats every step, so it never overflows;
        # overflow is checked after the timed region).
        from rtps_rx.shard import Exchange
        item = args.exchange
        probe_ex = Exchange(rx, n_rec, world, dist, dev, cap=max(n_rec, 1) if item == "descriptors" else None,
                            item=item)
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        probe_ex.bucket(outs)
        bcap = max(int(allreduce_max(probe_ex.counts.max().reshape(1)).item()), 1)
        del probe_ex
        exch = [Exchange(rx, n_rec, world, dist, dev, cap=bcap, item=item) for _ in range(2)]
        outs_pp = [outs, rx.alloc_outputs(n, n_rec)]
    slot = (0, 0)
    owned = [None, None]
    iouts = None
    if owner:
        # Owner-side exchange (rtps_rx_shard_*): every writer record that passes goes to its
        # writer's owner with its GAP bitmap / DATA_FRAG payload bytes.  Slots sized from a
        # first pack of this batch (largest (source, owner) pair over all ranks); anything
        # that does not fit would cross in the exact spill round, never be dropped.
        from rtps_rx.shard import OwnerShard, ITEM_BYTES_OWNER
        probe_sh = OwnerShard(rx, world, dist, dev, 1, 0)
        rx.parse_batch_device(arena, off_t, ln_t, n, outs)
        probe_sh.pack(arena, off_t, outs)
        c = probe_sh.counts("send")
        probe_sh.close()
        mx = allreduce_max(torch.tensor([int(c["n"].max()), int(c["bytes"].max())], dtype=torch.int64, device=dev))
        slot = (max(int(mx[0].item()), 1), int(mx[1].item()))
        shards = [OwnerShard(rx, world, dist, dev, slot[0], slot[1]) for _ in range(2)]
        outs_pp = [outs, rx.alloc_outputs(n, n_rec)]
    pending = [False, False]
    with_ingest = [False]

    def owner_ingest(b):
        """The owner's history-cache ingest of what batch b delivered to it (fresh writer proxies
        each step, so every step does the same work: all first copies accepted)."""
        nonlocal iouts
        ob = owned[b]
        if iouts is None or iouts["accept"].numel() < max(ob.n_records, 1):
            iouts = rx.alloc_ingest_outputs(max(ob.n_records, 1), n_matched_writers)
        rx.ingest_reset()
        rx.ingest(ob.arena, ob.off, ob.outs, iouts)

    def drain(b):
        if pending[b]:
            shards[b].finish()
            owned[b] = shards[b].unpack()
            pending[b] = False
            if with_ingest[0]:
                owner_ingest(b)

    def step(k):
        if world == 1:
            rx.parse_batch_device(arena, off_t, ln_t, n, outs)
            if with_ingest[0]:
                if iouts is None:
                    owner_ingest_n1()
                rx.ingest_reset()
                rx.ingest(arena, off_t, outs, iouts)
            return
        b = k & 1
        if owner:
            # batch k: parse + pack on the compute stream; meanwhile the host finishes batch
            # k-1 (its round 0 ran on the RCCL stream during this parse) and unpacks it for its
            # owners; then round 0 of batch k goes out
            rx.parse_batch_device(arena, off_t, ln_t, n, outs_pp[b])
            shards[b].pack(arena, off_t, outs_pp[b])
            drain(1 - b)
            shards[b].exchange()
            pending[b] = True
            return
        for w in works[b]:  # the exchange that last used buffer set b is done
            w.wait()
        rx.parse_batch_device(arena, off_t, ln_t, n, outs_pp[b])
        exch[b].bucket(outs_pp[b])
        works[b] = exch[b].exchange_async()

    def owner_ingest_n1():
        nonlocal iouts
        iouts = rx.alloc_ingest_outputs(max(n_rec, 1), n_matched_writers)

    def timed(steps, warmup):
        for k in range(warmup):
            step(k)
        if owner:  # the warmup's last batch is finished before the clock starts
            drain(0)
            drain(1)
        # One event pair around the whole timed region, on the parse stream: an event
        # recorded between steps costs each step 7-11 us of dispatch gap on MI355X
        # (scripts/diag_step_gap.py), so the kernel time is the per-step average over
        # back-to-back launches (both kernels plus the gaps between them).
        ev_start = torch.cuda.Event(enable_timing=True)
        ev_end = torch.cuda.Event(enable_timing=True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev_start.record(stream)
        for k in range(steps):
            step(warmup + k)
        if owner:  # the last batch's rounds and unpack belong to the timed steps
            drain((warmup + steps - 1) & 1)
        ev_end.record(stream)
        for ws in works:
            for w in ws:
                w.wait()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        wall = time.perf_counter() - t0
        if dist:
            wall = float(allreduce_max(torch.tensor([wall], dtype=torch.float64, device=dev)).item())
        return wall, ev_start.elapsed_time(ev_end) / steps

    wall, ev_ms = timed(args.steps, args.warmup)
    pipeline = None
    if (c5 or owner) and (owner or world == 1) and not args.no_owner_ingest and n_matched_writers:
        # the same steps ending where the N = 1 receive path ends: every owner ingests its
        # writers' records into the history cache (deliveries), timed as a second loop
        with_ingest[0] = True
        w2, e2 = timed(args.steps, args.warmup)
        with_ingest[0] = False
        torch.cuda.synchronize(dev)
        na = int(iouts["n_accepted"].item())
        na_all = int(allreduce_sum(torch.tensor([na], dtype=torch.int64, device=dev)).item())
        pipeline = {"what": "parse + owner exchange (pack, RCCL rounds, unpack) + history-cache ingest on every "
                            "owner (fresh writer proxies each step)" if world > 1 else
                            "parse + history-cache ingest (fresh writer proxies each step)",
                    "value": world * n / (w2 / args.steps), "unit": "datagrams/s",
                    "ms_per_step": w2 / args.steps * 1e3, "deliveries_per_step_all_ranks": na_all,
                    "deliveries_per_s": na_all / (w2 / args.steps)}

    # ---- results / sanity (outside the timed region) ----
    status = outs["status"][:n].cpu().numpy()
    alg_total = alg_reads = alg_writes = 0
    recs = None
    chunk = 1 << 23
    for c0 in range(0, n_rec, chunk):  # in chunks: C5 at N=1 holds 256M records (16 GB)
        rc = outs["records"][c0:min(n_rec, c0 + chunk)].cpu().numpy().reshape(-1).view(RECORD_DTYPE)
        if n_rec <= chunk:
            recs = rc
        _, r_, w_ = algorithmic_bytes(status if c0 == 0 else status[:0], rc, n if c0 == 0 else 0)
        alg_reads += r_
        alg_writes += w_
    alg_total = alg_reads + alg_writes
    total_bytes = float(ln.astype(np.int64).sum())
    ms_per_step = wall / args.steps * 1e3
    value = world * n / (wall / args.steps)
    result = {
        "metric": "RTPS datagrams/s + GiB/s parsed (device-resident), 1/2/4/8 MI355X",
        "value": value,
        "unit": "datagrams/s",
        # the datagram bytes the parse covers per second: NOT an HBM bandwidth (the parse is
        # zero-copy and reads only headers and fixed fields; roofline below has the bytes it moves)
        "gib_per_s_covered": world * total_bytes / (wall / args.steps) / 2**30,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if c5 else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic generator f(seed=0x52545053, idx), generated in HBM)",
        "config": {"workload": f"{args.workload}: {WORKLOAD_DESC[args.workload]}",
                   "datagrams_per_gpu": n, "bytes_per_gpu": int(total_bytes), "records_per_gpu": n_rec,
                   "ok_datagrams": int((status == 0).sum()), "matched_writers": n_matched_writers,
                   "parallelism": f"{world} ranks, datagram-sharded" + (
                       ", writer-GUID all-to-all (" + ("RCCL" if args.backend == "nccl" else "gloo") + ")"
                       if world > 1 else "")},
    }
    if world == 1:
        result["roofline"] = roofline(rx, args, arena, off_t, ln_t, n, outs, stream, total_bytes, alg_reads,
                                      alg_writes)
    else:
        result["roofline"] = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                              "traffic": None, "kernel_ms": ev_ms,
                              "note": "N>1: per-step time on the compute stream (parse + bucket, waiting for the "
                                      "exchange two steps back); the kernel roofline is the N=1 line's"}
    if world > 1 and c5:
        # the driver's N = 1 line is T (the headline config); C5's own one-GPU rate, for a
        # same-workload comparison, is the committed C5 N = 1 line (64M datagrams on one GPU)
        import glob
        ref = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_bench_C5_n1.json")))
        if ref:
            try:
                d1 = json.loads([l for l in open(ref[-1]) if l.startswith("{")][-1])
                result["config"]["c5_one_gpu"] = {"value": d1["value"], "unit": d1["unit"],
                                                  "source": os.path.relpath(ref[-1], REPO)}
            except (OSError, ValueError, KeyError, IndexError):
                pass
    if world > 1 and owner:
        last = owned[(args.warmup + args.steps - 1) & 1]
        result["config"]["received_records_rank0"] = int(last.n_records) if last is not None else 0
        rcv = shards[(args.warmup + args.steps - 1) & 1].counts("recv")
        result["config"]["exchange"] = {
            "mode": "owner-side exchange: fixed slots (equal-split RCCL group, pipelined with the next parse) "
                    "+ exact spill round when a slot overflows",
            "item": "16-B rtps_shard_item per writer submessage that passes (a DATA of a listed writer: its "
                    "writer-list index, SN, kind, flags, route, payload kind; another DATA adds its GUID and SN "
                    "(32-B blob); any other kind: its 64-B record + GAP bitmap / DATA_FRAG payload bytes in the "
                    "blob), owner = the shard's owner table; unpacked on the owner as one batch",
            "slot_items": slot[0], "slot_blob_bytes": slot[1],
            "bytes_sent_per_rank_per_step": (world - 1) * (slot[0] * ITEM_BYTES_OWNER + slot[1] + 32),
            "predicted_xgmi_ms": (slot[0] * ITEM_BYTES_OWNER + slot[1] + 32) / (XGMI_LINK_GBS * 1e9) * 1e3,
            "spilled_records_rank0": int((rcv["n"] - rcv["cut"]).sum()), "overflow": False}
    elif world > 1:
        got, split = exch[(args.warmup + args.steps - 1) & 1].gather_received()
        result["config"]["received_records_rank0"] = int(got.shape[0])
        ib = 16 if args.exchange == "descriptors" else 64
        result["config"]["exchange"] = {
            "mode": "padded equal-split all-to-all, pipelined with the next parse",
            "item": (f"{ib}-B rtps_xdesc of matched records, owner = writer set % world"
                     if ib == 16 else "64-B records, owner = writer-GUID hash % world"),
            "bucket_capacity": bcap, "bytes_sent_per_rank_per_step": world * bcap * ib,
            "overflow": any(e.overflowed() for e in exch)}
    if pipeline is not None:
        result["pipeline_with_ingest"] = pipeline
    fouts = None
    if world == 1 and not args.no_frag and args.workload == "C4" and recs is not None:
        fouts, result["frag_assemble"] = frag_leg(rx, arena, off_t, outs, n_rec, recs, stream, args.steps)
    leg_iouts = None
    if world == 1 and not args.no_ingest and n_matched_writers:
        leg_iouts, result["ingest"] = ingest_leg(rx, arena, off_t, outs, n_rec, recs, n_matched_writers, stream,
                                                 args.steps, fouts=fouts)
    if world == 1 and n_matched_writers and not c5:
        result["exchange_prediction"] = exchange_prediction(rx, arena, off_t, outs, dev)
    if world == 1 and not args.no_cdr:
        result["cdr_decode"] = cdr_decode_leg(rx, args.workload, arena, off_t, outs, n_rec, stream, args.steps,
                                              iouts=leg_iouts)
    if world == 1 and not args.no_c1:
        result["c1_loopback"] = c1_loopback(dev, stream)
        # the same subscriber fed by 4 publisher threads: what the receive loop sustains when
        # one sendmmsg thread (the C1 bound above) is not the limit
        result["c1_loopback_4_publishers"] = c1_loopback(dev, stream, n=400_000, publishers=4)
    if world == 1 and not args.no_e2e:
        result["end_to_end"] = end_to_end(rx, arena, off_t, ln_t, n, outs, n_rec, stream)
        if n_matched_writers:
            result["end_to_end"]["full_chain"] = full_chain(rx, args.workload, arena, off_t, ln_t, n, n_rec,
                                                            n_matched_writers)
            fc = result["end_to_end"]["full_chain"]
            fc["pipelined"] = full_chain_pipelined(rx, args.workload, arena, off_t, ln_t, n, n_matched_writers)
            fc["pipelined_64k"] = full_chain_pipelined(rx, args.workload, arena, off_t, ln_t, n, n_matched_writers,
                                                       batch=1 << 16)
            fc["pipelined_32k"] = full_chain_pipelined(rx, args.workload, arena, off_t, ln_t, n, n_matched_writers,
                                                       batch=1 << 15)
            fc["pipelined_best"] = max(("pipelined", "pipelined_64k", "pipelined_32k"),
                                       key=lambda k: fc[k]["datagrams_per_s"] if fc[k]["parity_ok"] else 0)
    if world == 1 and not args.no_ingest and n_matched_writers and args.workload == "C3" and not c5:
        result["topic_cache_spdp_repeats"] = spdp_repeats_leg(dev, stream, min(args.steps, 10))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline("C3" if c5 else args.workload, min(n, 1 << 20), match_table=tbl)
    rx.close()
    if shards is not None:
        for sh in shards:
            sh.close()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return result


if __name__ == "__main__":
    main()
