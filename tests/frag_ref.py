"""Test-side DataFrag helpers: a datagram builder and an independent pure-Python
model of the reference's sequential reassembly, used to check the C oracle
(oracle/rtps_oracle.c rtps_oracle_frag_batch) on small corpora.

The model transcribes FragmentAssembler / AssemblyBuffer
(rtps/fragment_assembler.rs:23-214) as Reader::handle_datafrag_msg drives it
(io_uring/rtps/reader.rs:563-647): the writer's fragment size is fixed by its
first DATA_FRAG, a buffer's size and fragment count by the first DATA_FRAG of
its SN, insert_frags copies min(fis*F, payload) bytes at (start-1)*F clamped
to the buffer and sets the bits; a complete buffer is emitted and dropped.
Where the reference panics (bit index past the count, byte range past the
buffer) the model clamps, like the device and the oracle.
"""
import struct

import numpy as np

from rtps_rx.records import DATA_FRAG, ROUTE_PASS

RTPS_HDR = b"RTPS\x02\x04\x01\x0f"


def datafrag_sub(writer_key, sn, frag_start, fis, frag_size, data_size, payload, le=True, key=False,
                 reader=b"\x00\x00\x00\x00"):
    e = "<" if le else ">"
    body = struct.pack(e + "HH", 0, 28) + reader + writer_key + struct.pack(e + "iI", sn >> 32, sn & 0xFFFFFFFF)
    body += struct.pack(e + "IHHI", frag_start, fis, frag_size, data_size) + bytes(payload)
    flags = (1 if le else 0) | (0x04 if key else 0)
    return bytes([0x16, flags]) + struct.pack(e + "H", len(body)) + body


def datagram(prefix, subs):
    return RTPS_HDR + bytes(prefix) + b"".join(subs)


class FragRef:
    """Sequential model; batch() consumes parse records of one batch."""

    def __init__(self):
        self.writer_f = {}
        self.bufs = {}
        self.now = 0

    def pending(self):
        return len(self.bufs)

    def gc(self, expire_before):
        """FragmentAssembler::garbage_collect_before (fragment_assembler.rs:216-224)."""
        self.bufs = {k: b for k, b in self.bufs.items() if b["modified"] >= expire_before}
        return len(self.bufs)

    def batch(self, arena, offs, recs):
        out = []  # (guid bytes, sn, data bytes, rec_idx, flags)
        for ri, r in enumerate(recs):
            if int(r["kind"]) != DATA_FRAG or not (int(r["route"]) & ROUTE_PASS):
                continue
            guid = bytes(r["prefix"]) + bytes(r["writer_id"])
            u = r["u"].tobytes()
            pl_off, pl_len, start, fis, fsz, ds = struct.unpack_from("<HHIHHI", u, 0)
            if guid not in self.writer_f:
                self.writer_f[guid] = fsz
            F = self.writer_f[guid]
            k = (guid, int(r["sn"]))
            if k not in self.bufs:
                self.bufs[k] = {"bytes": bytearray(ds), "count": ds // fsz + (ds % fsz > 0), "bits": set()}
            b = self.bufs[k]
            b["modified"] = self.now  # AssemblyBuffer::new / insert_frags (:54-61, :139)
            frm = (start - 1) * F
            to = min(frm + min(fis * F, pl_len), len(b["bytes"]))
            base = int(offs[int(r["dgram_idx"])]) + pl_off
            if to > frm:
                b["bytes"][frm:to] = bytes(arena[base:base + to - frm])
            for f in range(start - 1, start - 1 + fis):
                if f >= b["count"]:
                    break
                b["bits"].add(f)
            if len(b["bits"]) == b["count"]:
                out.append((guid, int(r["sn"]), bytes(b["bytes"]), ri, int(r["flags"])))
                del self.bufs[k]
        return out


def soup(n, seed, prefix_count=3, writers_per_prefix=2):
    """n datagrams of DATA_FRAG traffic with every anomaly the assembler has to
    replay in order: shuffled and repeated fragments (different bytes), several
    fragments per submessage, short payloads, writers that change their fragment
    size, SNs whose later fragments announce another data size, fragment bits
    past the buffer, KEY fragments, tiny samples (data_size < 4) and resends
    after completion."""
    rng = np.random.default_rng(seed)
    prefixes = [bytes(rng.integers(0, 256, 12, dtype=np.uint8)) for _ in range(prefix_count)]
    writers = [(p, bytes([0, 1, w, 0x02])) for p in prefixes for w in range(writers_per_prefix)]
    pending = []  # (prefix, wkey, sn, fsz, ds, next fragment list)
    sn_next = {w: 1 for w in range(len(writers))}
    fsz_of = {}
    out = []
    while len(out) < n:
        if not pending or rng.random() < 0.3:
            w = int(rng.integers(0, len(writers)))
            p, wk = writers[w]
            fsz = fsz_of.setdefault(w, int(rng.choice([2, 8, 16, 100, 1344])))
            if rng.random() < 0.05:
                fsz = int(rng.choice([8, 12, 64]))  # a writer changing its fragment size
            ds = int(rng.choice([1, 3, 4, fsz, 2 * fsz + 5, 5 * fsz, 9 * fsz + 1]))
            ds = max(ds, fsz)
            cnt = ds // fsz + (ds % fsz > 0)
            frags = list(range(1, cnt + 1))
            rng.shuffle(frags)
            if rng.random() < 0.2 and frags:
                frags.insert(int(rng.integers(0, len(frags) + 1)), frags[0])  # repeated fragment
            sn = sn_next[w]
            sn_next[w] += 1
            if rng.random() < 0.05:
                sn = max(1, sn - 1)  # resend of an older SN (maybe after completion)
            pending.append([p, wk, sn, fsz, ds, frags, bool(rng.random() < 0.1)])
        i = int(rng.integers(0, len(pending)))
        p, wk, sn, fsz, ds, frags, key = pending[i]
        if not frags:
            pending.pop(i)
            continue
        start = frags.pop(0)
        fis = 1
        cnt = ds // fsz + (ds % fsz > 0)
        if rng.random() < 0.15 and frags and frags[0] == start + 1:
            frags.pop(0)
            fis = 2
        if rng.random() < 0.03:
            fis += 2  # bits past the buffer's count for the last fragments
        want = min(fis * fsz, ds - (start - 1) * fsz)
        plen = want
        r = rng.random()
        if r < 0.05:
            plen = max(0, want - int(rng.integers(1, 5)))  # short payload
        elif r < 0.1:
            plen = want + int(rng.integers(1, 9))          # longer than the span
        ds_wire = ds
        if rng.random() < 0.03:
            ds_wire = ds + fsz  # a later fragment announcing another size
            if start > ds_wire // fsz + (ds_wire % fsz > 0):
                ds_wire = ds
        payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
        le = bool(rng.random() < 0.8)
        sub = datafrag_sub(wk, sn, start, fis, fsz, ds_wire, payload, le=le, key=key)
        if rng.random() < 0.1:  # a second DATA_FRAG in the same datagram
            j = int(rng.integers(0, len(pending)))
            p2, wk2, sn2, fsz2, ds2, frags2, key2 = pending[j]
            if frags2 and p2 == p:
                s2 = frags2.pop(0)
                w2 = min(fsz2, ds2 - (s2 - 1) * fsz2)
                sub += datafrag_sub(wk2, sn2, s2, 1, fsz2, ds2,
                                    bytes(rng.integers(0, 256, w2, dtype=np.uint8)), key=key2)
        out.append(datagram(p, [sub]))
    return out


class ReaderFragRef:
    """Per-reader model: Domain::handle_event hands a DATA_FRAG the receiver passes to
    user readers (ROUTE_PASS, not ROUTE_BUILTIN) to every reader that contains the
    writer's entity id, in EntityId order (dp_event_loop.rs:266-327; the targets of
    ingest_ref.IngestRef); each reader drops it when its Lifespan is exceeded
    (reader.rs:578-589: the receive Timestamp minus the source Timestamp, in ticks,
    wrapping, as a signed Duration) and otherwise feeds its own FragmentAssembler for
    the writer (:617-619, 638-647), modelled by a FragRef per (reader, writer)."""

    def __init__(self, readers, lifespan_ns=None, recv_ns=0):
        from ingest_ref import IngestRef
        self.route = IngestRef(readers)
        self.life = dict(lifespan_ns or {})
        self.recv_ns = recv_ns
        self.asm = {}

    def set_readers(self, readers):
        from ingest_ref import IngestRef
        self.route = IngestRef(readers)

    @staticmethod
    def _ticks(ns, signed=False):
        return ((ns // 10**9) << 32) + (((ns % 10**9) << 32) // 10**9)

    def batch(self, arena, offs, recs):
        from rtps_rx.records import ROUTE_BUILTIN, ROUTE_TS_VALID
        out = []  # (reader slot, guid, sn, bytes, rec_idx, flags)
        now = self._ticks(self.recv_ns)
        for ri, r in enumerate(recs):
            if int(r["kind"]) != DATA_FRAG or not (int(r["route"]) & ROUTE_PASS) or int(r["route"]) & ROUTE_BUILTIN:
                continue
            guid = bytes(r["prefix"]) + bytes(r["writer_id"])
            for reader, _proxy in self.route.targets(guid):
                slot = self.route.slot[reader]
                if slot in self.life and int(r["route"]) & ROUTE_TS_VALID:
                    src = (int(r["ts_sec"]) << 32) | int(r["ts_frac"])
                    elapsed = (now - src) & 0xFFFFFFFFFFFFFFFF
                    elapsed = elapsed - (1 << 64) if elapsed >= 1 << 63 else elapsed
                    if self._ticks(self.life[slot]) < elapsed:
                        continue
                a = self.asm.setdefault((slot, guid), FragRef())
                for g, sn, data, rj, fl in a.batch(arena, offs, recs[ri:ri + 1]):
                    out.append((slot, g, sn, data, ri, fl))
        return out


# ---- the per-reader scenario: two readers of one writer, one with a
# Lifespan, a third reader added mid-stream, a writer that changes its fragment size ----
RS_PREFIX = [bytes([0x01, 0x0f, 0xaa, k, 0, 0, 0, 0, 1, 0, 0, 0]) for k in (1, 2)]
RS_WRITER = [bytes([0, 1, k, 0x02]) for k in (1, 2)]
RS_READER = {11: bytes([0, 0, 1, 0x07]), 12: bytes([0, 0, 2, 0x07]), 13: bytes([0, 0, 3, 0x07])}
RS_RECV_NS = 1_700_000_100 * 10**9
RS_LIFESPAN = {12: 2 * 10**9}  # reader slot 12 (B): Lifespan 2 s


def reader_scenario_readers(with_c):
    """Readers A (11), B (12) and, from the second batch on, C (13); proxies appended so
    that existing proxies keep their positions."""
    from rtps_rx.records import Readers
    readers = [(RS_READER[11], 11, 0), (RS_READER[12], 12, 0)] + ([(RS_READER[13], 13, 0)] if with_c else [])
    g1, g2 = RS_PREFIX[0] + RS_WRITER[0], RS_PREFIX[1] + RS_WRITER[1]
    proxies = [(g1, 0), (g1, 1), (g2, 1)] + ([(g1, 2), (g2, 2)] if with_c else [])
    return Readers(readers, proxies)


def reader_scenario_single_readers():
    """Readers A (11) of W1 and B (12) of W2: every target set holds one reader (the
    library selects in place, without the per-target expansion)."""
    from rtps_rx.records import Readers
    g1, g2 = RS_PREFIX[0] + RS_WRITER[0], RS_PREFIX[1] + RS_WRITER[1]
    return Readers([(RS_READER[11], 11, 0), (RS_READER[12], 12, 0)], [(g1, 0), (g2, 1)])


def info_ts_sub(sec, frac, le=True, invalidate=False):
    e = "<" if le else ">"
    if invalidate:
        return bytes([0x09, (1 if le else 0) | 2]) + struct.pack(e + "H", 0)
    return bytes([0x09, 1 if le else 0]) + struct.pack(e + "HII", 8, sec, frac)


def reader_scenario(n, seed, sn0, frag_size):
    """n datagrams: samples of both writers fragmented at frag_size (W1) / 48 (W2),
    fragments shuffled across the batch, some repeated; each datagram may start with an
    INFO_TS 0.5, 1.5, 3 or 10 s before RS_RECV_NS (or none, or an invalidating one)."""
    rng = np.random.default_rng(seed)
    now_s = RS_RECV_NS // 10**9
    frags = []
    sn = {0: sn0, 1: sn0}
    while len(frags) < n:
        w = int(rng.integers(0, 2))
        F = frag_size if w == 0 else 48
        ds = int(rng.choice([F, 2 * F + 7, 3 * F, 5 * F - 1]))
        cnt = ds // F + (ds % F > 0)
        for k in range(1, cnt + 1):
            plen = min(F, ds - (k - 1) * F)
            frags.append((w, sn[w], k, F, ds, bytes(rng.integers(0, 256, plen, dtype=np.uint8))))
        sn[w] += 1
    order = rng.permutation(len(frags))
    out = []
    for i in order[:n]:
        w, s, k, F, ds, pl = frags[int(i)]
        subs = []
        t = rng.random()
        if t < 0.7:
            age = float(rng.choice([0.5, 1.5, 3.0, 10.0]))
            sec = now_s - int(age) - (1 if age % 1 else 0)
            frac = (1 << 31) if age % 1 else 0
            subs.append(info_ts_sub(sec, frac))
        elif t < 0.8:
            subs.append(info_ts_sub(0, 0, invalidate=True))
        subs.append(datafrag_sub(RS_WRITER[w], s, k, 1, F, ds, pl, le=bool(rng.random() < 0.85)))
        out.append(datagram(RS_PREFIX[w], subs))
        if rng.random() < 0.05:  # a repeated fragment
            out.append(datagram(RS_PREFIX[w], subs))
    return out[:n]
