"""Test-side history-cache ingest helpers: datagram builders for DATA /
HEARTBEAT / GAP traffic and an independent pure-Python model of the
reference's stateful-reader bookkeeping, used to check the C oracle
(oracle/rtps_oracle.c rtps_oracle_ingest_batch).

The model transcribes RtpsWriterProxy (rtps/rtps_writer_proxy.rs:17-355) with
its `changes` BTreeMap kept as a dict that is pruned exactly like the
reference prunes it (split_off / append in irrelevant_changes_range), driven as
Reader::handle_data_msg / handle_datafrag_msg / handle_heartbeat_msg /
handle_gap_msg drive it (io_uring/rtps/reader.rs:514-1116) for the records the
receiver passes (ROUTE_PASS) from matched writers (ROUTE_MATCHED).
"""
import struct

import numpy as np

from rtps_rx.records import DATA, HEARTBEAT, GAP, ROUTE_PASS, ROUTE_MATCHED, PK_DATA, PK_KEY, PK_KEY_HASH

RTPS_HDR = b"RTPS\x02\x04\x01\x0f"
ZERO_EID = b"\x00\x00\x00\x00"


def _sn(e, sn):
    return struct.pack(e + "iI", sn >> 32, sn & 0xFFFFFFFF)


def data_sub(writer_key, sn, le=True, payload=b"\x00\x01\x00\x00abcd", key=False, both=False, key_hash=None):
    """DATA (data.rs:57-144): D (or K) payload, or a KEY_HASH-only DATA (no payload)."""
    e = "<" if le else ">"
    flags = 1 if le else 0
    qos = b""
    if key_hash is not None:
        flags |= 0x02
        qos = struct.pack(e + "HH", 0x70, 16) + bytes(key_hash) + struct.pack(e + "HH", 1, 0)
        payload = b""
    elif both:
        flags |= 0x0C
    else:
        flags |= 0x08 if key else 0x04
    body = struct.pack(e + "HH", 0, 16) + ZERO_EID + writer_key + _sn(e, sn) + qos + bytes(payload)
    return bytes([0x15, flags]) + struct.pack(e + "H", len(body)) + body


def hb_sub(writer_key, first, last, count, le=True):
    e = "<" if le else ">"
    body = ZERO_EID + writer_key + _sn(e, first) + _sn(e, last) + struct.pack(e + "i", count)
    return bytes([0x07, (1 if le else 0) | 2]) + struct.pack(e + "H", len(body)) + body


def gap_sub(writer_key, start, base, bits, le=True):
    """GAP (gap.rs:23-46): gapStart, gapList = (base, numBits, bitmap MSB-first)."""
    e = "<" if le else ">"
    nb = len(bits)
    words = [0] * ((nb + 31) // 32)
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (31 - i % 32)
    body = ZERO_EID + writer_key + _sn(e, start) + _sn(e, base) + struct.pack(e + "I", nb)
    body += b"".join(struct.pack(e + "I", w) for w in words)
    return bytes([0x08, 1 if le else 0]) + struct.pack(e + "H", len(body)) + body


def info_dst_sub(prefix, le=True):
    e = "<" if le else ">"
    return bytes([0x0E, 1 if le else 0]) + struct.pack(e + "H", 12) + bytes(prefix)


def datagram(prefix, subs):
    return RTPS_HDR + bytes(prefix) + b"".join(subs)


class Proxy:
    """RtpsWriterProxy: ack_base, changes {sn: received?}, received_heartbeat_count."""

    def __init__(self):
        self.ack_base = 1
        self.changes = {}
        self.hb_count = 0

    def should_ignore(self, s):  # :202-204
        return s < self.ack_base or s in self.changes

    def advance(self):  # :338-355
        test = self.ack_base
        for sn in sorted(k for k in self.changes if k >= self.ack_base):
            if sn != test:
                break
            test += 1
            self.ack_base = test

    def received_add(self, s):  # :207-224
        self.changes[s] = True
        if s == self.ack_base:
            self.advance()

    def set_irrelevant(self, s):  # :226-239
        if s >= self.ack_base:
            self.changes[s] = None
        if s == self.ack_base:
            self.advance()

    def irrelevant_range(self, frm, until):  # :241-288
        if frm > until:
            return
        if frm <= self.ack_base:
            for k in [k for k in self.changes if frm <= k < until]:
                del self.changes[k]
            if until > self.ack_base:
                self.ack_base = until
                self.advance()
        else:
            for s in range(frm, until):
                self.changes[s] = None


class IngestRef:
    """Sequential model over the records of successive batches: every record the
    receiver passes (ROUTE_PASS) that is not a builtin pair (ROUTE_BUILTIN) goes to
    the readers that contain its writer's entity id, in EntityId order
    (dp_event_loop.rs:266-327, reader.rs:474-484), one writer proxy per
    (reader, writer GUID) (reader.rs:693-758)."""

    def __init__(self, readers):
        from rtps_rx.records import as_readers, READER_STATELESS
        rd = as_readers(readers)
        self.slot = [int(r["reader_slot"]) for r in rd.readers]
        self.flags = [int(r["flags"]) for r in rd.readers]
        self.eid = [bytes(r["entity_id"]) for r in rd.readers]
        self.order = sorted(range(len(rd.readers)), key=lambda i: self.eid[i])
        self.proxy_of = {}
        self.contains = [set() for _ in rd.readers]
        for k, p in enumerate(rd.proxies):
            g, r = bytes(p["writer_guid"]), int(p["reader"])
            self.proxy_of[(r, g)] = k
            if not self.flags[r] & READER_STATELESS:
                self.contains[r].add(g[12:])
        self.proxies = [Proxy() for _ in rd.proxies]

    def targets(self, guid):
        return [(r, self.proxy_of.get((r, guid))) for r in self.order if guid[12:] in self.contains[r]]

    def _sample(self, r, k, guid, sn):
        if k is None:
            return guid[15] & 0xF0 != 0  # no proxy: only a writer whose kind is not user-defined
        p = self.proxies[k]
        if p.should_ignore(sn) and self.eid[r] != SPDP_PARTICIPANT_READER:
            return False
        p.received_add(sn)
        return True

    def batch(self, arena, offs, recs, frag_samples=(), best_effort=False):
        """-> (deliveries [(record, reader slot)], ack_base per proxy)."""
        from rtps_rx.records import ROUTE_BUILTIN, WRITER_KINDS, READER_BEST_EFFORT
        at = {int(s["rec_idx"]): s for s in (frag_samples if frag_samples is not None else ())}
        out = []
        for i, r in enumerate(recs):
            route, kind = int(r["route"]), int(r["kind"])
            if not route & ROUTE_PASS or route & ROUTE_BUILTIN or kind not in WRITER_KINDS:
                continue
            guid = bytes(r["prefix"]) + bytes(r["writer_id"])
            for rd, k in self.targets(guid):
                p = self.proxies[k] if k is not None else None
                sn = int(r["sn"])
                u = r["u"].tobytes()
                if i in at:
                    s = at[i]
                    if int(s["status"]) != 1 and self._sample(rd, k, guid, int(s["sn"])):
                        out.append((i, self.slot[rd]))
                elif kind == DATA:
                    if int(r["payload_kind"]) in (PK_DATA, PK_KEY, PK_KEY_HASH) and self._sample(rd, k, guid, sn):
                        out.append((i, self.slot[rd]))
                elif kind == HEARTBEAT:
                    if best_effort or self.flags[rd] & READER_BEST_EFFORT or p is None:
                        continue
                    count = struct.unpack_from("<i", u, 8)[0]
                    if count <= p.hb_count:
                        continue
                    p.hb_count = count
                    p.irrelevant_range(0, sn)
                elif kind == GAP:
                    base, nb, boff = struct.unpack_from("<qIH", u, 0)
                    if p is None or sn <= 0 or base <= 0:
                        continue
                    p.irrelevant_range(sn, base)
                    bm = int(offs[int(r["dgram_idx"])]) + boff
                    le = int(r["flags"]) & 1
                    for b in range(nb):
                        w = bytes(arena[bm + 4 * (b // 32):bm + 4 * (b // 32) + 4])
                        word = struct.unpack("<I" if le else ">I", w)[0]
                        if word & (1 << (31 - b % 32)):
                            p.set_irrelevant(base + b)
        return out, [p.ack_base for p in self.proxies]


SPDP_PARTICIPANT_READER = bytes([0x00, 0x01, 0x00, 0xC7])
PREFIXES = [bytes([0xA0 + k] * 12) for k in range(4)]
OWN = bytes([0x01, 0x03, 0x00, 0x0c, 0x29, 0x2d, 0x31, 0xa2, 0x28, 0x20, 0x02, 0x08])


def writer_key(k):
    return bytes([0, 0, 1 + k, 0x02])


def table(n_prefix=3, n_writer=3):
    """Match table (compatibility form): writers (prefix p, key k) for p < n_prefix, k < n_writer,
    reader slot = p*n_writer+k; writer (prefix 0, key 0) also goes to a second reader (slot 77);
    writers of prefix 3 have no proxy."""
    from rtps_rx.records import pack_match_table
    ents = [(PREFIXES[p] + writer_key(k), p * n_writer + k) for p in range(n_prefix) for k in range(n_writer)]
    ents.append((PREFIXES[0] + writer_key(0), 77))
    return pack_match_table(ents), [g for g, _ in ents]


def stream(n, seed, sn_hi=60, n_prefix=4, n_writer=3, keys=None, sn_draw=None, gap_len=None):
    """n datagrams of reliable-reader traffic with every case the proxies have to
    replay in order: duplicate and out-of-order DATA, KEY and KEY_HASH samples,
    DATA whose payload decision fails, HEARTBEATs with stale counts and any
    firstSN (<= 0 too), valid and invalid GAPs with ranges and bitmaps, big- and
    little-endian submessages, writers outside the match table, and writer
    submessages after an INFO_DST to another participant (not passed).
    keys: writer entity ids to draw from (default writer_key(0 .. n_writer-1)).
    sn_draw(rng): the SN of a DATA, a HEARTBEAT's firstSN, a GAP's gapStart (default
    uniform in [-1, sn_hi)); gap_len(rng, start): a GAP's gapList.base (default start + [-3, 8))."""
    rng = np.random.default_rng(seed)
    draw = sn_draw or (lambda g: int(g.integers(-1, sn_hi)))
    keys = [writer_key(k) for k in range(n_writer)] if keys is None else list(keys)
    out = []
    for _ in range(n):
        p = int(rng.integers(n_prefix))
        subs = []
        if rng.random() < 0.05:
            subs.append(info_dst_sub(bytes([7] * 12)))
        for _ in range(int(rng.integers(1, 4))):
            wk = keys[int(rng.integers(len(keys)))]
            le = bool(rng.random() < 0.8)
            x = rng.random()
            if x < 0.55:
                sn = draw(rng)
                y = rng.random()
                if y < 0.08:
                    subs.append(data_sub(wk, sn, le, key=True))
                elif y < 0.12:
                    subs.append(data_sub(wk, sn, le, both=True))
                elif y < 0.16:
                    subs.append(data_sub(wk, sn, le, key_hash=bytes(range(16))))
                else:
                    subs.append(data_sub(wk, sn, le))
            elif x < 0.75:
                first = int(rng.integers(-2, sn_hi)) if sn_draw is None else draw(rng)
                subs.append(hb_sub(wk, first, first + int(rng.integers(0, 20)), int(rng.integers(-1, 12)), le))
            else:
                start = draw(rng)
                base = start + int(rng.integers(-3, 8)) if gap_len is None else gap_len(rng, start)
                nb = int(rng.integers(0, 70))
                bits = [bool(b) for b in rng.random(nb) < 0.4]
                subs.append(gap_sub(wk, start, base, bits, le))
        out.append(datagram(PREFIXES[p], subs))
    return out


# ---- a15: reader sets (dp_event_loop.rs:266-327, reader.rs:474-484, 693-758) ----
BUILTIN_KIND_KEY = bytes([0, 0, 9, 0xC2])   # a writer entity of builtin kind that is no discovery pair
VENDOR_KIND_KEY = bytes([0, 0, 10, 0x42])   # vendor-specific kind: not user-defined either


def a15_readers():
    """Readers listed out of EntityId order: two readers on one writer, a stateless reader with
    proxies, a BestEffort reader, the SPDP participant reader id (accepts duplicates), and
    builtin- / vendor-kind writers."""
    from rtps_rx.records import Readers, READER_STATELESS, READER_BEST_EFFORT
    P, wk = PREFIXES, writer_key
    readers = [(bytes([0, 0, 2, 0x07]), 11, 0),
               (bytes([0, 0, 1, 0x07]), 10, 0),
               (bytes([0, 0, 0, 0x04]), 12, READER_STATELESS),
               (bytes([0, 0, 3, 0x07]), 13, READER_BEST_EFFORT),
               (SPDP_PARTICIPANT_READER, 14, 0)]
    proxies = [(P[0] + wk(0), 1), (P[0] + wk(0), 0),     # one writer, two readers
               (P[1] + wk(0), 0), (P[0] + wk(1), 0),
               (P[0] + wk(2), 2), (P[1] + wk(2), 2),     # the stateless reader's: never targeted
               (P[2] + wk(1), 3),                         # BestEffort reader
               (P[0] + BUILTIN_KIND_KEY, 1),
               (P[1] + VENDOR_KIND_KEY, 4),
               (P[0] + wk(0), 4)]                         # the participant reader on writer 0 too
    return Readers(readers, proxies)


def a15_stream(n, seed, sn_hi=40):
    return stream(n, seed, sn_hi=sn_hi, keys=[writer_key(0), writer_key(1), writer_key(2), BUILTIN_KIND_KEY,
                                              VENDOR_KIND_KEY])
