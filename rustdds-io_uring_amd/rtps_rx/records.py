"""numpy views of the C-ABI output types (include/rtps_rx.h).

rtps_record is 64 bytes; its 16-byte kind-specific union is exposed as
several alternative dtypes over the same bytes (RECORD_DTYPE + per-kind
union dtypes applied to the `u` field).
"""
import numpy as np

# dgram status (rtps_dgram_status)
DGRAM_OK, DGRAM_SHORT, DGRAM_PING, DGRAM_RTPX, DGRAM_BAD_MAGIC, DGRAM_BAD_HEADER, \
    DGRAM_SUBMSG_ERR, DGRAM_TOO_LONG = range(8)
STATUS_NAMES = ["OK", "SHORT", "PING", "RTPX", "BAD_MAGIC", "BAD_HEADER", "SUBMSG_ERR", "TOO_LONG"]

# SubmessageKind (messages/submessages/submessage_kind.rs:17-34)
PAD, ACKNACK, HEARTBEAT, GAP, INFO_TS, INFO_SRC, INFO_REPLY_IP4, INFO_DST, INFO_REPLY, \
    NACK_FRAG, HEARTBEAT_FRAG, DATA, DATA_FRAG = \
    0x01, 0x06, 0x07, 0x08, 0x09, 0x0C, 0x0D, 0x0E, 0x0F, 0x12, 0x13, 0x15, 0x16
KIND_NAMES = {PAD: "PAD", ACKNACK: "ACKNACK", HEARTBEAT: "HEARTBEAT", GAP: "GAP", INFO_TS: "INFO_TS",
              INFO_SRC: "INFO_SRC", INFO_REPLY_IP4: "INFO_REPLY_IP4", INFO_DST: "INFO_DST",
              INFO_REPLY: "INFO_REPLY", NACK_FRAG: "NACK_FRAG", HEARTBEAT_FRAG: "HEARTBEAT_FRAG",
              DATA: "DATA", DATA_FRAG: "DATA_FRAG"}
WRITER_KINDS = (DATA, DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP)
READER_KINDS = (ACKNACK, NACK_FRAG)
INTERPRETER_KINDS = (INFO_TS, INFO_SRC, INFO_DST, INFO_REPLY)

ROUTE_PASS, ROUTE_TS_VALID, ROUTE_HAS_QOS, ROUTE_HAS_PAYLOAD, ROUTE_BUILTIN, ROUTE_MATCHED, ROUTE_TARGETED = \
    0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40

PK_NONE, PK_DATA, PK_KEY, PK_KEY_HASH = 0, 1, 2, 3
CK_ALIVE, CK_NOT_ALIVE_DISPOSED, CK_NOT_ALIVE_UNREGISTERED, CK_NONE = 0, 1, 2, 0xFF  # rtps_change_kind
PK_ERR_NO_CONTENT, PK_ERR_AMBIGUOUS, PK_ERR_SHORT = 0x81, 0x82, 0x83

NO_MATCH = 0xFFFF
NO_TARGET = 0xFFFFFFFF
NO_PROXY = 0xFFFFFFFF
READER_STATELESS, READER_BEST_EFFORT, TARGET_DUPLICATES_OK = 0x1, 0x2, 0x8000
MAX_DATAGRAM = 65536

RECORD_DTYPE = np.dtype([
    ("dgram_idx", "<u4"), ("sub_off", "<u2"), ("kind", "u1"), ("flags", "u1"),
    ("prefix", "u1", (12,)), ("writer_id", "u1", (4,)), ("reader_id", "u1", (4,)),
    ("aux16", "<u2"), ("route", "u1"), ("payload_kind", "u1"),
    ("sn", "<i8"), ("u", "u1", (16,)), ("ts_sec", "<u4"), ("ts_frac", "<u4"),
])
assert RECORD_DTYPE.itemsize == 64

U_DATA = np.dtype([("pl_off", "<u2"), ("pl_len", "<u2"), ("rep_id", "u1", (2,)), ("rep_opts", "u1", (2,)),
                   ("key_hash_off", "<u2"), ("status_info_off", "<u2"), ("rsi_off", "<u2"), ("change_kind", "u1"), ("_r", "u1")])
U_FRAG = np.dtype([("pl_off", "<u2"), ("pl_len", "<u2"), ("frag_start", "<u4"),
                   ("frags_in_sub", "<u2"), ("frag_size", "<u2"), ("data_size", "<u4")])
U_HB = np.dtype([("last_sn", "<i8"), ("count", "<i4"), ("_r", "<u4")])
U_HBFRAG = np.dtype([("last_frag_num", "<u4"), ("count", "<i4"), ("_r", "<u4", (2,))])
U_GAP = np.dtype([("list_base", "<i8"), ("num_bits", "<u4"), ("bitmap_off", "<u2"), ("_r", "<u2")])
U_ACKNACK = np.dtype([("count", "<i4"), ("_r", "<u4"), ("num_bits", "<u4"), ("bitmap_off", "<u2"), ("_r2", "<u2")])
U_NACKFRAG = np.dtype([("fns_base", "<u4"), ("count", "<i4"), ("num_bits", "<u4"), ("bitmap_off", "<u2"), ("_r", "<u2")])
U_INFOSRC = np.dtype([("version", "u1", (2,)), ("vendor", "u1", (2,)), ("_r", "<u4", (3,))])
U_INFOREPLY = np.dtype([("n_unicast", "<u4"), ("n_multicast", "<u4"), ("_r", "<u4", (2,))])
for _d in (U_DATA, U_FRAG, U_HB, U_HBFRAG, U_GAP, U_ACKNACK, U_NACKFRAG, U_INFOSRC, U_INFOREPLY):
    assert _d.itemsize == 16

UNION_BY_KIND = {DATA: U_DATA, DATA_FRAG: U_FRAG, HEARTBEAT: U_HB, HEARTBEAT_FRAG: U_HBFRAG, GAP: U_GAP,
                 ACKNACK: U_ACKNACK, NACK_FRAG: U_NACKFRAG, INFO_SRC: U_INFOSRC, INFO_REPLY: U_INFOREPLY}

MATCH_DTYPE = np.dtype([("writer_guid", "u1", (16,)), ("reader_slot", "<u2"), ("_pad", "<u2")])
# local readers and their writer proxies (rtps_reader / rtps_proxy / rtps_target / rtps_delivery)
READER_DTYPE = np.dtype([("entity_id", "u1", (4,)), ("reader_slot", "<u2"), ("flags", "<u2")])
PROXY_DTYPE = np.dtype([("writer_guid", "u1", (16,)), ("reader", "<u4")])
TARGET_DTYPE = np.dtype([("reader_slot", "<u2"), ("reader_flags", "<u2"), ("proxy", "<u4")])
DELIVERY_DTYPE = np.dtype([("rec_idx", "<u4"), ("reader_slot", "<u2"), ("flags", "<u2")])
DELIVERY_CACHED = 0x1  # rtps_delivery.flags: TopicCache::add_change stored the change
# topic caches (rtps_topic / rtps_topic_reader)
TOPIC_DTYPE = np.dtype([("topic", "<u4"), ("max_keep_samples", "<u4")])
TOPIC_READER_DTYPE = np.dtype([("reader_slot", "<u2"), ("_r", "<u2"), ("topic", "<u4")])
assert READER_DTYPE.itemsize == 8 and PROXY_DTYPE.itemsize == 20 and TARGET_DTYPE.itemsize == 8
assert DELIVERY_DTYPE.itemsize == 8

# exchange descriptor (rtps_xdesc): the compact cross-GPU form of a matched writer's record
XDESC_DTYPE = np.dtype([("sn", "<i8"), ("rec_idx", "<u4"), ("writer_kind", "<u4")])
assert XDESC_DTYPE.itemsize == 16

# DataFrag reassembly output (rtps_frag_sample, include/rtps_rx.h)
FRAG_OK, FRAG_SHORT, FRAG_NO_ROOM = 0, 1, 2
FRAG_SAMPLE_DTYPE = np.dtype([("writer_guid", "u1", (16,)), ("sn", "<i8"), ("heap_off", "<u8"),
                              ("data_size", "<u4"), ("rec_idx", "<u4"), ("flags", "u1"), ("status", "u1"),
                              ("reader_slot", "<u2"), ("_r2", "<u4")])
assert FRAG_SAMPLE_DTYPE.itemsize == 48
assert MATCH_DTYPE.itemsize == 20


def union_view(rec):
    """Kind-specific fields of one record (numpy void) as a dict."""
    dt = UNION_BY_KIND.get(int(rec["kind"]))
    if dt is None:
        return {}
    u = np.frombuffer(bytes(rec["u"]), dtype=dt)[0]
    return {n: (u[n].tolist() if hasattr(u[n], "tolist") else u[n]) for n in dt.names if not n.startswith("_")}


def record_to_dict(rec):
    d = {
        "dgram_idx": int(rec["dgram_idx"]), "sub_off": int(rec["sub_off"]), "kind": int(rec["kind"]),
        "kind_name": KIND_NAMES.get(int(rec["kind"]), hex(int(rec["kind"]))),
        "flags": int(rec["flags"]), "prefix": bytes(rec["prefix"]).hex(),
        "writer_id": bytes(rec["writer_id"]).hex(), "reader_id": bytes(rec["reader_id"]).hex(),
        "aux16": int(rec["aux16"]), "route": int(rec["route"]), "payload_kind": int(rec["payload_kind"]),
        "sn": int(rec["sn"]), "ts_sec": int(rec["ts_sec"]), "ts_frac": int(rec["ts_frac"]),
    }
    d.update(union_view(rec))
    return d


def max_records(lens):
    """Upper bound on records of a batch: every materialised submessage is >= 4 bytes."""
    lens = np.asarray(lens, dtype=np.int64)
    ok = (lens >= 20) & (lens <= MAX_DATAGRAM)
    return int(np.sum(np.where(ok, (lens - 20) // 4, 0)))


def pack_match_table(entries):
    """entries: iterable of (writer_guid: bytes[16], reader_slot: int)."""
    entries = list(entries)
    t = np.zeros(len(entries), dtype=MATCH_DTYPE)
    for i, (g, slot) in enumerate(entries):
        assert len(g) == 16 and 0 <= slot < NO_MATCH
        t[i]["writer_guid"] = np.frombuffer(bytes(g), dtype=np.uint8)
        t[i]["reader_slot"] = slot
    return t


class Readers:
    """The local readers and their writer proxies (rtps_rx_set_readers): the
    reference's available_readers (io_uring/rtps/message_receiver.rs:129), each
    Reader's matched_writers (io_uring/rtps/reader.rs:145)."""

    def __init__(self, readers=(), proxies=()):
        """readers: iterable of (entity_id bytes[4], reader_slot, flags);
        proxies: iterable of (writer_guid bytes[16], reader index)."""
        readers, proxies = list(readers), list(proxies)
        self.readers = np.zeros(len(readers), dtype=READER_DTYPE)
        for i, (eid, slot, flags) in enumerate(readers):
            assert len(eid) == 4
            self.readers[i]["entity_id"] = np.frombuffer(bytes(eid), dtype=np.uint8)
            self.readers[i]["reader_slot"] = slot
            self.readers[i]["flags"] = flags
        self.proxies = np.zeros(len(proxies), dtype=PROXY_DTYPE)
        for i, (g, r) in enumerate(proxies):
            assert len(g) == 16
            self.proxies[i]["writer_guid"] = np.frombuffer(bytes(g), dtype=np.uint8)
            self.proxies[i]["reader"] = r

    @property
    def n_proxies(self):
        return len(self.proxies)

    @classmethod
    def from_match(cls, entries):
        """The compatibility form (rtps_rx_set_match_table): every distinct slot is one
        reliable stateful reader (EntityId order = first appearance), every distinct
        (writer GUID, slot) pair one proxy."""
        t = entries if isinstance(entries, np.ndarray) else pack_match_table(entries)
        slots, readers, proxies, seen = {}, [], [], set()
        for e in t:
            slot = int(e["reader_slot"])
            if slot not in slots:
                r = len(readers)
                slots[slot] = r
                readers.append((bytes([(r >> 16) & 255, (r >> 8) & 255, r & 255, 0x07]), slot, 0))
            g = bytes(e["writer_guid"])
            if (slots[slot], g) in seen:
                continue
            seen.add((slots[slot], g))
            proxies.append((g, slots[slot]))
        return cls(readers, proxies)


def as_readers(table):
    """A Readers, a MATCH_DTYPE array, an iterable of (guid, slot) pairs, or None (no readers)."""
    if table is None:
        return Readers()
    if isinstance(table, Readers):
        return table
    return Readers.from_match(table)
