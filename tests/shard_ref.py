"""numpy reference of the writer-GUID owner hash and stable bucketing (test helper)."""
import numpy as np

from rtps_rx.records import WRITER_KINDS, READER_KINDS


def owner_np(recs, world):
    w = recs.view(np.uint32).reshape(-1, 16)[:, 2:6].astype(np.uint64)
    h = np.full(len(recs), 0x811C9DC5, dtype=np.uint64)
    for k in range(4):
        h = ((h ^ w[:, k]) * np.uint64(0x01000193)) & np.uint64(0xFFFFFFFF)
    m = np.uint64(0xFFFFFFFF)  # murmur3 fmix32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & m
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & m
    h ^= h >> np.uint64(16)
    owner = (h % np.uint64(world)).astype(np.int64)
    exch = np.isin(recs["kind"], WRITER_KINDS + READER_KINDS)
    return np.where(exch, owner, -1)


def bucket_np(recs, world):
    """(bucketed records, counts per destination): stable partition by owner."""
    o = owner_np(recs, world)
    keep = o >= 0
    idx = np.nonzero(keep)[0]
    order = idx[np.argsort(o[keep], kind="stable")]
    counts = np.bincount(o[keep], minlength=world).astype(np.int64)
    return recs[order], counts


def desc_bucket_np(recs, table_guids, world, entity_sets=None):
    """numpy reference of rtps_rx_bucket_descriptors: MATCHED records of table writers,
    owner = writer set index (rank of the GUID's first appearance) % world, and TARGETED-only
    records (a reader contains the writer's entity id, no proxy for the GUID) with owner =
    their entity set index % world (entity_sets[i]: the record's target set, numbered after
    the writer sets); stable; returns (list per owner of XDESC rows)."""
    from rtps_rx.records import XDESC_DTYPE, ROUTE_MATCHED, ROUTE_TARGETED
    index = {}
    for g in table_guids:
        index.setdefault(bytes(g), len(index))
    out = [[] for _ in range(world)]
    for i, r in enumerate(recs):
        route = int(r["route"])
        if route & ROUTE_MATCHED:
            k = index.get(bytes(r["prefix"]) + bytes(r["writer_id"]))
            if k is None:
                continue
        elif route & ROUTE_TARGETED and entity_sets is not None:
            k = int(entity_sets[i])
            assert k >= len(index), "a TARGETED-only record's set is an entity set"
        else:
            continue
        out[k % world].append((int(r["sn"]), i, (k << 8) | int(r["kind"])))
    return [np.array(o, dtype=XDESC_DTYPE) for o in out]


# ---- owner-side exchange (rtps_rx_shard_*): numpy model of pack / unpack ----
LEAD = 65536
COUNTS_DTYPE = np.dtype([("n", "<u8"), ("bytes", "<u8"), ("cut", "<u8"), ("cut_bytes", "<u8")])


def _blob(rec):
    """(offset in the datagram, bytes) the owner's consumers read of one record."""
    from rtps_rx.records import U_GAP, U_FRAG, GAP, DATA_FRAG
    k = int(rec["kind"])
    if k == GAP:
        g = np.frombuffer(bytes(rec["u"]), dtype=U_GAP)[0]
        nb = int(g["num_bits"])
        return int(g["bitmap_off"]), (4 * ((nb + 31) // 32) if nb else 0)
    if k == DATA_FRAG:
        f = np.frombuffer(bytes(rec["u"]), dtype=U_FRAG)[0]
        return int(f["pl_off"]), int(f["pl_len"])
    return 0, 0


def _r16(x):
    return (x + 15) // 16 * 16


def balanced_owner_table(guids, world):
    """The shard's default owner table (RTPS_OWNER_BALANCED): the writer GUIDs of the context's
    proxies dealt by rtps_rx_owner_assign -> {16-byte GUID: owner}."""
    from rtps_rx.shard import owner_assign
    guids = sorted(set(bytes(g) for g in guids))
    return dict(zip(guids, (int(x) for x in owner_assign(guids, world))))


EKEY = b"\xff" * 12  # an entity key's prefix (RTPS_OWNER_TOPIC: writers without a proxy, by entity id)


def topic_owner_keys(readers, topic_readers=()):
    """Python restatement of rtps_ctx_owner_keys(by_topic) over a Readers table: the keys (writer
    GUIDs of the writer sets in first-appearance order, then EKEY || entity id per entity set)
    and each key's group (the smallest key index of its group): keys whose target readers share
    a topic cache (topic_readers [(slot, topic)], else the reader's own) are one group."""
    from rtps_rx.records import as_readers, READER_STATELESS
    rd = as_readers(readers)
    flags = [int(r["flags"]) for r in rd.readers]
    slot = [int(r["reader_slot"]) for r in rd.readers]
    contains = [set() for _ in rd.readers]
    wsets = []
    for p in rd.proxies:
        r, g = int(p["reader"]), bytes(p["writer_guid"])
        if flags[r] & READER_STATELESS:
            continue
        contains[r].add(g[12:])
        if g not in wsets:
            wsets.append(g)
    esets = []
    for g in wsets:
        if g[12:] not in esets:
            esets.append(g[12:])
    keys = wsets + [EKEY + e for e in esets]
    topic_of = dict(topic_readers)
    group = list(range(len(keys)))

    def root(x):
        while group[x] != x:
            x = group[x]
        return x
    first_key = {}
    for w, k in enumerate(keys):
        for r in range(len(slot)):
            if flags[r] & READER_STATELESS or k[12:] not in contains[r]:
                continue
            t = topic_of.get(slot[r], ("own", slot[r]))
            if t not in first_key:
                first_key[t] = w
                continue
            a, b = root(w), root(first_key[t])
            if a != b:
                group[max(a, b)] = min(a, b)
    return keys, [root(w) for w in range(len(keys))]


def topic_owner_table(readers, topic_readers, world, prev=None):
    """The shard's RTPS_OWNER_TOPIC table: {16-byte key: owner} (prev: {key: owner} of the
    previous table, the sticky deal)."""
    from rtps_rx.shard import owner_assign
    keys, groups = topic_owner_keys(readers, topic_readers)
    pv = None if prev is None else [prev.get(k, -1) for k in keys]
    return dict(zip(keys, (int(x) for x in owner_assign(keys, world, groups=groups, prev=pv))))


def shard_items(recs, world, table=None):
    """Owner of every record that is an item (writer kinds with ROUTE_PASS), else -1: the
    writer's owner in `table` ({GUID: owner}, the shard's owner table), else (entity keys in
    the table) its entity id's owner, else the GUID hash."""
    from rtps_rx.records import ROUTE_PASS
    o = owner_np(recs, world)
    if table:
        g = recs.view(np.uint8).reshape(-1, 64)[:, 8:24]
        o = np.array([table.get(bytes(x), table.get(EKEY + bytes(x)[12:], int(h))) for x, h in zip(g, o)],
                     dtype=np.int64)
    writer = np.isin(recs["kind"], WRITER_KINDS) & ((recs["route"] & ROUTE_PASS) != 0)
    return np.where(writer, o, -1)


ITEM_DTYPE = np.dtype([("w0", "<u4"), ("src_rec", "<u4"), ("sn_lo", "<u4"), ("kind", "u1"), ("flags", "u1"),
                       ("route", "u1"), ("payload_kind", "u1")])
assert ITEM_DTYPE.itemsize == 16
COMPACT = 0x1  # w0 & 0xf of a compact DATA (RTPS_SHARD_COMPACT)
WLIST_MAX = 1 << 20


def writer_list(table):
    """The shard's writer list: the owner table's writer GUIDs (not its entity keys), ascending bytes."""
    return sorted(k for k in (table or {}) if not k.startswith(EKEY))


def _item_and_blob(arena, offs, r, i, windex):
    """(rtps_shard_item, blob bytes) of record r (index i of the source's parse output): a DATA of a
    listed writer (windex: GUID -> list index) whose SN's high word is 0..255 is its item alone
    (compact); another DATA sends its GUID and SN (32 B); any other kind its record (dgram_idx := i)
    and its consumers' bytes."""
    from rtps_rx.records import DATA
    it = np.zeros(1, dtype=ITEM_DTYPE)[0]
    it["kind"], it["flags"], it["route"], it["payload_kind"] = r["kind"], r["flags"], r["route"], r["payload_kind"]
    it["src_rec"] = i
    if int(r["kind"]) == DATA:
        g = bytes(r["prefix"]) + bytes(r["writer_id"])
        sn = int(r["sn"])
        hi, lo = (sn >> 32) & 0xFFFFFFFF, sn & 0xFFFFFFFF
        k = windex.get(g)
        if k is not None and k < WLIST_MAX and hi <= 0xFF:
            it["w0"] = COMPACT | (k << 4) | (hi << 24)
            it["sn_lo"] = lo
            return it, np.zeros(0, np.uint8)
        b = np.zeros(32, dtype=np.uint8)
        b[:16] = np.frombuffer(g, np.uint8)
        b[16:24] = np.frombuffer(np.int64(sn).tobytes(), np.uint8)
        it["w0"] = 32
        return it, b
    rel, ln = _blob(r)
    rc = r.copy()
    rc["dgram_idx"] = i
    b = np.zeros(64 + _r16(ln), dtype=np.uint8)
    b[:64] = np.frombuffer(rc.tobytes(), dtype=np.uint8)
    src = int(offs[int(r["dgram_idx"])]) + rel
    b[64:64 + ln] = arena[src:src + ln]
    it["w0"] = len(b)
    return it, b


def shard_pack_np(arena, offs, recs, world, cap, bcap, table=None):
    """Per destination d: dict(counts, slot_items, slot_blob (bcap bytes), spill_items, spill_blob)."""
    o = shard_items(recs, world, table)
    windex = {g: k for k, g in enumerate(writer_list(table))}
    out = []
    for d in range(world):
        idx = np.nonzero(o == d)[0]
        pairs = [_item_and_blob(arena, offs, recs[i], int(i), windex) for i in idx]
        items = np.array([p[0] for p in pairs], dtype=ITEM_DTYPE) if pairs else np.zeros(0, ITEM_DTYPE)
        blobs = [p[1] for p in pairs]
        sizes = np.array([len(b) for b in blobs], dtype=np.int64)
        boff = np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else np.zeros(0, np.int64)
        fits = (np.arange(len(items)) < cap) & (boff + sizes <= bcap)
        cut = int(np.argmin(fits)) if not fits.all() else len(items)
        assert fits[:cut].all() and not fits[cut:].any()  # a prefix
        cut_bytes = int(boff[cut]) if cut < len(items) else int(sizes.sum())
        stream = np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
        c = np.zeros(1, dtype=COUNTS_DTYPE)
        c[0] = (len(items), int(sizes.sum()), cut, cut_bytes)
        out.append({"counts": c, "slot_items": items[:cut], "slot_blob": stream[:cut_bytes],
                    "spill_items": items[cut:], "spill_blob": stream[cut_bytes:]})
    return out


def shard_unpack_np(received, table=None):
    """received: per source s (rank order) the dict shard_pack_np made for this owner (table: the
    owner table the packs used, whose writer list compact items name).
    -> (records with dgram_idx = i, dgram_off u64, arena u8, origin (rank u32, source record u32))."""
    from rtps_rx.records import RECORD_DTYPE, DATA
    wl = writer_list(table)
    rank, src = [], []
    items = [np.concatenate([x["slot_items"], x["spill_items"]]) for x in received]
    for s, it in enumerate(items):
        rank.append(np.full(len(it), s, dtype=np.uint32))
        src.append(it["src_rec"].astype(np.uint32))
    allit = np.concatenate(items) if items else np.zeros(0, dtype=ITEM_DTYPE)
    blobs = np.concatenate([np.zeros(LEAD, np.uint8)] + [np.concatenate([x["slot_blob"], x["spill_blob"]])
                                                          for x in received])
    out = np.zeros(len(allit), dtype=RECORD_DTYPE)
    off = np.zeros(len(out), dtype=np.uint64)
    pos = LEAD
    for i, it in enumerate(allit):
        w0 = int(it["w0"])
        if int(it["kind"]) == DATA:
            out[i]["kind"], out[i]["flags"] = it["kind"], it["flags"]
            out[i]["route"], out[i]["payload_kind"] = it["route"], it["payload_kind"]
            if w0 & 0xF == COMPACT:
                g = wl[(w0 >> 4) & (WLIST_MAX - 1)]
                out[i]["sn"] = ((w0 >> 24) << 32) | int(it["sn_lo"])
            else:
                g = blobs[pos:pos + 16].tobytes()
                out[i]["sn"] = np.frombuffer(blobs[pos + 16:pos + 24].tobytes(), "<i8")[0]
                pos += w0
            out[i]["prefix"] = np.frombuffer(g[:12], np.uint8)
            out[i]["writer_id"] = np.frombuffer(g[12:], np.uint8)
            off[i] = LEAD
        else:
            out[i] = np.frombuffer(blobs[pos:pos + 64].tobytes(), dtype=RECORD_DTYPE)[0]
            rel, _ = _blob(out[i])
            off[i] = pos + 64 - rel
            pos += w0
        out[i]["dgram_idx"] = i
    assert pos == len(blobs)
    return out, off, blobs, (np.concatenate(rank) if rank else np.zeros(0, np.uint32),
                             np.concatenate(src) if src else np.zeros(0, np.uint32))
