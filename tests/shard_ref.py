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


def shard_items(recs, world):
    """Owner of every record that is an item (writer kinds with ROUTE_PASS), else -1."""
    from rtps_rx.records import ROUTE_PASS
    o = owner_np(recs, world)
    writer = np.isin(recs["kind"], WRITER_KINDS) & ((recs["route"] & ROUTE_PASS) != 0)
    return np.where(writer, o, -1)


def shard_pack_np(arena, offs, recs, world, cap, bcap):
    """Per destination d: dict(counts, slot_recs, slot_blob (bcap bytes), spill_recs, spill_blob)."""
    o = shard_items(recs, world)
    out = []
    for d in range(world):
        idx = np.nonzero(o == d)[0]
        items = recs[idx]
        blobs = []
        for r in items:
            rel, ln = _blob(r)
            b = np.zeros(_r16(ln), dtype=np.uint8)
            src = int(offs[int(r["dgram_idx"])]) + rel
            b[:ln] = arena[src:src + ln]
            blobs.append(b)
        sizes = np.array([len(b) for b in blobs], dtype=np.int64)
        boff = np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else np.zeros(0, np.int64)
        fits = (np.arange(len(items)) < cap) & (boff + sizes <= bcap)
        cut = int(np.argmin(fits)) if not fits.all() else len(items)
        assert fits[:cut].all() and not fits[cut:].any()  # a prefix
        cut_bytes = int(boff[cut]) if cut < len(items) else int(sizes.sum())
        stream = np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
        c = np.zeros(1, dtype=COUNTS_DTYPE)
        c[0] = (len(items), int(sizes.sum()), cut, cut_bytes)
        out.append({"counts": c, "slot_recs": items[:cut], "slot_blob": stream[:cut_bytes],
                    "spill_recs": items[cut:], "spill_blob": stream[cut_bytes:]})
    return out


def shard_unpack_np(received):
    """received: per source s (rank order) the dict shard_pack_np made for this owner.
    -> (records with dgram_idx = i, dgram_off u64, arena u8, origin (rank u32, dgram_idx u32))."""
    rank, didx = [], []
    recs = [np.concatenate([x["slot_recs"], x["spill_recs"]]) for x in received]
    for s, r in enumerate(recs):
        rank.append(np.full(len(r), s, dtype=np.uint32))
        didx.append(r["dgram_idx"].astype(np.uint32))
    allr = np.concatenate(recs) if recs else np.zeros(0, dtype=received[0]["slot_recs"].dtype)
    blobs = np.concatenate([np.zeros(LEAD, np.uint8)] + [np.concatenate([x["slot_blob"], x["spill_blob"]])
                                                          for x in received])
    out = allr.copy()
    off = np.zeros(len(out), dtype=np.uint64)
    pos = LEAD
    for i, r in enumerate(out):
        rel, ln = _blob(r)
        off[i] = pos - rel
        pos += _r16(ln)
        out[i]["dgram_idx"] = i
    assert pos == len(blobs)
    return out, off, blobs, (np.concatenate(rank) if rank else np.zeros(0, np.uint32),
                             np.concatenate(didx) if didx else np.zeros(0, np.uint32))
