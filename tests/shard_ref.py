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


def desc_bucket_np(recs, table_guids, world):
    """numpy reference of rtps_rx_bucket_descriptors: MATCHED records of table writers,
    owner = writer set index (rank of the GUID's first appearance) % world, stable; returns
    (list per owner of XDESC rows)."""
    from rtps_rx.records import XDESC_DTYPE, ROUTE_MATCHED
    index = {}
    for g in table_guids:
        index.setdefault(bytes(g), len(index))
    out = [[] for _ in range(world)]
    for i, r in enumerate(recs):
        if not (int(r["route"]) & ROUTE_MATCHED):
            continue
        k = index.get(bytes(r["prefix"]) + bytes(r["writer_id"]))
        if k is None:
            continue
        out[k % world].append((int(r["sn"]), i, (k << 8) | int(r["kind"])))
    return [np.array(o, dtype=XDESC_DTYPE) for o in out]
