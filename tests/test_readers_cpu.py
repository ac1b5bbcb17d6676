"""CPU checks of the reader-set contract (a15, no GPU needed): the target sets the
library's host builder makes (rtps_rx_debug_target_sets, the code behind
rtps_rx_set_readers) against the oracle's literal available_readers scan
(dp_event_loop.rs:266-327, reader.rs:474-484, 712-739), their numbering, and the
validation errors."""
import ctypes

import numpy as np
import pytest

import ingest_ref as R
import oracle
from rtps_rx.records import (RECORD_DTYPE, TARGET_DTYPE, DATA, Readers, READER_STATELESS, NO_PROXY)


def _build(rd):
    import rtps_rx
    L = rtps_rx.lib()
    fn = L.rtps_rx_debug_target_sets
    fn.restype = ctypes.c_int
    P, U32 = ctypes.c_void_p, ctypes.c_uint32
    fn.argtypes = [P, U32, P, U32, P, U32, P, U32, ctypes.POINTER(U32), ctypes.POINTER(U32)]
    cap = 4096
    first = np.zeros(cap + 1, dtype=np.uint32)
    ent = np.zeros(cap, dtype=TARGET_DTYPE)
    ns, nw = U32(), U32()
    r, p = rd.readers, rd.proxies
    rc = fn(r.ctypes.data if len(r) else None, len(r), p.ctypes.data if len(p) else None, len(p),
            first.ctypes.data, cap, ent.ctypes.data, cap, ctypes.byref(ns), ctypes.byref(nw))
    if rc:
        return rc, None, None, 0
    return 0, first[:ns.value + 1], ent[:first[ns.value]], nw.value


def _fake_records(guids):
    recs = np.zeros(len(guids), dtype=RECORD_DTYPE)
    for i, g in enumerate(guids):
        recs[i]["kind"] = DATA
        recs[i]["prefix"] = np.frombuffer(g[:12], dtype=np.uint8)
        recs[i]["writer_id"] = np.frombuffer(g[12:], dtype=np.uint8)
    return recs


def _check_sets(rd):
    rc, first, ent, nw = _build(rd)
    assert rc == 0
    # writer sets: distinct GUIDs of non-stateless readers' proxies, first-appearance order
    wg = []
    for p in rd.proxies:
        if rd.readers[int(p["reader"])]["flags"] & READER_STATELESS:
            continue
        g = bytes(p["writer_guid"])
        if g not in wg:
            wg.append(g)
    eids = []
    for g in wg:
        if g[12:] not in eids:
            eids.append(g[12:])
    assert nw == len(wg) and len(first) - 1 == len(wg) + len(eids)
    unknown = bytes([0xEE] * 12)  # a prefix no proxy has: entity-only targeting
    o_off, o_ent = oracle.targets(_fake_records(wg + [unknown + e for e in eids]), rd)
    for s in range(len(first) - 1):
        got = ent[first[s]:first[s + 1]]
        exp = o_ent[int(o_off[s]):int(o_off[s + 1])]
        assert got.tobytes() == exp.tobytes(), s
        if s >= nw:
            assert (got["proxy"] == NO_PROXY).all()
    return first, ent


def test_a15_sets_match_oracle_scan():
    first, ent = _check_sets(R.a15_readers())
    assert np.max(np.diff(first)) >= 3  # writer 0: readers 10, 11 and the participant reader


def test_compat_table_sets_match_oracle_scan():
    tbl, _ = R.table()
    _check_sets(Readers.from_match(tbl))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_tables_match_oracle_scan(seed):
    rng = np.random.default_rng(seed)
    nr = int(rng.integers(1, 9))
    eids = rng.choice(200, size=nr, replace=False)
    readers = [(bytes([0, int(e) // 16, int(e) % 16, 0x07]), 100 + k, int(rng.integers(0, 4)) & 3)
               for k, e in enumerate(eids)]
    proxies, seen = [], set()
    for _ in range(int(rng.integers(0, 40))):
        g = R.PREFIXES[int(rng.integers(4))] + R.writer_key(int(rng.integers(5)))
        r = int(rng.integers(nr))
        if (g, r) not in seen:
            seen.add((g, r))
            proxies.append((g, r))
    _check_sets(Readers(readers, proxies))


def test_validation_errors():
    P = R.PREFIXES
    dup_reader = Readers([(b"\0\0\1\7", 1, 0), (b"\0\0\1\7", 2, 0)], [])
    dup_proxy = Readers([(b"\0\0\1\7", 1, 0)], [(P[0] + R.writer_key(0), 0)] * 2)
    bad_index = Readers([(b"\0\0\1\7", 1, 0)], [(P[0] + R.writer_key(0), 1)])
    for rd in (dup_reader, dup_proxy, bad_index):
        assert _build(rd)[0] == -1  # RTPS_RX_EINVAL
    assert _build(Readers())[0] == 0


_RT_FAIL_SCRIPT = r'''
import ctypes, sys
import numpy as np
sys.path[:0] = sys.argv[1:3]
import rtps_rx
from rtps_rx.records import Readers
L = rtps_rx.lib()
P, U32 = ctypes.c_void_p, ctypes.c_uint32
class View(ctypes.Structure):
    _fields_ = [(n, P) for n in ("gkeys", "gset", "ekeys", "eset", "set_first", "set_ent")] + \
               [(n, U32) for n in ("gmask", "emask", "n_writer_sets", "n_sets", "n_proxies", "max_set", "n_ent")]
L.rtps_rx_debug_rt_view_size.restype = U32
assert ctypes.sizeof(View) == L.rtps_rx_debug_rt_view_size(), "View must mirror ReaderDev exactly"
L.rtps_rx_debug_rt_new.restype = P
L.rtps_rx_debug_rt_free.argtypes = [P]
L.rtps_rx_debug_rt_set.argtypes = [P, P, U32, P, U32]
L.rtps_rx_debug_rt_view.argtypes = [P, ctypes.POINTER(View)]
def table(n_writers, slot):
    rd = Readers([(bytes([0, 0, slot, 7]), slot, 0)], [(bytes([9] * 12) + bytes([0, 0, w, 2]), 0) for w in range(n_writers)])
    return rd.readers, rd.proxies
def rt_set(t, rd):
    return L.rtps_rx_debug_rt_set(t, rd[0].ctypes.data, len(rd[0]), rd[1].ctypes.data, len(rd[1]))
def view(t):
    v = View(); L.rtps_rx_debug_rt_view(t, ctypes.byref(v)); return v
def words(addr, n):
    return np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(ctypes.c_uint32)), shape=(n,)).copy()
L.rtps_rx_debug_rt_host_mode(-1)
t = L.rtps_rx_debug_rt_new()
a, b = table(3, 1), table(40, 2)
assert rt_set(t, a) == 0
va = view(t)
ga = words(va.gset, va.gmask + 1)
for fail_at in range(1):  # the one table image buffer
    L.rtps_rx_debug_rt_host_mode(fail_at)
    assert rt_set(t, b) == -3, fail_at             # RTPS_RX_ENOMEM
    v = view(t)
    assert (v.gkeys, v.gset, v.ekeys, v.eset, v.set_first, v.set_ent) == \
           (va.gkeys, va.gset, va.ekeys, va.eset, va.set_first, va.set_ent), fail_at
    assert (v.gmask, v.n_sets, v.n_proxies) == (va.gmask, va.n_sets, va.n_proxies) == (va.gmask, 6, 3)
    assert np.array_equal(words(v.gset, v.gmask + 1), ga)
L.rtps_rx_debug_rt_host_mode(-1)
assert rt_set(t, b) == 0
vb = view(t)
assert vb.n_proxies == 40 and vb.n_sets == 80 and vb.gkeys
assert sorted(words(vb.gset, vb.gmask + 1).tolist())[:40] == list(range(40))
L.rtps_rx_debug_rt_free(t)
print("ok")
'''


def test_failed_set_readers_keeps_previous_table():
    """a set_readers whose allocation fails part-way must leave the previous
    device tables whole (build into new buffers, swap on success).  Host-memory mode of the
    table's allocator, failing its one image buffer (isolated process)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    r = subprocess.run([sys.executable, "-c", _RT_FAIL_SCRIPT, os.path.join(repo, "rustdds-io_uring_amd"), repo],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


_RT_IMAGE_SCRIPT = _RT_FAIL_SCRIPT.split("L.rtps_rx_debug_rt_host_mode(-1)\nt = ")[0] + r'''
L.rtps_rx_debug_rt_host_mode(-1)
RT_LDS_MAX = 48 * 1024
def lds_bytes(gcap, ecap):
    return gcap * 20 + ecap * 8
def pow2(n):
    p = 1
    while p < n:
        p <<= 1
    return p
def wide_table(n_writers):
    rd = Readers([(bytes([0, 0, 1, 7]), 1, 0)],
                 [(bytes([9] * 12) + bytes([0, w >> 8, w & 255, 2]), 0) for w in range(n_writers)])
    return rd.readers, rd.proxies
t = L.rtps_rx_debug_rt_new()
for n_writers in (3, 40, 256, 600, 1500):
    assert rt_set(t, wide_table(n_writers)) == 0
    v = view(t)
    gcap, ecap = v.gmask + 1, v.emask + 1
    # sparse slots (load <= 1/4) while the tables fit the LDS limit, else the dense ones (<= 1/2)
    if lds_bytes(pow2(4 * n_writers), pow2(4 * n_writers)) <= RT_LDS_MAX:
        assert gcap == pow2(4 * n_writers), (n_writers, gcap)
    else:
        assert gcap == pow2(2 * n_writers), (n_writers, gcap)
    # one image in the LDS layout: gkeys, gset, ekeys, eset, set_first, set_ent back to back
    assert v.gset == v.gkeys + 16 * gcap and v.ekeys == v.gset + 4 * gcap
    assert v.eset == v.ekeys + 4 * ecap and v.set_first == v.eset + 4 * ecap
    assert v.set_ent == v.set_first + 4 * (v.n_sets + 1)
    gs = words(v.gset, gcap)
    assert sorted(gs[gs != 0xFFFFFFFF].tolist()) == list(range(n_writers))
L.rtps_rx_debug_rt_free(t)
print("ok")
'''


def test_reader_table_image_layout():
    """Round 4: the reader tables are one device image in their LDS layout (staged by one flat
    copy), with hash slots at load <= 1/4 while they fit RT_LDS_MAX and <= 1/2 past it
    (host-memory mode of the table's allocator, isolated process)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    r = subprocess.run([sys.executable, "-c", _RT_IMAGE_SCRIPT, os.path.join(repo, "rustdds-io_uring_amd"), repo],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
