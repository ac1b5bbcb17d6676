"""The reference's own Reader unit tests as wire event streams (test helper).

Loads tests/golden/reader_known_answers.json (built by
tests/golden/make_reader_cases.py from the literals and assertions of
io_uring/rtps/reader.rs:1537-1988) and checks one ingest implementation
against it: `run(case, batch_fn)` where batch_fn(readers, arena, off, len)
returns (records, deliveries, ack_base, targets) for one batch, with state
carried across calls."""
import json
import os

import numpy as np

import oracle
from rtps_rx.records import Readers, NO_TARGET

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reader_known_answers.json")


def cases():
    with open(_PATH) as f:
        return json.load(f)["cases"]


def readers(case):
    return Readers([(bytes.fromhex(r["entity_id"]), r["reader_slot"], r["flags"]) for r in case["readers"]],
                   [(bytes.fromhex(p["writer_guid"]), p["reader"]) for p in case["proxies"]])


def check(case, batch_fn):
    """Feed the case's batches in order; assert every transcribed answer."""
    rd = readers(case)
    for k, b in enumerate(case["batches"]):
        arena, off, ln = oracle.pack([bytes.fromhex(d) for d in b["datagrams"]], align=4)
        recs, dels, ack, target = batch_fn(rd, arena, off, ln)
        label = f"{case['name']} batch {k}"
        got = [[int(d["rec_idx"]), int(d["reader_slot"])] for d in dels]
        assert got == b["deliveries"], f"{label}: deliveries {got} != {b['deliveries']}"
        if "ack_base" in b:
            assert np.asarray(ack).tolist() == b["ack_base"], f"{label}: all_ackable_before {ack} != {b['ack_base']}"
        if b.get("no_target"):
            assert all(int(t) == NO_TARGET for t in target), f"{label}: a stateless reader became a target"
        for d, exp in zip(dels, b.get("delivered", [])):
            r = recs[int(d["rec_idx"])]
            assert (bytes(r["prefix"]) + bytes(r["writer_id"])).hex() == exp["writer_guid"]
            assert int(r["sn"]) == exp["sn"]
            assert [int(r["ts_sec"]), int(r["ts_frac"])] == exp["ts"] and int(r["route"]) & 0x02
            u = r["u"].view(np.uint16)
            pl_off, pl_len = int(u[0]), int(u[1])
            dg = int(r["dgram_idx"])
            p = arena[int(off[dg]) + pl_off:int(off[dg]) + pl_off + pl_len].tobytes()
            assert p.hex() == exp["payload"], f"{label}: payload {p.hex()}"


def oracle_batch_fn():
    """batch_fn over the CPU oracle (parse with the readers, then the sequential ingest)."""
    state = {}

    def fn(rd, arena, off, ln):
        if "ing" not in state:
            state["ing"] = oracle.HistoryIngest(rd)
        st, recs, (toff, tent), _ = oracle.parse(arena, off, ln, match_table=rd)
        acc, dels, ack = state["ing"].batch(arena, off, recs)
        # the per-record target set is not in the oracle's output form: a record has a
        # target iff its expanded target list is non-empty
        target = np.where(np.diff(toff.astype(np.int64)) > 0, 0, NO_TARGET).astype(np.uint32)
        return recs, dels, ack, target
    return fn
