"""Compact view of a bench.py JSON line: the headline, the dominant kernel's roofline, the item
pass, the legs (ingest with / without topic caches, CDR, end to end incl. the full host chain,
the SPDP repeats case, the exchange prediction).  usage: python scripts/bench_summary.py FILE"""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline", {})
out = {"workload": d["config"]["workload"][:3], "value": d["value"], "ms_per_step": round(d["ms_per_step"] * 1e3, 1),
       "kernel": r.get("kernel"), "kernel_us": round((r.get("kernel_ms") or 0) * 1e3, 1), "frac": r.get("frac"),
       "item_us": round(r.get("item_kernel_ms", 0) * 1e3, 1), "emit_us": round(r.get("emit_kernel_ms", 0) * 1e3, 1),
       "item_pass_frac": r.get("item_pass_frac"), "attainable_frac": r.get("attainable_frac")}
ing = d.get("ingest", {})
out["ingest"] = {k: ing.get(k) for k in ("ms", "topic_cache_ms", "topic_cache_extra_ms", "frac", "window_overflow",
                                         "attainable_frac")}
e2e = d.get("end_to_end", {})
out["e2e"] = {k: (v.get("datagrams_per_s"), v.get("parity_ok")) for k, v in e2e.items() if isinstance(v, dict)
              and "datagrams_per_s" in v}
fc = e2e.get("full_chain", {})
out["full_chain"] = {k: (round(v["ms"], 2), v["datagrams_per_s"], v["parity_ok"]) for k, v in fc.items()
                     if isinstance(v, dict)}
sp = d.get("topic_cache_spdp_repeats", {})
out["spdp"] = {k: (round(v["ingest_ms"], 3), round(v["ingest_topic_cache_ms"], 3), v["parity_ok"]) for k, v in sp.items()
               if isinstance(v, dict)}
ex = d.get("exchange_prediction", {})
out["xgmi_ms"] = {k: round(v["predicted_xgmi_ms"], 3) for k, v in ex.items() if isinstance(v, dict)}
out["items_per_owner"] = {k: v["items_per_dest"] for k, v in ex.items() if isinstance(v, dict)}
out["cpu_baseline"] = d.get("cpu_baseline", {}).get("value")
print(json.dumps(out, indent=1))
