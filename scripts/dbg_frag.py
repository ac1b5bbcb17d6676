import sys, numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/rustdds-io_uring_amd", "/root/repo/tests"]
import oracle, frag_ref, rtps_rx
rx = rtps_rx.MessageReceiver(oracle.OWN_PREFIX, max_datagrams=1 << 16)
fa = oracle.FragAssembler()
arena, off, ln = oracle.pack(frag_ref.soup(3000, 1), align=1)
res, samples, heap, ns, used, npend = rx.assemble_batch(arena, off, ln)
st, recs, _, _ = oracle.parse(arena, off, ln, threads=8)
o_samples, o_heap, o_n, o_used = fa.batch(arena, off, recs)[:4]
bad = 0
for s in samples[samples["status"] != 2]:
    o, d = int(s["heap_off"]), int(s["data_size"])
    a, b = heap[o:o + d], o_heap[o:o + d]
    if a.tobytes() != b.tobytes():
        idx = np.nonzero(a != b)[0]
        print("sn", s["sn"], "size", d, "rec", s["rec_idx"], "diff", len(idx), "first", idx[:4], "last", idx[-4:], "gpu zeros", int((a[idx] == 0).sum()))
        bad += 1
        if bad > 6: break
print("bad", bad)
