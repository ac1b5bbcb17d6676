/*
 * rtps_gen.h — deterministic synthetic RTPS datagram generator f(seed, idx).
 *
 * Shared by the device generator kernel (rtps_rx.hip) and the host build
 * used by the CPU tests / CPU baseline (oracle/).  It produces datagrams
 * laid out exactly like the reference writer's MessageBuilder output:
 *   DATA      : octetsToInlineQos = 16, payload after the 20-byte DATA header
 *               (src/messages/submessages/data.rs:185-213, rtps/message.rs:146-325)
 *   DATA_FRAG : octetsToInlineQos = 28, one fragment per message
 *               (data_frag.rs:260-280, rtps/message.rs:326-464, io_uring/rtps/writer.rs:806-830)
 *   everything little-endian unless the workload asks for big-endian
 *   submessages (io_uring/rtps/writer.rs:332).
 * Workloads are the BASELINE configs.  This is input
 * production, not parsing: it contains no parse logic.
 *
 * Plain C99 so that gcc (oracle/) and hipcc (device) compile the same text.
 */
#ifndef RTPS_GEN_H
#define RTPS_GEN_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RG_HD __host__ __device__
#else
#define RG_HD
#endif

#define RG_SEED_DEFAULT 0x52545053ull /* "RTPS" */

/* participant prefix used as "own" by the tests: the target prefix of the
 * reference's receiver tests (rtps/message_receiver.rs:1138-1140). */
#define RG_OWN_PREFIX_INIT {0x01, 0x03, 0x00, 0x0c, 0x29, 0x2d, 0x31, 0xa2, 0x28, 0x20, 0x02, 0x08}

RG_HD static inline uint64_t rg_mix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
RG_HD static inline uint64_t rg_hash3(uint64_t a, uint64_t b, uint64_t c) {
  return rg_mix(a ^ rg_mix(b ^ rg_mix(c)));
}

typedef struct rg_rng { uint64_t s; } rg_rng;
RG_HD static inline uint32_t rg_next(rg_rng* r) {
  r->s = rg_mix(r->s);
  return (uint32_t)(r->s >> 17);
}
RG_HD static inline uint32_t rg_below(rg_rng* r, uint32_t n) { return n ? rg_next(r) % n : 0u; }

/* byte sink; out == 0 -> only count */
typedef struct rg_w {
  uint8_t* out;
  uint32_t pos;
  uint64_t fill_key; /* per-datagram key for payload fill words */
} rg_w;

RG_HD static inline void rg_put8(rg_w* w, uint32_t v) {
  if (w->out) w->out[w->pos] = (uint8_t)v;
  w->pos += 1;
}
RG_HD static inline void rg_put16(rg_w* w, uint32_t v, int le) {
  if (le) { rg_put8(w, v); rg_put8(w, v >> 8); }
  else { rg_put8(w, v >> 8); rg_put8(w, v); }
}
RG_HD static inline void rg_put32(rg_w* w, uint32_t v, int le) {
  if (le) { rg_put16(w, v & 0xffff, 1); rg_put16(w, v >> 16, 1); }
  else { rg_put16(w, v >> 16, 0); rg_put16(w, v & 0xffff, 0); }
}
RG_HD static inline void rg_put_bytes(rg_w* w, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) rg_put8(w, b[i]);
}
/* pseudo-random payload bytes; aligned word stores when possible */
RG_HD static inline void rg_put_fill(rg_w* w, uint32_t n) {
  if (!w->out) { w->pos += n; return; }
  uint32_t i = 0;
  while (i < n && ((w->pos & 3u) != 0)) { rg_put8(w, (uint32_t)rg_mix(w->fill_key + w->pos)); ++i; }
  if (((uintptr_t)(w->out) & 3u) == 0) {
    for (; i + 4 <= n; i += 4) {
      *(uint32_t*)(w->out + w->pos) = (uint32_t)rg_mix(w->fill_key + w->pos);
      w->pos += 4;
    }
  }
  for (; i < n; ++i) rg_put8(w, (uint32_t)rg_mix(w->fill_key + w->pos));
}
RG_HD static inline void rg_sn(rg_w* w, int64_t sn, int le) {
  rg_put32(w, (uint32_t)(uint64_t)((sn >> 32) & 0xffffffff), le);
  rg_put32(w, (uint32_t)(uint64_t)(sn & 0xffffffff), le);
}

/* writer w of the workload: GuidPrefix bytes (deterministic in seed, w) */
RG_HD static inline void rg_writer_prefix(uint64_t seed, uint32_t w, uint8_t p[12]) {
  uint64_t a = rg_hash3(seed, w, 0x5052454649ull);
  uint64_t b = rg_hash3(seed, w, 0x5052454650ull);
  p[0] = 0x01; p[1] = 0x0f;
  for (int i = 0; i < 8; ++i) p[2 + i] = (uint8_t)(a >> (8 * i));
  p[10] = (uint8_t)b; p[11] = (uint8_t)(b >> 8);
}
/* user-defined entity id of writer w: key (w+1, 3 bytes BE), kind 0x02 */
RG_HD static inline void rg_writer_eid(uint32_t w, uint8_t e[4]) {
  uint32_t k = w + 1u;
  e[0] = (uint8_t)(k >> 16); e[1] = (uint8_t)(k >> 8); e[2] = (uint8_t)k; e[3] = 0x02;
}

RG_HD static inline void rg_rtps_header(rg_w* w, const uint8_t prefix[12], uint32_t major) {
  rg_put8(w, 'R'); rg_put8(w, 'T'); rg_put8(w, 'P'); rg_put8(w, 'S');
  rg_put8(w, major); rg_put8(w, 4);   /* ProtocolVersion 2.4 */
  rg_put8(w, 0x01); rg_put8(w, 0x12); /* VendorId ATOSTEK */
  rg_put_bytes(w, prefix, 12);
}

/* A ShapeType sample {color: String, x: i32, y: i32, shapesize: i32} (the shapes demo
 * type of the reference's receiver test, rtps/message_receiver.rs:1250-1254) in classic
 * CDR after the encapsulation header, byte order le; values from the fill key (no rng
 * draws, so the rest of the datagram does not depend on it).  Returns bytes written,
 * 0 if n is too short (then the payload stays fill bytes). */
RG_HD static inline uint32_t rg_shape(rg_w* w, int le, uint32_t n) {
  const char* colors[8] = {"RED", "GREEN", "BLUE", "YELLOW", "ORANGE", "CYAN", "MAGENTA", "PURPLE"};
  const uint64_t h = rg_mix(w->fill_key ^ ((uint64_t)w->pos << 20));
  const char* c = colors[h & 7u];
  uint32_t len = 0;
  while (c[len]) ++len;
  const uint32_t str = 4u + ((len + 1u + 3u) & ~3u);
  if (n < str + 12u) return 0;
  rg_put32(w, len + 1u, le);
  for (uint32_t i = 0; i < len; ++i) rg_put8(w, (uint8_t)c[i]);
  for (uint32_t i = len; i < str - 4u; ++i) rg_put8(w, 0);  /* NUL + alignment of x */
  rg_put32(w, (uint32_t)((h >> 8) % 300u), le);
  rg_put32(w, (uint32_t)((h >> 24) % 300u), le);
  rg_put32(w, 10u + (uint32_t)((h >> 40) % 50u), le);
  return str + 12u;
}

/* DATA submessage with MessageBuilder::data_msg layout (otq = 16).  shape: a D payload
 * starts with a ShapeType sample (the C3 mix), the rest is fill. */
RG_HD static inline void rg_data(rg_w* w, int le, uint32_t flags_extra, const uint8_t rid[4],
                                 const uint8_t wid[4], int64_t sn, uint32_t qos_bytes,
                                 rg_rng* r, uint32_t payload, int shape) {
  uint32_t flags = (le ? 0x01u : 0x00u) | flags_extra;
  rg_put8(w, 0x15); rg_put8(w, flags);
  rg_put16(w, 20u + qos_bytes + payload, le);
  rg_put16(w, 0, le);  /* extraFlags */
  rg_put16(w, 16, le); /* octetsToInlineQos */
  rg_put_bytes(w, rid, 4);
  rg_put_bytes(w, wid, 4);
  rg_sn(w, sn, le);
  if (qos_bytes) {
    /* inline QoS: STATUS_INFO, [KEY_HASH], [RELATED_SAMPLE_IDENTITY], SENTINEL
       (pids: structure/parameter_id.rs:64-65,97; layout inline_qos.rs) */
    uint32_t left = qos_bytes - 4; /* sentinel */
    if (left >= 8) { rg_put16(w, 0x0071, le); rg_put16(w, 4, le); rg_put8(w, 0); rg_put8(w, 0); rg_put8(w, 0); rg_put8(w, 1 + rg_below(r, 3)); left -= 8; }
    if (left >= 20) { rg_put16(w, 0x0070, le); rg_put16(w, 16, le); rg_put_fill(w, 16); left -= 20; }
    if (left >= 28) { rg_put16(w, 0x0083, le); rg_put16(w, 24, le); rg_put_fill(w, 24); left -= 28; }
    while (left >= 4) { rg_put16(w, 0x0000, le); rg_put16(w, 0, le); left -= 4; } /* PID_PAD */
    rg_put16(w, 0x0001, le); rg_put16(w, 0, le); /* PID_SENTINEL */
  }
  if (payload) {
    /* SerializedPayload: encapsulation (CDR_LE / CDR_BE) + options, then data */
    rg_put8(w, 0x00); rg_put8(w, le ? 0x01 : 0x00); rg_put8(w, 0); rg_put8(w, 0);
    const uint32_t used = (shape && (flags & 0x04u)) ? rg_shape(w, le, payload - 4) : 0u;
    rg_put_fill(w, payload - 4 - used);
  }
}

/* Build datagram idx of workload wl into out (or only size it when out == 0).
 * Returns the datagram length.  max length: 1503 (C3), 1400 (C4). */
RG_HD static inline uint32_t rtps_gen_datagram(int wl, uint64_t seed, uint64_t idx,
                                               uint32_t n_writers, uint8_t* out) {
  rg_w w; w.out = out; w.pos = 0; w.fill_key = rg_hash3(seed, idx, 0x46494c4cull);
  rg_rng r; r.s = rg_hash3(seed, idx, wl);
  if (n_writers == 0) n_writers = 1;
  uint8_t prefix[12], wid[4];
  const uint8_t zero_eid[4] = {0, 0, 0, 0};

  if (wl == 1 || wl == 2) { /* T: 1024 B, C2: 300 B — one DATA each */
    uint32_t payload = (wl == 1) ? 980u : 256u;
    uint32_t wr = (uint32_t)(idx % n_writers);
    int64_t sn = (int64_t)(idx / n_writers) + 1;
    rg_writer_prefix(seed, wr, prefix);
    rg_writer_eid(wr, wid);
    rg_rtps_header(&w, prefix, 2);
    rg_data(&w, 1, 0x04, zero_eid, wid, sn, 0, &r, payload, 0);
    return w.pos;
  }

  if (wl == 4) { /* C4: DATA_FRAG, 64 KiB samples, 1344-B fragments, ±8 shuffle */
    const uint32_t frag_size = 1344u, data_size = 65536u, nfrag = 49u;
    uint64_t blk = idx / 8u; uint32_t j = (uint32_t)(idx % 8u);
    uint8_t perm[8];
    for (uint32_t i = 0; i < 8; ++i) perm[i] = (uint8_t)i;
    rg_rng pr; pr.s = rg_hash3(seed, blk, 0x5045524dull);
    for (uint32_t i = 7; i > 0; --i) { uint32_t k = rg_below(&pr, i + 1); uint8_t t = perm[i]; perm[i] = perm[k]; perm[k] = t; }
    uint64_t li = blk * 8u + perm[j];
    uint64_t g = li / nfrag; uint32_t k = (uint32_t)(li % nfrag);
    uint32_t wr = (uint32_t)(g % n_writers);
    int64_t sn = (int64_t)(g / n_writers) + 1;
    uint32_t fl = (k == nfrag - 1) ? (data_size - (nfrag - 1) * frag_size) : frag_size;
    rg_writer_prefix(seed, wr, prefix);
    rg_writer_eid(wr, wid);
    rg_rtps_header(&w, prefix, 2);
    rg_put8(&w, 0x16); rg_put8(&w, 0x01); rg_put16(&w, 32u + fl, 1);
    rg_put16(&w, 0, 1); rg_put16(&w, 28, 1);
    rg_put_bytes(&w, zero_eid, 4); rg_put_bytes(&w, wid, 4);
    rg_sn(&w, sn, 1);
    rg_put32(&w, k + 1u, 1);          /* fragmentStartingNum */
    rg_put16(&w, 1, 1);               /* fragmentsInSubmessage */
    rg_put16(&w, frag_size, 1);       /* fragmentSize */
    rg_put32(&w, data_size, 1);       /* sampleSize */
    if (k == 0) { rg_put8(&w, 0); rg_put8(&w, 1); rg_put8(&w, 0); rg_put8(&w, 0); rg_put_fill(&w, fl - 4); }
    else rg_put_fill(&w, fl);
    return w.pos;
  }

  /* C3: mixed stream, 16 writers (n_writers), 128..1500 B */
  uint32_t S = 128u + 4u * rg_below(&r, 344);
  uint32_t malformed = (rg_below(&r, 100) == 0) ? (1u + rg_below(&r, 8)) : 0u;
  uint32_t hw = rg_below(&r, n_writers);
  rg_writer_prefix(seed, hw, prefix);
  if (malformed == 5) { /* short datagram */
    rg_put8(&w, 'R'); rg_put8(&w, 'T'); rg_put8(&w, 'P'); rg_put8(&w, 'S');
    for (uint32_t i = 0; i < 8; ++i) rg_put8(&w, prefix[i]);
    return w.pos;
  }
  if (malformed == 6) { /* RTPS ping, 16 bytes */
    const uint8_t ping[16] = {'R', 'T', 'P', 'S', 2, 4, 1, 0x12, 0, 'D', 'D', 'S', 'P', 'I', 'N', 'G'};
    rg_put_bytes(&w, ping, 16);
    return w.pos;
  }
  uint32_t hdr_start = w.pos;
  rg_rtps_header(&w, prefix, (malformed == 4) ? 3u : 2u);
  if (malformed == 2 && out) { out[hdr_start + 3] = 'X'; }
  if (malformed == 3 && out) { out[hdr_start + 0] = 'X'; }
  const uint8_t own[12] = RG_OWN_PREFIX_INIT;
  int first_le = rg_below(&r, 10) != 0;
  uint32_t first_kind_pos = w.pos;
  if (rg_below(&r, 100) < 70) { /* INFO_TS */
    rg_put8(&w, 0x09); rg_put8(&w, first_le ? 1 : 0); rg_put16(&w, (malformed == 7) ? 0 : 8, first_le);
    rg_put32(&w, 1700000000u + (uint32_t)(idx & 0xffff), first_le);
    rg_put32(&w, rg_next(&r), first_le);
  } else { /* INFO_DST: 75 % own, 25 % someone else */
    uint8_t dst[12];
    if (rg_below(&r, 4) != 0) { for (int i = 0; i < 12; ++i) dst[i] = own[i]; }
    else rg_writer_prefix(seed ^ 0xd57ull, rg_below(&r, 1000), dst);
    rg_put8(&w, 0x0e); rg_put8(&w, first_le ? 1 : 0); rg_put16(&w, (malformed == 7) ? 8 : 12, first_le);
    rg_put_bytes(&w, dst, 12);
  }
  (void)first_kind_pos;
  uint32_t last_sub = w.pos;
  int have_data = 0;
  while (S - w.pos >= 48u) {
    uint32_t rem = S - w.pos;
    uint32_t pick = rg_below(&r, 100);
    int le = rg_below(&r, 10) != 0;
    uint32_t wr = rg_below(&r, n_writers);
    uint8_t weid[4]; rg_writer_eid(wr, weid);
    int64_t sn = 1 + (int64_t)rg_below(&r, 100000);
    last_sub = w.pos;
    if (pick < 60) { /* DATA */
      uint32_t qos = (rg_below(&r, 20) == 0) ? (4u + 4u * rg_below(&r, 16)) : 0u;
      if (24u + qos + 8u > rem) qos = 0;
      uint32_t avail = rem - 24u - qos;
      uint32_t payload;
      if (avail < 300u || rg_below(&r, 3) == 0) payload = avail;
      else payload = 8u + 4u * rg_below(&r, (avail - 8u) / 4u);
      uint32_t variant = rg_below(&r, 50);
      uint32_t fl = (qos ? 0x02u : 0u);
      if (variant == 0 && qos) { fl |= 0x00u; payload = 0; } /* key-hash-only DATA */
      else if (variant == 1) fl |= 0x08u;                      /* key payload */
      else fl |= 0x04u;                                        /* data payload */
      if (malformed == 8 && !have_data) {
        /* octetsToInlineQos < 16 -> DATA error (data.rs:86-91) */
        uint32_t at = w.pos;
        rg_data(&w, le, fl, zero_eid, weid, sn, qos, &r, payload, 1);
        if (out) { if (le) { out[at + 6] = 8; out[at + 7] = 0; } else { out[at + 6] = 0; out[at + 7] = 8; } }
      } else {
        rg_data(&w, le, fl, zero_eid, weid, sn, qos, &r, payload, 1);
      }
      have_data = 1;
    } else if (pick < 75) { /* HEARTBEAT (heartbeat.rs:21-49) */
      rg_put8(&w, 0x07); rg_put8(&w, (le ? 1u : 0u) | (rg_below(&r, 2) ? 2u : 0u)); rg_put16(&w, 28, le);
      rg_put_bytes(&w, zero_eid, 4); rg_put_bytes(&w, weid, 4);
      rg_sn(&w, 1, le); rg_sn(&w, sn, le); rg_put32(&w, rg_below(&r, 1000), le);
    } else if (pick < 85) { /* ACKNACK from one of our readers (ack_nack.rs:27-50) */
      uint32_t nb = rg_below(&r, 65), words = (nb + 31u) / 32u;
      uint8_t reid[4] = {0, 0, (uint8_t)(1 + rg_below(&r, 8)), 0x07};
      rg_put8(&w, 0x06); rg_put8(&w, (le ? 1u : 0u) | 2u); rg_put16(&w, 24u + 4u * words, le);
      rg_put_bytes(&w, reid, 4); rg_put_bytes(&w, weid, 4);
      rg_sn(&w, sn, le); rg_put32(&w, nb, le);
      for (uint32_t i = 0; i < words; ++i) rg_put32(&w, rg_next(&r), le);
      rg_put32(&w, rg_below(&r, 1000), le);
    } else if (pick < 95) { /* GAP (gap.rs:23-46) */
      uint32_t nb = rg_below(&r, 65), words = (nb + 31u) / 32u;
      rg_put8(&w, 0x08); rg_put8(&w, le ? 1u : 0u); rg_put16(&w, 28u + 4u * words, le);
      rg_put_bytes(&w, zero_eid, 4); rg_put_bytes(&w, weid, 4);
      rg_sn(&w, sn, le); rg_sn(&w, sn + 1, le); rg_put32(&w, nb, le);
      for (uint32_t i = 0; i < words; ++i) rg_put32(&w, rg_next(&r), le);
    } else if (rg_below(&r, 2)) { /* mid-datagram INFO_TS (sometimes invalidate) */
      if (rg_below(&r, 4) == 0) { rg_put8(&w, 0x09); rg_put8(&w, (le ? 1u : 0u) | 2u); rg_put16(&w, 0, le); }
      else { rg_put8(&w, 0x09); rg_put8(&w, le ? 1u : 0u); rg_put16(&w, 8, le); rg_put32(&w, 1700000000u + rg_below(&r, 1000), le); rg_put32(&w, rg_next(&r), le); }
    } else { /* INFO_SRC (info_source.rs:22-36) */
      uint8_t src[12]; rg_writer_prefix(seed, rg_below(&r, n_writers), src);
      rg_put8(&w, 0x0c); rg_put8(&w, le ? 1u : 0u); rg_put16(&w, 20, le);
      rg_put32(&w, 0, le); rg_put8(&w, 2); rg_put8(&w, 4); rg_put8(&w, 0x01); rg_put8(&w, 0x12);
      rg_put_bytes(&w, src, 12);
    }
  }
  if (S - w.pos >= 4u) { /* PAD to the chosen size (skipped by the parser) */
    uint32_t rem = S - w.pos;
    last_sub = w.pos;
    rg_put8(&w, 0x01); rg_put8(&w, 0x01); rg_put16(&w, rem - 4u, 1);
    rg_put_fill(&w, rem - 4u);
  }
  if (malformed == 1) { /* trailing 1..3 bytes -> SubmessageHeader read error */
    uint32_t extra = 1u + (uint32_t)(idx % 3u);
    rg_put_fill(&w, extra);
  }
  if (malformed == 8 && !have_data) { /* no DATA to corrupt: declare a too-long last submessage */
    if (out) { uint32_t len_at = last_sub + 2; int le = out[last_sub + 1] & 1;
      uint32_t cur = le ? (out[len_at] | (out[len_at + 1] << 8)) : ((out[len_at] << 8) | out[len_at + 1]);
      cur += 4u;
      if (le) { out[len_at] = (uint8_t)cur; out[len_at + 1] = (uint8_t)(cur >> 8); }
      else { out[len_at] = (uint8_t)(cur >> 8); out[len_at + 1] = (uint8_t)cur; } }
  }
  return w.pos;
}

/* Host: datagram lengths and 16-B aligned arena offsets. Returns arena bytes. */
static inline uint64_t rtps_gen_layout_host(int wl, uint64_t seed, uint64_t first_idx,
                                            uint32_t n_writers, uint32_t n, uint64_t* off,
                                            uint32_t* len) {
  uint64_t pos = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t l = rtps_gen_datagram(wl, seed, first_idx + i, n_writers, (uint8_t*)0);
    off[i] = pos;
    len[i] = l;
    pos += ((uint64_t)l + 15u) & ~(uint64_t)15u;
  }
  return pos;
}

#endif /* RTPS_GEN_H */
