/*
 * rtps_oracle.c — CPU restatement of the RustDDS receive-path parse.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path and the "port" CPU baseline of bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product library (rustdds-io_uring_amd/csrc) never links it.
 *
 * Parity pinning: the reference is Rust and cannot be built in this image
 * (no cargo/rustc, crates not vendored: SURVEY.md §0, §8c).  This
 * restatement is pinned by the reference's own wire vectors and
 * assertions, extracted into tests/golden/ by tests/golden/make_golden.py
 * (see tests/test_oracle_golden.py).  Behaviour of the third-party `speedy`
 * 0.8 reader that no vector covers (INFO_REPLY Option tag, trailing bytes
 * after fixed-size bodies) is "parity unpinned" and documented in DESIGN.md.
 *
 * Structure mirrors the reference:
 *   rtps_message_read_from_buffer   <- Message::read_from_buffer   rtps/message.rs:64-81
 *   submessage_read_from_buffer     <- Submessage::read_from_buffer rtps/submessage.rs:56-295
 *   data_deserialize                <- Data::deserialize_data      messages/submessages/data.rs:57-144
 *   datafrag_deserialize            <- DataFrag::deserialize       messages/submessages/data_frag.rs:121-257
 *   parameter_list_read             <- ParameterList::read_from    elements/parameter_list.rs:79-102
 *   number_set_read                 <- NumberSet::read_from        structure/sequence_number.rs:464-498
 *   handle_received_packet_2        <- io_uring/rtps/message_receiver.rs:232-287
 *   interpreter (iter_next)         <- io_uring/rtps/message_receiver.rs:56-119, 618-665, 289-295
 *   data_to_dds_data_kind           <- io_uring/rtps/reader.rs:760-833
 *   deduce_change_kind              <- io_uring/rtps/reader.rs:1158-1182, elements/inline_qos.rs:27-42,139-175
 *   builtin pairs                   <- io_uring/discovery/discovery.rs:2795-2816, 3075-3095
 *   oracle_targets                  <- io_uring/rtps/dp_event_loop.rs:266-327 (available_readers
 *                                      filtered by contains_writer, reader.rs:474-484), matched
 *                                      writer proxy by full GUID (reader.rs:712-739)
 *   rtps_oracle_cdr_decode          <- cdr_adapters.rs:246-275 + cdr-encoding 0.10 rules
 *   rtps_oracle_frag_batch          <- rtps/fragment_assembler.rs:23-214, reader.rs:563-647
 *   rtps_oracle_ingest_batch        <- rtps/rtps_writer_proxy.rs:202-355, reader.rs:514-1116
 *   rtps_oracle_topics_apply        <- TopicCache::add_change, structure/dds_cache.rs:210-284, 367-420
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rtps_rx.h"
#include "../rustdds-io_uring_amd/csrc/rtps_gen.h"

/* ------------------------------------------------------------------------ */
/* speedy-style reader over a byte slice (io::Cursor + Endianness)          */
/* ------------------------------------------------------------------------ */
typedef struct cursor {
  const uint8_t* buf; /* slice start */
  size_t len;         /* slice length */
  size_t pos;         /* cursor position */
  int le;             /* endianness_flag(flags): submessage_flag.rs:36-42 */
} cursor;

static int rd_u8(cursor* c, uint8_t* v) {
  if (c->pos + 1 > c->len) return -1;
  *v = c->buf[c->pos++];
  return 0;
}
static int rd_u16(cursor* c, uint16_t* v) {
  if (c->pos + 2 > c->len) return -1;
  const uint8_t* p = c->buf + c->pos;
  *v = c->le ? (uint16_t)(p[0] | (p[1] << 8)) : (uint16_t)((p[0] << 8) | p[1]);
  c->pos += 2;
  return 0;
}
static int rd_u32(cursor* c, uint32_t* v) {
  if (c->pos + 4 > c->len) return -1;
  const uint8_t* p = c->buf + c->pos;
  *v = c->le ? ((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24))
             : (((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
  c->pos += 4;
  return 0;
}
static int rd_bytes(cursor* c, uint8_t* out, size_t n) {
  if (c->pos + n > c->len) return -1;
  memcpy(out, c->buf + c->pos, n);
  c->pos += n;
  return 0;
}
/* EntityId::read_from: 3 key bytes + kind byte (structure/guid.rs:495-505) */
static int rd_entity_id(cursor* c, uint8_t e[4]) { return rd_bytes(c, e, 4); }
/* SequenceNumber::read_from: i32 high then u32 low (sequence_number.rs:169-182) */
static int rd_sn(cursor* c, int64_t* sn) {
  uint32_t hi, lo;
  if (rd_u32(c, &hi) || rd_u32(c, &lo)) return -1;
  *sn = (int64_t)(((int64_t)(int32_t)hi) * 4294967296LL) + (int64_t)lo;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* parsed submessage (one element of Message.submessages)                    */
/* ------------------------------------------------------------------------ */
enum body_class { BODY_WRITER = 1, BODY_READER = 2, BODY_INTERP = 3 };

typedef struct submsg {
  uint32_t off;   /* submessage header offset within the datagram */
  uint8_t kind, flags;
  uint32_t content_len;
  int cls;
  uint8_t reader_id[4], writer_id[4];
  int64_t sn, sn2;
  int32_t count;
  uint32_t num_bits, bitmap_off, u32a;
  /* DATA / DATA_FRAG */
  int has_qos, has_payload;
  uint32_t qos_len, pl_off, pl_len;
  uint32_t key_hash_off, status_info_off, rsi_off;
  int si_seen;
  uint32_t si_len;
  uint32_t frag_start, frags_in_sub, frag_size, data_size;
  /* interpreter */
  uint8_t prefix[12];
  int ts_valid;
  uint32_t ts_sec, ts_frac;
  uint8_t version[2], vendor[2];
  uint32_t n_uni, n_multi;
} submsg;

/* ParameterList::read_from (parameter_list.rs:79-102): loop { pid u16, length u16;
 * pid == PID_SENTINEL -> stop (value not read); else read exactly `length`
 * bytes }.  Also records the first KEY_HASH (value must be 16 bytes,
 * key.rs:64-68 / inline_qos.rs:44-53), STATUS_INFO (inline_qos.rs:28-42) and
 * RELATED_SAMPLE_IDENTITY(_CUSTOM) (inline_qos.rs:56-85) values.
 * `dgram_base` converts cursor positions to datagram offsets. */
static int parameter_list_read(cursor* c, uint32_t dgram_base, submsg* s) {
  int seen_kh = 0, seen_si = 0, seen_rsi = 0;
  for (;;) {
    uint16_t pid, plen;
    if (rd_u16(c, &pid) || rd_u16(c, &plen)) return -1;
    if (pid == 0x0001) return 0; /* PID_SENTINEL */
    if (c->pos + plen > c->len) return -1; /* reader.read_vec(length) */
    uint32_t value_off = dgram_base + (uint32_t)c->pos;
    if (pid == 0x0070 && !seen_kh) { seen_kh = 1; if (plen == 16) s->key_hash_off = value_off; }
    if (pid == 0x0071 && !seen_si) { seen_si = 1; s->status_info_off = value_off; s->si_seen = 1; s->si_len = plen; }
    if ((pid == 0x0083 || pid == 0x800f) && !seen_rsi) { seen_rsi = 1; s->rsi_off = value_off; }
    c->pos += plen;
  }
}

/* Data::deserialize_data (data.rs:57-144).  body = submessage content. */
static int data_deserialize(cursor* c, uint32_t dgram_base, uint8_t flags, submsg* s) {
  uint16_t extra_flags, otq;
  if (rd_u16(c, &extra_flags) || rd_u16(c, &otq)) return -1;
  if (rd_entity_id(c, s->reader_id) || rd_entity_id(c, s->writer_id)) return -1;
  if (rd_sn(c, &s->sn)) return -1;
  int expect_qos = (flags & 0x02) != 0;                    /* DATA_Flags::InlineQos */
  int expect_data = (flags & 0x04) != 0 || (flags & 0x08) != 0; /* Data || Key */
  if (otq < 16) return -1;                                  /* :86-91 */
  if (otq > 16) {                                           /* :95-116 */
    c->pos += (size_t)(otq - 16);
    if (c->pos > c->len) return -1;
  }
  uint32_t qos_start = (uint32_t)c->pos;
  if (expect_qos) {
    s->has_qos = 1;
    if (parameter_list_read(c, dgram_base, s)) return -1;
  }
  s->qos_len = (uint32_t)c->pos - qos_start;
  s->pl_off = dgram_base + (uint32_t)c->pos;
  s->pl_len = (uint32_t)(c->len - c->pos);
  s->has_payload = expect_data;                             /* :131-135 split_off(cursor) */
  return 0;
}

/* DataFrag::deserialize (data_frag.rs:121-257) and total_number_of_fragments (:97-119). */
static int datafrag_deserialize(cursor* c, uint32_t dgram_base, uint8_t flags, submsg* s) {
  uint16_t extra_flags, otq, frags_in_sub, frag_size;
  uint32_t frag_start, data_size;
  if (rd_u16(c, &extra_flags) || rd_u16(c, &otq)) return -1;
  if (rd_entity_id(c, s->reader_id) || rd_entity_id(c, s->writer_id)) return -1;
  if (rd_sn(c, &s->sn)) return -1;
  if (rd_u32(c, &frag_start) || rd_u16(c, &frags_in_sub) || rd_u16(c, &frag_size) || rd_u32(c, &data_size))
    return -1;
  int expect_qos = (flags & 0x02) != 0; /* DATAFRAG_Flags::InlineQos */
  if (otq < 28) return -1;
  if (otq > 28) {
    c->pos += (size_t)(otq - 28);
    if (c->pos > c->len) return -1;
  }
  uint32_t qos_start = (uint32_t)c->pos;
  if (expect_qos) {
    s->has_qos = 1;
    if (parameter_list_read(c, dgram_base, s)) return -1;
  }
  s->qos_len = (uint32_t)c->pos - qos_start;
  if (s->sn < 1) return -1;                                         /* :202-207 */
  if (frag_size < 1 || (uint32_t)frag_size > data_size) return -1;  /* :215-224 */
  s->pl_off = dgram_base + (uint32_t)c->pos;
  s->pl_len = (uint32_t)(c->len - c->pos);
  s->has_payload = 1;
  uint32_t total = data_size / frag_size + ((data_size % frag_size) > 0 ? 1u : 0u);
  if (frag_start < 1 || frag_start > total) return -1;              /* :244-254 */
  s->frag_start = frag_start;
  s->frags_in_sub = frags_in_sub;
  s->frag_size = frag_size;
  s->data_size = data_size;
  return 0;
}

/* NumberSet<N>::read_from (sequence_number.rs:464-498); base already read by caller. */
static int number_set_tail(cursor* c, uint32_t dgram_base, submsg* s) {
  uint32_t num_bits;
  if (rd_u32(c, &num_bits)) return -1;
  if (num_bits > 256) return -1;
  uint32_t words = (num_bits + 31u) / 32u;
  s->num_bits = num_bits;
  s->bitmap_off = dgram_base + (uint32_t)c->pos;
  for (uint32_t i = 0; i < words; ++i) {
    uint32_t wv;
    if (rd_u32(c, &wv)) return -1;
  }
  return 0;
}

/* Submessage::read_from_buffer (rtps/submessage.rs:56-295).
 * Returns 1 = materialised submessage, 0 = skipped (PAD / unknown), -1 = error.
 * `rem` = remaining bytes of the message starting at `m + off`. */
static int submessage_read_from_buffer(const uint8_t* m, uint32_t off, uint32_t rem,
                                       submsg* s, uint32_t* consumed) {
  /* SubmessageHeader::read_from (submessage_header.rs:14-35), minimum 4 bytes */
  if (rem < 4) return -1;
  uint8_t kind = m[off], flags = m[off + 1];
  int le = (flags & 0x01) != 0;
  uint16_t content_length = le ? (uint16_t)(m[off + 2] | (m[off + 3] << 8))
                               : (uint16_t)((m[off + 2] << 8) | m[off + 3]);
  uint32_t proposed;
  if (content_length == 0) {
    proposed = (kind == RTPS_PAD || kind == RTPS_INFO_TS) ? 0u : rem - 4u; /* :61-78 */
  } else {
    proposed = content_length;
  }
  if (4u + proposed > rem) return -1; /* :80-91 */
  *consumed = 4u + proposed;

  memset(s, 0, sizeof *s);
  s->off = off;
  s->kind = kind;
  s->flags = flags;
  s->content_len = proposed;
  cursor c = {m + off + 4, proposed, 0, le};
  uint32_t base = off + 4; /* datagram offset of body[0] */

  switch (kind) {
    case RTPS_DATA:
      s->cls = BODY_WRITER;
      return data_deserialize(&c, base, (uint8_t)(flags & 0x1f), s) ? -1 : 1;
    case RTPS_DATA_FRAG:
      s->cls = BODY_WRITER;
      return datafrag_deserialize(&c, base, (uint8_t)(flags & 0x0f), s) ? -1 : 1;
    case RTPS_GAP: /* Gap (gap.rs:23-46) */
      s->cls = BODY_WRITER;
      if (rd_entity_id(&c, s->reader_id) || rd_entity_id(&c, s->writer_id) || rd_sn(&c, &s->sn) ||
          rd_sn(&c, &s->sn2) || number_set_tail(&c, base, s))
        return -1;
      return 1;
    case RTPS_ACKNACK: /* AckNack (ack_nack.rs:27-50) */
      s->cls = BODY_READER;
      if (rd_entity_id(&c, s->reader_id) || rd_entity_id(&c, s->writer_id) || rd_sn(&c, &s->sn) ||
          number_set_tail(&c, base, s))
        return -1;
      if (rd_u32(&c, (uint32_t*)&s->count)) return -1;
      return 1;
    case RTPS_NACK_FRAG: /* NackFrag (nack_frag.rs:31-53): FragmentNumberSet base is u32 */
      s->cls = BODY_READER;
      if (rd_entity_id(&c, s->reader_id) || rd_entity_id(&c, s->writer_id) || rd_sn(&c, &s->sn) ||
          rd_u32(&c, &s->u32a) || number_set_tail(&c, base, s))
        return -1;
      if (rd_u32(&c, (uint32_t*)&s->count)) return -1;
      return 1;
    case RTPS_HEARTBEAT: /* Heartbeat (heartbeat.rs:21-49) */
      s->cls = BODY_WRITER;
      if (rd_entity_id(&c, s->reader_id) || rd_entity_id(&c, s->writer_id) || rd_sn(&c, &s->sn) ||
          rd_sn(&c, &s->sn2) || rd_u32(&c, (uint32_t*)&s->count))
        return -1;
      return 1;
    case RTPS_HEARTBEAT_FRAG: /* HeartbeatFrag (heartbeat_frag.rs:16-37) */
      s->cls = BODY_WRITER;
      if (rd_entity_id(&c, s->reader_id) || rd_entity_id(&c, s->writer_id) || rd_sn(&c, &s->sn) ||
          rd_u32(&c, &s->u32a) || rd_u32(&c, (uint32_t*)&s->count))
        return -1;
      return 1;
    case RTPS_INFO_DST: /* InfoDestination (info_destination.rs:20-25) */
      s->cls = BODY_INTERP;
      return rd_bytes(&c, s->prefix, 12) ? -1 : 1;
    case RTPS_INFO_SRC: { /* InfoSource (info_source.rs:22-36) */
      uint32_t unused;
      s->cls = BODY_INTERP;
      if (rd_u32(&c, &unused) || rd_bytes(&c, s->version, 2) || rd_bytes(&c, s->vendor, 2) ||
          rd_bytes(&c, s->prefix, 12))
        return -1;
      return 1;
    }
    case RTPS_INFO_TS: /* rtps/submessage.rs:211-225; Timestamp (structure/time.rs:37-56) */
      s->cls = BODY_INTERP;
      if (flags & 0x02) { s->ts_valid = 0; return 1; } /* Invalidate */
      if (rd_u32(&c, &s->ts_sec) || rd_u32(&c, &s->ts_frac)) return -1;
      s->ts_valid = 1;
      return 1;
    case RTPS_INFO_REPLY: { /* InfoReply (info_reply.rs:9-21): speedy Vec<Locator> + Option<Vec<Locator>> */
      uint32_t n1, n2 = 0xffffffffu;
      uint8_t tag;
      s->cls = BODY_INTERP;
      if (rd_u32(&c, &n1)) return -1;
      if ((uint64_t)n1 * 24u > (uint64_t)(c.len - c.pos)) return -1; /* Locator = i32 + u32 + 16 B */
      c.pos += (size_t)n1 * 24u;
      if (rd_u8(&c, &tag)) return -1;
      if (tag != 0) { /* parity unpinned: speedy Option tag (non-zero -> Some) */
        if (rd_u32(&c, &n2)) return -1;
        if ((uint64_t)n2 * 24u > (uint64_t)(c.len - c.pos)) return -1;
        c.pos += (size_t)n2 * 24u;
      }
      s->n_uni = n1;
      s->n_multi = n2;
      return 1;
    }
    case RTPS_PAD:
    default:
      /* PAD (:233-235); INFO_REPLY_IP4, SEC_* without `security`, vendor kinds (:278-293) */
      return 0;
  }
}

/* ------------------------------------------------------------------------ */
/* classification                                                            */
/* ------------------------------------------------------------------------ */
static const uint8_t E_UNKNOWN[4] = {0, 0, 0, 0};
static const uint8_t E_SEDP_PUB_W[4] = {0, 0, 3, 0xc2}, E_SEDP_PUB_R[4] = {0, 0, 3, 0xc7};
static const uint8_t E_SEDP_TOP_W[4] = {0, 0, 2, 0xc2}, E_SEDP_TOP_R[4] = {0, 0, 2, 0xc7};
static const uint8_t E_SEDP_SUB_W[4] = {0, 0, 4, 0xc2}, E_SEDP_SUB_R[4] = {0, 0, 4, 0xc7};
static const uint8_t E_SPDP_W[4] = {0, 1, 0, 0xc2}, E_SPDP_R[4] = {0, 1, 0, 0xc7};
static const uint8_t E_P2P_W[4] = {0, 2, 0, 0xc2}, E_P2P_R[4] = {0, 2, 0, 0xc7};

static int eid_eq(const uint8_t a[4], const uint8_t b[4]) { return memcmp(a, b, 4) == 0; }

/* Discovery2::handle_writer_msg pair test (io_uring/discovery/discovery.rs:2795-2816),
 * (receiver, sender) = (reader_id, writer_id) for writer submessages. */
static int builtin_writer_pair(const uint8_t rid[4], const uint8_t wid[4]) {
  if (eid_eq(rid, E_UNKNOWN))
    return eid_eq(wid, E_SEDP_PUB_W) || eid_eq(wid, E_SEDP_TOP_W) || eid_eq(wid, E_SPDP_W) ||
           eid_eq(wid, E_SEDP_SUB_W) || eid_eq(wid, E_P2P_W);
  return (eid_eq(rid, E_SEDP_PUB_R) && eid_eq(wid, E_SEDP_PUB_W)) ||
         (eid_eq(rid, E_SEDP_TOP_R) && eid_eq(wid, E_SEDP_TOP_W)) ||
         (eid_eq(rid, E_SEDP_SUB_R) && eid_eq(wid, E_SEDP_SUB_W));
}
/* Discovery2::handle_reader_submsg pair test (discovery.rs:3075-3095),
 * (receiver, sender) = (writer_id, reader_id) for ACKNACK / NACK_FRAG. */
static int builtin_reader_pair(const uint8_t rid[4], const uint8_t wid[4]) {
  return (eid_eq(wid, E_SEDP_PUB_W) && eid_eq(rid, E_SEDP_PUB_R)) ||
         (eid_eq(wid, E_SEDP_TOP_W) && eid_eq(rid, E_SEDP_TOP_R)) ||
         (eid_eq(wid, E_SEDP_SUB_W) && eid_eq(rid, E_SEDP_SUB_R)) ||
         (eid_eq(wid, E_SPDP_W) && eid_eq(rid, E_SPDP_R)) ||
         (eid_eq(wid, E_P2P_W) && eid_eq(rid, E_P2P_R));
}

/* The local readers: MessageReceiver::available_readers, a BTreeMap<EntityId,
 * Reader> (io_uring/rtps/message_receiver.rs:129), so iteration is in EntityId
 * byte order (EntityId derives Ord over {entity_key, entity_kind}, structure/guid.rs:208-216).
 * Each reader's matched_writers are the proxies naming it. */
typedef struct ox_proxy { uint32_t reader; uint8_t guid[16]; uint32_t index; } ox_proxy;
typedef struct ox_eid { uint8_t eid[4]; uint32_t order; uint32_t reader; } ox_eid;
typedef struct oracle_readers {
  const rtps_reader* r;
  uint32_t nr;
  const rtps_proxy* p;
  uint32_t np;
  uint32_t* order;  /* reader indices in EntityId order */
  /* lookup structures (the same relation, indexed so that a 1M-datagram batch with
   * hundreds of readers and proxies stays fast; oracle_targets gives their meaning) */
  ox_eid* eids;     /* (matched writer entity id, reader) of non-stateless readers, by (eid, EntityId order) */
  uint32_t n_eids;
  ox_proxy* px;     /* proxies by (reader, GUID) */
} oracle_readers;

static const oracle_readers* g_sort_ctx;
static int reader_cmp(const void* a, const void* b) {
  return memcmp(g_sort_ctx->r[*(const uint32_t*)a].entity_id, g_sort_ctx->r[*(const uint32_t*)b].entity_id, 4);
}
static int eid_cmp(const void* a, const void* b) {
  const ox_eid *x = (const ox_eid*)a, *y = (const ox_eid*)b;
  int c = memcmp(x->eid, y->eid, 4);
  return c ? c : (x->order > y->order) - (x->order < y->order);
}
static int px_cmp(const void* a, const void* b) {
  const ox_proxy *x = (const ox_proxy*)a, *y = (const ox_proxy*)b;
  if (x->reader != y->reader) return x->reader < y->reader ? -1 : 1;
  return memcmp(x->guid, y->guid, 16);
}
static void oracle_readers_init(oracle_readers* R, const rtps_reader* r, uint32_t nr, const rtps_proxy* p, uint32_t np) {
  R->r = r; R->nr = nr; R->p = p; R->np = np;
  R->order = (uint32_t*)malloc(sizeof(uint32_t) * (nr ? nr : 1));
  for (uint32_t i = 0; i < nr; ++i) R->order[i] = i;
  g_sort_ctx = R;  /* single-threaded setup */
  qsort(R->order, nr, sizeof(uint32_t), reader_cmp);
  uint32_t* rank = (uint32_t*)malloc(sizeof(uint32_t) * (nr ? nr : 1));
  for (uint32_t k = 0; k < nr; ++k) rank[R->order[k]] = k;
  R->eids = (ox_eid*)malloc(sizeof(ox_eid) * (np ? np : 1));
  R->px = (ox_proxy*)malloc(sizeof(ox_proxy) * (np ? np : 1));
  uint32_t ne = 0;
  for (uint32_t k = 0; k < np; ++k) {
    R->px[k].reader = p[k].reader;
    memcpy(R->px[k].guid, p[k].writer_guid, 16);
    R->px[k].index = k;
    if (p[k].reader >= nr || (r[p[k].reader].flags & RTPS_READER_STATELESS)) continue;
    memcpy(R->eids[ne].eid, p[k].writer_guid + 12, 4);
    R->eids[ne].order = rank[p[k].reader];
    R->eids[ne].reader = p[k].reader;
    ne++;
  }
  qsort(R->px, np, sizeof(ox_proxy), px_cmp);
  qsort(R->eids, ne, sizeof(ox_eid), eid_cmp);
  uint32_t w = 0;  /* one entry per (eid, reader) */
  for (uint32_t k = 0; k < ne; ++k)
    if (!w || memcmp(R->eids[w - 1].eid, R->eids[k].eid, 4) || R->eids[w - 1].reader != R->eids[k].reader)
      R->eids[w++] = R->eids[k];
  R->n_eids = w;
  free(rank);
}
static void oracle_readers_free(oracle_readers* R) { free(R->order); free(R->eids); free(R->px); }

/* matched_writers.get(&writer_guid) (reader.rs:712-739): the proxy index or RTPS_NO_PROXY */
static uint32_t matched_writer(const oracle_readers* R, uint32_t reader, const uint8_t prefix[12],
                               const uint8_t wid[4]) {
  ox_proxy key;
  key.reader = reader;
  memcpy(key.guid, prefix, 12);
  memcpy(key.guid + 12, wid, 4);
  const ox_proxy* f = (const ox_proxy*)bsearch(&key, R->px, R->np, sizeof(ox_proxy), px_cmp);
  return f ? f->index : RTPS_NO_PROXY;
}
static const uint8_t E_SPDP_R_ID[4] = {0x00, 0x01, 0x00, 0xc7};
/* The target readers of a writer submessage that is not a builtin pair
 * (Domain::handle_event, io_uring/rtps/dp_event_loop.rs:266-327):
 *   available_readers.values_mut().filter(|r| r.contains_writer(writer_entity_id))
 * i.e. in EntityId order, every reader that is not stateless and has a matched
 * writer with this ENTITY ID (Reader::contains_writer, reader.rs:474-484), each
 * with its proxy of the full writer GUID.  Writes up to cap targets into out
 * (may be NULL), returns the count; *matched = some target has a proxy. */
static uint32_t oracle_targets(const oracle_readers* R, const uint8_t prefix[12], const uint8_t wid[4],
                               rtps_target* out, uint32_t cap, int* matched) {
  *matched = 0;
  /* first (eid, *) entry: lower bound on eid */
  uint32_t lo = 0, hi = R->n_eids;
  while (lo < hi) {
    const uint32_t m = (lo + hi) / 2;
    if (memcmp(R->eids[m].eid, wid, 4) < 0) lo = m + 1; else hi = m;
  }
  uint32_t n = 0;
  for (uint32_t k = lo; k < R->n_eids && memcmp(R->eids[k].eid, wid, 4) == 0; ++k) {
    const uint32_t r = R->eids[k].reader;
    const uint32_t proxy = matched_writer(R, r, prefix, wid);
    if (proxy != RTPS_NO_PROXY) *matched = 1;
    if (out && n < cap) {
      out[n].reader_slot = R->r[r].reader_slot;
      out[n].reader_flags = (uint16_t)(R->r[r].flags |
                                       (memcmp(R->r[r].entity_id, E_SPDP_R_ID, 4) == 0 ? RTPS_TARGET_DUPLICATES_OK : 0));
      out[n].proxy = proxy;
    }
    n++;
  }
  return n;
}

/* Reader::data_to_dds_data (io_uring/rtps/reader.rs:760-833) +
 * SerializedPayload::from_bytes (serialized_payload.rs:86-110). */
static uint8_t data_to_dds_data_kind(const submsg* s) {
  int d = (s->flags & 0x04) != 0, k = (s->flags & 0x08) != 0;
  if (s->has_payload) {
    if (d && k) return RTPS_PK_ERR_AMBIGUOUS;
    if (s->pl_len < 4) return RTPS_PK_ERR_SHORT;
    return d ? RTPS_PK_DATA : RTPS_PK_KEY;
  }
  /* (None, false, false): needs a 16-byte KEY_HASH in the inline QoS */
  return s->key_hash_off ? RTPS_PK_KEY_HASH : RTPS_PK_ERR_NO_CONTENT;
}

/* Reader::deduce_change_kind (reader.rs:1158-1182) for the payload kinds that call it:
 * key (:779-785) and key hash (:787-813); Data is Alive (ddsdata.rs:45-50).
 * inline_qos None -> NotAliveDisposed.  InlineQos::status_info (inline_qos.rs:27-42):
 * the first PID_STATUS_INFO, or StatusInfo::empty() (Alive) if there is none;
 * StatusInfo::read_from reads four u8 (em[3], flags: :139-147), so a value shorter
 * than 4 bytes is an error -> NotAliveDisposed, and the byte order (rep id from the
 * E flag, submessage_flag.rs:25-31) never matters.  StatusInfo::change_kind
 * (:164-175): Disposed (0x1) first, then Unregistered (0x2), else Alive. */
static uint8_t deduce_change_kind(uint8_t pk, const submsg* s, const uint8_t* m) {
  if (pk == RTPS_PK_DATA) return RTPS_CK_ALIVE;
  if (pk != RTPS_PK_KEY && pk != RTPS_PK_KEY_HASH) return RTPS_CK_NONE;
  if (!s->has_qos) return RTPS_CK_NOT_ALIVE_DISPOSED;
  if (!s->si_seen) return RTPS_CK_ALIVE;
  if (s->si_len < 4) return RTPS_CK_NOT_ALIVE_DISPOSED;
  const uint8_t f = m[s->status_info_off + 3];
  if (f & 0x1) return RTPS_CK_NOT_ALIVE_DISPOSED;
  if (f & 0x2) return RTPS_CK_NOT_ALIVE_UNREGISTERED;
  return RTPS_CK_ALIVE;
}

/* ------------------------------------------------------------------------ */
/* one datagram: handle_received_packet_2 + Message::read_from_buffer +      */
/* the SubmessageIter2 interpreter                                            */
/* ------------------------------------------------------------------------ */
typedef struct oracle_cfg {
  uint8_t own[12];
  const oracle_readers* readers;
} oracle_cfg;

#define MAX_SUBMSGS (RTPS_MAX_DATAGRAM / 4)

/* returns status; writes up to cap records into recs (count in *n_out) */
static uint8_t oracle_datagram(const oracle_cfg* cfg, const uint8_t* m, uint32_t L, uint32_t dgram_idx,
                               submsg* subs /* scratch [MAX_SUBMSGS] */, rtps_record* recs,
                               uint32_t* n_out) {
  *n_out = 0;
  if (L > RTPS_MAX_DATAGRAM) return RTPS_DGRAM_TOO_LONG;
  /* message_receiver.rs:238-251 */
  if (L < 20) {
    if (L >= 16 && memcmp(m, "RTPS", 4) == 0 && memcmp(m + 9, "DDSPING", 7) == 0) return RTPS_DGRAM_PING;
    return RTPS_DGRAM_SHORT;
  }
  /* :254-271 */
  if (memcmp(m, "RTPS", 4) != 0) return memcmp(m, "RTPX", 4) == 0 ? RTPS_DGRAM_RTPX : RTPS_DGRAM_BAD_MAGIC;
  /* Header::valid (messages/header.rs:30-39): protocol id checked above, major <= 2 */
  if (m[4] > 2) return RTPS_DGRAM_BAD_HEADER;
  /* Message::read_from_buffer submessage loop (rtps/message.rs:74-78) */
  uint32_t nsub = 0, off = 20;
  while (off < L) {
    uint32_t used = 0;
    int r = submessage_read_from_buffer(m, off, L - off, &subs[nsub], &used);
    if (r < 0) return RTPS_DGRAM_SUBMSG_ERR;
    if (r > 0) nsub++;
    off += used;
  }
  /* handle_parsed_message_2 (:289-295): reset(), dest := own, src := header prefix */
  uint8_t src[12], dest[12];
  static const uint8_t zero12[12] = {0};
  memcpy(src, m + 8, 12);
  memcpy(dest, cfg->own, 12);
  int ts_valid = 0;
  uint32_t ts_sec = 0, ts_frac = 0;
  for (uint32_t i = 0; i < nsub; ++i) {
    const submsg* s = &subs[i];
    rtps_record* rec = &recs[i];
    memset(rec, 0, sizeof *rec);
    rec->dgram_idx = dgram_idx;
    rec->sub_off = (uint16_t)s->off;
    rec->kind = s->kind;
    rec->flags = s->flags;
    if (s->cls == BODY_INTERP) {
      /* handle_interpreter_submessage (message_receiver.rs:618-665) */
      switch (s->kind) {
        case RTPS_INFO_TS:
          ts_valid = s->ts_valid; ts_sec = s->ts_valid ? s->ts_sec : 0; ts_frac = s->ts_valid ? s->ts_frac : 0;
          memcpy(rec->prefix, src, 12);
          break;
        case RTPS_INFO_SRC:
          memcpy(src, s->prefix, 12);
          ts_valid = 0; ts_sec = 0; ts_frac = 0;
          memcpy(rec->prefix, s->prefix, 12);
          memcpy(rec->u.infosrc.version, s->version, 2);
          memcpy(rec->u.infosrc.vendor, s->vendor, 2);
          break;
        case RTPS_INFO_DST:
          if (memcmp(s->prefix, zero12, 12) == 0) memcpy(dest, cfg->own, 12);
          else memcpy(dest, s->prefix, 12);
          memcpy(rec->prefix, s->prefix, 12);
          break;
        case RTPS_INFO_REPLY:
          memcpy(rec->prefix, src, 12);
          rec->u.inforeply.n_unicast = s->n_uni;
          rec->u.inforeply.n_multicast = s->n_multi;
          break;
      }
      rec->aux16 = (uint16_t)s->content_len;
    } else {
      memcpy(rec->prefix, src, 12);
      memcpy(rec->writer_id, s->writer_id, 4);
      memcpy(rec->reader_id, s->reader_id, 4);
      rec->sn = s->sn;
      if (s->cls == BODY_WRITER) {
        /* SubmessageIter2::next writer filter (message_receiver.rs:75-84) */
        int pass = memcmp(dest, cfg->own, 12) == 0 || memcmp(dest, zero12, 12) == 0;
        if (pass) rec->route |= RTPS_ROUTE_PASS;
        if (builtin_writer_pair(s->reader_id, s->writer_id)) rec->route |= RTPS_ROUTE_BUILTIN;
        else {
          int matched = 0;
          if (oracle_targets(cfg->readers, src, s->writer_id, NULL, 0, &matched))
            rec->route |= RTPS_ROUTE_TARGETED | (matched ? RTPS_ROUTE_MATCHED : 0);
        }
      } else {
        rec->route |= RTPS_ROUTE_PASS; /* reader submessages always pass (:88-113) */
        if (builtin_reader_pair(s->reader_id, s->writer_id)) rec->route |= RTPS_ROUTE_BUILTIN;
      }
      switch (s->kind) {
        case RTPS_DATA:
          rec->aux16 = (uint16_t)s->qos_len;
          if (s->has_qos) rec->route |= RTPS_ROUTE_HAS_QOS;
          if (s->has_payload) rec->route |= RTPS_ROUTE_HAS_PAYLOAD;
          rec->u.data.pl_off = (uint16_t)s->pl_off;
          rec->u.data.pl_len = (uint16_t)s->pl_len;
          rec->payload_kind = data_to_dds_data_kind(s);
          if (rec->payload_kind == RTPS_PK_DATA || rec->payload_kind == RTPS_PK_KEY) {
            memcpy(rec->u.data.rep_id, m + s->pl_off, 2);
            memcpy(rec->u.data.rep_opts, m + s->pl_off + 2, 2);
          }
          rec->u.data.key_hash_off = (uint16_t)s->key_hash_off;
          rec->u.data.status_info_off = (uint16_t)s->status_info_off;
          rec->u.data.rsi_off = (uint16_t)s->rsi_off;
          rec->u.data.change_kind = deduce_change_kind(rec->payload_kind, s, m);
          break;
        case RTPS_DATA_FRAG:
          rec->aux16 = (uint16_t)s->qos_len;
          if (s->has_qos) rec->route |= RTPS_ROUTE_HAS_QOS;
          rec->route |= RTPS_ROUTE_HAS_PAYLOAD;
          rec->u.frag.pl_off = (uint16_t)s->pl_off;
          rec->u.frag.pl_len = (uint16_t)s->pl_len;
          rec->u.frag.frag_start = s->frag_start;
          rec->u.frag.frags_in_sub = (uint16_t)s->frags_in_sub;
          rec->u.frag.frag_size = (uint16_t)s->frag_size;
          rec->u.frag.data_size = s->data_size;
          break;
        case RTPS_HEARTBEAT:
          rec->aux16 = (uint16_t)s->content_len;
          rec->u.hb.last_sn = s->sn2;
          rec->u.hb.count = s->count;
          break;
        case RTPS_HEARTBEAT_FRAG:
          rec->aux16 = (uint16_t)s->content_len;
          rec->u.hbfrag.last_frag_num = s->u32a;
          rec->u.hbfrag.count = s->count;
          break;
        case RTPS_GAP:
          rec->aux16 = (uint16_t)s->content_len;
          rec->u.gap.list_base = s->sn2;
          rec->u.gap.num_bits = s->num_bits;
          rec->u.gap.bitmap_off = (uint16_t)s->bitmap_off;
          break;
        case RTPS_ACKNACK:
          rec->aux16 = (uint16_t)s->content_len;
          rec->u.acknack.count = s->count;
          rec->u.acknack.num_bits = s->num_bits;
          rec->u.acknack.bitmap_off = (uint16_t)s->bitmap_off;
          break;
        case RTPS_NACK_FRAG:
          rec->aux16 = (uint16_t)s->content_len;
          rec->u.nackfrag.fns_base = s->u32a;
          rec->u.nackfrag.count = s->count;
          rec->u.nackfrag.num_bits = s->num_bits;
          rec->u.nackfrag.bitmap_off = (uint16_t)s->bitmap_off;
          break;
      }
    }
    if (ts_valid) {
      rec->route |= RTPS_ROUTE_TS_VALID;
      rec->ts_sec = ts_sec;
      rec->ts_frac = ts_frac;
    }
  }
  *n_out = nsub;
  return RTPS_DGRAM_OK;
}

/* ------------------------------------------------------------------------ */
/* batch entry points (ctypes)                                               */
/* ------------------------------------------------------------------------ */
typedef struct slice_job {
  const oracle_cfg* cfg;
  const uint8_t* arena;
  const uint64_t* off;
  const uint32_t* len;
  uint32_t lo, hi;
  uint8_t* status;
  rtps_record* recs; /* thread-local */
  uint32_t* counts;  /* per datagram */
  uint64_t n_recs, cap;
  submsg* scratch;
} slice_job;

static void* run_slice(void* arg) {
  slice_job* j = (slice_job*)arg;
  j->n_recs = 0;
  for (uint32_t i = j->lo; i < j->hi; ++i) {
    uint32_t L = j->len[i];
    uint32_t nr = 0;
    uint64_t need = (L >= 20 && L <= RTPS_MAX_DATAGRAM) ? (uint64_t)(L - 20) / 4u : 0u;
    if (j->n_recs + need > j->cap) { /* grow thread-local buffers */
      uint64_t ncap = (j->cap + need) * 2 + 64;
      j->recs = (rtps_record*)realloc(j->recs, ncap * sizeof(rtps_record));
      j->cap = ncap;
    }
    j->status[i] = oracle_datagram(j->cfg, j->arena + j->off[i], L, i, j->scratch, j->recs + j->n_recs, &nr);
    j->counts[i] = nr;
    j->n_recs += nr;
  }
  return 0;
}

/* Parse a batch on `threads` host threads (contiguous slices).  Outputs are
 * identical to the device library's: status[n], records (ascending
 * (dgram_idx, sub_off)), rec_begin[n] (optional), total count; readers /
 * proxies as given to rtps_rx_set_readers.  Returns the total number of
 * records (records beyond max_records are not written). */
uint64_t rtps_oracle_parse(const uint8_t* arena, const uint64_t* off, const uint32_t* len, uint32_t n,
                           const uint8_t own[12], const rtps_reader* readers, uint32_t n_readers,
                           const rtps_proxy* proxies, uint32_t n_proxies,
                           uint8_t* status, rtps_record* records, uint64_t max_records,
                           uint32_t* rec_begin, int threads) {
  oracle_cfg cfg;
  oracle_readers R;
  oracle_readers_init(&R, readers, n_readers, proxies, n_proxies);
  memcpy(cfg.own, own, 12);
  cfg.readers = &R;
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > n && n > 0) threads = (int)n;
  uint32_t* counts = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  slice_job* jobs = (slice_job*)calloc((size_t)threads, sizeof(slice_job));
  pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].cfg = &cfg;
    jobs[t].arena = arena;
    jobs[t].off = off;
    jobs[t].len = len;
    jobs[t].lo = (uint32_t)((uint64_t)n * t / threads);
    jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
    jobs[t].status = status;
    jobs[t].counts = counts;
    jobs[t].scratch = (submsg*)malloc(sizeof(submsg) * MAX_SUBMSGS);
    if (threads > 1) pthread_create(&tids[t], 0, run_slice, &jobs[t]);
  }
  if (threads == 1) run_slice(&jobs[0]);
  else for (int t = 0; t < threads; ++t) pthread_join(tids[t], 0);
  uint64_t total = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t k = jobs[t].n_recs;
    if (records && total < max_records) {
      uint64_t w = (total + k <= max_records) ? k : max_records - total;
      memcpy(records + total, jobs[t].recs, w * sizeof(rtps_record));
    }
    total += k;
    free(jobs[t].recs);
    free(jobs[t].scratch);
  }
  if (rec_begin) {
    uint64_t acc = 0;
    for (uint32_t i = 0; i < n; ++i) { rec_begin[i] = (uint32_t)acc; acc += counts[i]; }
  }
  free(counts);
  free(jobs);
  free(tids);
  oracle_readers_free(&R);
  return total;
}

/* The target readers of every record (the user path of Domain::handle_event,
 * see oracle_targets): for record i, out[off[i] .. off[i+1]).  Only writer
 * kinds that are not a builtin pair have targets.  off: [m + 1].  Returns the
 * total (targets past cap are counted, not written). */
uint64_t rtps_oracle_targets(const rtps_record* recs, uint64_t m, const rtps_reader* readers, uint32_t n_readers,
                             const rtps_proxy* proxies, uint32_t n_proxies, uint64_t* off, rtps_target* out,
                             uint64_t cap) {
  oracle_readers R;
  oracle_readers_init(&R, readers, n_readers, proxies, n_proxies);
  uint64_t total = 0;
  rtps_target* tmp = (rtps_target*)malloc(sizeof(rtps_target) * (n_readers ? n_readers : 1));
  for (uint64_t i = 0; i < m; ++i) {
    off[i] = total;
    const rtps_record* r = &recs[i];
    const int writer_kind = r->kind == RTPS_DATA || r->kind == RTPS_DATA_FRAG || r->kind == RTPS_HEARTBEAT ||
                            r->kind == RTPS_HEARTBEAT_FRAG || r->kind == RTPS_GAP;
    if (!writer_kind || builtin_writer_pair(r->reader_id, r->writer_id)) continue;
    int matched = 0;
    const uint32_t k = oracle_targets(&R, r->prefix, r->writer_id, tmp, n_readers, &matched);
    for (uint32_t j = 0; j < k; ++j, ++total)
      if (total < cap) out[total] = tmp[j];
  }
  off[m] = total;
  free(tmp);
  oracle_readers_free(&R);
  return total;
}

/* Host-side synthetic generator (same f(seed, idx) as the device kernel). */
uint64_t rtps_oracle_gen_layout(int wl, uint64_t seed, uint64_t first_idx, uint32_t n_writers, uint32_t n,
                                uint64_t* off, uint32_t* len) {
  return rtps_gen_layout_host(wl, seed, first_idx, n_writers, n, off, len);
}
void rtps_oracle_gen_fill(int wl, uint64_t seed, uint64_t first_idx, uint32_t n_writers, uint32_t n,
                          const uint64_t* off, uint8_t* arena) {
  for (uint32_t i = 0; i < n; ++i) rtps_gen_datagram(wl, seed, first_idx + i, n_writers, arena + off[i]);
}
uint32_t rtps_oracle_record_size(void) { return (uint32_t)sizeof(rtps_record); }

/* ------------------------------------------------------------------------ */
/* CDR primitive decode (a18)                                                */
/*   deserialize_from_cdr_with_decoder_and_rep_id  serialization/cdr_adapters.rs:246-275 */
/*   CDRDeserializerAdapter::supported_encodings    cdr_adapters.rs:96-100     */
/*   -> external crate cdr-encoding 0.10 (not vendored): its published         */
/*      CdrDeserializer rules are restated here: classic CDR, every primitive  */
/*      aligned to its size relative to the first byte of the value (after the */
/*      4-byte encapsulation), padding skipped only when an element is read,   */
/*      string = u32 length incl. NUL + bytes (last byte dropped, contents     */
/*      must be UTF-8: str::from_utf8), bool byte must be 0 or 1, sequence =   */
/*      u32 count + elements, arrays have no length.  Parity pinned by the     */
/*      ShapeType "RED" vector (rtps/message_receiver.rs:1250-1254); the rest  */
/*      is "parity unpinned".                                                   */
/* ------------------------------------------------------------------------ */
typedef struct cdr_cur { const uint8_t* v; uint32_t len, pos; int le; } cdr_cur;

static uint32_t cdr_pad(uint32_t pos, uint32_t a) { return (a - (pos % a)) % a; }
static uint64_t cdr_get(const cdr_cur* c, uint32_t at, uint32_t size) {
  uint64_t x = 0;
  for (uint32_t k = 0; k < size; ++k) {
    uint64_t b = c->v[at + k];
    x |= c->le ? (b << (8 * k)) : (b << (8 * (size - 1 - k)));
  }
  return x;
}
/* std::str::from_utf8 acceptance */
static int utf8_ok(const uint8_t* s, uint32_t m) {
  uint32_t i = 0;
  while (i < m) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t need;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
    else return 0;
    if (i + need >= m) return 0; /* needs bytes i+1 .. i+need < m */
    if (s[i + 1] < lo || s[i + 1] > hi) return 0;
    for (uint32_t k = 2; k <= need; ++k) if (s[i + k] < 0x80 || s[i + k] > 0xBF) return 0;
    i += need + 1;
  }
  return 1;
}

static void cdr_store(uint8_t* row, uint32_t off, uint64_t x, uint32_t size) {
  for (uint32_t k = 0; k < size; ++k) row[off + k] = (uint8_t)(x >> (8 * k)); /* host = little-endian */
}

/* Composite elements (RTPS_CDR_SEQ_BEGIN / ARRAY_BEGIN ... END): serde's Vec<T> /
 * [T; N] through cdr-encoding's deserialize_seq / deserialize_tuple: a u32 count
 * (aligned to 4; arrays have none), then each element's fields in order, with no
 * alignment of the element's own.  cdr_match: the END that closes the BEGIN at k. */
static uint32_t cdr_match(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t k) {
  uint32_t depth = 0;
  for (uint32_t j = k; j < n_ops; ++j) {
    if (prog[j].kind == RTPS_CDR_SEQ_BEGIN || prog[j].kind == RTPS_CDR_ARRAY_BEGIN) depth++;
    else if (prog[j].kind == RTPS_CDR_END && --depth == 0) return j;
  }
  return n_ops;
}
/* the fewest wire bytes ops [a, b) can consume (0: they read nothing, so they cannot fail) */
static uint64_t cdr_min_wire(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t a, uint32_t b) {
  uint64_t m = 0;
  for (uint32_t k = a; k < b; ++k) {
    const rtps_cdr_op* op = &prog[k];
    switch (op->kind) {
      case RTPS_CDR_PRIM: m += op->size; break;
      case RTPS_CDR_BOOL: m += 1; break;
      case RTPS_CDR_ARRAY: m += (uint64_t)op->size * op->count; break;
      case RTPS_CDR_STRING: case RTPS_CDR_SEQ: case RTPS_CDR_SEQ_BEGIN: m += 4; break;
      case RTPS_CDR_ARRAY_BEGIN: {
        uint32_t j = cdr_match(prog, n_ops, k);
        m += (uint64_t)op->count * cdr_min_wire(prog, n_ops, k + 1, j);
        break;
      }
      default: break;
    }
    if (op->kind == RTPS_CDR_SEQ_BEGIN || op->kind == RTPS_CDR_ARRAY_BEGIN) k = cdr_match(prog, n_ops, k);
  }
  return m;
}
typedef struct cdr_frame { uint32_t begin, n, i, elem0, base; int write; } cdr_frame;

static uint8_t cdr_decode_one(const rtps_cdr_op* prog, uint32_t n_ops, const uint8_t* value, uint32_t len, int le,
                              uint8_t* row) {
  cdr_cur c = {value, len, 0, le};
  cdr_frame fr[RTPS_CDR_MAX_DEPTH];
  uint32_t depth = 0, base = 0; /* base: row offset of the current element (0: the row) */
  int write = 1;                /* 0 inside elements past a sequence's slot (n > count) */
  for (uint32_t k = 0; k < n_ops; ++k) {
    const rtps_cdr_op* op = &prog[k];
    uint32_t size = op->size;
    uint8_t* dst = row + base; /* elements past the slot are read (and validated), not stored */
    switch (op->kind) {
      case RTPS_CDR_PRIM:
      case RTPS_CDR_ARRAY: {
        uint32_t cnt = op->kind == RTPS_CDR_PRIM ? 1u : op->count;
        if (cnt == 0) break;
        uint32_t pad = cdr_pad(c.pos, size);
        if ((uint64_t)c.pos + pad + (uint64_t)cnt * size > c.len) return RTPS_CDR_EOF;
        c.pos += pad;
        if (write)
          for (uint32_t e = 0; e < cnt; ++e) cdr_store(dst, op->out_off + e * size, cdr_get(&c, c.pos + e * size, size), size);
        c.pos += cnt * size;
        break;
      }
      case RTPS_CDR_BOOL: {
        if (c.pos + 1 > c.len) return RTPS_CDR_EOF;
        uint8_t b = c.v[c.pos];
        if (b > 1) return RTPS_CDR_BAD_BOOL;
        if (write) dst[op->out_off] = b;
        c.pos += 1;
        break;
      }
      case RTPS_CDR_STRING: {
        uint32_t pad = cdr_pad(c.pos, 4);
        if ((uint64_t)c.pos + pad + 4 > c.len) return RTPS_CDR_EOF;
        c.pos += pad;
        uint32_t l = (uint32_t)cdr_get(&c, c.pos, 4);
        c.pos += 4;
        if ((uint64_t)c.pos + l > c.len) return RTPS_CDR_EOF;
        uint32_t m = l ? l - 1 : 0;
        if (!utf8_ok(c.v + c.pos, m)) return RTPS_CDR_BAD_UTF8;
        if (m > op->count) return RTPS_CDR_TOO_LONG;
        if (write) {
          cdr_store(dst, op->out_off, m, 4);
          memcpy(dst + op->out_off + 4, c.v + c.pos, m);
        }
        c.pos += l;
        break;
      }
      case RTPS_CDR_SEQ: {
        uint32_t pad = cdr_pad(c.pos, 4);
        if ((uint64_t)c.pos + pad + 4 > c.len) return RTPS_CDR_EOF;
        c.pos += pad;
        uint32_t n = (uint32_t)cdr_get(&c, c.pos, 4);
        c.pos += 4;
        if (n) {
          uint32_t pe = cdr_pad(c.pos, size);
          if ((uint64_t)c.pos + pe + (uint64_t)n * size > c.len) return RTPS_CDR_EOF;
          if (n > op->count) return RTPS_CDR_TOO_LONG;
          c.pos += pe;
          for (uint32_t e = 0; write && e < n; ++e)
            cdr_store(dst, op->out_off + 4 + e * size, cdr_get(&c, c.pos + e * size, size), size);
          c.pos += n * size;
        }
        if (write) cdr_store(dst, op->out_off, n, 4);
        break;
      }
      case RTPS_CDR_SEQ_BEGIN:
      case RTPS_CDR_ARRAY_BEGIN: {
        const int seq = op->kind == RTPS_CDR_SEQ_BEGIN;
        uint32_t n = op->count;
        if (seq) {
          uint32_t pad = cdr_pad(c.pos, 4);
          if ((uint64_t)c.pos + pad + 4 > c.len) return RTPS_CDR_EOF;
          c.pos += pad;
          n = (uint32_t)cdr_get(&c, c.pos, 4);
          c.pos += 4;
          if (write) cdr_store(dst, op->out_off, n, 4);
        }
        const uint32_t j = cdr_match(prog, n_ops, k);
        const int zero_wire = cdr_min_wire(prog, n_ops, k + 1, j) == 0;
        if (n > op->count && zero_wire) return RTPS_CDR_TOO_LONG;
        /* elements that read no bytes cannot fail and store nothing (zero-count arrays only) */
        if (n == 0 || zero_wire) { k = j; break; }
        cdr_frame f = {k, n, 0, base + op->out_off + (seq ? 4u : 0u), base, write};
        fr[depth++] = f;
        base = f.elem0;
        write = write && op->count > 0;
        break;
      }
      case RTPS_CDR_END: {
        cdr_frame* f = &fr[depth - 1];
        const rtps_cdr_op* b = &prog[f->begin];
        if (++f->i < f->n) {
          base = f->elem0 + f->i * b->stride;
          write = f->write && f->i < b->count;
          k = f->begin; /* the loop's ++k enters the element's first op */
        } else {
          depth--;
          base = f->base;
          write = f->write;
          if (f->n > b->count) return RTPS_CDR_TOO_LONG;
        }
        break;
      }
      default:
        return RTPS_CDR_TOO_LONG;
    }
  }
  return RTPS_CDR_OK;
}

/* Decode every record (see rtps_rx_cdr_decode in rtps_rx.h); rows are zeroed
 * unless the decode succeeds. */
void rtps_oracle_cdr_decode(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes, const uint8_t* arena,
                            const uint64_t* off, const rtps_record* recs, uint64_t n_recs, uint8_t* rows,
                            uint8_t* status) {
  for (uint64_t r = 0; r < n_recs; ++r) {
    const rtps_record* rec = &recs[r];
    uint8_t* row = rows + r * row_bytes;
    memset(row, 0, row_bytes);
    if (rec->kind != RTPS_DATA || rec->payload_kind != RTPS_PK_DATA) { status[r] = RTPS_CDR_NOT_DATA; continue; }
    /* SimpleDataReader::deserialize_with: rep id must be a supported encoding */
    const uint8_t* id = rec->u.data.rep_id;
    int le;
    if (id[0] == 0 && id[1] == 0) le = 0;                        /* CDR_BE    */
    else if (id[0] == 0 && (id[1] == 1 || id[1] == 3)) le = 1;   /* CDR_LE, PL_CDR_LE */
    else { status[r] = RTPS_CDR_BAD_ENCODING; continue; }
    const uint8_t* value = arena + off[rec->dgram_idx] + rec->u.data.pl_off + 4;
    uint8_t st = cdr_decode_one(prog, n_ops, value, (uint32_t)rec->u.data.pl_len - 4, le, row);
    if (st != RTPS_CDR_OK) memset(row, 0, row_bytes);
    status[r] = st;
  }
}

/* ------------------------------------------------------------------------ */
/* DataFrag reassembly                                */
/*   FragmentAssembler / AssemblyBuffer   rtps/fragment_assembler.rs:23-214  */
/*   driven by Reader::handle_datafrag_msg io_uring/rtps/reader.rs:563-647    */
/* Sequential restatement with state kept across batches.                    */
/* ------------------------------------------------------------------------ */
/* Assemblers are keyed by (writer GUID, reader word): one FragmentAssembler per
 * writer of each Reader (reader.rs:617-619, 638-647).  The reader word is 0 in the
 * reader-less form (rtps_oracle_frag_batch: one assembler per writer) and
 * slot | 0x10000 in rtps_oracle_frag_batch_readers. */
#define FA_KEY 20
typedef struct fa_writer { uint8_t guid[FA_KEY]; uint16_t frag_size; int used; } fa_writer;
typedef struct fa_buf {      /* AssemblyBuffer (:23-33) */
  uint8_t guid[FA_KEY];
  int64_t sn;
  uint32_t data_size, count, nset;
  uint8_t* bytes;            /* buffer_bytes, zero-initialised (:49-50) */
  uint8_t* bits;             /* received_bitmap */
  uint64_t modified;         /* modified_time (:31, :61, :139): the batch clock of its last fragment */
  int used;
} fa_buf;
typedef struct rtps_oracle_frag {
  fa_writer* w; size_t wcap, wn;
  fa_buf* b; size_t bcap, bn;
  uint64_t now;              /* the batch clock (Timestamp::now() of the batch's fragments) */
} rtps_oracle_frag;

static uint64_t fa_hash(const uint8_t* k, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= k[i]; h *= 1099511628211ull; }
  return h ^ (h >> 29);
}
static fa_writer* fa_writer_get(rtps_oracle_frag* f, const uint8_t guid[FA_KEY], int create) {
  if (create && (f->wn + 1) * 2 > f->wcap) {
    size_t ncap = f->wcap ? f->wcap * 2 : 64;
    fa_writer* nw = (fa_writer*)calloc(ncap, sizeof(fa_writer));
    for (size_t i = 0; i < f->wcap; ++i)
      if (f->w[i].used) {
        size_t j = fa_hash(f->w[i].guid, FA_KEY) & (ncap - 1);
        while (nw[j].used) j = (j + 1) & (ncap - 1);
        nw[j] = f->w[i];
      }
    free(f->w); f->w = nw; f->wcap = ncap;
  }
  if (!f->wcap) return NULL;
  size_t j = fa_hash(guid, FA_KEY) & (f->wcap - 1);
  while (f->w[j].used) {
    if (!memcmp(f->w[j].guid, guid, FA_KEY)) return &f->w[j];
    j = (j + 1) & (f->wcap - 1);
  }
  if (!create) return NULL;
  f->w[j].used = 1; memcpy(f->w[j].guid, guid, FA_KEY); f->wn++;
  return &f->w[j];
}
static void fa_key(uint8_t k[FA_KEY + 8], const uint8_t guid[FA_KEY], int64_t sn) {
  memcpy(k, guid, FA_KEY); memcpy(k + FA_KEY, &sn, 8);
}
static fa_buf* fa_buf_find(rtps_oracle_frag* f, const uint8_t guid[FA_KEY], int64_t sn, size_t* slot) {
  if (!f->bcap) return NULL;
  uint8_t k[FA_KEY + 8];
  fa_key(k, guid, sn);
  size_t j = fa_hash(k, FA_KEY + 8) & (f->bcap - 1);
  while (f->b[j].used) {
    if (f->b[j].used == 1 && f->b[j].sn == sn && !memcmp(f->b[j].guid, guid, FA_KEY)) { if (slot) *slot = j; return &f->b[j]; }
    j = (j + 1) & (f->bcap - 1);
  }
  return NULL;
}
static void fa_buf_rehash(rtps_oracle_frag* f, size_t ncap) {
  fa_buf* nb = (fa_buf*)calloc(ncap, sizeof(fa_buf));
  for (size_t i = 0; i < f->bcap; ++i)
    if (f->b[i].used == 1) {
      uint8_t k[FA_KEY + 8];
      fa_key(k, f->b[i].guid, f->b[i].sn);
      size_t j = fa_hash(k, FA_KEY + 8) & (ncap - 1);
      while (nb[j].used) j = (j + 1) & (ncap - 1);
      nb[j] = f->b[i];
    }
  free(f->b); f->b = nb; f->bcap = ncap;
}
static fa_buf* fa_buf_new(rtps_oracle_frag* f, const uint8_t guid[FA_KEY], int64_t sn) {
  if ((f->bn + 1) * 2 > f->bcap) fa_buf_rehash(f, f->bcap ? f->bcap * 2 : 64);
  uint8_t k[FA_KEY + 8];
  fa_key(k, guid, sn);
  size_t j = fa_hash(k, FA_KEY + 8) & (f->bcap - 1);
  while (f->b[j].used == 1) j = (j + 1) & (f->bcap - 1);
  memset(&f->b[j], 0, sizeof(fa_buf));
  f->b[j].used = 1; memcpy(f->b[j].guid, guid, FA_KEY); f->b[j].sn = sn; f->bn++;
  return &f->b[j];
}
static void fa_buf_drop(rtps_oracle_frag* f, fa_buf* b) {
  free(b->bytes); free(b->bits);
  b->bytes = NULL; b->bits = NULL;
  b->used = 2;  /* tombstone */
  f->bn--;
  fa_buf_rehash(f, f->bcap);  /* clears tombstones (test sizes: fine) */
}

rtps_oracle_frag* rtps_oracle_frag_new(void) { return (rtps_oracle_frag*)calloc(1, sizeof(rtps_oracle_frag)); }
void rtps_oracle_frag_free(rtps_oracle_frag* f) {
  if (!f) return;
  for (size_t i = 0; i < f->bcap; ++i) if (f->b[i].used == 1) { free(f->b[i].bytes); free(f->b[i].bits); }
  free(f->b); free(f->w); free(f);
}
uint64_t rtps_oracle_frag_pending(const rtps_oracle_frag* f) { return f->bn; }
void rtps_oracle_frag_set_clock(rtps_oracle_frag* f, uint64_t now_ns) { f->now = now_ns; }
/* FragmentAssembler::garbage_collect_before (rtps/fragment_assembler.rs:216-224): drop every
 * buffer whose modified_time < expire_before.  Returns the buffers left. */
uint64_t rtps_oracle_frag_gc(rtps_oracle_frag* f, uint64_t expire_before_ns) {
  for (size_t i = 0; i < f->bcap; ++i)
    if (f->b[i].used == 1 && f->b[i].modified < expire_before_ns) {
      free(f->b[i].bytes); free(f->b[i].bits);
      f->b[i].bytes = NULL; f->b[i].bits = NULL;
      f->b[i].used = 2;
      f->bn--;
    }
  if (f->bcap) fa_buf_rehash(f, f->bcap);
  return f->bn;
}

/* Reader::handle_datafrag_msg's assembler step for one DATA_FRAG record and one
 * assembler key (writer GUID || reader word): FragmentAssembler::new on first use
 * (fragment size of that first DATA_FRAG), AssemblyBuffer::new / insert_frags /
 * is_complete (fragment_assembler.rs:35-214).  A completed buffer becomes a sample
 * (descriptors beyond max_samples and bytes beyond heap_bytes are not written). */
static void fa_insert(rtps_oracle_frag* f, const uint8_t key[FA_KEY], const rtps_record* rec, uint64_t r,
                      uint16_t reader_slot, const uint8_t* arena, const uint64_t* off, rtps_frag_sample* samples,
                      uint64_t max_samples, uint8_t* heap, uint64_t heap_bytes, uint64_t* ns, uint64_t* used) {
  /* Reader::fragment_assembler_mutable: or_insert_with(FragmentAssembler::new(datafrag.fragment_size)) */
  fa_writer* w = fa_writer_get(f, key, 0);
  if (!w) { w = fa_writer_get(f, key, 1); w->frag_size = rec->u.frag.frag_size; }
  const uint32_t F = w->frag_size;
  /* assembly_buffers.entry(writer_sn).or_insert_with(|| AssemblyBuffer::new(datafrag)) */
  fa_buf* b = fa_buf_find(f, key, rec->sn, NULL);
  if (!b) {
    b = fa_buf_new(f, key, rec->sn);
    const uint32_t ds = rec->u.frag.data_size, fs = rec->u.frag.frag_size;  /* 1 <= fs <= ds (parse) */
    b->data_size = ds;
    b->count = ds / fs + (ds % fs > 0);  /* total_number_of_fragments, data_frag.rs:97-119 */
    b->bytes = (uint8_t*)calloc(ds ? ds : 1, 1);
    b->bits = (uint8_t*)calloc(b->count ? b->count : 1, 1);
  }
  b->modified = f->now;  /* AssemblyBuffer::new (:54-61) / insert_frags (:139) */
  /* insert_frags (:65-140) with frag_size = the assembler's F */
  const uint64_t start0 = (uint64_t)rec->u.frag.frag_start - 1;
  const uint64_t fis = rec->u.frag.frags_in_sub;
  const uint64_t pl_len = rec->u.frag.pl_len;
  const uint64_t from = start0 * F;
  uint64_t to = from + (fis * F < pl_len ? fis * F : pl_len);
  if (to > b->data_size) to = b->data_size;
  if (to > from)  /* reference: to < from panics (usize underflow); clamped to nothing here */
    memcpy(b->bytes + from, arena + off[rec->dgram_idx] + rec->u.frag.pl_off, (size_t)(to - from));
  for (uint64_t k = 0; k < fis; ++k) {
    const uint64_t bit = start0 + k;
    if (bit >= b->count) break;  /* reference: BitVec::set panics; ignored here */
    if (!b->bits[bit]) { b->bits[bit] = 1; b->nset++; }
  }
  if (b->nset == b->count) {  /* is_complete -> remove, SerializedPayload::from_bytes */
    if (*ns < max_samples) {
      rtps_frag_sample* sm = &samples[*ns];
      memset(sm, 0, sizeof(*sm));
      memcpy(sm->writer_guid, key, 16);
      sm->sn = rec->sn;
      sm->data_size = b->data_size;
      sm->rec_idx = (uint32_t)r;
      sm->flags = rec->flags;
      sm->reader_slot = reader_slot;
      sm->heap_off = *used;
      sm->status = b->data_size < 4 ? RTPS_FRAG_SHORT : RTPS_FRAG_OK;
      if (*used + b->data_size <= heap_bytes) memcpy(heap + *used, b->bytes, b->data_size);
      else sm->status = RTPS_FRAG_NO_ROOM;
    }
    *used += ((uint64_t)b->data_size + 15) & ~15ull;
    (*ns)++;
    fa_buf_drop(f, b);
  }
}

/* One batch without readers: every RTPS_DATA_FRAG record with ROUTE_PASS, in record
 * order, one assembler per writer (reader word 0).  Returns the completed samples. */
uint64_t rtps_oracle_frag_batch(rtps_oracle_frag* f, const uint8_t* arena, const uint64_t* off,
                                const rtps_record* recs, uint64_t n_recs, rtps_frag_sample* samples,
                                uint64_t max_samples, uint8_t* heap, uint64_t heap_bytes, uint64_t* heap_used) {
  uint64_t ns = 0, used = 0;
  for (uint64_t r = 0; r < n_recs; ++r) {
    const rtps_record* rec = &recs[r];
    if (rec->kind != RTPS_DATA_FRAG || !(rec->route & RTPS_ROUTE_PASS)) continue;
    uint8_t key[FA_KEY];
    memcpy(key, rec->prefix, 12);
    memcpy(key + 12, rec->writer_id, 4);
    memset(key + 16, 0, 4);
    fa_insert(f, key, rec, r, RTPS_NO_MATCH, arena, off, samples, max_samples, heap, heap_bytes, &ns, &used);
  }
  if (heap_used) *heap_used = used;
  return ns;
}

/* One batch with readers: Domain::handle_event hands each DATA_FRAG the receiver passes
 * to user readers (not a builtin pair) to every reader of its target set in turn
 * (dp_event_loop.rs:266-327; toff / tent = rtps_oracle_targets), and each reader's
 * handle_datafrag_msg (io_uring/rtps/reader.rs:563-636) first drops it when its
 * Lifespan has expired for the source timestamp (:578-589: lifespan.duration <
 * receive_timestamp.duration_since(source), Timestamp ticks wrapping-subtracted as
 * an i64 Duration, structure/time.rs:103-113), then feeds its own assembler for the
 * writer (:617-619, 638-647).  life: the Lifespan of each reader slot in Duration
 * ticks ([65536], INT64_MAX: none; NULL: none at all); recv_ticks: the batch's
 * Timestamp::now() as ticks.  Samples in completing order, each with its reader. */
uint64_t rtps_oracle_frag_batch_readers(rtps_oracle_frag* f, const uint8_t* arena, const uint64_t* off,
                                        const rtps_record* recs, uint64_t n_recs, const uint64_t* toff,
                                        const rtps_target* tent, const int64_t* life, uint64_t recv_ticks,
                                        rtps_frag_sample* samples, uint64_t max_samples, uint8_t* heap,
                                        uint64_t heap_bytes, uint64_t* heap_used) {
  uint64_t ns = 0, used = 0;
  for (uint64_t r = 0; r < n_recs; ++r) {
    const rtps_record* rec = &recs[r];
    if (rec->kind != RTPS_DATA_FRAG || !(rec->route & RTPS_ROUTE_PASS) || (rec->route & RTPS_ROUTE_BUILTIN)) continue;
    for (uint64_t k = toff[r]; k < toff[r + 1]; ++k) {
      const uint16_t slot = tent[k].reader_slot;
      if (life && life[slot] != INT64_MAX && (rec->route & RTPS_ROUTE_TS_VALID)) {
        const uint64_t src = ((uint64_t)rec->ts_sec << 32) | rec->ts_frac;
        if (life[slot] < (int64_t)(recv_ticks - src)) continue;  /* lifespan exceeded: return */
      }
      uint8_t key[FA_KEY];
      memcpy(key, rec->prefix, 12);
      memcpy(key + 12, rec->writer_id, 4);
      const uint32_t word = (uint32_t)slot | 0x10000u;
      memcpy(key + 16, &word, 4);
      fa_insert(f, key, rec, r, slot, arena, off, samples, max_samples, heap, heap_bytes, &ns, &used);
    }
  }
  if (heap_used) *heap_used = used;
  return ns;
}

/* ------------------------------------------------------------------------ */
/* History-cache ingest: the stateful reader's        */
/* writer-proxy bookkeeping, restated sequentially in record order.          */
/*   RtpsWriterProxy  rtps/rtps_writer_proxy.rs:17-355                        */
/*   Reader::handle_data_msg / process_received_data                          */
/*                    io_uring/rtps/reader.rs:514-561, 693-758                */
/*   Reader::handle_heartbeat_msg  reader.rs:859-917                          */
/*   Reader::handle_gap_msg        reader.rs:1060-1116                        */
/* The proxy's `changes` BTreeMap is a hash set of sequence numbers: only    */
/* membership is ever observed (should_ignore_change, advance_ack_base); the */
/* entries irrelevant_changes_range removes all lie below the new ack_base.   */
/* ------------------------------------------------------------------------ */
typedef struct ig_proxy {
  int64_t ack_base;   /* SequenceNumber::new(1) (rtps_writer_proxy.rs:96) */
  int32_t hb_count;   /* received_heartbeat_count, 0 */
  int64_t* set; uint8_t* used; size_t cap, n;
} ig_proxy;
typedef struct rtps_oracle_ingest {
  oracle_readers R;     /* the local readers and their proxies (copies) */
  rtps_reader* readers;
  rtps_proxy* proxies;
  ig_proxy* p;          /* one RtpsWriterProxy per proxy */
  rtps_target* tmp;
} rtps_oracle_ingest;

static size_t ig_h(int64_t s) { uint64_t x = (uint64_t)s * 0x9e3779b97f4a7c15ull; return (size_t)(x ^ (x >> 31)); }
static int ig_has(const ig_proxy* p, int64_t s) {
  if (!p->cap) return 0;
  for (size_t j = ig_h(s) & (p->cap - 1); p->used[j]; j = (j + 1) & (p->cap - 1))
    if (p->set[j] == s) return 1;
  return 0;
}
static void ig_add(ig_proxy* p, int64_t s) {
  if (ig_has(p, s)) return;
  if ((p->n + 1) * 2 > p->cap) {
    size_t ncap = p->cap ? p->cap * 2 : 64;
    int64_t* ns = (int64_t*)calloc(ncap, sizeof(int64_t));
    uint8_t* nu = (uint8_t*)calloc(ncap, 1);
    for (size_t i = 0; i < p->cap; ++i)
      if (p->used[i]) {
        size_t j = ig_h(p->set[i]) & (ncap - 1);
        while (nu[j]) j = (j + 1) & (ncap - 1);
        nu[j] = 1; ns[j] = p->set[i];
      }
    free(p->set); free(p->used); p->set = ns; p->used = nu; p->cap = ncap;
  }
  size_t j = ig_h(s) & (p->cap - 1);
  while (p->used[j]) j = (j + 1) & (p->cap - 1);
  p->used[j] = 1; p->set[j] = s; p->n++;
}
/* advance_ack_base (:338-355): move past a run of consecutive known changes */
static void ig_advance(ig_proxy* p) { while (ig_has(p, p->ack_base)) p->ack_base++; }
/* should_ignore_change (:202-204) */
static int ig_should_ignore(const ig_proxy* p, int64_t s) { return s < p->ack_base || ig_has(p, s); }
/* received_changes_add (:207-224) */
static void ig_received(ig_proxy* p, int64_t s) { ig_add(p, s); if (s == p->ack_base) ig_advance(p); }
/* set_irrelevant_change (:226-239) */
static void ig_irrelevant(ig_proxy* p, int64_t s) {
  if (s >= p->ack_base) ig_add(p, s);
  if (s == p->ack_base) ig_advance(p);
}
/* irrelevant_changes_range (:241-288) */
static void ig_irrelevant_range(ig_proxy* p, int64_t from, int64_t until) {
  if (from > until) return;  /* "negative range": error, nothing changes */
  if (from <= p->ack_base) {
    if (until > p->ack_base) { p->ack_base = until; ig_advance(p); }
  } else {
    for (int64_t s = from; s < until; ++s) ig_add(p, s);
  }
}

rtps_oracle_ingest* rtps_oracle_ingest_new(const rtps_reader* readers, uint32_t nr, const rtps_proxy* proxies,
                                           uint32_t np) {
  rtps_oracle_ingest* h = (rtps_oracle_ingest*)calloc(1, sizeof(rtps_oracle_ingest));
  h->readers = (rtps_reader*)calloc(nr ? nr : 1, sizeof(rtps_reader));
  h->proxies = (rtps_proxy*)calloc(np ? np : 1, sizeof(rtps_proxy));
  if (nr) memcpy(h->readers, readers, nr * sizeof(rtps_reader));
  if (np) memcpy(h->proxies, proxies, np * sizeof(rtps_proxy));
  oracle_readers_init(&h->R, h->readers, nr, h->proxies, np);
  h->p = (ig_proxy*)calloc(np ? np : 1, sizeof(ig_proxy));
  for (uint32_t e = 0; e < np; ++e) h->p[e].ack_base = 1; /* RtpsWriterProxy::new (rtps_writer_proxy.rs:96) */
  h->tmp = (rtps_target*)malloc(sizeof(rtps_target) * (nr ? nr : 1));
  return h;
}
/* New readers / proxies for an existing ingest: proxy state is kept by
 * position, as the device keeps it (rtps_rx_ingest: "indexed by proxy
 * position"); proxies past the old count start fresh (RtpsWriterProxy::new). */
void rtps_oracle_ingest_set_readers(rtps_oracle_ingest* h, const rtps_reader* readers, uint32_t nr,
                                    const rtps_proxy* proxies, uint32_t np) {
  const uint32_t old = h->R.np;
  for (uint32_t e = np; e < old; ++e) { free(h->p[e].set); free(h->p[e].used); }
  h->p = (ig_proxy*)realloc(h->p, sizeof(ig_proxy) * (np ? np : 1));
  for (uint32_t e = old; e < np; ++e) { memset(&h->p[e], 0, sizeof(ig_proxy)); h->p[e].ack_base = 1; }
  oracle_readers_free(&h->R);
  free(h->readers); free(h->proxies); free(h->tmp);
  h->readers = (rtps_reader*)calloc(nr ? nr : 1, sizeof(rtps_reader));
  h->proxies = (rtps_proxy*)calloc(np ? np : 1, sizeof(rtps_proxy));
  if (nr) memcpy(h->readers, readers, nr * sizeof(rtps_reader));
  if (np) memcpy(h->proxies, proxies, np * sizeof(rtps_proxy));
  oracle_readers_init(&h->R, h->readers, nr, h->proxies, np);
  h->tmp = (rtps_target*)malloc(sizeof(rtps_target) * (nr ? nr : 1));
}
void rtps_oracle_ingest_free(rtps_oracle_ingest* h) {
  if (!h) return;
  for (uint32_t e = 0; e < h->R.np; ++e) { free(h->p[e].set); free(h->p[e].used); }
  oracle_readers_free(&h->R);
  free(h->p); free(h->readers); free(h->proxies); free(h->tmp); free(h);
}

/* Reader::process_received_data for one target (io_uring/rtps/reader.rs:693-758):
 * 1 = the sample enters the reader's cache. */
static int ig_process_sample(rtps_oracle_ingest* h, const rtps_target* t, const uint8_t wid[4], int64_t sn) {
  if (t->proxy != RTPS_NO_PROXY) {
    ig_proxy* p = &h->p[t->proxy];
    if (ig_should_ignore(p, sn) && !(t->reader_flags & RTPS_TARGET_DUPLICATES_OK)) return 0;
    ig_received(p, sn);  /* writer_proxy.received_changes_add */
    return 1;
  }
  /* no writer proxy: dropped for user-defined writers, accepted otherwise (:734-739) */
  return (wid[3] & 0xF0) != 0x00;
}

/* One batch in record order (see rtps_rx_ingest in rtps_rx.h), every routed
 * record handed to each of its target readers in turn as Domain::handle_event
 * does (dp_event_loop.rs:266-327).  accept[m] = readers that took the record's
 * sample (saturating at 255); deliveries (record, reader slot) in order, count
 * returned (past max_del counted, not written); ack_base[n_proxies] (optional). */
uint64_t rtps_oracle_ingest_batch(rtps_oracle_ingest* h, const uint8_t* arena, const uint64_t* offs,
                                  const rtps_record* recs, uint64_t m, const rtps_frag_sample* frag, uint64_t nf,
                                  uint32_t flags, uint8_t* accept, rtps_delivery* del, uint64_t max_del,
                                  int64_t* ack_base) {
  /* the first completed sample of each record: the samples of one record are consecutive
   * (completing order), one per reader whose assembler completed it (or RTPS_NO_MATCH:
   * every reader of the record) */
  uint32_t* fidx = (uint32_t*)malloc((m ? m : 1) * sizeof(uint32_t));
  for (uint64_t i = 0; i < m; ++i) fidx[i] = 0xffffffffu;
  for (uint64_t s = nf; s-- > 0;)
    if (frag[s].rec_idx < m) fidx[frag[s].rec_idx] = (uint32_t)s;
  uint64_t nd = 0;
  for (uint64_t i = 0; i < m; ++i) {
    const rtps_record* r = &recs[i];
    accept[i] = 0;
    /* SubmessageIter2 passed it, and it is not a builtin pair (Discovery2 takes those) */
    if (!(r->route & RTPS_ROUTE_PASS) || builtin_writer_pair(r->reader_id, r->writer_id)) continue;
    const int writer_kind = r->kind == RTPS_DATA || r->kind == RTPS_DATA_FRAG || r->kind == RTPS_HEARTBEAT ||
                            r->kind == RTPS_HEARTBEAT_FRAG || r->kind == RTPS_GAP;
    if (!writer_kind) continue;
    int matched = 0;
    const uint32_t nt = oracle_targets(&h->R, r->prefix, r->writer_id, h->tmp, h->R.nr, &matched);
    uint32_t took = 0;
    for (uint32_t k = 0; k < nt; ++k) {
      const rtps_target* t = &h->tmp[k];
      ig_proxy* p = t->proxy != RTPS_NO_PROXY ? &h->p[t->proxy] : NULL;
      int acc = 0;
      if (fidx[i] != 0xffffffffu) {  /* completed DataFrag sample (handle_datafrag_msg :614-626) */
        const rtps_frag_sample* fs = NULL;  /* this reader's, or a writer-keyed one */
        for (uint64_t s = fidx[i]; s < nf && frag[s].rec_idx == i && !fs; ++s)
          if (frag[s].reader_slot == RTPS_NO_MATCH || frag[s].reader_slot == t->reader_slot) fs = &frag[s];
        if (fs && fs->status != RTPS_FRAG_SHORT) acc = ig_process_sample(h, t, r->writer_id, fs->sn);
      } else if (r->kind == RTPS_DATA) {
        if (r->payload_kind != RTPS_PK_DATA && r->payload_kind != RTPS_PK_KEY && r->payload_kind != RTPS_PK_KEY_HASH)
          continue;  /* data_to_dds_data failed: no process_received_data (reader.rs:552-558) */
        acc = ig_process_sample(h, t, r->writer_id, r->sn);
      } else if (r->kind == RTPS_HEARTBEAT) {
        /* BestEffort (or stateless) readers ignore HEARTBEATs (:871-881), no proxy: ignored (:885-891) */
        if ((flags & RTPS_INGEST_BEST_EFFORT) || (t->reader_flags & RTPS_READER_BEST_EFFORT) || !p) continue;
        if (r->u.hb.count <= p->hb_count) continue;  /* already seen (reader.rs:902-905) */
        p->hb_count = r->u.hb.count;
        ig_irrelevant_range(p, 0, r->sn);            /* irrelevant_changes_up_to(first_sn) */
      } else if (r->kind == RTPS_GAP) {
        if (!p) continue;                            /* no writer proxy (:1076-1086) */
        const int64_t start = r->sn, base = r->u.gap.list_base;
        if (start <= 0 || base <= 0) continue;       /* validity (reader.rs:1087-1102) */
        ig_irrelevant_range(p, start, base);
        const uint8_t* bm = arena + offs[r->dgram_idx] + r->u.gap.bitmap_off;
        const int le = r->flags & 1;
        for (uint32_t b = 0; b < r->u.gap.num_bits; ++b) {  /* NumberSetIter (sequence_number.rs:543-557) */
          const uint8_t* w = bm + 4 * (b / 32);
          uint32_t word = le ? (uint32_t)w[0] | ((uint32_t)w[1] << 8) | ((uint32_t)w[2] << 16) | ((uint32_t)w[3] << 24)
                             : ((uint32_t)w[0] << 24) | ((uint32_t)w[1] << 16) | ((uint32_t)w[2] << 8) | (uint32_t)w[3];
          if (word & (1u << (31 - b % 32))) ig_irrelevant(p, base + (int64_t)b);
        }
      }
      if (acc) {
        if (nd < max_del) { del[nd].rec_idx = (uint32_t)i; del[nd].reader_slot = t->reader_slot; del[nd].flags = 0; }
        nd++;
        took++;
      }
    }
    accept[i] = (uint8_t)(took < 255 ? took : 255);
  }
  if (ack_base)
    for (uint32_t e = 0; e < h->R.np; ++e) ack_base[e] = h->p[e].ack_base;
  free(fidx);
  return nd;
}

/* ------------------------------------------------------------------------ */
/* Topic caches: TopicCache::add_change (structure/dds_cache.rs:210-284)    */
/* over the deliveries of rtps_oracle_ingest_batch, in order.  The cache's   */
/* `changes` BTreeMap is keyed by receive instant, i.e. insertion order; the */
/* garbage collection remove_changes_before(ZERO) (:367-420) removes only    */
/* the oldest (`ts < ZERO` never holds, so may_remove never exceeds          */
/* must_remove), so the live changes are always the insertions with index   */
/* in [E, I) (I = insertions so far, E = removed so far), and a GC sets      */
/* E = max(E, I - max_keep).  sequence_numbers (:134-135) maps (writer GUID, */
/* SN) to a live change: here the key's last insertion index, live iff >= E. */
/* ------------------------------------------------------------------------ */
typedef struct tc_ent { uint8_t guid[16]; int64_t sn; uint32_t topic; uint64_t idx; } tc_ent;
typedef struct rtps_oracle_topics {
  uint32_t nt;           /* topics: [0, nt) configured, then one private topic per unmapped slot */
  uint32_t topic_of[65536];
  uint64_t* I; uint64_t* E; uint32_t* K;
  uint32_t cap_t;
  tc_ent* map; uint8_t* used; size_t cap, n;
} rtps_oracle_topics;

static size_t tc_h(const uint8_t g[16], int64_t sn, uint32_t t) {
  uint64_t x = 0x9e3779b97f4a7c15ull ^ t;
  for (int i = 0; i < 16; ++i) x = (x ^ g[i]) * 0x100000001b3ull;
  x = (x ^ (uint64_t)sn) * 0xff51afd7ed558ccdull;
  return (size_t)(x ^ (x >> 29));
}
static tc_ent* tc_find(rtps_oracle_topics* h, const uint8_t g[16], int64_t sn, uint32_t t) {
  if (!h->cap) return NULL;
  for (size_t j = tc_h(g, sn, t) & (h->cap - 1); h->used[j]; j = (j + 1) & (h->cap - 1))
    if (h->map[j].topic == t && h->map[j].sn == sn && !memcmp(h->map[j].guid, g, 16)) return &h->map[j];
  return NULL;
}
static void tc_put(rtps_oracle_topics* h, const uint8_t g[16], int64_t sn, uint32_t t, uint64_t idx) {
  tc_ent* e = tc_find(h, g, sn, t);
  if (e) { e->idx = idx; return; }
  if ((h->n + 1) * 2 > h->cap) {
    size_t ncap = h->cap ? h->cap * 2 : 1024;
    tc_ent* nm = (tc_ent*)calloc(ncap, sizeof(tc_ent));
    uint8_t* nu = (uint8_t*)calloc(ncap, 1);
    for (size_t i = 0; i < h->cap; ++i)
      if (h->used[i]) {
        size_t j = tc_h(h->map[i].guid, h->map[i].sn, h->map[i].topic) & (ncap - 1);
        while (nu[j]) j = (j + 1) & (ncap - 1);
        nu[j] = 1; nm[j] = h->map[i];
      }
    free(h->map); free(h->used); h->map = nm; h->used = nu; h->cap = ncap;
  }
  size_t j = tc_h(g, sn, t) & (h->cap - 1);
  while (h->used[j]) j = (j + 1) & (h->cap - 1);
  h->used[j] = 1;
  memcpy(h->map[j].guid, g, 16); h->map[j].sn = sn; h->map[j].topic = t; h->map[j].idx = idx;
  h->n++;
}
/* topics[n] = (topic id, max_keep_samples); readers[m] = (reader slot, topic id) */
rtps_oracle_topics* rtps_oracle_topics_new(const rtps_topic* topics, uint32_t n, const rtps_topic_reader* readers,
                                           uint32_t m) {
  rtps_oracle_topics* h = (rtps_oracle_topics*)calloc(1, sizeof(rtps_oracle_topics));
  h->nt = n;
  h->cap_t = n + 65536u;
  h->I = (uint64_t*)calloc(h->cap_t, 8); h->E = (uint64_t*)calloc(h->cap_t, 8); h->K = (uint32_t*)calloc(h->cap_t, 4);
  for (uint32_t t = 0; t < n; ++t) h->K[t] = topics[t].max_keep_samples ? topics[t].max_keep_samples : 1u;
  for (uint32_t s = 0; s < 65536u; ++s) { h->topic_of[s] = n + s; h->K[n + s] = 64; }  /* private topic per slot */
  for (uint32_t r = 0; r < m; ++r)
    for (uint32_t t = 0; t < n; ++t)
      if (topics[t].topic == readers[r].topic) h->topic_of[readers[r].reader_slot] = t;
  return h;
}
void rtps_oracle_topics_free(rtps_oracle_topics* h) {
  if (!h) return;
  free(h->I); free(h->E); free(h->K); free(h->map); free(h->used); free(h);
}
/* remove_changes_before(ZERO) on every topic (DDSCache::garbage_collect) */
void rtps_oracle_topics_gc(rtps_oracle_topics* h) {
  for (uint32_t t = 0; t < h->cap_t; ++t)
    if (h->I[t] - h->E[t] > h->K[t]) h->E[t] = h->I[t] - h->K[t];
}
/* add_change for every delivery in order (the change of record rec_idx: writer GUID =
 * prefix || writer_id, SN = the record's sn, which a DATA_FRAG's completed sample shares);
 * sets RTPS_DELIVERY_CACHED in del[k].flags when it is stored.  Returns the stored count. */
uint64_t rtps_oracle_topics_apply(rtps_oracle_topics* h, const rtps_record* recs, uint64_t m, rtps_delivery* del,
                                  uint64_t nd) {
  uint64_t stored = 0;
  for (uint64_t k = 0; k < nd; ++k) {
    del[k].flags &= (uint16_t)~RTPS_DELIVERY_CACHED;
    if (del[k].rec_idx >= m) continue;
    const rtps_record* r = &recs[del[k].rec_idx];
    uint8_t g[16];
    memcpy(g, r->prefix, 12); memcpy(g + 12, r->writer_id, 4);
    const uint32_t t = h->topic_of[del[k].reader_slot];
    /* garbage collection first, at every 64th sequence number ((sn as usize) % 64 == 0, :230-238) */
    if (((uint64_t)r->sn & 63u) == 0 && h->I[t] - h->E[t] > h->K[t]) h->E[t] = h->I[t] - h->K[t];
    const tc_ent* e = tc_find(h, g, r->sn, t);
    if (e && e->idx >= h->E[t]) continue;  /* find_by_sn hit: duplicate, not stored (:241-252) */
    tc_put(h, g, r->sn, t, h->I[t]);       /* insert_sn + changes.insert (:254-256) */
    h->I[t]++;
    del[k].flags |= RTPS_DELIVERY_CACHED;
    stored++;
  }
  return stored;
}
