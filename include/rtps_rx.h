/*
 * rtps_rx.h — C ABI of the MI355X-native RTPS receive-path parser.
 *
 * Drop-in boundary for the rx parse of RustDDS (w-utter/rustdds-io_uring).
 * The functions below replace, for a *batch* of datagrams at once:
 *
 *   Message::read_from_buffer(&Bytes) -> io::Result<Message>
 *       src/rtps/message.rs:64-81
 *   MessageReceiver::handle_received_packet_2(&mut self, &Bytes)
 *       -> Option<SubmessageIter2>          src/io_uring/rtps/message_receiver.rs:232-287
 *   SubmessageIter2::next -> PassedSubmessage  (interpreter state, dest filter)
 *       src/io_uring/rtps/message_receiver.rs:56-119, 618-665, 289-295
 *   builtin-pair / matched-writer classification feeding Reader::handle_data_msg
 *       src/io_uring/discovery/discovery.rs:2795-2816, 3075-3095
 *       src/io_uring/rtps/dp_event_loop.rs:266-327, src/io_uring/rtps/reader.rs:474-484
 *   payload-kind decision of Reader::data_to_dds_data + SerializedPayload::from_bytes
 *       src/io_uring/rtps/reader.rs:760-833, src/messages/submessages/elements/serialized_payload.rs:86-110
 *
 * Plain C types only (no torch, no HIP types): a Rust caller binds this with
 * bindgen / a hand-written `extern "C"` block.
 *
 * Output model
 * ------------
 * For every input datagram i the library writes status[i] (RTPS_DGRAM_*).
 * For every submessage the reference *materialises* in Message.submessages
 * (everything except PAD and unknown / vendor / security kinds) of a datagram
 * whose status is RTPS_DGRAM_OK, one 64-byte rtps_record is written.
 * Records are in the reference's order: ascending (dgram_idx, sub_off).
 * A datagram whose status is not OK has zero records (the reference drops
 * the whole datagram on any submessage error: message.rs:75,
 * message_receiver.rs:275-282).
 *
 * All multi-byte record fields are host (little-endian) integers already
 * converted from the submessage's own byte order (flags bit 0).
 * GUID prefixes / entity ids are raw wire bytes.
 * Offsets (sub_off, pl_off, ...) are relative to the start of the datagram.
 */
#ifndef RTPS_RX_H
#define RTPS_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTPS_RX_ABI_VERSION 2u /* 2: reader sets (rtps_rx_set_readers), u32 targets, deliveries */

/* Largest datagram the record layout can address (u16 offsets).  The
 * reference's io_uring provided buffers are 64 KiB each
 * (src/io_uring/network/udp_listener.rs:7,27), so no datagram it can
 * receive is longer. */
#define RTPS_MAX_DATAGRAM 65536u

/* ---- per-datagram status (handle_received_packet_2 outcome) ------------ */
enum rtps_dgram_status {
  RTPS_DGRAM_OK = 0,         /* parsed; records emitted                          */
  RTPS_DGRAM_SHORT = 1,      /* len < 20, not a ping   (message_receiver.rs:238-251) */
  RTPS_DGRAM_PING = 2,       /* len < 20, "RTPS"...."DDSPING"                     */
  RTPS_DGRAM_RTPX = 3,       /* magic "RTPX"           (:254-266)                 */
  RTPS_DGRAM_BAD_MAGIC = 4,  /* other magic            (:267-271)                 */
  RTPS_DGRAM_BAD_HEADER = 5, /* version major > 2      (messages/header.rs:30-39)  */
  RTPS_DGRAM_SUBMSG_ERR = 6, /* any submessage read error -> whole datagram dropped */
  RTPS_DGRAM_TOO_LONG = 7    /* len > RTPS_MAX_DATAGRAM (cannot come from a UDP socket) */
};

/* ---- submessage kinds (messages/submessages/submessage_kind.rs:17-34) --- */
enum rtps_kind {
  RTPS_PAD = 0x01,
  RTPS_ACKNACK = 0x06,
  RTPS_HEARTBEAT = 0x07,
  RTPS_GAP = 0x08,
  RTPS_INFO_TS = 0x09,
  RTPS_INFO_SRC = 0x0c,
  RTPS_INFO_REPLY_IP4 = 0x0d,
  RTPS_INFO_DST = 0x0e,
  RTPS_INFO_REPLY = 0x0f,
  RTPS_NACK_FRAG = 0x12,
  RTPS_HEARTBEAT_FRAG = 0x13,
  RTPS_DATA = 0x15,
  RTPS_DATA_FRAG = 0x16
};

/* ---- rtps_record.route bits -------------------------------------------- */
/* PASS: SubmessageIter2::next would yield this submessage
 *   writer kinds: dest == own || dest == UNKNOWN   (message_receiver.rs:75-84)
 *   reader kinds: always                            (message_receiver.rs:88-113)
 *   interpreter kinds: never (state change only)    (message_receiver.rs:70-73) */
#define RTPS_ROUTE_PASS 0x01u
#define RTPS_ROUTE_TS_VALID 0x02u    /* a source timestamp is in effect (ts_sec/ts_frac) */
#define RTPS_ROUTE_HAS_QOS 0x04u     /* DATA / DATA_FRAG: inline QoS present (Q flag)    */
#define RTPS_ROUTE_HAS_PAYLOAD 0x08u /* DATA with D|K, DATA_FRAG: serialized payload    */
#define RTPS_ROUTE_BUILTIN 0x10u     /* (reader_id, writer_id) is a builtin discovery pair */
/* Writer kinds that are not a builtin pair go to the local readers
 * (io_uring/rtps/dp_event_loop.rs:266-327): */
#define RTPS_ROUTE_MATCHED 0x20u     /* some target reader has a writer proxy for the full writer GUID */
#define RTPS_ROUTE_TARGETED 0x40u    /* some local reader contains_writer(writer_id) (reader.rs:474-484) */

/* ---- rtps_record.payload_kind (Reader::data_to_dds_data, reader.rs:760-833) */
enum rtps_payload_kind {
  RTPS_PK_NONE = 0,           /* not a DATA submessage                            */
  RTPS_PK_DATA = 1,           /* (payload, D=1, K=0) -> DDSData::Data              */
  RTPS_PK_KEY = 2,            /* (payload, D=0, K=1) -> DDSData::DisposeByKey      */
  RTPS_PK_KEY_HASH = 3,       /* (none, 0, 0) + 16-byte PID_KEY_HASH -> DisposeByKeyHash */
  RTPS_PK_ERR_NO_CONTENT = 0x81, /* (none, 0, 0) without a usable KEY_HASH           */
  RTPS_PK_ERR_AMBIGUOUS = 0x82,  /* D=1 and K=1                                       */
  RTPS_PK_ERR_SHORT = 0x83       /* payload shorter than the 4-byte encapsulation header */
};

/* ---- rtps_record.u.data.change_kind: the sample's ChangeKind
 * (Reader::deduce_change_kind, reader.rs:1158-1182, for key / key-hash payload
 * kinds; Data -> Alive, ddsdata.rs:45-50) */
enum rtps_change_kind {
  RTPS_CK_ALIVE = 0,
  RTPS_CK_NOT_ALIVE_DISPOSED = 1,
  RTPS_CK_NOT_ALIVE_UNREGISTERED = 2,
  RTPS_CK_NONE = 0xFF         /* payload_kind is not a sample (RTPS_PK_ERR_*)       */
};

/* ---- one parsed submessage (64 bytes) ----------------------------------- */
typedef struct rtps_record {
  uint32_t dgram_idx;   /*  0 index of the datagram in the batch                   */
  uint16_t sub_off;     /*  4 offset of the submessage header in the datagram      */
  uint8_t kind;         /*  6 SubmessageKind                                       */
  uint8_t flags;        /*  7 raw submessage flags byte                            */
  uint8_t prefix[12];   /*  8 writer/reader kinds: source GuidPrefix in effect
                              (writer GUID = prefix||writer_id, reader_submsg source);
                              INFO_DST / INFO_SRC: the prefix the submessage carries;
                              INFO_TS / INFO_REPLY: source prefix in effect            */
  uint8_t writer_id[4]; /* 20 EntityId (raw)                                       */
  uint8_t reader_id[4]; /* 24 EntityId (raw)                                       */
  uint16_t aux16;       /* 28 DATA/DATA_FRAG: inline-QoS length incl. sentinel
                              (qos_off = pl_off - aux16); other kinds: body length   */
  uint8_t route;        /* 30 RTPS_ROUTE_* bits                                    */
  uint8_t payload_kind; /* 31 rtps_payload_kind (DATA only)                        */
  int64_t sn;           /* 32 DATA/DATA_FRAG/HB_FRAG/NACK_FRAG: writerSN;
                              HEARTBEAT: firstSN; GAP: gapStart; ACKNACK: readerSNState.base */
  union {               /* 40 kind-specific (16 bytes)                             */
    struct { uint16_t pl_off, pl_len; uint8_t rep_id[2], rep_opts[2];
             uint16_t key_hash_off, status_info_off, rsi_off;
             uint8_t change_kind, _r; } data;   /* change_kind: rtps_change_kind */
    struct { uint16_t pl_off, pl_len; uint32_t frag_start;
             uint16_t frags_in_sub, frag_size; uint32_t data_size; } frag;
    struct { int64_t last_sn; int32_t count; uint32_t _r; } hb;
    struct { uint32_t last_frag_num; int32_t count; uint32_t _r[2]; } hbfrag;
    struct { int64_t list_base; uint32_t num_bits; uint16_t bitmap_off, _r; } gap;
    struct { int32_t count; uint32_t _r; uint32_t num_bits; uint16_t bitmap_off, _r2; } acknack;
    struct { uint32_t fns_base; int32_t count; uint32_t num_bits; uint16_t bitmap_off, _r; } nackfrag;
    struct { uint8_t version[2], vendor[2]; uint32_t _r[3]; } infosrc;
    struct { uint32_t n_unicast, n_multicast; uint32_t _r[2]; } inforeply; /* n_multicast = 0xFFFFFFFF: None */
    uint8_t raw[16];
  } u;
  uint32_t ts_sec;      /* 56 source timestamp in effect (iff route & TS_VALID)    */
  uint32_t ts_frac;     /* 60                                                     */
} rtps_record;

#ifdef __cplusplus
#define RTPS_RX_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RTPS_RX_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif
RTPS_RX_STATIC_ASSERT(sizeof(rtps_record) == 64, "rtps_record must be 64 bytes");
RTPS_RX_STATIC_ASSERT(offsetof(rtps_record, sn) == 32, "rtps_record.sn at 32");
RTPS_RX_STATIC_ASSERT(offsetof(rtps_record, u) == 40, "rtps_record.u at 40");
RTPS_RX_STATIC_ASSERT(offsetof(rtps_record, ts_sec) == 56, "rtps_record.ts_sec at 56");

/* ---- local readers and their writer proxies (classification, a15) -------
 * The reference routes a writer submessage that is not a builtin pair to
 *   available_readers.values_mut().filter(|r| r.contains_writer(writer_id))
 *                                          io_uring/rtps/dp_event_loop.rs:266-275
 * where available_readers is a BTreeMap keyed by the reader's EntityId
 * (io_uring/rtps/message_receiver.rs:129) and contains_writer tests the ENTITY
 * ID of every matched writer, and is false for a stateless reader
 * (io_uring/rtps/reader.rs:474-484).  Each target reader then looks its
 * writer proxy up by the FULL writer GUID (matched_writers, a BTreeMap<GUID,
 * RtpsWriterProxy>, reader.rs:145, 712-738): with a proxy the sample is
 * deduplicated; without one it is dropped for a user-defined writer entity
 * kind and accepted otherwise (reader.rs:734-739).
 * The caller describes every reader and every (reader, writer GUID) proxy;
 * the library turns them into TARGET SETS, one per distinct outcome:
 *   - writer sets 0 .. W-1: one per distinct writer GUID that has a proxy in a
 *     non-stateless reader, numbered in order of first appearance in proxies[];
 *   - entity sets W .. W+E-1: one per distinct writer entity id of those
 *     proxies, first-appearance order (a writer GUID with no proxy whose
 *     entity id some reader contains).
 * A set lists its target readers in EntityId order with, per reader, the
 * proxy of the record's writer GUID (writer sets) or RTPS_NO_PROXY.  A
 * writer-kind record that is not a builtin pair gets target = the writer set
 * of prefix||writer_id if there is one (RTPS_ROUTE_MATCHED | TARGETED), else
 * the entity set of writer_id (RTPS_ROUTE_TARGETED), else RTPS_NO_TARGET. */
#define RTPS_READER_STATELESS 0x1u   /* like_stateless: never a target (reader.rs:474-484)            */
#define RTPS_READER_BEST_EFFORT 0x2u /* Reliability BestEffort: HEARTBEATs ignored (reader.rs:870-881) */
/* set by the library in rtps_target.reader_flags for a reader whose entity id is
 * SPDP_BUILTIN_PARTICIPANT_READER: it accepts duplicate samples (reader.rs:712-722) */
#define RTPS_TARGET_DUPLICATES_OK 0x8000u
typedef struct rtps_reader {
  uint8_t entity_id[4];  /* the reader's EntityId: its available_readers key (unique, orders the sets) */
  uint16_t reader_slot;  /* caller-defined handle reported in targets and deliveries */
  uint16_t flags;        /* RTPS_READER_* */
} rtps_reader;
typedef struct rtps_proxy {  /* one RtpsWriterProxy: an entry of the reader's matched_writers */
  uint8_t writer_guid[16];   /* prefix[12] || entity_id[4]; unique per reader */
  uint32_t reader;           /* index into the readers[] array */
} rtps_proxy;
typedef struct rtps_target {  /* one target reader of a target set */
  uint16_t reader_slot;
  uint16_t reader_flags;      /* the reader's RTPS_READER_* | RTPS_TARGET_DUPLICATES_OK */
  uint32_t proxy;             /* index into proxies[] of (this reader, the writer GUID), or RTPS_NO_PROXY */
} rtps_target;
#define RTPS_NO_TARGET 0xFFFFFFFFu
#define RTPS_NO_PROXY 0xFFFFFFFFu

/* Compatibility form: (writer GUID, reader slot) pairs.  Every distinct slot
 * becomes one reliable, stateful reader (EntityId order = order of first
 * appearance), every pair one proxy of that reader (repeated pairs once). */
typedef struct rtps_match {
  uint8_t writer_guid[16]; /* prefix[12] || entity_id[4] */
  uint16_t reader_slot;    /* caller-defined local reader index (< 0xFFFF) */
  uint16_t _pad;
} rtps_match;

#define RTPS_NO_MATCH 0xFFFFu

/* ---- context ------------------------------------------------------------ */
typedef struct rtps_rx_config {
  uint32_t abi_version;    /* RTPS_RX_ABI_VERSION */
  int32_t device;          /* HIP device ordinal */
  uint8_t own_prefix[12];  /* participant GuidPrefix (MessageReceiver::new) */
  uint32_t max_datagrams;  /* largest batch this context will parse */
  uint32_t flags;          /* reserved, 0 */
} rtps_rx_config;

/* Output buffers of one batch.  All pointers are DEVICE pointers (the
 * caller owns them).  records/match have room for max_records entries;
 * records past max_records are counted but not written. */
typedef struct rtps_rx_out {
  uint8_t* status;          /* [n]            required */
  rtps_record* records;     /* [max_records]  required */
  uint64_t max_records;
  uint32_t* target;         /* [max_records]  optional: target set of the record or RTPS_NO_TARGET */
  uint32_t* rec_begin;      /* [n]            optional: index of datagram i's first record */
  uint64_t* n_records;      /* [1]            required: total records of the batch */
} rtps_rx_out;

typedef struct rtps_rx_ctx rtps_rx_ctx;

/* error codes (negative) */
#define RTPS_RX_OK 0
#define RTPS_RX_EINVAL (-1)
#define RTPS_RX_EHIP (-2)
#define RTPS_RX_ENOMEM (-3)
#define RTPS_RX_ETOOBIG (-4)
#define RTPS_RX_EABI (-5)
#define RTPS_RX_EABORTED (-6) /* the RCCL communicator was aborted (and freed) after a failed
                                 group: forget the handle, do not destroy it, make a new one */

/* MessageReceiver::new(participant_guid_prefix, None)  (message_receiver.rs:158-182) */
int rtps_rx_create(const rtps_rx_config* cfg, rtps_rx_ctx** out_ctx);
int rtps_rx_destroy(rtps_rx_ctx* ctx);
/* Launch on the caller's hipStream_t.  NULL = the HIP null (default)
 * stream; RTPS_RX_OWN_STREAM = the context's own non-blocking stream
 * (the default after rtps_rx_create). */
#define RTPS_RX_OWN_STREAM ((void*)(intptr_t)-1)
int rtps_rx_set_stream(rtps_rx_ctx* ctx, void* hip_stream);
/* Replace the local readers and their writer proxies (Domain registration +
 * Reader::matched_writer_add).  RTPS_RX_EINVAL for a repeated reader entity id,
 * a repeated (reader, writer GUID) proxy or a reader index out of range.
 * Ingest state is kept per proxy index (see rtps_rx_ingest). */
int rtps_rx_set_readers(rtps_rx_ctx* ctx, const rtps_reader* readers, uint32_t n_readers,
                        const rtps_proxy* proxies, uint32_t n_proxies);
/* Compatibility form of rtps_rx_set_readers (see rtps_match): proxy i = the
 * i-th distinct (writer GUID, slot) pair. */
int rtps_rx_set_match_table(rtps_rx_ctx* ctx, const rtps_match* table, uint32_t n);
/* Host view of the current target sets: set t lists entries[first[t] .. first[t+1]).
 * Valid until the next set_readers / set_match_table. */
int rtps_rx_target_table(const rtps_rx_ctx* ctx, const uint32_t** first, const rtps_target** entries,
                         uint32_t* n_sets);
/* Parse n datagrams: datagram i = arena[dgram_off[i] .. dgram_off[i]+dgram_len[i]).
 * arena, dgram_off, dgram_len are DEVICE pointers.  Asynchronous on the
 * context's stream; call rtps_rx_sync (or synchronise the stream) before
 * reading the outputs. */
int rtps_rx_parse_batch(rtps_rx_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* dgram_off, const uint32_t* dgram_len, uint32_t n,
                        const rtps_rx_out* out);
int rtps_rx_sync(rtps_rx_ctx* ctx);
/* Performance hint: the number of records most datagrams of the coming
 * batches produce (default 1: one DATA per datagram; 2 for INFO_TS+DATA).
 * Tiles of 256 datagrams that all match it are written in a single pass;
 * any other tile costs a second walk.  When most tiles of the previous batch
 * did not match, the context switches by itself to a chained pass made for
 * mixed traffic (each tile counts, learns its exact position from its
 * predecessors, then writes); 0 selects that pass always.  Results never
 * depend on the hint. */
int rtps_rx_set_spec_hint(rtps_rx_ctx* ctx, uint32_t records_per_datagram);
const char* rtps_rx_strerror(int code);

/* Multi-GPU sharding (>= 2 GPUs): stable partition of the writer/reader-kind
 * records (interpreter records are not exchanged) by owner GPU =
 * fmix32(fnv1a32(prefix || writer_id)) % n_dest (FNV-1a over the GUID's four
 * little-endian words, then the murmur3 finaliser).
 * recs/n_records are a parse_batch output (device); out has room for
 * max_records records; dest_counts[n_dest] (device u64) receives the bucket
 * sizes; bucket d starts at sum(dest_counts[0..d)).  Input order is kept
 * inside each bucket.  New: the reference has one process and no exchange. */
int rtps_rx_bucket_by_writer(rtps_rx_ctx* ctx, const rtps_record* recs, const uint64_t* n_records,
                             uint64_t max_records, uint32_t n_dest, rtps_record* out, uint64_t* dest_counts);
/* Same partition into fixed-capacity buckets: bucket d occupies
 * out[d*cap, (d+1)*cap); records past position cap of their bucket are not
 * written (dest_counts[d] > cap tells the caller).  Lets the exchange use an
 * equal-split all-to-all whose sizes need no device-to-host round trip. */
int rtps_rx_bucket_by_writer_padded(rtps_rx_ctx* ctx, const rtps_record* recs, const uint64_t* n_records,
                                    uint64_t max_records, uint32_t n_dest, uint64_t cap, rtps_record* out,
                                    uint64_t* dest_counts);

/* Exchange descriptors (>= 2 GPUs): the compact form of a targeted writer's
 * record that crosses xGMI instead of the 64-byte record.  Only records with
 * RTPS_ROUTE_MATCHED or RTPS_ROUTE_TARGETED are exchanged (writer submessages
 * that reach some reader, with or without a proxy: what a reader's per-writer
 * state consumes, io_uring/rtps/reader.rs handle_*_msg, and the proxy-less
 * samples of non-user-defined writers it accepts, :734-739).  Owner GPU =
 * target set index % n_dest (writer sets first, in the order the proxies list
 * them, then entity sets): writers are spread round-robin, so the owners are
 * balanced whatever the GUID hash does; payloads and full records stay on the
 * source GPU (rec_idx). */
typedef struct rtps_xdesc {
  int64_t sn;            /* writer sequence number */
  uint32_t rec_idx;      /* index of the full record in the source rank's parse output */
  uint32_t writer_kind;  /* target set index << 8 | submessage kind */
} rtps_xdesc;
/* Stable partition of the targeted records' descriptors into n_dest buckets of
 * cap descriptors each (out[d*cap, (d+1)*cap)); dest_counts as in
 * rtps_rx_bucket_by_writer_padded.  Needs readers (RTPS_RX_EINVAL without). */
int rtps_rx_bucket_descriptors(rtps_rx_ctx* ctx, const rtps_record* recs, const uint64_t* n_records,
                               uint64_t max_records, uint32_t n_dest, uint64_t cap, rtps_xdesc* out,
                               uint64_t* dest_counts);

/* ---- the exchange over RCCL (>= 2 GPUs) -------------------
 * One process (rank) per GPU; the communicator is an RCCL ncclComm_t passed as
 * void*: create it with rtps_rx_exchange_unique_id on one rank, an out-of-band
 * broadcast of the 128 bytes (the host's own control channel), and
 * rtps_rx_exchange_comm_init on every rank; or pass a ncclComm_t the host
 * already has.  New: the reference has one process and no collective. */
#define RTPS_RX_EXCHANGE_ID_BYTES 128
int rtps_rx_exchange_unique_id(uint8_t id[RTPS_RX_EXCHANGE_ID_BYTES]);
int rtps_rx_exchange_comm_init(const uint8_t id[RTPS_RX_EXCHANGE_ID_BYTES], int n_ranks, int rank, int device,
                               void** comm);
int rtps_rx_exchange_comm_destroy(void* comm);
/* Equal-split all-to-all of fixed-capacity buckets (the output of
 * rtps_rx_bucket_by_writer_padded or rtps_rx_bucket_descriptors): bucket d
 * (send + d*cap*item_bytes) goes to rank d, rank s's bucket for this rank lands
 * at recv + s*cap*item_bytes; the true bucket sizes travel alongside
 * (send_counts[n_ranks] -> recv_counts[n_ranks], device u64; a size > cap means
 * that bucket overflowed).  One ncclGroupStart/End of ncclSend/ncclRecv per
 * peer on hip_stream (NULL: the context's stream; a separate stream lets the
 * exchange of batch k overlap the parse of batch k+1): asynchronous, no host
 * round trip. */
int rtps_rx_exchange(rtps_rx_ctx* ctx, void* comm, void* hip_stream, const void* send, const uint64_t* send_counts,
                     uint64_t cap, uint32_t item_bytes, void* recv, uint64_t* recv_counts);

/* ---- owner-side exchange: what a writer's owner GPU consumes (>= 2 GPUs) ----
 * The per-writer state of the receive path (fragment assembly and the writer
 * proxies: io_uring/rtps/reader.rs:563-758, rtps/rtps_writer_proxy.rs:202-355,
 * structure/dds_cache.rs:241-252) is only right where ALL of a writer's
 * submessages meet: on its owner GPU.  rtps_rx_shard_* move there every record
 * that state consumes, so that the owner runs rtps_rx_frag_assemble and
 * rtps_rx_ingest as one GPU would on the whole stream:
 *   - items: every writer-kind record that passes (RTPS_ROUTE_PASS: DATA,
 *     DATA_FRAG, HEARTBEAT, HEARTBEAT_FRAG, GAP), owner = the writer's owner in the
 *     shard's owner table (rtps_rx_shard_set_owners below; default: the context's
 *     writers dealt evenly), else fmix32(fnv1a32(prefix || writer_id)) % n_ranks.
 *     What crosses is a 16-byte rtps_shard_item per record and a "blob".  A DATA
 *     of a writer in the shard's writer list (the owner table's writer GUIDs in
 *     ascending byte order; every rank builds the same table) whose SN's high word
 *     is 0..255 is its item alone ("compact": the writer's list index, the SN,
 *     kind, flags, route, payload kind: what the owner's ingest reads; its payload
 *     stays on the source GPU, zero-copy, and `origin` names the record there); any
 *     other DATA sends its writer GUID and SN in a 32-byte blob; any other kind
 *     sends its whole 64-byte record in the blob, followed by the arena bytes the
 *     owner's consumers read (a GAP's bitmap words, a DATA_FRAG's payload), 16-byte
 *     aligned;
 *   - order: rank r parses the r-th contiguous chunk of the stream, so the
 *     records an owner receives, concatenated in source-rank order, are its
 *     writers' records in stream order;
 *   - capacity: round 0 moves fixed slots (cap records and bcap blob bytes per
 *     peer: equal splits, no host round trip).  A source's records past its slot
 *     go in a second round of exact size (the spill) once the host has read the
 *     counts, so nothing is dropped whatever the traffic mix.
 * Sequence per batch: rtps_rx_parse_batch, rtps_rx_shard_pack (context stream),
 * rtps_rx_shard_exchange (round 0, asynchronous), rtps_rx_shard_finish (waits
 * for the counts; spill round if needed), rtps_rx_shard_unpack -> an owner batch
 * for rtps_rx_frag_assemble / rtps_rx_ingest on the same context.
 * New: the reference has one process and no exchange. */
typedef struct rtps_shard rtps_shard;
typedef struct rtps_shard_item {  /* one exchanged writer record (16 bytes) */
  uint32_t w0;         /* compact DATA: 1 | the writer's list index << 4 (< 2^20) | the SN's high word << 24;
                          else the item's blob bytes (a multiple of 16: the low nibble tells them apart):
                          32 for a DATA (its writer GUID, SN, 8 zero bytes), else 64 + its consumers'
                          bytes rounded to 16 (its record, dgram_idx = src_rec, then those bytes) */
  uint32_t src_rec;    /* the record's index in the source rank's parse output */
  uint32_t sn_lo;      /* compact DATA: the SN's low word; else 0 */
  uint8_t kind, flags, route, payload_kind;
} rtps_shard_item;
RTPS_RX_STATIC_ASSERT(sizeof(rtps_shard_item) == 16, "rtps_shard_item must be 16 bytes");
#define RTPS_SHARD_COMPACT 0x1u  /* rtps_shard_item.w0 & 0xf: a compact DATA */
typedef struct rtps_shard_counts {  /* one (source, destination) pair */
  uint64_t n;          /* items */
  uint64_t bytes;      /* blob bytes (multiple of 16) */
  uint64_t cut;        /* items in the fixed slot: the first `cut` (the rest is spill) */
  uint64_t cut_bytes;  /* blob bytes of those items */
} rtps_shard_counts;
#define RTPS_SHARD_LEAD 65536u  /* zero bytes ahead of the owner arena's blobs */
typedef struct rtps_owner_batch {  /* DEVICE pointers owned by the shard, valid until its next unpack */
  const uint8_t* arena;            /* RTPS_SHARD_LEAD zero bytes, then the received blobs */
  uint64_t arena_len;
  const uint64_t* dgram_off;       /* [n_records]: record i's dgram_idx is i, its blob is at
                                      arena + dgram_off[i] + (u.gap.bitmap_off | u.frag.pl_off) */
  const rtps_record* records;      /* [n_records], stream order; every field as parsed except dgram_idx,
                                      for a DATA only kind, flags, route, payload_kind, the writer GUID
                                      and sn (the rest stays at its origin) */
  const uint64_t* origin;          /* [n_records]: source rank << 32 | the record's index in the source
                                      rank's parse output */
  const uint64_t* n_records_dev;   /* device u64 (for the consumers' n_records argument) */
  uint64_t n_records;              /* host copy */
} rtps_owner_batch;
/* cap: items per peer slot (>= 1); bcap: blob bytes per peer slot (a multiple of 16). */
int rtps_rx_shard_create(rtps_rx_ctx* ctx, uint32_t n_ranks, uint64_t cap, uint64_t bcap, rtps_shard** out);
int rtps_rx_shard_destroy(rtps_shard* s);
/* Source side: partition this rank's parse output by owner into the fixed slots and
 * the spill, with the blobs (asynchronous on the context's stream). */
int rtps_rx_shard_pack(rtps_shard* s, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                       const rtps_record* records, const uint64_t* n_records, uint64_t max_records);
/* Round 0 over RCCL (comm as for rtps_rx_exchange): one ncclGroupStart/End of, per peer,
 * the counts, the record slot and the blob slot, on hip_stream (NULL: the context's
 * stream), after the pack; then the counts are copied to the host.  Asynchronous. */
int rtps_rx_shard_exchange(rtps_shard* s, void* comm, void* hip_stream);
/* Waits for round 0's counts; if any pair overflowed its slot, moves the spill in a
 * second group of exact sizes (both ends know them from the counts).  Every failure
 * of rtps_rx_shard_finish, and a failed group in rtps_rx_shard_exchange /
 * rtps_rx_exchange, aborts the communicator (RTPS_RX_EABORTED): it is freed, and the
 * peers' pending operations fail instead of waiting forever.  rtps_rx_shard_unpack
 * refuses (RTPS_RX_EINVAL) a batch with a spill that rtps_rx_shard_finish did not move. */
int rtps_rx_shard_finish(rtps_shard* s, void* comm, void* hip_stream);
/* Owner side: every received record as one batch (reads the received counts: a host sync). */
int rtps_rx_shard_unpack(rtps_shard* s, rtps_owner_batch* out);
/* The same protocol over a host-driven transport (e.g. gloo): the buffers round 0
 * moves and the spill areas.  Spill layouts: send side, destination d's records at
 * sum_{d' < d} n_d' and its bytes at sum_{d' < d} bytes_d' (the spilled ones are
 * [cut, n) / [cut_bytes, bytes) of that range); receive side, source s's spilled
 * records at sum_{s' < s} (n - cut), its bytes at sum_{s' < s} (bytes - cut_bytes). */
typedef struct rtps_shard_buffers {
  void* send_slots;        /* [n_ranks * cap] rtps_shard_item; peer d's slot at d * cap */
  void* send_blob;         /* [n_ranks * bcap] */
  void* send_counts;       /* [n_ranks] rtps_shard_counts */
  void* recv_slots;
  void* recv_blob;
  void* recv_counts;
  void* send_spill;
  void* send_blob_spill;
  void* recv_spill;
  void* recv_blob_spill;
  uint64_t recv_spill_cap;       /* items */
  uint64_t recv_blob_spill_cap;  /* bytes */
} rtps_shard_buffers;
int rtps_rx_shard_buffers(rtps_shard* s, rtps_shard_buffers* out);
/* Grow the receive spill to hold `records` records and `bytes` blob bytes. */
int rtps_rx_shard_reserve_spill(rtps_shard* s, uint64_t records, uint64_t bytes);

/* Writer -> owner assignment of the items.  An owner's step time follows its busiest
 * owner, and a hash of few writers leaves owners unequal (16 writers over 8 ranks: one
 * idle, one with 1.5x the mean), so the shard keeps a table of the context's writers
 * (the writer GUIDs of its proxies) dealt over the ranks; a writer not in it goes by
 * fmix32(fnv1a32(GUID)) % n_ranks.  Every rank must make the same calls (readers, topics,
 * set_owners, packs) in the same order: the deal is a function of them alone (not of the
 * order inside a table).
 *   RTPS_OWNER_BALANCED  every writer its own group (the default while no topic is set);
 *   RTPS_OWNER_TOPIC     writers whose target readers share a topic cache (a topic of
 *     rtps_rx_set_topics, or a reader's own cache) are one group, so one owner holds
 *     all of a TopicCache's changes, as RTPS_INGEST_TOPIC_CACHE on owner batches needs (the
 *     cache's GC spans its writers, dds_cache.rs:367-420).  The group also holds an ENTITY
 *     KEY per entity id that a reader contains (0xff x 12 || entity id): a writer without a
 *     proxy that reaches the topic by entity id (rt_classify's entity sets) goes to that
 *     group's owner.  The default once rtps_rx_set_topics has configured a topic, unless
 *     set_owners chose a mode;
 *   RTPS_OWNER_HASH      no table (every writer by the hash).
 * rtps_rx_ingest refuses RTPS_INGEST_TOPIC_CACHE (RTPS_RX_EINVAL) on a context with a
 * shard of >= 2 ranks in another mode: its topic caches would diverge.
 * The table is STICKY: when the readers or topics change, the next pack (re)builds it,
 * and every writer the previous table held keeps its owner (its writer proxy, far set,
 * DataFrag assemblies and topic-cache changes live there); new writers are dealt onto the
 * ranks' loads.  Only a topic group that comes to join writers of different owners moves
 * the smaller part to the owner holding most of its weight: those writers' state stays
 * behind on the old owner (as after rtps_rx_ingest_reset there).  set_owners deals afresh
 * (an explicit rebalance with the same state caveat for every writer that moves).
 * Groups are dealt by total weight, largest first, each to the least-loaded owner (ties:
 * the group's smallest GUID, the lowest rank); equal weights deal the sorted GUIDs
 * round-robin.  guids[n][16] / weights[n] (optional): weights of writers (e.g. their
 * records in the previous batches); a listed writer the context does not know joins
 * the table as a group of its own; unlisted writers weigh 1. */
#define RTPS_OWNER_BALANCED 0u
#define RTPS_OWNER_HASH 1u
#define RTPS_OWNER_TOPIC 2u
int rtps_rx_shard_set_owners(rtps_shard* s, uint32_t mode, const uint8_t* guids, const uint64_t* weights,
                             uint32_t n);
/* The owner rank of a writer GUID under the shard's current assignment (host; a table the
 * next pack would rebuild is answered from that rebuild, without committing it), or a
 * negative RTPS_RX_* code. */
int rtps_rx_shard_owner(rtps_shard* s, const uint8_t guid[16]);
/* The deal itself, on the host (no GPU): writers[n][16], weights[n] (NULL: 1 each),
 * groups[n] (NULL: every writer its own; else writer w is in group groups[w] < n) ->
 * owners[n] < n_ranks. */
int rtps_rx_owner_assign(const uint8_t* writers, const uint64_t* weights, const uint32_t* groups, uint32_t n,
                         uint32_t n_ranks, uint32_t* owners);
/* The sticky deal: prev[n] (NULL: none) = each writer's owner in the previous table, or -1
 * for a new one.  A group with owned members goes to the rank holding most of their weight
 * (each owned member counts weight + 1; ties: the lowest rank), and the other groups are
 * dealt as above onto the loads those leave. */
int rtps_rx_owner_assign_sticky(const uint8_t* writers, const uint64_t* weights, const uint32_t* groups, uint32_t n,
                                uint32_t n_ranks, const int32_t* prev, uint32_t* owners);

/* ---- batch CDR decode (a18) ----------------------------------------------
 * Replaces the per-sample decode
 *   SimpleDataReader::deserialize_with -> DA::from_bytes_with(&payload.value, rep_id, ..)
 *       io_uring/dds/with_key/simpledatareader.rs:137-160, dds/adapters.rs:128-139
 *   -> deserialize_from_cdr_with_decoder_and_rep_id   serialization/cdr_adapters.rs:246-275
 *   -> cdr_encoding::CdrDeserializer (external crate cdr-encoding 0.10)
 * The type is a "program" of ops (a struct's fields in order; nested structs
 * flatten because classic CDR aligns each primitive to its own size relative
 * to the first byte after the 4-byte encapsulation header).  Sequences and
 * arrays of non-primitive elements (strings, structs, sequences) are a
 * SEQ_BEGIN / ARRAY_BEGIN op, the element's ops, and an END op.  Every DATA
 * record with payload_kind == RTPS_PK_DATA is decoded into a row of row_bytes
 * at rows + record_index * row_bytes (host byte order). */
enum rtps_cdr_op_kind {
  RTPS_CDR_PRIM = 1,        /* size 1/2/4/8 (ints, f32, f64, unit enum = u32)                          */
  RTPS_CDR_BOOL = 2,        /* 1 byte, must be 0 or 1                                                   */
  RTPS_CDR_STRING = 3,      /* u32 length incl. NUL + bytes, UTF-8 checked; count = max chars (no NUL) */
  RTPS_CDR_SEQ = 4,         /* u32 n + n primitives of `size`; count = max elements                     */
  RTPS_CDR_ARRAY = 5,       /* count primitives of `size`, no length                                    */
  RTPS_CDR_SEQ_BEGIN = 6,   /* u32 n + n elements = the ops up to the matching END; count = max elements */
  RTPS_CDR_ARRAY_BEGIN = 7, /* count elements = the ops up to the matching END, no length               */
  RTPS_CDR_END = 8          /* closes the innermost open SEQ_BEGIN / ARRAY_BEGIN (size, count, out_off 0) */
};
/* Row layout: each op owns a slot that starts at out_off (4-aligned) and spans
 * a multiple of 4 bytes; sibling slots must not overlap and must lie inside
 * their container (the row, or one element):
 *   PRIM  align4(size)           value (host order), zero-extended
 *   BOOL  4                      byte 0 = 0/1, rest 0
 *   STRING 4 + align4(count)     u32 chars, then the chars, zero tail (no NUL)
 *   SEQ   4 + align4(size*count) u32 n, then n elements, zero tail
 *   ARRAY align4(size*count)     count elements
 *   SEQ_BEGIN   4 + count*stride u32 n, then element i at +4 + i*stride (i < n)
 *   ARRAY_BEGIN count*stride     element i at i*stride
 * The ops between a BEGIN and its END lay out ONE element: their out_off are
 * relative to the element's start and their slots lie inside [0, stride).
 * Bytes not covered by a slot (elements >= n included) are zero.  A row whose
 * decode fails is all zero.  Nesting depth <= RTPS_CDR_MAX_DEPTH.
 * A sequence longer than its slot (n > count) is RTPS_CDR_TOO_LONG once its
 * elements have been read (so a malformed element reports the reference's own
 * error); elements that occupy no wire bytes cannot fail and report it at once. */
typedef struct rtps_cdr_op {
  uint8_t kind;      /* rtps_cdr_op_kind */
  uint8_t size;      /* primitive size for PRIM / SEQ / ARRAY */
  uint16_t stride;   /* SEQ_BEGIN / ARRAY_BEGIN: row bytes per element (multiple of 4, >= 4); else 0 */
  uint32_t count;    /* STRING: max chars; SEQ / SEQ_BEGIN: max elements; ARRAY / ARRAY_BEGIN: elements */
  uint32_t out_off;  /* byte offset of the slot in the row / element (multiple of 4) */
} rtps_cdr_op;
enum rtps_cdr_status {
  RTPS_CDR_OK = 0,
  RTPS_CDR_NOT_DATA = 1,        /* record is not a DATA with payload_kind == RTPS_PK_DATA   */
  RTPS_CDR_BAD_ENCODING = 2,    /* rep id not in {CDR_BE, CDR_LE, PL_CDR_LE} (cdr_adapters.rs:96-100) */
  RTPS_CDR_EOF = 3,             /* payload ends before the type does                        */
  RTPS_CDR_BAD_BOOL = 4,        /* bool byte not 0/1                                        */
  RTPS_CDR_BAD_UTF8 = 5,        /* string bytes are not UTF-8                               */
  RTPS_CDR_TOO_LONG = 6         /* string/sequence longer than the row slot (not a reference error) */
};
#define RTPS_CDR_MAX_DEPTH 4u
#define RTPS_CDR_MAX_OPS 64u
/* prog: host array of n_ops ops (copied at the call).  arena / dgram_off: the
 * batch given to rtps_rx_parse_batch; records / n_records: its outputs.
 * rows: [max_records * row_bytes] (row_bytes a multiple of 4), row_status:
 * [max_records]; rows/statuses [0, min(*n_records, max_records)) are written.
 * Asynchronous on the context's stream.  RTPS_RX_EINVAL for a malformed program. */
int rtps_rx_cdr_decode(rtps_rx_ctx* ctx, const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes,
                       const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                       const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                       uint8_t* rows, uint8_t* row_status);
/* The same decode into COMPACT rows: row k decodes the record named by list entry k, a
 * u32 record index at list + k * list_stride (device), for k < min(*n_list, max_list):
 * e.g. the rtps_ingest_out deliveries (list = accepted, list_stride =
 * sizeof(rtps_delivery), n_list = n_accepted), so only the samples that entered a
 * history cache are decoded, as the reference decodes only the samples a DataReader
 * takes (SimpleDataReader::deserialize_with per cache change,
 * io_uring/dds/with_key/simpledatareader.rs:137-237).  A list entry naming a record
 * that is not a DATA sample (or >= min(*n_records, max_records)) gets
 * RTPS_CDR_NOT_DATA and a zero row.  list_stride: a multiple of 4, >= 4. */
int rtps_rx_cdr_decode_list(rtps_rx_ctx* ctx, const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes,
                            const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                            const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                            const void* list, uint32_t list_stride, const uint64_t* n_list, uint64_t max_list,
                            uint8_t* rows, uint8_t* row_status);

/* ---- DataFrag reassembly ---------------------------
 * Replaces the per-reader FragmentAssembler / AssemblyBuffer
 * (rtps/fragment_assembler.rs:23-214) driven by Reader::handle_datafrag_msg
 * (io_uring/rtps/reader.rs:563-636), for every DATA_FRAG record with
 * RTPS_ROUTE_PASS of a parse_batch output, in record order:
 *   - per writer GUID the fragment size is the one of its first DATA_FRAG ever
 *     (FragmentAssembler::new :163-169, reader.rs:638-647);
 *   - per (writer GUID, SN) an assembly buffer of data_size bytes and
 *     ceil(data_size / fragment_size) fragment bits is created from the first
 *     DATA_FRAG of that SN (AssemblyBuffer::new :35-63);
 *   - each DATA_FRAG copies min(frags_in_submessage * F, payload length) bytes
 *     to (fragment_starting_num - 1) * F, clamped to the buffer, and sets its
 *     fragment bits (insert_frags :65-140);
 *   - when every bit is set the sample is emitted and the buffer dropped
 *     (new_datafrag :172-214, is_complete :142-144).
 * With readers set (rtps_rx_set_readers), every reader has its own assembler per
 * writer, as every Reader has its own FragmentAssembler per writer GUID
 * (reader.rs:617-619, 638-647): a DATA_FRAG record is assembled once for every
 * reader of its target set (records that are a builtin pair or reach no reader are
 * not assembled: Discovery2 / nobody takes them), the fragment size is the one of
 * that reader's first DATA_FRAG of the writer, and a reader whose Lifespan
 * (rtps_rx_set_reader_lifespan) has expired for the record's source timestamp
 * skips it (handle_datafrag_msg :578-589).  A reader added later starts with no
 * buffers; the others keep theirs.  Without readers, one assembler per writer
 * takes every DATA_FRAG that passes (the form the reader-less tests use).
 * State (fragment sizes, incomplete buffers) persists in the context
 * across batches.  Completed samples are emitted in completing-record order
 * (then target-set order), each with the reader whose assembler completed it;
 * their SerializedPayload bytes (incl. the 4-byte encapsulation) are written
 * back to back (16-byte aligned) into `heap`.  Inputs the reference rejects
 * by panicking (fragment bits past the buffer's count, byte ranges past its
 * end) are clamped here. */
typedef struct rtps_frag_sample {
  uint8_t writer_guid[16]; /* source prefix || writer_id */
  int64_t sn;
  uint64_t heap_off;       /* offset of the sample bytes in the heap */
  uint32_t data_size;      /* bytes of the SerializedPayload (incl. encapsulation) */
  uint32_t rec_idx;        /* record (of this batch) that completed the sample */
  uint8_t flags;           /* DATA_FRAG flags of the completing record (0x04 Key: dispose by key) */
  uint8_t status;          /* rtps_frag_status */
  uint16_t reader_slot;    /* the reader whose assembler completed it; RTPS_NO_MATCH (no readers set):
                              every reader of the completing record's target set */
  uint32_t _r2;
} rtps_frag_sample;
enum rtps_frag_status {
  RTPS_FRAG_OK = 0,
  RTPS_FRAG_SHORT = 1,     /* data_size < 4: SerializedPayload::from_bytes fails, no DDSData (:189-198) */
  RTPS_FRAG_NO_ROOM = 2    /* heap too small: descriptor only, bytes not written */
};
typedef struct rtps_frag_out {
  rtps_frag_sample* samples; /* [max_samples] */
  uint64_t max_samples;
  uint8_t* heap;             /* [heap_bytes] */
  uint64_t heap_bytes;
  uint64_t* n_samples;       /* device u64: completed samples (may exceed max_samples) */
  uint64_t* heap_used;       /* device u64: bytes the samples need */
  uint64_t* n_pending;       /* device u64: incomplete buffers carried to the next batch */
} rtps_frag_out;
/* Assemble one parsed batch (asynchronous).  arena / dgram_off / records /
 * n_records / max_records: the batch and its parse_batch output. */
int rtps_rx_frag_assemble(rtps_rx_ctx* ctx, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                          const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                          const rtps_frag_out* out);
/* Drop every incomplete buffer and the writer fragment sizes (a new reader). */
int rtps_rx_frag_reset(rtps_rx_ctx* ctx);
/* Assembly-buffer expiry (FragmentAssembler::garbage_collect_before,
 * fragment_assembler.rs:216-224, called by the reader with now - expiry,
 * reader.rs:1338-1340).  set_clock: the time (ns; any monotonic u64 clock) the
 * next batches stamp on every buffer they create or extend (AssemblyBuffer::
 * modified_time :54-61, :139).  gc: drop the incomplete buffers last modified
 * before expire_before_ns (asynchronous); *n_pending (device u64) = the buffers
 * left.  A dropped (writer, SN) that receives fragments later starts a new
 * buffer, as in the reference. */
int rtps_rx_frag_set_clock(rtps_rx_ctx* ctx, uint64_t now_ns);
int rtps_rx_frag_gc(rtps_rx_ctx* ctx, uint64_t expire_before_ns, uint64_t* n_pending);
/* Lifespan QoS of a reader (by reader_slot) for the DataFrag assembly: a DATA_FRAG
 * whose source timestamp is older than the receive time by more than the lifespan
 * is dropped for that reader (reader.rs:578-589, Duration/Timestamp tick arithmetic,
 * structure/time.rs:85-113).  lifespan_ns < 0: none (the default). */
int rtps_rx_set_reader_lifespan(rtps_rx_ctx* ctx, uint16_t reader_slot, int64_t lifespan_ns);
/* The receive time (Timestamp::now(), ns since the UNIX epoch) the next batches'
 * Lifespan checks use; 0 (the default): the host's clock at each assemble call. */
int rtps_rx_frag_set_receive_time(rtps_rx_ctx* ctx, uint64_t unix_ns);

/* ---- history-cache ingest ---------------------------
 * Replaces, for every target reader of every routed writer submessage, the
 * writer-proxy bookkeeping that decides which samples enter that reader's
 * history cache:
 *   Reader::handle_data_msg -> process_received_data      io_uring/rtps/reader.rs:514-561, 693-758
 *     RtpsWriterProxy::should_ignore_change, received_changes_add, advance_ack_base
 *                                                         rtps/rtps_writer_proxy.rs:202-224, 338-355
 *   Reader::handle_datafrag_msg, completed samples        reader.rs:563-636
 *   Reader::handle_heartbeat_msg (Reliable readers only): count check, then
 *     irrelevant_changes_up_to(first_sn)                  reader.rs:859-917, rtps_writer_proxy.rs:241-292
 *   Reader::handle_gap_msg: gapStart > 0 and gapList.base > 0, then
 *     irrelevant_changes_range(gapStart, gapList.base) and set_irrelevant_change
 *     for every listed SN                                 reader.rs:1060-1116, rtps_writer_proxy.rs:226-239
 *   TopicCache::add_change (flags & RTPS_INGEST_TOPIC_CACHE: see below)
 *                                                         structure/dds_cache.rs:210-284
 * Events are the records of a parse_batch output with RTPS_ROUTE_PASS, in
 * record order, delivered to every reader of their target set in set order
 * (dp_event_loop.rs:272-326): DATA with payload_kind DATA / KEY / KEY_HASH and
 * completed DataFrag samples (status != RTPS_FRAG_SHORT, placed at their
 * completing record) are samples; HEARTBEAT and GAP update the proxy's state.
 * For one (record, target reader):
 *   - a sample with a proxy enters the reader's cache iff the proxy does not
 *     ignore it: sn >= all_ackable_before and sn not in the proxy's change set
 *     (received or irrelevant), or always for a RTPS_TARGET_DUPLICATES_OK
 *     reader (process_received_data, reader.rs:693-733);
 *   - a sample without a proxy enters iff the writer's entity kind is not
 *     user-defined (kind & 0xF0 != 0, reader.rs:734-739; guid.rs:168-170);
 *   - a completed DataFrag sample goes only to the reader whose assembler
 *     completed it (rtps_frag_sample.reader_slot; RTPS_NO_MATCH: every reader of
 *     the record's target set); at most 64 readers per target set take such samples;
 *   - HEARTBEAT / GAP without a proxy, HEARTBEAT for a BestEffort reader: no
 *     effect (reader.rs:871-891, 1071-1086).
 * Every accepted (record, reader) pair is one delivery: process_received_data
 * returned true (reader.rs:693-758), so Domain::handle_event calls on_read for a
 * DATA (dp_event_loop.rs:284-299) and the reader hands the change to its topic's
 * TopicCache::add_change (make_cache_change, reader.rs:1185-1205).  Whether that
 * add_change STORES it is the topic cache's own duplicate check, which this call
 * decides too when flags has RTPS_INGEST_TOPIC_CACHE: the delivery's
 * RTPS_DELIVERY_CACHED flag (see "topic caches" below).  State per proxy
 * (all_ackable_before, the change set above it, received_heartbeat_count)
 * persists in the context across batches; it is indexed by proxy position, so
 * keep proxies in place (append new ones) or call rtps_rx_ingest_reset after
 * reordering them.
 * The change set is a bitmap over RTPS_INGEST_WINDOW sequence numbers from
 * all_ackable_before plus, per proxy, a FAR SET: every covered SN beyond that window
 * (samples and GAPs further ahead), a hash set in device memory that grows with it
 * (no fixed bound; a batch may add any number of far SNs to any proxy), decided
 * exactly by first cover (all_ackable_before continues through the set).  Before
 * a batch's far samples are decided the context makes room in its pool for
 * 8 x (the batch's far candidates + 256 per GAP + 2^16) + twice the far-set slots
 * in use, growing the pool between batches (on the per-proxy path without a count
 * read-back: from the previous batch's far items).  A GAP whose range starts at or
 * below all_ackable_before only moves it (a threshold, as the reference's
 * irrelevant_changes_range does), whatever its length.  Only a batch whose other
 * GAPs cover more SNs beyond the window than that room finds it full, and then those proxies' far
 * samples are accepted without the duplicate check and counted in
 * *n_window_overflow (the reference's BTreeMap inserts such a range SN by SN). */
#define RTPS_INGEST_WINDOW (1u << 17)
#define RTPS_INGEST_BEST_EFFORT 0x1u /* flags: treat every reader as BestEffort (HEARTBEATs ignored) */
#define RTPS_INGEST_TOPIC_CACHE 0x2u /* flags: also run the topic caches' add_change (RTPS_DELIVERY_CACHED) */
typedef struct rtps_delivery {  /* one sample a reader accepted (process_received_data == true) */
  uint32_t rec_idx;             /* the record (completing record of a DataFrag sample) */
  uint16_t reader_slot;
  uint16_t flags;               /* RTPS_DELIVERY_*; 0 without RTPS_INGEST_TOPIC_CACHE */
} rtps_delivery;
/* TopicCache::add_change stored the change: its (writer GUID, SN) was not in the topic's
 * cache (find_by_sn missed, structure/dds_cache.rs:241-276) */
#define RTPS_DELIVERY_CACHED 0x1u
typedef struct rtps_ingest_out {
  uint8_t* accept;              /* [max_records] device: readers whose cache the record's sample enters
                                   (saturating at 255); 0 = none */
  rtps_delivery* accepted;      /* [max_accepted] device: deliveries, ascending (record, set order) */
  uint64_t max_accepted;        /* deliveries past it are counted but not written */
  uint64_t* n_accepted;         /* device u64: deliveries of the batch */
  int64_t* ack_base;            /* device, optional: all_ackable_before() of every proxy after the batch */
  uint64_t* n_window_overflow;  /* device u64, optional */
} rtps_ingest_out;
/* arena / dgram_off / records / n_records / max_records: the batch and its
 * parse_batch output (GAP bitmaps are read from the arena).  frag / n_frag /
 * max_frag: optional rtps_rx_frag_assemble output of the same batch (device;
 * NULL = none).  Asynchronous on the context's stream; needs readers. */
int rtps_rx_ingest(rtps_rx_ctx* ctx, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                   const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                   const rtps_frag_sample* frag, const uint64_t* n_frag, uint64_t max_frag, uint32_t flags,
                   const rtps_ingest_out* out);
/* Forget every writer proxy's state (all_ackable_before = 1, empty change set, count 0),
 * as re-created RtpsWriterProxy entries start (rtps_writer_proxy.rs:62-90).  The topic
 * caches keep their changes, as the reference's TopicCache outlives its readers' proxies:
 * a re-sent (writer GUID, SN) that a fresh proxy accepts is still dropped by add_change's
 * find_by_sn while the topic holds it (dds_cache.rs:241-276).  rtps_rx_topic_reset empties
 * the caches. */
int rtps_rx_ingest_reset(rtps_rx_ctx* ctx);

/* ---- topic caches (TopicCache::add_change, structure/dds_cache.rs:113-420) ----
 * A reader hands every change it accepts to its topic's TopicCache (one per topic
 * name, shared by every reader of the topic: DDSCache, io_uring/dds/cache.rs:10-41),
 * whose add_change
 *   1. garbage-collects first when the change's SN is a multiple of 64
 *      (add_change_internal :230-238 -> remove_changes_before(ZERO) :367-420):
 *      the oldest changes (receive-instant order = insertion order) are removed
 *      until at most max_keep_samples remain;
 *   2. drops the change if the topic already holds (writer GUID, SN) (find_by_sn
 *      :241-252, 270-276), else stores it.
 * max_keep_samples = max(ResourceLimits.max_samples (default 64), KeepLast depth)
 * over the topic's QoS, and at least 1 (update_keep_limits :165-197).  A reader slot
 * without a topic here has a topic cache of its own with max_keep_samples 64 (the
 * reference's defaults).  The periodic DDSCache::garbage_collect (the CacheCleaning
 * timer, io_uring/rtps/dp_event_loop.rs:385-389, io_uring/dds/cache.rs:43-51) is
 * rtps_rx_topic_gc.  Set the topics before the readers receive traffic: setting them
 * empties every topic cache.  A batch whose ingest overflowed its capacities
 * (*n_window_overflow > 0: samples accepted without the duplicate check) has every delivery
 * checked against its topic's live changes, so CACHED stays add_change's answer for the
 * deliveries made.  Owner batches (rtps_rx_shard_*): a topic cache's GC spans all of its
 * writers, so its changes must all meet on one owner: RTPS_OWNER_TOPIC (the shard's default
 * once topics are set; the ingest refuses the topic caches under another mode). */
typedef struct rtps_topic {
  uint32_t topic;             /* caller-defined topic id */
  uint32_t max_keep_samples;  /* >= 1 */
} rtps_topic;
typedef struct rtps_topic_reader {
  uint16_t reader_slot;       /* a reader (rtps_reader.reader_slot) ... */
  uint16_t _r;
  uint32_t topic;             /* ... of this topic (one of topics[].topic) */
} rtps_topic_reader;
int rtps_rx_set_topics(rtps_rx_ctx* ctx, const rtps_topic* topics, uint32_t n_topics,
                       const rtps_topic_reader* readers, uint32_t n_readers);
/* DDSCache::garbage_collect: every topic cache trimmed to its max_keep_samples
 * newest changes (asynchronous). */
int rtps_rx_topic_gc(rtps_rx_ctx* ctx);
/* Empty every topic cache (a new DDSCache); the writer proxies keep their state. */
int rtps_rx_topic_reset(rtps_rx_ctx* ctx);

/* ---- UDP batch receive into a datagram arena -----
 * Replaces the receive side of the reference: a UDPListener per locator with
 * an io_uring RecvMulti (multishot recv) on a provided-buffer ring of
 * 128 x 64 KiB (io_uring/network/udp_listener.rs:7-27, 101-209), whose
 * completions Domain::handle_event copies out one at a time
 * (io_uring/rtps/dp_event_loop.rs:190-211: Bytes::copy_from_slice, then
 * handle_received_packet_2).  Here the provided buffers are the slots of a
 * caller-owned arena (pinned host memory that the GPU parses zero-copy, or
 * copies to HBM): the kernel writes each datagram straight into its slot and
 * a batch is a list of (arena offset, length) pairs ready for
 * rtps_rx_parse_batch, with no per-datagram copy.  A batch's slots stay out
 * of the receive pool until released.  Backend: io_uring multishot recv on a
 * registered buffer ring (IORING_REGISTER_PBUF_RING); where io_uring is not
 * available (seccomp, old kernel) the same slots are filled with recvmmsg.
 * Host-side code: no GPU is involved. */
#define RTPS_UDP_REUSE 0x1u          /* SO_REUSEADDR + SO_REUSEPORT (udp_listener.rs:41-51)      */
#define RTPS_UDP_FORCE_RECVMMSG 0x2u /* do not try io_uring                                      */
#define RTPS_UDP_SQPOLL 0x4u         /* io_uring with a kernel poll thread (IORING_SETUP_SQPOLL): the
                                       kernel keeps landing datagrams in slots while the host is busy;
                                       falls back to a plain ring where it is refused              */
enum rtps_udp_backend { RTPS_UDP_IO_URING = 1, RTPS_UDP_RECVMMSG = 2, RTPS_UDP_IO_URING_SQPOLL = 3 };
typedef struct rtps_udp_config {
  uint32_t abi_version;      /* RTPS_RX_ABI_VERSION */
  uint32_t ipv4_addr;        /* bind address, host byte order (0 = INADDR_ANY) */
  uint16_t port;             /* 0 = ephemeral (rtps_udp_port) */
  uint16_t flags;            /* RTPS_UDP_* */
  uint32_t multicast_group;  /* host byte order, 0 = none (joined on INADDR_ANY) */
  uint8_t* arena;            /* caller memory of slot_bytes * n_slots bytes */
  uint32_t slot_bytes;       /* bytes per datagram slot: multiple of 16, 32..65536 */
  uint32_t n_slots;          /* power of two, 2..32768 */
  uint32_t rcvbuf_bytes;     /* SO_RCVBUF request, 0 = system default */
} rtps_udp_config;
typedef struct rtps_udp_rx rtps_udp_rx;
int rtps_udp_open(const rtps_udp_config* cfg, rtps_udp_rx** out);
int rtps_udp_close(rtps_udp_rx* rx);
int rtps_udp_port(const rtps_udp_rx* rx);     /* bound UDP port */
int rtps_udp_backend(const rtps_udp_rx* rx);  /* rtps_udp_backend */
/* Take up to max_n received datagrams, waiting up to timeout_ms for the first
 * (-1: forever, 0: poll).  off / len: host arrays of max_n, filled in arrival
 * order with arena offsets (slot * slot_bytes) and lengths.  Returns the count
 * (>= 0) or a negative RTPS_RX_* code.  *truncated (optional) += datagrams
 * longer than slot_bytes, which are dropped. */
int rtps_udp_recv_batch(rtps_udp_rx* rx, uint64_t* off, uint32_t* len, uint32_t max_n, int timeout_ms,
                        uint64_t* truncated);
/* Give the slots of n datagrams of a batch (their offsets) back to the receive pool. */
int rtps_udp_release(rtps_udp_rx* rx, const uint64_t* off, uint32_t n);
/* Loopback publisher side for tests and the C1 plumbing bench: sendmmsg of n
 * datagrams arena[off[i] .. off[i]+len[i]) to ipv4_addr:port (host order).
 * Returns datagrams sent or a negative RTPS_RX_* code. */
int rtps_udp_send_batch(uint32_t ipv4_addr, uint16_t port, const uint8_t* arena, const uint64_t* off,
                        const uint32_t* len, uint32_t n);

/* ---- native receive loop: UDP arena -> GPU parse -> ingest -> decode --------
 * Replaces the per-datagram receive loop of the reference's event loop:
 *   Domain::handle_event, Variant::DataRecv      io_uring/rtps/dp_event_loop.rs:162-211
 *     buffer_from_cqe / try_fix_err (ENOBUFS)    io_uring/discovery/traffic.rs:167-189, 246-284
 *     Bytes::copy_from_slice + handle_received_packet_2, then the reader's
 *     handle_*_msg per submessage                 dp_event_loop.rs:206-211, 266-327
 * with a batch loop on the calling thread: take every datagram that has
 * landed in the arena (up to max_batch; the first one waits up to wait_ms),
 * launch the parse (zero-copy from the arena), the history-cache ingest and
 * the CDR decode on the context's stream, then finish the PREVIOUS batch while
 * the GPU works: wait for it, hand its outputs to on_batch, give its slots
 * back to the receive pool.  Two batches are in flight at most (double-
 * buffered offsets, outputs and events).  The arena must be device-visible
 * (pinned host memory, or memory the GPU maps). */
#define RTPS_PUMP_INGEST 0x1u /* run rtps_rx_ingest on every batch (needs a match table) */
#define RTPS_PUMP_CDR 0x2u    /* run rtps_rx_cdr_decode with cdr_prog on every batch       */
typedef struct rtps_pump_buffers { /* outputs of one in-flight batch: caller-owned DEVICE memory */
  rtps_rx_out out;          /* status [max_batch]; records / match [out.max_records]; n_records */
  rtps_ingest_out ingest;   /* RTPS_PUMP_INGEST: accept / accepted [out.max_records], n_accepted */
  uint8_t* rows;            /* RTPS_PUMP_CDR: [out.max_records * cdr_row_bytes] */
  uint8_t* row_status;      /* RTPS_PUMP_CDR: [out.max_records] */
} rtps_pump_buffers;
typedef struct rtps_pump_batch {
  uint64_t seq;                  /* batch number, from 0 */
  uint32_t buffer;               /* which of the two rtps_pump_buffers holds the outputs */
  uint32_t n_datagrams;
  const uint64_t* dgram_off;     /* [n] host (pinned) arena offsets, arrival order */
  const uint32_t* dgram_len;     /* [n] */
  uint64_t n_records;            /* host copy of *out.n_records */
  uint64_t n_accepted;           /* host copy of *ingest.n_accepted (0 without ingest) */
} rtps_pump_batch;
/* Called on the pump's thread once a batch's GPU work is done, before its
 * slots are released (the arena bytes are still valid).  Non-zero: stop. */
typedef int (*rtps_pump_fn)(void* user, const rtps_pump_batch* batch);
typedef struct rtps_pump_config {
  uint32_t abi_version;        /* RTPS_RX_ABI_VERSION */
  uint32_t flags;              /* RTPS_PUMP_* */
  uint32_t max_batch;          /* datagrams per GPU batch, 1..ctx max_datagrams */
  int32_t wait_ms;             /* wait for the first datagram of a batch (>= 0) */
  uint64_t stop_after;         /* stop after this many datagrams (0 = no limit) */
  uint32_t idle_stop_ms;       /* stop after this long without a datagram (0 = no limit) */
  uint32_t ingest_flags;       /* RTPS_INGEST_* for rtps_rx_ingest */
  const rtps_cdr_op* cdr_prog; /* RTPS_PUMP_CDR: the sample type (see rtps_rx_cdr_decode) */
  uint32_t cdr_n_ops;
  uint32_t cdr_row_bytes;
  const rtps_pump_buffers* buffers; /* [2]; a batch is cut where its record bound
                                       sum((len-20)/4) would exceed out.max_records */
  rtps_pump_fn on_batch;       /* optional */
  void* user;
  const volatile uint32_t* stop; /* optional: non-zero (from any thread) stops the loop */
} rtps_pump_config;
/* Updated while the loop runs (relaxed 64-bit stores: another thread may poll
 * them, e.g. for flow control); final when rtps_rx_pump returns. */
typedef struct rtps_pump_stats {
  uint64_t datagrams;   /* received and handed to the GPU */
  uint64_t completed;   /* datagrams of finished batches (slots released) */
  uint64_t batches;
  uint64_t records;
  uint64_t accepted;
  uint64_t truncated;   /* datagrams longer than a slot (dropped by the receive) */
  uint64_t first_ns;    /* CLOCK_MONOTONIC when the first batch was received */
  uint64_t last_ns;     /* CLOCK_MONOTONIC when the last batch finished */
} rtps_pump_stats;
/* arena / arena_len: the memory given to rtps_udp_open.  Returns RTPS_RX_OK
 * when a stop condition ends the loop, or a negative code.  The batches in
 * flight are finished before it returns; datagrams already received but left
 * out of a batch by a capacity cut are dropped (their slots released) when the
 * loop stops. */
int rtps_rx_pump(rtps_rx_ctx* ctx, rtps_udp_rx* udp, const uint8_t* arena, uint64_t arena_len,
                 const rtps_pump_config* cfg, rtps_pump_stats* stats);

/* Upper bound on records for datagram lengths (host arrays): sum((len-20)/4). */
uint64_t rtps_rx_max_records_host(const uint32_t* dgram_len, uint32_t n);

/* ---- synthetic workload generator (device) ------------------------------
 * Deterministic f(seed, idx) datagrams shaped like MessageBuilder output
 * (src/rtps/message.rs:146-562, io_uring/rtps/writer.rs:681-893).
 * workload: RTPS_WL_* ; dgram_off/dgram_len are DEVICE arrays already filled
 * (rtps_gen_layout_host computes them). */
enum rtps_workload {
  RTPS_WL_C2 = 2,   /* 1M x 300 B, one DATA each, 256 B CDR payload             */
  RTPS_WL_T = 1,    /* 1M x 1024 B, one DATA each (north-star target)            */
  RTPS_WL_C3 = 3,   /* mixed DATA/HB/ACKNACK/GAP/INFO_*, 128..1500 B, 16 writers  */
  RTPS_WL_C4 = 4    /* DATA_FRAG: 64 KiB samples in 1400 B datagrams, 16 writers */
};
int rtps_rx_generate(rtps_rx_ctx* ctx, int workload, uint64_t seed, uint64_t first_idx,
                     uint32_t n_writers, uint8_t* arena, const uint64_t* dgram_off,
                     const uint32_t* dgram_len, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* RTPS_RX_H */
