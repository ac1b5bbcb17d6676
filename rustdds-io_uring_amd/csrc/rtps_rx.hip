// rtps_rx.hip — MI355X (gfx950) RTPS receive-path parser + C ABI (include/rtps_rx.h).
//
// The parse kernels (A or C, then B: see "Ordered output" below) replace, for a
// whole batch of datagrams:
//   MessageReceiver::handle_received_packet_2      io_uring/rtps/message_receiver.rs:232-287
//   Message::read_from_buffer + Submessage::read_from_buffer
//                                                  rtps/message.rs:64-81, rtps/submessage.rs:56-295
//   the per-kind readers in src/messages/**        (data.rs:57-144, data_frag.rs:121-257, ...)
//   SubmessageIter2 interpreter + dest filter      io_uring/rtps/message_receiver.rs:56-119, 618-665
//   builtin-pair / matched-writer classification   io_uring/discovery/discovery.rs:2795-2816,3075-3095
//   Reader::data_to_dds_data payload decision      io_uring/rtps/reader.rs:760-833
//
// Layout / mapping:
//   * one LANE per datagram, 256 datagrams (4 wave64s) per workgroup "tile";
//     the submessage chain of a datagram is a serial pointer chase, so the
//     parallelism is across datagrams;
//   * the datagram bytes are never copied: each submessage is read through a
//     register window (16-B buffer loads at the submessage start, the second
//     16 B only for kinds that read them; every fixed field at a compile-time
//     offset), variable-offset fields (inline-QoS parameters, AckNack count,
//     ...) by 4-byte loads; payload bytes stay in HBM (zero-copy spans, like
//     the reference's Bytes slices);
//   * records are placed in the reference's order (ascending dgram, sub_off):
//     walk 1 counts, walk 2 writes the 64-B records at their final index,
//     speculatively (one record per datagram: kernel A), after a look-back
//     over the predecessors' counts (mixed traffic: kernel C), or after all
//     counts are known (kernel B);
//   * all arena reads go through a bounds-checked buffer resource (reads past
//     the arena return 0 and never fault).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

// the diagnostic / tuning builds that need the rejected passes (diag/mixed_passes.inc)
#if (defined(RTPS_ITEM_DIAG) || defined(RTPS_EM_STAMPS) || defined(RTPS_LDS_STAMPS)) && !defined(RTPS_DIAG_PASSES)
#define RTPS_DIAG_PASSES
#endif

#include "../../include/rtps_rx.h"
#include "rtps_gen.h"
#include "rtps_cdr.h"
#include "rtps_frag.h"
#include "rtps_ctx.h"
#include "rtps_ingest.h"
#include "rtps_readers.h"
#include "rtps_topic.h"

namespace {

constexpr uint32_t TILE = 256;  // datagrams per workgroup
constexpr uint32_t WAVES = TILE / 64;
#ifndef RTPS_WAVES_PER_SIMD
#define RTPS_WAVES_PER_SIMD 6  // 80 VGPRs, no spill; SGPR use caps a CU at 6 such workgroups anyway
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct KParams {
  const uint8_t* arena;
  uint64_t arena_len;
  const uint64_t* dgram_off;
  const uint32_t* dgram_len;
  uint32_t n;
  uint32_t own0, own1, own2;  // own GuidPrefix as 3 little-endian words
  uint8_t* status;
  rtps_record* records;
  uint64_t max_records;
  uint32_t* target_out;
  uint32_t* rec_begin;
  uint64_t* n_records;
  ReaderDev rt;               // local readers -> target sets (rt.gkeys == null: none)
  uint32_t rt_lds;            // 1: the reader tables are staged in dynamic LDS by every workgroup
  uint64_t* scratch;          // per-tile counts / prefixes (Scratch)
  uint64_t* chain;            // per-tile look-back words (chained launch only), tagged with ch_epoch
  uint32_t* mixed_out;        // pinned host [2]: tiles of the batch not uniform k_spec, tiles (launch choice)
  uint32_t ch_spin_limit;     // polls before a chained tile leaves itself to kernel B
  uint32_t ch_epoch;          // chained launch number (never 0): tags the look-back words of this launch
};

// ---------------------------------------------------------------------------
// arena access: byte offsets are relative to the lane's datagram start
// ---------------------------------------------------------------------------
struct Src {
  __amdgpu_buffer_rsrc_t rsrc;  // wave-uniform, base = arena + tile_base
  uint32_t base;                // datagram start relative to the descriptor base
  uint32_t avail;               // bytes addressable through the descriptor
};

__device__ __forceinline__ uint32_t ld_u8_raw(const Src& s, uint32_t a) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(s.rsrc, a, 0, 0);
}
// 16 bytes at datagram offset o (unaligned). Bytes past the arena read as 0.
__device__ __forceinline__ u32x4 ld16(const Src& s, uint32_t o) {
  uint32_t a = s.base + o;
  if ((uint64_t)a + 16u <= s.avail) return __builtin_amdgcn_raw_buffer_load_b128(s.rsrc, a, 0, 0);
  u32x4 r = {0u, 0u, 0u, 0u};
  for (uint32_t k = 0; k < 16; ++k) {
    uint32_t b = ((uint64_t)a + k < s.avail) ? ld_u8_raw(s, a + k) : 0u;
    r[k >> 2] |= b << (8u * (k & 3u));
  }
  return r;
}
// 4 bytes at datagram offset o (unaligned), raw wire order packed little-endian.
__device__ __forceinline__ uint32_t ld4(const Src& s, uint32_t o) {
  uint32_t a = s.base + o;
  if ((uint64_t)a + 4u <= s.avail) return __builtin_amdgcn_raw_buffer_load_b32(s.rsrc, a, 0, 0);
  uint32_t r = 0;
  for (uint32_t k = 0; k < 4; ++k)
    if ((uint64_t)a + k < s.avail) r |= ld_u8_raw(s, a + k) << (8u * k);
  return r;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// wire dword -> value in the submessage byte order
__device__ __forceinline__ uint32_t e32(uint32_t raw, bool le) { return le ? raw : bswap32(raw); }
// wire u16 stored in the low (sel=0) or high (sel=1) half of a raw dword
__device__ __forceinline__ uint32_t e16(uint32_t raw, uint32_t sel, bool le) {
  uint32_t v = (raw >> (16u * sel)) & 0xffffu;
  return le ? v : (((v & 0xffu) << 8) | (v >> 8));
}
__device__ __forceinline__ int64_t sn_of(uint32_t hi_raw, uint32_t lo_raw, bool le) {
  // SequenceNumber::read_from: i32 high, u32 low (sequence_number.rs:169-182)
  return (int64_t)(((uint64_t)(int64_t)(int32_t)e32(hi_raw, le)) << 32) + (int64_t)e32(lo_raw, le);
}

// 36-byte window at a submessage start: w[0] = header, w[1..8] = body dwords
// (the largest fixed field, DATA_FRAG sampleSize, ends at body byte 32).
struct Win {
  uint32_t w[12];
};
template <class S>
__device__ __forceinline__ void load_win(const S& s, uint32_t o, Win& W) {
  u32x4 a = ld16(s, o), b = ld16(s, o + 16);
  W.w[0] = a[0]; W.w[1] = a[1]; W.w[2] = a[2]; W.w[3] = a[3];
  W.w[4] = b[0]; W.w[5] = b[1]; W.w[6] = b[2]; W.w[7] = b[3];
  W.w[8] = ld4(s, o + 32); W.w[9] = 0; W.w[10] = 0; W.w[11] = 0;
}
// Kinds whose reader needs body bytes past 12 (window dwords 4..7): every
// per-lane gather instruction costs the texture unit about one cycle per
// active lane, so the second 16 bytes (and the DATA_FRAG sampleSize dword) are
// fetched only by the lanes that use them.  Counting (WRITE=false) needs only
// the NumberSet sizes and the DATA_FRAG fields; writing needs every fixed field.
template <bool WRITE>
__device__ __forceinline__ bool win_needs_tail(uint32_t kind) {
  const uint32_t count_mask = (1u << RTPS_GAP) | (1u << RTPS_ACKNACK) | (1u << RTPS_NACK_FRAG);
  const uint32_t write_mask = count_mask | (1u << RTPS_DATA) | (1u << RTPS_HEARTBEAT) |
                              (1u << RTPS_HEARTBEAT_FRAG) | (1u << RTPS_INFO_SRC);
  if (kind == RTPS_DATA_FRAG) return true;
  return kind < 32u && (((WRITE ? write_mask : count_mask) >> kind) & 1u);
}
template <bool WRITE, class S>
__device__ __forceinline__ void load_win_lazy(const S& s, uint32_t o, Win& W) {
  const u32x4 a = ld16(s, o);
  W.w[0] = a[0]; W.w[1] = a[1]; W.w[2] = a[2]; W.w[3] = a[3];
  const uint32_t kind = a[0] & 0xffu;
  u32x4 b = {0u, 0u, 0u, 0u};
  if (win_needs_tail<WRITE>(kind)) b = ld16(s, o + 16);
  W.w[4] = b[0]; W.w[5] = b[1]; W.w[6] = b[2]; W.w[7] = b[3];
  W.w[8] = (kind == RTPS_DATA_FRAG) ? ld4(s, o + 32) : 0u;
  W.w[9] = 0; W.w[10] = 0; W.w[11] = 0;
}
// prefetch form: header + body 0..28 (DATA_FRAG's sampleSize dword is fetched
// when the kind is known)
template <class S>
__device__ __forceinline__ void load_win_pf(const S& s, uint32_t o, Win& W) {
  const u32x4 a = ld16(s, o), b = ld16(s, o + 16);
  W.w[0] = a[0]; W.w[1] = a[1]; W.w[2] = a[2]; W.w[3] = a[3];
  W.w[4] = b[0]; W.w[5] = b[1]; W.w[6] = b[2]; W.w[7] = b[3];
  W.w[8] = 0; W.w[9] = 0; W.w[10] = 0; W.w[11] = 0;
}
// the first submessage always starts at byte 20: its window comes from the
// 64-byte head (bytes 0..64) already in registers
__device__ __forceinline__ void head_win(const uint32_t* H, Win& W) {
#pragma unroll
  for (int k = 0; k < 11; ++k) W.w[k] = H[5 + k];
  W.w[11] = 0;
}

// builtin (reader_id, writer_id) pairs; entity ids as raw little-endian-packed words
// (bytes k0 k1 k2 kind -> k0 | k1<<8 | k2<<16 | kind<<24)
__device__ __forceinline__ uint32_t eid(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t kind) {
  return k0 | (k1 << 8) | (k2 << 16) | (kind << 24);
}
// Discovery2::handle_writer_msg (io_uring/discovery/discovery.rs:2795-2816)
__device__ __forceinline__ bool builtin_writer_pair(uint32_t rid, uint32_t wid) {
  const uint32_t SEDP_PUB_W = eid(0, 0, 3, 0xc2), SEDP_PUB_R = eid(0, 0, 3, 0xc7);
  const uint32_t SEDP_TOP_W = eid(0, 0, 2, 0xc2), SEDP_TOP_R = eid(0, 0, 2, 0xc7);
  const uint32_t SEDP_SUB_W = eid(0, 0, 4, 0xc2), SEDP_SUB_R = eid(0, 0, 4, 0xc7);
  const uint32_t SPDP_W = eid(0, 1, 0, 0xc2), P2P_W = eid(0, 2, 0, 0xc2);
  if (rid == 0u)
    return wid == SEDP_PUB_W || wid == SEDP_TOP_W || wid == SPDP_W || wid == SEDP_SUB_W || wid == P2P_W;
  return (rid == SEDP_PUB_R && wid == SEDP_PUB_W) || (rid == SEDP_TOP_R && wid == SEDP_TOP_W) ||
         (rid == SEDP_SUB_R && wid == SEDP_SUB_W);
}
// Discovery2::handle_reader_submsg (discovery.rs:3075-3095): (writer_id, reader_id)
__device__ __forceinline__ bool builtin_reader_pair(uint32_t rid, uint32_t wid) {
  return (wid == eid(0, 0, 3, 0xc2) && rid == eid(0, 0, 3, 0xc7)) ||
         (wid == eid(0, 0, 2, 0xc2) && rid == eid(0, 0, 2, 0xc7)) ||
         (wid == eid(0, 0, 4, 0xc2) && rid == eid(0, 0, 4, 0xc7)) ||
         (wid == eid(0, 1, 0, 0xc2) && rid == eid(0, 1, 0, 0xc7)) ||
         (wid == eid(0, 2, 0, 0xc2) && rid == eid(0, 2, 0, 0xc7));
}

// Reader tables (rtps_readers.h) of up to RT_LDS_MAX bytes are staged in LDS
// by every parse workgroup, in dynamic shared memory sized by the launch, so
// small tables cost no occupancy; larger ones are probed in global memory (L2).
extern __shared__ u32x4 s_mt_dyn[];
__device__ __forceinline__ void mt_stage(const KParams& p) {
  if (p.rt_lds) rt_stage(p.rt, reinterpret_cast<uint32_t*>(s_mt_dyn));
}
__device__ __forceinline__ uint32_t target_lookup(const KParams& p, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                                  uint32_t& route) {
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(s_mt_dyn);
  return p.rt_lds ? rt_classify<true>(p.rt, lds, a, b, c, d, route) : rt_classify<false>(p.rt, lds, a, b, c, d, route);
}

// One record being assembled in registers (16 dwords = 64 bytes).
struct Rec {
  uint32_t d[16];
};
__device__ __forceinline__ void rec_clear(Rec& r) {
#pragma unroll
  for (int i = 0; i < 16; ++i) r.d[i] = 0u;
}
// Record stores: the output is written once and read by the next stage (or the host) well
// after the L2 has turned over, so the streaming (nontemporal) form when RTPS_NT_RECORDS.
#ifndef RTPS_NT_RECORDS
#define RTPS_NT_RECORDS 1  // T kernel 46.6 -> 43.0 us (round 5)
#endif
__device__ __forceinline__ void rec_st16(u32x4* p, const u32x4& v) {
#if RTPS_NT_RECORDS
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void rec_store(rtps_record* dst, const Rec& r) {
  u32x4* p = reinterpret_cast<u32x4*>(dst);
  rec_st16(p + 0, u32x4{r.d[0], r.d[1], r.d[2], r.d[3]});
  rec_st16(p + 1, u32x4{r.d[4], r.d[5], r.d[6], r.d[7]});
  rec_st16(p + 2, u32x4{r.d[8], r.d[9], r.d[10], r.d[11]});
  rec_st16(p + 3, u32x4{r.d[12], r.d[13], r.d[14], r.d[15]});
}

// ParameterList::read_from (elements/parameter_list.rs:79-102) over the body
// starting at body position pos; records the first KEY_HASH (16-byte value
// required, dds/key.rs:64-68), STATUS_INFO and RELATED_SAMPLE_IDENTITY values,
// and the first STATUS_INFO's flags octet (SI_ABSENT / SI_ERROR: none / shorter
// than the 4 octets StatusInfo::read_from reads, inline_qos.rs:139-147).
// Returns false on a read error.
constexpr uint32_t SI_ABSENT = 0x100u, SI_ERROR = 0x200u;
template <class S>
__device__ __forceinline__ bool param_list(const S& s, uint32_t body_off, uint32_t blen, bool le,
                                           uint32_t& pos, uint32_t& kh, uint32_t& si, uint32_t& rsi,
                                           uint32_t& si_flags) {
  bool seen_kh = false, seen_si = false, seen_rsi = false;
  for (;;) {
    if (pos + 4u > blen) return false;
    uint32_t raw = ld4(s, body_off + pos);
    uint32_t pid = e16(raw, 0, le), plen = e16(raw, 1, le);
    pos += 4u;
    if (pid == 0x0001u) return true;  // PID_SENTINEL: value not read
    if (pos + plen > blen) return false;
    uint32_t voff = body_off + pos;
    if (pid == 0x0070u && !seen_kh) { seen_kh = true; if (plen == 16u) kh = voff; }
    if (pid == 0x0071u && !seen_si) {
      seen_si = true;
      si = voff;
      si_flags = plen >= 4u ? (ld4(s, voff) >> 24) : SI_ERROR;  // octets em[3], then the flags
    }
    if ((pid == 0x0083u || pid == 0x800fu) && !seen_rsi) { seen_rsi = true; rsi = voff; }
    pos += plen;
  }
}

// submessage kinds the reference materialises in Message.submessages (every
// kind except PAD and unknown / vendor / security ones, rtps/submessage.rs:233-235, 278-293)
constexpr uint32_t EMIT_MASK = (1u << RTPS_ACKNACK) | (1u << RTPS_HEARTBEAT) | (1u << RTPS_GAP) |
                               (1u << RTPS_INFO_TS) | (1u << RTPS_INFO_SRC) | (1u << RTPS_INFO_DST) |
                               (1u << RTPS_INFO_REPLY) | (1u << RTPS_NACK_FRAG) | (1u << RTPS_HEARTBEAT_FRAG) |
                               (1u << RTPS_DATA) | (1u << RTPS_DATA_FRAG);
__device__ __forceinline__ bool emits(uint32_t kind) { return kind < 32u && ((EMIT_MASK >> kind) & 1u); }

// Submessage::read_from_buffer length rule (rtps/submessage.rs:61-78): a zero
// octetsToNextHeader means "to the end of the message" except for PAD / INFO_TS
__device__ __forceinline__ uint32_t eff_len(uint32_t kind, uint32_t clen, uint32_t rem) {
  return clen != 0u ? clen : ((kind == RTPS_PAD || kind == RTPS_INFO_TS) ? 0u : rem - 4u);
}

// Reader::deduce_change_kind (reader.rs:1158-1182) for the DATA payload kinds that
// call it (key: :779-785, key hash: :787-813); Data -> Alive (ddsdata.rs:45-50).
// No inline QoS -> NotAliveDisposed; inline QoS without STATUS_INFO ->
// StatusInfo::empty() -> Alive (inline_qos.rs:27-42); a STATUS_INFO shorter than
// 4 octets fails to deserialise -> NotAliveDisposed; else StatusInfo::change_kind
// (inline_qos.rs:164-175): Disposed bit, then Unregistered bit, else Alive.  The
// octet order never matters: StatusInfo reads four u8.
__device__ __forceinline__ uint32_t change_kind(uint32_t pk, bool q, uint32_t si_flags) {
  if (pk == RTPS_PK_DATA) return RTPS_CK_ALIVE;
  if (pk != RTPS_PK_KEY && pk != RTPS_PK_KEY_HASH) return RTPS_CK_NONE;
  if (!q || si_flags == SI_ERROR) return RTPS_CK_NOT_ALIVE_DISPOSED;
  if (si_flags == SI_ABSENT) return RTPS_CK_ALIVE;
  return (si_flags & 1u) ? RTPS_CK_NOT_ALIVE_DISPOSED : (si_flags & 2u) ? RTPS_CK_NOT_ALIVE_UNREGISTERED : RTPS_CK_ALIVE;
}

// What the body reader of one submessage produced.
struct SubOut {
  uint32_t cls;  // 0 not materialised, 1 writer kind, 2 reader kind, 3 interpreter kind
  uint32_t route, pk, aux16, rid, wid;
};

// The per-kind body readers of src/messages/submessages/** for one submessage
// whose window W starts at its header (W.w[0]).  Validates exactly what the
// reference reader rejects; WRITE additionally fills the kind-specific record
// words R.d[8..13] (and R.d[2..4] / R.d[10..11] for INFO_DST / INFO_SRC /
// INFO_REPLY).  Returns false on a read error (the datagram is dropped).
// TRUSTED: the submessage is known valid (its datagram's count walk passed): the checks are skipped.
#ifndef RTPS_TRUSTED_WRITE
#define RTPS_TRUSTED_WRITE 1
#endif
#define SB_CHECK(c) do { if (!TRUSTED && (c)) return false; } while (0)
template <bool WRITE, bool TRUSTED = false, class S>
__device__ __forceinline__ bool sub_body(const S& s, const Win& W, uint32_t kind, uint32_t flags, bool le,
                                         uint32_t body, uint32_t blen, Rec& R, SubOut& so) {
  so.cls = 0; so.route = 0; so.pk = 0; so.aux16 = blen; so.rid = 0; so.wid = 0;
  switch (kind) {
    case RTPS_DATA: {  // Data::deserialize_data (data.rs:57-144)
      SB_CHECK(blen < 20u);
      uint32_t otq = e16(W.w[1], 1, le);
      SB_CHECK(otq < 16u);
      uint32_t pos = 20u;
      if (otq > 16u) { pos = 4u + otq; SB_CHECK(pos > blen); }
      uint32_t fl = flags & 0x1fu;
      bool q = (fl & 0x02u) != 0u, dk = (fl & 0x0cu) != 0u;
      uint32_t qstart = pos, kh = 0, si = 0, rsi = 0, si_flags = SI_ABSENT;
      { const bool plok = !q || param_list(s, body, blen, le, pos, kh, si, rsi, si_flags); SB_CHECK(!plok); }
      so.cls = 1;
      if (WRITE) {
        so.rid = W.w[2]; so.wid = W.w[3];
        int64_t sn = sn_of(W.w[4], W.w[5], le);
        uint32_t pl_off = body + pos, pl_len = blen - pos;
        so.aux16 = pos - qstart;
        if (q) so.route |= RTPS_ROUTE_HAS_QOS;
        if (dk) so.route |= RTPS_ROUTE_HAS_PAYLOAD;
        // Reader::data_to_dds_data (reader.rs:760-833)
        uint32_t enc = 0;
        if (dk) {
          bool d = (fl & 0x04u) != 0u, k = (fl & 0x08u) != 0u;
          if (d && k) so.pk = RTPS_PK_ERR_AMBIGUOUS;
          else if (pl_len < 4u) so.pk = RTPS_PK_ERR_SHORT;
          else {
            so.pk = d ? RTPS_PK_DATA : RTPS_PK_KEY;
            enc = (pos == 20u) ? W.w[6] : ld4(s, pl_off);  // rep_id[2] + options[2]
          }
        } else {
          so.pk = kh ? RTPS_PK_KEY_HASH : RTPS_PK_ERR_NO_CONTENT;
        }
        R.d[8] = (uint32_t)sn; R.d[9] = (uint32_t)((uint64_t)sn >> 32);
        R.d[10] = pl_off | (pl_len << 16);
        R.d[11] = enc;
        R.d[12] = kh | (si << 16);
        R.d[13] = rsi | (change_kind(so.pk, q, si_flags) << 16);
      }
      return true;
    }
    case RTPS_DATA_FRAG: {  // DataFrag::deserialize (data_frag.rs:121-257)
      SB_CHECK(blen < 32u);
      uint32_t otq = e16(W.w[1], 1, le);
      SB_CHECK(otq < 28u);
      uint32_t pos = 32u;
      if (otq > 28u) { pos = 4u + otq; SB_CHECK(pos > blen); }
      bool q = (flags & 0x02u) != 0u;
      uint32_t qstart = pos, kh = 0, si = 0, rsi = 0, si_flags = SI_ABSENT;
      { const bool plok = !q || param_list(s, body, blen, le, pos, kh, si, rsi, si_flags); SB_CHECK(!plok); }
      int64_t sn = sn_of(W.w[4], W.w[5], le);
      SB_CHECK(sn < 1);
      uint32_t frag_start = e32(W.w[6], le);
      uint32_t frags_in_sub = e16(W.w[7], 0, le), frag_size = e16(W.w[7], 1, le);
      uint32_t data_size = e32(W.w[8], le);
      SB_CHECK(frag_size < 1u || frag_size > data_size);
      uint32_t total = data_size / frag_size + ((data_size % frag_size) ? 1u : 0u);
      SB_CHECK(frag_start < 1u || frag_start > total);
      so.cls = 1;
      if (WRITE) {
        so.rid = W.w[2]; so.wid = W.w[3];
        so.aux16 = pos - qstart;
        if (q) so.route |= RTPS_ROUTE_HAS_QOS;
        so.route |= RTPS_ROUTE_HAS_PAYLOAD;
        uint32_t pl_off = body + pos, pl_len = blen - pos;
        R.d[8] = (uint32_t)sn; R.d[9] = (uint32_t)((uint64_t)sn >> 32);
        R.d[10] = pl_off | (pl_len << 16);
        R.d[11] = frag_start;
        R.d[12] = frags_in_sub | (frag_size << 16);
        R.d[13] = data_size;
      }
      return true;
    }
    case RTPS_HEARTBEAT: {  // Heartbeat (heartbeat.rs:21-49): 28 bytes
      SB_CHECK(blen < 28u);
      so.cls = 1;
      if (WRITE) {
        so.rid = W.w[1]; so.wid = W.w[2];
        int64_t first = sn_of(W.w[3], W.w[4], le), last = sn_of(W.w[5], W.w[6], le);
        R.d[8] = (uint32_t)first; R.d[9] = (uint32_t)((uint64_t)first >> 32);
        R.d[10] = (uint32_t)last; R.d[11] = (uint32_t)((uint64_t)last >> 32);
        R.d[12] = e32(W.w[7], le);
      }
      return true;
    }
    case RTPS_HEARTBEAT_FRAG: {  // HeartbeatFrag (heartbeat_frag.rs:16-37): 24 bytes
      SB_CHECK(blen < 24u);
      so.cls = 1;
      if (WRITE) {
        so.rid = W.w[1]; so.wid = W.w[2];
        int64_t sn = sn_of(W.w[3], W.w[4], le);
        R.d[8] = (uint32_t)sn; R.d[9] = (uint32_t)((uint64_t)sn >> 32);
        R.d[10] = e32(W.w[5], le);
        R.d[11] = e32(W.w[6], le);
      }
      return true;
    }
    case RTPS_GAP: {  // Gap (gap.rs:23-46): rid wid gapStart SNSet
      SB_CHECK(blen < 28u);
      uint32_t nb = e32(W.w[7], le);
      SB_CHECK(nb > 256u);
      uint32_t words = (nb + 31u) >> 5;
      SB_CHECK(28u + 4u * words > blen);
      so.cls = 1;
      if (WRITE) {
        so.rid = W.w[1]; so.wid = W.w[2];
        int64_t gs = sn_of(W.w[3], W.w[4], le), lb = sn_of(W.w[5], W.w[6], le);
        R.d[8] = (uint32_t)gs; R.d[9] = (uint32_t)((uint64_t)gs >> 32);
        R.d[10] = (uint32_t)lb; R.d[11] = (uint32_t)((uint64_t)lb >> 32);
        R.d[12] = nb;
        R.d[13] = body + 28u;
      }
      return true;
    }
    case RTPS_ACKNACK: {  // AckNack (ack_nack.rs:27-50): rid wid SNSet count
      SB_CHECK(blen < 20u);
      uint32_t nb = e32(W.w[5], le);
      SB_CHECK(nb > 256u);
      uint32_t words = (nb + 31u) >> 5;
      SB_CHECK(24u + 4u * words > blen);
      so.cls = 2;
      if (WRITE) {
        so.rid = W.w[1]; so.wid = W.w[2];
        int64_t base = sn_of(W.w[3], W.w[4], le);
        R.d[8] = (uint32_t)base; R.d[9] = (uint32_t)((uint64_t)base >> 32);
        R.d[10] = e32(ld4(s, body + 20u + 4u * words), le);
        R.d[12] = nb;
        R.d[13] = body + 20u;
      }
      return true;
    }
    case RTPS_NACK_FRAG: {  // NackFrag (nack_frag.rs:31-53): rid wid sn FNSet count
      SB_CHECK(blen < 24u);
      uint32_t nb = e32(W.w[6], le);
      SB_CHECK(nb > 256u);
      uint32_t words = (nb + 31u) >> 5;
      SB_CHECK(28u + 4u * words > blen);
      so.cls = 2;
      if (WRITE) {
        so.rid = W.w[1]; so.wid = W.w[2];
        int64_t sn = sn_of(W.w[3], W.w[4], le);
        R.d[8] = (uint32_t)sn; R.d[9] = (uint32_t)((uint64_t)sn >> 32);
        R.d[10] = e32(W.w[5], le);
        R.d[11] = e32(ld4(s, body + 24u + 4u * words), le);
        R.d[12] = nb;
        R.d[13] = body + 24u;
      }
      return true;
    }
    case RTPS_INFO_TS:  // rtps/submessage.rs:211-225 (Invalidate flag: no body read)
      SB_CHECK(!(flags & 0x02u) && blen < 8u);
      so.cls = 3;
      return true;
    case RTPS_INFO_SRC:  // InfoSource (info_source.rs:22-36)
      SB_CHECK(blen < 20u);
      so.cls = 3;
      if (WRITE) R.d[10] = W.w[2];
      return true;
    case RTPS_INFO_DST:  // InfoDestination (info_destination.rs:20-25)
      SB_CHECK(blen < 12u);
      so.cls = 3;
      if (WRITE) { R.d[2] = W.w[1]; R.d[3] = W.w[2]; R.d[4] = W.w[3]; }
      return true;
    case RTPS_INFO_REPLY: {  // InfoReply (info_reply.rs:9-21): Vec<Locator> + Option<Vec<Locator>>
      SB_CHECK(blen < 4u);
      uint32_t n1 = e32(W.w[1], le), n2 = 0xffffffffu;
      uint64_t pos = 4u + 24ull * n1;
      SB_CHECK(pos > blen);
      SB_CHECK(pos + 1u > blen);
      uint32_t tag = ld4(s, body + (uint32_t)pos) & 0xffu;
      pos += 1u;
      if (tag != 0u) {
        SB_CHECK(pos + 4u > blen);
        n2 = e32(ld4(s, body + (uint32_t)pos), le);
        pos += 4u;
        SB_CHECK(pos + 24ull * n2 > blen);
      }
      so.cls = 3;
      if (WRITE) { R.d[10] = n1; R.d[11] = n2; }
      return true;
    }
    default:  // PAD, INFO_REPLY_IP4, SEC_*, vendor and unknown kinds: skipped (:233-235, :278-293)
      return true;
  }
}

// Interpreter state in effect *after* a submessage (SubmessageIter2,
// io_uring/rtps/message_receiver.rs:56-119, 618-665).
struct Interp {
  uint32_t src0, src1, src2;  // source GuidPrefix
  bool dst_ok;                // dest == own || dest == UNKNOWN
  bool ts_valid;
  uint32_t ts_sec, ts_frac;
};

// Common tail of a record: ids, source prefix, the SubmessageIter2 writer
// filter (:75-84), builtin / target-set classification, timestamp, word 7.
// Returns the record's target set.
__device__ __forceinline__ uint32_t rec_finish(const KParams& p, Rec& R, const SubOut& so, uint32_t kind,
                                               const Interp& st) {
  uint32_t route = so.route;
  uint32_t tgt = RTPS_NO_TARGET;
  if (kind != RTPS_INFO_DST) { R.d[2] = st.src0; R.d[3] = st.src1; R.d[4] = st.src2; }
  if (so.cls != 3) {
    R.d[5] = so.wid; R.d[6] = so.rid;
    if (so.cls == 1) {
      if (st.dst_ok) route |= RTPS_ROUTE_PASS;
      if (builtin_writer_pair(so.rid, so.wid)) route |= RTPS_ROUTE_BUILTIN;
      else tgt = target_lookup(p, st.src0, st.src1, st.src2, so.wid, route);
    } else {
      route |= RTPS_ROUTE_PASS;
      if (builtin_reader_pair(so.rid, so.wid)) route |= RTPS_ROUTE_BUILTIN;
    }
  }
  if (st.ts_valid) { route |= RTPS_ROUTE_TS_VALID; R.d[14] = st.ts_sec; R.d[15] = st.ts_frac; }
  R.d[7] = (so.aux16 & 0xffffu) | (route << 16) | (so.pk << 24);
  return tgt;
}

// SubmessageIter2 interpreter transitions (message_receiver.rs:618-665)
__device__ __forceinline__ void interp_update(const KParams& p, Interp& st, const Win& W, uint32_t kind,
                                              uint32_t flags, bool le) {
  if (kind == RTPS_INFO_TS) {  // Invalidate flag -> None
    st.ts_valid = !(flags & 0x02u);
    st.ts_sec = st.ts_valid ? e32(W.w[1], le) : 0u;
    st.ts_frac = st.ts_valid ? e32(W.w[2], le) : 0u;
  } else if (kind == RTPS_INFO_SRC) {  // new source, timestamp cleared (:626-636)
    st.src0 = W.w[3]; st.src1 = W.w[4]; st.src2 = W.w[5];
    st.ts_valid = false; st.ts_sec = 0u; st.ts_frac = 0u;
  } else if (kind == RTPS_INFO_DST) {  // UNKNOWN -> own (:656-662)
    const uint32_t a = W.w[1], b = W.w[2], c = W.w[3];
    st.dst_ok = ((a | b | c) == 0u) || (a == p.own0 && b == p.own1 && c == p.own2);
  }
}

// Walk one datagram on one lane.  WRITE=false: validate + count materialised
// submessages.  WRITE=true (datagram known OK): write its records starting at
// record index `ridx`, to p.records[ridx + k], or, when stage != nullptr, to
// the LDS staging buffer stage[ridx + k - stage_first] (the caller copies it out).
template <bool WRITE>
__device__ uint32_t walk(const KParams& p, const Src& s, const uint32_t* H, uint32_t L, uint32_t dgram_idx,
                         uint64_t ridx, uint32_t& nrec, u32x4* stage = nullptr, uint32_t* stage_match = nullptr,
                         uint64_t stage_first = 0) {
  nrec = 0;
  if (L > RTPS_MAX_DATAGRAM) return RTPS_DGRAM_TOO_LONG;
  const uint32_t MAGIC_RTPS = 0x53505452u, MAGIC_RTPX = 0x58505452u;  // "RTPS" / "RTPX"
  if (L < 20u) {  // message_receiver.rs:238-251
    if (L >= 16u && H[0] == MAGIC_RTPS && (H[2] >> 8) == 0x534444u /* "DDS" */ &&
        H[3] == 0x474e4950u /* "PING" */)
      return RTPS_DGRAM_PING;
    return RTPS_DGRAM_SHORT;
  }
  if (H[0] != MAGIC_RTPS) return H[0] == MAGIC_RTPX ? RTPS_DGRAM_RTPX : RTPS_DGRAM_BAD_MAGIC;
  if ((H[1] & 0xffu) > 2u) return RTPS_DGRAM_BAD_HEADER;  // ProtocolVersion major
  // handle_parsed_message_2 (:289-295): src := header prefix, dest := own, ts := None
  Interp st{H[2], H[3], H[4], true, false, 0u, 0u};
  uint32_t o = 20;
  // WRITE: the window of the next submessage is loaded before this record's
  // stores are issued.  vmcnt counts stores too, so a load issued after them
  // would make the next iteration wait for their write acknowledgements.
  // The count walk takes its first window from the head before the loop, so
  // the head's registers are dead in it.
  Win Wn, W;
  if (WRITE) head_win(H, Wn);
  else head_win(H, W);
  while (o < L) {
    uint32_t rem = L - o;
    if (rem < 4u) return RTPS_DGRAM_SUBMSG_ERR;  // SubmessageHeader needs 4 bytes
    if (WRITE) {
      W = Wn;
      if (o != 20u && (W.w[0] & 0xffu) == RTPS_DATA_FRAG) W.w[8] = ld4(s, o + 32u);
    } else if (o != 20u) {
      load_win_lazy<WRITE>(s, o, W);
    }
    uint32_t kind = W.w[0] & 0xffu, flags = (W.w[0] >> 8) & 0xffu;
    bool le = (flags & 1u) != 0u;
    uint32_t eff = eff_len(kind, e16(W.w[0], 1, le), rem);
    if (4u + eff > rem) return RTPS_DGRAM_SUBMSG_ERR;
    if (WRITE && o + 4u + eff < L) load_win_pf(s, o + 4u + eff, Wn);
    Rec R;
    if (WRITE) rec_clear(R);
    SubOut so;
    if (!sub_body<WRITE, WRITE && RTPS_TRUSTED_WRITE != 0>(s, W, kind, flags, le, o + 4u, eff, R, so))
      return RTPS_DGRAM_SUBMSG_ERR;  // (WRITE: the datagram passed its count walk)
    interp_update(p, st, W, kind, flags, le);
    if (so.cls != 0u) {
      if (WRITE) {
        R.d[0] = dgram_idx;
        R.d[1] = o | (kind << 16) | (flags << 24);
        const uint32_t mslot = rec_finish(p, R, so, kind, st);
        const uint64_t r = ridx + nrec;
        if (stage) {
          u32x4* q = stage + (r - stage_first) * 4u;
          q[0] = u32x4{R.d[0], R.d[1], R.d[2], R.d[3]};
          q[1] = u32x4{R.d[4], R.d[5], R.d[6], R.d[7]};
          q[2] = u32x4{R.d[8], R.d[9], R.d[10], R.d[11]};
          q[3] = u32x4{R.d[12], R.d[13], R.d[14], R.d[15]};
          stage_match[r - stage_first] = mslot;
        } else if (r < p.max_records) {
          rec_store(p.records + r, R);
          if (p.target_out) p.target_out[r] = mslot;
        }
      }
      nrec++;
    }
    o += 4u + eff;
  }
  return RTPS_DGRAM_OK;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// ---------------------------------------------------------------------------
// Ordered output:
//   A  rtps_parse_spec_kernel  one workgroup per tile of 256 datagrams (blockIdx
//      order): walk 1 counts each datagram's records; a tile in which every
//      datagram has exactly k_spec records ("speculative" tile) walks again and
//      writes its records at tile*256*k_spec + local prefix, which is the final
//      position whenever every earlier tile is speculative too.  Every tile
//      publishes its count and flags (info[], below).
//   C  rtps_parse_chain_kernel  replaces A for mixed traffic: count walk, the
//      exact prefix from the predecessors' published counts (two-level
//      look-back, bounded polls), then the writing walk.
//   B  rtps_parse_fix_kernel   persistent, after A or C: reduces the tile
//      counts (n_records), reports the batch's mix for the next launch choice,
//      and walks the tiles not yet written at their exact positions
//      (overwriting any speculative writes there).
// One-DATA-per-datagram traffic (T, C2, C4) finishes in A; mixed traffic (C3)
// in C.  A and B have no spin-waits, tickets or grid barriers.
// ---------------------------------------------------------------------------
struct TileCtx {
  uint32_t i;      // datagram index of this lane
  bool valid, addressable;
  uint32_t L;
  Src s;
  uint32_t H[16];  // datagram bytes 0..64
};

// arenas below this size are addressed from their start (datagram offset + in-datagram
// offset < 2^32 - 2^17); larger ones from each wave's smallest datagram offset
#ifndef RTPS_ARENA_DIRECT
#define RTPS_ARENA_DIRECT ((1ull << 32) - (1ull << 17))
#endif
constexpr uint64_t ARENA_DIRECT = RTPS_ARENA_DIRECT;  // (0: every arena per wave; variant builds)
// load this lane's (offset, length), build the wave's buffer descriptor
// (base = the arena, or for arenas of 4 GiB and more the min offset over the wave:
// no workgroup barrier) and the 64-byte head
template <uint32_t TS = TILE>
__device__ __forceinline__ void tile_src(const KParams& p, uint32_t tile, TileCtx& t, bool enabled = true,
                                         uint32_t tid = threadIdx.x) {
  t.i = tile * TS + tid;
  t.valid = enabled && tid < TS && t.i < p.n;
  const uint64_t off = t.valid ? p.dgram_off[t.i] : ~0ull;
  t.L = t.valid ? p.dgram_len[t.i] : 0u;
  uint64_t tb = 0;  // descriptor base: the arena itself when every in-datagram offset fits 32 bits
  if (p.arena_len >= ARENA_DIRECT) {  // (uniform) larger arenas: the wave's smallest datagram offset
    uint64_t m = off;
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) {
      uint64_t y = __shfl_xor(m, d, 64);
      m = y < m ? y : m;
    }
    tb = m > p.arena_len ? p.arena_len : m;
    uint32_t tb_lo = __builtin_amdgcn_readfirstlane((uint32_t)tb);
    uint32_t tb_hi = __builtin_amdgcn_readfirstlane((uint32_t)(tb >> 32));
    tb = ((uint64_t)tb_hi << 32) | tb_lo;
  }
  uint64_t avail64 = p.arena_len - tb;
  uint32_t avail = __builtin_amdgcn_readfirstlane(avail64 > 0xffffffffull ? 0xffffffffu : (uint32_t)avail64);
  t.s.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.arena + tb), (short)0, (int)avail,
                                               0x00020000);
  t.s.avail = avail;
  const uint64_t rel = t.valid ? off - tb : 0;
  t.addressable = t.valid && off <= p.arena_len && (uint64_t)t.L <= p.arena_len - off && rel + t.L <= avail;
  t.s.base = (uint32_t)rel;
}
// tile_src plus the 64-byte head
template <uint32_t TS = TILE>
__device__ __forceinline__ void load_tile(const KParams& p, uint32_t tile, TileCtx& t, bool enabled = true,
                                          uint32_t tid = threadIdx.x) {
  tile_src<TS>(p, tile, t, enabled, tid);
  u32x4 a = {0u, 0u, 0u, 0u}, b = a, c = a, d = a;
  if (t.addressable) {
    a = ld16(t.s, 0); b = ld16(t.s, 16); c = ld16(t.s, 32);
    // bytes 48..63 serve only the first submessage's window, which a DATA there
    // does not read (its fields and encapsulation end at byte 48): skipping them
    // saves a line fetch wherever they begin a new 128-B line
    if ((b[1] & 0xffu) != RTPS_DATA) d = ld16(t.s, 48);
  }
  t.H[0] = a[0]; t.H[1] = a[1]; t.H[2] = a[2]; t.H[3] = a[3];
  t.H[4] = b[0]; t.H[5] = b[1]; t.H[6] = b[2]; t.H[7] = b[3];
  t.H[8] = c[0]; t.H[9] = c[1]; t.H[10] = c[2]; t.H[11] = c[3];
  t.H[12] = d[0]; t.H[13] = d[1]; t.H[14] = d[2]; t.H[15] = d[3];
}

__device__ __forceinline__ uint32_t count_lane(const KParams& p, TileCtx& t, uint32_t& cnt) {
  cnt = 0;
  uint32_t st = RTPS_DGRAM_OK;
  if (t.valid) {
    if (!t.addressable) st = RTPS_DGRAM_TOO_LONG;
    else st = walk<false>(p, t.s, t.H, t.L, t.i, 0, cnt);
    if (st != RTPS_DGRAM_OK) cnt = 0;
  }
  return st;
}

// scratch layout (all written before being read in every launch, except flag[]):
//   u32 flag[4]          flag[parity] = 1 if any tile of the launch is non-speculative
//                        (plain stores of the same value); kernel B clears flag[parity ^ 1]
//   u32 info[n_tiles]    see below
//   u16 dcount[n]        records per datagram, written for non-speculative tiles only
// info[tile] = records | INFO_NONSPEC (B must account per datagram) | INFO_WRITTEN (the
// chained kernel already wrote the tile at its exact position: B only counts it) |
// INFO_MIXED (some datagram does not have k_spec records: sizes the next launch's choice)
constexpr uint32_t INFO_NONSPEC = 0x80000000u, INFO_WRITTEN = 0x40000000u, INFO_MIXED = 0x20000000u,
                   INFO_COUNT = 0x1fffffffu;
struct Scratch {
  uint32_t* flag;
  uint32_t* info;
  uint16_t* dcount;
};
__device__ __forceinline__ Scratch scratch_of(uint64_t* base, uint32_t n_tiles) {
  Scratch x;
  x.flag = reinterpret_cast<uint32_t*>(base);
  x.info = x.flag + 4;
  x.dcount = reinterpret_cast<uint16_t*>(x.info + ((n_tiles + 3u) & ~3u));
  return x;
}

constexpr uint32_t STAGE_RECS = TILE;  // LDS staging for speculative tiles with k_spec == 1
__global__ __launch_bounds__(TILE, RTPS_WAVES_PER_SIMD) void rtps_parse_spec_kernel(KParams p, uint32_t n_tiles,
                                                                                     uint32_t k_spec, uint32_t parity) {
  __shared__ uint32_t s_wave_sum[WAVES], s_wave_bad[WAVES];
  __shared__ u32x4 s_stage[STAGE_RECS * 4];
  __shared__ uint32_t s_stage_match[STAGE_RECS];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t tile = blockIdx.x;
  mt_stage(p);  // visible after the __syncthreads below, before the writing walk
  TileCtx t;
  load_tile(p, tile, t);
  uint32_t cnt;
  const uint32_t st = count_lane(p, t, cnt);
  const uint32_t incl = wave_incl_scan(cnt, lane);
  const uint64_t bad = __ballot(t.valid && cnt != k_spec);
  if (lane == 63) { s_wave_sum[wave] = incl; s_wave_bad[wave] = bad != 0ull; }
  __syncthreads();
  uint32_t wave_off = 0, agg = 0, nonspec = 0;
#pragma unroll
  for (uint32_t w = 0; w < WAVES; ++w) {
    uint32_t v = s_wave_sum[w];
    if (w < wave) wave_off += v;
    agg += v;
    nonspec |= s_wave_bad[w];
  }
  Scratch x = scratch_of(p.scratch, n_tiles);
  if (tid == 0) {
    x.info[tile] = agg | (nonspec ? INFO_NONSPEC | INFO_MIXED : 0u);  // read by kernel B (next launch)
    if (nonspec) x.flag[parity] = 1u;
  }
  if (t.valid) {
    p.status[t.i] = (uint8_t)st;
    if (nonspec) x.dcount[t.i] = (uint16_t)cnt;
  }
  if (!nonspec) {
    const uint64_t tile_first = (uint64_t)tile * TILE * k_spec;
    const uint64_t my_first = tile_first + wave_off + (incl - cnt);
    const bool stage = k_spec == 1u;  // agg == valid datagrams <= STAGE_RECS
    if (t.valid) {
      if (p.rec_begin) p.rec_begin[t.i] = (uint32_t)my_first;
      if (cnt) {
        uint32_t n2;
        if (stage) walk<true>(p, t.s, t.H, t.L, t.i, my_first, n2, s_stage, s_stage_match, tile_first);
        else walk<true>(p, t.s, t.H, t.L, t.i, my_first, n2);
      }
    }
    if (stage) {  // coalesced copy-out: 16 B per lane, contiguous per wave instruction
      __syncthreads();
      const uint64_t lim = p.max_records > tile_first ? p.max_records - tile_first : 0;
      const uint32_t nrec = agg < lim ? agg : (uint32_t)lim;
      u32x4* dst = reinterpret_cast<u32x4*>(p.records + tile_first);
      for (uint32_t k = tid; k < nrec * 4u; k += TILE) rec_st16(dst + k, s_stage[k]);
      if (p.target_out)
        for (uint32_t k = tid; k < nrec; k += TILE) p.target_out[tile_first + k] = s_stage_match[k];
    }
  }
}


// sum of info[lo, hi) counts and the first tile B must walk, over the workgroup
__device__ __forceinline__ void reduce_info(const uint32_t* info, uint32_t lo, uint32_t hi, uint64_t* s_sum,
                                            uint32_t* s_min, uint64_t& sum, uint32_t& first_bad) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint64_t acc = 0;
  uint32_t fb = 0xffffffffu;
  for (uint32_t t = lo + tid; t < hi; t += TILE) {
    uint32_t v = info[t];
    acc += v & INFO_COUNT;
    if ((v & (INFO_NONSPEC | INFO_WRITTEN)) == INFO_NONSPEC && t < fb) fb = t;
  }
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    acc += __shfl_xor(acc, d, 64);
    uint32_t y = __shfl_xor(fb, d, 64);
    fb = y < fb ? y : fb;
  }
  if (lane == 0) { s_sum[wave] = acc; s_min[wave] = fb; }
  __syncthreads();
  sum = 0;
  first_bad = 0xffffffffu;
#pragma unroll
  for (uint32_t w = 0; w < WAVES; ++w) {
    sum += s_sum[w];
    first_bad = s_min[w] < first_bad ? s_min[w] : first_bad;
  }
  __syncthreads();
}

// Kernel B: every workgroup first reduces the tile counts of kernel A (16 KB
// per 1M datagrams, L2-resident) to find the first non-speculative tile f and
// the total; workgroup 0 publishes the total.  Tiles f.. are then re-walked in
// a grid-stride loop, each at its exact prefix.
// TS: datagrams per tile of the first kernel (256 for A and C, LT for the LDS-tile kernel D)
template <uint32_t TS>
__global__ __launch_bounds__(TILE, RTPS_WAVES_PER_SIMD) void rtps_parse_fix_kernel(KParams p, uint32_t n_tiles,
                                                                                    uint32_t k_spec, uint32_t parity) {
  __shared__ uint32_t s_wave_sum[WAVES];
  __shared__ uint64_t s_rsum[WAVES];
  __shared__ uint32_t s_rmin[WAVES];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  Scratch x = scratch_of(p.scratch, n_tiles);
  if (blockIdx.x == 0 && tid == 0) x.flag[parity ^ 1u] = 0u;  // for the next launch
  if (__builtin_amdgcn_readfirstlane(x.flag[parity]) == 0u) {
    // every tile was speculative: every datagram has exactly k_spec records
    if (blockIdx.x == 0 && tid == 0) {
      *p.n_records = (uint64_t)p.n * k_spec;
      p.mixed_out[0] = 0u;
      p.mixed_out[1] = n_tiles;
    }
    return;
  }
  uint64_t total;
  uint32_t first;
  reduce_info(x.info, 0, n_tiles, s_rsum, s_rmin, total, first);
  if (blockIdx.x == 0) {
    uint32_t mixed = 0;
    for (uint32_t t = tid; t < n_tiles; t += TILE) mixed += (x.info[t] & INFO_MIXED) != 0u;
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) mixed += __shfl_xor(mixed, d, 64);
    if (lane == 0) s_wave_sum[wave] = mixed;
    __syncthreads();
    if (tid == 0) {
      *p.n_records = total;
      p.mixed_out[0] = s_wave_sum[0] + s_wave_sum[1] + s_wave_sum[2] + s_wave_sum[3];
      p.mixed_out[1] = n_tiles;
    }
    __syncthreads();  // s_wave_sum reuse below
  }
  if (first > n_tiles) first = n_tiles;
  uint32_t tile = first + blockIdx.x;
  if (tile >= n_tiles) return;
  mt_stage(p);
  __syncthreads();
  uint64_t prefix, dummy_sum;
  uint32_t dummy_min;
  reduce_info(x.info, 0, tile, s_rsum, s_rmin, prefix, dummy_min);
  for (;;) {
    const uint32_t info = x.info[tile];
    const uint32_t i = tile * TS + tid;
    // non-speculative tiles stored their per-datagram counts; speculative tiles
    // (after the first non-speculative one) have exactly k_spec per datagram
    uint32_t cnt = 0;
    if (tid < TS && i < p.n) cnt = (info & INFO_NONSPEC) ? (uint32_t)x.dcount[i] : k_spec;
    const bool skip = (info & INFO_WRITTEN) != 0;  // written in place by the chained kernel
    const uint32_t incl = wave_incl_scan(cnt, lane);
    if (lane == 63) s_wave_sum[wave] = incl;
    __syncthreads();
    uint32_t wave_off = 0;
#pragma unroll
    for (uint32_t w = 0; w < WAVES; ++w)
      if (w < wave) wave_off += s_wave_sum[w];
    const uint64_t my_first = prefix + wave_off + (incl - cnt);
    TileCtx t;
    load_tile<TS>(p, tile, t, !skip);
    if (t.valid) {
      if (p.rec_begin) p.rec_begin[t.i] = (uint32_t)my_first;
      if (cnt) {  // cnt > 0 implies status OK
        uint32_t n2;
        walk<true>(p, t.s, t.H, t.L, t.i, my_first, n2);
      }
    }
    __syncthreads();  // s_wave_sum reuse
    const uint32_t next = tile + gridDim.x;
    if (next >= n_tiles) break;
    reduce_info(x.info, tile, next, s_rsum, s_rmin, dummy_sum, dummy_min);
    prefix += dummy_sum;
    tile = next;
  }
}

// ---------------------------------------------------------------------------
// E / S / W: the item pass for mixed traffic (the default
// since round 4).  The chained kernel C spends its time in three places: the
// count walk, the look-back wait, and a second walk that re-fetches every
// submessage to write it.  Here the count walk leaves behind what the write
// needs, so no kernel waits on another tile and no lane chases a chain twice:
//   E rtps_parse_item_kernel  one workgroup per tile of 256 datagrams: the count
//     walk (status, records per datagram) appends one 16-B ITEM per materialised
//     submessage to its wave's slab of CAPW items, at a position taken with a
//     wave ballot in the walk loop (no atomics, no ordering between tiles):
//       [0] sub_off | src_off << 16   src_off: datagram offset of the source prefix
//                                     in effect (8: the header's; INFO_SRC at o: o + 12)
//       [1] j | lane << 16 | dst_ok << 22 | ts_valid << 23 | kind << 24
//                                     j: the record's index inside its datagram
//       [2] ts_sec  [3] ts_frac       the timestamp in effect (host order)
//     A wave whose items overflow its slab is flagged; W walks its datagrams.
//   S rtps_parse_scan_kernel  one workgroup: exclusive scan of the tile counts,
//     n_records, the launch-choice report (what kernel B does after A / C).
//   W rtps_parse_emit_kernel  one workgroup per tile: one thread per item, in slab
//     order (coalesced item loads): the item names the kind, so the submessage
//     window is ONE gather issued at once (16 B, + 16 B for kinds that read body
//     bytes past 12), the source prefix comes from a per-datagram LDS stage, the
//     interpreter state from the item; the per-kind reader and the record tail are
//     the walk's own (sub_body / rec_finish); the record goes to tile prefix +
//     datagram's local first record + j.
// ---------------------------------------------------------------------------
#ifndef RTPS_IT_CAPW
#define RTPS_IT_CAPW 512u
#endif
constexpr uint32_t CAPW = RTPS_IT_CAPW;  // items per wave slab (C3 averages 243 per 64 datagrams)
// Wide items (48 B): the item also carries the submessage's 32-B window as the walk loaded it
// (with the tail the record's reader needs), so that the record pass reads it coalesced with
// the item instead of gathering it from the datagram again.
#ifndef RTPS_IT_WIDE
#define RTPS_IT_WIDE 0  // measured: E +49 us, W -11 us on C3
#endif
constexpr uint32_t IW = RTPS_IT_WIDE ? 3u : 1u;  // u32x4 per item
constexpr uint32_t WCNT_OVERFLOW = 0x80000000u;
constexpr uint32_t DI_NOREC = 0x80000000u;  // dinfo[0]: the datagram has no records
#ifndef RTPS_IT_WAVES_PER_SIMD
#define RTPS_IT_WAVES_PER_SIMD 8
#endif
#ifndef RTPS_EM_WAVES_PER_SIMD
#define RTPS_EM_WAVES_PER_SIMD 8
#endif

// The count walk of walk<false> plus the items.  wpos: the wave's slab position,
// the same in every active lane (each iteration advances it by the ballot's count).
__device__ uint32_t item_walk(const KParams& p, const Src& s, const uint32_t* H, uint32_t L, uint32_t lane,
                              u32x4* slab, uint32_t& wpos, uint32_t& nrec) {
  nrec = 0;
  if (L > RTPS_MAX_DATAGRAM) return RTPS_DGRAM_TOO_LONG;
  const uint32_t MAGIC_RTPS = 0x53505452u, MAGIC_RTPX = 0x58505452u;
  if (L < 20u) {  // message_receiver.rs:238-251
    if (L >= 16u && H[0] == MAGIC_RTPS && (H[2] >> 8) == 0x534444u && H[3] == 0x474e4950u) return RTPS_DGRAM_PING;
    return RTPS_DGRAM_SHORT;
  }
  if (H[0] != MAGIC_RTPS) return H[0] == MAGIC_RTPX ? RTPS_DGRAM_RTPX : RTPS_DGRAM_BAD_MAGIC;
  if ((H[1] & 0xffu) > 2u) return RTPS_DGRAM_BAD_HEADER;
  // handle_parsed_message_2 (:289-295): src := header prefix, dest := own, ts := None
  Interp st{H[2], H[3], H[4], true, false, 0u, 0u};
  uint32_t src_off = 8u;
  const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t o = 20;
  // the first window comes from the head, before the loop: the head's registers are dead in it
  Win W;
  head_win(H, W);
  while (o < L) {
    const uint32_t rem = L - o;
    if (rem < 4u) return RTPS_DGRAM_SUBMSG_ERR;
    if (o != 20u) load_win_lazy<RTPS_IT_WIDE != 0>(s, o, W);
    const uint32_t kind = W.w[0] & 0xffu, flags = (W.w[0] >> 8) & 0xffu;
    const bool le = (flags & 1u) != 0u;
    const uint32_t eff = eff_len(kind, e16(W.w[0], 1, le), rem);
    if (4u + eff > rem) return RTPS_DGRAM_SUBMSG_ERR;
    Rec R;
    SubOut so;
    if (!sub_body<false>(s, W, kind, flags, le, o + 4u, eff, R, so)) return RTPS_DGRAM_SUBMSG_ERR;
    interp_update(p, st, W, kind, flags, le);  // (INFO_SRC's prefix words are not loaded here: src_off)
    if (kind == RTPS_INFO_SRC) src_off = o + 12u;
    const bool em = so.cls != 0u;
    const uint64_t m = __ballot(em);
    if (em) {
      const uint32_t pos = wpos + (uint32_t)__popcll(m & lt);
      if (pos < CAPW) {
        const u32x4 iv{o | (src_off << 16),
                       nrec | (lane << 16) | ((st.dst_ok ? 1u : 0u) << 22) | ((st.ts_valid ? 1u : 0u) << 23) |
                           (kind << 24),
                       st.ts_sec, st.ts_frac};
        slab[pos * IW] = iv;
        if (IW == 3u) {
          slab[pos * IW + 1] = u32x4{W.w[0], W.w[1], W.w[2], W.w[3]};
          slab[pos * IW + 2] = u32x4{W.w[4], W.w[5], W.w[6], W.w[7]};
        }
      }
      nrec++;
    }
    wpos += (uint32_t)__popcll(m);
    o += 4u + eff;
  }
  return RTPS_DGRAM_OK;
}

__global__ __launch_bounds__(TILE, RTPS_IT_WAVES_PER_SIMD) void rtps_parse_item_kernel(KParams p, uint32_t n_tiles,
                                                                                     uint32_t k_spec, u32x4* items,
                                                                                     uint32_t* wcnt, u32x4* dinfo) {
  __shared__ uint32_t s_wave_sum[WAVES], s_wave_bad[WAVES];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: the slab base in SGPRs)
  const uint32_t tile = blockIdx.x;
  TileCtx t;
  load_tile(p, tile, t);
  u32x4* slab = items + (size_t)(tile * WAVES + wave) * CAPW * IW;
  uint32_t cnt = 0, wpos = 0, st = RTPS_DGRAM_OK;
  if (t.valid) {
    if (!t.addressable) st = RTPS_DGRAM_TOO_LONG;
    else st = item_walk(p, t.s, t.H, t.L, lane, slab, wpos, cnt);
    if (st != RTPS_DGRAM_OK) cnt = 0;
  }
  const uint32_t incl = dinfo ? wave_incl_scan(cnt, lane) : 0u;
  // the wave's item total: the position of the lane that walked longest
  uint32_t wtot = wpos, wsum = cnt;
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    const uint32_t y = __shfl_xor(wtot, d, 64);
    wtot = y > wtot ? y : wtot;
    wsum += __shfl_xor(wsum, d, 64);
  }
  const uint64_t bad = __ballot(t.valid && cnt != k_spec);
  if (lane == 0) {
    s_wave_sum[wave] = wsum;
    s_wave_bad[wave] = bad != 0ull;
    wcnt[tile * WAVES + wave] = wtot > CAPW ? WCNT_OVERFLOW : wtot;
  }
  Scratch x = scratch_of(p.scratch, n_tiles);
  if (t.valid) {
    p.status[t.i] = (uint8_t)st;
    if (!dinfo) x.dcount[t.i] = (uint16_t)cnt;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t agg = 0, mixed = 0;
#pragma unroll
    for (uint32_t w = 0; w < WAVES; ++w) { agg += s_wave_sum[w]; mixed |= s_wave_bad[w]; }
    x.info[tile] = agg | INFO_NONSPEC | (mixed ? INFO_MIXED : 0u);
  }
  if (dinfo && t.valid) {  // the record pass's per-datagram prologue, one coalesced 16-B word
    uint32_t woff = 0;
#pragma unroll
    for (uint32_t w = 0; w < WAVES; ++w) woff += w < wave ? s_wave_sum[w] : 0u;
    dinfo[t.i] = u32x4{(woff + incl - cnt) | (cnt ? 0u : DI_NOREC), t.H[2], t.H[3], t.H[4]};
  }
}

// S: one workgroup of 1024 threads, 4 tiles per thread per round
constexpr uint32_t SCAN_T = 1024;
__global__ __launch_bounds__(SCAN_T) void rtps_parse_scan_kernel(KParams p, uint32_t n_tiles, uint32_t parity,
                                                                 uint64_t* tprefix) {
  __shared__ uint64_t s_w[SCAN_T / 64];
  __shared__ uint32_t s_m[SCAN_T / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  Scratch x = scratch_of(p.scratch, n_tiles);
  uint64_t carry = 0;
  uint32_t mixed = 0;
  for (uint32_t base = 0; base < n_tiles; base += 4u * SCAN_T) {
    const uint32_t t0 = base + 4u * tid;
    uint32_t c[4];
    if (t0 + 3u < n_tiles) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(x.info + t0);  // info is 16-B aligned
      c[0] = v[0]; c[1] = v[1]; c[2] = v[2]; c[3] = v[3];
    } else {
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) c[k] = t0 + k < n_tiles ? x.info[t0 + k] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) { mixed += (c[k] & INFO_MIXED) != 0u; c[k] &= INFO_COUNT; }
    const uint64_t own = (uint64_t)c[0] + c[1] + c[2] + c[3];
    uint64_t incl = own;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint64_t before = carry, total = carry;
#pragma unroll
    for (uint32_t w = 0; w < SCAN_T / 64; ++w) {
      const uint64_t v = s_w[w];
      if (w < wave) before += v;
      total += v;
    }
    uint64_t e = before + incl - own;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (t0 + k < n_tiles) tprefix[t0 + k] = e;
      e += c[k];
    }
    carry = total;
    __syncthreads();  // s_w reuse
  }
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) mixed += __shfl_xor(mixed, d, 64);
  if (lane == 0) s_m[wave] = mixed;
  __syncthreads();
  if (tid == 0) {
    uint32_t m = 0;
    for (uint32_t w = 0; w < SCAN_T / 64; ++w) m += s_m[w];
    *p.n_records = carry;
    p.mixed_out[0] = m;
    p.mixed_out[1] = n_tiles;
    x.flag[parity ^ 1u] = 0u;  // kernel B's invariant for the next launch (B does not run after S)
  }
}

// The item of slab position k, its datagram's fields (lane permutes: every lane of the
// wave calls this) and the record it becomes: R, its target set, its index r (~0: none).
__device__ __forceinline__ void em2_item(const KParams& p, const Src& s0, const u32x4 it, bool act, const u32x4 di,
                                         uint32_t doff, uint32_t dlen, uint32_t dg0, uint64_t prefix, Rec& R,
                                         uint32_t& tgt, uint64_t& r) {
  const uint32_t d = (it[1] >> 16) & 63u;
  const uint32_t rb = __shfl(di[0], d, 64);
  const uint32_t base = __shfl(doff, d, 64), len = __shfl(dlen, d, 64);
  const uint32_t pf0 = __shfl(di[1], d, 64), pf1 = __shfl(di[2], d, 64), pf2 = __shfl(di[3], d, 64);
  r = ~0ull;
  tgt = RTPS_NO_TARGET;
  if (!act || (rb & DI_NOREC)) return;  // (a datagram dropped after this item)
  const uint32_t o = it[0] & 0xffffu, src_off = it[0] >> 16;
  const uint32_t j = it[1] & 0xffffu, kind = it[1] >> 24;
  Src s = s0;
  s.base = base;
  Win W;
  {
    const u32x4 a = ld16(s, o);
    u32x4 bq = {0u, 0u, 0u, 0u};
    if (win_needs_tail<true>(kind)) bq = ld16(s, o + 16u);
    W.w[0] = a[0]; W.w[1] = a[1]; W.w[2] = a[2]; W.w[3] = a[3];
    W.w[4] = bq[0]; W.w[5] = bq[1]; W.w[6] = bq[2]; W.w[7] = bq[3];
    W.w[8] = kind == RTPS_DATA_FRAG ? ld4(s, o + 32u) : 0u;
    W.w[9] = 0u; W.w[10] = 0u; W.w[11] = 0u;
  }
  Interp st;
  if (src_off == 8u) {
    st.src0 = pf0; st.src1 = pf1; st.src2 = pf2;
  } else {  // an INFO_SRC's prefix is in effect
    const u32x4 q = ld16(s, src_off);
    st.src0 = q[0]; st.src1 = q[1]; st.src2 = q[2];
  }
  st.dst_ok = ((it[1] >> 22) & 1u) != 0u;
  st.ts_valid = ((it[1] >> 23) & 1u) != 0u;
  st.ts_sec = it[2];
  st.ts_frac = it[3];
  const uint32_t flags = (W.w[0] >> 8) & 0xffu;
  const bool le = (flags & 1u) != 0u;
  const uint32_t eff = eff_len(kind, e16(W.w[0], 1, le), len - o);
  rec_clear(R);
  SubOut so;
  sub_body<true, RTPS_TRUSTED_WRITE != 0>(s, W, kind, flags, le, o + 4u, eff, R, so);  // validated by E's walk
  R.d[0] = dg0 + d;
  R.d[1] = o | (kind << 16) | (flags << 24);
  tgt = rec_finish(p, R, so, kind, st);
  r = prefix + rb + j;
}

// ---------------------------------------------------------------------------
// W2 rtps_parse_emit2_kernel: wave w of a workgroup takes E's wave slab w of each tile
// of its grid stride.  The reader tables are staged once per workgroup; after that no
// wave waits for another (no barrier, no per-tile prologue scan).  The per-datagram
// prologue is one coalesced 16-B word E wrote (dinfo: the datagram's tile-local first
// record, its header prefix) plus the (offset, length) arrays: lane l holds datagram l
// of the slab, and an item takes its datagram's fields with lane permutes.  The
// descriptor base is E's (the arena, or for large arenas the wave's smallest offset),
// so every datagram E walked is addressable here.
// Records are taken in RECORD ORDER: the wave first maps its records to their slab positions
// in LDS (record q of the wave = item k, from the item's datagram and index j), then takes
// them 64 at a time: the 64 lanes of a round read neighbouring submessages (a datagram's
// submessages share lines and DRAM rows) and their 64 records are 4 KB back to back, stored
// through a 1-KB LDS stage so that each store instruction writes 1 KB of consecutive bytes.
// (Slab order, E's walk-step-major order, measured 254 us against 210 on C3)
#ifndef RTPS_EM2_WAVES_PER_SIMD
#define RTPS_EM2_WAVES_PER_SIMD 6  // 80 VGPRs, no spill (the LDS caps the CU at 24 waves anyway)
#endif
#ifndef RTPS_EM2_TRANSPOSE
#define RTPS_EM2_TRANSPOSE 1  // 0: per-lane 64-B record stores (measured slower)
#endif
#ifndef RTPS_EM2_NT  // W2's record stores streamed: C3 W2 188 -> 177 us (round 5)
#define RTPS_EM2_NT 1
#endif
#ifndef RTPS_EM2_THREADS
#define RTPS_EM2_THREADS 512  // two tiles per workgroup (one reader-table copy for 8 waves; 256 / 768: slower)
#endif
constexpr uint32_t EM2T = RTPS_EM2_THREADS, EM2_TPB = EM2T / TILE;
static_assert(EM2T % TILE == 0, "whole tiles per workgroup");
// Tile order of W2's grid stride.  0: ascending.  1: descending, so that the first tiles W2
// takes are the last E walked (their lines and items are the likeliest still in the Infinity
// Cache).  2: descending inside each XCD: workgroup b (XCD b % 8, as the dispatcher deals
// workgroups round robin) takes only tiles t = b (mod 8), the ones E's workgroup t walked on
// the same XCD, so E's items and dinfo words can still be in that XCD's L2.
#ifndef RTPS_EM2_ORDER
#define RTPS_EM2_ORDER 2  // C3 step 316 -> 307 us, W2 168 -> 165.4 (1: 309.5 us; scripts/gpu_variant_ab.sh)
#endif
constexpr uint32_t XCDS = 8;
struct Em2Seq {  // the tiles one wave of a W2 workgroup takes, in order
  uint32_t x, step, mx, n_tiles;  // ORDER 2: its XCD, stride, tiles of that XCD
  uint32_t m;                     // position in the sequence
};
__device__ __forceinline__ Em2Seq em2_seq(uint32_t n_tiles, uint32_t sub) {
  Em2Seq q;
  q.n_tiles = n_tiles;
  if (RTPS_EM2_ORDER == 2 && gridDim.x % XCDS == 0) {
    q.x = blockIdx.x % XCDS;
    q.step = (gridDim.x / XCDS) * EM2_TPB;
    q.m = (blockIdx.x / XCDS) * EM2_TPB + sub;
    q.mx = n_tiles > q.x ? (n_tiles - q.x + XCDS - 1) / XCDS : 0u;
  } else {
    q.x = ~0u;
    q.step = gridDim.x * EM2_TPB;
    q.m = blockIdx.x * EM2_TPB + sub;
    q.mx = n_tiles;
  }
  return q;
}
__device__ __forceinline__ bool em2_more(const Em2Seq& q) { return q.m < q.mx; }
__device__ __forceinline__ uint32_t em2_tile(const Em2Seq& q) {
  if (q.x != ~0u) return q.x + XCDS * (q.mx - 1u - q.m);
  return RTPS_EM2_ORDER ? q.n_tiles - 1u - q.m : q.m;
}
__global__ __launch_bounds__(EM2T, RTPS_EM2_WAVES_PER_SIMD) void rtps_parse_emit2_kernel(
    KParams p, uint32_t n_tiles, const u32x4* __restrict__ items, const uint32_t* __restrict__ wcnt,
    const uint64_t* __restrict__ tprefix, const u32x4* __restrict__ dinfo) {
  static_assert(!RTPS_IT_WIDE, "W2 takes 16-B items");
  __shared__ uint16_t s_map[(EM2T / 64u) * CAPW];  // the waves' record -> slab position maps
#if RTPS_EM2_TRANSPOSE
  __shared__ u32x4 s_stage[(EM2T / 64u) * 64u];    // 1 KB per wave
#endif
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t wave = wv % WAVES, sub = wv / WAVES;  // the wave's slab in its tile, the workgroup's tile
  uint16_t* map = s_map + wv * CAPW;
  mt_stage(p);
  __syncthreads();
  for (Em2Seq sq = em2_seq(n_tiles, sub); em2_more(sq); sq.m += sq.step) {
    const uint32_t tile = em2_tile(sq);
    const uint32_t wc = __builtin_amdgcn_readfirstlane(wcnt[tile * WAVES + wave]);
    const uint64_t prefix = tprefix[tile];
    TileCtx t;
    tile_src(p, tile, t, true, wave * 64u + lane);
    const u32x4 di = t.valid ? dinfo[t.i] : u32x4{DI_NOREC, 0u, 0u, 0u};
    const uint32_t first = di[0] & ~DI_NOREC;
    if (t.valid && p.rec_begin) p.rec_begin[t.i] = (uint32_t)(prefix + first);
    if (wc & WCNT_OVERFLOW) continue;  // walked below
    const u32x4* slab = items + (size_t)(tile * WAVES + wave) * CAPW;
    const uint32_t doff = t.s.base, dlen = t.L;
    const uint32_t dg0 = tile * TILE + wave * 64u;
    // record q of the wave (q = the datagram's first record - the wave's + j) <- slab position k
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(first);  // lane 0: the wave's first record
    uint32_t nr = 0;
    for (uint32_t b = 0; b < wc; b += 64u) {
      const uint32_t k = b + lane;
      const uint32_t m1 = k < wc ? slab[k][1] : 0u;
      const uint32_t rb = __shfl(di[0], (m1 >> 16) & 63u, 64);
      const bool keep = k < wc && !(rb & DI_NOREC);
      if (keep) map[rb - wbase + (m1 & 0xffffu)] = (uint16_t)k;
      nr += (uint32_t)__popcll(__ballot(keep));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t b = 0; b < nr; b += 64u) {
      const uint32_t q = b + lane;
      const bool act = q < nr;
      const u32x4 it = act ? slab[map[q]] : u32x4{0u, 0u, 0u, 0u};
      Rec R;
      uint32_t tgt;
      uint64_t r;
      em2_item(p, t.s, it, act, di, doff, dlen, dg0, prefix, R, tgt, r);
      // lane l holds record r0 + l: the 64 records are 4 KB back to back
      const uint64_t r0 = prefix + wbase + b;
      const uint32_t nact = nr - b < 64u ? nr - b : 64u;
      if (p.target_out && r < p.max_records) p.target_out[r] = tgt;
#if RTPS_EM2_TRANSPOSE
      // through the wave's 1-KB stage, a quarter of the records at a time: lanes 16c .. 16c+15
      // write their records, then every lane stores 16 B of them, so each store instruction
      // writes 1 KB of consecutive records
      u32x4* stg = s_stage + wv * 64u;
#pragma unroll
      for (uint32_t c = 0; c < 4u; ++c) {
        if ((lane >> 4) == c) {
          u32x4* q4 = stg + (lane & 15u) * 4u;
          q4[0] = u32x4{R.d[0], R.d[1], R.d[2], R.d[3]};
          q4[1] = u32x4{R.d[4], R.d[5], R.d[6], R.d[7]};
          q4[2] = u32x4{R.d[8], R.d[9], R.d[10], R.d[11]};
          q4[3] = u32x4{R.d[12], R.d[13], R.d[14], R.d[15]};
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const u32x4 v = stg[lane];
        const uint32_t rl = 16u * c + (lane >> 2);  // the record (of the 64) whose quarter lane l stores
        if (rl < nact && r0 + rl < p.max_records) {
#if RTPS_EM2_NT
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p.records + r0 + rl) + (lane & 3u));
#else
          reinterpret_cast<u32x4*>(p.records + r0 + rl)[lane & 3u] = v;
#endif
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads before the next quarter's writes
        __builtin_amdgcn_wave_barrier();
      }
#else
      if (r < p.max_records) rec_store(p.records + r, R);
#endif
      (void)r0; (void)nact;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // map reads before the next tile's writes
    __builtin_amdgcn_wave_barrier();
  }
  // slabs whose items did not fit (rare): walk the wave's datagrams, after the item loop so
  // that its registers do not carry the walk's
  for (Em2Seq sq = em2_seq(n_tiles, sub); em2_more(sq); sq.m += sq.step) {
    const uint32_t tile = em2_tile(sq);
    if (!(wcnt[tile * WAVES + wave] & WCNT_OVERFLOW)) continue;
    TileCtx th;
    load_tile(p, tile, th, true, wave * 64u + lane);
    const uint32_t di0 = th.valid ? dinfo[th.i][0] : DI_NOREC;
    if (th.valid && !(di0 & DI_NOREC)) {
      uint32_t n2;
      walk<true>(p, th.s, th.H, th.L, th.i, tprefix[tile] + di0, n2);
    }
  }
}

#ifdef RTPS_DIAG_PASSES  // the measured, rejected passes for mixed traffic (variant builds)
#include "diag/mixed_passes.inc"
#endif
#ifdef RTPS_ITEM_DIAG  // diagnostic variant builds only (scripts/diag_item_pass.py)
#include "diag/item_pass_kernel.inc"
#endif

// device-side synthetic generator: one lane per datagram
__global__ void rtps_gen_kernel(int wl, uint64_t seed, uint64_t first_idx, uint32_t n_writers,
                                uint8_t* arena, const uint64_t* off, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rtps_gen_datagram(wl, seed, first_idx + i, n_writers, arena + off[i]);
}


// ---------------------------------------------------------------------------
// writer-GUID sharding for >= 2 GPUs: stable partition of
// the writer/reader-kind records by owner = owner_hash(prefix || writer_id) %
// n_dest.  Three launches: per-tile histogram, per-destination scan over
// tiles, stable scatter (wave ballots keep input order inside a bucket).
// ---------------------------------------------------------------------------
constexpr uint32_t MAX_DEST = 64;

// Owner rank of a writer GUID: FNV-1a over its four words, then the murmur3
// finaliser (fmix32).  The match table's fold (h ^ h >> 15) leaves the low bits
// tied to a few input bits: over C3's 256 writers it splits 25 / 75 % at 2 ranks,
// fmix32 within 5 %.
__device__ __forceinline__ uint32_t owner_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = 0x811c9dc5u;
  h = (h ^ a) * 0x01000193u; h = (h ^ b) * 0x01000193u;
  h = (h ^ c) * 0x01000193u; h = (h ^ d) * 0x01000193u;
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}

__device__ __forceinline__ uint32_t owner_of(const rtps_record* r, uint32_t n_dest) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(r);
  uint32_t kind = (d[1] >> 16) & 0xffu;
  bool exch = kind == RTPS_DATA || kind == RTPS_DATA_FRAG || kind == RTPS_HEARTBEAT || kind == RTPS_GAP ||
              kind == RTPS_HEARTBEAT_FRAG || kind == RTPS_ACKNACK || kind == RTPS_NACK_FRAG;
  if (!exch) return 0xffffffffu;
  return owner_hash(d[2], d[3], d[4], d[5]) % n_dest;
}

// descriptor mode: writer records that reach a reader (MATCHED, or TARGETED by entity id
// only: the proxy-less samples a reader accepts from non-user-defined writers,
// reader.rs:734-739), owner = target set index % n_dest
struct DescOwner {
  ReaderDev rt;
};
__device__ __forceinline__ uint32_t desc_entry(const rtps_record* r, const DescOwner& m) {
  if (!(r->route & (RTPS_ROUTE_MATCHED | RTPS_ROUTE_TARGETED))) return 0xffffffffu;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(r);
  uint32_t r2 = 0;
  const uint32_t t = rt_classify<false>(m.rt, nullptr, d[2], d[3], d[4], d[5], r2);
  return t == RTPS_NO_TARGET ? 0xffffffffu : t;
}
template <bool DESC>
__device__ __forceinline__ uint32_t owner_sel(const rtps_record* r, uint32_t n_dest, const DescOwner& m) {
  if (DESC) {
    const uint32_t e = desc_entry(r, m);
    return e == 0xffffffffu ? e : e % n_dest;
  }
  return owner_of(r, n_dest);
}

template <bool DESC>
__global__ __launch_bounds__(TILE) void bucket_hist_kernel(const rtps_record* recs, const uint64_t* n_rec,
                                                            uint32_t n_dest, uint32_t* hist, DescOwner m) {
  __shared__ uint32_t h[MAX_DEST];
  if (threadIdx.x < n_dest) h[threadIdx.x] = 0;
  __syncthreads();
  uint64_t i = (uint64_t)blockIdx.x * TILE + threadIdx.x;
  if (i < *n_rec) {
    uint32_t o = owner_sel<DESC>(recs + i, n_dest, m);
    if (o != 0xffffffffu) atomicAdd(&h[o], 1u);
  }
  __syncthreads();
  if (threadIdx.x < n_dest) hist[(uint64_t)blockIdx.x * n_dest + threadIdx.x] = h[threadIdx.x];
}

// one workgroup per destination d: exclusive scan of hist[t][d] over the tiles
// t (offsets inside bucket d), and the bucket size dest_counts[d]
__global__ __launch_bounds__(TILE) void bucket_scan_kernel(uint32_t* hist, uint32_t tiles, uint32_t n_dest,
                                                            uint64_t* dest_counts) {
  __shared__ uint32_t wsum[WAVES];
  const uint32_t d = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < tiles; t0 += TILE) {
    const uint32_t t = t0 + tid;
    const uint32_t v = t < tiles ? hist[(uint64_t)t * n_dest + d] : 0u;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = carry, total = carry;
    for (uint32_t w = 0; w < WAVES; ++w) {
      if (w < wave) before += wsum[w];
      total += wsum[w];
    }
    if (t < tiles) hist[(uint64_t)t * n_dest + d] = before + incl - v;
    carry = total;
    __syncthreads();
  }
  if (tid == 0) dest_counts[d] = carry;
}

// cap == 0: bucket d starts at sum(dest_counts[0..d)); cap > 0: at d * cap, and
// records at positions >= cap inside their bucket are dropped
template <bool DESC>
__global__ __launch_bounds__(TILE) void bucket_scatter_kernel(const rtps_record* recs, const uint64_t* n_rec,
                                                               uint32_t n_dest, const uint32_t* offs,
                                                               const uint64_t* dest_counts, uint64_t cap,
                                                               void* out_v, DescOwner m) {
  __shared__ uint32_t wcnt[WAVES][MAX_DEST];
  __shared__ uint64_t base[MAX_DEST];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  if (tid == 0) {
    uint64_t acc = 0;
    for (uint32_t d = 0; d < n_dest; ++d) { base[d] = cap ? d * cap : acc; acc += dest_counts[d]; }
  }
  uint64_t i = (uint64_t)blockIdx.x * TILE + tid;
  const uint32_t ent = (DESC && i < *n_rec) ? desc_entry(recs + i, m) : 0xffffffffu;
  uint32_t o = (i < *n_rec) ? (DESC ? (ent == 0xffffffffu ? ent : ent % n_dest) : owner_of(recs + i, n_dest))
                            : 0xffffffffu;
  uint32_t rank = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
  for (uint32_t d = 0; d < n_dest; ++d) {
    uint64_t m = __ballot(o == d);
    if (o == d) rank = (uint32_t)__popcll(m & lt);
    if (lane == 0) wcnt[wave][d] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (o != 0xffffffffu) {
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += wcnt[w][o];
    const uint64_t pos = (uint64_t)offs[(uint64_t)blockIdx.x * n_dest + o] + before + rank;
    if (cap == 0 || pos < cap) {
      if (DESC) {
        const rtps_record* r = recs + i;
        rtps_xdesc x;
        x.sn = r->sn;
        x.rec_idx = (uint32_t)i;
        x.writer_kind = (ent << 8) | r->kind;
        reinterpret_cast<rtps_xdesc*>(out_v)[base[o] + pos] = x;
      } else {
        const u32x4* src = reinterpret_cast<const u32x4*>(recs + i);
        u32x4* dp = reinterpret_cast<u32x4*>(reinterpret_cast<rtps_record*>(out_v) + base[o] + pos);
        u32x4 a = src[0], b = src[1], c = src[2], e = src[3];
        dp[0] = a; dp[1] = b; dp[2] = c; dp[3] = e;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// per-reader DataFrag assembly (rtps_rx_frag_assemble with readers set): every
// reader has its own FragmentAssembler per writer (Reader::fragment_assembler_mutable,
// io_uring/rtps/reader.rs:617-619, 638-647), fed the DATA_FRAGs Domain::handle_event
// routes to it (dp_event_loop.rs:266-327) minus those its Lifespan drops
// (handle_datafrag_msg :578-589).  The batch is expanded into one copy of each
// such record per target reader, the reader word (slot | 0x10000) in the copy's
// reader_id; the assembly keys (rtps_frag.hip) include that word.
// ---------------------------------------------------------------------------
constexpr int64_t NO_LIFESPAN = INT64_MAX;
struct FragX {
  const rtps_record* recs;
  const uint64_t* n_rec;
  uint64_t max;
  ReaderDev rt;
  const int64_t* life;   // [65536] Lifespan of reader slot s in Duration ticks, NO_LIFESPAN: none
  uint64_t recv_ticks;   // Timestamp::now() of the batch as ticks (seconds << 32 | fraction)
  uint32_t any_life;
  uint32_t* cnt;         // [max] copies of record i
  uint32_t* off;         // [max] exclusive scan of cnt
  rtps_record* xrec;     // [max_x] the copies
  uint32_t* emap;        // [max_x] copy -> record
  uint64_t* n_x;
};
// the target-set entries [b, e) of a DATA_FRAG record the user readers receive, or b == e
__device__ __forceinline__ void frag_targets(const FragX& a, const rtps_record* r, uint32_t& b, uint32_t& e) {
  b = e = 0;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(r);
  const uint32_t kind = (d[1] >> 16) & 0xffu, route = (d[7] >> 16) & 0xffu;
  if (kind != RTPS_DATA_FRAG || !(route & RTPS_ROUTE_PASS) || !(route & RTPS_ROUTE_TARGETED) ||
      (route & RTPS_ROUTE_BUILTIN))
    return;
  uint32_t r2 = 0;
  const uint32_t set = rt_classify<false>(a.rt, nullptr, d[2], d[3], d[4], d[5], r2);
  if (set == RTPS_NO_TARGET) return;
  b = a.rt.set_first[set];
  e = a.rt.set_first[set + 1];
}
// Lifespan check of handle_datafrag_msg (reader.rs:578-589): a source timestamp and a
// Lifespan, and lifespan.duration < receive_timestamp.duration_since(source)
// (structure/time.rs:85-113: wrapping tick difference as i64; Duration orders as ticks)
__device__ __forceinline__ bool frag_expired(const FragX& a, const rtps_record* r, uint32_t slot) {
  if (!a.any_life) return false;
  const int64_t L = a.life[slot];
  if (L == NO_LIFESPAN || !(r->route & RTPS_ROUTE_TS_VALID)) return false;
  const uint64_t src = ((uint64_t)r->ts_sec << 32) | r->ts_frac;
  return L < (int64_t)(a.recv_ticks - src);
}
__global__ __launch_bounds__(TILE) void frag_x_count(FragX a) {
  const uint64_t n = *a.n_rec < a.max ? *a.n_rec : a.max;
  for (uint64_t i = (uint64_t)blockIdx.x * TILE + threadIdx.x; i < a.max; i += (uint64_t)gridDim.x * TILE) {
    uint32_t c = 0;
    if (i < n) {
      uint32_t b, e;
      frag_targets(a, a.recs + i, b, e);
      for (uint32_t k = b; k < e; ++k) c += frag_expired(a, a.recs + i, a.rt.set_ent[k].reader_slot) ? 0u : 1u;
    }
    a.cnt[i] = c;
  }
}
__global__ __launch_bounds__(TILE) void frag_x_fill(FragX a) {
  const uint64_t n = *a.n_rec < a.max ? *a.n_rec : a.max;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.n_x = a.max ? (uint64_t)a.off[a.max - 1] + a.cnt[a.max - 1] : 0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * TILE + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TILE) {
    if (!a.cnt[i]) continue;
    uint32_t b, e;
    frag_targets(a, a.recs + i, b, e);
    const rtps_record* r = a.recs + i;
    uint32_t w[16];
    const u32x4* q = reinterpret_cast<const u32x4*>(r);
#pragma unroll
    for (int k = 0; k < 4; ++k) { const u32x4 v = q[k]; w[4 * k] = v[0]; w[4 * k + 1] = v[1]; w[4 * k + 2] = v[2]; w[4 * k + 3] = v[3]; }
    uint32_t o = a.off[i];
    for (uint32_t k = b; k < e; ++k) {
      const uint32_t slot = a.rt.set_ent[k].reader_slot;
      if (frag_expired(a, r, slot)) continue;
      w[6] = slot | 0x10000u;  // reader_id: the reader word of the assembly key
      u32x4* d = reinterpret_cast<u32x4*>(a.xrec + o);
      d[0] = u32x4{w[0], w[1], w[2], w[3]}; d[1] = u32x4{w[4], w[5], w[6], w[7]};
      d[2] = u32x4{w[8], w[9], w[10], w[11]}; d[3] = u32x4{w[12], w[13], w[14], w[15]};
      a.emap[o] = (uint32_t)i;
      ++o;
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
struct rtps_rx_ctx {
  int device = 0;
  uint8_t own[12] = {0};
  uint32_t max_datagrams = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint64_t* scratch = nullptr;  // per-tile counts / prefixes (Scratch)
  size_t scratch_words = 0;
  ReaderTable* readers = nullptr;  // local readers -> target sets (rtps_readers.h)
  uint32_t* bucket_hist = nullptr;
  size_t bucket_bytes = 0;
  uint32_t resident_blocks = 1024;
  uint32_t launch_parity = 0;
  uint32_t k_spec = 1;  // speculated records per datagram (0 disables nothing: see set_spec_hint)
  FragState* frag = nullptr;  // DataFrag reassembly state (created on first use)
  IngestState* ingest = nullptr;  // history-cache ingest state (created on first use)
  TopicState* topics = nullptr;   // topic caches (created on first use)
  uint64_t* chain = nullptr;      // look-back words of the chained launch [chain_words(tiles) + 2]
  uint32_t* mixed = nullptr;      // pinned: {mixed tiles, tiles} of the last finished batch (kernel B)
#ifdef RTPS_DIAG_PASSES
  uint32_t ch_spin_limit = CH_SPIN_LIMIT;
#else
  uint32_t ch_spin_limit = 0;
#endif
  uint32_t ch_epoch = 0;          // last chained launch's epoch (words start zeroed: epoch 0 is never used)
  uint32_t chain_tiles = 0;       // tiles the chain words are sized for
  uint32_t mixed_pass = 2;        // pass for mixed traffic: 2 = the item pass (E / S / W2); diagnostic builds
                                  // (RTPS_DIAG_PASSES): 0 = chained lane walk (C), 1 = LDS tiles (D), 3 = E' / W'
  u32x4* it_items = nullptr;      // item pass: wave slabs [tiles * WAVES * CAPW]
  uint32_t* it_wcnt = nullptr;    // item pass: items per wave slab [tiles * WAVES]
  uint64_t* it_prefix = nullptr;  // item pass: tile record prefixes [tiles]
  u32x4* it_dinfo = nullptr;      // item pass: per-datagram prologue of the record pass [tiles * TILE]
  uint64_t* tc_ovf = nullptr;     // device u64: the ingest's window overflows when the caller asks for none
  uint64_t readers_version = 0;   // bumped by set_readers / set_match_table / set_topics (owner tables follow it)
  uint32_t emit = 2;              // record pass: 2 = W2 (rtps_parse_emit2_kernel); 1 = round 4's W (diagnostic builds)
  uint32_t emit_grid = 0, emit_grid_lds = ~0u;  // W2's resident grid and the LDS size it was computed for
  uint32_t it_tiles = 0;          // tiles the item-pass buffers are sized for
  u32x4* rs_recs = nullptr;       // (diagnostic builds) record-slab pass: wave slabs of records
  uint32_t* rs_meta = nullptr;    //   (j | lane << 16) per slab record
  uint32_t* rs_tgt = nullptr;     //   target set per slab record
  uint32_t* rs_wcnt = nullptr;    //   records per wave slab
  uint64_t* rs_prefix = nullptr;  //   tile record prefixes
  uint32_t rs_tiles = 0;
  // per-reader DataFrag assembly (frag_x_*): Lifespans by reader slot, the batch's receive time, the expansion
  int64_t* life = nullptr;        // [65536] device, NO_LIFESPAN where none
  bool any_life = false;
  uint64_t recv_ns = 0;           // rtps_rx_frag_set_receive_time (0: the host's clock at each assemble)
  uint32_t *fx_cnt = nullptr, *fx_off = nullptr, *fx_emap = nullptr;
  rtps_record* fx_rec = nullptr;
  uint64_t* fx_n = nullptr;
  uint64_t fx_cap = 0, fx_xcap = 0;
  void* fx_tmp = nullptr;
  size_t fx_tmp_bytes = 0;
  std::vector<rtps_shard*> shards;  // owner-side exchanges created on this context (rtps_ctx_shard_attach)
};

uint64_t rtps_ctx_readers_version(const rtps_rx_ctx* c) { return c->readers_version; }

void rtps_ctx_owner_keys(const rtps_rx_ctx* c, bool by_topic, std::vector<uint8_t>& keys,
                         std::vector<uint32_t>& group) {
  uint32_t nw = 0, ne = 0;
  const uint8_t* g = c->readers ? rt_writer_guids(c->readers, &nw) : nullptr;
  const uint8_t* e = (by_topic && c->readers) ? rt_entity_ids(c->readers, &ne) : nullptr;
  keys.assign(g, g + 16ull * nw);
  for (uint32_t k = 0; k < ne; ++k) {  // entity keys: OWNER_EKEY_PREFIX x 12, then the entity id
    keys.insert(keys.end(), 12, OWNER_EKEY_PREFIX);
    keys.insert(keys.end(), e + 4ull * k, e + 4ull * k + 4);
  }
  const uint32_t nk = nw + ne;
  group.resize(nk);
  for (uint32_t w = 0; w < nk; ++w) group[w] = w;
  if (!by_topic || !nk) return;
  const uint32_t* first = nullptr;
  const rtps_target* ent = nullptr;
  uint32_t n_sets = 0;
  rt_host(c->readers, &first, &ent, &n_sets);
  auto root = [&](uint32_t x) {
    while (group[x] != x) x = group[x] = group[group[x]];
    return x;
  };
  std::vector<uint32_t> topic_key;  // topic cache -> the first key seen feeding it
  std::vector<uint32_t> topic;      // (parallel) topic cache ids
  // key w is target set w: writer sets first, then entity sets (rtps_readers.cpp)
  for (uint32_t w = 0; w < nk && w < n_sets; ++w)
    for (uint32_t k = first[w]; k < first[w + 1]; ++k) {
      // the reader's topic cache: a configured topic, or its own (no topics set: one per slot)
      const uint32_t t = c->topics ? rtps_topic_of_slot(c->topics, ent[k].reader_slot) : ent[k].reader_slot;
      uint32_t j = 0;
      while (j < topic.size() && topic[j] != t) ++j;
      if (j == topic.size()) { topic.push_back(t); topic_key.push_back(w); continue; }
      const uint32_t a = root(w), b = root(topic_key[j]);
      if (a != b) group[a > b ? a : b] = a < b ? a : b;  // the smaller index is the root
    }
  for (uint32_t w = 0; w < nk; ++w) group[w] = root(w);
}

bool rtps_ctx_topics_configured(const rtps_rx_ctx* c) { return c->topics && rtps_topic_n_configured(c->topics) > 0; }

void rtps_ctx_shard_attach(rtps_rx_ctx* c, rtps_shard* s, bool attach) {
  auto& v = c->shards;
  v.erase(std::remove(v.begin(), v.end(), s), v.end());
  if (attach) v.push_back(s);
}

bool rtps_ctx_topic_split(const rtps_rx_ctx* c) {
  for (const rtps_shard* s : c->shards)
    if (rtps_shard_splits_topics(s)) return true;
  return false;
}

static int hip_fail(hipError_t e) { return e == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP; }
#ifdef RTPS_DIAG_PASSES
#include "diag/mixed_passes_host.inc"
#endif

extern "C" {

int rtps_rx_create(const rtps_rx_config* cfg, rtps_rx_ctx** out_ctx) {
  if (!cfg || !out_ctx) return RTPS_RX_EINVAL;
  if (cfg->abi_version != RTPS_RX_ABI_VERSION) return RTPS_RX_EABI;
  rtps_rx_ctx* c = new (std::nothrow) rtps_rx_ctx();
  if (!c) return RTPS_RX_ENOMEM;
  c->device = cfg->device;
  memcpy(c->own, cfg->own_prefix, 12);
  c->max_datagrams = cfg->max_datagrams;
  if (hipSetDevice(c->device) != hipSuccess) { delete c; return RTPS_RX_EHIP; }
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) { delete c; return RTPS_RX_EHIP; }
  c->stream = c->own_stream;
#ifdef RTPS_DIAG_PASSES
  if (const char* e = getenv("RTPS_RX_MIXED_PASS"))  // A/B measurements
    c->mixed_pass = (e[0] == '1') ? 1u : (e[0] == '0') ? 0u : (e[0] == '3') ? 3u : 2u;
  if (const char* e = getenv("RTPS_RX_EMIT"))  // A/B measurements of the record pass
    c->emit = (e[0] == '1') ? 1u : 2u;
#endif
  {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess && cus > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rtps_parse_fix_kernel<TILE>, TILE, 0) == hipSuccess &&
        per_cu > 0)
      c->resident_blocks = (uint32_t)cus * (uint32_t)per_cu;
  }
#ifdef RTPS_DIAG_PASSES  // scratch and look-back words sized for the smallest tile (LT datagrams, kernel D)
  size_t tiles = ((size_t)cfg->max_datagrams + LT - 1) / LT;
  const size_t chain_bytes = chain_words((uint32_t)(tiles ? tiles : 1)) * sizeof(uint64_t);
#else
  size_t tiles = ((size_t)cfg->max_datagrams + TILE - 1) / TILE;
  const size_t chain_bytes = 16;
#endif
  if (tiles == 0) tiles = 1;
  // u32 flag[4] | u32 info[tiles rounded to 4] | u16 dcount[max_datagrams]
  c->scratch_words = 2 + ((tiles + 3) & ~(size_t)3) / 2 + ((size_t)cfg->max_datagrams + 3) / 4 + 2;
  if (hipMalloc(&c->scratch, c->scratch_words * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->scratch, 0, c->scratch_words * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&c->chain, chain_bytes) != hipSuccess || hipMemset(c->chain, 0, chain_bytes) != hipSuccess ||
      hipHostMalloc(&c->mixed, 2 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
    (void)hipFree(c->scratch);
    (void)hipFree(c->chain);
    if (c->mixed) (void)hipHostFree(c->mixed);
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return RTPS_RX_ENOMEM;
  }
  c->mixed[0] = c->mixed[1] = 0u;
  c->chain_tiles = (uint32_t)tiles;
  *out_ctx = c;
  return RTPS_RX_OK;
}

int rtps_rx_destroy(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->scratch);
  (void)hipFree(c->chain);
  if (c->mixed) (void)hipHostFree(c->mixed);
  rt_free(c->readers);
  (void)hipFree(c->bucket_hist);
  rtps_frag_state_free(c->frag);
  rtps_ingest_state_free(c->ingest);
  rtps_topic_state_free(c->topics);
  {
    void* it[] = {c->it_items, c->it_wcnt, c->it_prefix, c->it_dinfo, c->rs_recs, c->rs_meta, c->rs_tgt, c->rs_wcnt,
                  c->rs_prefix, c->tc_ovf};
    for (void* q : it) if (q) (void)hipFree(q);
  }
  {
    void* fx[] = {c->life, c->fx_cnt, c->fx_off, c->fx_emap, c->fx_rec, c->fx_n, c->fx_tmp};
    for (void* q : fx) if (q) (void)hipFree(q);
  }
  (void)hipStreamDestroy(c->own_stream);
  delete c;
  return RTPS_RX_OK;
}

int rtps_rx_set_stream(rtps_rx_ctx* c, void* s) {
  if (!c) return RTPS_RX_EINVAL;
  c->stream = (s == RTPS_RX_OWN_STREAM) ? c->own_stream : (hipStream_t)s;
  return RTPS_RX_OK;
}

static int readers_table(rtps_rx_ctx* c) {
  if (!c->readers) c->readers = rt_new();
  return c->readers ? RTPS_RX_OK : RTPS_RX_ENOMEM;
}

// the topic caches follow the readers (which topics have one reader, fresh proxies)
static int topics_follow(rtps_rx_ctx* c) {
  if (!c->topics) return RTPS_RX_OK;
  const uint32_t* first = nullptr;
  const rtps_target* ent = nullptr;
  uint32_t n_sets = 0;
  rt_host(c->readers, &first, &ent, &n_sets);
  return rtps_topic_readers_changed(c->topics, first, ent, n_sets, c->stream);
}

int rtps_rx_set_readers(rtps_rx_ctx* c, const rtps_reader* readers, uint32_t n_readers, const rtps_proxy* proxies,
                        uint32_t n_proxies) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  c->readers_version++;
  int rc = readers_table(c);
  if (!rc) rc = rt_set(c->readers, readers, n_readers, proxies, n_proxies, c->stream);
  return rc ? rc : topics_follow(c);
}

int rtps_rx_set_match_table(rtps_rx_ctx* c, const rtps_match* t, uint32_t n) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  c->readers_version++;
  int rc = readers_table(c);
  if (!rc) rc = rt_set_match(c->readers, t, n, c->stream);
  return rc ? rc : topics_follow(c);
}

static int topics_state(rtps_rx_ctx* c) {
  if (c->topics) return RTPS_RX_OK;
  c->topics = rtps_topic_state_new(c->device);
  if (!c->topics) return RTPS_RX_ENOMEM;
  const uint32_t* first = nullptr;
  const rtps_target* ent = nullptr;
  uint32_t n_sets = 0;
  if (c->readers) rt_host(c->readers, &first, &ent, &n_sets);
  return rtps_topic_configure(c->topics, nullptr, 0, nullptr, 0, first, ent, n_sets, c->stream);
}

int rtps_rx_set_topics(rtps_rx_ctx* c, const rtps_topic* topics, uint32_t n_topics, const rtps_topic_reader* readers,
                       uint32_t n_readers) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  c->readers_version++;
  int rc = topics_state(c);
  if (rc) return rc;
  const uint32_t* first = nullptr;
  const rtps_target* ent = nullptr;
  uint32_t n_sets = 0;
  if (c->readers) rt_host(c->readers, &first, &ent, &n_sets);
  return rtps_topic_configure(c->topics, topics, n_topics, readers, n_readers, first, ent, n_sets, c->stream);
}

int rtps_rx_topic_gc(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  if (!c->topics) return RTPS_RX_OK;
  (void)hipSetDevice(c->device);
  return rtps_topic_gc(c->topics, c->stream);
}

int rtps_rx_target_table(const rtps_rx_ctx* c, const uint32_t** first, const rtps_target** entries, uint32_t* n_sets) {
  if (!c) return RTPS_RX_EINVAL;
  rt_host(c->readers, first, entries, n_sets);
  return RTPS_RX_OK;
}

// phases: 1 = the first kernel (A, or the item pass's walk E), 2 = the finishing kernels (B, or
// the item pass's scan S and record pass W2; 2 | 4: W2 alone); *first_kernel (optional): the
// first kernel chosen, 1 = A (rtps_parse_spec_kernel), 4 = E (rtps_parse_item_kernel); the
// diagnostic builds' rejected passes (RTPS_DIAG_PASSES): 2 = C, 3 = D, 5 = E'
static int parse_launch(rtps_rx_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                        const uint32_t* dgram_len, uint32_t n, const rtps_rx_out* out, uint32_t phases,
                        uint32_t* first_kernel) {
  if (!c || !out || !out->status || !out->records || !out->n_records) return RTPS_RX_EINVAL;
  if (n && (!arena || !dgram_off || !dgram_len)) return RTPS_RX_EINVAL;
  if (n > c->max_datagrams) return RTPS_RX_ETOOBIG;
  (void)hipSetDevice(c->device);
  if (n == 0) return hip_fail(hipMemsetAsync(out->n_records, 0, sizeof(uint64_t), c->stream));
  uint32_t tiles = (n + TILE - 1) / TILE;  // one tile = one workgroup = 256 datagrams
  KParams p;
  p.arena = arena;
  p.arena_len = arena_len;
  p.dgram_off = dgram_off;
  p.dgram_len = dgram_len;
  p.n = n;
  memcpy(&p.own0, c->own + 0, 4);
  memcpy(&p.own1, c->own + 4, 4);
  memcpy(&p.own2, c->own + 8, 4);
  p.status = out->status;
  p.records = out->records;
  p.max_records = out->max_records;
  p.target_out = out->target;
  p.rec_begin = out->rec_begin;
  p.n_records = out->n_records;
  p.rt = rt_dev(c->readers);
  p.rt_lds = rt_fits_lds(p.rt) ? 1u : 0u;
  p.scratch = c->scratch;
  const uint32_t parity = c->launch_parity;
  const uint32_t mt_lds = p.rt_lds ? rt_lds_bytes(p.rt.gmask + 1u, p.rt.emask + 1u) : 0u;
  c->launch_parity ^= 1u;
  p.chain = c->chain;
  p.mixed_out = c->mixed;
  p.ch_spin_limit = c->ch_spin_limit;
  p.ch_epoch = 0u;  // set below for a chained launch (diagnostic builds)
  // Launch choice, a performance decision only (both give the same output): the item
  // pass for mixed traffic when the spec hint is 0, or when most tiles of the last
  // finished batch were mixed (reported to pinned memory; read without a sync, so it
  // may lag a batch); else the speculative pass.
  const uint32_t mixed = __atomic_load_n(&c->mixed[0], __ATOMIC_RELAXED);
  const uint32_t seen = __atomic_load_n(&c->mixed[1], __ATOMIC_RELAXED);
  const bool mixed_traffic = c->k_spec == 0 || (seen >= 16u && 2u * mixed > seen);
  const uint32_t k = c->k_spec ? c->k_spec : 1u;
  const bool item = mixed_traffic && c->mixed_pass == 2u;
#ifdef RTPS_DIAG_PASSES
  if (mixed_traffic && !item) {
    const int rc = diag_mixed_launch(c, p, tiles, k, parity, mt_lds, phases, first_kernel);
    return rc;
  }
#endif
  if (first_kernel) *first_kernel = item ? 4u : 1u;
  if (item) {  // E (phases 1), then S and W2 (phases 2); no kernel B
    if (tiles > c->it_tiles || !c->it_items) {
      if (hipStreamSynchronize(c->stream) != hipSuccess) return RTPS_RX_EHIP;
      void* q[] = {c->it_items, c->it_wcnt, c->it_prefix, c->it_dinfo};
      for (void* b : q) if (b) (void)hipFree(b);
      c->it_items = nullptr; c->it_wcnt = nullptr; c->it_prefix = nullptr; c->it_dinfo = nullptr; c->it_tiles = 0;
      const uint32_t t = (uint32_t)(((size_t)c->max_datagrams + TILE - 1) / TILE) > tiles
                             ? (uint32_t)(((size_t)c->max_datagrams + TILE - 1) / TILE) : tiles;
      if (hipMalloc(&c->it_items, (size_t)t * WAVES * CAPW * IW * sizeof(u32x4)) != hipSuccess ||
          hipMalloc(&c->it_wcnt, (size_t)t * WAVES * sizeof(uint32_t)) != hipSuccess ||
          hipMalloc(&c->it_prefix, (size_t)t * sizeof(uint64_t)) != hipSuccess ||
          hipMalloc(&c->it_dinfo, (size_t)t * TILE * sizeof(u32x4)) != hipSuccess)
        return RTPS_RX_ENOMEM;
      c->it_tiles = t;
    }
    const bool w2 = c->emit == 2u;  // (1: the round-4 record pass W, diagnostic builds)
    if (w2 && c->emit_grid_lds != mt_lds) {  // resident W2 workgroups for this LDS size
      int cus = 0, per_cu = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rtps_parse_emit2_kernel, EM2T, mt_lds) != hipSuccess)
        return RTPS_RX_EHIP;
      c->emit_grid = (uint32_t)(cus > 0 ? cus : 1) * (uint32_t)(per_cu > 0 ? per_cu : 1);
      c->emit_grid_lds = mt_lds;
    }
    if (phases & 1u)
      hipLaunchKernelGGL(rtps_parse_item_kernel, dim3(tiles), dim3(TILE), 0, c->stream, p, tiles, k, c->it_items,
                         c->it_wcnt, w2 ? c->it_dinfo : nullptr);
    if (phases & 2u) {
      if (!(phases & 4u))  // (4: the record pass alone, on the previous launch's scan: bench.py's timing)
        hipLaunchKernelGGL(rtps_parse_scan_kernel, dim3(1), dim3(SCAN_T), 0, c->stream, p, tiles, parity,
                           c->it_prefix);
      if (w2) {
        const uint32_t groups = (tiles + EM2_TPB - 1) / EM2_TPB;
        const uint32_t g = c->emit_grid < groups ? c->emit_grid : groups;
        hipLaunchKernelGGL(rtps_parse_emit2_kernel, dim3(g), dim3(EM2T), mt_lds, c->stream, p, tiles, c->it_items,
                           c->it_wcnt, c->it_prefix, c->it_dinfo);
      } else {
#ifdef RTPS_DIAG_PASSES
        hipLaunchKernelGGL(rtps_parse_emit_kernel, dim3(tiles), dim3(EMT), mt_lds, c->stream, p, tiles, c->it_items,
                           c->it_wcnt, c->it_prefix);
#else
        return RTPS_RX_EINVAL;
#endif
      }
    }
    return hip_fail(hipGetLastError());
  }
  if (phases & 1u)
    hipLaunchKernelGGL(rtps_parse_spec_kernel, dim3(tiles), dim3(TILE), mt_lds, c->stream, p, tiles, c->k_spec,
                       parity);
  const uint32_t grid = tiles < c->resident_blocks ? tiles : c->resident_blocks;
  if (phases & 2u)
    hipLaunchKernelGGL(rtps_parse_fix_kernel<TILE>, dim3(grid), dim3(TILE), mt_lds, c->stream, p, tiles, k, parity);
  return hip_fail(hipGetLastError());
}

int rtps_rx_parse_batch(rtps_rx_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                        const uint32_t* dgram_len, uint32_t n, const rtps_rx_out* out) {
  return parse_launch(c, arena, arena_len, dgram_off, dgram_len, n, out, 3u, nullptr);
}

/* measurement hook (not part of the public header): launch only the parse's first
   kernel (phases 1) or only the finishing kernels (phases 2: B, or the item pass's S and
   W), so bench.py can time the kernels alone with HIP events.  A full
   rtps_rx_parse_batch afterwards restores the per-launch bookkeeping (run two).  Phases 2 | 4 on
   the item pass: the record pass W alone (the scan S of the previous launch stays valid).
   *first_kernel: 1 = spec (A), 2 = chained (C), 3 = chained LDS tiles (D), 4 = item pass (E). */
int rtps_rx_debug_parse_phases(rtps_rx_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                               const uint32_t* dgram_len, uint32_t n, const rtps_rx_out* out, uint32_t phases,
                               uint32_t* first_kernel) {
  return parse_launch(c, arena, arena_len, dgram_off, dgram_len, n, out, phases, first_kernel);
}

int rtps_rx_set_spec_hint(rtps_rx_ctx* c, uint32_t records_per_datagram) {
  if (!c || records_per_datagram > 0xffffu) return RTPS_RX_EINVAL;
  c->k_spec = records_per_datagram;
  return RTPS_RX_OK;
}

int rtps_rx_sync(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  return hip_fail(hipStreamSynchronize(c->stream));
}

const char* rtps_rx_strerror(int code) {
  switch (code) {
    case RTPS_RX_OK: return "ok";
    case RTPS_RX_EINVAL: return "invalid argument";
    case RTPS_RX_EHIP: return "HIP runtime error";
    case RTPS_RX_ENOMEM: return "out of device memory";
    case RTPS_RX_ETOOBIG: return "batch larger than the context's max_datagrams";
    case RTPS_RX_EABI: return "ABI version mismatch";
    case RTPS_RX_EABORTED: return "RCCL communicator aborted (freed): make a new one";
    default: return "unknown error";
  }
}

uint64_t rtps_rx_max_records_host(const uint32_t* len, uint32_t n) {
  uint64_t t = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (len[i] >= 20 && len[i] <= RTPS_MAX_DATAGRAM) t += (len[i] - 20) / 4;
  return t;
}

int rtps_rx_generate(rtps_rx_ctx* c, int wl, uint64_t seed, uint64_t first_idx, uint32_t n_writers,
                     uint8_t* arena, const uint64_t* off, const uint32_t* len, uint32_t n) {
  (void)len;
  if (!c || (n && (!arena || !off))) return RTPS_RX_EINVAL;
  if (wl < 1 || wl > 4) return RTPS_RX_EINVAL;
  if (n == 0) return RTPS_RX_OK;
  (void)hipSetDevice(c->device);
  hipLaunchKernelGGL(rtps_gen_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, wl, seed, first_idx,
                     n_writers, arena, off, n);
  return hip_fail(hipGetLastError());
}

/* host copy of the generator's layout (same f(seed, idx) as the device kernel) */
uint64_t rtps_rx_gen_layout_host(int wl, uint64_t seed, uint64_t first_idx, uint32_t n_writers, uint32_t n,
                                 uint64_t* off, uint32_t* len) {
  return rtps_gen_layout_host(wl, seed, first_idx, n_writers, n, off, len);
}


static int bucket_impl(rtps_rx_ctx* c, const rtps_record* recs, const uint64_t* n_records, uint64_t max_records,
                       uint32_t n_dest, uint64_t cap, void* out, uint64_t* dest_counts, bool desc) {
  if (!c || !recs || !n_records || !out || !dest_counts || n_dest < 1 || n_dest > MAX_DEST) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  uint64_t tiles64 = (max_records + TILE - 1) / TILE;
  if (tiles64 == 0) return hip_fail(hipMemsetAsync(dest_counts, 0, n_dest * sizeof(uint64_t), c->stream));
  if (tiles64 > 0xffffffffull) return RTPS_RX_ETOOBIG;
  uint32_t tiles = (uint32_t)tiles64;
  size_t need = (size_t)tiles * n_dest * sizeof(uint32_t);
  if (need > c->bucket_bytes) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->bucket_hist);
    c->bucket_hist = nullptr; c->bucket_bytes = 0;
    if (hipMalloc(&c->bucket_hist, need) != hipSuccess) return RTPS_RX_ENOMEM;
    c->bucket_bytes = need;
  }
  DescOwner m{rt_dev(c->readers)};
  if (desc) {
    hipLaunchKernelGGL(bucket_hist_kernel<true>, dim3(tiles), dim3(TILE), 0, c->stream, recs, n_records, n_dest,
                       c->bucket_hist, m);
  } else {
    hipLaunchKernelGGL(bucket_hist_kernel<false>, dim3(tiles), dim3(TILE), 0, c->stream, recs, n_records, n_dest,
                       c->bucket_hist, m);
  }
  hipLaunchKernelGGL(bucket_scan_kernel, dim3(n_dest), dim3(TILE), 0, c->stream, c->bucket_hist, tiles, n_dest,
                     dest_counts);
  if (desc) {
    hipLaunchKernelGGL(bucket_scatter_kernel<true>, dim3(tiles), dim3(TILE), 0, c->stream, recs, n_records, n_dest,
                       c->bucket_hist, dest_counts, cap, out, m);
  } else {
    hipLaunchKernelGGL(bucket_scatter_kernel<false>, dim3(tiles), dim3(TILE), 0, c->stream, recs, n_records, n_dest,
                       c->bucket_hist, dest_counts, cap, out, m);
  }
  return hip_fail(hipGetLastError());
}

int rtps_rx_bucket_by_writer(rtps_rx_ctx* c, const rtps_record* recs, const uint64_t* n_records,
                             uint64_t max_records, uint32_t n_dest, rtps_record* out, uint64_t* dest_counts) {
  return bucket_impl(c, recs, n_records, max_records, n_dest, 0, out, dest_counts, false);
}

int rtps_rx_bucket_by_writer_padded(rtps_rx_ctx* c, const rtps_record* recs, const uint64_t* n_records,
                                    uint64_t max_records, uint32_t n_dest, uint64_t cap, rtps_record* out,
                                    uint64_t* dest_counts) {
  if (cap == 0) return RTPS_RX_EINVAL;
  return bucket_impl(c, recs, n_records, max_records, n_dest, cap, out, dest_counts, false);
}

int rtps_rx_bucket_descriptors(rtps_rx_ctx* c, const rtps_record* recs, const uint64_t* n_records,
                               uint64_t max_records, uint32_t n_dest, uint64_t cap, rtps_xdesc* out,
                               uint64_t* dest_counts) {
  if (!c || cap == 0 || rt_dev(c->readers).gkeys == nullptr) return RTPS_RX_EINVAL;
  return bucket_impl(c, recs, n_records, max_records, n_dest, cap, out, dest_counts, true);
}

/* a18: batch CDR decode (rtps_cdr.hip).  The program is validated here so
 * the kernel can trust every op (sizes, slot bounds inside the row). */
static int cdr_prog(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes, CdrProg& P) {
  if (!prog || n_ops > RTPS_CDR_MAX_OPS || row_bytes == 0 || (row_bytes & 3u) || row_bytes > (1u << 20))
    return RTPS_RX_EINVAL;
  memset(&P, 0, sizeof(P));
  for (uint32_t k = 0; k < n_ops; ++k) {
    const rtps_cdr_op& op = prog[k];
    const uint64_t sz = op.size;
    const bool pow2 = sz == 1 || sz == 2 || sz == 4 || sz == 8;
    uint64_t field;
    switch (op.kind) {
      case RTPS_CDR_PRIM: if (!pow2) return RTPS_RX_EINVAL; field = sz; break;
      case RTPS_CDR_BOOL: field = 1; break;
      case RTPS_CDR_STRING: field = 4ull + op.count; break;
      case RTPS_CDR_SEQ: if (!pow2) return RTPS_RX_EINVAL; field = 4ull + sz * op.count; break;
      case RTPS_CDR_ARRAY: if (!pow2) return RTPS_RX_EINVAL; field = sz * op.count; break;
      default: return RTPS_RX_EINVAL;
    }
    if ((uint64_t)op.out_off + field > row_bytes) return RTPS_RX_EINVAL;
    P.ops[k] = op;
  }
  P.n_ops = n_ops;
  P.row_bytes = row_bytes;
  return rtps_cdr_build_slots(P) ? RTPS_RX_OK : RTPS_RX_EINVAL;
}

// Validates the program and launches the decode: the slot-parallel kernel for flat
// programs, the lane-per-row one for composite programs (SEQ_BEGIN / ARRAY_BEGIN).
static int cdr_run(rtps_rx_ctx* c, const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes, const CdrArgs& a) {
  (void)hipSetDevice(c->device);
  // tuning knob: RTPS_CDR_NESTED=1 runs flat programs through the lane-per-row kernel too
  static const bool force_nested = [] { const char* e = getenv("RTPS_CDR_NESTED"); return e && e[0] == '1'; }();
  if (rtps_cdr_is_composite(prog, n_ops) || force_nested) {
    CdrNest N;
    if (!rtps_cdr_build_nested(prog, n_ops, row_bytes, N)) return RTPS_RX_EINVAL;
    return rtps_cdr_launch_nested(c->stream, N, a, c->resident_blocks) == 0 ? RTPS_RX_OK : RTPS_RX_EHIP;
  }
  CdrProg P;
  const int rc = cdr_prog(prog, n_ops, row_bytes, P);
  if (rc) return rc;
  return rtps_cdr_launch(c->stream, P, a, c->resident_blocks) == 0 ? RTPS_RX_OK : RTPS_RX_EHIP;
}
static bool cdr_prog_ok(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes) {
  if (!prog || n_ops > RTPS_CDR_MAX_OPS || row_bytes == 0 || (row_bytes & 3u) || row_bytes > (1u << 20)) return false;
  if (rtps_cdr_is_composite(prog, n_ops)) {
    CdrNest N;
    return rtps_cdr_build_nested(prog, n_ops, row_bytes, N);
  }
  CdrProg P;
  return cdr_prog(prog, n_ops, row_bytes, P) == RTPS_RX_OK;
}

int rtps_rx_cdr_decode(rtps_rx_ctx* c, const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes,
                       const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                       const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                       uint8_t* rows, uint8_t* row_status) {
  if (!c || !cdr_prog_ok(prog, n_ops, row_bytes)) return RTPS_RX_EINVAL;
  if (!records || !n_records || (max_records && (!arena || !dgram_off || !rows || !row_status))) return RTPS_RX_EINVAL;
  if (max_records == 0) return RTPS_RX_OK;
  CdrArgs a{arena, arena_len, dgram_off, records, n_records, max_records, rows, row_status, nullptr, 0, nullptr, 0};
  return cdr_run(c, prog, n_ops, row_bytes, a);
}

int rtps_rx_cdr_decode_list(rtps_rx_ctx* c, const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes,
                            const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                            const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                            const void* list, uint32_t list_stride, const uint64_t* n_list, uint64_t max_list,
                            uint8_t* rows, uint8_t* row_status) {
  if (!c || !cdr_prog_ok(prog, n_ops, row_bytes)) return RTPS_RX_EINVAL;
  if (!records || !n_records || !n_list || list_stride < 4 || (list_stride & 3u)) return RTPS_RX_EINVAL;
  if (max_list && (!list || !arena || !dgram_off || !rows || !row_status)) return RTPS_RX_EINVAL;
  if (max_list == 0) return RTPS_RX_OK;
  CdrArgs a{arena, arena_len, dgram_off, records, n_records, max_records, rows, row_status,
            static_cast<const uint8_t*>(list), list_stride, n_list, max_list};
  return cdr_run(c, prog, n_ops, row_bytes, a);
}

/* DataFrag reassembly (rtps_frag.hip) */
int rtps_rx_frag_assemble(rtps_rx_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                          const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                          const rtps_frag_out* out) {
  if (!c || !records || !n_records || !out || !out->n_samples || !out->heap_used || !out->n_pending) return RTPS_RX_EINVAL;
  if ((out->max_samples && !out->samples) || (out->heap_bytes && !out->heap)) return RTPS_RX_EINVAL;
  if (max_records && (!arena || !dgram_off)) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->frag) {
    c->frag = rtps_frag_state_new(c->device);
    if (!c->frag) return RTPS_RX_ENOMEM;
  }
  const ReaderDev rd = rt_dev(c->readers);
  FragSel sel;
  memset(&sel, 0, sizeof sel);
  if (rd.gkeys == nullptr)  // no readers: one assembler per writer for every DATA_FRAG that passes
    return rtps_frag_assemble(c->frag, c->stream, arena, arena_len, dgram_off, records, n_records, max_records, out,
                              sel, nullptr);
  if (!c->life) {
    if (hipMalloc(&c->life, 65536 * sizeof(int64_t)) != hipSuccess) return RTPS_RX_ENOMEM;
    std::vector<int64_t> none(65536, NO_LIFESPAN);
    if (hipMemcpy(c->life, none.data(), 65536 * sizeof(int64_t), hipMemcpyHostToDevice) != hipSuccess)
      return RTPS_RX_EHIP;
  }
  uint64_t now_ns = c->recv_ns;
  if (!now_ns) {  // Timestamp::now() (structure/time.rs:58-65): the host's wall clock at this batch
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    now_ns = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
  }
  // Timestamp::from_nanos (time.rs:78-83) as ticks
  const uint64_t recv_ticks = ((now_ns / 1000000000ull) << 32) + (((now_ns % 1000000000ull) << 32) / 1000000000ull);
  sel.rt = rd;
  sel.life = c->life;
  sel.any_life = c->any_life ? 1u : 0u;
  sel.recv_ticks = recv_ticks;
  if (rd.max_set <= 1u) {  // every record reaches one reader at most: select it in place, no copies
    sel.mode = 1;
    return rtps_frag_assemble(c->frag, c->stream, arena, arena_len, dgram_off, records, n_records, max_records, out,
                              sel, nullptr);
  }
  // larger target sets: one assembler per (reader, writer), over the batch expanded per target reader
  sel.mode = 2;
  const uint64_t max_x = max_records * (rd.max_set ? rd.max_set : 1u);
  if (max_x > 0x7fffffffull) return RTPS_RX_ETOOBIG;
  if (max_records > c->fx_cap || max_x > c->fx_xcap || !c->fx_n) {
    if (hipStreamSynchronize(c->stream) != hipSuccess) return RTPS_RX_EHIP;
    void* fx[] = {c->fx_cnt, c->fx_off, c->fx_emap, c->fx_rec, c->fx_n, c->fx_tmp};
    for (void* q : fx) if (q) (void)hipFree(q);
    c->fx_cnt = c->fx_off = c->fx_emap = nullptr; c->fx_rec = nullptr; c->fx_n = nullptr; c->fx_tmp = nullptr;
    c->fx_cap = c->fx_xcap = 0; c->fx_tmp_bytes = 0;
    const uint64_t m = max_records ? max_records : 1, x = max_x ? max_x : 1;
    size_t tb = 0;
    if (hipMalloc(&c->fx_cnt, m * 4) != hipSuccess || hipMalloc(&c->fx_off, m * 4) != hipSuccess ||
        hipMalloc(&c->fx_emap, x * 4) != hipSuccess || hipMalloc(&c->fx_rec, x * sizeof(rtps_record)) != hipSuccess ||
        hipMalloc(&c->fx_n, 8) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, tb, c->fx_cnt, c->fx_off, (int)m, c->stream) != hipSuccess ||
        hipMalloc(&c->fx_tmp, tb ? tb : 16) != hipSuccess)
      return RTPS_RX_ENOMEM;
    c->fx_tmp_bytes = tb;
    c->fx_cap = m;
    c->fx_xcap = x;
  }
  const uint64_t m = max_records ? max_records : 1;
  FragX a{records, n_records, max_records, rd, c->life, recv_ticks, c->any_life ? 1u : 0u, c->fx_cnt, c->fx_off,
          c->fx_rec, c->fx_emap, c->fx_n};
  const uint32_t g = (uint32_t)((m + TILE - 1) / TILE < 8192 ? (m + TILE - 1) / TILE : 8192);
  if (max_records == 0) {
    if (hipMemsetAsync(c->fx_n, 0, 8, c->stream) != hipSuccess) return RTPS_RX_EHIP;
  } else {
    hipLaunchKernelGGL(frag_x_count, dim3(g), dim3(TILE), 0, c->stream, a);
    size_t tb = c->fx_tmp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(c->fx_tmp, tb, c->fx_cnt, c->fx_off, (int)max_records, c->stream) !=
        hipSuccess)
      return RTPS_RX_EHIP;
    hipLaunchKernelGGL(frag_x_fill, dim3(g), dim3(TILE), 0, c->stream, a);
  }
  if (hipGetLastError() != hipSuccess) return RTPS_RX_EHIP;
  return rtps_frag_assemble(c->frag, c->stream, arena, arena_len, dgram_off, c->fx_rec, c->fx_n, max_x, out, sel,
                            c->fx_emap);
}

/* per-reader Lifespan QoS for the DataFrag assembly (reader.rs:578-589): lifespan_ns < 0 = none */
int rtps_rx_set_reader_lifespan(rtps_rx_ctx* c, uint16_t reader_slot, int64_t lifespan_ns) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->life) {
    if (hipMalloc(&c->life, 65536 * sizeof(int64_t)) != hipSuccess) return RTPS_RX_ENOMEM;
    std::vector<int64_t> none(65536, NO_LIFESPAN);
    if (hipMemcpy(c->life, none.data(), 65536 * sizeof(int64_t), hipMemcpyHostToDevice) != hipSuccess)
      return RTPS_RX_EHIP;
  }
  int64_t ticks = NO_LIFESPAN;
  if (lifespan_ns >= 0) {  // Duration::from_nanos (structure/duration.rs:60-67) as ticks
    const int64_t sec = lifespan_ns / 1000000000ll, frac = ((lifespan_ns % 1000000000ll) << 32) / 1000000000ll;
    ticks = (int64_t)(((uint64_t)(int64_t)(int32_t)sec << 32) + (uint64_t)(uint32_t)frac);
    c->any_life = true;
  }
  if (hipStreamSynchronize(c->stream) != hipSuccess ||
      hipMemcpy(c->life + reader_slot, &ticks, sizeof ticks, hipMemcpyHostToDevice) != hipSuccess)
    return RTPS_RX_EHIP;
  return RTPS_RX_OK;
}

/* the receive time (Timestamp::now(), ns since the UNIX epoch) of the next batches' DATA_FRAGs for
   the Lifespan check; 0: the host's clock at each rtps_rx_frag_assemble */
int rtps_rx_frag_set_receive_time(rtps_rx_ctx* c, uint64_t unix_ns) {
  if (!c) return RTPS_RX_EINVAL;
  c->recv_ns = unix_ns;
  return RTPS_RX_OK;
}

int rtps_rx_frag_reset(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  if (!c->frag) return RTPS_RX_OK;
  (void)hipSetDevice(c->device);
  return rtps_frag_state_reset(c->frag, c->stream);
}

int rtps_rx_frag_set_clock(rtps_rx_ctx* c, uint64_t now_ns) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->frag) {
    c->frag = rtps_frag_state_new(c->device);
    if (!c->frag) return RTPS_RX_ENOMEM;
  }
  rtps_frag_set_clock(c->frag, now_ns);
  return RTPS_RX_OK;
}

int rtps_rx_frag_gc(rtps_rx_ctx* c, uint64_t expire_before_ns, uint64_t* n_pending) {
  if (!c || !n_pending) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->frag) return hipMemsetAsync(n_pending, 0, 8, c->stream) == hipSuccess ? RTPS_RX_OK : RTPS_RX_EHIP;
  return rtps_frag_gc(c->frag, c->stream, expire_before_ns, n_pending);
}

/* history-cache ingest (rtps_ingest.hip) */
int rtps_rx_ingest(rtps_rx_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* dgram_off,
                   const rtps_record* records, const uint64_t* n_records, uint64_t max_records,
                   const rtps_frag_sample* frag, const uint64_t* n_frag, uint64_t max_frag, uint32_t flags,
                   const rtps_ingest_out* out) {
  if (!c || !records || !n_records || !out || !out->accept || !out->accepted || !out->n_accepted) return RTPS_RX_EINVAL;
  const ReaderDev rd = rt_dev(c->readers);
  if (rd.gkeys == nullptr) return RTPS_RX_EINVAL;
  if (max_records && (!arena || !dgram_off)) return RTPS_RX_EINVAL;
  if (flags & ~(RTPS_INGEST_BEST_EFFORT | RTPS_INGEST_TOPIC_CACHE)) return RTPS_RX_EINVAL;
  if (frag && (!n_frag || !max_frag)) return RTPS_RX_EINVAL;
  // a topic cache's GC spans all of its writers (dds_cache.rs:210-276, 367-420): on owner batches
  // they must all meet on one owner, which only RTPS_OWNER_TOPIC guarantees
  if ((flags & RTPS_INGEST_TOPIC_CACHE) && rtps_ctx_topic_split(c)) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->ingest) {
    c->ingest = rtps_ingest_state_new(c->device);
    if (!c->ingest) return RTPS_RX_ENOMEM;
  }
  // with the topic caches, the batch's window-overflow count goes where the topic step reads it
  rtps_ingest_out o = *out;
  if ((flags & RTPS_INGEST_TOPIC_CACHE) && !o.n_window_overflow) {
    if (!c->tc_ovf && hipMalloc(&c->tc_ovf, sizeof(uint64_t)) != hipSuccess) return RTPS_RX_ENOMEM;
    o.n_window_overflow = c->tc_ovf;
  }
  if (!(flags & RTPS_INGEST_TOPIC_CACHE))
    return rtps_ingest_batch(c->ingest, c->stream, rd, arena, arena_len, dgram_off, records, n_records, max_records,
                             frag, n_frag, max_frag, flags, &o);
  // the topic caches' add_change over the deliveries (rtps_topic.hip), queued by the ingest
  // behind its deliveries (gated by its verdict where it queues its plain path ahead)
  int rc = topics_state(c);
  if (rc) return rc;
  struct TopicTail {
    rtps_rx_ctx* c;
    const rtps_record* records;
    const uint64_t* n_records;
    uint64_t max_records;
    const rtps_ingest_out* o;
  } tt{c, records, n_records, max_records, &o};
  const IngestTail tail{[](void* p, const uint64_t* gate) -> int {
                          const TopicTail& a = *static_cast<const TopicTail*>(p);
                          return rtps_topic_apply(a.c->topics, a.c->stream, a.records, a.n_records, a.max_records,
                                                  a.o->accepted, a.o->n_accepted, a.o->max_accepted,
                                                  a.o->n_window_overflow, gate);
                        },
                        &tt};
  return rtps_ingest_batch(c->ingest, c->stream, rd, arena, arena_len, dgram_off, records, n_records, max_records,
                           frag, n_frag, max_frag, flags & ~RTPS_INGEST_TOPIC_CACHE, &o, &tail);
}

/* test / measurement hook (not part of the public header): the ingest's
   per-batch path, 0 = chosen per batch, 1 = global marks / merge, 2 = one
   workgroup per proxy (same results), 3 = global with the first-cover-key merge,
   4 = per proxy with the radix sort instead of the proxy bucketing */
int rtps_rx_debug_ingest_path(rtps_rx_ctx* c, uint32_t path) {
  if (!c || path > 4u) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->ingest) {
    c->ingest = rtps_ingest_state_new(c->device);
    if (!c->ingest) return RTPS_RX_ENOMEM;
  }
  rtps_ingest_set_path(c->ingest, path);
  return RTPS_RX_OK;
}

/* test hook (not part of the public header): the reassembly's key sort, 0 = the
   bucket sort of rtps_bsort.h up to its size limit, 1 = rocprim's device sort always
   (same results) */
int rtps_rx_debug_frag_sort(rtps_rx_ctx* c, uint32_t mode) {
  if (!c || mode > 1u) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (!c->frag) {
    c->frag = rtps_frag_state_new(c->device);
    if (!c->frag) return RTPS_RX_ENOMEM;
  }
  rtps_frag_set_sort(c->frag, (int)mode);
  return RTPS_RX_OK;
}

/* tuning hook (not part of the public header): see rtps_ingest_proxy_stamps */
int rtps_rx_debug_proxy_stamps(rtps_rx_ctx* c, uint64_t* host, uint64_t n) {
  if (!c || !host) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  if (hipStreamSynchronize(c->stream) != hipSuccess) return RTPS_RX_EHIP;
  return rtps_ingest_proxy_stamps(host, n);
}

int rtps_rx_ingest_reset(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  (void)hipSetDevice(c->device);
  const int rc = c->ingest ? rtps_ingest_state_reset(c->ingest, c->stream) : RTPS_RX_OK;
  if (rc || !c->topics) return rc;
  return rtps_topic_proxies_reset(c->topics, c->stream);
}

int rtps_rx_topic_reset(rtps_rx_ctx* c) {
  if (!c) return RTPS_RX_EINVAL;
  if (!c->topics) return RTPS_RX_OK;
  (void)hipSetDevice(c->device);
  return rtps_topic_reset(c->topics, c->stream);
}

uint32_t rtps_rx_record_size(void) { return (uint32_t)sizeof(rtps_record); }

/* test hook (not part of the public header): polls before a chained tile gives up and
   leaves itself to kernel B; 0 makes most tiles give up, exercising that fallback */
int rtps_rx_debug_set_chain_spin_limit(rtps_rx_ctx* c, uint32_t limit) {
  if (!c) return RTPS_RX_EINVAL;
#ifdef RTPS_DIAG_PASSES
  c->ch_spin_limit = limit;
  return RTPS_RX_OK;
#else
  (void)limit;
  return RTPS_RX_EINVAL;  // (no chained pass in the product build)
#endif
}

/* tuning hook (not part of the public header): per-tile phase stamps (s_memrealtime,
   100 MHz; STAMP_N per tile) of the last launch of kernel D or W, in diagnostic builds
   with RTPS_LDS_STAMPS / RTPS_EM_STAMPS; RTPS_RX_EINVAL otherwise */
int rtps_rx_debug_lds_stamps(rtps_rx_ctx* c, uint64_t* host, uint64_t n) {
#if defined(RTPS_DIAG_PASSES) && (defined(RTPS_LDS_STAMPS) || defined(RTPS_EM_STAMPS))
  if (!c || !host) return RTPS_RX_EINVAL;
  if (n > (uint64_t)STAMP_TILES * STAMP_N) n = (uint64_t)STAMP_TILES * STAMP_N;
  (void)hipSetDevice(c->device);
  if (hipStreamSynchronize(c->stream) != hipSuccess) return RTPS_RX_EHIP;
  return hip_fail(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lds_stamps), n * 8, 0, hipMemcpyDeviceToHost));
#else
  (void)c; (void)host; (void)n;
  return RTPS_RX_EINVAL;
#endif
}

/* test / measurement hook (not part of the public header): the pass used for mixed
   traffic, 2 = the item pass (rtps_parse_item_kernel / scan / emit2, the product's only
   one); diagnostic builds (RTPS_DIAG_PASSES) also 0 = the chained lane walk
   (rtps_parse_chain_kernel), 1 = LDS tiles (rtps_parse_lds_kernel), 3 = the record-slab
   pass.  Same results.  RTPS_RX_EINVAL for a pass this build does not have. */
int rtps_rx_debug_set_mixed_pass(rtps_rx_ctx* c, uint32_t pass) {
#ifdef RTPS_DIAG_PASSES
  if (!c || pass > 3u) return RTPS_RX_EINVAL;
#else
  if (!c || pass != 2u) return RTPS_RX_EINVAL;
#endif
  c->mixed_pass = pass;
  return RTPS_RX_OK;
}

/* test / measurement hook (not part of the public header): the item pass's record pass,
   2 = rtps_parse_emit2_kernel (the product's); diagnostic builds also 1 = round 4's
   rtps_parse_emit_kernel.  Same results.  Returns the pass in effect (0 selects nothing
   new), or RTPS_RX_EINVAL for a pass this build does not have. */
int rtps_rx_debug_emit(rtps_rx_ctx* c, uint32_t emit) {
#ifdef RTPS_DIAG_PASSES
  if (!c || emit > 2u) return RTPS_RX_EINVAL;
#else
  if (!c || (emit != 0u && emit != 2u)) return RTPS_RX_EINVAL;
#endif
  if (emit) c->emit = emit;
  return (int)c->emit;
}

/* test hook (not part of the public header): the last chained launch's epoch, so
   that a test can run chained launches across the 32-bit wrap (diagnostic builds) */
int rtps_rx_debug_set_chain_epoch(rtps_rx_ctx* c, uint32_t epoch) {
  if (!c) return RTPS_RX_EINVAL;
#ifdef RTPS_DIAG_PASSES
  c->ch_epoch = epoch;
  return RTPS_RX_OK;
#else
  (void)epoch;
  return RTPS_RX_EINVAL;
#endif
}

#ifdef RTPS_ITEM_DIAG
#include "diag/item_pass_host.inc"
#endif

/* diagnostics (not part of the public header): copy the first k scratch words */
int rtps_rx_debug_scratch(rtps_rx_ctx* c, uint64_t* host, uint32_t k) {
  if (!c || !host || k > c->scratch_words) return RTPS_RX_EINVAL;
  (void)hipStreamSynchronize(c->stream);
  return hip_fail(hipMemcpy(host, c->scratch, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
}

}  // extern "C"

// internal accessors (rtps_ctx.h)
hipStream_t rtps_ctx_stream(const rtps_rx_ctx* c) { return c->stream; }
int rtps_ctx_device(const rtps_rx_ctx* c) { return c->device; }
uint32_t rtps_ctx_max_datagrams(const rtps_rx_ctx* c) { return c->max_datagrams; }
