// rtps_shard.h — internal state of the owner-side exchange (rtps_shard.hip:
// pack / unpack kernels; rtps_exchange.cpp: the RCCL rounds).  Not installed;
// the public contract is the rtps_rx_shard_* section of include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/rtps_rx.h"

constexpr uint32_t SHARD_MAX_RANKS = 64;
// what crosses xGMI per writer record: rtps_shard_item (include/rtps_rx.h); a compact DATA is the
// item alone, any other kind the item + a blob (a DATA's GUID and SN; else its 64-B record + the
// bytes its consumers read)
typedef rtps_shard_item shard_item;
static_assert(sizeof(shard_item) == 16, "16-B exchange items");
constexpr uint32_t SHARD_WLIST_MAX = 1u << 20;  // writers a compact item can name

struct rtps_shard {
  rtps_rx_ctx* ctx = nullptr;
  int device = 0;
  uint32_t n_ranks = 0;
  uint64_t cap = 0, bcap = 0;  // fixed slot per peer: records, blob bytes (multiple of 16)
  // ---- send side (this rank as a source) ----
  shard_item* s_slots = nullptr;         // [n_ranks * cap]
  uint8_t* s_blob = nullptr;              // [n_ranks * bcap]
  rtps_shard_counts* s_counts = nullptr;  // [n_ranks] device
  shard_item* s_spill = nullptr;         // exact layout: dest d at sum_{d' < d} n_d'
  uint64_t s_spill_cap = 0;
  uint8_t* s_bspill = nullptr;            // exact layout: dest d at sum_{d' < d} bytes_d'
  uint64_t s_bspill_cap = 0;
  uint32_t* hist = nullptr;               // [tiles * n_ranks] x {records, bytes}
  uint64_t* hscan = nullptr;              // [tiles * n_ranks] x {record offset, byte offset}
  uint64_t hist_tiles = 0;
  // ---- receive side (this rank as the owner) ----
  shard_item* r_slots = nullptr;         // [n_ranks * cap]: source s's slot at s * cap
  uint8_t* r_blob = nullptr;              // [n_ranks * bcap]
  rtps_shard_counts* r_counts = nullptr;  // [n_ranks] device: what source s sent this rank
  shard_item* r_spill = nullptr;         // source s's spill at sum_{s' < s} (n - cut)
  uint64_t r_spill_cap = 0;
  uint8_t* r_bspill = nullptr;            // source s's spilled bytes at sum_{s' < s} (bytes - cut_bytes)
  uint64_t r_bspill_cap = 0;
  // ---- host copies of the counts (pinned), filled by the exchange ----
  rtps_shard_counts* h_send = nullptr;
  rtps_shard_counts* h_recv = nullptr;
  hipEvent_t packed = nullptr;     // recorded after pack on the context stream
  hipEvent_t counts_ev = nullptr;  // recorded after the counts' device-to-host copies (exchange stream)
  hipEvent_t done = nullptr;       // recorded after the last exchange round (exchange stream)
  bool exchanged = false;          // the counts were copied by rtps_rx_shard_exchange
  bool finished = false;           // rtps_rx_shard_finish ran after that exchange (the spill, if any, moved)
  // ---- the owner batch ----
  shard_item* o_item = nullptr;  // the received items, source order
  rtps_record* o_rec = nullptr;
  uint64_t* o_off = nullptr;
  uint64_t* o_origin = nullptr;
  uint64_t* o_size = nullptr;  // blob bytes per record, then (scanned in place) its blob offset
  uint64_t* o_boff = nullptr;
  uint64_t o_cap = 0;
  uint8_t* o_arena = nullptr;
  uint64_t o_arena_cap = 0;
  uint64_t* o_n = nullptr;  // device u64
  void* cub_tmp = nullptr;
  size_t cub_bytes = 0;
  // ---- writer -> owner table (rtps_rx_shard_set_owners) ----
  uint32_t owner_mode = RTPS_OWNER_BALANCED;
  bool mode_explicit = false;      // rtps_rx_shard_set_owners chose the mode (else: TOPIC once topics are set)
  std::vector<uint8_t> x_guid;     // the caller's extra writers (16 B each) and their weights
  std::vector<uint64_t> x_weight;
  uint64_t owner_version = ~0ull;  // the context's readers version the table follows (~0: build at the next pack)
  uint32_t t_mode = ~0u;           // the mode the table was dealt in (~0u: none yet)
  std::vector<uint8_t> t_guid;     // host copy of the table: keys (writer GUIDs, entity keys) and their owners
  std::vector<uint32_t> t_owner;
  bool t_ent = false;              // the table has entity keys (RTPS_OWNER_TOPIC)
  uint32_t* d_okeys = nullptr;     // device: [ocap * 4] GUID words, open addressing by rt_hash16
  uint32_t* d_oval = nullptr;      // [ocap] owner | (writer-list index + 1) << 8 (0: an entity key), ~0 = empty
  uint32_t ocap = 0;               // 0: no table (every writer by the GUID hash)
  uint32_t* d_wlist = nullptr;     // [n_wlist * 4] the table's writer GUIDs, ascending bytes (compact items)
  uint32_t n_wlist = 0, wlist_cap = 0;
};

// grow-only device buffer (contents are not kept); false on allocation failure
bool shard_reserve(void** p, uint64_t* cap, uint64_t need_bytes);
