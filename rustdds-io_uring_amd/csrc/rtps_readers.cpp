// rtps_readers.cpp — host builder of the target sets (see rtps_readers.h).
//
// Readers are kept in EntityId order, the iteration order of the reference's
// available_readers BTreeMap<EntityId, Reader> (io_uring/rtps/message_receiver.rs:129;
// EntityId derives Ord over {entity_key[3], entity_kind}: byte order, structure/guid.rs:208-216).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <new>
#include <utility>
#include <vector>

#include "rtps_readers.h"

namespace {
typedef std::array<uint8_t, 16> Guid;
static_assert(sizeof(Guid) == 16, "GUIDs back to back");
typedef std::array<uint8_t, 4> Eid;
// EntityId::SPDP_BUILTIN_PARTICIPANT_READER {0x00,0x01,0x00}, 0xc7 (structure/guid.rs)
const Eid SPDP_PARTICIPANT_READER = {0x00, 0x01, 0x00, 0xc7};

uint32_t pow2_at_least(uint64_t n) {
  uint32_t c = 16;
  while (c < n) c <<= 1;
  return c;
}
uint32_t word(const uint8_t* p) {
  uint32_t w;
  memcpy(&w, p, 4);
  return w;
}
}  // namespace

struct ReaderTable {
  std::vector<uint32_t> first;     // [n_sets + 1]
  std::vector<rtps_target> ent;
  std::vector<Guid> wguid;         // [n_writer_sets] the writer GUID of each writer set
  std::vector<Eid> eids;           // [n_sets - n_writer_sets] the writer entity id of each entity set
  uint32_t n_writer_sets = 0, n_proxies = 0, max_set = 0;
  bool active = false;
  // device images
  uint32_t *gkeys = nullptr, *gset = nullptr, *ekeys = nullptr, *eset = nullptr, *dfirst = nullptr;
  rtps_target* dent = nullptr;
  uint32_t gcap = 0, ecap = 0;
};

ReaderTable* rt_new() { return new (std::nothrow) ReaderTable(); }

// Device memory of the tables.  rt_set builds the image into a fresh buffer and
// swaps it in only when all of it is uploaded, so a failed call leaves the
// previous table whole (readers and proxies of the last successful call).  The
// operations are indirect so that a CPU test can run rt_set on host memory with
// an injected allocation failure (rtps_rx_debug_rt_* below).
struct DevMem {
  void* (*alloc)(size_t);
  void (*release)(void*);
  bool (*upload)(void* dst, const void* src, size_t n);
  bool (*sync)(hipStream_t);
};
namespace {
void* hip_alloc(size_t n) {
  void* p = nullptr;
  return hipMalloc(&p, n ? n : 1) == hipSuccess ? p : nullptr;
}
void hip_release(void* p) { if (p) (void)hipFree(p); }
bool hip_upload(void* d, const void* s, size_t n) { return !n || hipMemcpy(d, s, n, hipMemcpyHostToDevice) == hipSuccess; }
bool hip_sync(hipStream_t st) { return hipStreamSynchronize(st) == hipSuccess; }
int g_fail_at = -1, g_allocs = 0;  // host-memory test mode: fail the g_fail_at-th allocation
void* host_alloc(size_t n) { return g_allocs++ == g_fail_at ? nullptr : malloc(n ? n : 1); }
void host_release(void* p) { free(p); }
bool host_upload(void* d, const void* s, size_t n) { if (n) memcpy(d, s, n); return true; }
bool host_sync(hipStream_t) { return true; }
DevMem g_mem = {hip_alloc, hip_release, hip_upload, hip_sync};
}  // namespace

void rt_free(ReaderTable* t) {
  if (!t) return;
  g_mem.release(t->gkeys);  // the one image buffer (gkeys is its base)
  delete t;
}

namespace {
struct Built {  // host image of a reader table
  std::vector<uint32_t> first;
  std::vector<rtps_target> ent;
  std::vector<Guid> wguid;
  std::vector<Eid> eids;
  std::vector<uint32_t> gkeys, gset, ekeys, eset;
  uint32_t gcap = 0, ecap = 0, n_writer_sets = 0, max_set = 0;
};

int build(const rtps_reader* readers, uint32_t nr, const rtps_proxy* proxies, uint32_t np, Built& out) {
  if ((nr && !readers) || (np && !proxies)) return RTPS_RX_EINVAL;
  if (nr > 0xffffu) return RTPS_RX_ETOOBIG;
  // ---- validation: unique reader entity ids, proxies keyed (reader, GUID) uniquely ----
  std::vector<uint32_t> order(nr);
  for (uint32_t i = 0; i < nr; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return memcmp(readers[a].entity_id, readers[b].entity_id, 4) < 0;
  });
  for (uint32_t k = 1; k < nr; ++k)
    if (memcmp(readers[order[k - 1]].entity_id, readers[order[k]].entity_id, 4) == 0) return RTPS_RX_EINVAL;
  std::map<std::pair<uint32_t, Guid>, uint32_t> proxy_of;  // (reader, GUID) -> proxy index
  std::vector<std::vector<Eid>> contains(nr);                // entity ids of each reader's matched writers
  std::vector<Guid> wsets;                                   // writer sets, first appearance
  std::map<Guid, uint32_t> wset_of;
  std::vector<Eid> esets;
  std::map<Eid, uint32_t> eset_of;
  for (uint32_t i = 0; i < np; ++i) {
    const rtps_proxy& p = proxies[i];
    if (p.reader >= nr) return RTPS_RX_EINVAL;
    Guid g;
    memcpy(g.data(), p.writer_guid, 16);
    if (!proxy_of.emplace(std::make_pair(p.reader, g), i).second) return RTPS_RX_EINVAL;
    if (readers[p.reader].flags & RTPS_READER_STATELESS) continue;  // contains_writer() is false
    Eid e;
    memcpy(e.data(), p.writer_guid + 12, 4);
    contains[p.reader].push_back(e);
    if (wset_of.emplace(g, (uint32_t)wsets.size()).second) wsets.push_back(g);
  }
  for (const Guid& g : wsets) {
    Eid e;
    memcpy(e.data(), g.data() + 12, 4);
    if (eset_of.emplace(e, (uint32_t)esets.size()).second) esets.push_back(e);
  }
  for (auto& c : contains) {
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
  }
  auto reader_contains = [&](uint32_t r, const Eid& e) {
    return std::binary_search(contains[r].begin(), contains[r].end(), e);
  };
  auto rflags = [&](uint32_t r) {
    uint16_t f = readers[r].flags;
    if (memcmp(readers[r].entity_id, SPDP_PARTICIPANT_READER.data(), 4) == 0) f |= RTPS_TARGET_DUPLICATES_OK;
    return f;
  };
  // ---- target sets ----
  std::vector<uint32_t> first;
  std::vector<rtps_target> ent;
  uint32_t max_set = 0;
  const uint32_t n_sets = (uint32_t)(wsets.size() + esets.size());
  first.reserve(n_sets + 1);
  for (uint32_t s = 0; s < n_sets; ++s) {
    first.push_back((uint32_t)ent.size());
    const bool wset = s < wsets.size();
    Eid e;
    if (wset) memcpy(e.data(), wsets[s].data() + 12, 4);
    else e = esets[s - wsets.size()];
    for (uint32_t k = 0; k < nr; ++k) {
      const uint32_t r = order[k];
      if ((readers[r].flags & RTPS_READER_STATELESS) || !reader_contains(r, e)) continue;
      rtps_target x;
      x.reader_slot = readers[r].reader_slot;
      x.reader_flags = rflags(r);
      x.proxy = RTPS_NO_PROXY;
      if (wset) {
        auto it = proxy_of.find(std::make_pair(r, wsets[s]));
        if (it != proxy_of.end()) x.proxy = it->second;
      }
      ent.push_back(x);
    }
    max_set = std::max(max_set, (uint32_t)(ent.size() - first.back()));
  }
  first.push_back((uint32_t)ent.size());
  // ---- hash tables ----
  uint32_t gcap = pow2_at_least((uint64_t)RT_SLACK * wsets.size()), ecap = pow2_at_least((uint64_t)RT_SLACK * esets.size());
  if (rt_lds_bytes(gcap, ecap) > RT_LDS_MAX) {  // the sparse tables would leave LDS: the dense ones
    gcap = pow2_at_least((uint64_t)RT_SLACK_MIN * wsets.size());
    ecap = pow2_at_least((uint64_t)RT_SLACK_MIN * esets.size());
  }
  std::vector<uint32_t> gkeys((size_t)gcap * 4, 0u), gset(gcap, RTPS_NO_TARGET), ekeys(ecap, 0u),
      eset(ecap, RTPS_NO_TARGET);
  for (uint32_t s = 0; s < wsets.size(); ++s) {
    const uint8_t* g = wsets[s].data();
    const uint32_t a = word(g), b = word(g + 4), c = word(g + 8), d = word(g + 12);
    uint32_t i = rt_hash16(a, b, c, d) & (gcap - 1);
    while (gset[i] != RTPS_NO_TARGET) i = (i + 1) & (gcap - 1);
    gkeys[4 * (size_t)i] = a; gkeys[4 * (size_t)i + 1] = b; gkeys[4 * (size_t)i + 2] = c; gkeys[4 * (size_t)i + 3] = d;
    gset[i] = s;
  }
  for (uint32_t s = 0; s < esets.size(); ++s) {
    const uint32_t d = word(esets[s].data());
    uint32_t i = rt_hash4(d) & (ecap - 1);
    while (eset[i] != RTPS_NO_TARGET) i = (i + 1) & (ecap - 1);
    ekeys[i] = d;
    eset[i] = (uint32_t)wsets.size() + s;
  }
  out.first.swap(first);
  out.ent.swap(ent);
  out.gkeys.swap(gkeys); out.gset.swap(gset); out.ekeys.swap(ekeys); out.eset.swap(eset);
  out.gcap = gcap; out.ecap = ecap;
  out.n_writer_sets = (uint32_t)wsets.size();
  out.max_set = max_set;
  out.wguid.swap(wsets);
  out.eids.swap(esets);
  return RTPS_RX_OK;
}
}  // namespace

int rt_set(ReaderTable* t, const rtps_reader* readers, uint32_t nr, const rtps_proxy* proxies, uint32_t np,
           hipStream_t stream) {
  if (!t) return RTPS_RX_EINVAL;
  Built b;
  const int rc = build(readers, nr, proxies, np, b);
  if (rc) return rc;
  const uint32_t gcap = b.gcap, ecap = b.ecap;
  std::vector<uint32_t>&gkeys = b.gkeys, &gset = b.gset, &ekeys = b.ekeys, &eset = b.eset, &first = b.first;
  std::vector<rtps_target>& ent = b.ent;
  // ---- upload into new buffers; swap them in only when every step succeeded ----
  if (!g_mem.sync(stream)) return RTPS_RX_EHIP;  // the previous batch may still read the old tables
  // one buffer, the arrays back to back (ReaderDev: the LDS image, then the target sets)
  static_assert(sizeof(rtps_target) == 8 && alignof(rtps_target) <= 4, "target entries at word offsets");
  const void* src[6] = {gkeys.data(), gset.data(), ekeys.data(), eset.data(), first.data(), ent.data()};
  const size_t bytes[6] = {gkeys.size() * 4, gset.size() * 4, ekeys.size() * 4, eset.size() * 4, first.size() * 4,
                           ent.size() * sizeof(rtps_target)};
  size_t off[7] = {0};
  for (int k = 0; k < 6; ++k) off[k + 1] = off[k] + bytes[k];
  uint8_t* img = static_cast<uint8_t*>(g_mem.alloc(off[6]));
  if (!img) return RTPS_RX_ENOMEM;
  for (int k = 0; k < 6; ++k)
    if (!g_mem.upload(img + off[k], src[k], bytes[k])) {
      g_mem.release(img);
      return RTPS_RX_EHIP;
    }
  g_mem.release(t->gkeys);  // (the previous image: gkeys is its base)
  t->gkeys = (uint32_t*)(img + off[0]); t->gset = (uint32_t*)(img + off[1]); t->ekeys = (uint32_t*)(img + off[2]);
  t->eset = (uint32_t*)(img + off[3]); t->dfirst = (uint32_t*)(img + off[4]); t->dent = (rtps_target*)(img + off[5]);
  t->gcap = gcap;  // the images above are exactly gcap / ecap slots
  t->ecap = ecap;
  t->first.swap(first);
  t->ent.swap(ent);
  t->wguid.swap(b.wguid);
  t->eids.swap(b.eids);
  t->n_writer_sets = b.n_writer_sets;
  t->n_proxies = np;
  t->max_set = b.max_set;
  t->active = nr > 0;
  return RTPS_RX_OK;
}

int rt_set_match(ReaderTable* t, const rtps_match* m, uint32_t n, hipStream_t stream) {
  if (!t || (n && !m)) return RTPS_RX_EINVAL;
  std::vector<rtps_reader> readers;
  std::map<uint16_t, uint32_t> reader_of;
  std::vector<rtps_proxy> proxies;
  std::map<std::pair<uint32_t, Guid>, bool> seen;
  for (uint32_t k = 0; k < n; ++k) {
    if (m[k].reader_slot == RTPS_NO_MATCH) return RTPS_RX_EINVAL;
    auto it = reader_of.find(m[k].reader_slot);
    if (it == reader_of.end()) {
      const uint32_t r = (uint32_t)readers.size();
      rtps_reader x;
      // EntityId order = order of first appearance: big-endian reader number, user reader kind
      x.entity_id[0] = (uint8_t)(r >> 16); x.entity_id[1] = (uint8_t)(r >> 8); x.entity_id[2] = (uint8_t)r;
      x.entity_id[3] = 0x07;
      x.reader_slot = m[k].reader_slot;
      x.flags = 0;
      readers.push_back(x);
      it = reader_of.emplace(m[k].reader_slot, r).first;
    }
    Guid g;
    memcpy(g.data(), m[k].writer_guid, 16);
    if (!seen.emplace(std::make_pair(it->second, g), true).second) continue;
    rtps_proxy p;
    memcpy(p.writer_guid, m[k].writer_guid, 16);
    p.reader = it->second;
    proxies.push_back(p);
  }
  return rt_set(t, readers.data(), (uint32_t)readers.size(), proxies.data(), (uint32_t)proxies.size(), stream);
}

ReaderDev rt_dev(const ReaderTable* t) {
  ReaderDev r;
  memset(&r, 0, sizeof r);
  if (!t || !t->active) return r;
  r.gkeys = t->gkeys; r.gset = t->gset; r.ekeys = t->ekeys; r.eset = t->eset;
  r.set_first = t->dfirst; r.set_ent = t->dent;
  r.gmask = t->gcap - 1; r.emask = t->ecap - 1;
  r.n_writer_sets = t->n_writer_sets;
  r.n_sets = (uint32_t)t->first.size() - 1;
  r.n_proxies = t->n_proxies;
  r.max_set = t->max_set;
  r.n_ent = t->first.empty() ? 0u : t->first.back();
  return r;
}

const uint8_t* rt_writer_guids(const ReaderTable* t, uint32_t* n) {
  const bool on = t && t->active && !t->wguid.empty();
  *n = on ? (uint32_t)t->wguid.size() : 0u;
  return on ? t->wguid[0].data() : nullptr;
}

const uint8_t* rt_entity_ids(const ReaderTable* t, uint32_t* n) {
  const bool on = t && t->active && !t->eids.empty();
  *n = on ? (uint32_t)t->eids.size() : 0u;
  return on ? t->eids[0].data() : nullptr;
}

void rt_host(const ReaderTable* t, const uint32_t** first, const rtps_target** ent, uint32_t* n_sets) {
  static const uint32_t zero = 0;
  const bool on = t && t->active && !t->first.empty();
  if (first) *first = on ? t->first.data() : &zero;
  if (ent) *ent = on ? t->ent.data() : nullptr;
  if (n_sets) *n_sets = on ? (uint32_t)t->first.size() - 1 : 0;
}

/* test hook (not part of the public header, no GPU needed): the target sets
   rtps_rx_set_readers would build.  first: [n_sets + 1] (cap_sets + 1 room),
   ent: [cap_ent].  Returns RTPS_RX_OK, RTPS_RX_ETOOBIG when the room is short,
   or the validation error. */
extern "C" int rtps_rx_debug_target_sets(const rtps_reader* readers, uint32_t nr, const rtps_proxy* proxies,
                                         uint32_t np, uint32_t* first, uint32_t cap_sets, rtps_target* ent,
                                         uint32_t cap_ent, uint32_t* n_sets, uint32_t* n_writer_sets) {
  Built b;
  const int rc = build(readers, nr, proxies, np, b);
  if (rc) return rc;
  *n_sets = (uint32_t)b.first.size() - 1;
  *n_writer_sets = b.n_writer_sets;
  if (*n_sets > cap_sets || b.ent.size() > cap_ent) return RTPS_RX_ETOOBIG;
  memcpy(first, b.first.data(), b.first.size() * 4);
  if (!b.ent.empty()) memcpy(ent, b.ent.data(), b.ent.size() * sizeof(rtps_target));
  return RTPS_RX_OK;
}

/* test hooks (not part of the public header, no GPU needed): a reader table on
   host memory whose fail_at-th buffer allocation fails (-1: none), to check that
   a failed rtps_rx_set_readers leaves the previous table in place. */
extern "C" {
int rtps_rx_debug_rt_host_mode(int fail_at) {
  g_mem = {host_alloc, host_release, host_upload, host_sync};
  g_fail_at = fail_at;
  g_allocs = 0;
  return RTPS_RX_OK;
}
void* rtps_rx_debug_rt_new(void) { return rt_new(); }
void rtps_rx_debug_rt_free(void* t) { rt_free(static_cast<ReaderTable*>(t)); }
int rtps_rx_debug_rt_set(void* t, const rtps_reader* readers, uint32_t nr, const rtps_proxy* proxies, uint32_t np) {
  return rt_set(static_cast<ReaderTable*>(t), readers, nr, proxies, np, nullptr);
}
/* the device view rt_dev returns (pointers into the table's buffers) */
/* sizeof(ReaderDev): a debug hook's caller must mirror the struct exactly (rtps_rx_debug_rt_view
   writes the whole struct) */
uint32_t rtps_rx_debug_rt_view_size(void) { return (uint32_t)sizeof(ReaderDev); }
static_assert(sizeof(ReaderDev) == 6 * sizeof(void*) + 8 * sizeof(uint32_t),
              "ReaderDev changed: update the debug mirrors (tests/test_readers_cpu.py View)");
int rtps_rx_debug_rt_view(const void* t, ReaderDev* out) {
  if (!out) return RTPS_RX_EINVAL;
  *out = rt_dev(static_cast<const ReaderTable*>(t));
  return RTPS_RX_OK;
}
}
