// rtps_rx.hpp — C++17 RAII mirror of the receive path over the C ABI (rtps_rx.h).
//
// Same object model as the reference (and the Python mirror):
//   rtps_rx::MessageReceiver(own_prefix)       io_uring/rtps/message_receiver.rs:158-182
//   .handle_received_batch(arena, off, len)    batch form of handle_received_packet_2 (:232-287)
//   .read_from_buffer(datagram)                Message::read_from_buffer (rtps/message.rs:64-81), one datagram
//   BatchResult::submessages(i)                Message.submessages of datagram i
//   BatchResult::passed_submessages(i)         what SubmessageIter2::next yields (:56-119):
//                                              PassedSubmessage::{Writer, Reader(source prefix)}
// Host code only: device memory comes from the HIP runtime, the parse from the library.
#pragma once
#include <hip/hip_runtime_api.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtps_rx.h"

namespace rtps_rx {

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};
inline void check(int rc, const char* what) {
  if (rc != RTPS_RX_OK) throw Error(std::string(what) + ": " + rtps_rx_strerror(rc));
}
inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
class DeviceBuffer {
 public:
  explicit DeviceBuffer(size_t n) : n_(n) { hip_check(hipMalloc(&p_, (n ? n : 1) * sizeof(T)), "hipMalloc"); }
  ~DeviceBuffer() { (void)hipFree(p_); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  T* get() const { return p_; }
  size_t size() const { return n_; }
  void upload(const T* src, size_t n) { hip_check(hipMemcpy(p_, src, n * sizeof(T), hipMemcpyHostToDevice), "H2D"); }
  void download(T* dst, size_t n) const {
    hip_check(hipMemcpy(dst, p_, n * sizeof(T), hipMemcpyDeviceToHost), "D2H");
  }

 private:
  T* p_ = nullptr;
  size_t n_;
};

inline bool is_writer_kind(uint8_t k) {
  return k == RTPS_DATA || k == RTPS_DATA_FRAG || k == RTPS_HEARTBEAT || k == RTPS_HEARTBEAT_FRAG || k == RTPS_GAP;
}

// PassedSubmessage (io_uring/rtps/message_receiver.rs:39-43)
struct PassedSubmessage {
  enum class Kind { Writer, Reader } kind;
  const rtps_record* rec;               // the parsed submessage
  std::array<uint8_t, 12> source_prefix;  // Reader(_, GuidPrefix); writer GUID prefix for Writer
};

struct BatchResult {
  std::vector<uint8_t> status;
  std::vector<rtps_record> records;
  std::vector<uint32_t> target;  // target set per record (RTPS_NO_TARGET: none)
  std::vector<uint32_t> rec_begin;
  uint64_t n_records = 0;

  std::pair<const rtps_record*, const rtps_record*> submessages(size_t i) const {
    if (status[i] != RTPS_DGRAM_OK) return {nullptr, nullptr};
    size_t lo = rec_begin[i], hi = i + 1 < rec_begin.size() ? rec_begin[i + 1] : (size_t)n_records;
    return {records.data() + lo, records.data() + hi};
  }
  std::vector<PassedSubmessage> passed_submessages(size_t i) const {
    std::vector<PassedSubmessage> v;
    auto r = submessages(i);
    for (const rtps_record* p = r.first; p != r.second; ++p) {
      if (!(p->route & RTPS_ROUTE_PASS)) continue;
      PassedSubmessage s;
      s.kind = is_writer_kind(p->kind) ? PassedSubmessage::Kind::Writer : PassedSubmessage::Kind::Reader;
      s.rec = p;
      std::memcpy(s.source_prefix.data(), p->prefix, 12);
      v.push_back(s);
    }
    return v;
  }
};

class MessageReceiver {
 public:
  MessageReceiver(const std::array<uint8_t, 12>& own_prefix, int device = 0, uint32_t max_datagrams = 1u << 20)
      : max_datagrams_(max_datagrams) {
    rtps_rx_config cfg{};
    cfg.abi_version = RTPS_RX_ABI_VERSION;
    cfg.device = device;
    std::memcpy(cfg.own_prefix, own_prefix.data(), 12);
    cfg.max_datagrams = max_datagrams;
    check(rtps_rx_create(&cfg, &ctx_), "rtps_rx_create");
  }
  ~MessageReceiver() { rtps_rx_destroy(ctx_); }
  MessageReceiver(const MessageReceiver&) = delete;
  MessageReceiver& operator=(const MessageReceiver&) = delete;

  rtps_rx_ctx* handle() const { return ctx_; }
  void set_match_table(const std::vector<rtps_match>& t) {
    check(rtps_rx_set_match_table(ctx_, t.data(), (uint32_t)t.size()), "rtps_rx_set_match_table");
  }
  // available_readers + each Reader's matched_writers (see rtps_rx_set_readers)
  void set_readers(const std::vector<rtps_reader>& readers, const std::vector<rtps_proxy>& proxies) {
    check(rtps_rx_set_readers(ctx_, readers.data(), (uint32_t)readers.size(), proxies.data(),
                              (uint32_t)proxies.size()),
          "rtps_rx_set_readers");
  }
  // the target readers of a record's target set (empty for RTPS_NO_TARGET)
  std::vector<rtps_target> targets(uint32_t target) const {
    const uint32_t* first = nullptr;
    const rtps_target* ent = nullptr;
    uint32_t n = 0;
    check(rtps_rx_target_table(ctx_, &first, &ent, &n), "rtps_rx_target_table");
    if (target == RTPS_NO_TARGET || target >= n) return {};
    return std::vector<rtps_target>(ent + first[target], ent + first[target + 1]);
  }

  // host datagrams in (arena + offsets + lengths), host results out
  BatchResult handle_received_batch(const std::vector<uint8_t>& arena, const std::vector<uint64_t>& off,
                                    const std::vector<uint32_t>& len) {
    const uint32_t n = (uint32_t)len.size();
    const uint64_t cap = rtps_rx_max_records_host(len.data(), n);
    DeviceBuffer<uint8_t> d_arena(arena.size());
    DeviceBuffer<uint64_t> d_off(n), d_n(1);
    DeviceBuffer<uint32_t> d_len(n), d_rb(n);
    DeviceBuffer<uint8_t> d_status(n);
    DeviceBuffer<rtps_record> d_recs(cap);
    DeviceBuffer<uint32_t> d_target(cap);
    d_arena.upload(arena.data(), arena.size());
    d_off.upload(off.data(), n);
    d_len.upload(len.data(), n);
    rtps_rx_out out{d_status.get(), d_recs.get(), cap, d_target.get(), d_rb.get(), d_n.get()};
    check(rtps_rx_parse_batch(ctx_, d_arena.get(), arena.size(), d_off.get(), d_len.get(), n, &out),
          "rtps_rx_parse_batch");
    check(rtps_rx_sync(ctx_), "rtps_rx_sync");
    BatchResult r;
    d_n.download(&r.n_records, 1);
    const size_t kept = r.n_records < cap ? (size_t)r.n_records : (size_t)cap;
    r.status.resize(n);
    r.rec_begin.resize(n);
    r.records.resize(kept);
    r.target.resize(kept);
    d_status.download(r.status.data(), n);
    d_rb.download(r.rec_begin.data(), n);
    d_recs.download(r.records.data(), kept);
    d_target.download(r.target.data(), kept);
    return r;
  }

  // Message::read_from_buffer for one datagram: status + its submessages
  BatchResult read_from_buffer(const std::vector<uint8_t>& datagram) {
    return handle_received_batch(datagram, {0}, {(uint32_t)datagram.size()});
  }

 private:
  rtps_rx_ctx* ctx_ = nullptr;
  uint32_t max_datagrams_;
};

}  // namespace rtps_rx
