// Parity check through the C++ mirror (include/rtps_rx.hpp): parse a batch
// dumped by tests/test_cpp_mirror.py and compare with the oracle's outputs.
// usage: receiver_check <dir>   (dir holds arena.bin off.bin len.bin own.bin status.bin records.bin)
#include <cstdio>
#include <fstream>
#include <iterator>

#include "rtps_rx.hpp"

template <class T>
static std::vector<T> load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<T> v(b.size() / sizeof(T));
  std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::string d = argv[1];
  auto arena = load<uint8_t>(d + "/arena.bin");
  auto off = load<uint64_t>(d + "/off.bin");
  auto len = load<uint32_t>(d + "/len.bin");
  auto own_v = load<uint8_t>(d + "/own.bin");
  auto status = load<uint8_t>(d + "/status.bin");
  auto recs = load<rtps_record>(d + "/records.bin");
  std::array<uint8_t, 12> own{};
  std::memcpy(own.data(), own_v.data(), 12);
  try {
    rtps_rx::MessageReceiver rx(own, 0, (uint32_t)len.size());
    auto r = rx.handle_received_batch(arena, off, len);
    bool ok = r.status == status && r.n_records == recs.size() &&
              std::memcmp(r.records.data(), recs.data(), recs.size() * sizeof(rtps_record)) == 0;
    size_t passed = 0;
    for (size_t i = 0; i < len.size(); ++i) passed += r.passed_submessages(i).size();
    // single-datagram API == the batch result for that datagram
    auto one = rx.read_from_buffer(std::vector<uint8_t>(arena.begin() + off[0], arena.begin() + off[0] + len[0]));
    auto s0 = r.submessages(0);
    ok = ok && one.status[0] == r.status[0] && (size_t)one.n_records == (size_t)(s0.second - s0.first);
    std::printf("%s: %zu datagrams, %llu records, %zu passed submessages\n", ok ? "OK" : "MISMATCH", len.size(),
                (unsigned long long)r.n_records, passed);
    return ok ? 0 : 1;
  } catch (const std::exception& e) {
    std::printf("ERROR %s\n", e.what());
    return 3;
  }
}
