// rtps_udp.cpp — UDP batch receive into a datagram arena.
//
// The reference receives with one io_uring RecvMulti per socket on a provided
// buffer ring (io_uring/network/udp_listener.rs:101-209) and copies every
// completion into a fresh Bytes before parsing it
// (io_uring/rtps/dp_event_loop.rs:190-211).  Here the provided buffers are the
// slots of the caller's arena, so the kernel writes each datagram where the
// batch parser (rtps_rx_parse_batch) reads it: a batch is (offset, length)
// pairs, no copy.  The ring is driven through the raw io_uring syscalls
// (linux/io_uring.h; liburing is not needed); a recvmmsg backend fills the same
// slots where io_uring is unavailable.
#include <errno.h>
#include <linux/io_uring.h>
#include <netinet/in.h>
#include <poll.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <new>
#include <vector>

#include "../../include/rtps_rx.h"

// Kernel ABI this image's 5.15 uapi headers predate (stable since Linux 5.19 /
// 6.0; the running kernel is checked at open and the recvmmsg backend is used
// when it refuses).
#ifndef IORING_RECV_MULTISHOT
#define IORING_RECV_MULTISHOT (1U << 1)
#endif
constexpr unsigned REGISTER_PBUF_RING = 22;  // IORING_REGISTER_PBUF_RING
struct uring_buf {                            // struct io_uring_buf
  uint64_t addr;
  uint32_t len;
  uint16_t bid;
  uint16_t resv;
};
struct uring_buf_ring {                       // struct io_uring_buf_ring: tail overlays bufs[0].resv
  union {
    struct { uint64_t resv1; uint32_t resv2; uint16_t resv3; uint16_t tail; };
    uring_buf bufs[1];
  };
};
struct uring_buf_reg {                        // struct io_uring_buf_reg
  uint64_t ring_addr;
  uint32_t ring_entries;
  uint16_t bgid;
  uint16_t flags;
  uint64_t resv[3];
};
static_assert(sizeof(uring_buf) == 16 && sizeof(uring_buf_reg) == 40, "io_uring buffer-ring ABI");

namespace {

constexpr uint16_t BGID = 0x5254;  // buffer group id of the arena slots
constexpr uint64_t UD_RECV = 1;    // user_data of the multishot recv

int sys_setup(unsigned entries, io_uring_params* p) { return (int)syscall(__NR_io_uring_setup, entries, p); }
int sys_enter(int fd, unsigned submit, unsigned min_complete, unsigned flags) {
  return (int)syscall(__NR_io_uring_enter, fd, submit, min_complete, flags, nullptr, 0);
}
int sys_register(int fd, unsigned op, void* arg, unsigned n) { return (int)syscall(__NR_io_uring_register, fd, op, arg, n); }

template <typename T>
T* at(void* base, uint32_t off) { return reinterpret_cast<T*>(static_cast<uint8_t*>(base) + off); }

}  // namespace

struct rtps_udp_rx {
  int sock = -1;
  int backend = 0;
  uint8_t* arena = nullptr;
  uint32_t slot_bytes = 0, n_slots = 0;
  uint16_t port = 0;
  // io_uring
  int ring = -1;
  void* sq_map = nullptr;
  size_t sq_map_len = 0;
  void* cq_map = nullptr;
  size_t cq_map_len = 0;
  io_uring_sqe* sqes = nullptr;
  size_t sqes_len = 0;
  unsigned *sq_head = nullptr, *sq_tail = nullptr, *sq_mask = nullptr, *sq_array = nullptr;
  unsigned *cq_head = nullptr, *cq_tail = nullptr, *cq_mask = nullptr;
  io_uring_cqe* cqes = nullptr;
  uring_buf_ring* br = nullptr;  // provided-buffer ring (n_slots entries)
  size_t br_len = 0;
  uint16_t br_tail = 0;
  bool armed = false;
  bool sqpoll = false;              // a kernel thread issues the recv and runs its completions
  unsigned* sq_flags = nullptr;
  uint32_t provided = 0;            // slots currently owned by the kernel
  // recvmmsg
  std::vector<uint32_t> free_slots;
  std::vector<mmsghdr> msgs;
  std::vector<iovec> iovs;
};

static void ring_teardown(rtps_udp_rx* r) {
  if (r->br) munmap(r->br, r->br_len);
  if (r->sqes) munmap(r->sqes, r->sqes_len);
  if (r->cq_map && r->cq_map != r->sq_map) munmap(r->cq_map, r->cq_map_len);
  if (r->sq_map) munmap(r->sq_map, r->sq_map_len);
  if (r->ring >= 0) close(r->ring);
  r->br = nullptr; r->sqes = nullptr; r->cq_map = nullptr; r->sq_map = nullptr; r->ring = -1;
}

// one more slot for the kernel (visible after ring_publish)
static void ring_provide(rtps_udp_rx* r, uint32_t slot) {
  const uint32_t mask = r->n_slots - 1u;
  uring_buf* b = &r->br->bufs[r->br_tail & mask];
  b->addr = (uint64_t)(uintptr_t)(r->arena + (uint64_t)slot * r->slot_bytes);
  b->len = r->slot_bytes;
  b->bid = (uint16_t)slot;
  r->br_tail++;
  r->provided++;
}
static void ring_publish(rtps_udp_rx* r) { __atomic_store_n(&r->br->tail, r->br_tail, __ATOMIC_RELEASE); }

// (re)arm the multishot recv: every datagram completes into a provided slot
static int ring_arm(rtps_udp_rx* r) {
  const unsigned tail = *r->sq_tail, idx = tail & *r->sq_mask;
  io_uring_sqe* e = &r->sqes[idx];
  memset(e, 0, sizeof(*e));
  e->opcode = IORING_OP_RECV;
  e->fd = r->sock;
  e->ioprio = IORING_RECV_MULTISHOT;
  e->flags = IOSQE_BUFFER_SELECT;
  e->buf_group = BGID;
  e->msg_flags = MSG_TRUNC;  // report the datagram's real length (truncation detection)
  e->user_data = UD_RECV;
  r->sq_array[idx] = idx;
  __atomic_store_n(r->sq_tail, tail + 1u, __ATOMIC_RELEASE);
  if (r->sqpoll) {  // the poll thread takes the entry; wake it if it went idle
    if (__atomic_load_n(r->sq_flags, __ATOMIC_ACQUIRE) & IORING_SQ_NEED_WAKEUP)
      (void)sys_enter(r->ring, 0, 0, IORING_ENTER_SQ_WAKEUP);
    for (int spin = 0; __atomic_load_n(r->sq_head, __ATOMIC_ACQUIRE) != tail + 1u; ++spin) {
      if (spin > 100000) return RTPS_RX_EINVAL;
      if (__atomic_load_n(r->sq_flags, __ATOMIC_ACQUIRE) & IORING_SQ_NEED_WAKEUP)
        (void)sys_enter(r->ring, 0, 0, IORING_ENTER_SQ_WAKEUP);
      usleep(10);
    }
  } else if (sys_enter(r->ring, 1, 0, 0) != 1) {
    return RTPS_RX_EINVAL;
  }
  r->armed = true;
  return RTPS_RX_OK;
}

static bool ring_setup(rtps_udp_rx* r, bool sqpoll) {
  io_uring_params p;
  memset(&p, 0, sizeof(p));
  p.flags = IORING_SETUP_CQSIZE | (sqpoll ? IORING_SETUP_SQPOLL : 0u);
  p.cq_entries = 2u * r->n_slots;  // every provided slot can hold one completion, plus errors
  p.sq_thread_idle = 100;          // ms the poll thread spins before it sleeps
  r->ring = sys_setup(8, &p);
  if (r->ring < 0) return false;
  r->sqpoll = sqpoll;
  r->sq_map_len = p.sq_off.array + p.sq_entries * sizeof(unsigned);
  r->cq_map_len = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
  const bool single = (p.features & IORING_FEAT_SINGLE_MMAP) != 0;
  if (single && r->cq_map_len > r->sq_map_len) r->sq_map_len = r->cq_map_len;
  r->sq_map = mmap(nullptr, r->sq_map_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->ring, IORING_OFF_SQ_RING);
  if (r->sq_map == MAP_FAILED) { r->sq_map = nullptr; ring_teardown(r); return false; }
  r->cq_map = single ? r->sq_map
                     : mmap(nullptr, r->cq_map_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->ring,
                            IORING_OFF_CQ_RING);
  if (r->cq_map == MAP_FAILED) { r->cq_map = nullptr; ring_teardown(r); return false; }
  r->sqes_len = p.sq_entries * sizeof(io_uring_sqe);
  void* sq = mmap(nullptr, r->sqes_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->ring, IORING_OFF_SQES);
  if (sq == MAP_FAILED) { ring_teardown(r); return false; }
  r->sqes = static_cast<io_uring_sqe*>(sq);
  r->sq_head = at<unsigned>(r->sq_map, p.sq_off.head);
  r->sq_tail = at<unsigned>(r->sq_map, p.sq_off.tail);
  r->sq_mask = at<unsigned>(r->sq_map, p.sq_off.ring_mask);
  r->sq_array = at<unsigned>(r->sq_map, p.sq_off.array);
  r->sq_flags = at<unsigned>(r->sq_map, p.sq_off.flags);
  r->cq_head = at<unsigned>(r->cq_map, p.cq_off.head);
  r->cq_tail = at<unsigned>(r->cq_map, p.cq_off.tail);
  r->cq_mask = at<unsigned>(r->cq_map, p.cq_off.ring_mask);
  r->cqes = at<io_uring_cqe>(r->cq_map, p.cq_off.cqes);
  // the arena slots as a registered provided-buffer ring
  r->br_len = ((size_t)r->n_slots * sizeof(uring_buf) + 4095) & ~(size_t)4095;
  void* br = mmap(nullptr, r->br_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
  if (br == MAP_FAILED) { ring_teardown(r); return false; }
  r->br = static_cast<uring_buf_ring*>(br);
  uring_buf_reg reg;
  memset(&reg, 0, sizeof(reg));
  reg.ring_addr = (uint64_t)(uintptr_t)br;
  reg.ring_entries = r->n_slots;
  reg.bgid = BGID;
  if (sys_register(r->ring, REGISTER_PBUF_RING, &reg, 1) != 0) { ring_teardown(r); return false; }
  r->br_tail = 0;
  for (uint32_t s = 0; s < r->n_slots; ++s) ring_provide(r, s);
  ring_publish(r);
  if (ring_arm(r) != RTPS_RX_OK) { ring_teardown(r); return false; }
  // a kernel without multishot recv completes the request at once with an error
  const unsigned head = *r->cq_head;
  if (head != __atomic_load_n(r->cq_tail, __ATOMIC_ACQUIRE)) {
    const io_uring_cqe* c = &r->cqes[head & *r->cq_mask];
    if (c->res < 0 && !(c->flags & IORING_CQE_F_BUFFER)) { ring_teardown(r); return false; }
  }
  return true;
}

static int64_t now_ms() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000 + t.tv_nsec / 1000000;
}

static int ring_recv(rtps_udp_rx* r, uint64_t* off, uint32_t* len, uint32_t max_n, int timeout_ms, uint64_t* trunc) {
  uint32_t n = 0;
  const int64_t deadline = timeout_ms > 0 ? now_ms() + timeout_ms : 0;
  for (;;) {
    // multishot completions are posted from task work, which runs when this
    // thread enters the kernel: enter once so arrived datagrams show up
    (void)sys_enter(r->ring, 0, 0, IORING_ENTER_GETEVENTS);
    unsigned head = *r->cq_head;
    const unsigned tail = __atomic_load_n(r->cq_tail, __ATOMIC_ACQUIRE);
    bool reprovide = false;
    while (head != tail && n < max_n) {
      const io_uring_cqe* c = &r->cqes[head & *r->cq_mask];
      if (c->user_data == UD_RECV) {
        if (!(c->flags & IORING_CQE_F_MORE)) r->armed = false;  // multishot ended (-ENOBUFS: no free slot)
        if (c->flags & IORING_CQE_F_BUFFER) {
          const uint32_t slot = c->flags >> IORING_CQE_BUFFER_SHIFT;
          r->provided--;
          if (c->res >= 0 && (uint32_t)c->res <= r->slot_bytes) {
            off[n] = (uint64_t)slot * r->slot_bytes;
            len[n] = (uint32_t)c->res;
            ++n;
          } else {  // longer than a slot: dropped, slot goes straight back
            if (c->res > 0 && trunc) ++*trunc;
            ring_provide(r, slot);
            reprovide = true;
          }
        } else if (c->res < 0 && c->res != -ENOBUFS) {
          __atomic_store_n(r->cq_head, head + 1u, __ATOMIC_RELEASE);
          return RTPS_RX_EINVAL;
        }
      }
      ++head;
    }
    __atomic_store_n(r->cq_head, head, __ATOMIC_RELEASE);
    if (reprovide) ring_publish(r);
    // re-arm after -ENOBUFS once slots are back (traffic.rs:246-284 does the same on error 105)
    if (!r->armed && r->provided > 0) {
      const int rc = ring_arm(r);
      if (rc != RTPS_RX_OK) return rc;
    }
    if (n > 0 || timeout_ms == 0) return (int)n;
    if (!r->armed) return 0;  // no slot to receive into: the caller must release
    int wait = -1;
    if (timeout_ms > 0) {
      const int64_t left = deadline - now_ms();
      if (left <= 0) return 0;
      wait = (int)left;
    }
    pollfd pf{r->ring, POLLIN, 0};
    if (poll(&pf, 1, wait) < 0 && errno != EINTR) return RTPS_RX_EINVAL;
  }
}

static int mmsg_recv(rtps_udp_rx* r, uint64_t* off, uint32_t* len, uint32_t max_n, int timeout_ms, uint64_t* trunc) {
  if (r->free_slots.empty()) return 0;
  if (timeout_ms != 0) {
    pollfd pf{r->sock, POLLIN, 0};
    if (poll(&pf, 1, timeout_ms) <= 0) return 0;
  }
  uint32_t n = 0;
  while (n < max_n && !r->free_slots.empty()) {
    uint32_t k = max_n - n;
    if (k > r->free_slots.size()) k = (uint32_t)r->free_slots.size();
    uint32_t* slots = r->free_slots.data() + (r->free_slots.size() - k);  // the k slots popped next
    for (uint32_t j = 0; j < k; ++j) {
      r->iovs[j].iov_base = r->arena + (uint64_t)slots[k - 1 - j] * r->slot_bytes;
      r->iovs[j].iov_len = r->slot_bytes;
      memset(&r->msgs[j], 0, sizeof(mmsghdr));
      r->msgs[j].msg_hdr.msg_iov = &r->iovs[j];
      r->msgs[j].msg_hdr.msg_iovlen = 1;
    }
    const int got = recvmmsg(r->sock, r->msgs.data(), k, MSG_DONTWAIT, nullptr);
    if (got <= 0) break;
    std::vector<uint32_t> back;  // slots of truncated datagrams (dropped) and unused ones
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t slot = slots[k - 1 - j];
      if ((int)j < got && !(r->msgs[j].msg_hdr.msg_flags & MSG_TRUNC)) {
        off[n] = (uint64_t)slot * r->slot_bytes;
        len[n] = r->msgs[j].msg_len;
        ++n;
      } else {
        if ((int)j < got && trunc) ++*trunc;
        back.push_back(slot);
      }
    }
    r->free_slots.resize(r->free_slots.size() - k);
    for (size_t j = back.size(); j-- > 0;) r->free_slots.push_back(back[j]);
    if ((uint32_t)got < k) break;
  }
  return (int)n;
}

extern "C" {

int rtps_udp_open(const rtps_udp_config* cfg, rtps_udp_rx** out) {
  if (!cfg || !out || !cfg->arena) return RTPS_RX_EINVAL;
  if (cfg->abi_version != RTPS_RX_ABI_VERSION) return RTPS_RX_EABI;
  const uint32_t B = cfg->slot_bytes, N = cfg->n_slots;
  if (B < 32 || B > 65536 || (B & 15u) || N < 2 || N > 32768 || (N & (N - 1u))) return RTPS_RX_EINVAL;
  rtps_udp_rx* r = new (std::nothrow) rtps_udp_rx();
  if (!r) return RTPS_RX_ENOMEM;
  r->arena = cfg->arena;
  r->slot_bytes = B;
  r->n_slots = N;
  r->sock = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, IPPROTO_UDP);
  if (r->sock < 0) { delete r; return RTPS_RX_EINVAL; }
  int one = 1;
  if (cfg->flags & RTPS_UDP_REUSE) {
    (void)setsockopt(r->sock, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    (void)setsockopt(r->sock, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  }
  if (cfg->rcvbuf_bytes) {
    int v = (int)cfg->rcvbuf_bytes;
    (void)setsockopt(r->sock, SOL_SOCKET, SO_RCVBUF, &v, sizeof(v));
  }
  sockaddr_in a;
  memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  a.sin_port = htons(cfg->port);
  a.sin_addr.s_addr = htonl(cfg->ipv4_addr);
  if (bind(r->sock, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) { close(r->sock); delete r; return RTPS_RX_EINVAL; }
  if (cfg->multicast_group) {
    ip_mreq m;
    m.imr_multiaddr.s_addr = htonl(cfg->multicast_group);
    m.imr_interface.s_addr = htonl(INADDR_ANY);
    if (setsockopt(r->sock, IPPROTO_IP, IP_ADD_MEMBERSHIP, &m, sizeof(m)) != 0) {
      close(r->sock); delete r; return RTPS_RX_EINVAL;
    }
  }
  socklen_t al = sizeof(a);
  (void)getsockname(r->sock, reinterpret_cast<sockaddr*>(&a), &al);
  r->port = ntohs(a.sin_port);
  const bool try_ring = !(cfg->flags & RTPS_UDP_FORCE_RECVMMSG);
  if (try_ring && (((cfg->flags & RTPS_UDP_SQPOLL) && ring_setup(r, true)) || ring_setup(r, false))) {
    r->backend = RTPS_UDP_IO_URING;
  } else {
    r->backend = RTPS_UDP_RECVMMSG;
    r->free_slots.resize(N);
    for (uint32_t s = 0; s < N; ++s) r->free_slots[s] = N - 1u - s;  // pop order 0, 1, 2, ...
    r->msgs.resize(N);
    r->iovs.resize(N);
  }
  *out = r;
  return RTPS_RX_OK;
}

int rtps_udp_close(rtps_udp_rx* r) {
  if (!r) return RTPS_RX_EINVAL;
  ring_teardown(r);
  if (r->sock >= 0) close(r->sock);
  delete r;
  return RTPS_RX_OK;
}

int rtps_udp_port(const rtps_udp_rx* r) { return r ? (int)r->port : RTPS_RX_EINVAL; }
int rtps_udp_backend(const rtps_udp_rx* r) {
  if (!r) return RTPS_RX_EINVAL;
  return r->backend == RTPS_UDP_IO_URING && r->sqpoll ? RTPS_UDP_IO_URING_SQPOLL : r->backend;
}

int rtps_udp_recv_batch(rtps_udp_rx* r, uint64_t* off, uint32_t* len, uint32_t max_n, int timeout_ms,
                        uint64_t* truncated) {
  if (!r || (max_n && (!off || !len))) return RTPS_RX_EINVAL;
  if (max_n == 0) return 0;
  return r->backend == RTPS_UDP_IO_URING ? ring_recv(r, off, len, max_n, timeout_ms, truncated)
                                         : mmsg_recv(r, off, len, max_n, timeout_ms, truncated);
}

int rtps_udp_release(rtps_udp_rx* r, const uint64_t* off, uint32_t n) {
  if (!r || (n && !off)) return RTPS_RX_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (off[i] % r->slot_bytes || off[i] / r->slot_bytes >= r->n_slots) return RTPS_RX_EINVAL;
  if (r->backend == RTPS_UDP_IO_URING) {
    for (uint32_t i = 0; i < n; ++i) ring_provide(r, (uint32_t)(off[i] / r->slot_bytes));
    ring_publish(r);
    if (!r->armed && r->provided > 0) return ring_arm(r);
  } else {
    for (uint32_t i = 0; i < n; ++i) r->free_slots.push_back((uint32_t)(off[i] / r->slot_bytes));
  }
  return RTPS_RX_OK;
}

int rtps_udp_send_batch(uint32_t ipv4_addr, uint16_t port, const uint8_t* arena, const uint64_t* off,
                        const uint32_t* len, uint32_t n) {
  if (n && (!arena || !off || !len)) return RTPS_RX_EINVAL;
  const int s = socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, IPPROTO_UDP);
  if (s < 0) return RTPS_RX_EINVAL;
  int sz = 8 << 20;
  (void)setsockopt(s, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  sockaddr_in a;
  memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  a.sin_addr.s_addr = htonl(ipv4_addr);
  constexpr uint32_t K = 256;
  mmsghdr msgs[K];
  iovec iov[K];
  uint32_t sent = 0, stalls = 0;
  while (sent < n) {
    const uint32_t k = (n - sent) < K ? (n - sent) : K;
    for (uint32_t j = 0; j < k; ++j) {
      iov[j].iov_base = const_cast<uint8_t*>(arena + off[sent + j]);
      iov[j].iov_len = len[sent + j];
      memset(&msgs[j], 0, sizeof(mmsghdr));
      msgs[j].msg_hdr.msg_name = &a;
      msgs[j].msg_hdr.msg_namelen = sizeof(a);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
    }
    const int got = sendmmsg(s, msgs, k, 0);
    if (got <= 0) {
      // a full device/socket queue is transient (ENOBUFS, EAGAIN): wait for room and retry
      if (got < 0 && (errno == ENOBUFS || errno == EAGAIN || errno == EINTR) && ++stalls < 100000) {
        pollfd pf{s, POLLOUT, 0};
        (void)poll(&pf, 1, 1);
        continue;
      }
      break;
    }
    sent += (uint32_t)got;
  }
  close(s);
  return (int)sent;
}

}  // extern "C"
