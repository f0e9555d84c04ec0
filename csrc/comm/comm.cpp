// First-party collective communication layer (SURVEY §1.2 "L0 comm", §2.5, §2.7, §5.8).
//
// The reference's workers and PS talk over TF 1.4's gRPC runtime: a server per
// task bound to its cluster-spec endpoint (examples/workdir/mnist_replica.py:117-122),
// variables placed on the PS tasks (:137-141) and pulled / pushed on every step
// (:256).  Here the same traffic is RCCL over xGMI, driven from this library:
//
//   bootstrap   rank 0 (the chief) listens on a TCP port of its node and every
//               other rank connects (the address travels through the job's
//               endpoint registry / rendezvous store); rank 0 hands out the
//               128-byte unique id it got from ncclGetUniqueId plus every rank's
//               address, then each rank calls ncclCommInitRank.  One TCP
//               exchange per communicator, nothing after it.
//   collectives all-reduce / reduce-scatter / all-gather / broadcast / reduce
//               and grouped point-to-point send / recv (the async PS and the
//               embedding all-to-all) straight on the caller's flat buffers, on
//               the HIP stream the caller passes (parallel/comm.py gives every
//               communicator its own stream and hands the result back with an
//               event, so the optimizer waits only for the buckets it reads).
//
// Two interchangeable backends behind one C ABI:
//   "rccl"  librccl resolved at run time: the copy the process already has
//           mapped (PyTorch-ROCm links one) or /opt/rocm/lib/librccl.so.1 — one
//           RCCL per process, whoever loaded it first.
//   "host"  the same collectives over host memory and a TCP mesh between the
//           ranks: the CPU build of this layer, so the communicator logic
//           (bootstrap, collective semantics, grouping, error paths) is tested
//           against gloo on a machine without a GPU (tests/test_comm_cpu.py).
//           Reductions run in rank order, so every rank gets identical bits.
//
// Every entry point returns 0 or an error code; kfc_last_error() describes it.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <link.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#define KFC_API extern "C" __attribute__((visibility("default")))

namespace kfc {

// ncclDataType_t / ncclRedOp_t values (rccl.h), so the RCCL backend passes them through
enum Dtype { I8 = 0, U8 = 1, I32 = 2, U32 = 3, I64 = 4, U64 = 5, F16 = 6, F32 = 7, F64 = 8, BF16 = 9, NDT = 10 };
enum Op { SUM = 0, PROD = 1, MAX = 2, MIN = 3, AVG = 4, NOPS = 5 };
enum Err { OK = 0, E_ARG = 1, E_SYS = 2, E_TIMEOUT = 3, E_PROTO = 4, E_LIB = 5, E_RCCL = 6, E_STATE = 7 };
constexpr uint32_t kMagic = 0x4b464331;  // "KFC1"
constexpr int kIdBytes = 128;

thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

static size_t dsize(int dt) {
  switch (dt) {
    case I8: case U8: return 1;
    case F16: case BF16: return 2;
    case I32: case U32: case F32: return 4;
    case I64: case U64: case F64: return 8;
    default: return 0;
  }
}

using Clock = std::chrono::steady_clock;
static int64_t ms_left(Clock::time_point deadline) {
  return std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
}

// ------------------------------------------------------------------ TCP helpers
static void set_nodelay(int fd) {
  int one = 1;
  (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

static int wait_fd(int fd, short ev, Clock::time_point deadline) {
  for (;;) {
    const int64_t left = ms_left(deadline);
    if (left <= 0) return fail(E_TIMEOUT, "timed out waiting on a peer socket");
    pollfd p{fd, ev, 0};
    const int r = poll(&p, 1, (int)std::min<int64_t>(left, 1000));
    if (r > 0) {
      if (p.revents & (POLLERR | POLLNVAL)) return fail(E_SYS, "peer socket error");
      return OK;
    }
    if (r < 0 && errno != EINTR) return fail(E_SYS, std::string("poll: ") + strerror(errno));
  }
}

static int send_all(int fd, const void* buf, size_t n, Clock::time_point deadline) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (k > 0) { p += k; n -= (size_t)k; continue; }
    if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
      return fail(E_SYS, std::string("send: ") + strerror(errno));
    if (int rc = wait_fd(fd, POLLOUT, deadline)) return rc;
  }
  return OK;
}

static int recv_all(int fd, void* buf, size_t n, Clock::time_point deadline) {
  char* p = static_cast<char*>(buf);
  while (n) {
    const ssize_t k = ::recv(fd, p, n, MSG_DONTWAIT);
    if (k > 0) { p += k; n -= (size_t)k; continue; }
    if (k == 0) return fail(E_PROTO, "peer closed the connection");
    if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
      return fail(E_SYS, std::string("recv: ") + strerror(errno));
    if (int rc = wait_fd(fd, POLLIN, deadline)) return rc;
  }
  return OK;
}

static int make_listener(const char* host, int port, int* out_port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -fail(E_SYS, std::string("socket: ") + strerror(errno));
  int one = 1;
  (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (!host || !*host || inet_pton(AF_INET, host, &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 256) != 0) {
    const std::string m = std::string("bind/listen ") + (host ? host : "*") + ":" + std::to_string(port) + ": " +
                          strerror(errno);
    ::close(fd);
    return -fail(E_SYS, m);
  }
  socklen_t l = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &l);
  if (out_port) *out_port = ntohs(a.sin_port);
  return fd;
}

static int accept_one(int lfd, Clock::time_point deadline, uint32_t* peer_ip) {
  if (int rc = wait_fd(lfd, POLLIN, deadline)) return -rc;
  sockaddr_in a{};
  socklen_t l = sizeof(a);
  const int fd = accept(lfd, (sockaddr*)&a, &l);
  if (fd < 0) return -fail(E_SYS, std::string("accept: ") + strerror(errno));
  if (peer_ip) *peer_ip = a.sin_addr.s_addr;
  set_nodelay(fd);
  return fd;
}

static int connect_to(uint32_t ip, int port, Clock::time_point deadline) {
  for (;;) {  // the listener may not be up yet: retry until the deadline
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return -fail(E_SYS, std::string("socket: ") + strerror(errno));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = ip;
    if (::connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    ::close(fd);
    if (ms_left(deadline) <= 0) return -fail(E_TIMEOUT, "timed out connecting to port " + std::to_string(port));
    usleep(20000);
  }
}

static int resolve(const char* host, uint32_t* ip) {
  if (inet_pton(AF_INET, host, ip) == 1) return OK;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) return fail(E_ARG, std::string("cannot resolve ") + host);
  *ip = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr.s_addr;
  freeaddrinfo(res);
  return OK;
}

// ------------------------------------------------------------------ backends
struct Backend {
  int world = 1, rank = 0;
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  virtual int all_reduce(const void* s, void* r, size_t n, int dt, int op, void* st) = 0;
  virtual int reduce_scatter(const void* s, void* r, size_t rc, int dt, int op, void* st) = 0;
  virtual int all_gather(const void* s, void* r, size_t sc, int dt, void* st) = 0;
  virtual int broadcast(const void* s, void* r, size_t n, int dt, int root, void* st) = 0;
  virtual int reduce(const void* s, void* r, size_t n, int dt, int op, int root, void* st) = 0;
  virtual int send(const void* s, size_t n, int dt, int peer, void* st) = 0;
  virtual int recv(void* r, size_t n, int dt, int peer, void* st) = 0;
  virtual int group_start() = 0;
  virtual int group_end() = 0;
  // receive ONE message from whichever peer sends first (host backend: the async
  // parameter server's request loop); *src = that peer
  virtual int recv_any(void*, size_t, int, int* src, int64_t) {
    *src = -1;
    return fail(E_ARG, std::string("recv_any: not supported by the ") + name() + " backend");
  }
  virtual int async_error() { return OK; }
  virtual void abort() {}
};

// ---- RCCL, resolved at run time
struct RcclApi {
  void* lib = nullptr;
  std::string path;
  typedef struct { char internal[kIdBytes]; } UniqueId;
  int (*getUniqueId)(UniqueId*) = nullptr;
  int (*commInitRank)(void**, int, UniqueId, int) = nullptr;
  int (*commDestroy)(void*) = nullptr;
  int (*commAbort)(void*) = nullptr;
  int (*commGetAsyncError)(void*, int*) = nullptr;
  const char* (*getErrorString)(int) = nullptr;
  int (*getVersion)(int*) = nullptr;
  int (*allReduce)(const void*, void*, size_t, int, int, void*, void*) = nullptr;
  int (*reduceScatter)(const void*, void*, size_t, int, int, void*, void*) = nullptr;
  int (*allGather)(const void*, void*, size_t, int, void*, void*) = nullptr;
  int (*broadcast)(const void*, void*, size_t, int, int, void*, void*) = nullptr;
  int (*reduce)(const void*, void*, size_t, int, int, int, void*, void*) = nullptr;
  int (*send)(const void*, size_t, int, int, void*, void*) = nullptr;
  int (*recv)(void*, size_t, int, int, void*, void*) = nullptr;
  int (*groupStart)() = nullptr;
  int (*groupEnd)() = nullptr;
};

static int find_loaded_rccl(dl_phdr_info* info, size_t, void* data) {
  const char* n = info->dlpi_name;
  if (n && strstr(n, "librccl")) {
    *static_cast<std::string*>(data) = n;
    return 1;
  }
  return 0;
}

static RcclApi* rccl_api() {
  static std::once_flag once;
  static RcclApi api;
  static std::string err;
  std::call_once(once, [] {
    std::string loaded;
    dl_iterate_phdr(find_loaded_rccl, &loaded);
    std::vector<std::string> cands;
    if (const char* e = getenv("KFC_RCCL_LIB")) cands.push_back(e);
    if (!loaded.empty()) cands.push_back(loaded);
    cands.push_back("/opt/rocm/lib/librccl.so.1");
    cands.push_back("librccl.so.1");
    cands.push_back("librccl.so");
    for (const auto& c : cands) {
      api.lib = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (api.lib) { api.path = c; break; }
    }
    if (!api.lib) { err = "librccl not found"; return; }
    bool ok = true;
    auto sym = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(api.lib, name));
      if (!fp) { ok = false; err += std::string(" missing ") + name; }
    };
    sym(api.getUniqueId, "ncclGetUniqueId");
    sym(api.commInitRank, "ncclCommInitRank");
    sym(api.commDestroy, "ncclCommDestroy");
    sym(api.commAbort, "ncclCommAbort");
    sym(api.commGetAsyncError, "ncclCommGetAsyncError");
    sym(api.getErrorString, "ncclGetErrorString");
    sym(api.getVersion, "ncclGetVersion");
    sym(api.allReduce, "ncclAllReduce");
    sym(api.reduceScatter, "ncclReduceScatter");
    sym(api.allGather, "ncclAllGather");
    sym(api.broadcast, "ncclBroadcast");
    sym(api.reduce, "ncclReduce");
    sym(api.send, "ncclSend");
    sym(api.recv, "ncclRecv");
    sym(api.groupStart, "ncclGroupStart");
    sym(api.groupEnd, "ncclGroupEnd");
    if (!ok) { dlclose(api.lib); api.lib = nullptr; }
  });
  if (!api.lib) {
    fail(E_LIB, "RCCL backend unavailable: " + err);
    return nullptr;
  }
  return &api;
}

struct Rccl : Backend {
  RcclApi* api;
  void* comm = nullptr;
  explicit Rccl(RcclApi* a) : api(a) {}
  ~Rccl() override {
    if (comm) api->commDestroy(comm);
  }
  const char* name() const override { return "rccl"; }
  int chk(int r, const char* what) {
    if (r == 0) return OK;
    return fail(E_RCCL, std::string(what) + ": " + api->getErrorString(r));
  }
  int all_reduce(const void* s, void* r, size_t n, int dt, int op, void* st) override {
    return chk(api->allReduce(s, r, n, dt, op, comm, st), "ncclAllReduce");
  }
  int reduce_scatter(const void* s, void* r, size_t rc, int dt, int op, void* st) override {
    return chk(api->reduceScatter(s, r, rc, dt, op, comm, st), "ncclReduceScatter");
  }
  int all_gather(const void* s, void* r, size_t sc, int dt, void* st) override {
    return chk(api->allGather(s, r, sc, dt, comm, st), "ncclAllGather");
  }
  int broadcast(const void* s, void* r, size_t n, int dt, int root, void* st) override {
    return chk(api->broadcast(s, r, n, dt, root, comm, st), "ncclBroadcast");
  }
  int reduce(const void* s, void* r, size_t n, int dt, int op, int root, void* st) override {
    return chk(api->reduce(s, r, n, dt, op, root, comm, st), "ncclReduce");
  }
  int send(const void* s, size_t n, int dt, int peer, void* st) override {
    return chk(api->send(s, n, dt, peer, comm, st), "ncclSend");
  }
  int recv(void* r, size_t n, int dt, int peer, void* st) override {
    return chk(api->recv(r, n, dt, peer, comm, st), "ncclRecv");
  }
  int group_start() override { return chk(api->groupStart(), "ncclGroupStart"); }
  int group_end() override { return chk(api->groupEnd(), "ncclGroupEnd"); }
  int async_error() override {
    int e = 0;
    if (int r = api->commGetAsyncError(comm, &e)) return chk(r, "ncclCommGetAsyncError");
    return chk(e, "RCCL async error");
  }
  void abort() override {
    if (comm) { api->commAbort(comm); comm = nullptr; }
  }
};

// ---- host backend: the same collectives over host memory + a TCP mesh
static inline float h2f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t f;
  if (e == 0) {
    if (m == 0) f = s;
    else {  // subnormal
      int ee = -1;
      uint32_t mm = m;
      do { mm <<= 1; ee++; } while (!(mm & 0x400));
      f = s | (uint32_t)(127 - 15 - ee) << 23 | (mm & 0x3ff) << 13;
    }
  } else if (e == 31) f = s | 0x7f800000u | m << 13;
  else f = s | (e + 112) << 23 | m << 13;
  float x;
  memcpy(&x, &f, 4);
  return x;
}
static inline uint16_t f2h(float x) {  // round to nearest even
  uint32_t f;
  memcpy(&f, &x, 4);
  const uint32_t s = (f >> 16) & 0x8000;
  const int e = (int)((f >> 23) & 0xff) - 127 + 15;
  uint32_t m = f & 0x7fffff;
  if (((f >> 23) & 0xff) == 0xff) return (uint16_t)(s | 0x7c00 | (m ? 0x200 : 0));
  if (e >= 31) return (uint16_t)(s | 0x7c00);
  if (e <= 0) {
    if (e < -10) return (uint16_t)s;
    m |= 0x800000;
    const int sh = 14 - e;
    uint32_t v = m >> sh;
    const uint32_t rem = m & ((1u << sh) - 1), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (v & 1))) v++;
    return (uint16_t)(s | v);
  }
  uint32_t v = (uint32_t)e << 10 | m >> 13;
  const uint32_t rem = m & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (v & 1))) v++;
  return (uint16_t)(s | v);
}
static inline float b2f(uint16_t b) {
  const uint32_t f = (uint32_t)b << 16;
  float x;
  memcpy(&x, &f, 4);
  return x;
}
static inline uint16_t f2b(float x) {
  uint32_t f;
  memcpy(&f, &x, 4);
  if ((f & 0x7fffffff) > 0x7f800000) return (uint16_t)((f >> 16) | 0x40);
  return (uint16_t)((f + 0x7fff + ((f >> 16) & 1)) >> 16);
}

template <class T>
static T apply_op(T a, T b, int op) {
  switch (op) {
    case PROD: return a * b;
    case MAX: return a > b ? a : b;
    case MIN: return a < b ? a : b;
    default: return a + b;
  }
}

// out[i] = src[0][i] (op) src[1][i] (op) ... in rank order; AVG divides by n at the end
template <class T, class Acc>
static void fold_typed(std::vector<const char*>& src, char* out, size_t n, int op, Acc (*ld)(T), T (*st)(Acc)) {
  const size_t k = src.size();
  for (size_t i = 0; i < n; i++) {
    Acc a = ld(reinterpret_cast<const T*>(src[0])[i]);
    for (size_t j = 1; j < k; j++) a = apply_op<Acc>(a, ld(reinterpret_cast<const T*>(src[j])[i]), op);
    if (op == AVG) a = a / (Acc)k;
    reinterpret_cast<T*>(out)[i] = st(a);
  }
}
template <class T> static T ident_ld(T v) { return v; }
template <class T> static T ident_st(T v) { return v; }

static void fold(std::vector<const char*>& src, char* out, size_t n, int dt, int op) {
  switch (dt) {
    case I8: fold_typed<int8_t, int8_t>(src, out, n, op, ident_ld, ident_st); break;
    case U8: fold_typed<uint8_t, uint8_t>(src, out, n, op, ident_ld, ident_st); break;
    case I32: fold_typed<int32_t, int32_t>(src, out, n, op, ident_ld, ident_st); break;
    case U32: fold_typed<uint32_t, uint32_t>(src, out, n, op, ident_ld, ident_st); break;
    case I64: fold_typed<int64_t, int64_t>(src, out, n, op, ident_ld, ident_st); break;
    case U64: fold_typed<uint64_t, uint64_t>(src, out, n, op, ident_ld, ident_st); break;
    case F32: fold_typed<float, float>(src, out, n, op, ident_ld, ident_st); break;
    case F64: fold_typed<double, double>(src, out, n, op, ident_ld, ident_st); break;
    case F16: fold_typed<uint16_t, float>(src, out, n, op, h2f, f2h); break;
    case BF16: fold_typed<uint16_t, float>(src, out, n, op, b2f, f2b); break;
  }
}

struct Host : Backend {
  std::vector<int> fds;  // fds[peer], -1 for self
  int64_t timeout_ms = 300000;
  struct XOp {
    int peer;
    bool is_send;
    char* buf;
    size_t len;
  };
  std::vector<XOp> queued;  // grouped point-to-point ops
  int depth = 0;
  int rr = 0;                 // recv_any: last peer served
  std::vector<char> closed;   // recv_any: peers whose connection ended
  ~Host() override {
    for (int fd : fds)
      if (fd >= 0) ::close(fd);
  }
  const char* name() const override { return "host"; }

  // Run a batch of point-to-point transfers to completion: per peer, the sends
  // and the receives each proceed in posting order (both sides post matching
  // sequences), every peer's head transfer progresses concurrently.  Each
  // message carries an 8-byte length header that the receiver checks.
  int run(std::vector<XOp>& ops) {
    const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    struct Q {
      std::vector<size_t> s, r;  // op indices
      size_t si = 0, ri = 0, soff = 0, roff = 0;
      uint64_t shdr = 0, rhdr = 0;
    };
    std::vector<Q> q(world);
    for (size_t i = 0; i < ops.size(); i++) {
      const XOp& o = ops[i];
      if (o.peer < 0 || o.peer >= world || o.peer == rank) return fail(E_ARG, "invalid peer " + std::to_string(o.peer));
      (o.is_send ? q[o.peer].s : q[o.peer].r).push_back(i);
    }
    for (;;) {
      std::vector<pollfd> pf;
      std::vector<int> who;
      for (int p = 0; p < world; p++) {
        short ev = 0;
        if (q[p].si < q[p].s.size()) ev |= POLLOUT;
        if (q[p].ri < q[p].r.size()) ev |= POLLIN;
        if (ev) { pf.push_back(pollfd{fds[p], ev, 0}); who.push_back(p); }
      }
      if (pf.empty()) return OK;
      const int64_t left = ms_left(deadline);
      if (left <= 0) return fail(E_TIMEOUT, "host collective timed out (a peer never posted the matching op)");
      const int r = poll(pf.data(), pf.size(), (int)std::min<int64_t>(left, 1000));
      if (r < 0 && errno != EINTR) return fail(E_SYS, std::string("poll: ") + strerror(errno));
      for (size_t k = 0; k < pf.size(); k++) {
        Q& Qp = q[who[k]];
        const int fd = pf[k].fd;
        if (pf[k].revents & (POLLERR | POLLNVAL)) return fail(E_SYS, "peer socket error");
        if ((pf[k].revents & POLLOUT) && Qp.si < Qp.s.size()) {  // send: header then payload
          const XOp& o = ops[Qp.s[Qp.si]];
          Qp.shdr = o.len;
          for (;;) {
            const size_t tot = 8 + o.len;
            if (Qp.soff == tot) { Qp.si++; Qp.soff = 0; break; }
            const char* p = Qp.soff < 8 ? reinterpret_cast<const char*>(&Qp.shdr) + Qp.soff : o.buf + (Qp.soff - 8);
            const size_t n = Qp.soff < 8 ? 8 - Qp.soff : tot - Qp.soff;
            const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (w > 0) { Qp.soff += (size_t)w; continue; }
            if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) break;
            return fail(E_SYS, std::string("send: ") + strerror(errno));
          }
        }
        if ((pf[k].revents & (POLLIN | POLLHUP)) && Qp.ri < Qp.r.size()) {
          const XOp& o = ops[Qp.r[Qp.ri]];
          for (;;) {
            const size_t tot = 8 + o.len;
            if (Qp.roff == tot) { Qp.ri++; Qp.roff = 0; break; }
            char* p = Qp.roff < 8 ? reinterpret_cast<char*>(&Qp.rhdr) + Qp.roff : o.buf + (Qp.roff - 8);
            const size_t n = Qp.roff < 8 ? 8 - Qp.roff : tot - Qp.roff;
            const ssize_t g = ::recv(fd, p, n, MSG_DONTWAIT);
            if (g > 0) {
              Qp.roff += (size_t)g;
              if (Qp.roff == 8 && Qp.rhdr != o.len)
                return fail(E_PROTO, "message size mismatch from rank " + std::to_string(who[k]) + ": got " +
                                         std::to_string(Qp.rhdr) + " B, expected " + std::to_string(o.len) + " B");
              continue;
            }
            if (g == 0) return fail(E_PROTO, "rank " + std::to_string(who[k]) + " closed its connection");
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
            return fail(E_SYS, std::string("recv: ") + strerror(errno));
          }
        }
      }
    }
  }

  int all_reduce(const void* s, void* r, size_t n, int dt, int op, void*) override {
    const size_t b = n * dsize(dt);
    std::vector<std::vector<char>> tmp(world);
    std::vector<XOp> ops;
    for (int p = 0; p < world; p++) {
      tmp[p].resize(b);
      if (p == rank) memcpy(tmp[p].data(), s, b);
      else {
        ops.push_back({p, true, const_cast<char*>(static_cast<const char*>(s)), b});
        ops.push_back({p, false, tmp[p].data(), b});
      }
    }
    if (int rc = run(ops)) return rc;
    std::vector<const char*> src;
    for (auto& t : tmp) src.push_back(t.data());
    fold(src, static_cast<char*>(r), n, dt, op);
    return OK;
  }
  int reduce_scatter(const void* s, void* r, size_t rc, int dt, int op, void*) override {
    const size_t b = rc * dsize(dt);
    const char* sb = static_cast<const char*>(s);
    std::vector<std::vector<char>> tmp(world);
    std::vector<XOp> ops;
    for (int p = 0; p < world; p++) {
      tmp[p].resize(b);
      if (p == rank) memcpy(tmp[p].data(), sb + (size_t)rank * b, b);
      else {
        ops.push_back({p, true, const_cast<char*>(sb + (size_t)p * b), b});
        ops.push_back({p, false, tmp[p].data(), b});
      }
    }
    if (int e = run(ops)) return e;
    std::vector<const char*> src;
    for (auto& t : tmp) src.push_back(t.data());
    fold(src, static_cast<char*>(r), rc, dt, op);
    return OK;
  }
  int all_gather(const void* s, void* r, size_t sc, int dt, void*) override {
    const size_t b = sc * dsize(dt);
    char* rb = static_cast<char*>(r);
    std::vector<char> own(static_cast<const char*>(s), static_cast<const char*>(s) + b);  // s may alias r
    std::vector<XOp> ops;
    for (int p = 0; p < world; p++)
      if (p != rank) {
        ops.push_back({p, true, own.data(), b});
        ops.push_back({p, false, rb + (size_t)p * b, b});
      }
    if (int e = run(ops)) return e;
    memcpy(rb + (size_t)rank * b, own.data(), b);
    return OK;
  }
  int broadcast(const void* s, void* r, size_t n, int dt, int root, void*) override {
    const size_t b = n * dsize(dt);
    std::vector<XOp> ops;
    if (rank == root) {
      if (s != r) memmove(r, s, b);
      for (int p = 0; p < world; p++)
        if (p != rank) ops.push_back({p, true, static_cast<char*>(r), b});
    } else {
      ops.push_back({root, false, static_cast<char*>(r), b});
    }
    return run(ops);
  }
  int reduce(const void* s, void* r, size_t n, int dt, int op, int root, void*) override {
    const size_t b = n * dsize(dt);
    std::vector<XOp> ops;
    if (rank != root) {
      ops.push_back({root, true, const_cast<char*>(static_cast<const char*>(s)), b});
      return run(ops);
    }
    std::vector<std::vector<char>> tmp(world);
    for (int p = 0; p < world; p++) {
      tmp[p].resize(b);
      if (p == rank) memcpy(tmp[p].data(), s, b);
      else ops.push_back({p, false, tmp[p].data(), b});
    }
    if (int e = run(ops)) return e;
    std::vector<const char*> src;
    for (auto& t : tmp) src.push_back(t.data());
    fold(src, static_cast<char*>(r), n, dt, op);
    return OK;
  }
  int send(const void* s, size_t n, int dt, int peer, void*) override {
    XOp o{peer, true, const_cast<char*>(static_cast<const char*>(s)), n * dsize(dt)};
    if (depth > 0) { queued.push_back(o); return OK; }
    std::vector<XOp> ops{o};
    return run(ops);
  }
  int recv(void* r, size_t n, int dt, int peer, void*) override {
    XOp o{peer, false, static_cast<char*>(r), n * dsize(dt)};
    if (depth > 0) { queued.push_back(o); return OK; }
    std::vector<XOp> ops{o};
    return run(ops);
  }
  // Wait until a peer's socket is readable and receive its next message with the
  // normal directed path.  Peers are scanned round-robin from the last one served
  // (no starvation); a peer whose connection closed with nothing left to read
  // (a finished worker) is skipped from then on.
  int recv_any(void* r, size_t n, int dt, int* src, int64_t tmo_ms) override {
    *src = -1;
    if (depth > 0) return fail(E_STATE, "recv_any inside a group");
    const auto deadline = Clock::now() + std::chrono::milliseconds(tmo_ms > 0 ? tmo_ms : timeout_ms);
    if (closed.size() != (size_t)world) closed.assign(world, 0);
    for (;;) {
      std::vector<pollfd> pf;
      std::vector<int> who;
      for (int k = 1; k <= world; k++) {
        const int p = (rr + k) % world;
        if (p == rank || closed[p]) continue;
        pf.push_back(pollfd{fds[p], POLLIN, 0});
        who.push_back(p);
      }
      if (pf.empty()) return fail(E_PROTO, "recv_any: every peer closed its connection");
      const int64_t left = ms_left(deadline);
      if (left <= 0) return fail(E_TIMEOUT, "recv_any timed out (no peer sent a message)");
      const int rc = poll(pf.data(), pf.size(), (int)std::min<int64_t>(left, 1000));
      if (rc < 0 && errno != EINTR) return fail(E_SYS, std::string("poll: ") + strerror(errno));
      for (size_t k = 0; k < pf.size(); k++) {
        if (!(pf[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        char b;
        const ssize_t g = ::recv(pf[k].fd, &b, 1, MSG_PEEK | MSG_DONTWAIT);
        if (g == 0) { closed[who[k]] = 1; continue; }  // orderly close, nothing pending
        if (g < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) continue;
        if (g < 0) return fail(E_SYS, std::string("recv: ") + strerror(errno));
        rr = who[k];
        *src = who[k];
        XOp o{who[k], false, static_cast<char*>(r), n * dsize(dt)};
        std::vector<XOp> ops{o};
        return run(ops);
      }
    }
  }
  int group_start() override {
    depth++;
    return OK;
  }
  int group_end() override {
    if (depth <= 0) return fail(E_STATE, "group_end without group_start");
    if (--depth > 0) return OK;
    std::vector<XOp> ops;
    ops.swap(queued);
    return run(ops);
  }
};

// ------------------------------------------------------------------ communicator
struct Comm {
  std::unique_ptr<Backend> be;
  std::mutex mu;  // backward hooks may issue from autograd's device thread
  int in_group = 0;
};

struct Hello {
  uint32_t magic;
  int32_t rank, world, mesh_port;
};

}  // namespace kfc

using namespace kfc;

KFC_API const char* kfc_last_error() { return g_err.c_str(); }

KFC_API int kfc_dtype_size(int dt) { return (int)dsize(dt); }

// Rank 0's bootstrap listener: host "" = every interface, port 0 = ephemeral.
// Returns the listening fd (>= 0) and the bound port, or -error.
KFC_API int kfc_listen(const char* host, int port, int* out_port) { return make_listener(host, port, out_port); }

KFC_API void kfc_close_fd(int fd) {
  if (fd >= 0) ::close(fd);
}

// Path of the librccl the "rccl" backend resolved ("" if none); loads it on first call.
KFC_API const char* kfc_rccl_path() {
  RcclApi* a = rccl_api();
  return a ? a->path.c_str() : "";
}

KFC_API int kfc_rccl_version() {
  RcclApi* a = rccl_api();
  int v = 0;
  if (a) a->getVersion(&v);
  return v;
}

// Create a communicator.  backend: "rccl" | "host".  Rank 0 passes its listener
// (kfc_listen; closed here) and ignores root_host / root_port; other ranks connect
// to root_host:root_port.  Returns the handle, or nullptr (kfc_last_error()).
KFC_API void* kfc_comm_init(const char* backend, int world, int rank, const char* root_host, int root_port,
                            int listen_fd, int timeout_ms) {
  if (world < 1 || rank < 0 || rank >= world) {
    fail(E_ARG, "bad world / rank");
    return nullptr;
  }
  const bool host = backend && strcmp(backend, "host") == 0;
  if (!host && !(backend && strcmp(backend, "rccl") == 0)) {
    fail(E_ARG, std::string("unknown backend ") + (backend ? backend : "(null)"));
    return nullptr;
  }
  RcclApi* api = nullptr;
  if (!host && !(api = rccl_api())) return nullptr;
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 300000);
  RcclApi::UniqueId id{};
  // host backend: every rank opens a mesh listener and reports its port
  int mesh_fd = -1, mesh_port = 0;
  if (host && world > 1) {
    mesh_fd = make_listener(nullptr, 0, &mesh_port);
    if (mesh_fd < 0) return nullptr;
  }
  std::vector<uint32_t> ips(world, 0);
  std::vector<int32_t> ports(world, 0);
  auto cleanup = [&]() {
    if (mesh_fd >= 0) ::close(mesh_fd);
  };
  if (rank == 0) {
    if (!host) {
      if (int r = api->getUniqueId(&id)) {
        fail(E_RCCL, std::string("ncclGetUniqueId: ") + api->getErrorString(r));
        if (listen_fd >= 0) ::close(listen_fd);
        cleanup();
        return nullptr;
      }
    }
    ports[0] = mesh_port;
    ips[0] = htonl(INADDR_LOOPBACK);
    std::vector<int> peers(world, -1);
    int err = OK;
    for (int k = 1; k < world && !err; k++) {
      uint32_t ip = 0;
      const int fd = accept_one(listen_fd, deadline, &ip);
      if (fd < 0) { err = -fd; break; }
      Hello h{};
      if ((err = recv_all(fd, &h, sizeof(h), deadline))) { ::close(fd); break; }
      if (h.magic != kMagic || h.world != world || h.rank <= 0 || h.rank >= world || peers[h.rank] >= 0) {
        ::close(fd);
        err = fail(E_PROTO, "bootstrap: bad hello (rank " + std::to_string(h.rank) + ", world " +
                                std::to_string(h.world) + ")");
        break;
      }
      peers[h.rank] = fd;
      ips[h.rank] = ip;
      ports[h.rank] = h.mesh_port;
    }
    if (listen_fd >= 0) ::close(listen_fd);
    for (int p = 1; p < world && !err; p++) {
      const uint32_t m = kMagic;
      if ((err = send_all(peers[p], &m, 4, deadline))) break;
      if ((err = send_all(peers[p], &id, sizeof(id), deadline))) break;
      if ((err = send_all(peers[p], ips.data(), 4 * world, deadline))) break;
      err = send_all(peers[p], ports.data(), 4 * world, deadline);
    }
    for (int fd : peers)
      if (fd >= 0) ::close(fd);
    if (err) { cleanup(); return nullptr; }
  } else {
    uint32_t rip = 0;
    if (resolve(root_host && *root_host ? root_host : "127.0.0.1", &rip)) { cleanup(); return nullptr; }
    const int fd = connect_to(rip, root_port, deadline);
    if (fd < 0) { cleanup(); return nullptr; }
    Hello h{kMagic, rank, world, mesh_port};
    uint32_t m = 0;
    int err = send_all(fd, &h, sizeof(h), deadline);
    if (!err) err = recv_all(fd, &m, 4, deadline);
    if (!err && m != kMagic) err = fail(E_PROTO, "bootstrap: bad reply");
    if (!err) err = recv_all(fd, &id, sizeof(id), deadline);
    if (!err) err = recv_all(fd, ips.data(), 4 * world, deadline);
    if (!err) err = recv_all(fd, ports.data(), 4 * world, deadline);
    ::close(fd);
    if (err) { cleanup(); return nullptr; }
    ips[0] = rip;  // the root's address as this rank reached it
  }
  auto c = std::make_unique<Comm>();
  if (host) {
    auto h = std::make_unique<Host>();
    h->world = world;
    h->rank = rank;
    h->timeout_ms = timeout_ms > 0 ? timeout_ms : 300000;
    h->fds.assign(world, -1);
    int err = OK;
    // mesh: connect to every lower rank (their listeners exist: the table came after
    // they opened them), then accept every higher rank; each connector sends its rank
    for (int p = 0; p < rank && !err; p++) {
      const int fd = connect_to(ips[p], ports[p], deadline);
      if (fd < 0) { err = -fd; break; }
      const int32_t me = rank;
      if ((err = send_all(fd, &me, 4, deadline))) { ::close(fd); break; }
      h->fds[p] = fd;
    }
    for (int k = rank + 1; k < world && !err; k++) {
      const int fd = accept_one(mesh_fd, deadline, nullptr);
      if (fd < 0) { err = -fd; break; }
      int32_t who = -1;
      if ((err = recv_all(fd, &who, 4, deadline))) { ::close(fd); break; }
      if (who <= rank || who >= world || h->fds[who] >= 0) {
        ::close(fd);
        err = fail(E_PROTO, "mesh: unexpected peer " + std::to_string(who));
        break;
      }
      h->fds[who] = fd;
    }
    cleanup();
    if (err) return nullptr;
    for (int fd : h->fds)
      if (fd >= 0) fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    c->be = std::move(h);
  } else {
    auto r = std::make_unique<Rccl>(api);
    r->world = world;
    r->rank = rank;
    if (int e = api->commInitRank(&r->comm, world, id, rank)) {
      fail(E_RCCL, std::string("ncclCommInitRank: ") + api->getErrorString(e));
      r->comm = nullptr;
      return nullptr;
    }
    c->be = std::move(r);
  }
  return c.release();
}

#define KFC_COMM(h)                                               \
  Comm* c = static_cast<Comm*>(h);                                \
  if (!c || !c->be) return fail(E_STATE, "null communicator"); \
  std::lock_guard<std::mutex> lk(c->mu)

static int chk_args(int dt, int op) {
  if (dsize(dt) == 0) return fail(E_ARG, "bad dtype " + std::to_string(dt));
  if (op < 0 || op >= NOPS) return fail(E_ARG, "bad reduction op " + std::to_string(op));
  return OK;
}

KFC_API const char* kfc_backend(void* h) {
  Comm* c = static_cast<Comm*>(h);
  return c && c->be ? c->be->name() : "";
}

KFC_API int kfc_all_reduce(void* h, const void* s, void* r, size_t n, int dt, int op, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, op)) return e;
  return c->be->all_reduce(s, r, n, dt, op, stream);
}

KFC_API int kfc_reduce_scatter(void* h, const void* s, void* r, size_t recvcount, int dt, int op, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, op)) return e;
  return c->be->reduce_scatter(s, r, recvcount, dt, op, stream);
}

KFC_API int kfc_all_gather(void* h, const void* s, void* r, size_t sendcount, int dt, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  return c->be->all_gather(s, r, sendcount, dt, stream);
}

KFC_API int kfc_broadcast(void* h, const void* s, void* r, size_t n, int dt, int root, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  if (root < 0 || root >= c->be->world) return fail(E_ARG, "bad root");
  return c->be->broadcast(s, r, n, dt, root, stream);
}

KFC_API int kfc_reduce(void* h, const void* s, void* r, size_t n, int dt, int op, int root, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, op)) return e;
  if (root < 0 || root >= c->be->world) return fail(E_ARG, "bad root");
  return c->be->reduce(s, r, n, dt, op, root, stream);
}

KFC_API int kfc_send(void* h, const void* s, size_t n, int dt, int peer, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  return c->be->send(s, n, dt, peer, stream);
}

KFC_API int kfc_recv(void* h, void* r, size_t n, int dt, int peer, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  return c->be->recv(r, n, dt, peer, stream);
}

// one message from whichever peer sends first (host backend); *src = its rank;
// timeout_ms <= 0: the communicator's timeout
KFC_API int kfc_recv_any(void* h, void* r, size_t n, int dt, int* src, int timeout_ms) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  return c->be->recv_any(r, n, dt, src, timeout_ms);
}

// All-to-all with per-peer element counts / offsets (the embedding exchange): one
// grouped batch of send / recv, the local block copied by the caller.
KFC_API int kfc_all_to_all_v(void* h, const void* s, const int64_t* scount, const int64_t* soff, void* r,
                             const int64_t* rcount, const int64_t* roff, int dt, void* stream) {
  KFC_COMM(h);
  if (int e = chk_args(dt, SUM)) return e;
  const size_t es = dsize(dt);
  Backend* b = c->be.get();
  if (int e = b->group_start()) return e;
  int err = OK;
  for (int p = 0; p < b->world && !err; p++) {
    if (p == b->rank) continue;
    if (scount[p] > 0) err = b->send(static_cast<const char*>(s) + soff[p] * es, (size_t)scount[p], dt, p, stream);
    if (!err && rcount[p] > 0) err = b->recv(static_cast<char*>(r) + roff[p] * es, (size_t)rcount[p], dt, p, stream);
  }
  const int e2 = b->group_end();
  return err ? err : e2;
}

KFC_API int kfc_group_start(void* h) {
  KFC_COMM(h);
  c->in_group++;
  return c->be->group_start();
}

KFC_API int kfc_group_end(void* h) {
  KFC_COMM(h);
  if (c->in_group <= 0) return fail(E_STATE, "group_end without group_start");
  c->in_group--;
  return c->be->group_end();
}

KFC_API int kfc_async_error(void* h) {
  KFC_COMM(h);
  return c->be->async_error();
}

KFC_API void kfc_comm_abort(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c) return;
  if (c->be) c->be->abort();
  delete c;
}

KFC_API void kfc_comm_destroy(void* h) { delete static_cast<Comm*>(h); }
