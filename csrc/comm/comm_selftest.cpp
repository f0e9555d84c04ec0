// Native self-test of the first-party collective layer (csrc/comm/comm.cpp), built
// WITHOUT Python under ASan+UBSan and under TSan (kubeflow_controller_amd/
// _build.py: build_sanitized("asan"|"tsan", target="comm")).
//
// W ranks run as threads of this one process on the host backend (the same code
// paths the RCCL backend shares: bootstrap, the per-communicator mutex, grouping,
// argument checks; the host backend's own socket mesh, partial-I/O offsets and
// rank-order folds).  Every collective is checked element by element against
// values computed here from rank-distinct inputs, so an offset or ordering error
// shows up as a wrong element, not only as a crash.  Each rank also hands its
// communicator to a second thread half way through (what autograd's device thread
// does with the bucket collectives), so TSan sees the mutex-ordered hand-off.
//
// Exit status: 0 = every check passed; 1 = a check failed; a sanitizer report
// exits with the code _build.run_sanitized sets (23 ASan/UBSan, 25 TSan).
#include "comm.cpp"

#include <atomic>
#include <condition_variable>
#include <thread>

namespace {

constexpr int W = 3;
std::atomic<int> g_fail{0}, g_pass{0};
std::mutex g_port_mu;
std::condition_variable g_port_cv;
int g_port = 0;  // rank 0's bootstrap port, published to the other rank threads

void check(bool ok, int rank, const char* what, long i = -1) {
  if (ok) {
    g_pass++;
    return;
  }
  g_fail++;
  std::fprintf(stderr, "FAIL rank %d: %s (element %ld) %s\n", rank, what, i, kfc_last_error());
}

// value of element i contributed by rank r (distinct per rank and element, exact in fp32)
float val(int r, size_t i) { return (float)(r * 1000 + (int)(i % 997)) + 0.25f * (float)r; }

void* make(int rank, int timeout_ms) {
  if (rank == 0) {
    int port = 0;
    const int fd = kfc_listen("127.0.0.1", 0, &port);
    if (fd < 0) return nullptr;
    {
      std::lock_guard<std::mutex> lk(g_port_mu);
      g_port = port;
    }
    g_port_cv.notify_all();
    return kfc_comm_init("host", W, 0, nullptr, 0, fd, timeout_ms);
  }
  int port;
  {
    std::unique_lock<std::mutex> lk(g_port_mu);
    g_port_cv.wait(lk, [] { return g_port != 0; });
    port = g_port;
  }
  return kfc_comm_init("host", W, rank, "127.0.0.1", port, -1, timeout_ms);
}

void collectives(void* c, int rank, size_t n) {
  // all-reduce (sum, max) fp32, out of place and in place
  std::vector<float> s(n), r(n);
  for (size_t i = 0; i < n; i++) s[i] = val(rank, i);
  check(kfc_all_reduce(c, s.data(), r.data(), n, F32, SUM, nullptr) == 0, rank, "all_reduce rc");
  for (size_t i = 0; i < n; i++) {
    float e = 0.f;
    for (int p = 0; p < W; p++) e += val(p, i);
    if (r[i] != e) { check(false, rank, "all_reduce sum", (long)i); break; }
  }
  check(kfc_all_reduce(c, s.data(), s.data(), n, F32, MAX, nullptr) == 0, rank, "all_reduce max rc");
  for (size_t i = 0; i < n; i++)
    if (s[i] != val(W - 1, i)) { check(false, rank, "all_reduce max in place", (long)i); break; }
  // reduce-scatter: rank p receives block p of the sum
  const size_t blk = n / W;
  std::vector<float> rs(blk);
  for (size_t i = 0; i < n; i++) s[i] = val(rank, i);
  check(kfc_reduce_scatter(c, s.data(), rs.data(), blk, F32, SUM, nullptr) == 0, rank, "reduce_scatter rc");
  for (size_t i = 0; i < blk; i++) {
    float e = 0.f;
    for (int p = 0; p < W; p++) e += val(p, rank * blk + i);
    if (rs[i] != e) { check(false, rank, "reduce_scatter", (long)i); break; }
  }
  // all-gather of rank-distinct blocks, the own block aliasing the output
  std::vector<float> ag(blk * W, -1.f);
  for (size_t i = 0; i < blk; i++) ag[rank * blk + i] = val(rank, i);
  check(kfc_all_gather(c, ag.data() + rank * blk, ag.data(), blk, F32, nullptr) == 0, rank, "all_gather rc");
  for (int p = 0; p < W; p++)
    for (size_t i = 0; i < blk; i++)
      if (ag[p * blk + i] != val(p, i)) { check(false, rank, "all_gather", (long)(p * blk + i)); p = W; break; }
  // broadcast from the last rank, reduce (int64) to rank 1
  std::vector<float> b(n);
  for (size_t i = 0; i < n; i++) b[i] = val(rank, i);
  check(kfc_broadcast(c, b.data(), b.data(), n, F32, W - 1, nullptr) == 0, rank, "broadcast rc");
  for (size_t i = 0; i < n; i++)
    if (b[i] != val(W - 1, i)) { check(false, rank, "broadcast", (long)i); break; }
  std::vector<int64_t> li(n), lo(n, 0);
  for (size_t i = 0; i < n; i++) li[i] = (int64_t)rank * 1000003 + (int64_t)i;
  check(kfc_reduce(c, li.data(), lo.data(), n, I64, SUM, 1, nullptr) == 0, rank, "reduce rc");
  if (rank == 1)
    for (size_t i = 0; i < n; i++) {
      int64_t e = 0;
      for (int p = 0; p < W; p++) e += (int64_t)p * 1000003 + (int64_t)i;
      if (lo[i] != e) { check(false, rank, "reduce", (long)i); break; }
    }
  // bf16 all-reduce in rank order (identical bits everywhere)
  std::vector<uint16_t> hb(n), hr(n);
  for (size_t i = 0; i < n; i++) hb[i] = f2b(val(rank, i) * 0.001f);
  check(kfc_all_reduce(c, hb.data(), hr.data(), n, BF16, SUM, nullptr) == 0, rank, "bf16 all_reduce rc");
  for (size_t i = 0; i < n; i++) {
    float a = b2f(f2b(val(0, i) * 0.001f));
    for (int p = 1; p < W; p++) a = a + b2f(f2b(val(p, i) * 0.001f));
    if (hr[i] != f2b(a)) { check(false, rank, "bf16 all_reduce", (long)i); break; }
  }
}

void point_to_point(void* c, int rank, size_t n) {
  // uneven all-to-all-v: rank r sends (r + p + 1) * 7 elements to p
  std::vector<int64_t> sc(W), so(W), rc(W), ro(W);
  int64_t st = 0, rt = 0;
  for (int p = 0; p < W; p++) {
    sc[p] = (rank + p + 1) * 7;
    rc[p] = (p + rank + 1) * 7;
    so[p] = st;
    ro[p] = rt;
    st += sc[p];
    rt += rc[p];
  }
  std::vector<float> s(st), r(rt, -1.f);
  for (int p = 0; p < W; p++)
    for (int64_t i = 0; i < sc[p]; i++) s[so[p] + i] = (float)(rank * 100000 + p * 1000 + i);
  check(kfc_all_to_all_v(c, s.data(), sc.data(), so.data(), r.data(), rc.data(), ro.data(), F32, nullptr) == 0, rank,
        "all_to_all_v rc");
  for (int p = 0; p < W; p++) {
    if (p == rank) continue;  // the caller copies its own block
    for (int64_t i = 0; i < rc[p]; i++)
      if (r[ro[p] + i] != (float)(p * 100000 + rank * 1000 + i)) { check(false, rank, "all_to_all_v", (long)i); break; }
  }
  // grouped ring send / recv of a large message (forces partial socket I/O)
  const int nxt = (rank + 1) % W, prv = (rank + W - 1) % W;
  const size_t big = n * 64;
  std::vector<float> out(big), in(big, 0.f);
  for (size_t i = 0; i < big; i++) out[i] = val(rank, i);
  check(kfc_group_start(c) == 0, rank, "group_start");
  check(kfc_send(c, out.data(), big, F32, nxt, nullptr) == 0, rank, "send");
  check(kfc_recv(c, in.data(), big, F32, prv, nullptr) == 0, rank, "recv");
  check(kfc_group_end(c) == 0, rank, "group_end");
  for (size_t i = 0; i < big; i++)
    if (in[i] != val(prv, i)) { check(false, rank, "ring send/recv", (long)i); break; }
  // any-source receive: every other rank sends one message to rank 0, in any order
  if (rank == 0) {
    std::vector<int> seen(W, 0);
    for (int k = 1; k < W; k++) {
      int32_t msg = -1;
      int src = -1;
      check(kfc_recv_any(c, &msg, 1, I32, &src, 0) == 0, rank, "recv_any rc");
      check(src > 0 && src < W && msg == src * 11 && !seen[src], rank, "recv_any source / payload");
      if (src > 0 && src < W) seen[src] = 1;
    }
  } else {
    const int32_t msg = rank * 11;
    check(kfc_send(c, &msg, 1, I32, 0, nullptr) == 0, rank, "send to recv_any");
  }
  // a size mismatch fails on both ends instead of corrupting the receiver
  if (rank < 2) {
    std::vector<float> x(16, 1.f);
    const int e = rank == 0 ? kfc_send(c, x.data(), 16, F32, 1, nullptr) : kfc_recv(c, x.data(), 8, F32, 0, nullptr);
    check(rank == 0 || e == E_PROTO, rank, "size mismatch detected");
  }
}

void rank_main(int rank) {
  void* c = make(rank, 20000);
  check(c != nullptr, rank, "comm_init");
  if (!c) return;
  check(std::string(kfc_backend(c)) == "host", rank, "backend name");
  // argument checks
  float x = 0.f;
  check(kfc_all_reduce(c, &x, &x, 1, 77, SUM, nullptr) == E_ARG, rank, "bad dtype rejected");
  check(kfc_broadcast(c, &x, &x, 1, F32, W, nullptr) == E_ARG, rank, "bad root rejected");
  check(kfc_group_end(c) == E_STATE, rank, "group_end without start rejected");
  collectives(c, rank, 3 * 4099);  // odd block sizes
  // hand the communicator to another thread for the next batch (autograd's device thread)
  std::thread t([&] { collectives(c, rank, 3 * 17); });
  t.join();
  point_to_point(c, rank, 4099);
  kfc_comm_destroy(c);
}

}  // namespace

int main() {
  std::vector<std::thread> th;
  for (int r = 0; r < W; r++) th.emplace_back(rank_main, r);
  for (auto& t : th) t.join();
  // bootstrap failure path: a rank that never finds its root times out cleanly
  void* lone = kfc_comm_init("host", 2, 1, "127.0.0.1", 1, -1, 300);
  check(lone == nullptr, 1, "timeout without a root");
  std::printf("comm selftest: %d passed, %d failed\n", g_pass.load(), g_fail.load());
  return g_fail.load() ? 1 : 0;
}
