// Native self-test of the control-plane runtime core (runtime_core.h), built
// without Python under the sanitizers ("use ASAN/UBSAN builds of
// the C++ host code"; the reference's Makefile:22-29 has no `-race` either):
//
//   clang++ -std=c++17 -O1 -g -fsanitize=address,undefined ...  (memory / UB)
//   clang++ -std=c++17 -O1 -g -fsanitize=thread ...             (data races)
//
// (ROCm's clang++: gcc-11's TSan misses pthread_cond_clockwait and reports a
// false double lock on every timed condition-variable wait.)
//
// Driven by `python -m kubeflow_controller_amd._build --sanitize` and
// tests/test_sanitizers_cpu.py.  Host code only: nothing here touches a GPU.
//
// What it exercises, concurrently where the controller is concurrent:
//   * rate limiters: exponential backoff sequence / cap / forget
//     (default_rate_limiters.go:54-105), token bucket burst, MaxOf;
//   * WorkQueue: N producers x M workers over a small key space — an item is
//     never held by two workers at once, every add is eventually processed,
//     shutdown wakes blocked getters (queue.go:33-158);
//   * delayed adds: earliest-deadline wins, fake-clock drain (delaying_queue.go);
//   * queue construction/destruction churn (waiter thread lifetime);
//   * ControllerExpectations under concurrent raise/lower (controller_utils.go:136-288);
//   * process launcher: exit codes, signals, process-group kill, log capture.
#include "runtime_core.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

static int g_checks = 0, g_fail = 0;

#define CHECK(cond)                                                         \
  do {                                                                      \
    ++g_checks;                                                             \
    if (!(cond)) {                                                          \
      ++g_fail;                                                             \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                       \
  } while (0)

static bool near(double a, double b) { return std::fabs(a - b) <= 1e-9 * std::max(1.0, std::fabs(b)); }

static void test_rate_limiters() {
  ExpFailureLimiter e(0.005, 1.0);
  CHECK(near(e.when("a"), 0.005));
  CHECK(near(e.when("a"), 0.010));
  CHECK(near(e.when("a"), 0.020));
  CHECK(e.num_requeues("a") == 3);
  CHECK(near(e.when("b"), 0.005));
  for (int i = 0; i < 2000; ++i) e.when("a");  // 2^2000 overflows to inf -> capped
  CHECK(near(e.when("a"), 1.0));
  e.forget("a");
  CHECK(e.num_requeues("a") == 0);
  CHECK(near(e.when("a"), 0.005));

  g_fake_now = 100.0;
  g_fake = true;
  BucketLimiter b(10.0, 3);
  CHECK(b.when("x") == 0.0);
  CHECK(b.when("x") == 0.0);
  CHECK(b.when("x") == 0.0);
  CHECK(near(b.when("x"), 0.1));  // burst spent: one token every 1/qps
  g_fake_now = g_fake_now.load() + 10.0;
  CHECK(b.when("x") == 0.0);  // refilled (capped at burst)
  g_fake = false;

  auto d = default_controller_rate_limiter();
  CHECK(near(d->when("k"), 0.005));
  CHECK(d->num_requeues("k") == 1);
  d->forget("k");
  CHECK(d->num_requeues("k") == 0);

  // concurrent hammering of one limiter (mutex-protected failure map)
  ExpFailureLimiter c(0.001, 10.0);
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&c, t] {
      for (int i = 0; i < 2000; ++i) {
        std::string k = "job-" + std::to_string((i + t) % 16);
        c.when(k);
        if (i % 7 == 0) c.forget(k);
        c.num_requeues(k);
      }
    });
  for (auto &th : ts) th.join();
  CHECK(true);
}

static void test_queue_dedup_and_exclusive_processing() {
  constexpr int kKeys = 32, kProducers = 6, kWorkers = 6, kAddsPerProducer = 3000;
  WorkQueue q("stress", default_controller_rate_limiter());
  std::vector<std::atomic<int>> holders(kKeys);
  std::vector<std::atomic<long>> last_add(kKeys), last_done(kKeys);
  for (int i = 0; i < kKeys; ++i) holders[i] = 0, last_add[i] = 0, last_done[i] = 0;
  std::atomic<long> seq{0}, processed{0};
  std::atomic<int> overlap{0};

  std::vector<std::thread> workers;
  for (int w = 0; w < kWorkers; ++w)
    workers.emplace_back([&] {
      for (;;) {
        auto r = q.get(-1.0);
        if (r.second) return;  // shutdown
        int k = std::atoi(r.first->c_str() + 4);
        if (holders[k].fetch_add(1) != 0) overlap.fetch_add(1);
        long s = seq.load();  // everything added before this point is covered
        std::this_thread::yield();
        holders[k].fetch_sub(1);
        long prev = last_done[k].load();
        while (prev < s && !last_done[k].compare_exchange_weak(prev, s)) {
        }
        processed.fetch_add(1);
        q.done(*r.first);
      }
    });
  std::vector<std::thread> producers;
  for (int p = 0; p < kProducers; ++p)
    producers.emplace_back([&, p] {
      for (int i = 0; i < kAddsPerProducer; ++i) {
        int k = (i * 7 + p) % kKeys;
        long s = seq.fetch_add(1) + 1;
        long prev = last_add[k].load();
        while (prev < s && !last_add[k].compare_exchange_weak(prev, s)) {
        }
        q.add("key-" + std::to_string(k));
        if (i % 97 == 0) std::this_thread::yield();
      }
    });
  for (auto &t : producers) t.join();
  // drain: every key's last add must be followed by a processing that started after it
  for (int spin = 0; spin < 2000; ++spin) {
    bool all = q.len() == 0;
    for (int k = 0; all && k < kKeys; ++k) all = last_done[k].load() >= last_add[k].load();
    if (all) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  for (int k = 0; k < kKeys; ++k) CHECK(last_done[k].load() >= last_add[k].load());
  CHECK(overlap.load() == 0);
  CHECK(processed.load() > 0);
  CHECK(processed.load() <= (long)kProducers * kAddsPerProducer);  // dedup never inflates
  q.shut_down();
  for (auto &t : workers) t.join();  // shutdown wakes every blocked get
  CHECK(q.shutting_down());
  q.add("late");
  CHECK(q.len() == 0);  // adds after shutdown are dropped
}

static void test_dirty_while_processing() {
  WorkQueue q("dirty", default_controller_rate_limiter());
  q.add("a");
  auto r = q.get(0.5);
  CHECK(r.first && *r.first == "a");
  q.add("a");  // re-add while processing: deferred to done()
  q.add("a");
  CHECK(q.len() == 0);
  q.done("a");
  CHECK(q.len() == 1);
  r = q.get(0.5);
  CHECK(r.first && *r.first == "a");
  q.done("a");
  CHECK(q.len() == 0);
  r = q.get(0.01);  // timeout: no item, not shutdown
  CHECK(!r.first && !r.second);
}

static void test_delayed_adds() {
  g_fake_now = 1000.0;
  g_fake = true;
  {
    WorkQueue q("delay", default_controller_rate_limiter());
    q.add_after("x", 5.0);
    q.add_after("x", 2.0);  // earlier deadline wins
    q.add_after("x", 9.0);  // later one ignored
    q.add_after("y", 3.0);
    CHECK(q.num_waiting() == 2);
    q.poll_delayed();
    CHECK(q.len() == 0);
    g_fake_now = 1002.5;
    q.poll_delayed();
    CHECK(q.len() == 1);
    CHECK(q.num_waiting() == 1);
    g_fake_now = 1010.0;
    q.poll_delayed();
    CHECK(q.len() == 2);
    CHECK(q.num_waiting() == 0);
    q.add_rate_limited("z");  // 5 ms backoff on the fake clock
    CHECK(q.num_requeues("z") == 1);
    g_fake_now = 1010.01;
    q.poll_delayed();
    CHECK(q.len() == 3);
    q.forget("z");
    CHECK(q.num_requeues("z") == 0);
  }
  g_fake = false;
  // real clock: the waiter thread moves due items without a poll
  WorkQueue q("delay-real", default_controller_rate_limiter());
  for (int i = 0; i < 64; ++i) q.add_after("r" + std::to_string(i), 0.001 * (i % 8));
  for (int spin = 0; spin < 500 && q.len() < 64; ++spin) std::this_thread::sleep_for(std::chrono::milliseconds(2));
  CHECK(q.len() == 64);
}

static void test_queue_lifetime_churn() {
  for (int i = 0; i < 200; ++i) {
    WorkQueue q("churn-" + std::to_string(i), default_controller_rate_limiter());
    q.add_after("a", 0.5);  // pending delayed item at destruction
    q.add("b");
    if (i % 2) q.shut_down();
  }
  // a getter blocked when another thread shuts the queue down
  WorkQueue q("blocked", default_controller_rate_limiter());
  std::atomic<bool> woke{false};
  std::thread t([&] {
    auto r = q.get(-1.0);
    woke = r.second && !r.first;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  q.shut_down();
  t.join();
  CHECK(woke.load());
}

static void test_expectations() {
  Expectations e(300.0);
  CHECK(e.satisfied("ns/job"));  // absent
  e.set("ns/job", 4, 0);
  CHECK(!e.satisfied("ns/job"));
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; ++t) ts.emplace_back([&] { e.lower("ns/job", 1, 0); });
  for (auto &th : ts) th.join();
  CHECK(e.satisfied("ns/job"));
  // concurrent raise/lower balance out
  e.set("ns/b", 0, 0);
  ts.clear();
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 1000; ++i) {
        e.raise("ns/b", 1, 1);
        e.lower("ns/b", 1, 1);
        e.satisfied("ns/b");
        e.get("ns/b");
      }
    });
  for (auto &th : ts) th.join();
  auto g = e.get("ns/b");
  CHECK(g && std::get<0>(*g) <= 0 && std::get<1>(*g) <= 0);
  // TTL expiry on the fake clock
  g_fake_now = 50.0;
  g_fake = true;
  Expectations s(300.0);
  s.set("k", 2, 0);
  CHECK(!s.satisfied("k"));
  g_fake_now = 351.0;
  CHECK(s.satisfied("k"));
  g_fake = false;
  s.erase("k");
  CHECK(!s.get("k"));
}

static std::pair<int, int> wait_exit(int pid) {
  for (int i = 0; i < 1000; ++i) {
    auto r = poll_process(pid);
    if (r) return *r;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return {-2, 0};
}

static void test_process_launcher() {
  std::map<std::string, std::string> env{{"PATH", "/usr/bin:/bin"}, {"KFA_SELFTEST", "hello"}};
  int pid = spawn_process({"/bin/sh", "-c", "exit 3"}, env, "", "");
  CHECK(pid > 0);
  auto r = wait_exit(pid);
  CHECK(r.first == 3 && r.second == 0);

  char tmpl[] = "/tmp/kfa_selftest_XXXXXX";
  int fd = mkstemp(tmpl);
  CHECK(fd >= 0);
  close(fd);
  pid = spawn_process({"sh", "-c", "echo $KFA_SELFTEST; pwd; echo err >&2"}, env, "/tmp", tmpl);
  r = wait_exit(pid);
  CHECK(r.first == 0);
  std::ifstream f(tmpl);
  std::stringstream ss;
  ss << f.rdbuf();
  CHECK(ss.str().find("hello") != std::string::npos);
  CHECK(ss.str().find("/tmp") != std::string::npos);
  CHECK(ss.str().find("err") != std::string::npos);
  std::remove(tmpl);

  // process-group kill reaches the grandchild too
  pid = spawn_process({"/bin/sh", "-c", "sleep 30 & wait"}, env, "", "");
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  CHECK(pid_alive(pid));
  CHECK(kill_group(pid, SIGTERM));
  r = wait_exit(pid);
  CHECK(r.first == 128 + SIGTERM && r.second == SIGTERM);
  CHECK(!kill_group(-1, SIGTERM));
  CHECK(poll_process(pid)->first == -1);  // already reaped

  bool threw = false;
  try {
    spawn_process({}, env, "", "");
  } catch (const std::runtime_error &) {
    threw = true;
  }
  CHECK(threw);
  threw = false;
  try {
    spawn_process({"/nonexistent/kfa-binary"}, env, "", "");
  } catch (const std::runtime_error &) {
    threw = true;
  }
  CHECK(threw);
}

#ifdef KFA_SELFTEST_INJECT
// Deliberate defects, compiled only into the canary build that proves the
// sanitizer is live (tests/test_sanitizers_cpu.py expects it to be caught).
static void inject_defect() {
#if defined(__SANITIZE_THREAD__) || (defined(__has_feature) && __has_feature(thread_sanitizer))
  static long racy = 0;  // unsynchronised read-modify-write from two threads
  std::thread a([] { for (int i = 0; i < 100000; ++i) ++racy; });
  std::thread b([] { for (int i = 0; i < 100000; ++i) ++racy; });
  a.join();
  b.join();
  std::printf("racy=%ld\n", racy);
#else
  volatile int idx = 8;
  int *p = new int[8];
  p[idx] = 1;  // heap-buffer-overflow
  std::printf("%d\n", p[0]);
  delete[] p;
#endif
}
#endif

int main() {
#ifdef KFA_SELFTEST_INJECT
  inject_defect();
#endif
  test_rate_limiters();
  test_queue_dedup_and_exclusive_processing();
  test_dirty_while_processing();
  test_delayed_adds();
  test_queue_lifetime_churn();
  test_expectations();
  test_process_launcher();
  std::printf("runtime selftest: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
