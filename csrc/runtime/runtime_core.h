#pragma once
// Native control-plane runtime core for the TFJob controller: no Python
// dependency, so the same code is bound by runtime.cpp (pybind11 module
// `kubeflow_controller_amd._native_runtime`) and driven directly by the
// sanitizer self-test (selftest.cpp, ASan+UBSan and TSan builds).
//
// The reference gets these from vendored Go (client-go / kubernetes):
//   * WorkQueue + RateLimitingQueue + DelayingQueue
//       VCG/util/workqueue/queue.go:33-158, delaying_queue.go, rate_limitting_queue.go:20-69
//   * ItemExponentialFailureRateLimiter / BucketRateLimiter / MaxOf
//       VCG/util/workqueue/default_rate_limiters.go:39-105
//   * ControllerExpectations (TTL 5 min)
//       VKC/controller_utils.go:56-67, 136-288
//   * the kubelet's process lifecycle (here: posix_spawn into a new session,
//     a reaper that reports exit codes, process-group kill)
//
// The bindings release the GIL around blocking calls.  Time comes from a monotonic clock
// that tests can freeze (`set_fake_clock`) to exercise TTL / backoff paths.
#include <spawn.h>
#include <signal.h>
#include <fcntl.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <optional>
#include <queue>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

extern char **environ;

// ----------------------------------------------------------------------------- clock
static std::atomic<bool> g_fake{false};
static std::atomic<double> g_fake_now{0.0};

static double now_s() {
  if (g_fake.load()) return g_fake_now.load();
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ----------------------------------------------------------------------------- rate limiters
struct RateLimiter {
  virtual ~RateLimiter() = default;
  virtual double when(const std::string &item) = 0;
  virtual void forget(const std::string &item) = 0;
  virtual int num_requeues(const std::string &item) = 0;
};

// 5ms * 2^failures, capped (default_rate_limiters.go:54-105)
struct ExpFailureLimiter : RateLimiter {
  double base, maxd;
  std::mutex mu;
  std::unordered_map<std::string, int> failures;
  ExpFailureLimiter(double b, double m) : base(b), maxd(m) {}
  double when(const std::string &item) override {
    std::lock_guard<std::mutex> g(mu);
    int exp = failures[item]++;
    double backoff = base * std::pow(2.0, (double)exp);
    if (!std::isfinite(backoff) || backoff > maxd) return maxd;
    return backoff;
  }
  void forget(const std::string &item) override {
    std::lock_guard<std::mutex> g(mu);
    failures.erase(item);
  }
  int num_requeues(const std::string &item) override {
    std::lock_guard<std::mutex> g(mu);
    auto it = failures.find(item);
    return it == failures.end() ? 0 : it->second;
  }
};

// golang.org/x/time/rate token bucket: Reserve().Delay()  (default_rate_limiters.go:39-45)
struct BucketLimiter : RateLimiter {
  double qps, burst, tokens, last;
  std::mutex mu;
  BucketLimiter(double q, int b) : qps(q), burst(b), tokens(b), last(now_s()) {}
  double when(const std::string &) override {
    std::lock_guard<std::mutex> g(mu);
    double t = now_s();
    tokens = std::min(burst, tokens + (t - last) * qps);
    last = t;
    tokens -= 1.0;
    return tokens < 0 ? -tokens / qps : 0.0;
  }
  void forget(const std::string &) override {}
  int num_requeues(const std::string &) override { return 0; }
};

struct MaxOfLimiter : RateLimiter {
  std::vector<std::shared_ptr<RateLimiter>> ls;
  explicit MaxOfLimiter(std::vector<std::shared_ptr<RateLimiter>> l) : ls(std::move(l)) {}
  double when(const std::string &item) override {
    double r = 0;
    for (auto &l : ls) r = std::max(r, l->when(item));
    return r;
  }
  void forget(const std::string &item) override {
    for (auto &l : ls) l->forget(item);
  }
  int num_requeues(const std::string &item) override {
    int r = 0;
    for (auto &l : ls) r = std::max(r, l->num_requeues(item));
    return r;
  }
};

static std::shared_ptr<RateLimiter> default_controller_rate_limiter() {
  return std::make_shared<MaxOfLimiter>(std::vector<std::shared_ptr<RateLimiter>>{
      std::make_shared<ExpFailureLimiter>(0.005, 1000.0), std::make_shared<BucketLimiter>(10.0, 100)});
}

// ----------------------------------------------------------------------------- work queue
// Dedup FIFO with processing/dirty sets: an item is never handed to two
// workers at once and re-adds while processing are deferred to Done().
// Delayed adds live in a min-heap drained by a waiter thread.
class WorkQueue {
 public:
  WorkQueue(std::string name, std::shared_ptr<RateLimiter> limiter)
      : name_(std::move(name)), limiter_(std::move(limiter)) {
    waiter_ = std::thread([this] { wait_loop(); });
  }
  ~WorkQueue() {
    shut_down();
    if (waiter_.joinable()) waiter_.join();
  }

  void add(const std::string &item) {
    std::lock_guard<std::mutex> g(mu_);
    add_locked(item);
  }
  int len() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)queue_.size();
  }
  // returns (item, shutdown); item is empty when shutdown or timeout
  std::pair<std::optional<std::string>, bool> get(double timeout) {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [this] { return !queue_.empty() || shutting_down_; };
    if (timeout < 0) {
      cv_.wait(lk, pred);
    } else if (!cv_.wait_for(lk, std::chrono::duration<double>(timeout), pred)) {
      return {std::nullopt, false};
    }
    if (queue_.empty()) return {std::nullopt, true};
    std::string item = queue_.front();
    queue_.pop_front();
    processing_.insert(item);
    dirty_.erase(item);
    return {item, false};
  }
  void done(const std::string &item) {
    std::lock_guard<std::mutex> g(mu_);
    processing_.erase(item);
    if (dirty_.count(item)) {
      queue_.push_back(item);
      cv_.notify_one();
    }
  }
  void shut_down() {
    {
      std::lock_guard<std::mutex> g(mu_);
      shutting_down_ = true;
    }
    cv_.notify_all();
    wcv_.notify_all();
  }
  bool shutting_down() {
    std::lock_guard<std::mutex> g(mu_);
    return shutting_down_;
  }
  void add_after(const std::string &item, double delay) {
    if (delay <= 0) {
      add(item);
      return;
    }
    std::lock_guard<std::mutex> g(mu_);
    if (shutting_down_) return;
    double ready = now_s() + delay;
    auto it = waiting_at_.find(item);
    if (it != waiting_at_.end() && it->second <= ready) return;  // keep earliest
    waiting_at_[item] = ready;
    heap_.push({ready, item});
    wcv_.notify_all();
  }
  void add_rate_limited(const std::string &item) { add_after(item, limiter_->when(item)); }
  void forget(const std::string &item) { limiter_->forget(item); }
  int num_requeues(const std::string &item) { return limiter_->num_requeues(item); }
  int num_waiting() {
    std::lock_guard<std::mutex> g(mu_);
    return (int)waiting_at_.size();
  }
  // Test hook for the fake clock: move due delayed items into the queue now.
  void poll_delayed() {
    std::lock_guard<std::mutex> g(mu_);
    drain_ready_locked(now_s());
  }
  const std::string &name() const { return name_; }

 private:
  void add_locked(const std::string &item) {
    if (shutting_down_) return;
    if (dirty_.count(item)) return;
    dirty_.insert(item);
    if (processing_.count(item)) return;
    queue_.push_back(item);
    cv_.notify_one();
  }
  void drain_ready_locked(double t) {
    while (!heap_.empty() && heap_.top().first <= t) {
      auto e = heap_.top();
      heap_.pop();
      auto it = waiting_at_.find(e.second);
      if (it == waiting_at_.end() || it->second != e.first) continue;  // superseded
      waiting_at_.erase(it);
      add_locked(e.second);
    }
  }
  void wait_loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!shutting_down_) {
      double t = now_s();
      drain_ready_locked(t);
      double wait = 0.25;  // re-check cadence (also picks up fake-clock moves)
      if (!heap_.empty()) wait = std::min(wait, std::max(0.0, heap_.top().first - t));
      wcv_.wait_for(lk, std::chrono::duration<double>(wait));
    }
  }

  std::string name_;
  std::shared_ptr<RateLimiter> limiter_;
  std::mutex mu_;
  std::condition_variable cv_, wcv_;
  std::deque<std::string> queue_;
  std::unordered_set<std::string> dirty_, processing_;
  bool shutting_down_ = false;
  using Entry = std::pair<double, std::string>;
  std::priority_queue<Entry, std::vector<Entry>, std::greater<Entry>> heap_;
  std::unordered_map<std::string, double> waiting_at_;
  std::thread waiter_;
};

// ----------------------------------------------------------------------------- expectations
class Expectations {
 public:
  explicit Expectations(double ttl) : ttl_(ttl) {}
  // SatisfiedExpectations: fulfilled, expired, or absent  (controller_utils.go:176-207)
  bool satisfied(const std::string &key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(key);
    if (it == m_.end()) return true;
    const Exp &e = it->second;
    if (e.add <= 0 && e.del <= 0) return true;
    if (now_s() - e.ts > ttl_) return true;
    return false;
  }
  // ExpectCreations == SetExpectations(key, add, 0): overwrite (reference quirk)
  void set(const std::string &key, long add, long del) {
    std::lock_guard<std::mutex> g(mu_);
    m_[key] = Exp{add, del, now_s()};
  }
  // RaiseExpectations: accumulate (used to fix the overwrite quirk)
  void raise(const std::string &key, long add, long del) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(key);
    if (it == m_.end() || (it->second.add <= 0 && it->second.del <= 0)) {
      m_[key] = Exp{add, del, now_s()};
    } else {
      it->second.add += add;
      it->second.del += del;
    }
  }
  void lower(const std::string &key, long add, long del) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(key);
    if (it == m_.end()) return;
    it->second.add -= add;
    it->second.del -= del;
  }
  void erase(const std::string &key) {
    std::lock_guard<std::mutex> g(mu_);
    m_.erase(key);
  }
  std::optional<std::tuple<long, long, double>> get(const std::string &key) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(key);
    if (it == m_.end()) return std::nullopt;
    return std::make_tuple(it->second.add, it->second.del, it->second.ts);
  }

 private:
  struct Exp {
    long add, del;
    double ts;
  };
  double ttl_;
  std::mutex mu_;
  std::unordered_map<std::string, Exp> m_;
};

// ----------------------------------------------------------------------------- process launcher
// posix_spawn into a new session (so the whole replica tree can be signalled
// as a process group), stdout+stderr appended to a log file.
static int spawn_process(const std::vector<std::string> &argv, const std::map<std::string, std::string> &env,
                         const std::string &cwd, const std::string &log_path) {
  if (argv.empty()) throw std::runtime_error("spawn: empty argv");
  posix_spawn_file_actions_t fa;
  posix_spawnattr_t at;
  posix_spawn_file_actions_init(&fa);
  posix_spawnattr_init(&at);
  short flags = POSIX_SPAWN_SETSID | POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF;
  posix_spawnattr_setflags(&at, flags);
  sigset_t empty, all;
  sigemptyset(&empty);
  sigfillset(&all);
  posix_spawnattr_setsigmask(&at, &empty);
  posix_spawnattr_setsigdefault(&at, &all);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  if (!log_path.empty()) {
    posix_spawn_file_actions_addopen(&fa, 1, log_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    posix_spawn_file_actions_adddup2(&fa, 1, 2);
  }
#if defined(__GLIBC__) && ((__GLIBC__ > 2) || (__GLIBC__ == 2 && __GLIBC_MINOR__ >= 29))
  if (!cwd.empty()) posix_spawn_file_actions_addchdir_np(&fa, cwd.c_str());
#endif
  std::vector<std::string> envs;
  for (auto &kv : env) envs.push_back(kv.first + "=" + kv.second);
  std::vector<char *> cargv, cenv;
  for (auto &s : argv) cargv.push_back(const_cast<char *>(s.c_str()));
  cargv.push_back(nullptr);
  for (auto &s : envs) cenv.push_back(const_cast<char *>(s.c_str()));
  cenv.push_back(nullptr);
  pid_t pid = 0;
  int rc = posix_spawnp(&pid, cargv[0], &fa, &at, cargv.data(), cenv.data());
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&at);
  if (rc != 0) throw std::runtime_error(std::string("spawn ") + argv[0] + ": " + strerror(rc));
  return (int)pid;
}

// Non-blocking reap of one specific child. Returns None while it runs,
// else (exit_code, term_signal).
static std::optional<std::pair<int, int>> poll_process(int pid) {
  int st = 0;
  pid_t r = waitpid((pid_t)pid, &st, WNOHANG);
  if (r == 0) return std::nullopt;
  if (r < 0) return std::make_pair(-1, 0);  // not our child / already reaped
  if (WIFEXITED(st)) return std::make_pair(WEXITSTATUS(st), 0);
  if (WIFSIGNALED(st)) return std::make_pair(128 + WTERMSIG(st), WTERMSIG(st));
  return std::nullopt;
}

static bool kill_group(int pid, int sig) {
  if (pid <= 0) return false;
  return ::killpg((pid_t)pid, sig) == 0 || ::kill((pid_t)pid, sig) == 0;
}

static bool pid_alive(int pid) { return pid > 0 && ::kill((pid_t)pid, 0) == 0; }

