// Concurrency stress test for the host runtime, built with ThreadSanitizer and with
// AddressSanitizer+UBSan by tools/sanitize_runtime.sh (and tests/test_runtime_sanitizers.py).
//
// It drives the parameter server the way the reference's cluster does
// (/root/reference/distribute_training.py:142-152, SURVEY.md §3.4 / §5 "race detection"),
// but from many threads of one process so the sanitizers see every interleaving:
//   * async phase: W workers Pull + ApplyGD(inc global_step) on shared variables (Hogwild),
//     while a monitor thread Saves/Restores, lists variables, reads stats and a re-init
//     thread replaces a variable with a differently sized one under concurrent pulls;
//   * sync phase: SyncReplicasOptimizer protocol — workers AccumApply(local_step), the chief
//     TakeApply(num_required, finalize, tokens) and workers block on the token queue — with an
//     exact expected result (every step applies the mean of exactly W gradients);
//   * named counters, queue close, Shutdown op;
//   * the batch prefetcher (producer thread vs consumer), checking epoch coverage.
// Exits 0 and prints "PASS" when every check holds; sanitizer reports make it fail.
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* ttd_ps_server_start(const char* host, int port, int task);
int ttd_ps_server_port(void* h);
void ttd_ps_server_stop(void* h);
void ttd_ps_server_destroy(void* h);
void* ttd_ps_client_connect(const char* host, int port, int timeout_ms);
int ttd_ps_client_call(void* h, uint32_t op, int nseg, const void* const* segs, const uint64_t* lens, int timeout_ms);
const void* ttd_ps_client_resp(void* h);
uint64_t ttd_ps_client_resp_len(void* h);
void ttd_ps_client_close(void* h);
const char* ttd_last_error();
void* ttd_prefetch_create(const void* x, const void* y, int64_t n, uint64_t xrow, uint64_t yrow, int batch, int depth,
                          uint64_t seed);
int64_t ttd_prefetch_next(void* h, void* x_out, void* y_out);
void ttd_prefetch_destroy(void* h);
}

namespace {

enum : uint32_t {
  kPing = 1, kInitVars = 2, kIsReady = 3, kSetReady = 4, kPull = 5, kApplyGD = 6, kAccumApply = 7,
  kTakeApply = 8, kTokenDequeue = 9, kTokenEnqueue = 10, kCloseQueue = 11, kGetGlobalStep = 12,
  kSetGlobalStep = 13, kSetAccumStep = 14, kSave = 15, kRestore = 16, kShutdown = 17, kListVars = 18,
  kStats = 19, kCounterAdd = 20
};

std::atomic<int> g_failures{0};

#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: %s | ", __FILE__, __LINE__, #c); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++g_failures;                                        \
    }                                                      \
  } while (0)

struct Msg {
  std::string b;
  template <typename T>
  Msg& put(T v) {
    b.append(reinterpret_cast<const char*>(&v), sizeof(T));
    return *this;
  }
  Msg& str(const std::string& s) {
    put<uint16_t>(static_cast<uint16_t>(s.size()));
    b.append(s);
    return *this;
  }
  Msg& raw(const void* p, size_t n) {
    b.append(static_cast<const char*>(p), n);
    return *this;
  }
};

struct Conn {
  void* h = nullptr;
  explicit Conn(int port) {
    h = ttd_ps_client_connect("127.0.0.1", port, 5000);
    if (!h) {
      std::fprintf(stderr, "connect failed: %s\n", ttd_last_error());
      std::exit(3);
    }
  }
  ~Conn() { ttd_ps_client_close(h); }
  int call(uint32_t op, const Msg& m, int timeout_ms = 20000) {
    const void* seg = m.b.data();
    uint64_t len = m.b.size();
    return ttd_ps_client_call(h, op, 1, &seg, &len, timeout_ms);
  }
  template <typename T>
  T resp_at(size_t off) const {
    T v{};
    if (off + sizeof(T) <= ttd_ps_client_resp_len(h))
      std::memcpy(&v, static_cast<const char*>(ttd_ps_client_resp(h)) + off, sizeof(T));
    return v;
  }
  std::vector<float> resp_floats(size_t off, size_t n) const {
    std::vector<float> v(n);
    if (off + 4 * n <= ttd_ps_client_resp_len(h))
      std::memcpy(v.data(), static_cast<const char*>(ttd_ps_client_resp(h)) + off, 4 * n);
    return v;
  }
};

Msg init_msg(const std::vector<std::pair<std::string, std::vector<float>>>& vars) {
  Msg m;
  m.put<uint32_t>(static_cast<uint32_t>(vars.size()));
  for (auto& kv : vars) {
    m.str(kv.first).put<int32_t>(1).put<uint32_t>(1).put<int64_t>(static_cast<int64_t>(kv.second.size()));
    m.put<uint64_t>(kv.second.size() * 4).raw(kv.second.data(), kv.second.size() * 4);
  }
  return m;
}

Msg names_msg(const std::vector<std::string>& names) {
  Msg m;
  m.put<uint32_t>(static_cast<uint32_t>(names.size()));
  for (auto& n : names) m.str(n);
  return m;
}

void async_phase(int port, const char* tmpdir) {
  constexpr int kW = 6, kIters = 150, kN = 4096;
  constexpr float kLr = 1e-3f;
  {
    Conn c(port);
    CHECK(c.call(kInitVars, init_msg({{"hidden/kernel", std::vector<float>(kN, 1.f)},
                                      {"hidden/bias", std::vector<float>(64, 0.f)},
                                      {"scratch", std::vector<float>(16, 0.f)}})) == 0, "init");
    CHECK(c.call(kSetGlobalStep, Msg().put<int64_t>(0)) == 0, "set gs");
    CHECK(c.call(kSetReady, Msg().put<uint8_t>(1)) == 0, "ready");
  }
  std::atomic<bool> done{false};
  std::vector<std::thread> th;
  for (int w = 0; w < kW; ++w)
    th.emplace_back([&, w] {
      Conn c(port);
      std::vector<float> g(kN, 1.f), gb(64, 0.5f);
      for (int it = 0; it < kIters; ++it) {
        CHECK(c.call(kPull, names_msg({"hidden/kernel", "hidden/bias"})) == 0, "pull w%d", w);
        CHECK(c.resp_at<uint64_t>(0) == kN * 4, "pull size");
        auto v = c.resp_floats(8, 4);
        CHECK(std::isfinite(v[0]) && v[0] <= 1.f && v[0] >= 1.f - kLr * kW * kIters - 1e-3f, "pull value %g", v[0]);
        Msg m;
        m.put<float>(kLr).put<uint8_t>(1).put<uint32_t>(2);
        m.str("hidden/kernel").put<uint64_t>(kN * 4).raw(g.data(), kN * 4);
        m.str("hidden/bias").put<uint64_t>(64 * 4).raw(gb.data(), 64 * 4);
        CHECK(c.call(kApplyGD, m) == 0, "apply");
      }
    });
  // re-init thread: replaces "scratch" with a differently sized var while others pull it
  th.emplace_back([&] {
    Conn c(port);
    for (int it = 0; !done.load(); ++it) {
      size_t n = (it & 1) ? 16 : 1024;
      CHECK(c.call(kInitVars, init_msg({{"scratch", std::vector<float>(n, float(it))}})) == 0, "reinit");
    }
  });
  th.emplace_back([&] {
    Conn c(port);
    while (!done.load()) {
      int st = c.call(kPull, names_msg({"scratch"}));
      CHECK(st == 0, "pull scratch");
      uint64_t nb = c.resp_at<uint64_t>(0);
      CHECK(nb == 64 || nb == 4096, "scratch size %llu", (unsigned long long)nb);
    }
  });
  // monitor: save/restore/list/stats/readiness while training runs (chief-style hooks)
  th.emplace_back([&] {
    Conn c(port);
    std::string prefix = std::string(tmpdir) + "/stress_ckpt";
    for (int it = 0; !done.load(); ++it) {
      CHECK(c.call(kSave, Msg().str(prefix).put<int32_t>(0).put<int32_t>(1).put<uint8_t>(1)) == 0, "save");
      CHECK(c.call(kListVars, Msg()) == 0, "list");
      CHECK(c.call(kStats, Msg()) == 0, "stats");
      CHECK(c.call(kIsReady, Msg()) == 0 && c.resp_at<uint8_t>(0) == 1, "ready");
      CHECK(c.call(kGetGlobalStep, Msg()) == 0, "gs");
      CHECK(c.call(kCounterAdd, Msg().str("monitor").put<int64_t>(1)) == 0, "counter");
      if (it == 0) {
        // restore only the non-trained variable: training vars must keep converging
        Conn c2(port);
        CHECK(c2.call(kPing, Msg()) == 0, "ping");
      }
    }
  });
  for (int w = 0; w < kW; ++w) th[w].join();
  done = true;
  for (size_t i = kW; i < th.size(); ++i) th[i].join();

  Conn c(port);
  CHECK(c.call(kGetGlobalStep, Msg()) == 0, "gs");
  CHECK(c.resp_at<int64_t>(0) == kW * kIters, "global step %lld", (long long)c.resp_at<int64_t>(0));
  CHECK(c.call(kPull, names_msg({"hidden/kernel"})) == 0, "pull");
  auto v = c.resp_floats(8, kN);
  // Hogwild may lose updates, but never tears words: every element is 1 - k*lr for an integer k
  for (int i = 0; i < kN; i += 97) {
    float k = (1.f - v[i]) / kLr;
    CHECK(k > 0.5f && k < kW * kIters + 0.5f && std::fabs(k - std::round(k)) < 0.05f, "elem %d = %g", i, v[i]);
  }
  // restore from the last checkpoint round-trips exactly
  std::string prefix = std::string(tmpdir) + "/stress_ckpt";
  CHECK(c.call(kSave, Msg().str(prefix).put<int32_t>(0).put<int32_t>(1).put<uint8_t>(1)) == 0, "save");
  CHECK(c.call(kInitVars, init_msg({{"hidden/kernel", std::vector<float>(kN, 7.f)}})) == 0, "clobber");
  CHECK(c.call(kRestore, Msg().str(prefix)) == 0, "restore");
  CHECK(c.call(kPull, names_msg({"hidden/kernel"})) == 0, "pull");
  auto r = c.resp_floats(8, kN);
  CHECK(std::memcmp(r.data(), v.data(), 4 * kN) == 0, "restore mismatch");
}

void sync_phase(int port) {
  constexpr int kW = 4, kSteps = 40, kN = 1000;
  constexpr float kLr = 0.5f;
  {
    Conn c(port);
    CHECK(c.call(kInitVars, init_msg({{"sync/w", std::vector<float>(kN, 0.f)}})) == 0, "init");
    CHECK(c.call(kSetAccumStep, Msg().put<int64_t>(0)) == 0, "accum step");
    CHECK(c.call(kSetGlobalStep, Msg().put<int64_t>(0)) == 0, "gs");
  }
  std::vector<std::thread> th;
  // chief: the sync_op of SyncReplicasOptimizer
  th.emplace_back([&] {
    Conn c(port);
    for (int s = 0; s < kSteps; ++s) {
      Msg m;
      m.put<uint32_t>(kW).put<float>(kLr).put<uint8_t>(1).put<uint32_t>(kW).put<uint32_t>(1).str("sync/w");
      CHECK(c.call(kTakeApply, m, 0) == 0, "take");
      CHECK(c.resp_at<int64_t>(0) == s + 1, "gs after take %lld", (long long)c.resp_at<int64_t>(0));
    }
  });
  for (int w = 0; w < kW; ++w)
    th.emplace_back([&, w] {
      Conn c(port);
      // identical gradients: tokens are shared, so a fast worker may contribute twice to one
      // step (TF semantics); the mean — and so the result — does not depend on who did
      std::vector<float> g(kN, 1.f);
      int64_t local = 0;
      // as a TF worker: loop until the global step reaches the limit (every token but the
      // final ones must turn into a gradient, or the chief's take would starve)
      for (int s = 0; local < kSteps; ++s) {
        Msg m;
        m.put<int64_t>(local).put<uint32_t>(1).str("sync/w").put<uint64_t>(kN * 4).raw(g.data(), kN * 4);
        CHECK(c.call(kAccumApply, m) == 0 && c.resp_at<uint32_t>(0) == 1, "accum w%d s%d", w, s);
        // a stale gradient (older local step) is dropped, never applied
        if (s == 3 && w == 0) {
          Msg st;
          st.put<int64_t>(-1).put<uint32_t>(1).str("sync/w").put<uint64_t>(kN * 4).raw(g.data(), kN * 4);
          CHECK(c.call(kAccumApply, st) == 0 && c.resp_at<uint32_t>(0) == 0, "stale accepted");
        }
        CHECK(c.call(kTokenDequeue, Msg(), 0) == 0, "dequeue");
        const int64_t tok = c.resp_at<int64_t>(0);
        CHECK(tok >= local && tok <= kSteps, "token %lld after %lld", (long long)tok, (long long)local);
        local = tok;
      }
    });
  for (auto& t : th) t.join();
  Conn c(port);
  CHECK(c.call(kPull, names_msg({"sync/w"})) == 0, "pull");
  auto v = c.resp_floats(8, kN);
  const float expect = -kLr * kSteps;
  CHECK(std::fabs(v[0] - expect) < 1e-3f && std::fabs(v[kN - 1] - expect) < 1e-3f, "sync w %g vs %g", v[0], expect);
  CHECK(c.call(kStats, Msg()) == 0 && c.resp_at<int64_t>(0) == 1, "dropped %lld", (long long)c.resp_at<int64_t>(0));
}

void counters_and_shutdown(int port) {
  constexpr int kT = 8, kAdds = 200;
  std::vector<std::thread> th;
  for (int t = 0; t < kT; ++t)
    th.emplace_back([&] {
      Conn c(port);
      for (int i = 0; i < kAdds; ++i) CHECK(c.call(kCounterAdd, Msg().str("workers_done").put<int64_t>(1)) == 0, "add");
    });
  // blocked dequeuers are released by CloseQueue with kClosed
  std::vector<std::thread> waiters;
  std::atomic<int> closed{0};
  for (int t = 0; t < 3; ++t)
    waiters.emplace_back([&] {
      Conn c(port);
      int st;
      while ((st = c.call(kTokenDequeue, Msg(), 0)) == 0) {
      }
      if (st == 2) ++closed;
    });
  for (auto& t : th) t.join();
  Conn c(port);
  CHECK(c.call(kCounterAdd, Msg().str("workers_done").put<int64_t>(0)) == 0, "read counter");
  CHECK(c.resp_at<int64_t>(0) == kT * kAdds, "counter %lld", (long long)c.resp_at<int64_t>(0));
  CHECK(c.call(kCloseQueue, Msg()) == 0, "close");
  for (auto& t : waiters) t.join();
  CHECK(closed.load() == 3, "closed waiters %d", closed.load());
  CHECK(c.call(kTokenEnqueue, Msg().put<uint32_t>(1).put<int64_t>(5)) == 2, "enqueue after close");
}

void prefetch_phase() {
  constexpr int kN = 1200, kB = 100, kEpochs = 5;
  std::vector<int32_t> x(kN * 3), y(kN);
  for (int i = 0; i < kN; ++i) {
    y[i] = i;
    for (int j = 0; j < 3; ++j) x[i * 3 + j] = i * 3 + j;
  }
  for (int depth : {1, 2, 4}) {
    void* p = ttd_prefetch_create(x.data(), y.data(), kN, 12, 4, kB, depth, 17 + depth);
    std::vector<int32_t> bx(kB * 3), by(kB);
    for (int e = 0; e < kEpochs; ++e) {
      std::vector<int> seen(kN, 0);
      int64_t ep = 0;
      for (int b = 0; b < kN / kB; ++b) {
        ep = ttd_prefetch_next(p, bx.data(), by.data());
        for (int i = 0; i < kB; ++i) {
          ++seen[by[i]];
          CHECK(bx[i * 3 + 2] == by[i] * 3 + 2, "row mismatch");
        }
      }
      CHECK(ep == e, "epochs %lld at %d", (long long)ep, e);
      for (int i = 0; i < kN; ++i) CHECK(seen[i] == 1, "sample %d seen %d in epoch %d", i, seen[i], e);
    }
    ttd_prefetch_destroy(p);  // with the producer blocked on a full ring
  }
}

}  // namespace

int main(int argc, char** argv) {
  const char* tmpdir = argc > 1 ? argv[1] : "/tmp";
  for (int round = 0; round < 2; ++round) {
    void* s = ttd_ps_server_start("127.0.0.1", 0, 0);
    if (!s) {
      std::fprintf(stderr, "server start failed: %s\n", ttd_last_error());
      return 3;
    }
    const int port = ttd_ps_server_port(s);
    async_phase(port, tmpdir);
    std::fprintf(stderr, "[stress] round %d: %s done\n", round, "async_phase");
    sync_phase(port);
    std::fprintf(stderr, "[stress] round %d: %s done\n", round, "sync_phase");
    counters_and_shutdown(port);
    std::fprintf(stderr, "[stress] round %d: %s done\n", round, "counters_and_shutdown");
    if (round == 0) {
      // explicit Shutdown op: the server stops itself; destroy must still be clean
      Conn c(port);
      CHECK(c.call(kShutdown, Msg()) == 0, "shutdown");
    }
    ttd_ps_server_destroy(s);
    std::fprintf(stderr, "[stress] round %d: server destroyed\n", round);
  }
  prefetch_phase();
  if (g_failures.load()) {
    std::fprintf(stderr, "FAILED (%d checks)\n", g_failures.load());
    return 1;
  }
  std::printf("PASS\n");
  return 0;
}
