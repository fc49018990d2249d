// Parameter-server runtime: the native equivalent of what `tf.train.Server(cluster,
// job_name="ps", ...)` + `server.join()` provide to the reference
// (/root/reference/distribute_training.py:173-181) and of the PS-resident kernels its
// worker graphs execute remotely:
//   * a variable store (VariableV2 on /job:ps/task:k, placed by replica_device_setter,
//     distribute_training.py:186-190),
//   * ApplyGradientDescent + AssignAdd(global_step) for async (Hogwild, no locking) updates
//     (distribute_training.py:149-152),
//   * per-variable ConditionalAccumulators (stale-gradient drop, blocking take of the mean)
//     and the `sync_token_q` FIFO token queue used by SyncReplicasOptimizer
//     (distribute_training.py:142-148),
//   * SaveV2/RestoreV2 of this task's shard (bundle.cc), readiness flag for the
//     chief/worker session-creation barrier, and an explicit Shutdown so PS processes
//     exit (fixes SURVEY.md §2.9 Q6).
//
// Transport: plain TCP, one thread per connection, length-prefixed binary frames:
//   request  = u32 magic 'TTDP' | u32 op | u64 body_len | body
//   response = u32 status        | u64 body_len | body
// The matching client lives at the bottom of this file; Python drives both via ctypes.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

extern "C" {
void* ttd_bundle_writer_open(const char* prefix, int shard_id, int num_shards);
int ttd_bundle_writer_add(void* h, const char* key, int dtype, int ndims, const int64_t* shape, const void* data,
                          uint64_t nbytes);
int ttd_bundle_writer_finish(void* h);
void* ttd_bundle_reader_open(const char* prefix);
int ttd_bundle_reader_num_entries(void* h);
const char* ttd_bundle_reader_key(void* h, int i);
int ttd_bundle_reader_entry(void* h, const char* key, int* dtype, int64_t* shape, uint64_t* nbytes, int* shard_id,
                            uint64_t* offset, uint32_t* masked_crc);
int ttd_bundle_reader_read(void* h, const char* key, void* out, uint64_t nbytes);
void ttd_bundle_reader_close(void* h);
}

namespace {

constexpr uint32_t kMagic = 0x50445454;  // "TTDP"

enum Op : uint32_t {
  kPing = 1,
  kInitVars = 2,
  kIsReady = 3,
  kSetReady = 4,
  kPull = 5,
  kApplyGD = 6,
  kAccumApply = 7,
  kTakeApply = 8,
  kTokenDequeue = 9,
  kTokenEnqueue = 10,
  kCloseQueue = 11,
  kGetGlobalStep = 12,
  kSetGlobalStep = 13,
  kSetAccumStep = 14,
  kSave = 15,
  kRestore = 16,
  kShutdown = 17,
  kListVars = 18,
  kStats = 19,
  kCounterAdd = 20,
};

enum Status : uint32_t { kOk = 0, kErr = 1, kClosed = 2, kNotFound = 3, kShuttingDown = 4 };

constexpr int kDtFloat = 1;
constexpr int kDtInt64 = 9;

struct Accumulator {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<float> sum;
  int64_t count = 0;
  int64_t step = 0;
  int64_t dropped = 0;
};

// Variable storage. Workers read (Pull) and update (ApplyGD) without locking, exactly as
// TF1's Hogwild `use_locking=False` kernels; to keep that well-defined under the C++
// memory model (and clean under ThreadSanitizer) every element access is a relaxed 32-bit
// atomic (a plain mov on x86: lost updates are allowed, torn words are not).
struct Var {
  int dtype = kDtFloat;
  std::vector<int64_t> shape;
  std::vector<uint32_t> words;  // float32 or int64 payload as 32-bit words
  Accumulator acc;
  size_t nbytes() const { return words.size() * 4; }
  size_t numel() const { return nbytes() / (dtype == kDtInt64 ? 8 : 4); }
  void load(char* dst) const {  // relaxed snapshot
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (size_t i = 0; i < words.size(); ++i) {
      uint32_t w = __atomic_load_n(&words[i], __ATOMIC_RELAXED);
      std::memcpy(d + i, &w, 4);
    }
  }
  void store(const char* src) {
    for (size_t i = 0; i < words.size(); ++i) {
      uint32_t w;
      std::memcpy(&w, src + 4 * i, 4);
      __atomic_store_n(&words[i], w, __ATOMIC_RELAXED);
    }
  }
  // w += a * g, elementwise-atomic, not RMW-atomic. `g` may be unaligned (request body).
  void axpy(float a, const void* gp) {
    const char* g = static_cast<const char*>(gp);
    for (size_t i = 0; i < words.size(); ++i) {
      uint32_t u = __atomic_load_n(&words[i], __ATOMIC_RELAXED);
      float w, gi;
      std::memcpy(&w, &u, 4);
      std::memcpy(&gi, g + 4 * i, 4);
      w += a * gi;
      std::memcpy(&u, &w, 4);
      __atomic_store_n(&words[i], u, __ATOMIC_RELAXED);
    }
  }
};
using VarPtr = std::shared_ptr<Var>;  // a Pull racing a re-init keeps its Var alive

// Cursor over a request body.
struct Body {
  const char* p;
  const char* end;
  bool ok = true;
  template <typename T>
  T get() {
    T v{};
    if (p + sizeof(T) > end) {
      ok = false;
      return v;
    }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint16_t n = get<uint16_t>();
    if (!ok || p + n > end) {
      ok = false;
      return {};
    }
    std::string s(p, n);
    p += n;
    return s;
  }
  const char* bytes(uint64_t n) {
    if (p + n > end) {
      ok = false;
      return nullptr;
    }
    const char* b = p;
    p += n;
    return b;
  }
};

template <typename T>
void put(std::string* s, T v) {
  s->append(reinterpret_cast<const char*>(&v), sizeof(T));
}

bool send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool recv_all(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

class Server {
 public:
  Server(int port, int task_index) : port_(port), task_(task_index) {}

  bool start(const char* bind_host) {
    lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) return fail("socket()");
    int one = 1;
    ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port_));
    if (!bind_host || !*bind_host || std::string(bind_host) == "0.0.0.0")
      a.sin_addr.s_addr = htonl(INADDR_ANY);
    else if (::inet_pton(AF_INET, bind_host, &a.sin_addr) != 1)
      a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) return fail("bind() port " + std::to_string(port_));
    if (::listen(lfd_, 128) != 0) return fail("listen()");
    if (port_ == 0) {
      socklen_t len = sizeof(a);
      ::getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &len);
      port_ = ntohs(a.sin_port);
    }
    accept_thread_ = std::thread([this] { accept_loop(); });
    return true;
  }

  int port() const { return port_; }

  void join() {
    std::unique_lock<std::mutex> lk(stop_mu_);
    stop_cv_.wait(lk, [this] { return stopping_.load(); });
  }

  void stop() {
    {
      std::unique_lock<std::mutex> lk(stop_mu_);
      if (stopping_.exchange(true)) {
        // Another thread is tearing down: wait until it is done.
        stop_cv_.wait(lk, [this] { return stopped_; });
        return;
      }
    }
    stop_cv_.notify_all();
    close_queue();
    {
      std::lock_guard<std::mutex> lk(vars_mu_);
      for (auto& kv : vars_) {
        std::lock_guard<std::mutex> al(kv.second->acc.mu);
        kv.second->acc.cv.notify_all();
      }
    }
    ::shutdown(lfd_, SHUT_RDWR);
    ::close(lfd_);
    if (accept_thread_.joinable()) accept_thread_.join();
    std::vector<std::thread> ts;
    {
      std::lock_guard<std::mutex> lk(conn_mu_);
      for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
      ts.swap(conn_threads_);
    }
    for (auto& t : ts)
      if (t.joinable()) t.join();
    std::lock_guard<std::mutex> lk(stop_mu_);
    stopped_ = true;
    stop_cv_.notify_all();  // under the lock: a waiter may destroy the server once it returns
  }

  ~Server() {
    stop();
    std::thread t;
    {
      std::lock_guard<std::mutex> lk(stop_mu_);
      t.swap(shutdown_thread_);
    }
    if (t.joinable()) t.join();
  }

  bool stopping() const { return stopping_.load(); }

 private:
  bool fail(const std::string& m) {
    ttd::set_error(m + ": " + std::strerror(errno));
    return false;
  }

  void accept_loop() {
    while (!stopping_) {
      int fd = ::accept(lfd_, nullptr, nullptr);
      if (fd < 0) {
        if (stopping_) break;
        if (errno == EINTR) continue;
        break;
      }
      int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> lk(conn_mu_);
      conn_fds_.push_back(fd);
      conn_threads_.emplace_back([this, fd] { serve(fd); });
    }
  }

  void serve(int fd) {
    std::vector<char> body;
    std::string resp;
    while (!stopping_) {
      uint32_t hdr[2];
      uint64_t blen;
      if (!recv_all(fd, hdr, 8) || !recv_all(fd, &blen, 8)) break;
      if (hdr[0] != kMagic) break;
      body.resize(blen);
      if (blen && !recv_all(fd, body.data(), blen)) break;
      resp.clear();
      Body b{body.data(), body.data() + blen};
      uint32_t st = handle(hdr[1], b, &resp);
      uint64_t rl = resp.size();
      if (!send_all(fd, &st, 4) || !send_all(fd, &rl, 8) || (rl && !send_all(fd, resp.data(), rl))) break;
      if (hdr[1] == kShutdown) {
        // Tear down off this connection thread (stop() joins it); the destructor joins this
        // thread, so a Shutdown racing ttd_ps_server_destroy never touches a freed server.
        std::lock_guard<std::mutex> lk(stop_mu_);
        if (!shutdown_thread_.joinable()) shutdown_thread_ = std::thread([this] { stop(); });
        break;
      }
    }
    {
      std::lock_guard<std::mutex> lk(conn_mu_);
      for (auto it = conn_fds_.begin(); it != conn_fds_.end(); ++it)
        if (*it == fd) {
          conn_fds_.erase(it);
          break;
        }
      ::close(fd);
    }
  }

  VarPtr find(const std::string& name) {
    std::lock_guard<std::mutex> lk(vars_mu_);
    auto it = vars_.find(name);
    return it == vars_.end() ? nullptr : it->second;
  }

  void close_queue() {
    std::lock_guard<std::mutex> lk(q_mu_);
    q_closed_ = true;
    q_cv_.notify_all();
  }

  void enqueue_tokens(uint32_t n, int64_t v) {
    std::lock_guard<std::mutex> lk(q_mu_);
    for (uint32_t i = 0; i < n; ++i) q_.push_back(v);
    q_cv_.notify_all();
  }

  uint32_t handle(uint32_t op, Body& b, std::string* out) {
    switch (op) {
      case kPing:
        put<int32_t>(out, task_);
        return kOk;
      case kInitVars: {
        uint32_t n = b.get<uint32_t>();
        for (uint32_t i = 0; i < n && b.ok; ++i) {
          std::string name = b.str();
          int32_t dt = b.get<int32_t>();
          uint32_t nd = b.get<uint32_t>();
          std::vector<int64_t> shape(nd);
          for (uint32_t d = 0; d < nd; ++d) shape[d] = b.get<int64_t>();
          uint64_t nb = b.get<uint64_t>();
          const char* data = b.bytes(nb);
          if (!b.ok || nb % 4) break;
          std::lock_guard<std::mutex> lk(vars_mu_);
          auto it = vars_.find(name);
          if (it != vars_.end() && it->second->nbytes() == nb) {
            it->second->store(data);  // keep accumulator state
          } else {
            auto v = std::make_shared<Var>();
            v->dtype = dt;
            v->shape = shape;
            v->words.resize(nb / 4);
            std::memcpy(v->words.data(), data, nb);
            vars_[name] = std::move(v);
          }
        }
        return b.ok ? kOk : kErr;
      }
      case kIsReady:
        put<uint8_t>(out, ready_.load() ? 1 : 0);
        put<int64_t>(out, generation_.load());
        return kOk;
      case kSetReady:
        ready_ = b.get<uint8_t>() != 0;
        ++generation_;
        return kOk;
      case kPull: {
        uint32_t n = b.get<uint32_t>();
        for (uint32_t i = 0; i < n && b.ok; ++i) {
          std::string name = b.str();
          VarPtr v = find(name);
          if (!v) {
            out->assign(name);
            return kNotFound;
          }
          put<uint64_t>(out, v->nbytes());
          const size_t at = out->size();
          out->resize(at + v->nbytes());
          v->load(&(*out)[at]);  // Hogwild read, as TF1 (no locking)
        }
        return b.ok ? kOk : kErr;
      }
      case kApplyGD: {
        float lr = b.get<float>();
        uint8_t inc = b.get<uint8_t>();
        uint32_t n = b.get<uint32_t>();
        for (uint32_t i = 0; i < n && b.ok; ++i) {
          std::string name = b.str();
          uint64_t nb = b.get<uint64_t>();
          const char* g = b.bytes(nb);  // unaligned: read with memcpy
          if (!b.ok) break;
          VarPtr v = find(name);
          if (!v || v->dtype != kDtFloat || v->nbytes() != nb) {
            out->assign(name);
            return kNotFound;
          }
          v->axpy(-lr, g);  // ApplyGradientDescent, use_locking=False
        }
        int64_t gs = inc ? global_step_.fetch_add(1) + 1 : global_step_.load();
        put<int64_t>(out, gs);
        return b.ok ? kOk : kErr;
      }
      case kAccumApply: {
        int64_t local_step = b.get<int64_t>();
        uint32_t n = b.get<uint32_t>();
        uint32_t accepted = 0;
        for (uint32_t i = 0; i < n && b.ok; ++i) {
          std::string name = b.str();
          uint64_t nb = b.get<uint64_t>();
          const char* g = b.bytes(nb);  // unaligned: read with memcpy
          if (!b.ok) break;
          VarPtr v = find(name);
          if (!v || v->nbytes() != nb) {
            out->assign(name);
            return kNotFound;
          }
          Accumulator& a = v->acc;
          std::lock_guard<std::mutex> lk(a.mu);
          if (local_step < a.step) {  // stale: silently dropped (ConditionalAccumulator)
            ++a.dropped;
            continue;
          }
          const size_t m = nb / 4;
          if (a.sum.size() != m) a.sum.assign(m, 0.f);
          for (size_t k = 0; k < m; ++k) {
            float gk;
            std::memcpy(&gk, g + 4 * k, 4);
            a.sum[k] += gk;
          }
          ++a.count;
          ++accepted;
          a.cv.notify_all();
        }
        put<uint32_t>(out, accepted);
        return b.ok ? kOk : kErr;
      }
      case kTakeApply: {
        // sync_op of SyncReplicasOptimizer for this task's variables:
        //   take_grad(num_required) (blocks, returns mean, resets, step += 1) -> GD apply,
        //   then (finalize) global_step += 1 and enqueue `tokens` tokens of the new step.
        uint32_t num_required = b.get<uint32_t>();
        float lr = b.get<float>();
        uint8_t finalize = b.get<uint8_t>();
        uint32_t tokens = b.get<uint32_t>();
        uint32_t n = b.get<uint32_t>();
        std::vector<VarPtr> vs;
        for (uint32_t i = 0; i < n && b.ok; ++i) {
          std::string name = b.str();
          VarPtr v = find(name);
          if (!v) {
            out->assign(name);
            return kNotFound;
          }
          vs.push_back(v);
        }
        if (!b.ok) return kErr;
        for (VarPtr& v : vs) {
          Accumulator& a = v->acc;
          std::unique_lock<std::mutex> lk(a.mu);
          a.cv.wait(lk, [&] { return stopping_.load() || a.count >= static_cast<int64_t>(num_required); });
          if (stopping_) return kShuttingDown;
          const float inv = 1.0f / static_cast<float>(a.count);
          if (a.sum.size() == v->numel()) v->axpy(-lr * inv, a.sum.data());
          std::fill(a.sum.begin(), a.sum.end(), 0.f);
          a.count = 0;
          ++a.step;
        }
        int64_t gs = global_step_.load();
        if (finalize) {
          gs = global_step_.fetch_add(1) + 1;
          enqueue_tokens(tokens, gs);
        }
        put<int64_t>(out, gs);
        return kOk;
      }
      case kTokenDequeue: {
        std::unique_lock<std::mutex> lk(q_mu_);
        q_cv_.wait(lk, [&] { return q_closed_ || !q_.empty(); });
        if (q_.empty()) return kClosed;
        put<int64_t>(out, q_.front());
        q_.pop_front();
        return kOk;
      }
      case kTokenEnqueue: {
        uint32_t n = b.get<uint32_t>();
        int64_t v = b.get<int64_t>();
        if (!b.ok) return kErr;
        {
          std::lock_guard<std::mutex> lk(q_mu_);
          if (q_closed_) return kClosed;
        }
        enqueue_tokens(n, v);
        return kOk;
      }
      case kCloseQueue:
        close_queue();
        return kOk;
      case kGetGlobalStep:
        put<int64_t>(out, global_step_.load());
        return kOk;
      case kSetGlobalStep:
        global_step_ = b.get<int64_t>();
        return b.ok ? kOk : kErr;
      case kSetAccumStep: {
        int64_t s = b.get<int64_t>();
        std::lock_guard<std::mutex> lk(vars_mu_);
        for (auto& kv : vars_) {
          Accumulator& a = kv.second->acc;
          std::lock_guard<std::mutex> al(a.mu);
          a.step = s;
          a.count = 0;
          std::fill(a.sum.begin(), a.sum.end(), 0.f);
        }
        return kOk;
      }
      case kSave: {
        std::string prefix = b.str();
        int32_t shard = b.get<int32_t>();
        int32_t nshards = b.get<int32_t>();
        uint8_t with_gs = b.get<uint8_t>();
        if (!b.ok) return kErr;
        void* w = ttd_bundle_writer_open(prefix.c_str(), shard, nshards);
        if (!w) {
          out->assign(ttd_last_error_str());
          return kErr;
        }
        std::vector<char> snap;
        std::lock_guard<std::mutex> lk(vars_mu_);
        for (auto& kv : vars_) {
          Var* v = kv.second.get();
          snap.resize(v->nbytes());
          v->load(snap.data());
          if (ttd_bundle_writer_add(w, kv.first.c_str(), v->dtype, static_cast<int>(v->shape.size()),
                                    v->shape.data(), snap.data(), snap.size()) != 0) {
            out->assign(ttd_last_error_str());
            ttd_bundle_writer_finish(w);
            return kErr;
          }
        }
        if (with_gs) {
          int64_t gs = global_step_.load();
          if (ttd_bundle_writer_add(w, "global_step", kDtInt64, 0, nullptr, &gs, 8) != 0) {
            out->assign(ttd_last_error_str());
            ttd_bundle_writer_finish(w);
            return kErr;
          }
        }
        if (ttd_bundle_writer_finish(w) != 0) {
          out->assign(ttd_last_error_str());
          return kErr;
        }
        return kOk;
      }
      case kRestore: {
        std::string prefix = b.str();
        if (!b.ok) return kErr;
        void* r = ttd_bundle_reader_open(prefix.c_str());
        if (!r) {
          out->assign(ttd_last_error_str());
          return kErr;
        }
        uint32_t restored = 0;
        std::lock_guard<std::mutex> lk(vars_mu_);
        int ne = ttd_bundle_reader_num_entries(r);
        for (int i = 0; i < ne; ++i) {
          std::string key = ttd_bundle_reader_key(r, i);
          int dt;
          int64_t shape[32];
          uint64_t nb;
          int nd = ttd_bundle_reader_entry(r, key.c_str(), &dt, shape, &nb, nullptr, nullptr, nullptr);
          if (nd < 0) continue;
          if (key == "global_step") {
            if (task_ != 0) continue;  // the global step lives on ps task 0
            int64_t gs = 0;
            if (ttd_bundle_reader_read(r, key.c_str(), &gs, 8) == 0) global_step_ = gs;
            ++restored;
            continue;
          }
          auto it = vars_.find(key);
          if (it == vars_.end()) continue;  // owned by another PS task
          Var* v = it->second.get();
          if (v->nbytes() != nb) continue;
          std::vector<char> buf(nb);
          if (ttd_bundle_reader_read(r, key.c_str(), buf.data(), nb) == 0) {
            v->store(buf.data());
            ++restored;
          }
        }
        ttd_bundle_reader_close(r);
        put<uint32_t>(out, restored);
        return kOk;
      }
      case kShutdown:
        return kOk;
      case kListVars: {
        std::lock_guard<std::mutex> lk(vars_mu_);
        put<uint32_t>(out, static_cast<uint32_t>(vars_.size()));
        for (auto& kv : vars_) {
          put<uint16_t>(out, static_cast<uint16_t>(kv.first.size()));
          out->append(kv.first);
          put<int32_t>(out, kv.second->dtype);
          put<uint32_t>(out, static_cast<uint32_t>(kv.second->shape.size()));
          for (int64_t d : kv.second->shape) put<int64_t>(out, d);
        }
        return kOk;
      }
      case kCounterAdd: {  // named int64 counters (e.g. "workers_done" for coordinated shutdown)
        std::string name = b.str();
        int64_t d = b.get<int64_t>();
        if (!b.ok) return kErr;
        std::lock_guard<std::mutex> lk(vars_mu_);
        const int64_t v = (counters_[name] += d);
        put<int64_t>(out, v);
        return kOk;
      }
      case kStats: {
        int64_t dropped = 0, step = -1;
        std::lock_guard<std::mutex> lk(vars_mu_);
        for (auto& kv : vars_) {
          std::lock_guard<std::mutex> al(kv.second->acc.mu);
          dropped += kv.second->acc.dropped;
          step = kv.second->acc.step;
        }
        size_t qn;
        {
          std::lock_guard<std::mutex> ql(q_mu_);
          qn = q_.size();
        }
        put<int64_t>(out, dropped);
        put<int64_t>(out, step);
        put<int64_t>(out, static_cast<int64_t>(qn));
        return kOk;
      }
      default:
        return kErr;
    }
  }

  static const char* ttd_last_error_str();

  int port_;
  int task_;
  int lfd_ = -1;
  std::thread accept_thread_;
  std::mutex conn_mu_;
  std::vector<int> conn_fds_;
  std::vector<std::thread> conn_threads_;
  std::mutex stop_mu_;
  std::condition_variable stop_cv_;
  std::atomic<bool> stopping_{false};
  bool stopped_ = false;
  std::thread shutdown_thread_;

  std::mutex vars_mu_;
  std::map<std::string, VarPtr> vars_;
  std::atomic<bool> ready_{false};
  std::atomic<int64_t> generation_{0};
  std::atomic<int64_t> global_step_{0};
  std::map<std::string, int64_t> counters_;

  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<int64_t> q_;
  bool q_closed_ = false;
};

}  // namespace

extern "C" const char* ttd_last_error();
const char* Server::ttd_last_error_str() { return ttd_last_error(); }

TTD_EXPORT void* ttd_ps_server_start(const char* bind_host, int port, int task_index) {
  auto* s = new Server(port, task_index);
  if (!s->start(bind_host)) {
    delete s;
    return nullptr;
  }
  return s;
}
TTD_EXPORT int ttd_ps_server_port(void* h) { return static_cast<Server*>(h)->port(); }
TTD_EXPORT void ttd_ps_server_join(void* h) { static_cast<Server*>(h)->join(); }
TTD_EXPORT void ttd_ps_server_stop(void* h) { static_cast<Server*>(h)->stop(); }
TTD_EXPORT int ttd_ps_server_stopping(void* h) { return static_cast<Server*>(h)->stopping() ? 1 : 0; }
TTD_EXPORT void ttd_ps_server_destroy(void* h) {
  auto* s = static_cast<Server*>(h);
  s->stop();
  delete s;
}

// ----------------------------------------------------------------------------- client
namespace {
struct Client {
  int fd = -1;
  std::string resp;
  std::mutex mu;
};
}  // namespace

TTD_EXPORT void* ttd_ps_client_connect(const char* host, int port, int timeout_ms) {
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string h = (host && *host && std::string(host) != "localhost") ? host : "127.0.0.1";
  if (::getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    ttd::set_error("cannot resolve " + h);
    return nullptr;
  }
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) {
    ::freeaddrinfo(res);
    ttd::set_error("socket() failed");
    return nullptr;
  }
  if (timeout_ms > 0) {
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  }
  if (::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    ::freeaddrinfo(res);
    ::close(fd);
    ttd::set_error("connect to " + h + ":" + std::to_string(port) + " failed: " + std::strerror(errno));
    return nullptr;
  }
  ::freeaddrinfo(res);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  auto* c = new Client;
  c->fd = fd;
  return c;
}

// Sends op with a body gathered from `nseg` segments and waits for the response.
// Returns the server status (>=0) or -1 on a transport error (peer gone).
// `recv_timeout_ms` <= 0 waits forever (blocking ops such as token dequeue).
TTD_EXPORT int ttd_ps_client_call(void* h, uint32_t op, int nseg, const void* const* segs, const uint64_t* lens,
                                  int recv_timeout_ms) {
  auto* c = static_cast<Client*>(h);
  std::lock_guard<std::mutex> lk(c->mu);
  uint64_t total = 0;
  for (int i = 0; i < nseg; ++i) total += lens[i];
  uint32_t hdr[2] = {kMagic, op};
  timeval tv{0, 0};
  if (recv_timeout_ms > 0) tv = timeval{recv_timeout_ms / 1000, (recv_timeout_ms % 1000) * 1000};
  ::setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  if (!send_all(c->fd, hdr, 8) || !send_all(c->fd, &total, 8)) {
    ttd::set_error("send failed (peer unavailable)");
    return -1;
  }
  for (int i = 0; i < nseg; ++i)
    if (lens[i] && !send_all(c->fd, segs[i], lens[i])) {
      ttd::set_error("send failed (peer unavailable)");
      return -1;
    }
  uint32_t st;
  uint64_t rl;
  if (!recv_all(c->fd, &st, 4) || !recv_all(c->fd, &rl, 8)) {
    ttd::set_error("recv failed (peer unavailable or timeout)");
    return -1;
  }
  c->resp.resize(rl);
  if (rl && !recv_all(c->fd, &c->resp[0], rl)) {
    ttd::set_error("recv body failed");
    return -1;
  }
  return static_cast<int>(st);
}

TTD_EXPORT const void* ttd_ps_client_resp(void* h) { return static_cast<Client*>(h)->resp.data(); }
TTD_EXPORT uint64_t ttd_ps_client_resp_len(void* h) { return static_cast<Client*>(h)->resp.size(); }
// Unblocks a call in progress on another thread (no lock): the peer read fails and the
// blocked ttd_ps_client_call returns -1. Used to cancel blocking takes/dequeues at shutdown.
TTD_EXPORT void ttd_ps_client_abort(void* h) {
  auto* c = static_cast<Client*>(h);
  if (c) ::shutdown(c->fd, SHUT_RDWR);
}

TTD_EXPORT void ttd_ps_client_close(void* h) {
  auto* c = static_cast<Client*>(h);
  if (!c) return;
  ::shutdown(c->fd, SHUT_RDWR);
  ::close(c->fd);
  delete c;
}
