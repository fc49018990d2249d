// Native batch prefetcher: a background thread assembles shuffled mini-batches into a
// ring of `depth` host buffers while the trainer computes — the multi-threaded input queue
// of the reference's "ReadByQueue" branch (/root/reference/README.md:7), with exactly the
// epoch semantics of TF1's DataSet.next_batch (distribute_training.py:224):
// shuffle at the start and at every epoch boundary; a batch crossing the boundary is the
// tail of the old permutation followed by the head of the new one.
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "common.h"

namespace {

struct Slot {
  std::vector<uint8_t> x, y;
  int64_t epochs = 0;
  bool full = false;
};

struct Prefetcher {
  const uint8_t* x;
  const uint8_t* y;
  int64_t n;
  size_t xrow, yrow;
  int batch;
  std::vector<Slot> ring;
  std::mt19937_64 rng;
  std::vector<int64_t> perm;
  int64_t idx = 0, epochs = 0;
  size_t head = 0, tail = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool stop = false;
  std::thread th;

  void shuffle() {
    for (int64_t i = n - 1; i > 0; --i) {
      std::uniform_int_distribution<int64_t> d(0, i);
      std::swap(perm[i], perm[d(rng)]);
    }
  }

  void fill(Slot& s) {
    int64_t pos = 0;
    while (pos < batch) {
      if (idx >= n) {
        ++epochs;
        shuffle();
        idx = 0;
      }
      const int64_t take = std::min<int64_t>(batch - pos, n - idx);
      for (int64_t k = 0; k < take; ++k) {
        const int64_t src = perm[idx + k];
        std::memcpy(&s.x[(pos + k) * xrow], x + src * xrow, xrow);
        std::memcpy(&s.y[(pos + k) * yrow], y + src * yrow, yrow);
      }
      pos += take;
      idx += take;
    }
    s.epochs = epochs;
  }

  void run() {
    for (;;) {
      Slot* s;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !ring[head].full; });
        if (stop) return;
        s = &ring[head];
      }
      fill(*s);
      {
        std::lock_guard<std::mutex> lk(mu);
        s->full = true;
        head = (head + 1) % ring.size();
      }
      cv.notify_all();
    }
  }
};

}  // namespace

TTD_EXPORT void* ttd_prefetch_create(const void* x, const void* y, int64_t n, uint64_t xrow, uint64_t yrow, int batch,
                                     int depth, uint64_t seed) {
  if (n <= 0 || batch <= 0 || depth <= 0) {
    ttd::set_error("bad prefetch arguments");
    return nullptr;
  }
  auto* p = new Prefetcher;
  p->x = static_cast<const uint8_t*>(x);
  p->y = static_cast<const uint8_t*>(y);
  p->n = n;
  p->xrow = xrow;
  p->yrow = yrow;
  p->batch = batch;
  p->ring.resize(depth);
  for (auto& s : p->ring) {
    s.x.resize(static_cast<size_t>(batch) * xrow);
    s.y.resize(static_cast<size_t>(batch) * yrow);
  }
  p->rng.seed(seed);
  p->perm.resize(n);
  for (int64_t i = 0; i < n; ++i) p->perm[i] = i;
  p->shuffle();
  p->th = std::thread([p] { p->run(); });
  return p;
}

// Copies the next batch out; returns the number of completed epochs after it.
TTD_EXPORT int64_t ttd_prefetch_next(void* h, void* x_out, void* y_out) {
  auto* p = static_cast<Prefetcher*>(h);
  Slot* s;
  {
    std::unique_lock<std::mutex> lk(p->mu);
    p->cv.wait(lk, [&] { return p->ring[p->tail].full; });
    s = &p->ring[p->tail];
  }
  std::memcpy(x_out, s->x.data(), s->x.size());
  std::memcpy(y_out, s->y.data(), s->y.size());
  const int64_t ep = s->epochs;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    s->full = false;
    p->tail = (p->tail + 1) % p->ring.size();
  }
  p->cv.notify_all();
  return ep;
}

TTD_EXPORT void ttd_prefetch_destroy(void* h) {
  auto* p = static_cast<Prefetcher*>(h);
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    p->stop = true;
  }
  p->cv.notify_all();
  if (p->th.joinable()) p->th.join();
  delete p;
}
