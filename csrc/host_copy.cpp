// Host-side strided copies and a persistent worker pool.
//
// Reference: memcopy!/memcopy_threads! (src/update_halo.jl:755-774) copy flat
// halo buffers with Julia threads above GG_THREADCOPY_THRESHOLD bytes. Here the
// same threshold gates a persistent std::thread pool (no OpenMP runtime, so the
// library never fights PyTorch's libgomp for threads).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>

#include "igg/copy.hpp"

namespace igg {
namespace {

class Pool {
 public:
  Pool() {
    unsigned hw = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("IGG_HOST_THREADS")) hw = static_cast<unsigned>(std::atoi(e));
    nworkers_ = std::max(1u, std::min(hw, 64u)) - 1;  // caller participates
    for (unsigned i = 0; i < nworkers_; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  unsigned size() const { return nworkers_ + 1; }

  void run(int64_t nchunks, const std::function<void(int64_t)>& body) {
    std::lock_guard<std::mutex> run_lock(run_m_);  // one parallel region at a time
    {
      std::lock_guard<std::mutex> lk(m_);
      body_ = &body;
      next_.store(0);
      nchunks_ = nchunks;
      pending_ = nworkers_;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    body_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      int64_t c = next_.fetch_add(1);
      if (c >= nchunks_) break;
      (*body_)(c);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }

  unsigned nworkers_ = 0;
  std::vector<std::thread> threads_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* body_ = nullptr;
  std::atomic<int64_t> next_{0};
  int64_t nchunks_ = 0;
  unsigned pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

Pool& pool() {
  static Pool p;
  return p;
}

template <typename T>
void copy_rows(const Copy2D& c, int64_t o0, int64_t o1) {
  const T* src = reinterpret_cast<const T*>(c.src);
  T* dst = reinterpret_cast<T*>(c.dst);
  const size_t row_bytes = static_cast<size_t>(c.n_inner) * sizeof(T);
  for (int64_t o = o0; o < o1; ++o) {
    const T* s = src + o * c.src_so;
    T* d = dst + o * c.dst_so;
    if (c.src_si == 1 && c.dst_si == 1) {
      std::memcpy(d, s, row_bytes);
    } else {
      for (int64_t i = 0; i < c.n_inner; ++i) d[i * c.dst_si] = s[i * c.src_si];
    }
  }
}

struct alignas(16) B16 { uint64_t x, y; };

void copy_range(const Copy2D& c, int eb, int64_t o0, int64_t o1) {
  switch (eb) {
    case 1: copy_rows<uint8_t>(c, o0, o1); break;
    case 2: copy_rows<uint16_t>(c, o0, o1); break;
    case 4: copy_rows<uint32_t>(c, o0, o1); break;
    case 8: copy_rows<uint64_t>(c, o0, o1); break;
    case 16: copy_rows<B16>(c, o0, o1); break;
    default: fail("host_copy2d: unsupported element size ", eb, " bytes");
  }
}

}  // namespace

void host_parallel_for(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn) {
  if (n <= 0) return;
  grain = std::max<int64_t>(1, grain);
  const int64_t nchunks = (n + grain - 1) / grain;
  if (nchunks == 1 || pool().size() == 1) { fn(0, n); return; }
  std::function<void(int64_t)> body = [&](int64_t ch) {
    fn(ch * grain, std::min(n, (ch + 1) * grain));
  };
  pool().run(nchunks, body);
}

void host_copy2d(const std::vector<Copy2D>& copies, int elem_bytes) {
  for (const Copy2D& c : copies) {
    const int64_t bytes = c.n_outer * c.n_inner * elem_bytes;
    if (bytes <= 0) continue;
    if (bytes < THREADCOPY_THRESHOLD || c.n_outer < 2) {
      copy_range(c, elem_bytes, 0, c.n_outer);
    } else {
      const int64_t rows_per_chunk =
          std::max<int64_t>(1, c.n_outer / (4 * static_cast<int64_t>(pool().size())));
      host_parallel_for(c.n_outer, rows_per_chunk,
                        [&](int64_t o0, int64_t o1) { copy_range(c, elem_bytes, o0, o1); });
    }
  }
}

}  // namespace igg
