// Native edge-serving runtime: latency histogram, activation arena planner, pinned frame
// ring, native hipGraph serve loop.  See kv_runtime.h for the design.
#include "kv_runtime.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>

namespace kvrt {

// ===========================================================================
// LatencyHist
// ===========================================================================
int LatencyHist::bucket_of(double us) {
  if (!(us >= 1.0)) return 0;  // also catches NaN
  int e;
  const double m = std::frexp(us, &e);  // us = m * 2^e, m in [0.5, 1)
  const int ex = e - 1;                 // us in [2^ex, 2^(ex+1))
  if (ex >= kMaxExp) return kBuckets - 1;
  int sub = (int)((m * 2.0 - 1.0) * kSub);
  sub = std::min(std::max(sub, 0), kSub - 1);
  return 1 + ex * kSub + sub;
}

double LatencyHist::bucket_lo(int b) {
  if (b <= 0) return 0.0;
  if (b >= kBuckets - 1) return std::ldexp(1.0, kMaxExp);
  const int ex = (b - 1) / kSub, sub = (b - 1) % kSub;
  return std::ldexp(1.0 + (double)sub / kSub, ex);
}

double LatencyHist::bucket_hi(int b) {
  if (b <= 0) return 1.0;
  if (b >= kBuckets - 1) return std::ldexp(1.0, kMaxExp + 1);
  const int ex = (b - 1) / kSub, sub = (b - 1) % kSub;
  return std::ldexp(1.0 + (double)(sub + 1) / kSub, ex);
}

void LatencyHist::add(int64_t* hist, double us) {
  hist[bucket_of(us)] += 1;
  hist[kBuckets] += 1;
  hist[kBuckets + 1] += (int64_t)std::llround(std::max(us, 0.0) * 1e3);
}

double LatencyHist::quantile(const int64_t* hist, double q) {
  const int64_t n = hist[kBuckets];
  if (n <= 0) return 0.0;
  q = std::min(std::max(q, 0.0), 1.0);
  // rank of the q-quantile (nearest-rank), interpolated linearly inside its bucket
  const double target = q * (double)(n - 1);
  int64_t seen = 0;
  for (int b = 0; b < kBuckets; ++b) {
    const int64_t c = hist[b];
    if (c == 0) continue;
    if ((double)(seen + c - 1) >= target) {
      const double frac = c > 1 ? (target - (double)seen) / (double)(c - 1) : 0.5;
      const double lo = bucket_lo(b), hi = bucket_hi(b);
      return lo + std::min(std::max(frac, 0.0), 1.0) * (hi - lo);
    }
    seen += c;
  }
  return bucket_lo(kBuckets - 1);
}

double LatencyHist::mean(const int64_t* hist) {
  const int64_t n = hist[kBuckets];
  return n > 0 ? (double)hist[kBuckets + 1] / 1e3 / (double)n : 0.0;
}

// ===========================================================================
// ArenaPlan: greedy by size (largest first); each tensor takes the lowest aligned
// offset whose [off, off+size) range does not collide with an already placed tensor
// whose lifetime overlaps.  O(n^2) -- n is a few hundred per model.
// ===========================================================================
int64_t arena_plan(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                   const std::vector<int64_t>& last, int64_t align,
                   std::vector<int64_t>* offsets) {
  const size_t n = sizes.size();
  if (first.size() != n || last.size() != n || align <= 0) return -1;
  offsets->assign(n, -1);
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    if (sizes[a] != sizes[b]) return sizes[a] > sizes[b];
    return first[a] < first[b];
  });
  auto up = [align](int64_t v) { return (v + align - 1) / align * align; };
  std::vector<size_t> placed;
  int64_t total = 0;
  std::vector<std::pair<int64_t, int64_t>> busy;  // [lo, hi) ranges of overlapping tensors
  for (size_t idx : order) {
    if (sizes[idx] < 0 || last[idx] < first[idx]) return -1;
    busy.clear();
    for (size_t j : placed)
      if (first[j] <= last[idx] && first[idx] <= last[j])
        busy.emplace_back((*offsets)[j], (*offsets)[j] + up(sizes[j]));
    std::sort(busy.begin(), busy.end());
    int64_t off = 0;
    const int64_t need = up(sizes[idx]);
    for (const auto& r : busy) {
      if (off + need <= r.first) break;  // fits in the gap before r
      off = std::max(off, r.second);
    }
    (*offsets)[idx] = off;
    total = std::max(total, off + need);
    placed.push_back(idx);
  }
  return total;
}

int64_t arena_live_peak(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                        const std::vector<int64_t>& last) {
  std::vector<std::pair<int64_t, int64_t>> ev;  // (time, +/-size); frees after allocs at t+1
  for (size_t i = 0; i < sizes.size(); ++i) {
    ev.emplace_back(first[i] * 2, sizes[i]);
    ev.emplace_back(last[i] * 2 + 1, -sizes[i]);
  }
  std::sort(ev.begin(), ev.end());
  int64_t cur = 0, peak = 0;
  for (const auto& e : ev) {
    cur += e.second;
    peak = std::max(peak, cur);
  }
  return peak;
}

// ===========================================================================
// FrameRing
// ===========================================================================
FrameRing::FrameRing(int slots, size_t slot_bytes) : slot_bytes_(slot_bytes) {
  slots = std::max(slots, 1);
  slots_.resize(slots, nullptr);
  state_.assign(slots, kFree);
  seq_.assign(slots, -1);
  order_.assign(slots, 0);
  slot_pinned_.assign(slots, 1);
  for (int i = 0; i < slots; ++i) {
    void* p = nullptr;
    // pinned so hipMemcpyAsync is a true DMA; a host with no GPU (tests, build box)
    // falls back to ordinary aligned memory
    if (hipHostMalloc(&p, slot_bytes ? slot_bytes : 1, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      p = std::aligned_alloc(4096, (slot_bytes + 4095) / 4096 * 4096 + 4096);
      pinned_ = false;
      slot_pinned_[i] = 0;
    }
    slots_[i] = p;
  }
}

FrameRing::~FrameRing() {
  close();
  for (int i = 0; i < slots(); ++i) {
    if (!slots_[i]) continue;
    if (slot_pinned_[i]) {
      (void)hipHostFree(slots_[i]);
    } else {
      std::free(slots_[i]);
    }
  }
}

int FrameRing::acquire_write(int timeout_ms, bool drop_oldest) {
  std::unique_lock<std::mutex> lk(mu_);
  auto pick = [&]() -> int {
    for (int i = 0; i < slots(); ++i)
      if (state_[i] == kFree) return i;
    if (drop_oldest) {  // recycle the oldest frame nobody is reading yet
      int best = -1;
      for (int i = 0; i < slots(); ++i)
        if (state_[i] == kReady && (best < 0 || order_[i] < order_[best])) best = i;
      if (best >= 0) dropped_.fetch_add(1);
      return best;
    }
    return -1;
  };
  int got = -1;
  const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(std::max(timeout_ms, 0)), [&] {
    if (closed_) return true;
    got = pick();
    return got >= 0;
  });
  if (!ok || closed_ || got < 0) return -1;
  state_[got] = kWriting;
  return got;
}

void FrameRing::publish(int i, int64_t seq) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (i < 0 || i >= slots() || state_[i] != kWriting) return;
    state_[i] = kReady;
    seq_[i] = seq;
    order_[i] = ++stamp_;
  }
  cv_.notify_all();
}

int FrameRing::acquire_read(int timeout_ms, int64_t* seq) {
  std::unique_lock<std::mutex> lk(mu_);
  int got = -1;
  auto pick = [&]() {
    got = -1;
    for (int i = 0; i < slots(); ++i)
      if (state_[i] == kReady && (got < 0 || order_[i] < order_[got])) got = i;
    return got >= 0;
  };
  const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(std::max(timeout_ms, 0)),
                               [&] { return pick() || closed_; });
  if (!ok || got < 0) return -1;
  state_[got] = kReading;
  if (seq) *seq = seq_[got];
  return got;
}

void FrameRing::release(int i) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (i < 0 || i >= slots() || state_[i] != kReading) return;
    state_[i] = kFree;
  }
  cv_.notify_all();
}

void FrameRing::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

int FrameRing::ready() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)std::count(state_.begin(), state_.end(), (int)kReady);
}

// ===========================================================================
// ServeLoop
// ===========================================================================
namespace {
struct InFlight {
  hipEvent_t start = nullptr, stop = nullptr;
  int slot = -1;
  bool live = false;
};
}  // namespace

int serve_loop(hipGraphExec_t exec, hipStream_t stream, int64_t n_steps, int depth,
               int64_t* hist, FrameRing* ring, void* dev_input, int ring_timeout_ms,
               ServeStats* stats) {
  if (!exec || n_steps < 0 || (ring && !dev_input)) return -1;
  depth = std::max(1, std::min(depth, 64));
  std::vector<InFlight> fl(depth);
  hipError_t err = hipSuccess;
  for (auto& f : fl) {
    if ((err = hipEventCreate(&f.start)) != hipSuccess) break;
    if ((err = hipEventCreate(&f.stop)) != hipSuccess) break;
  }
  ServeStats st;
  auto drain = [&](InFlight& f) -> hipError_t {
    if (!f.live) return hipSuccess;
    hipError_t e = hipEventSynchronize(f.stop);
    if (e != hipSuccess) return e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, f.start, f.stop);
    if (e != hipSuccess) return e;
    st.device_ms += ms;
    if (hist) LatencyHist::add(hist, (double)ms * 1e3);
    if (ring && f.slot >= 0) ring->release(f.slot);
    f.slot = -1;
    f.live = false;
    return hipSuccess;
  };
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t s = 0; err == hipSuccess && s < n_steps; ++s) {
    InFlight& f = fl[s % depth];
    if ((err = drain(f)) != hipSuccess) break;  // bounded in-flight window
    if ((err = hipEventRecord(f.start, stream)) != hipSuccess) break;
    if (ring) {
      int64_t seq = 0;
      const int slot = ring->acquire_read(ring_timeout_ms, &seq);
      if (slot >= 0) {
        err = hipMemcpyAsync(dev_input, ring->slot_ptr(slot), ring->slot_bytes(),
                             hipMemcpyHostToDevice, stream);
        if (err != hipSuccess) {
          ring->release(slot);
          break;
        }
        f.slot = slot;
        st.frames_in++;
      }
    }
    if ((err = hipGraphLaunch(exec, stream)) != hipSuccess) break;
    if ((err = hipEventRecord(f.stop, stream)) != hipSuccess) break;
    f.live = true;
    st.steps++;
  }
  for (auto& f : fl) {
    const hipError_t e = drain(f);
    if (err == hipSuccess) err = e;
  }
  st.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (auto& f : fl) {
    if (f.slot >= 0 && ring) ring->release(f.slot);
    if (f.start) (void)hipEventDestroy(f.start);
    if (f.stop) (void)hipEventDestroy(f.stop);
  }
  if (stats) *stats = st;
  return err == hipSuccess ? 0 : -(int)err;
}

}  // namespace kvrt
