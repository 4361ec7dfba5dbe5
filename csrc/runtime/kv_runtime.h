// Native edge-serving runtime (host C++; HIP runtime API only, no kernels).
//
// The reference (levi106/kvedge) has no runtime of its own: its "serving loop" is the
// IoT Edge module container started by edgeAgent (cast :2890/:3524).
// This is the MI355X-native piece that sits under the Python module app
// (kvedge_amd/module/app.py) and the inference engine (kvedge_amd/engine):
//
//   * LatencyHist  -- fixed-layout log-linear histogram of step latencies.  The bucket
//                     array is a plain int64 vector so replicas merge it with ONE RCCL /
//                     gloo all_reduce(SUM) and read fleet p50/p99.
//   * ArenaPlan    -- static activation-memory planner: tensors with (size, first_use,
//                     last_use) get offsets in one slab, greedy-by-size with interval
//                     conflicts.  The engine uses it to size the per-GPU batch against the
//                     288 GB HBM budget instead of guessing.
//   * ServeLoop    -- replays an instantiated hipGraphExec_t (torch.cuda.CUDAGraph's
//                     raw_cuda_graph_exec()) from native code with a bounded number of
//                     steps in flight, timing every step with HIP events into a
//                     LatencyHist, optionally copying a frame batch from a pinned host ring
//                     into the graph's fixed input buffer before each replay.  No Python,
//                     no GIL in the serving hot loop.
//   * FrameRing    -- pinned-host ring of frame slots filled by producer threads (camera /
//                     network ingest) and drained by ServeLoop; blocking hand-off with
//                     condition variables, drop-oldest policy when the GPU falls behind.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <vector>

namespace kvrt {

// ---------------------------------------------------------------------------
// LatencyHist: values in microseconds.  Buckets: [0,1) us, then per power of two
// 2^e .. 2^(e+1) us (e = 0..kMaxExp-1) split into kSub linear sub-buckets; the last
// bucket is an overflow.  Relative bucket width <= 1/kSub (3.1 %).
// ---------------------------------------------------------------------------
struct LatencyHist {
  static constexpr int kSub = 32;
  static constexpr int kMaxExp = 32;                   // up to 2^32 us (~71 min)
  static constexpr int kBuckets = 1 + kMaxExp * kSub + 1;

  static int bucket_of(double us);
  static double bucket_lo(int b);
  static double bucket_hi(int b);

  // Layout: kBuckets int64 counters, then {count, sum_ns}.  Every field merges by
  // plain addition, so an all_reduce(SUM) of the whole vector merges replicas.
  static constexpr int kLen = kBuckets + 2;
  static void add(int64_t* hist, double us);
  static double quantile(const int64_t* hist, double q);  // q in [0, 1]; 0 if empty
  static int64_t count(const int64_t* hist) { return hist[kBuckets]; }
  static double mean(const int64_t* hist);
};

// ---------------------------------------------------------------------------
// ArenaPlan: offsets for tensors with overlapping lifetimes [first, last] (inclusive
// op indices).  Returns the slab size; offsets[i] is aligned to `align`.
// ---------------------------------------------------------------------------
int64_t arena_plan(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                   const std::vector<int64_t>& last, int64_t align,
                   std::vector<int64_t>* offsets);
// sum over time of live bytes, maximised (a lower bound for any plan)
int64_t arena_live_peak(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                        const std::vector<int64_t>& last);

// ---------------------------------------------------------------------------
// FrameRing
// ---------------------------------------------------------------------------
class FrameRing {
 public:
  FrameRing(int slots, size_t slot_bytes);  // pinned host memory (hipHostMalloc)
  ~FrameRing();
  FrameRing(const FrameRing&) = delete;
  FrameRing& operator=(const FrameRing&) = delete;

  int slots() const { return (int)slots_.size(); }
  size_t slot_bytes() const { return slot_bytes_; }
  // producer: get a free slot (blocks up to timeout_ms; -1 on timeout / closed), fill
  // it, publish it.  With drop_oldest, a full ring recycles the oldest ready slot.
  int acquire_write(int timeout_ms, bool drop_oldest);
  void* slot_ptr(int i) { return slots_[i]; }
  void publish(int i, int64_t seq);
  // consumer: oldest ready slot (blocks up to timeout_ms; -1 on timeout / closed)
  int acquire_read(int timeout_ms, int64_t* seq);
  void release(int i);
  void close();
  int64_t dropped() const { return dropped_.load(); }
  int ready() const;
  bool pinned() const { return pinned_; }

 private:
  enum State : int { kFree = 0, kWriting = 1, kReady = 2, kReading = 3 };
  std::vector<void*> slots_;
  std::vector<int> state_;
  std::vector<char> slot_pinned_;
  std::vector<int64_t> seq_;
  std::vector<int64_t> order_;  // publish order stamp per slot
  int64_t stamp_ = 0;
  size_t slot_bytes_;
  bool closed_ = false;
  bool pinned_ = true;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<int64_t> dropped_{0};
};

// ---------------------------------------------------------------------------
// ServeLoop
// ---------------------------------------------------------------------------
struct ServeStats {
  int64_t steps = 0;
  double wall_s = 0.0;     // host wall clock from first launch to last completion
  double device_ms = 0.0;  // sum of per-step device time (event pairs)
  int64_t frames_in = 0;   // batches taken from the ring
};

// Replays `exec` n_steps times on `stream`.  Up to `depth` (>= 1) steps are in flight;
// each step is bracketed by a pair of events whose elapsed time is added to `hist`
// (LatencyHist layout, may be null).  If `ring` is non-null, each step first takes one
// ready slot (waiting up to ring_timeout_ms; on timeout the step reuses the last
// frames) and copies slot_bytes into `dev_input` with hipMemcpyAsync on the same
// stream; the slot is released once that copy has completed.
// Returns 0, or a negative hipError_t on failure.
int serve_loop(hipGraphExec_t exec, hipStream_t stream, int64_t n_steps, int depth,
               int64_t* hist, FrameRing* ring, void* dev_input, int ring_timeout_ms,
               ServeStats* stats);

}  // namespace kvrt
