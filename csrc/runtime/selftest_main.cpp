// Host self-test of the native serving runtime (kv_runtime.h).  Runs on the CPU build
// box (no GPU: the serve-loop part is skipped) and on the MI355X (serve loop over a
// captured hipGraph of a memset + memcpy).  Also the target of the AddressSanitizer
// build (kvedge_amd/_build.py --asan): sanitizers apply to host code only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "kv_runtime.h"

using namespace kvrt;

static int g_fail = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static void test_hist() {
  std::vector<int64_t> h(LatencyHist::kLen, 0);
  // buckets are contiguous and monotone
  for (int b = 0; b + 1 < LatencyHist::kBuckets; ++b)
    CHECK(LatencyHist::bucket_hi(b) == LatencyHist::bucket_lo(b + 1));
  for (double us : {0.5, 1.0, 1.5, 3.0, 1000.0, 1e6, 12345.6})
    CHECK(LatencyHist::bucket_lo(LatencyHist::bucket_of(us)) <= us + 1e-9 &&
          us < LatencyHist::bucket_hi(LatencyHist::bucket_of(us)));
  std::mt19937 rng(1);
  std::uniform_real_distribution<double> u(1000.0, 2000.0);
  std::vector<double> v;
  for (int i = 0; i < 20000; ++i) {
    v.push_back(u(rng));
    LatencyHist::add(h.data(), v.back());
  }
  std::sort(v.begin(), v.end());
  for (double q : {0.5, 0.9, 0.99}) {
    const double exact = v[(size_t)(q * (v.size() - 1))];
    const double est = LatencyHist::quantile(h.data(), q);
    CHECK(std::fabs(est - exact) / exact < 0.035);
  }
  CHECK(LatencyHist::count(h.data()) == 20000);
  CHECK(std::fabs(LatencyHist::mean(h.data()) - 1500.0) < 15.0);
  // merge by addition == histogram of the union
  std::vector<int64_t> a(LatencyHist::kLen, 0), b(LatencyHist::kLen, 0), ab(LatencyHist::kLen, 0);
  for (int i = 0; i < 100; ++i) {
    LatencyHist::add(a.data(), 10.0 + i);
    LatencyHist::add(b.data(), 500.0 + i);
    LatencyHist::add(ab.data(), 10.0 + i);
    LatencyHist::add(ab.data(), 500.0 + i);
  }
  for (int i = 0; i < LatencyHist::kLen; ++i) a[i] += b[i];
  CHECK(a == ab);
}

static void test_arena() {
  // chain a->b->c: a and c may share memory, b may not overlap either
  std::vector<int64_t> sizes = {100, 200, 100}, first = {0, 1, 2}, last = {1, 2, 3}, off;
  const int64_t total = arena_plan(sizes, first, last, 64, &off);
  CHECK(total == 128 + 256);
  CHECK(off[0] == off[2] || off[0] + 128 <= off[2] || off[2] + 128 <= off[0]);
  // random instances: no two live-overlapping tensors overlap in memory; total >= peak
  std::mt19937 rng(7);
  for (int it = 0; it < 200; ++it) {
    const int n = 1 + (int)(rng() % 60);
    sizes.assign(n, 0), first.assign(n, 0), last.assign(n, 0);
    for (int i = 0; i < n; ++i) {
      sizes[i] = 1 + (int64_t)(rng() % 5000);
      first[i] = rng() % 100;
      last[i] = first[i] + rng() % 20;
    }
    const int64_t t = arena_plan(sizes, first, last, 256, &off);
    CHECK(t >= arena_live_peak(sizes, first, last));
    for (int i = 0; i < n; ++i) {
      CHECK(off[i] % 256 == 0);
      for (int j = i + 1; j < n; ++j) {
        const bool live = first[i] <= last[j] && first[j] <= last[i];
        const bool mem = off[i] < off[j] + sizes[j] && off[j] < off[i] + sizes[i];
        CHECK(!(live && mem));
      }
    }
  }
  CHECK(arena_plan({1}, {2}, {1}, 64, &off) == -1);  // bad interval
}

static void test_ring() {
  FrameRing ring(3, 1024);
  CHECK(ring.slots() == 3);
  CHECK(ring.acquire_read(0, nullptr) == -1);  // empty
  // producer thread publishes 200 frames, consumer checks order and content
  const int n = 200;
  std::thread prod([&] {
    for (int i = 0; i < n; ++i) {
      const int s = ring.acquire_write(2000, false);
      if (s < 0) return;
      std::memset(ring.slot_ptr(s), i & 0xff, ring.slot_bytes());
      ring.publish(s, i);
    }
  });
  int64_t expect = 0;
  while (expect < n) {
    int64_t seq = -1;
    const int s = ring.acquire_read(2000, &seq);
    if (s < 0) break;
    CHECK(seq == expect);
    CHECK(static_cast<unsigned char*>(ring.slot_ptr(s))[1023] == (unsigned char)(seq & 0xff));
    ring.release(s);
    ++expect;
  }
  prod.join();
  CHECK(expect == n);
  // drop-oldest when the consumer stalls
  FrameRing r2(2, 16);
  for (int i = 0; i < 5; ++i) {
    const int s = r2.acquire_write(10, true);
    CHECK(s >= 0);
    r2.publish(s, i);
  }
  CHECK(r2.dropped() == 3);
  int64_t seq = -1;
  int s = r2.acquire_read(0, &seq);
  CHECK(s >= 0 && seq == 3);
  r2.release(s);
  r2.close();
  CHECK(r2.acquire_write(10, false) == -1);
}

static void test_serve_loop() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    std::printf("serve_loop: no GPU, skipped\n");
    return;
  }
  const size_t bytes = 1 << 20;
  void *in = nullptr, *out = nullptr;
  CHECK(hipMalloc(&in, bytes) == hipSuccess);
  CHECK(hipMalloc(&out, bytes) == hipSuccess);
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess);
  CHECK(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, s) == hipSuccess);
  CHECK(hipStreamEndCapture(s, &g) == hipSuccess);
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess);
  FrameRing ring(4, bytes);
  std::thread prod([&] {
    for (int i = 0; i < 32; ++i) {
      const int k = ring.acquire_write(2000, false);
      if (k < 0) return;
      std::memset(ring.slot_ptr(k), 0x40 + (i & 7), bytes);
      ring.publish(k, i);
    }
  });
  std::vector<int64_t> h(LatencyHist::kLen, 0);
  ServeStats st;
  const int rc = serve_loop(ge, s, 32, 3, h.data(), &ring, in, 2000, &st);
  prod.join();
  CHECK(rc == 0);
  CHECK(st.steps == 32 && st.frames_in == 32);
  CHECK(LatencyHist::count(h.data()) == 32);
  unsigned char last = 0;
  CHECK(hipMemcpy(&last, out, 1, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(last == 0x40 + 7);
  std::printf("serve_loop: %lld steps, p50 %.1f us, wall %.3f ms\n", (long long)st.steps,
              LatencyHist::quantile(h.data(), 0.5), st.wall_s * 1e3);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  (void)hipFree(in);
  (void)hipFree(out);
}

int main() {
  test_hist();
  test_arena();
  test_ring();
  test_serve_loop();
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
