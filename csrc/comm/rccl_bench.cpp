// C5: native RCCL collective bandwidth bench, rccl-tests style.
//
// One process drives every visible GPU (ncclCommInitAll) -- on one MI355X node that is
// the xGMI hive; inside one-GPU VMs use the torch.distributed variant
// (tools/allreduce_bench.py) which runs one process per VM.  For each message size it
// times all_reduce(sum), broadcast and all_gather with HIP events and reports
//   algBW = bytes / time,  busBW = algBW * factor  (all_reduce 2(n-1)/n,
//   all_gather (n-1)/n, broadcast 1)   -- the numbers to compare against the
// per-link xGMI ceiling (~153 GB/s per direction per link; rings are per-link bound).
//
// usage: kv_rccl_bench [min_bytes] [max_bytes] [iters] [dtype: bf16|fp32]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                       \
      std::exit(2);                                                                 \
    }                                                                               \
  } while (0)
#define NCCLCHK(x)                                                                  \
  do {                                                                              \
    ncclResult_t r_ = (x);                                                          \
    if (r_ != ncclSuccess) {                                                        \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, \
                   __LINE__);                                                       \
      std::exit(3);                                                                 \
    }                                                                               \
  } while (0)

enum Coll { kAllReduce, kBroadcast, kAllGather };

static double run(Coll c, std::vector<ncclComm_t>& comms, std::vector<hipStream_t>& st,
                  std::vector<void*>& sbuf, std::vector<void*>& rbuf, size_t count,
                  ncclDataType_t dt, int iters) {
  const int n = (int)comms.size();
  auto launch = [&]() {
    NCCLCHK(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
      if (c == kAllReduce)
        NCCLCHK(ncclAllReduce(sbuf[i], rbuf[i], count, dt, ncclSum, comms[i], st[i]));
      else if (c == kBroadcast)
        NCCLCHK(ncclBroadcast(sbuf[i], rbuf[i], count, dt, 0, comms[i], st[i]));
      else
        NCCLCHK(ncclAllGather(sbuf[i], rbuf[i], count / n, dt, comms[i], st[i]));
    }
    NCCLCHK(ncclGroupEnd());
  };
  for (int w = 0; w < 3; ++w) launch();
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipStreamSynchronize(st[i]));
  }
  HIPCHK(hipSetDevice(0));
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  HIPCHK(hipEventRecord(a, st[0]));
  for (int it = 0; it < iters; ++it) launch();
  HIPCHK(hipSetDevice(0));
  HIPCHK(hipEventRecord(b, st[0]));
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipStreamSynchronize(st[i]));
  }
  HIPCHK(hipSetDevice(0));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  HIPCHK(hipEventDestroy(a));
  HIPCHK(hipEventDestroy(b));
  return ms / iters * 1e-3;  // seconds per op
}

int main(int argc, char** argv) {
  size_t min_b = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8;
  size_t max_b = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (size_t)1 << 30;
  int iters = argc > 3 ? std::atoi(argv[3]) : 20;
  std::string dts = argc > 4 ? argv[4] : "bf16";
  const ncclDataType_t dt = dts == "fp32" ? ncclFloat32 : ncclBfloat16;
  const size_t esz = dts == "fp32" ? 4 : 2;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (n < 1) {
    std::fprintf(stderr, "no GPU\n");
    return 1;
  }
  std::vector<ncclComm_t> comms(n);
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  NCCLCHK(ncclCommInitAll(comms.data(), n, devs.data()));
  std::vector<hipStream_t> st(n);
  std::vector<void*> sbuf(n), rbuf(n);
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    HIPCHK(hipMalloc(&sbuf[i], max_b));
    HIPCHK(hipMalloc(&rbuf[i], max_b));
    HIPCHK(hipMemset(sbuf[i], 0, max_b));
  }
  const char* names[] = {"all_reduce", "broadcast", "all_gather"};
  const double f_ar = n > 1 ? 2.0 * (n - 1) / n : 0.0;
  const double f_ag = n > 1 ? (double)(n - 1) / n : 0.0;
  for (size_t bytes = min_b; bytes <= max_b; bytes *= 4) {
    size_t count = bytes / esz;
    if (count < (size_t)n) continue;
    count -= count % n;
    for (int c = 0; c < 3; ++c) {
      const double t = run((Coll)c, comms, st, sbuf, rbuf, count, dt, iters);
      const double alg = count * esz / t / 1e9;
      const double bus = alg * (c == kAllReduce ? f_ar : c == kAllGather ? f_ag : 1.0);
      std::printf("{\"coll\": \"%s\", \"n_gpus\": %d, \"bytes\": %zu, \"dtype\": \"%s\", "
                  "\"us\": %.2f, \"algbw_GBps\": %.2f, \"busbw_GBps\": %.2f}\n",
                  names[c], n, count * esz, dts.c_str(), t * 1e6, alg, bus);
    }
  }
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipFree(sbuf[i]));
    HIPCHK(hipFree(rbuf[i]));
    ncclCommDestroy(comms[i]);
  }
  return 0;
}
