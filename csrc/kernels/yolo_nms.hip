#include <stdlib.h>
// K9 YOLOv8 decode and K10 class-aware NMS for gfx950.  SURVEY.md §2.5, §7.3(2).
//
// Decode: one workgroup per 64 consecutive anchors of one (image, level): the
// 64 x (64 + nc) bf16 rows are contiguous, so they are copied into LDS with
// coalesced 16-B loads; then FOUR lanes per anchor: lane p does the DFL (softmax
// over 16 bins, expectation) of box side p -- which alone gives box coordinate p --
// and the class max over classes [p*nc/4, (p+1)*nc/4); the class max is merged with
// two xor-shuffles (sigmoid is monotonic: sigmoid(max logit) == max sigmoid).
// (The first version was one thread per anchor reading its 288-B row with scalar
// loads: 600 us at batch 64, 20x the HBM time of the 155 MB it reads.)
//
// NMS: one workgroup per image (latency-bound by nature):
//   1. compaction of candidates with score > conf into an LDS key array
//      key = score_bits << 32 | ~index  (descending key = score desc, index asc)
//   2. bitonic sort of up to 16384 keys in LDS (128 KiB of the CU's 160 KiB)
//   3. greedy suppression in chunks of 64 candidates, ONE WAVE64 LANE PER BOX:
//      all 8 waves test the chunk against interleaved eighths of the kept list
//      (ballot -> LDS), then wave 0 resolves the 64x64 in-chunk IoU matrix with
//      64-bit lane masks and v_readlane, and appends survivors in rank order.
//      Stops at max_det.
#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kRegMax = 16;
constexpr float kMaxWH = 7680.f;  // class offset for class-aware NMS
constexpr int kMaxCand = 16384;

constexpr int kDecAnch = 64;  // anchors per workgroup (256 threads = 4 lanes per anchor)

// NC > 0: the class count is a compile-time constant (COCO's 80), so the staging loop's
// row / chunk split is a multiply-shift instead of a runtime divide (a ~20-instruction VALU
// expansion per 16-B chunk on gfx9).  NC = 0: any nc % 8 == 0 at run time.
template <int NC>
__global__ __launch_bounds__(256) void yolo_decode_kernel(
    const bf16* __restrict__ f0, const bf16* __restrict__ f1, const bf16* __restrict__ f2,
    int h0, int w0, int h1, int w1, int h2, int w2, int s0, int s1, int s2, int N, int nc_rt,
    float* __restrict__ boxes, float* __restrict__ scores, int* __restrict__ cls) {
  const int nc = NC > 0 ? NC : nc_rt;
  extern __shared__ __attribute__((aligned(16))) bf16 tile[];  // [64][ch + 8]
  const int A0 = h0 * w0, A1 = h1 * w1, A2 = h2 * w2;
  const int A = A0 + A1 + A2;
  const int nb0 = (A0 + kDecAnch - 1) / kDecAnch, nb1 = (A1 + kDecAnch - 1) / kDecAnch;
  const int nb2 = (A2 + kDecAnch - 1) / kDecAnch, nbt = nb0 + nb1 + nb2;
  const int n = blockIdx.x / nbt;
  int r = blockIdx.x - n * nbt;
  const bf16* f;
  int Al, w, stride, abase;
  if (r < nb0) {
    f = f0; Al = A0; w = w0; stride = s0; abase = 0;
  } else if (r < nb0 + nb1) {
    r -= nb0; f = f1; Al = A1; w = w1; stride = s1; abase = A0;
  } else {
    r -= nb0 + nb1; f = f2; Al = A2; w = w2; stride = s2; abase = A0 + A1;
  }
  const int ch = 4 * kRegMax + nc, chp = ch + 8, c8 = ch / 8;
  const int a0 = r * kDecAnch;
  const int cnt = min(kDecAnch, Al - a0);
  const bf16* src = f + ((long long)n * Al + a0) * ch;
  for (int q = threadIdx.x; q < cnt * c8; q += 256) {  // coalesced: rows are contiguous
    const int row = q / c8, cc = q - row * c8;
    *reinterpret_cast<bf16x8*>(tile + row * chp + cc * 8) =
        *reinterpret_cast<const bf16x8*>(src + (long long)q * 8);
  }
  __syncthreads();
  const int a = threadIdx.x >> 2, p = threadIdx.x & 3;
  if (a >= cnt) return;  // whole 4-lane groups leave together; no barrier follows
  const bf16* row = tile + a * chp;
  // DFL for side p
  const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(row + p * 16);
  const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(row + p * 16 + 8);
  float x[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[j] = (float)v0[j];
    x[8 + j] = (float)v1[j];
  }
  float mx = x[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) mx = fmaxf(mx, x[j]);
  float se = 0.f, sw = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float e = __expf(x[j] - mx);
    se += e;
    sw += e * (float)j;
  }
  const float dist = sw / se;
  const int al = a0 + a;
  // al / w via a float reciprocal: al < 2^16, and (al + 0.5) / w sits >= 0.5 / w away from
  // an integer, far beyond the float rounding error, so the floor is exact
  const int iy = (int)(((float)al + 0.5f) * __frcp_rn((float)w));
  const float ax = (float)(al - iy * w) + 0.5f, ay = (float)iy + 0.5f;
  // p: 0 -> x1 = ax - l, 1 -> y1 = ay - t, 2 -> x2 = ax + r, 3 -> y2 = ay + b
  const float base = (p & 1) ? ay : ax;
  const long long i = (long long)n * A + abase + al;
  boxes[i * 4 + p] = (p < 2 ? base - dist : base + dist) * (float)stride;
  // class max over this lane's quarter, then across the 4 lanes (ties -> lower class)
  const int cq = nc / 4;
  const bf16* cr = row + 4 * kRegMax + p * cq;
  float best = -INFINITY;
  int bc = p * cq;
  if ((cq & 3) == 0) {
    // 8-B LDS reads (cq*2 bytes per lane quarter is 8-B aligned; rows are 16-B aligned):
    // 4x fewer ds_read issues than the u16 loop, same first-max tie rule
    for (int c = 0; c < cq; c += 4) {
      const bf16x4 v4 = *reinterpret_cast<const bf16x4*>(cr + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = (float)v4[j];
        if (v > best) { best = v; bc = p * cq + c + j; }
      }
    }
  } else {
    for (int c = 0; c < cq; ++c) {
      const float v = (float)cr[c];
      if (v > best) { best = v; bc = p * cq + c; }
    }
  }
#pragma unroll
  for (int o = 1; o <= 2; o <<= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oc = __shfl_xor(bc, o, 64);
    if (ob > best || (ob == best && oc < bc)) { best = ob; bc = oc; }
  }
  if (p == 0) {
    scores[i] = sigmoidf_(best);
    cls[i] = bc;
  }
}

// IoU(a, b) > thr, without the divide: inter > thr * max(union, 1e-9)
__device__ __forceinline__ bool iou_gt(float ax1, float ay1, float ax2, float ay2, float bx1,
                                       float by1, float bx2, float by2, float thr) {
  const float iw = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f);
  const float ih = fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float inter = iw * ih;
  const float aa = (ax2 - ax1) * (ay2 - ay1);
  const float ab = (bx2 - bx1) * (by2 - by1);
  return inter > thr * fmaxf(aa + ab - inter, 1e-9f);
}

constexpr int kNmsWaves = 16;  // 1024 threads: the slowest image sets the kernel time (one workgroup per image)
constexpr int kSel = 768;      // top-set target size (rank-sortable: <= kRankSortMax)
constexpr int kSelMax = 2048;  // top-set capacity (a wider threshold bin -> full sort)
constexpr int kBins = 2048;    // score-bit histogram bins
constexpr int kRankSortMax = 1024;  // rank sort up to here (<= 2 keys per thread), bitonic above

__global__ __launch_bounds__(64 * kNmsWaves) void nms_kernel(const float* __restrict__ boxes,
                                                  const float* __restrict__ scores,
                                                  const int* __restrict__ cls, int A,
                                                  float conf, float iou_thr, int max_det,
                                                  float* __restrict__ out,
                                                  int* __restrict__ count, int diag) {
  __shared__ __attribute__((aligned(16))) unsigned long long keys[kMaxCand];
  __shared__ __attribute__((aligned(16))) float kept[4 * 320];
  __shared__ int kept_c[320];
  __shared__ unsigned long long supp[kNmsWaves];
  __shared__ unsigned long long rowp[kNmsWaves][64];
  __shared__ unsigned long long sel[kSelMax];  // the top set; its first 8 KB hold the histogram first
  __shared__ int s_nk;
  __shared__ int ncand;
  __shared__ int s_n2, s_T, s_nsel;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const unsigned long long t_start = (diag & 4) ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const float* sc = scores + (long long)n * A;
  // wave-aggregated compaction: one LDS atomic per wave and pass (popcount of the ballot)
  // instead of one per candidate -- with random-init heads nearly all 8400 anchors pass
  // conf, and 8400 atomics on one LDS word serialise (key order does not matter: sorted next)
  // All of this thread's scores are loaded up front (A <= kMaxCand: at most kIt per thread),
  // so the HBM latency is paid once, not once per pass of the ballot loop below.
  constexpr int kIt = kMaxCand / (64 * kNmsWaves);
  auto compact = [&]() __attribute__((always_inline)) {
    if (tid == 0) ncand = 0;
    __syncthreads();
    const int ln = tid & 63;
    float sv[kIt];
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      const int a = i * 64 * kNmsWaves + tid;
      sv[i] = a < A ? sc[a] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kIt; ++i) {  // uniform trip count: whole waves ballot
      if (i * 64 * kNmsWaves >= A) break;
      const int a = i * 64 * kNmsWaves + tid;
      const float s = sv[i];
      const bool take = a < A && s > conf;
      const unsigned long long m = __ballot(take);
      int base = 0;
      if (ln == 0 && m) base = atomicAdd(&ncand, (int)__popcll(m));
      base = __shfl(base, 0);
      if (take) {
        const int slot = base + (int)__popcll(m & ((1ull << ln) - 1ull));
        if (slot < kMaxCand)
          keys[slot] = ((unsigned long long)__float_as_uint(s) << 32) | (0xFFFFFFFFu - (unsigned)a);
      }
    }
    __syncthreads();
  };
  compact();
  const int cnt = min(ncand, kMaxCand);
  // diag bit 2: per-phase wall-clock stamps (s_memrealtime, 100 MHz) -> the image's output rows
  unsigned long long t_ph[4] = {t_start, 0, 0, 0};
  // bitonic sort of K[0, n) (padded with zero keys to a power of two), descending
  auto bitonic = [&](unsigned long long* K, int n) __attribute__((always_inline)) {
    int P = 64;
    while (P < n) P <<= 1;
    for (int i = n + tid; i < P; i += blockDim.x) K[i] = 0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P; i += blockDim.x) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const unsigned long long a = K[i], b = K[ixj];
            const bool desc = (i & k) == 0;
            if (desc ? (a < b) : (a > b)) {
              K[i] = b;
              K[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    }
  };
  // rank sort: each thread counts the keys above its own with broadcast LDS reads and writes
  // its key to that slot -- one pass, one barrier.  Keys are unique (the index is in the low
  // word), so the ranks are a permutation.
  auto rank_sort = [&](const unsigned long long* src, unsigned long long* dst, int n)
      __attribute__((always_inline)) {
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
      const int i = i0 + tid;
      const unsigned long long key = i < n ? src[i] : 0ull;
      int r = 0;
      for (int j = 0; j < n; ++j) r += src[j] > key;
      if (i < n) dst[r] = key;
    }
    __syncthreads();
  };
  // Top-set selection.  Greedy NMS reads candidates in score order and usually reaches
  // max_det long before the end of the list, so only the head needs sorting: a 2048-bin
  // histogram of the score bits gives the lowest bin T whose suffix holds >= kSel keys;
  // keys in bins >= T are exactly the top keys of the total (score, index) order (equal
  // scores share a bin).  They are compacted and sorted alone (<= 2048 instead of up to
  // 16384 keys: the full sort was most of the 179 us the b192 step spent in NMS,
  // profiles/r3_v7_yolov8n_b192_op_roofline.md row 64); the rest is sorted only if the top
  // set runs out before max_det.
  const unsigned lo = conf > 0.f ? __float_as_uint(conf) : 0u;
  const unsigned span = 0x3F800000u - lo;  // scores are sigmoids: (conf, 1]
  const int shift = max(0, 32 - __clz((int)(span | 1u)) - 11);
  auto bin_of = [&](unsigned long long key) __attribute__((always_inline)) {
    return min(kBins - 1, (int)((((unsigned)(key >> 32)) - lo) >> shift));
  };
  unsigned long long* K = keys;
  int nsel = cnt;
  bool sorted = false;  // the top set already came out of its sort (bucket or fallback)
  bool clobbered = false;  // keys[] now holds the sorted top set, not all candidates
  int rest_T = -1;         // threshold bin of the top set (the rest = keys below it)
  if (cnt > kSel) {
    int* hist = reinterpret_cast<int*>(sel);
    for (int i = tid; i < kBins; i += blockDim.x) hist[i] = 0;
    if (tid == 0) s_n2 = 0;
    __syncthreads();
    for (int i = tid; i < cnt; i += blockDim.x) atomicAdd(&hist[bin_of(keys[i])], 1);
    __syncthreads();
    if (tid < 64) {  // wave 0: lane L owns bins [32 L, 32 L + 32)
      int sum = 0;
      for (int b = 0; b < 32; ++b) sum += hist[tid * 32 + b];
      int suf = sum;  // suffix sum over lanes >= L
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_down(suf, off);
        if (tid + off < 64) suf += v;
      }
      const unsigned long long hit = __ballot(suf >= kSel);
      const int lt = 63 - __clzll((long long)hit);  // highest lane whose suffix reaches kSel
      if (tid == lt) {
        int acc = suf - sum, T = tid * 32;
        for (int b = 31; b >= 0; --b) {
          acc += hist[tid * 32 + b];
          if (acc >= kSel) {
            T = tid * 32 + b;
            break;
          }
        }
        s_T = T;
        s_nsel = acc;
      }
    }
    __syncthreads();
    // Bucket sort of the top set (the 2048-key bitonic network was 43 of
    // the ~100 us a crowded image spends in NMS, profiles/r4_v5_nms_probe.txt).  The
    // histogram already orders the keys by bin; each top-set bin gets a descending slot range
    // (suffix sums of its counts), keys are scattered into their bin's range with one LDS
    // atomic each, and only keys that share a bin are ranked against each other.  The bin
    // cursors live in the free tail of keys[] (cnt <= kMaxCand - kBins / 2 -- the top set
    // of a 640x640 image has at most 8400 candidates); a bin with more than kBinRankMax keys
    // (a degenerate score pile-up) falls back to the bitonic network.
    constexpr int kBinRankMax = 64;
    int* cur = reinterpret_cast<int*>(keys + (kMaxCand - kBins / 2));
    // measured level-to-slower than the bitonic network on the bench's decode output (101.3
    // vs 96.7 us per b256 slice, profiles/r5_v5_nms_probe_bucket.txt: the kernel is set by
    // its slowest image, whose compaction and suppression dominate), so opt-in (diag bit 3)
    const bool bucket = s_nsel <= kSelMax && cnt <= kMaxCand - kBins / 2 && (diag & 8);
    if (bucket) {
      const int T = s_T;
      if (tid < 64) {  // wave 0: lane L owns bins [32 L, 32 L + 32); descending exclusive sums
        int sum = 0, mx = 0;
        for (int b = 0; b < 32; ++b) {
          const int bb = tid * 32 + b;
          const int c = bb >= T ? hist[bb] : 0;
          sum += c;
          mx = max(mx, c);
        }
        int suf = sum;  // inclusive suffix over lanes >= L
        for (int off = 1; off < 64; off <<= 1) {
          const int v = __shfl_down(suf, off);
          if (tid + off < 64) suf += v;
        }
        int run = suf - sum;  // slots taken by the bins above this lane's
        for (int b = 31; b >= 0; --b) {
          const int bb = tid * 32 + b;
          cur[bb] = run;  // start of bin bb (the scatter advances it to the bin's end)
          run += bb >= T ? hist[bb] : 0;
        }
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off));
        if (tid == 0) s_n2 = mx;
      }
      __syncthreads();
      const int binmax = s_n2;
      __syncthreads();  // every thread has read s_n2 before the fallback below reuses it
      if (binmax <= kBinRankMax) {
        for (int i = tid; i < cnt; i += blockDim.x) {
          const unsigned long long key = keys[i];
          const int b = bin_of(key);
          if (b >= T) sel[atomicAdd(&cur[b], 1)] = key;
        }
        __syncthreads();
        // rank inside the bin: cur[b] is now the bin's end, its start the end of bin b + 1
        const int ns = s_nsel;
        unsigned long long mine[kSelMax / (64 * kNmsWaves)];
        int dst[kSelMax / (64 * kNmsWaves)];
#pragma unroll
        for (int k = 0; k < kSelMax / (64 * kNmsWaves); ++k) {
          const int i = tid + k * 64 * kNmsWaves;
          dst[k] = -1;
          if (i < ns) {
            const unsigned long long key = sel[i];
            const int b = bin_of(key);
            const int lo0 = b + 1 < kBins ? cur[b + 1] : 0, hi0 = cur[b];
            int r = 0;
            for (int j = lo0; j < hi0; ++j) r += sel[j] > key;
            mine[k] = key;
            dst[k] = lo0 + r;
          }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSelMax / (64 * kNmsWaves); ++k)
          if (dst[k] >= 0) sel[dst[k]] = mine[k];
        __syncthreads();
        K = sel;
        nsel = ns;
      }
    }
    if (s_nsel <= kSelMax && K == keys) {
      const int T = s_T;
      rest_T = T;
      const int ln = tid & 63;
      if (tid == 0) s_n2 = 0;
      __syncthreads();
      for (int i0 = 0; i0 < cnt; i0 += blockDim.x) {  // wave-aggregated, as the compaction
        const int i = i0 + tid;
        const unsigned long long key = i < cnt ? keys[i] : 0ull;
        const bool take = i < cnt && bin_of(key) >= T;
        const unsigned long long m = __ballot(take);
        int base = 0;
        if (ln == 0 && m) base = atomicAdd(&s_n2, (int)__popcll(m));
        base = __shfl(base, 0);
        if (take) sel[base + (int)__popcll(m & ((1ull << ln) - 1ull))] = key;
      }
      __syncthreads();
      K = sel;
      nsel = s_n2;
      if (!(diag & 2)) {
        if (nsel <= kRankSortMax) {
          // one rank pass into keys[0, nsel) instead of the bitonic network's log^2
          // barrier-separated stages (a 1382-candidate image: ~28 us of bitonic, r5 probe);
          // keys[] is rebuilt from the scores if the top set runs out (fallback below)
          rank_sort(sel, keys, nsel);
          K = keys;
          clobbered = true;
        } else {
          bitonic(K, nsel);
        }
      }
      sorted = true;
    }
  }
  if (diag & 4) t_ph[1] = __builtin_amdgcn_s_memrealtime();
  // Small sets (random-init heads: ~100 candidates per image) are sorted by rank: each thread
  // counts the keys above its own with broadcast LDS reads and writes its key to that slot --
  // one pass and one barrier instead of the bitonic network's log^2 barrier-separated stages
  // (28 at 128 keys, 42 us per image measured: profiles/r4_v5_nms_probe.txt).  Keys are unique
  // (the index is in the low word), so the ranks are a permutation.
  if (K == sel && cnt > kSel) sorted = true;  // the bucket sort above
  if (!(diag & 2) && !sorted) {
    if (K == keys && nsel <= kRankSortMax) {
      rank_sort(keys, sel, nsel);
      K = sel;
    } else {
      bitonic(K, nsel);  // diag bit 1: no top-set sort (timing only)
    }
  }
  if (diag & 4) t_ph[2] = __builtin_amdgcn_s_memrealtime();
  float* o = out + (long long)n * max_det * 6;
  const int lane = tid & 63, wv = tid >> 6;
  const float* bx = boxes + (long long)n * A * 4;
  const int* cl = cls + (long long)n * A;
  int nk = 0;
  // greedy suppression over the sorted K[from, to), continuing the kept list
  auto greedy = [&](const unsigned long long* K, int from, int to) __attribute__((always_inline)) {
    // the chunk's class / box gathers (random global reads) are issued one chunk ahead, so
    // their latency hides under the previous chunk's IoU tests and barriers (the images
    // with crowded candidate sets walk ~20 chunks: 58 us of suppression at b192,
    // profiles/r4_v5_nms_probe.txt)
    int pc = -1;
    float4 praw = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned long long pkey = 0ull;
    auto fetch = [&](int b) __attribute__((always_inline)) {
      const int ci = b + lane;
      pc = -1;
      if (ci < to) {
        pkey = K[ci];
        const int idx = (int)(0xFFFFFFFFu - (unsigned)(pkey & 0xFFFFFFFFull));
        pc = cl[idx];
        praw = *reinterpret_cast<const float4*>(bx + idx * 4);
      }
    };
    if (from < to) fetch(from);
    for (int base = from; base < to && nk < max_det; base += 64) {
      // every wave holds the same 64 candidates (lane = candidate)
      const int ci = base + lane;
      const bool valid = ci < to;
      float x1 = 0, y1 = 0, x2 = 0, y2 = 0, s = 0;
      const float4 raw = valid ? praw : make_float4(0.f, 0.f, 0.f, 0.f);
      const int c = valid ? pc : -1;
      if (valid) s = __uint_as_float((unsigned)(pkey >> 32));
      if (base + 64 < to) fetch(base + 64);
      if (valid) {
        const float off = (float)c * kMaxWH;
        x1 = raw.x + off;
        y1 = raw.y + off;
        x2 = raw.z + off;
        y2 = raw.w + off;
      }
      // 1. against the kept list, split over the NMS_WAVES waves (j = wv, wv + W, ...):
      // independent LDS reads, no early exit, so the loads pipeline instead of one
      // LDS round trip per kept box (the one-wave version was 290 us at batch 64 on
      // images with ~1000 candidates).  Other classes never overlap: compare class first.
      bool sup = false;
      for (int j = wv; j < nk; j += kNmsWaves) {
        const float4 kb = *reinterpret_cast<const float4*>(kept + 4 * j);
        sup |= kept_c[j] == c && iou_gt(x1, y1, x2, y2, kb.x, kb.y, kb.z, kb.w, iou_thr);
      }
      // 2. in-chunk: which LATER lanes this lane's box suppresses, also split over the
      // waves (j = wv, wv + W, ...); j is wave-uniform, so the other box comes from
      // v_readlane (scalar broadcast), not an LDS-routed shuffle
      const int lim = min(64, to - base);
      unsigned long long row = 0ull;
      for (int j = wv; j < lim; j += kNmsWaves) {
        const float bx1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x1), j));
        const float by1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, y1), j));
        const float bx2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x2), j));
        const float by2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, y2), j));
        if (j > lane && iou_gt(x1, y1, x2, y2, bx1, by1, bx2, by2, iou_thr)) row |= 1ull << j;
      }
      rowp[wv][lane] = row;
      const unsigned long long sb = __ballot(sup);
      if (lane == 0) supp[wv] = sb;
      __syncthreads();
      if (wv == 0) {
        unsigned long long dead = 0ull;
        row = 0ull;
#pragma unroll
        for (int w = 0; w < kNmsWaves; ++w) {
          dead |= supp[w];
          row |= rowp[w][lane];
        }
        const bool alive = valid && !((dead >> lane) & 1ull);
        unsigned long long todo = __ballot(alive), live = 0ull;
        const unsigned rlo = (unsigned)row, rhi = (unsigned)(row >> 32);
        // survivors in rank order: only the set bits are visited (a crowded chunk behind a
        // full kept list has few), each one striking the later boxes it overlaps
        while (todo) {
          const int j = __builtin_ctzll(todo);
          const unsigned long long rj =
              ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)rhi, j) << 32) |
              (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)rlo, j);
          live |= 1ull << j;
          todo &= ~(rj | (1ull << j));
        }
        // 3. append survivors in rank order
        const bool keep = (live >> lane) & 1ull;
        const int rank = __popcll(live & ((1ull << lane) - 1ull));
        const int pos = nk + rank;
        if (keep && pos < max_det) {
          *reinterpret_cast<float4*>(kept + 4 * pos) = make_float4(x1, y1, x2, y2);
          kept_c[pos] = c;
          float* r = o + pos * 6;  // original (un-offset) coordinates: exact, no fp32 cancellation
          r[0] = raw.x;
          r[1] = raw.y;
          r[2] = raw.z;
          r[3] = raw.w;
          r[4] = s;
          r[5] = (float)c;
        }
        if (lane == 0) s_nk = min(nk + (int)__popcll(live), max_det);
      }
      __syncthreads();
      nk = s_nk;
    }
  };
  if (!(diag & 1)) greedy(K, 0, nsel);  // diag bit 0: no suppression (timing only)
  else nk = max_det;
  if (nk < max_det && nsel < cnt) {
    // the top set ran out: sort everything (its first nsel keys are the top set again,
    // in the same order) and continue after them; the rank-sorted top set overwrote the
    // head of keys[], so the candidates are compacted from the scores again first (the
    // same set: compaction order does not matter, the sort fixes it)
    if (clobbered) compact();
    const int nrest = cnt - nsel;
    if (rest_T >= 0 && nrest <= kRankSortMax && !(diag & 2)) {
      // only the keys BELOW the top set still need an order: compact them (bin < T) into
      // sel, rank-sort them into keys[0, nrest) and continue the greedy there -- they all
      // rank below every top-set key, so this is the full sort's tail (the crowded image's
      // bitonic network over every candidate was ~25 us of the slowest image, r6 probe)
      const int ln = tid & 63;
      if (tid == 0) s_n2 = 0;
      __syncthreads();
      for (int i0 = 0; i0 < cnt; i0 += blockDim.x) {
        const int i = i0 + tid;
        const unsigned long long key = i < cnt ? keys[i] : 0ull;
        const bool take = i < cnt && bin_of(key) < rest_T;
        const unsigned long long m = __ballot(take);
        int base = 0;
        if (ln == 0 && m) base = atomicAdd(&s_n2, (int)__popcll(m));
        base = __shfl(base, 0);
        if (take) sel[base + (int)__popcll(m & ((1ull << ln) - 1ull))] = key;
      }
      __syncthreads();
      rank_sort(sel, keys, nrest);
      greedy(keys, 0, nrest);
    } else {
      bitonic(keys, cnt);
      greedy(keys, nsel, cnt);
    }
  }
  for (int i = nk * 6 + tid; i < max_det * 6; i += blockDim.x) o[i] = 0.f;
  if (tid == 0) count[n] = nk;
  if (diag & 4) {
    t_ph[3] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (tid == 0) {  // phase durations in 10-ns ticks: compaction+select, sort, suppression
      o[0] = (float)(t_ph[1] - t_ph[0]);
      o[1] = (float)(t_ph[2] - t_ph[1]);
      o[2] = (float)(t_ph[3] - t_ph[2]);
    }
  }
}

}  // namespace
}  // namespace kvedge

using namespace kvedge;

extern "C" int kv_yolo_decode(const void* f0, const void* f1, const void* f2, int h0, int w0,
                              int h1, int w1, int h2, int w2, int s0, int s1, int s2, int N,
                              int nc, float* boxes, float* scores, int* cls, hipStream_t s) {
  if (nc % 8) return -1;
  const int ch = 4 * kRegMax + nc;
  const unsigned lds = (unsigned)(kDecAnch * (ch + 8) * 2);
  if (lds > 64 * 1024) return -2;
  auto nb = [](int a) { return (a + kDecAnch - 1) / kDecAnch; };
  const long long g = (long long)N * (nb(h0 * w0) + nb(h1 * w1) + nb(h2 * w2));
  if (g <= 0) return 0;
  if (h0 * w0 >= 65536 || h1 * w1 >= 65536 || h2 * w2 >= 65536) return -3;
  hipLaunchKernelGGL(nc == 80 ? yolo_decode_kernel<80> : yolo_decode_kernel<0>, dim3((unsigned)g),
                     dim3(256), lds, s, (const bf16*)f0,
                     (const bf16*)f1, (const bf16*)f2, h0, w0, h1, w1, h2, w2, s0, s1, s2, N, nc,
                     boxes, scores, cls);
  return hipGetLastError() == hipSuccess ? 0 : -100;
}

extern "C" int kv_nms(const float* boxes, const float* scores, const int* cls, int N, int A,
                      float conf_thres, float iou_thres, int max_det, float* out, int* count,
                      hipStream_t s) {
  if (max_det > 300 || max_det <= 0 || A > kMaxCand) return -1;
  if (N <= 0) return 0;
  // KVEDGE_NMS_DIAG (timing experiments only; outputs wrong): bit 0 skips the greedy
  // suppression, bit 1 the top-set sort; bit 2 writes per-phase durations into each image's
  // first output row; bit 3 (outputs right) sorts the top set with the histogram bucket sort
  // instead of the bitonic network (A/B)
  const char* dg = getenv("KVEDGE_NMS_DIAG");
  hipLaunchKernelGGL(nms_kernel, dim3(N), dim3(64 * kNmsWaves), 0, s, boxes, scores, cls, A, conf_thres,
                     iou_thres, max_det, out, count, dg ? atoi(dg) : 0);
  return hipGetLastError() == hipSuccess ? 0 : -100;
}
