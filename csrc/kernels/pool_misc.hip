// K4 (BN fallback), K5 (max pool, SPPF), K6 (global avg pool), K7 (softmax),
// K8 (nearest 2x upsample into a concat slice), K11 (synthetic frames),
// K12 (uint8 -> normalized bf16 NHWC4).  SURVEY.md §2.5.
//
// All of these are HBM-bound streaming ops: every lane moves 16 B (8 bf16
// channels) per access (cdna_hip_programming.md Guideline 13), grids are capped
// at 256 CUs x 8 blocks and grid-stride the rest (Guideline 11).
#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kBlock = 256;
inline unsigned grid_for(long long work) {
  long long g = (work + kBlock - 1) / kBlock;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

__device__ __forceinline__ bf16x8 max8(bf16x8 a, bf16x8 b) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = f2bf(fmaxf((float)a[i], (float)b[i]));
  return r;
}

// ---- K5 max pool ----------------------------------------------------------
__global__ __launch_bounds__(kBlock) void maxpool_kernel(const bf16* __restrict__ x,
                                                         bf16* __restrict__ y, int N, int H,
                                                         int W, int C, int ldx, int x_coff,
                                                         int ldy, int y_coff, int k, int stride,
                                                         int pad, int Ho, int Wo) {
  const int C8 = C / 8;
  const long long total = (long long)N * Ho * Wo * C8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long long pix = i / C8;
    const int wo = (int)(pix % Wo);
    pix /= Wo;
    const int ho = (int)(pix % Ho);
    const int n = (int)(pix / Ho);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    const int h0 = ho * stride - pad, w0 = wo * stride - pad;
    for (int r = 0; r < k; ++r) {
      const int hi = h0 + r;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int s = 0; s < k; ++s) {
        const int wi = w0 + s;
        if ((unsigned)wi >= (unsigned)W) continue;
        const bf16x8 v =
            *reinterpret_cast<const bf16x8*>(x + ((long long)(n * H + hi) * W + wi) * ldx + x_coff + c8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], (float)v[j]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(m[j]);
    *reinterpret_cast<bf16x8*>(y + ((long long)(n * Ho + ho) * Wo + wo) * ldy + y_coff + c8 * 8) = o;
  }
}

// ---- K5b SPPF: y1 = mp5(x), y2 = mp5(y1) = mp9(x), y3 = mp13(x) ------------
// (Composition of stride-1 max filters with -inf padding is the max over the summed
// window, so chaining gives exactly mp5 / mp9 / mp13 of x.)
// Separable, LDS-resident, chained: one workgroup per (image, 16-channel group) runs the
// three 5x5 pools as they are defined (y_k = mp5(y_{k-1})), each as a radius-2 row max
// into LDS image t and a radius-2 column max back into image a, which then holds y_k and
// is also written to its global slice.  Two LDS images (not four: x plus the three
// radius-2/4/6 row-max images of the previous version) -> 2.5x the workgroups per CU, and
// 5 + 5 reads per output per stage instead of 13 + (5 + 9 + 13) for the whole pass.
constexpr int kSppfCg = 16;  // channels per workgroup
typedef short sppf_i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned sppf_key2(unsigned w) {
  const sppf_i16x2 x = __builtin_bit_cast(sppf_i16x2, w);
  return __builtin_bit_cast(unsigned, x ^ ((x >> 15) & (short)0x7fff));
}
__device__ __forceinline__ uint4 sppf_key4(uint4 v) {
  return make_uint4(sppf_key2(v.x), sppf_key2(v.y), sppf_key2(v.z), sppf_key2(v.w));
}
__device__ __forceinline__ unsigned sppf_max2(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(sppf_i16x2, a),
                                                                __builtin_bit_cast(sppf_i16x2, b)));
}
__device__ __forceinline__ uint4 sppf_max4(uint4 a, uint4 b) {
  return make_uint4(sppf_max2(a.x, b.x), sppf_max2(a.y, b.y), sppf_max2(a.z, b.z), sppf_max2(a.w, b.w));
}
__global__ __launch_bounds__(kBlock) void sppf_kernel(bf16* __restrict__ buf, int N, int H,
                                                      int W, int C) {
  extern __shared__ __attribute__((aligned(16))) bf16 sp[];  // 2 x [H*W][16]
  const int HW = H * W;
  const int ncg = C / kSppfCg;
  const int n = blockIdx.x / ncg, cg = blockIdx.x - n * ncg;
  const int ld = 4 * C;
  bf16* a = sp;
  bf16* t = sp + HW * kSppfCg;
  bf16* base = buf + (long long)n * HW * ld + cg * kSppfCg;
  for (int q = threadIdx.x; q < HW * 2; q += kBlock) {  // 2 x 16 B per pixel
    const int pix = q >> 1, hf = q & 1;
    *reinterpret_cast<uint4*>(a + pix * kSppfCg + hf * 8) =
        sppf_key4(*reinterpret_cast<const uint4*>(base + (long long)pix * ld + hf * 8));
  }
  // Max on order-preserving int16 keys, two channels per v_pk_max_i16: key(x) = x ^ 0x7fff
  // for negative bf16 x (sign set: the magnitude bits flipped, so a larger magnitude orders
  // lower), x otherwise.  The map is its own inverse and exact; the previous float path spent
  // 8 converts + 8 fmax per 16-B read.  x is stored as keys.  Out-of-image taps are clamped
  // onto in-window pixels (a duplicate never changes a max): the tap loops have no branches.
  for (int k = 1; k <= 3; ++k) {
    __syncthreads();  // a complete (keys of x or y_{k-1})
    for (int q = threadIdx.x; q < HW * 2; q += kBlock) {  // t = row max, radius 2
      const int pix = q >> 1, hf = q & 1;
      const int y = pix / W, x = pix - y * W;
      uint4 m = *reinterpret_cast<const uint4*>(a + pix * kSppfCg + hf * 8);
#pragma unroll
      for (int dx = -2; dx <= 2; ++dx) {
        if (dx == 0) continue;
        const int xi = min(max(x + dx, 0), W - 1);
        m = sppf_max4(m, *reinterpret_cast<const uint4*>(a + (y * W + xi) * kSppfCg + hf * 8));
      }
      *reinterpret_cast<uint4*>(t + pix * kSppfCg + hf * 8) = m;
    }
    __syncthreads();  // t complete; a no longer read
    for (int q = threadIdx.x; q < HW * 2; q += kBlock) {  // a = y_k = column max of t
      const int pix = q >> 1, hf = q & 1;
      const int y = pix / W, x = pix - y * W;
      uint4 m = *reinterpret_cast<const uint4*>(t + pix * kSppfCg + hf * 8);
#pragma unroll
      for (int dy = -2; dy <= 2; ++dy) {
        if (dy == 0) continue;
        const int yi = min(max(y + dy, 0), H - 1);
        m = sppf_max4(m, *reinterpret_cast<const uint4*>(t + (yi * W + x) * kSppfCg + hf * 8));
      }
      if (k < 3) *reinterpret_cast<uint4*>(a + pix * kSppfCg + hf * 8) = m;
      *reinterpret_cast<uint4*>(base + (long long)pix * ld + k * C + hf * 8) = sppf_key4(m);
    }
  }
}

// ---- K6 global average pool: one thread per (n, 8 channels) ----------------
// 8 lanes per output chunk (8 channels of one image), each summing every 8th pixel, then a
// 3-step xor-shuffle reduction.  One lane per chunk walking all HW pixels serialised 49
// dependent-address loads per lane: at batch 1 (256 chunks, one workgroup) that was 15 us,
// the longest non-conv kernel of the edge step (profiles/r3_v7_resnet50_b1_forward_splitk.md).
__global__ __launch_bounds__(kBlock) void avgpool_kernel(const bf16* __restrict__ x,
                                                         bf16* __restrict__ y, int N, int HW,
                                                         int C) {
  const int C8 = C / 8;
  const long long total = (long long)N * C8 * 8;
  const float inv = 1.0f / (float)HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {  // total % 64 == 0: whole waves iterate
    const int part = (int)(i & 7);
    const long long o = i >> 3;
    const int c8 = (int)(o % C8);
    const int n = (int)(o / C8);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16* p = x + (long long)n * HW * C + c8 * 8;
    for (int q = part; q < HW; q += 8) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(p + (long long)q * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], off);
    if (part == 0) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = f2bf(s[j] * inv);
      *reinterpret_cast<bf16x8*>(y + (long long)n * C + c8 * 8) = r;
    }
  }
}

// ---- K6+K1 fused head for edge batches: logits = fc(global_avgpool(x)) -----------------
// At batch 1-16 the classifier is a GEMV (K = 2048, N = 1000): as a tiled GEMM it was a
// 16-32-workgroup launch walking 32 K steps (~13 us), after a separate pooling launch.  Here
// workgroup (column block of 64, image) pools the image's C channels into LDS (rounded to
// bf16, as the pooling kernel stores them), then each of its 8 waves dots 8 weight rows with
// it: 16-B weight loads, a wave reduction per column.  One launch, weights read once per
// image.  Every column block needs the whole pooled vector, so the image is pooled once per
// block: 16 blocks at ncls = 1000 (was 32 with 32-column blocks), each splitting
// the HW pixels of a channel chunk over kPfSplit threads so the pooling pass is
// ceil(HW / kPfSplit) loads deep instead of HW.
constexpr int kPfThreads = 512, kPfCols = 64;
__global__ __launch_bounds__(kPfThreads) void pooled_fc_kernel(const bf16* __restrict__ x, int HW,
                                                               int C, const bf16* __restrict__ w,
                                                               int ldw, const float* __restrict__ bias,
                                                               bf16* __restrict__ y, int ncls,
                                                               int split) {
  extern __shared__ float pf_smem[];  // [split][C] partial sums, then [C] pooled (slot 0)
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bf16* xb = x + (size_t)b * HW * C;
  const int C8 = C / 8;
  for (int it = tid; it < C8 * split; it += kPfThreads) {
    const int c8 = it % C8, part = it / C8;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
    for (int q = part; q < HW; q += split) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(xb + (size_t)q * C + c8 * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += (float)v[e];
    }
    float4* dst = reinterpret_cast<float4*>(pf_smem + part * C + c8 * 8);
    dst[0] = make_float4(s[0], s[1], s[2], s[3]);
    dst[1] = make_float4(s[4], s[5], s[6], s[7]);
  }
  __syncthreads();
  const float inv = 1.0f / (float)HW;
  for (int c = tid; c < C; c += kPfThreads) {
    float t = pf_smem[c];
    for (int part = 1; part < split; ++part) t += pf_smem[part * C + c];
    pf_smem[c] = (float)f2bf(t * inv);
  }
  __syncthreads();
  const float* pooled = pf_smem;
  for (int j = 0; j < kPfCols / 8; ++j) {
    const int n = blockIdx.x * kPfCols + wv * 8 + j;  // wave-uniform
    if (n >= ncls) break;
    const bf16* wr = w + (size_t)n * ldw;
    float acc = 0.f;
    for (int k = lane * 8; k < C; k += 512) {
      const bf16x8 wk = *reinterpret_cast<const bf16x8*>(wr + k);
      const float4 p0 = *reinterpret_cast<const float4*>(pooled + k);  // ds_read_b128
      const float4 p1 = *reinterpret_cast<const float4*>(pooled + k + 4);
      acc += (float)wk[0] * p0.x + (float)wk[1] * p0.y + (float)wk[2] * p0.z + (float)wk[3] * p0.w;
      acc += (float)wk[4] * p1.x + (float)wk[5] * p1.y + (float)wk[6] * p1.z + (float)wk[7] * p1.w;
    }
    acc = wave_sum(acc);
    if (lane == 0) y[(size_t)b * ncls + n] = f2bf(acc + (bias ? bias[n] : 0.f));
  }
}

// ---- K7 row softmax + argmax: one wave64 per row ---------------------------
__global__ __launch_bounds__(kBlock) void softmax_kernel(const bf16* __restrict__ x,
                                                         float* __restrict__ y,
                                                         int64_t* __restrict__ amax, int rows,
                                                         int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* xr = x + (long long)row * cols;
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  if (cols <= 1024 && (cols & 7) == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
    // register-resident row (ResNet-50's 1000 classes): each lane loads 16 contiguous
    // columns as two 16-B vectors ONCE; max / sum / store run from registers.  The strided
    // loop below reads the row three times with 2-B loads: ~10 us at batch 1, a whole
    // edge-batch step's worth of per-kernel floor
    float v[16];
    const int c0 = lane * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = c0 + 8 * h;  // a chunk of 8 is either all in range or all past cols
      bf16x8 q = {};
      if (c < cols) q = *reinterpret_cast<const bf16x8*>(xr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[8 * h + e] = c < cols ? (float)q[e] : -INFINITY;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (v[i] > mx) { mx = v[i]; arg = c0 + i; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      v[i] = __expf(v[i] - mx);  // exp(-inf) = 0 past cols
      sum += v[i];
    }
    const float inv = 1.0f / wave_sum(sum);
    float* yr = y + (long long)row * cols;
#pragma unroll
    for (int h = 0; h < 4; ++h)
      if (c0 + 4 * h < cols)
        *reinterpret_cast<float4*>(yr + c0 + 4 * h) =
            make_float4(v[4 * h] * inv, v[4 * h + 1] * inv, v[4 * h + 2] * inv, v[4 * h + 3] * inv);
    if (lane == 0 && amax) amax[row] = arg;
    return;
  }
  for (int c = lane; c < cols; c += 64) {
    const float v = (float)xr[c];
    if (v > mx) { mx = v; arg = c; }
  }
  // wave argmax (ties -> lowest index)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  float sum = 0.f;
  for (int c = lane; c < cols; c += 64) sum += __expf((float)xr[c] - mx);
  sum = wave_sum(sum);
  const float inv = 1.0f / sum;
  float* yr = y + (long long)row * cols;
  for (int c = lane; c < cols; c += 64) yr[c] = __expf((float)xr[c] - mx) * inv;
  if (lane == 0 && amax) amax[row] = arg;
}

// ---- K8 nearest 2x upsample into a channel slice ---------------------------
// One thread per SOURCE 16-B vector: one load, four stores (the 2x2 block it
// feeds).  32-bit index math (host checks N*H*W*C/8 < 2^31); the grid is sized to
// the work, so each thread runs its body at most a few times.
__global__ __launch_bounds__(kBlock) void upsample2x_kernel(const bf16* __restrict__ x,
                                                            bf16* __restrict__ y, int N, int H,
                                                            int W, int C, int ldx, int x_coff,
                                                            int ldy, int y_coff) {
  const int C8 = C >> 3;
  const int total = N * H * W * C8;
  const int Wo = 2 * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    const int pix = i / C8;              // (n*H + h)*W + w
    const int w = pix % W;
    const int nh = pix / W;              // n*H + h
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long long)pix * ldx + x_coff + c8 * 8);
    // output row n*Ho + 2h = 2*nh, columns 2w and 2w+1
    bf16* r0 = y + ((long long)(2 * nh) * Wo + 2 * w) * ldy + y_coff + c8 * 8;
    bf16* r1 = r0 + (long long)Wo * ldy;
    *reinterpret_cast<bf16x8*>(r0) = v;
    *reinterpret_cast<bf16x8*>(r0 + ldy) = v;
    *reinterpret_cast<bf16x8*>(r1) = v;
    *reinterpret_cast<bf16x8*>(r1 + ldy) = v;
  }
}

// ---- K11 synthetic frames: counter-based hash RNG (splitmix64) --------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Each thread produces 8 bytes.  Frames are a smooth gradient + hashed noise so
// that they are not constant (constant inputs flatter DVFS, guide rule 25).
__device__ __forceinline__ void synth_body(uint8_t* y, long long total8, uint64_t seed,
                                           uint64_t step) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total8;
       i += (long long)gridDim.x * blockDim.x) {
    const uint64_t h = splitmix64(seed ^ (step * 0xD1B54A32D192ED03ull) ^ (uint64_t)i);
    *reinterpret_cast<uint64_t*>(y + i * 8) = h;
  }
}

__global__ __launch_bounds__(kBlock) void synth_kernel(uint8_t* y, long long total8,
                                                       uint64_t seed, uint64_t step) {
  synth_body(y, total8, seed, step);
}

// step[0] = step counter.  bump_done (step has a second slot, step[1] = blocks finished,
// zero between launches): the LAST block to finish advances the counter for the next step
// -- every block read step[0] before it counted itself finished -- so no separate one-thread
// bump launch (~5 us per step at edge batches, where a step is ~50 launches)
__global__ __launch_bounds__(kBlock) void synth_dev_kernel(uint8_t* y, long long total8,
                                                           uint64_t seed, uint64_t* step,
                                                           int bump_done) {
  const uint64_t s = *step;
  synth_body(y, total8, seed, s);
  if (!bump_done) return;
  __syncthreads();  // every thread of this block has read step[0]
  if (threadIdx.x == 0) {
    // relaxed: the only ordering needed is every block's READ of step[0] before the last
    // block's increment, and each block consumed its read before the barrier above.  (An
    // acq_rel ticket writes back the whole L2 per block on gfx950: 19 -> 91 us at b640.)
    const unsigned long long prev = __hip_atomic_fetch_add(
        reinterpret_cast<unsigned long long*>(step + 1), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1ull) {
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(step + 1), 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(step), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void bump_kernel(uint64_t* step) { *step += 1; }

// ---- K12 uint8 NHWC3 -> bf16 NHWC4 normalized ------------------------------
__global__ __launch_bounds__(kBlock) void preprocess_kernel(const uint8_t* __restrict__ x,
                                                            bf16* __restrict__ y, long long pix,
                                                            float m0, float m1, float m2,
                                                            float s0, float s1, float s2) {
  // two pixels per thread: 6 input bytes -> 16 output bytes
  const long long pairs = pix / 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < pairs;
       i += (long long)gridDim.x * blockDim.x) {
    const uint8_t* p = x + i * 6;
    bf16x8 o;
    o[0] = f2bf(((float)p[0] * (1.f / 255.f) - m0) * s0);
    o[1] = f2bf(((float)p[1] * (1.f / 255.f) - m1) * s1);
    o[2] = f2bf(((float)p[2] * (1.f / 255.f) - m2) * s2);
    o[3] = f2bf(0.f);
    o[4] = f2bf(((float)p[3] * (1.f / 255.f) - m0) * s0);
    o[5] = f2bf(((float)p[4] * (1.f / 255.f) - m1) * s1);
    o[6] = f2bf(((float)p[5] * (1.f / 255.f) - m2) * s2);
    o[7] = f2bf(0.f);
    *reinterpret_cast<bf16x8*>(y + i * 8) = o;
  }
}

// ---- K12b uint8 NHWC3 -> bf16 space-to-depth NHWC16 normalized ------------
// y[n, by, bx, (dy*2+dx)*4 + c] = norm(x[n, 2by+dy, 2bx+dx, c]), c == 3 -> 0.
// Turns a stride-2 KxK stem conv into a stride-1 ceil(K/2)-tap conv over 16
// channels (kvedge_amd.models.layers.DeployedConv.stem_s2d): every MFMA k-chunk is
// then one aligned 16-B load and the stem runs on the general implicit-GEMM path.
__global__ __launch_bounds__(kBlock) void preprocess_s2d_kernel(
    const uint8_t* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, float m0,
    float m1, float m2, float s0, float s1, float s2) {
  const int Hs = H / 2, Ws = W / 2;
  const long long total = (long long)N * Hs * Ws;
  const float mm[3] = {m0, m1, m2}, ss[3] = {s0, s1, s2};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int bx = (int)(i % Ws);
    const long long t = i / Ws;
    const int by = (int)(t % Hs);
    const int n = (int)(t / Hs);
    bf16x8 o[2];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const uint8_t* p = x + (((long long)n * H + 2 * by + dy) * W + 2 * bx) * 3;
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          o[dy][dx * 4 + c] = f2bf(((float)p[dx * 3 + c] * (1.f / 255.f) - mm[c]) * ss[c]);
        o[dy][dx * 4 + 3] = f2bf(0.f);
      }
    }
    bf16x8* q = reinterpret_cast<bf16x8*>(y + i * 16);
    q[0] = o[0];
    q[1] = o[1];
  }
}

// ---- K4 fallback BN / affine ------------------------------------------------
__global__ __launch_bounds__(kBlock) void bn_kernel(const bf16* __restrict__ x,
                                                    bf16* __restrict__ y,
                                                    const float* __restrict__ sc,
                                                    const float* __restrict__ sh,
                                                    long long total8, int C, int relu) {
  const int C8 = C / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total8;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)v[j] * sc[c + j] + sh[c + j];
      if (relu) f = fmaxf(f, 0.f);
      o[j] = f2bf(f);
    }
    *reinterpret_cast<bf16x8*>(y + i * 8) = o;
  }
}

}  // namespace
}  // namespace kvedge

using namespace kvedge;

#define KV_CHECK_LAUNCH() return hipGetLastError() == hipSuccess ? 0 : -100

extern "C" int kv_maxpool2d(const void* x, void* y, int N, int H, int W, int C, int ldx,
                            int x_coff, int ldy, int y_coff, int k, int stride, int pad, int Ho,
                            int Wo, hipStream_t s) {
  if (C % 8 || ldx % 8 || x_coff % 8 || ldy % 8 || y_coff % 8) return -1;
  const long long work = (long long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_kernel, dim3(grid_for(work)), dim3(kBlock), 0, s,
                     (const bf16*)x, (bf16*)y, N, H, W, C, ldx, x_coff, ldy, y_coff, k, stride,
                     pad, Ho, Wo);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_sppf_pool(void* buf, int N, int H, int W, int C, hipStream_t s) {
  if (C % kSppfCg) return -1;
  const long long lds = 2LL * H * W * kSppfCg * 2;
  if (lds > 160 * 1024) return -2;  // 2 LDS images of the 16-channel slice must fit
  const long long g = (long long)N * (C / kSppfCg);
  if (g <= 0) return 0;
  hipLaunchKernelGGL(sppf_kernel, dim3((unsigned)g), dim3(kBlock), (unsigned)lds, s, (bf16*)buf, N,
                     H, W, C);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_global_avgpool(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  if (C % 64) return -1;  // whole waves per grid-stride step (the shuffle needs every lane)
  const long long work = (long long)N * (C / 8) * 8;
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_for(work)), dim3(kBlock), 0, s, (const bf16*)x,
                     (bf16*)y, N, HW, C);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_pooled_fc(const void* x, int N, int HW, int C, const void* w, int ldw,
                            const float* bias, void* y, int ncls, hipStream_t s) {
  if (N <= 0 || C % 8 || ldw < C || ldw % 8 || C > 16384) return -1;
  // pixel split of the pooling pass: enough (channel chunk, part) items for the 512 threads,
  // while the [split][C] fp32 partials fit in 64 KB of LDS
  int split = 1;
  while (split < 8 && (C / 8) * split < kPfThreads && (split * 2) * C * 4 <= 65536) split *= 2;
  hipLaunchKernelGGL(pooled_fc_kernel, dim3((unsigned)((ncls + kPfCols - 1) / kPfCols), (unsigned)N),
                     dim3(kPfThreads), (unsigned)(split * C * sizeof(float)), s, (const bf16*)x, HW,
                     C, (const bf16*)w, ldw, bias, (bf16*)y, ncls, split);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_softmax_rows(const void* x, float* y, int64_t* argmax, int rows, int cols,
                               hipStream_t s) {
  const unsigned g = (unsigned)((rows + 3) / 4);
  if (g == 0) return 0;
  hipLaunchKernelGGL(softmax_kernel, dim3(g), dim3(kBlock), 0, s, (const bf16*)x, y, argmax,
                     rows, cols);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_upsample2x(const void* x, void* y, int N, int H, int W, int C, int ldx,
                             int x_coff, int ldy, int y_coff, hipStream_t s) {
  if (C % 8 || ldx % 8 || x_coff % 8 || ldy % 8 || y_coff % 8) return -1;
  const long long work = (long long)N * H * W * (C / 8);
  if (work >= (1ll << 31)) return -1;
  long long g = (work + kBlock - 1) / kBlock;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(upsample2x_kernel, dim3((unsigned)(g < 1 ? 1 : g)), dim3(kBlock), 0, s,
                     (const bf16*)x, (bf16*)y, N, H, W, C, ldx, x_coff, ldy, y_coff);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_synth_frames(uint8_t* y, int N, int H, int W, uint64_t seed, uint64_t step,
                               hipStream_t s) {
  const long long bytes = (long long)N * H * W * 3;
  if (bytes % 8) return -1;
  hipLaunchKernelGGL(synth_kernel, dim3(grid_for(bytes / 8)), dim3(kBlock), 0, s, y, bytes / 8,
                     seed, step);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_synth_frames_dev(uint8_t* y, int N, int H, int W, uint64_t seed,
                                   uint64_t* step, int bump_done, hipStream_t s) {
  const long long bytes = (long long)N * H * W * 3;
  if (bytes % 8) return -1;
  // the in-kernel ticket costs one same-address atomic per block: at 2048 blocks (batch
  // 640+) those serialise to ~13 us, more than the separate one-thread launch; at edge
  // batches (tens of blocks) it is free and saves the launch
  const unsigned g = grid_for(bytes / 8);
  const int in_kernel = bump_done && g <= 256;
  hipLaunchKernelGGL(synth_dev_kernel, dim3(g), dim3(kBlock), 0, s, y, bytes / 8, seed, step,
                     in_kernel);
  if (!in_kernel) hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, s, step);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_preprocess(const uint8_t* x, void* y, int N, int H, int W, const float* mean3,
                             const float* inv_std3, hipStream_t s) {
  const long long pix = (long long)N * H * W;
  if (pix % 2) return -1;
  hipLaunchKernelGGL(preprocess_kernel, dim3(grid_for(pix / 2)), dim3(kBlock), 0, s, x, (bf16*)y,
                     pix, mean3[0], mean3[1], mean3[2], inv_std3[0], inv_std3[1], inv_std3[2]);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_preprocess_s2d(const uint8_t* x, void* y, int N, int H, int W,
                                 const float* mean3, const float* inv_std3, hipStream_t s) {
  if (H % 2 || W % 2) return -1;
  const long long work = (long long)N * (H / 2) * (W / 2);
  hipLaunchKernelGGL(preprocess_s2d_kernel, dim3(grid_for(work)), dim3(kBlock), 0, s, x,
                     (bf16*)y, N, H, W, mean3[0], mean3[1], mean3[2], inv_std3[0], inv_std3[1],
                     inv_std3[2]);
  KV_CHECK_LAUNCH();
}

extern "C" int kv_batchnorm_nhwc(const void* x, void* y, const float* scale, const float* shift,
                                 int64_t rows, int C, int relu, hipStream_t s) {
  if (C % 8) return -1;
  const long long total8 = rows * (long long)C / 8;
  hipLaunchKernelGGL(bn_kernel, dim3(grid_for(total8)), dim3(kBlock), 0, s, (const bf16*)x,
                     (bf16*)y, scale, shift, total8, C, relu);
  KV_CHECK_LAUNCH();
}
