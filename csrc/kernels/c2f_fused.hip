// v13: YOLOv8 C2f block with one 16-channel shortcut bottleneck as ONE launch (the b2 block
// of YOLOv8n: C2f(32, 32, n=1, shortcut) at 160 x 160):
//
//   t = SiLU(W1 . x + b1)                      1x1 32 -> 32;  a = t[:16], s = t[16:]
//   u = SiLU(conv3x3(s; Wm1) + bm1)            3x3 16 -> 16
//   v = s + SiLU(conv3x3(u; Wm2) + bm2)        3x3 16 -> 16, shortcut after the activation
//   y = SiLU(W2 . [a, s, v] + b2)              1x1 48 -> 32
//
// Unfused, the block is four launches that move 224 channels per pixel through HBM (t, u, v
// written and re-read, the 48-channel concat read): the in-graph table of the YOLOv8n bench
// step (profiles/r5_v6_graph_layers_yolo_b512.md, rows 1-4) puts it at ~2 ms of the 10.8 ms
// step against ~0.3 ms of compulsory traffic (x read, y written: 64 channels per pixel).
// Here x is read once and y written once; t / u stay in LDS rings.
//
// Decomposition: a workgroup (W / 16 waves, one 16-pixel block each) sweeps a strip of S
// output rows of one image top to bottom, two rows per iteration, with row rings in LDS (s and
// a: 6 rows, u: 4 rows; zero columns either side for the 3x3 padding, zero rows outside the
// image):
//   phase 1: u of rows o + 1, o + 2 from s rows o .. o + 3
//   barrier
//   phase 2: t of rows o + 4, o + 5 from x (in registers, loaded an iteration ahead);
//            v from u rows o - 1 .. o + 2 and s; y of rows o, o + 1 from a, s and v
//   barrier
// One barrier per row: every slot a phase writes was last read in the other phase of the
// previous iteration.  In each phase a wave has two rows' independent MFMA chains, and their
// LDS fragment reads are all issued first.  The strip's first rows repeat two rows of t and
// one of u of the strip above (halo).  (The first form ran one row per iteration with three
// steps and two barriers per row: 469 us at b256 vs 441 us with the reads hoisted;
// profiles/r5_v10_c2f_probe.md, r5_v11_c2f_probe_wave_per_block.txt.)
//
// MFMA: v_mfma_f32_16x16x32_bf16, weights as the first operand (D = W . X^T: a lane's four
// accumulators are four consecutive output channels of one pixel).  The 3x3s run K = 9 taps
// x 16 channels as five 32-wide steps, lane quarter q of step j reading tap 2j + q / 2 (the
// tenth tap's weights are zero; its activations are read from a real pixel, so never NaN).
// The concat's v part is fed to cv2 straight from the 3x3's accumulators: lane (pixel, q)
// holds v channels 4q .. 4q + 3, so cv2's second K step takes them as k = 8q .. 8q + 3 with
// zeros in k = 8q + 4 .. 8q + 7, and the weights are read in that permuted order -- v never
// goes through LDS.
#include <stdlib.h>

#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kC2fRS = 6, kC2fRU = 4, kC2fRA = 6;  // two rows per iteration (below)
typedef unsigned int c2f_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int c2f_u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kC2fOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t c2f_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes),
                                           0x00020000);
}

// SiLU of four accumulators (the bias is already in them: the MFMA chains start from it),
// two at a time in packed fp32 (v_pk_mul / v_pk_add): per element one exp and one rcp plus
// 1.5 packed ops.  The kernel is VALU-issue-bound (profiles/r5_v12_c2f_probe_two_rows.txt)
typedef float c2f_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ floatx4 c2f_silu4f(floatx4 v) {
  floatx4 o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const c2f_f2 x = {v[2 * h], v[2 * h + 1]};
    const c2f_f2 t = x * c2f_f2{-1.4426950408889634f, -1.4426950408889634f};
    c2f_f2 d = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
    d = d + c2f_f2{1.f, 1.f};
    const c2f_f2 y = x * c2f_f2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    o[2 * h] = y[0];
    o[2 * h + 1] = y[1];
  }
  return o;
}
__device__ __forceinline__ bf16x4 c2f_pack4(floatx4 v) {
  bf16x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
  return o;
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, 3) void c2f16_kernel(const KvC2fParams p, int diag) {
  constexpr int BPW = 1;  // one 16-pixel block per wave: W = 16 x WAVES
  extern __shared__ __attribute__((aligned(16))) char c2f_lds[];
  constexpr int W = 16 * WAVES;
  constexpr int WP = W + 2;  // one zero column either side
  bf16* const sring = reinterpret_cast<bf16*>(c2f_lds);  // [RS][WP][16]
  bf16* const uring = sring + kC2fRS * WP * 16;          // [RU][WP][16]
  bf16* const aring = uring + kC2fRU * WP * 16;          // [RA][W][16]

  const int strips = p.H / p.S;
  const int img = blockIdx.x / strips;
  const int s0 = (blockIdx.x - img * strips) * p.S, s1 = s0 + p.S;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int H = p.H;

  // ---- zero the padding columns of the s / u rings (never written by the steps)
  for (int i = threadIdx.x; i < (kC2fRS + kC2fRU) * 2 * 2; i += WAVES * 64) {
    const int slot = i >> 2, side = (i >> 1) & 1, half = i & 1;
    bf16* row = slot < kC2fRS ? sring + slot * WP * 16 : uring + (slot - kC2fRS) * WP * 16;
    *reinterpret_cast<c2f_u32x4*>(row + (side ? WP - 1 : 0) * 16 + half * 8) = c2f_u32x4{0, 0, 0, 0};
  }

  // ---- weights and biases in registers (every wave needs all of them)
  const __amdgpu_buffer_rsrc_t rw1 = c2f_rsrc(p.w1, 32LL * p.ldw1 * 2);
  const __amdgpu_buffer_rsrc_t rwm1 = c2f_rsrc(p.wm1, 16LL * p.ldwm * 2);
  const __amdgpu_buffer_rsrc_t rwm2 = c2f_rsrc(p.wm2, 16LL * p.ldwm * 2);
  const __amdgpu_buffer_rsrc_t rw2 = c2f_rsrc(p.w2, 32LL * p.ldw2 * 2);
  bf16x8 w1f[2], wm1f[5], wm2f[5], w2f0[2], w2f1[2];
  // biases live in LDS (96 floats; registers are the limit: 3 waves per SIMD)
  float* const bias_lds = reinterpret_cast<float*>(aring + kC2fRA * W * 16);  // b1 | bm1 | bm2 | b2
  for (int i = threadIdx.x; i < 96; i += WAVES * 64)
    bias_lds[i] = i < 32 ? p.b1[i] : i < 48 ? p.bm1[i - 32] : i < 64 ? p.bm2[i - 48] : p.b2[i - 64];
  auto bias4 = [&](int off) __attribute__((always_inline)) -> floatx4 {
    return *reinterpret_cast<const floatx4*>(bias_lds + off + q * 4);
  };
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int row = nb * 16 + r16;
    w1f[nb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                             rw1, (unsigned)(row * p.ldw1 + q * 8) * 2u, 0, 0));
    w2f0[nb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              rw2, (unsigned)(row * p.ldw2 + q * 8) * 2u, 0, 0));
    // cv2's v columns in the accumulator order: k = 8q + e <- v channel 4q + e (e < 4)
    const c2f_u32x2 lo = __builtin_amdgcn_raw_buffer_load_b64(
        rw2, (unsigned)(row * p.ldw2 + 32 + q * 4) * 2u, 0, 0);
    w2f1[nb] = __builtin_bit_cast(bf16x8, c2f_u32x4{lo[0], lo[1], 0u, 0u});
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int tap = 2 * j + (q >> 1);
    const unsigned off = tap < 9 ? (unsigned)(r16 * p.ldwm + tap * 16 + (q & 1) * 8) * 2u : kC2fOOB;
    wm1f[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rwm1, off, 0, 0));
    wm2f[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rwm2, off, 0, 0));
  }

  // diag bit 1: identity instead of SiLU (timing only)
  // bias-seeded accumulator -> SiLU (diag bit 1: identity, timing only) -> bf16
  auto c2f_act4 = [&](floatx4 acc) __attribute__((always_inline)) -> bf16x4 {
    return c2f_pack4((diag & 1) ? acc : c2f_silu4f(acc));
  };

  // 3x3 tap of lane quarter q in step j (the tenth tap re-reads tap 8: finite, weight 0)
  int tdy[5], tdx[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int tap = min(2 * j + (q >> 1), 8);
    tdy[j] = tap / 3;
    tdx[j] = tap % 3;
  }

  // ---- x rows: lane (pixel r16 of block b, quarter q) loads channels 8q .. 8q + 7
  const __amdgpu_buffer_rsrc_t rx = c2f_rsrc(p.x, (long long)p.N * H * W * p.ldx * 2);
  const __amdgpu_buffer_rsrc_t ry = c2f_rsrc(p.y, (long long)p.N * H * W * p.ldy * 2);
  auto load_x = [&](int r, c2f_u32x4 (&dst)[BPW]) __attribute__((always_inline)) {
    const bool ok = r >= 0 && r < H && r <= s1 + 3 && !(diag & 2);
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
      const int px = (w + WAVES * b) * 16 + r16;
      const unsigned off =
          ok ? (unsigned)(((img * H + r) * W + px) * p.ldx + p.x_coff + q * 8) * 2u : kC2fOOB;
      dst[b] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
    }
  };
  auto slot_s = [](int r) { return (r + 2 * kC2fRS) % kC2fRS; };
  auto slot_u = [](int r) { return (r + 2 * kC2fRU) % kC2fRU; };
  auto slot_a = [](int r) { return (r + 2 * kC2fRA) % kC2fRA; };

  // step A: t of row r -> a ring (channels 0-15) and s ring (16-31; zero outside the image)
  auto stepA = [&](int r, const c2f_u32x4 (&xr)[BPW]) __attribute__((always_inline)) {
    const bool in = r >= 0 && r < H;
    bf16* srow = sring + slot_s(r) * WP * 16;
    bf16* arow = aring + slot_a(r) * W * 16;
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
      const int px = (w + WAVES * b) * 16 + r16;
      const bf16x8 xf = __builtin_bit_cast(bf16x8, xr[b]);
      const floatx4 ta = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[0], xf, bias4(0), 0, 0, 0);
      const floatx4 ts = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[1], xf, bias4(16), 0, 0, 0);
      bf16x4 sv = c2f_act4(ts);
      if (!in) sv = bf16x4{0, 0, 0, 0};
      *reinterpret_cast<bf16x4*>(arow + px * 16 + q * 4) = c2f_act4(ta);
      *reinterpret_cast<bf16x4*>(srow + (px + 1) * 16 + q * 4) = sv;
    }
  };
  // 3x3 16 -> 16 over three rows of a ring (rows r - 1 .. r + 1 at slots sl[0..2])
  // 3x3 16 -> 16: the five fragment reads of a block (rows r - 1 .. r + 1 of a ring at slots
  // sl[0..2]) are issued for every block of the wave before the first MFMA (hipcc otherwise
  // serialises read -> wait -> MFMA per tap: ~5 LDS round trips per block and step)
  // Step j's taps are 2j (lanes q < 2) and 2j + 1 (q >= 2): both halves read the same ring row
  // except in step 1 (taps 2 and 3), so the row base is a scalar and the per-lane part of the
  // address (pixel, tap column, channel half) is precomputed once
  const int px_w = w * 16 + r16;
  const bool qhi = q >= 2;
  const int fbase = px_w * 16 + (q & 1) * 8;  // bf16 units: pixel + channel half
  const int fhi = qhi ? 16 : 0;               // one pixel further for the high half
  auto frags3 = [&](const bf16* ring, const int (&sl)[3], int /*px*/, bf16x8 (&fr)[5])
      __attribute__((always_inline)) {
    static_range<0, 5>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr int tlo = 2 * j, thi = 2 * j + 1 < 9 ? 2 * j + 1 : 8;
      constexpr int dlo = tlo / 3, dhi = thi / 3, xlo = tlo % 3, xhi = thi % 3;
      const bf16* row = ring + sl[dlo] * WP * 16;
      if constexpr (dhi != dlo) row = qhi ? ring + sl[dhi] * WP * 16 : row;
      fr[j] = *reinterpret_cast<const bf16x8*>(row + fbase + xlo * 16 + (xhi - xlo) * fhi);
    });
  };
  // step B: u of rows r, r + 1 from s rows r - 1 .. r + 2 (zero outside the image); the two
  // rows' fragment reads go first, then their MFMA chains interleaved
  auto stepB = [&](int r) __attribute__((always_inline)) {
    const int px = w * 16 + r16;
    bf16x8 fr[2][5];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int sl[3] = {slot_s(r + i - 1), slot_s(r + i), slot_s(r + i + 1)};
      frags3(sring, sl, px, fr[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc[2] = {bias4(32), bias4(32)};
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm1f[j], fr[i][j], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool in = r + i >= 0 && r + i < H;
      bf16x4 uv = c2f_act4(acc[i]);
      if (!in) uv = bf16x4{0, 0, 0, 0};
      *reinterpret_cast<bf16x4*>(uring + slot_u(r + i) * WP * 16 + (px + 1) * 16 + q * 4) = uv;
    }
  };
  // step C: v and y of output rows o, o + 1
  auto stepC = [&](int o) __attribute__((always_inline)) {
    const int px = w * 16 + r16;
    bf16x8 fr[2][5], as[2];
    bf16x4 sres[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int sl[3] = {slot_u(o + i - 1), slot_u(o + i), slot_u(o + i + 1)};
      const bf16* srow = sring + slot_s(o + i) * WP * 16;
      const bf16* arow = aring + slot_a(o + i) * W * 16;
      frags3(uring, sl, px, fr[i]);
      sres[i] = *reinterpret_cast<const bf16x4*>(srow + (px + 1) * 16 + q * 4);
      // cv2's first K step: [a | s] channels 8q .. 8q + 7 of the concat
      as[i] = q < 2 ? *reinterpret_cast<const bf16x8*>(arow + px * 16 + q * 8)
                    : *reinterpret_cast<const bf16x8*>(srow + (px + 1) * 16 + (q - 2) * 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    floatx4 m[2] = {bias4(48), bias4(48)};
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        m[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm2f[j], fr[i][j], m[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x8 vf;
      const bf16x4 mv = c2f_act4(m[i]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // rounded to bf16 before and after the shortcut add, as the four-launch path does
        vf[e] = f2bf((float)mv[e] + (float)sres[i][e]);
        vf[4 + e] = (bf16)0.f;
      }
      const size_t ybase = ((size_t)(img * H + o + i) * W + px) * p.ldy + p.y_coff;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        floatx4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f0[nb], as[i], bias4(64 + nb * 16),
                                                              0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f1[nb], vf, acc, 0, 0, 0);
        const bf16x4 yv = c2f_act4(acc);
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(c2f_u32x2, yv), ry,
            (diag & 4) ? kC2fOOB : (unsigned)(ybase + nb * 16 + q * 4) * 2u, 0, 0);
      }
    }
  };

  __syncthreads();  // biases and the zero columns are in LDS
  // ---- prologue: t of rows s0 - 2 .. s0 + 3, u of rows s0 - 1, s0
  {
    c2f_u32x4 xp[6][BPW];
#pragma unroll
    for (int i = 0; i < 6; ++i) load_x(s0 - 2 + i, xp[i]);
#pragma unroll
    for (int i = 0; i < 6; ++i) stepA(s0 - 2 + i, xp[i]);
  }
  c2f_u32x4 xr[2][2][BPW];  // x of rows o + 4, o + 5 for this and the next iteration
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int i = 0; i < 2; ++i) load_x(s0 + 4 + 2 * k + i, xr[k][i]);
  __syncthreads();
  stepB(s0 - 1);
  // ---- sweep, two output rows per iteration and one barrier per row:
  //   phase 1: u of rows o + 1, o + 2          (s rows o .. o + 3 are in the ring)
  //   phase 2: t of rows o + 4, o + 5; v and y of rows o, o + 1
  // Every slot a phase writes was last read in the other phase of the previous iteration
  // (ring sizes: s 6, a 6, u 4).  S is a multiple of 4, so the x register ring is static.
  for (int o = s0; o < s1; o += 4) {
    static_range<0, 2>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int oo = o + 2 * k;
      stepB(oo + 1);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        stepA(oo + 4 + i, xr[k][i]);
        load_x(oo + 8 + i, xr[k][i]);
      }
      stepC(oo);
      __syncthreads();
    });
  }
}

}  // namespace

int c2f16_lds_bytes(int W) {
  return ((kC2fRS + kC2fRU) * (W + 2) + kC2fRA * W) * 16 * 2 + 96 * 4;  // + biases
}

// KVEDGE_C2F_DIAG (timing experiments, tools/c2f_probe.py): 1 identity activations, 2 no x
// loads, 4 no y stores (bit 8, y staged through LDS for whole-pixel stores, measured slower:
// profiles/r5_v10_c2f_probe.md, removed)
int c2f_diag() {
  const char* e = getenv("KVEDGE_C2F_DIAG");
  return e ? atoi(e) : 0;
}

}  // namespace kvedge

using namespace kvedge;

extern "C" int kv_c2f16_supported(int H, int W, int S) {
  return (W == 160 || W == 80) && S > 0 && S % 4 == 0 && H % S == 0;
}

extern "C" int kv_c2f16_fused(const KvC2fParams* p, hipStream_t stream) {
  if (!kv_c2f16_supported(p->H, p->W, p->S)) return -8;
  if (p->ldx % 8 || p->x_coff % 8 || p->ldy % 4 || p->y_coff % 4 || p->ldw1 < 32 ||
      p->ldw2 < 48 || p->ldwm < 144)
    return -3;
  const int lds = c2f16_lds_bytes(p->W);
  const int diag = c2f_diag();
  const unsigned grid = (unsigned)(p->N * (p->H / p->S));
  if (grid == 0) return 0;
  const void* fn = p->W == 160 ? reinterpret_cast<const void*>(&c2f16_kernel<10>)
                               : reinterpret_cast<const void*>(&c2f16_kernel<5>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  if (p->W == 160)
    hipLaunchKernelGGL(c2f16_kernel<10>, dim3(grid), dim3(10 * 64), (unsigned)lds, stream, *p, diag);
  else
    hipLaunchKernelGGL(c2f16_kernel<5>, dim3(grid), dim3(5 * 64), (unsigned)lds, stream, *p, diag);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
