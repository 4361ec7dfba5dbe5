// v6 — A-resident N-loop 1x1 GEMM (+bias, residual, activation), gfx950.
//
// For the low-K, wide-N expand convs of ResNet-50 (conv3 of stages 2-4: K = 128..512,
// N = 512..2048, plus the residual add) every other family is latency-bound, not
// bandwidth-bound: with K = 256 a 128x128 output tile is only 4 K steps, so each tile is a
// chain of ~4 exposed DMA latencies plus an epilogue, and two workgroups per CU cannot
// cover it (stage-3 expand + residual: 170 us for 578 MB at batch 640, 3.4 TB/s; hipBLASLt
// is no better on the bare GEMM, profiles/r1_v11_hipblaslt_yardstick.md).
//
// This family turns the loop inside out.  A workgroup owns BM = 16 x NW output rows (128
// with the 8 waves every tile uses):
//  * its A rows (BM x K, <= 64 KB) are DMA'd into LDS ONCE and stay resident;
//  * it walks every N tile (BN = 64 channels) of the layer with the weights streamed
//    through a D-slot LDS ring -- the weights (<= 2 MB) are shared by every workgroup, so
//    they come from L2, at L2 latency, and the ring runs unbroken across N tiles;
//  * each N tile's residual is DMA'd into an RD-slot LDS ring RD - 1 tiles ahead (HBM
//    latency hidden behind whole tiles of MFMAs), and the epilogue works in place on that
//    slot: y = act2(act1(acc + bias) + res) is written back over the residual, then leaves
//    with 16-B buffer stores.  The bias table sits in LDS too.
// HBM then sees exactly A once, the residual once and y once, and every VMEM operation in
// the loop is either an LDS DMA (kv_lds_dma16, invisible to hipcc's wait-count pass) or a
// buffer store that is issued by every wave unconditionally (out-of-range rows and
// channels are dropped by the descriptor's range check).  The per-wave op sequence is thus
// fixed at compile time and every wait is an exact counted `s_waitcnt vmcnt(n)` computed by
// NlSched below -- no wait ever drains the prefetches in flight.
//
// MFMA: v_mfma_f32_16x16x32_bf16 with the operand swap of the other families (D = W . A^T:
// a lane's 4 accumulators are 4 consecutive channels of one pixel); NW waves in (NW / 2) x 2,
// each a 32 x 32 sub-tile of the BM x 64 N tile.  LDS images use the [row][64] bf16 layout with the 16-B chunk swizzle
// c ^ ((r >> 1) & 7) applied on the DMA source address (conv_glds.hip).
#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kNlOOB = 0x7ffffff0;  // byte offset past every operand: DMA zero-fills, store drops
constexpr int kNlBN = 64;
constexpr int kNlLdsMax = 160 * 1024;

template <int I>
struct NlIC {
  static constexpr int value = I;
};
template <int N, int I = 0, class F>
__device__ __forceinline__ void nl_static_for(F&& f) {
  if constexpr (I < N) {
    f(NlIC<I>{});
    nl_static_for<N, I + 1>(f);
  }
}

template <int N>
__device__ __forceinline__ void nl_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-wave VMEM issue order (every wave issues the same sequence):
//   prologue: bias table, A chunks 0..NK-1, R(0..RD-2), B(0..D-2)
//   step s (tile t = s / NK, k = s % NK): WAIT(B(s)) | barrier | B(s + D - 1) |
//       k == 0: R(t + RD - 1) | MFMAs | k == NK-1: WAIT(R(t)) ... epilogue ... stores(t)
// In-order completion makes "B(s) landed" = vmcnt(#ops issued after B(s)).
template <int NK, int D, int RD, int NW, int KS2 = 1>
struct NlSched {
  // per-wave instructions: a weight stage is 8 KB (8 DMA instructions over NW waves); an A
  // chunk, a residual tile and a tile's stores are BM x 128 B = 2 instructions per wave
  // (KS2 64-wide K chunks per step: a weight stage is KS2 x 8 KB)
  static constexpr int kB = KS2 * 8 / NW, kR = 2, kS = 2, kA = 2 * NK * KS2;
  static constexpr int steps_ops(int u) {  // ops of steps 0 .. u-1 (incl. their R / stores)
    return u * kB + ((u + NK - 1) / NK) * kR + (u / NK) * kS;
  }
  static constexpr int pro() { return kA + (RD - 1) * kR + (D - 1) * kB; }
  static constexpr int after_B(int s) {  // cumulative ops up to and including B(s)
    if (s <= D - 2) return kA + (RD - 1) * kR + (s + 1) * kB;
    return pro() + steps_ops(s - (D - 1)) + kB;
  }
  static constexpr int after_R(int t) {  // cumulative ops up to and including R(t)
    if (t <= RD - 2) return kA + (t + 1) * kR;
    return pro() + steps_ops((t - (RD - 1)) * NK) + kB + kR;
  }
  static constexpr int wait_B(int s) { return pro() + steps_ops(s) - after_B(s); }
  static constexpr int wait_E(int t) {
    const int s = (t + 1) * NK - 1;
    return pro() + steps_ops(s) + kB + (s % NK == 0 ? kR : 0) - after_R(t);
  }
  static constexpr int kFar = 16;
  // first tile from which every wait equals its steady-state (periodic) value
  static constexpr int steady_from() {
    int t0 = 0;
    for (int t = 0; t < kFar; ++t) {
      bool same = wait_E(t) == wait_E(kFar);
      for (int k = 0; k < NK; ++k) same = same && wait_B(t * NK + k) == wait_B(kFar * NK + k);
      if (!same) t0 = t + 1;
    }
    return t0;
  }
  static constexpr int kSteady = steady_from();
  static constexpr int steady_B(int k) { return wait_B(kFar * NK + k); }
  static constexpr int steady_E() { return wait_E(kFar); }
  static constexpr int safe_B(int k) {  // min over the warm-up tiles: never under-waits
    int m = steady_B(k);
    for (int t = 0; t <= kSteady; ++t) m = wait_B(t * NK + k) < m ? wait_B(t * NK + k) : m;
    return m;
  }
  static constexpr int safe_E() {
    int m = steady_E();
    for (int t = 0; t <= kSteady; ++t) m = wait_E(t) < m ? wait_E(t) : m;
    return m;
  }
};

__device__ __forceinline__ int nl_sw(int r) { return (r >> 1) & 7; }

// BM = 16 * NW rows per workgroup (NW waves, 2 x (NW / 2) of 32 x 32 sub-tiles).
// DUAL: the bottleneck's conv3 + fused downsample as one GEMM (mode 4): A chunks below K1
// come from x (row m), the rest from x2 at the strided pixel (img, ho * s2, wo * s2); only
// the resident-A prologue differs.
// KS2: 64-wide K chunks per ring step (2 = 128-wide steps: half the barriers and waits per
// MFMA, the same ring bytes); NK = K steps per N tile = Kpad / (64 KS2).
template <int NK, int D, int RD, int NW, bool DUAL = false, int KS2 = 1>
__global__ __launch_bounds__(64 * NW, 1) void conv_nloop_kernel(const KvConvParams p, int ntiles) {
  using S = NlSched<NK, D, RD, NW, KS2>;
  constexpr int NC = NK * KS2;  // 64-wide K chunks of A
  constexpr int kNlNT = 64 * NW, BM = 16 * NW, BPW = 8 / NW;  // BPW: weight DMAs per wave
  static_assert(NW == 2 || NW == 4 || NW == 8, "waves");
  static_assert(S::steady_B(0) <= 63 && S::steady_E() <= 63, "vmcnt range");
  static_assert(S::kSteady < S::kFar, "schedule must become periodic");
  constexpr int BN = kNlBN;
  constexpr int A_BYTES = NC * BM * 128, B_CHUNK = BN * 128, B_STAGE = KS2 * B_CHUNK;
  constexpr int R_SLOT = BM * BN * 2;
  constexpr int B_OFF = A_BYTES, R_OFF = B_OFF + D * B_STAGE, BIAS_OFF = R_OFF + RD * R_SLOT;
  extern __shared__ __attribute__((aligned(16))) char nl_smem[];
  char* const lds = nl_smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv >> 1, wn = wv & 1;  // 32-row block, 32-channel half of the N tile
  const int nbm = (p.M + BM - 1) / BM;
  const int m0 = xcd_remap(blockIdx.x, nbm) * BM;

  const kv_i32x4 rx = kv_rsrc4(p.x, p.N * p.H * p.W * p.ldx * 2);
  const kv_i32x4 rw = kv_rsrc4(p.w, p.Cout * p.Kpad * 2);
  const kv_i32x4 rx2 = kv_rsrc4(DUAL ? p.x2 : p.x, DUAL ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);
  const kv_i32x4 rr = kv_rsrc4(p.res, p.res ? p.M * p.ldr * 2 : 0);
  const kv_i32x4 rb = kv_rsrc4(p.bias, p.bias ? p.Cout * 4 : 0);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.M * p.ldy * 2, 0x00020000);

  // DMA lane roles: 8 rows x 8 chunks of 16 B per instruction; 2 instructions per wave
  // cover the BM = 16 NW rows of A / a residual tile (BPW per wave for a weight chunk);
  // row r's logical chunk (lane & 7) ^ sw(r) lands at position lane & 7
  const int lrow = lane >> 3, pch = lane & 7;
  int arow_off[2], a2_off[2], r_src[2], lc8[2], b_src[BPW];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wv * 2 + i) * 8 + lrow;
    const int lc = pch ^ nl_sw(row);
    lc8[i] = lc * 8;
    const int m = m0 + row;
    arow_off[i] = m < p.M ? (m * p.ldx + p.x_coff + lc * 8) * 2 : kNlOOB;
    r_src[i] = m < p.M ? (m * p.ldr + p.r_coff + lc * 8) * 2 : kNlOOB;
    a2_off[i] = kNlOOB;
    if (DUAL && m < p.M) {
      const int hw = p.Ho * p.Wo, img = m / hw, rem = m - img * hw;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      a2_off[i] = (((img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2) * p.ldx2 + lc * 8) * 2;
    }
  }
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int row = (wv * BPW + i) * 8 + lrow;
    b_src[i] = (row * p.Kpad + ((pch ^ nl_sw(row)) * 8)) * 2;  // + n-tile base + k chunk
  }

  auto issue_B = [&](int s) __attribute__((always_inline)) {
    const int t = s / NK, kc = (s - (s / NK) * NK) * KS2;
    char* dst = lds + B_OFF + (s % D) * B_STAGE;
#pragma unroll
    for (int j = 0; j < KS2; ++j)
#pragma unroll
      for (int i = 0; i < BPW; ++i) {
        const int n = t * BN + (wv * BPW + i) * 8 + lrow;
        const int v = (t < ntiles && n < p.Cout) ? b_src[i] + (t * BN * p.Kpad + (kc + j) * 64) * 2 : kNlOOB;
        kv_lds_dma16(rw, dst + j * B_CHUNK + (wv * BPW + i) * 1024, v);
      }
  };
  auto issue_R = [&](int t) __attribute__((always_inline)) {
    char* dst = lds + R_OFF + (t % RD) * R_SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = t * BN + lc8[i];
      const int v = (t < ntiles && n < p.Cout && r_src[i] != kNlOOB) ? r_src[i] + t * BN * 2 : kNlOOB;
      kv_lds_dma16(rr, dst + (wv * 2 + i) * 1024, v);
    }
  };

  // ---- prologue -------------------------------------------------------------
  {
    const int bt = (p.Cout * 4 + NW * 1024 - 1) / (NW * 1024);  // 1-KB DMAs per wave
    for (int i = 0; i < bt; ++i) {
      const int off = (i * NW + wv) * 1024;
      kv_lds_dma16(rb, lds + BIAS_OFF + off, off + lane * 16);
    }
  }
#pragma unroll
  for (int kc = 0; kc < NC; ++kc)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      char* dst = lds + kc * (BM * 128) + (wv * 2 + i) * 1024;
      if constexpr (DUAL) {  // K1 and K - K1 are multiples of 64: no K tails
        if (kc * 64 < p.K1) {
          kv_lds_dma16(rx, dst, arow_off[i] != kNlOOB ? arow_off[i] + kc * 128 : kNlOOB);
        } else {
          kv_lds_dma16(rx2, dst, a2_off[i] != kNlOOB ? a2_off[i] + (kc * 64 - p.K1) * 2 : kNlOOB);
        }
      } else {
        const int v = (arow_off[i] != kNlOOB && kc * 64 + lc8[i] < p.Cin) ? arow_off[i] + kc * 128 : kNlOOB;
        kv_lds_dma16(rx, dst, v);
      }
    }
#pragma unroll
  for (int t = 0; t < RD - 1; ++t) issue_R(t);
#pragma unroll
  for (int s = 0; s < D - 1; ++s) issue_B(s);

  const int fr = lane & 15, fh = lane >> 4;
  floatx4 acc[2][2];

  dispatch_act(p.act, p.res != nullptr, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
      const bool warm = t < S::kSteady;
      nl_static_for<NK>([&](auto kcc) __attribute__((always_inline)) {
        constexpr int k = decltype(kcc)::value;
        const int s = t * NK + k;
        if (warm) nl_wait_vm<S::safe_B(k)>();
        else nl_wait_vm<S::steady_B(k)>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue_B(s + D - 1);
        if constexpr (k == 0) issue_R(t + RD - 1);
#pragma unroll
        for (int j = 0; j < KS2; ++j) {
          const char* As = lds + (k * KS2 + j) * (BM * 128);
          const char* Bs = lds + B_OFF + (s % D) * B_STAGE + j * B_CHUNK;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const int q = ks * 4 + fh;
            bf16x8 af[2], bfg[2];
#pragma unroll
            for (int tm = 0; tm < 2; ++tm) {
              const int row = wm * 32 + tm * 16 + fr;
              af[tm] = *reinterpret_cast<const bf16x8*>(As + row * 128 + ((q ^ nl_sw(row)) << 4));
            }
#pragma unroll
            for (int tn = 0; tn < 2; ++tn) {
              const int row = wn * 32 + tn * 16 + fr;
              bfg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + ((q ^ nl_sw(row)) << 4));
            }
#pragma unroll
            for (int tn = 0; tn < 2; ++tn)
#pragma unroll
              for (int tm = 0; tm < 2; ++tm)
                acc[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[tn], af[tm], acc[tn][tm], 0, 0, 0);
          }
        }
      });
      // ---- epilogue of tile t: residual slot t % RD holds R(t); y overwrites it in place
      if (warm) nl_wait_vm<S::safe_E()>();
      else nl_wait_vm<S::steady_E()>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      char* Rs = lds + R_OFF + (t % RD) * R_SLOT;
      const float* bias_t = reinterpret_cast<const float*>(lds + BIAS_OFF) + t * BN;
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        const int c0 = wn * 32 + tn * 16 + fh * 4;
        const float4 bv = t * BN + c0 < p.Cout ? *reinterpret_cast<const float4*>(bias_t + c0)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) {
          const int row = wm * 32 + tm * 16 + fr;
          bf16x4* ptr = reinterpret_cast<bf16x4*>(Rs + row * 128 + (((c0 >> 3) ^ nl_sw(row)) << 4) +
                                                  (c0 & 7) * 2);
          const bf16x4 rv = *ptr;
          bf16x4 o;
          o[0] = f2bf(act_c<act2>(act_c<act1>(acc[tn][tm][0] + bv.x) + (float)rv[0]));
          o[1] = f2bf(act_c<act2>(act_c<act1>(acc[tn][tm][1] + bv.y) + (float)rv[1]));
          o[2] = f2bf(act_c<act2>(act_c<act1>(acc[tn][tm][2] + bv.z) + (float)rv[2]));
          o[3] = f2bf(act_c<act2>(act_c<act1>(acc[tn][tm][3] + bv.w) + (float)rv[3]));
          *ptr = o;
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = tid + kNlNT * i;
        const int row = idx >> 3, c = idx & 7;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(Rs + row * 128 + ((c ^ nl_sw(row)) << 4));
        const int m = m0 + row, n = t * BN + c * 8;
        const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kNlOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(kv_i32x4, v), ry, off, 0, 0);
      }
    }
  });
  // the ring's prefetches past the last tile are still landing in LDS: drain them before
  // the workgroup's LDS can be handed to the next workgroup on this CU
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Host self-check of the counted-wait schedule (tests/test_conv_nloop_sched_cpu.py): replays
// one wave's VMEM issue order for 3 x kFar N tiles exactly as the kernel issues it and
// requires every wait the kernel uses to be <= the exact count of ops issued after the
// awaited one (a larger count would let the wave read LDS before its DMA lands), and equal
// to it from the steady tile on (a smaller one only over-waits).  Returns 0 when the
// schedule is safe, else a code naming the first violation.
template <int NK, int D, int RD, int NW, int KS2>
int nl_sched_check() {
  using S = NlSched<NK, D, RD, NW, KS2>;
  constexpr int T = 3 * S::kFar, NS = T * NK + D + 1;
  long long endB[NS] = {}, endR[T + RD + 1] = {};
  long long pos = S::kA;  // bias table DMAs precede everything that is waited on
  for (int t = 0; t < RD - 1; ++t) endR[t] = (pos += S::kR);
  for (int s = 0; s < D - 1; ++s) endB[s] = (pos += S::kB);
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < NK; ++k) {
      const int s = t * NK + k;
      const long long exact = pos - endB[s];
      const int used = t < S::kSteady ? S::safe_B(k) : S::steady_B(k);
      if (used > exact || (t >= S::kSteady && used != exact) || used > 63) return 1000 + s;
      endB[s + D - 1] = (pos += S::kB);
      if (k == 0) endR[t + RD - 1] = (pos += S::kR);
    }
    const long long exact = pos - endR[t];
    const int used = t < S::kSteady ? S::safe_E() : S::steady_E();
    if (used > exact || (t >= S::kSteady && used != exact) || used > 63) return 2000 + t;
    pos += S::kS;
  }
  return 0;
}

typedef void (*NlFn)(const KvConvParams, int);

struct NlTile {
  int nk, d, rd, nw, dual, ks2;  // nk: K steps per N tile of ks2 x 64 K each
  NlFn fn;
  int (*sched_check)();
};

// one table row: the kernel and its schedule check from the same template arguments
template <int NK, int D, int RD, int NW, bool DUAL = false, int KS2 = 1>
constexpr NlTile nl_tile() {
  return NlTile{NK, D, RD, NW, DUAL ? 1 : 0, KS2, &conv_nloop_kernel<NK, D, RD, NW, DUAL, KS2>,
                &nl_sched_check<NK, D, RD, NW, KS2>};
}

// LDS = A (K x BM x 2) + d x 8 KB weight ring + rd x BM x 128 B residual ring + the bias
// table (Cout x 4 B, rounded up to nw KB).  Measured at batch 640 (profiles/r2_v18_*):
// one 8-wave workgroup per CU with BM = 128 and a 5-7 slot ring beats two or three smaller
// workgroups per CU (BM 64 / 32: 155-234 us on the stage-3 expand against 136-147 us), and
// warp-specialised forms (8 compute waves + 1, 2 or 4 waves issuing every residual DMA and
// store, so the weight waits never queue behind HBM-latency ops in the in-order vmcnt) lost
// too: 155-180 us (profiles/r2_v18_nloop_tile_probe.md, rounds d and e).
static const NlTile kNlTiles[] = {
    nl_tile<2, 6, 2, 8>(),  // K = 128 (stage-2 expand)
    nl_tile<4, 6, 2, 8>(),  // K = 256 (stage-3 expand)
    nl_tile<4, 7, 2, 8>(),  // K = 256, 7-slot ring (160 KB)
    nl_tile<4, 4, 3, 8>(),  // K = 256, residual two tiles ahead
    nl_tile<4, 5, 2, 8>(),  // K = 256, 5-slot ring
    // fused downsample (dual, no residual: a 1-slot staging ring for the epilogue)
    nl_tile<6, 5, 1, 8, true>(),   // K = 128 + 256 (stage 2)
    nl_tile<6, 4, 1, 8, true>(),   // K = 128 + 256, 4-slot ring
    nl_tile<12, 5, 1, 4, true>(),  // K = 256 + 512 (stage 3), BM 64
    // 128-wide K steps (two 64-chunks per ring slot): stage-3 expand 143 -> 136 us at b640;
    // the K = 128 and dual forms of this step lost (266 vs 245 us, 391 vs 353 us) and are not
    // instantiated (profiles/r2_v18_nloop_tile_probe.md, round f)
    nl_tile<2, 3, 2, 8, false, 2>(),  // K = 256
    nl_tile<2, 3, 1, 8, false, 2>(),  // K = 256, 1-slot residual
};

}  // namespace

int nloop_num_tiles() { return (int)(sizeof(kNlTiles) / sizeof(kNlTiles[0])); }

// 0 if every v6 tile's counted-wait schedule is safe (host-side replay), else
// tile * 10000 + the violation code of nl_sched_check
int nloop_sched_check() {
  for (int i = 0; i < nloop_num_tiles(); ++i)
    if (const int rc = kNlTiles[i].sched_check()) return i * 10000 + rc;
  return 0;
}

int nloop_lds_bytes(int tile, int cout) {
  const NlTile& e = kNlTiles[tile];
  const int bm = 16 * e.nw;
  return e.nk * e.ks2 * bm * 128 + e.d * e.ks2 * kNlBN * 128 + e.rd * bm * kNlBN * 2 +
         ((cout * 4 + e.nw * 1024 - 1) / (e.nw * 1024)) * (e.nw * 1024);
}

int nloop_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= nloop_num_tiles()) return -6;
  const NlTile& e = kNlTiles[tile];
  if (p->n_t || p->in_u8) return -8;
  if (e.dual) {  // conv3 + fused downsample only
    if (p->mode != 4 || p->res || !p->x2 || p->up2 || p->x2_coff || p->K1 % 64 ||
        (p->Kpad - p->K1) % 64 ||
        (long long)p->N * p->H2 * p->W2 * p->ldx2 * 2 >= kNlOOB)
      return -8;
  } else if (p->mode != 1) {
    return -8;  // 1x1 stride-1 GEMM
  }
  if (p->Kpad != e.nk * e.ks2 * 64 || (!e.dual && p->Cin > p->Kpad)) return -8;
  if ((long long)p->M * p->ldy * 2 >= kNlOOB || (p->res && (long long)p->M * p->ldr * 2 >= kNlOOB) ||
      (long long)p->N * p->H * p->W * p->ldx * 2 >= kNlOOB || (long long)p->Cout * p->Kpad * 2 >= kNlOOB)
    return -9;
  const int lds = nloop_lds_bytes(tile, p->Cout);
  if (lds > kNlLdsMax) return -11;
  const int bm = 16 * e.nw;
  const int nbm = (p->M + bm - 1) / bm, ntiles = (p->Cout + kNlBN - 1) / kNlBN;
  if (nbm <= 0 || ntiles <= 0) return 0;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(e.fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(e.fn, dim3((unsigned)nbm), dim3(64 * e.nw), (unsigned)lds, stream, *p, ntiles);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
