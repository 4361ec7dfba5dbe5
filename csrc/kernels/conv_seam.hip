// v9 -- bottleneck seam: conv3 (+bias +residual, ReLU) -> next block's conv1, one launch.
//
// Stages 2-4 of ResNet-50 end every bottleneck with an expand conv3 (K3 = 128 / 256 / 512
// -> Cout = 4 K3, + residual) whose output y is immediately re-read by the next block's
// 1x1 reduce conv1 (Cout -> N1 = K3, or 2 K3 at a stage boundary).  As two launches the
// pair moves A + R + y (write) + y (read) + z bytes and runs each half at its own
// latency-bound rate (profiles/r3_v12_resnet50_b640_roofline.md rows 25/26: 137 + 83 us
// per stage-3 seam at batch 640 against a 96 + 54 us HBM floor).  Fused, y never makes the
// HBM round trip and the conv1 MFMAs overlap the conv3 memory stream.
//
// Structure (the v6 A-resident N-loop, conv_nloop.hip, extended):
//  * one 8-wave workgroup per CU owns BM = 128 output rows; its A rows (BM x K3) are
//    DMA'd into LDS once and stay resident;
//  * it walks the T = Cout / 64 y tiles.  Tile t: 64-channel conv3 tile from A and W3
//    (NK3 64-deep K steps), epilogue y = ReLU(acc + b3 + R(t)) in place over the residual
//    slot, y tile stored with 16-B stores -- and the SAME LDS tile is then the A operand
//    of a 64-deep K slice of conv1: z[BM][N1] += y_t . W1[:, 64t : 64t + 64]^T (NZ = N1/64
//    steps of 64 z channels each).  z stays in registers (NZ x 16 floats per lane) across
//    the whole tile walk and leaves once, ReLU(z + b1), at the end;
//  * W3 and W1 stream through ONE ring of 8-KB stages (64 rows x 64 K, bf16): per tile NK3
//    W3 stages then NZ W1 stages.  The weights are shared by every workgroup, so they come
//    from L2; each workgroup reads W3 + W1 once (1 MB at stage 3);
//  * the residual of tile t is DMA'd RD - 1 tiles ahead into an RD-slot ring.
// Every VMEM op is an LDS DMA (kv_lds_dma16, invisible to hipcc's wait-count pass) or an
// unconditional buffer store, so every wave issues a fixed op sequence and every wait is an
// exact counted `s_waitcnt vmcnt(n)` from the constexpr replay SmSched below.
//
// MFMA v_mfma_f32_16x16x32_bf16 with the operand swap (D = W . A^T: a lane's accumulators
// are 4 consecutive channels of one pixel); 8 waves as 4 (rows) x 2 (channel halves), each
// a 32 x 32 sub-tile of every 128 x 64 (tile, stage) product, conv3 and conv1 alike.
#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kSmOOB = 0x7ffffff0;  // byte offset past every operand: DMA zero-fills, store drops
constexpr int kSmLdsMax = 160 * 1024;

template <int I>
struct SmIC {
  static constexpr int value = I;
};
template <int N, int I = 0, class F>
__device__ __forceinline__ void sm_static_for(F&& f) {
  if constexpr (I < N) {
    f(SmIC<I>{});
    sm_static_for<N, I + 1>(f);
  }
}

template <int N>
__device__ __forceinline__ void sm_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-wave VMEM issue order (every wave issues the same sequence; bias DMAs come first and
// are older than everything waited on):
//   prologue: A chunks (2 per 64-K chunk), R(0 .. RD-2) (2 each), B(0 .. D-2) (kB each)
//   tile t, ring step j = 0 .. SPT-1 (s = t SPT + j; SY conv3 steps, then SZ conv1 steps):
//     j == SY: WAIT(R(t)) | y epilogue | y stores (2)
//     WAIT(B(s)) | barrier | B(s + D - 1) | j == 0: R(t + RD - 1) | MFMAs
// vmcnt counts in issue order, so "X landed" = vmcnt(#ops issued after X).  The waits are
// computed by replaying that sequence at compile time.
template <int SY, int SZ, int D, int RD, int KB, int NA>
struct SmSched {
  static constexpr int SPT = SY + SZ;
  static constexpr int kB = KB, kR = 2, kS = 2, kA = NA;  // NA: A-chunk DMAs per wave
  static constexpr int kFar = 12;
  static constexpr int kTiles = kFar + 2;
  // kind 0: wait before reading ring stage s; kind 1: wait before tile t's epilogue;
  // kind 2 (XP): the wait at step s that covers stage s + 1 (its fragments are read during
  // step s, one step ahead of their MFMAs)
  static constexpr int wait(int kind, int idx) {
    long endB[kTiles * SPT + D + 2] = {};
    long endR[kTiles + RD + 2] = {};
    long pos = kA;
    for (int t = 0; t < RD - 1; ++t) endR[t] = (pos += kR);
    for (int s = 0; s < D - 1; ++s) endB[s] = (pos += kB);
    for (int t = 0; t < kTiles; ++t) {
      for (int j = 0; j < SPT; ++j) {
        const int s = t * SPT + j;
        if (j == SY) {
          if (kind == 1 && idx == t) return (int)(pos - endR[t]);
          pos += kS;
        }
        if (kind == 0 && idx == s) return (int)(pos - endB[s]);
        if (kind == 2 && idx == s) return D >= 3 ? (int)(pos - endB[s + 1]) : -1;
        endB[s + D - 1] = (pos += kB);
        if (j == 0) endR[t + RD - 1] = (pos += kR);
      }
    }
    return -1;
  }
  static constexpr int wB(int t, int j) { return wait(0, t * SPT + j); }
  static constexpr int wE(int t) { return wait(1, t); }
  static constexpr int wXB(int t, int j) { return wait(2, t * SPT + j); }
  static constexpr int steady_from() {
    int t0 = 0;
    for (int t = 0; t < kFar; ++t) {
      bool same = wE(t) == wE(kFar);
      for (int j = 0; j < SPT; ++j)
        same = same && wB(t, j) == wB(kFar, j) && wXB(t, j) == wXB(kFar, j);
      if (!same) t0 = t + 1;
    }
    return t0;
  }
  static constexpr int kSteady = steady_from();
  static constexpr int safe_B(int j) {  // min over the warm-up tiles: never under-waits
    int m = wB(kFar, j);
    for (int t = 0; t <= kSteady; ++t) m = wB(t, j) < m ? wB(t, j) : m;
    return m;
  }
  static constexpr int safe_XB(int j) {
    int m = wXB(kFar, j);
    for (int t = 0; t <= kSteady; ++t) m = wXB(t, j) < m ? wXB(t, j) : m;
    return m;
  }
  static constexpr int safe_E() {
    int m = wE(kFar);
    for (int t = 0; t <= kSteady; ++t) m = wE(t) < m ? wE(t) : m;
    return m;
  }
  static constexpr bool ok(bool xp = false) {
    for (int t = 0; t <= kFar; ++t) {
      if (wE(t) < 0 || wE(t) > 63) return false;
      for (int j = 0; j < SPT; ++j) {
        if (wB(t, j) < 0 || wB(t, j) > 63) return false;
        if (xp && (wXB(t, j) < 0 || wXB(t, j) > 63)) return false;
      }
    }
    return kSteady < kFar;
  }
};

__device__ __forceinline__ int sm_sw(int r) { return (r >> 1) & 7; }

// Workgroup barrier for LDS hand-offs only: this wave's LDS ops retired, then s_barrier.
// (__syncthreads()' fence may also wait for the wave's global stores, and vmcnt drains in
// order, so it would drain every ring prefetch behind them.)
__device__ __forceinline__ void sm_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NC3 / NZC: 64-wide chunks of K3 (conv3's K) / of N1 (conv1's output channels).
// NW waves (BM = 16 NW rows, (NW / 2) x 2 waves of 32 x 32); KS2 64-chunks per ring stage
// (2 = 16-KB stages: half the waits and barriers per MFMA).  NW = 4 tiles fit 80 KB of LDS,
// so two workgroups share a CU and one's ring waits hide under the other's MFMAs.
// AREG: each wave keeps its 32 rows of A (conv3's input) in VGPRs (NC3 x 16 registers)
// instead of LDS: the conv3 steps then read only weight fragments from LDS (0.5 ds_read_b128
// per MFMA instead of 1.0 -- the LDS-bound part of the step), and the freed LDS deepens the
// weight ring.
// XP (AREG forms): cross-step fragment prefetch.  The wait + barrier at step s covers ring
// stage s + 1, and step s reads stage s + 1's weight fragments into the other register set
// while its own MFMAs consume the set read during step s - 1: no step starts with an LDS
// round trip behind the barrier (the conv1 steps' y-tile A reads stay in-step: y is written
// by the epilogue at the start of the tile's first conv1 step).
template <int NC3, int NZC, int D, int RD, int NW = 8, int KS2 = 1, bool AREG = false,
          bool XP = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void conv_seam_kernel(const KvConvParams p, int ntiles) {
  static_assert(NW == 4 || NW == 8, "waves");
  static_assert(NC3 % KS2 == 0 && NZC % KS2 == 0, "whole chunks per ring stage");
  constexpr int SY = NC3 / KS2, SZ = NZC / KS2, BPW = 8 / NW;  // BPW: DMAs per wave per chunk
  using S = SmSched<SY, SZ, D, RD, KS2 * BPW, AREG ? 0 : 2 * NC3>;
  static_assert(S::ok(XP), "counted-wait schedule out of range or not periodic");
  constexpr int SPT = S::SPT, BM = 16 * NW, NT = 64 * NW;
  static_assert(!XP || (AREG && D >= 3 && SPT % 2 == 0),
                "XP: A in VGPRs, stage s + 1 issued before step s, register sets by step parity");
  constexpr int A_BYTES = AREG ? 0 : NC3 * BM * 128, B_CHUNK = 64 * 128, B_STAGE = KS2 * B_CHUNK;
  constexpr int R_SLOT = BM * 64 * 2;
  constexpr int B_OFF = A_BYTES, R_OFF = B_OFF + D * B_STAGE, BIAS_OFF = R_OFF + RD * R_SLOT;
  constexpr int BIAS_ROUND = NW * 1024;  // bias DMAs: 1 KB per wave-instruction
  extern __shared__ __attribute__((aligned(16))) char sm_smem[];
  char* const lds = sm_smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv >> 1, wn = wv & 1;  // 32-row block, 32-channel half of each chunk
  const int nbm = (p.M + BM - 1) / BM;
  const int m0 = xcd_remap(blockIdx.x, nbm) * BM;
  const int Cout = p.Cout, N1 = p.n_t;
  const int b1_off = BIAS_OFF + ((Cout * 4 + BIAS_ROUND - 1) / BIAS_ROUND) * BIAS_ROUND;

  const kv_i32x4 rx = kv_rsrc4(p.x, p.M * p.ldx * 2);
  const kv_i32x4 rw3 = kv_rsrc4(p.w, Cout * p.Kpad * 2);
  const kv_i32x4 rw1 = kv_rsrc4(p.w_t, N1 * Cout * 2);
  const kv_i32x4 rr = kv_rsrc4(p.res, p.M * p.ldr * 2);
  const kv_i32x4 rb3 = kv_rsrc4(p.bias, Cout * 4);
  const kv_i32x4 rb1 = kv_rsrc4(p.bias_t, N1 * 4);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.M * p.ldy * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz =
      __builtin_amdgcn_make_buffer_rsrc(p.z, (short)0, p.M * p.ldz * 2, 0x00020000);

  // DMA lane roles: 8 rows x 8 chunks of 16 B per instruction; row r's logical chunk
  // (lane & 7) ^ sw(r) lands at position lane & 7 (the read side XORs it back)
  const int lrow = lane >> 3, pch = lane & 7;
  int arow_off[2], r_src[2], lc8[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wv * 2 + i) * 8 + lrow;
    const int lc = pch ^ sm_sw(row);
    lc8[i] = lc * 8;
    const int m = m0 + row;
    arow_off[i] = m < p.M ? (m * p.ldx + p.x_coff + lc * 8) * 2 : kSmOOB;
    r_src[i] = m < p.M ? (m * p.ldr + p.r_coff + lc * 8) * 2 : kSmOOB;
  }
  int w3_src[BPW], w1_src[BPW], brow[BPW];
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    brow[i] = (wv * BPW + i) * 8 + lrow;
    const int bch = (pch ^ sm_sw(brow[i])) * 8;
    w3_src[i] = (brow[i] * p.Kpad + bch) * 2;
    w1_src[i] = (brow[i] * Cout + bch) * 2;
  }

  // ring stage (tile tt, step jj): jj < SY -> W3 rows 64 tt.., K chunks jj KS2 ..; else W1
  // rows 64 ((jj - SY) KS2 + c).., K = y channels 64 tt..
  auto issue_B = [&](int tt, auto JJ) __attribute__((always_inline)) {
    constexpr int jj = decltype(JJ)::value;
    const int s = tt * SPT + jj;
    char* dst = lds + B_OFF + (s % D) * B_STAGE;
#pragma unroll
    for (int c = 0; c < KS2; ++c)
#pragma unroll
      for (int i = 0; i < BPW; ++i) {
        char* d = dst + c * B_CHUNK + (wv * BPW + i) * 1024;
        if constexpr (jj < SY) {
          const int n = tt * 64 + brow[i];
          const int v = (tt < ntiles && n < Cout) ? w3_src[i] + (tt * 64 * p.Kpad + (jj * KS2 + c) * 64) * 2 : kSmOOB;
          kv_lds_dma16(rw3, d, v);
        } else {
          const int zc = (jj - SY) * KS2 + c;
          const int zr = zc * 64 + brow[i];
          const int v = (tt < ntiles && zr < N1) ? w1_src[i] + (zc * 64 * Cout + tt * 64) * 2 : kSmOOB;
          kv_lds_dma16(rw1, d, v);
        }
      }
  };
  auto issue_R = [&](int tt) __attribute__((always_inline)) {
    char* dst = lds + R_OFF + (tt % RD) * R_SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = tt * 64 + lc8[i];
      const int v = (tt < ntiles && n < Cout && r_src[i] != kSmOOB) ? r_src[i] + tt * 128 : kSmOOB;
      kv_lds_dma16_nt(rr, dst + (wv * 2 + i) * 1024, v);  // see the y store
    }
  };

  // ---- prologue ---------------------------------------------------------------
  for (int i = 0; i < (Cout * 4 + BIAS_ROUND - 1) / BIAS_ROUND; ++i) {
    const int off = (i * NW + wv) * 1024;
    kv_lds_dma16(rb3, lds + BIAS_OFF + off, off + lane * 16);
  }
  for (int i = 0; i < (N1 * 4 + BIAS_ROUND - 1) / BIAS_ROUND; ++i) {
    const int off = (i * NW + wv) * 1024;
    kv_lds_dma16(rb1, lds + b1_off + off, off + lane * 16);
  }
  // AREG: the wave's A fragments straight from global memory into VGPRs, in MFMA operand
  // layout (lane (fr, fh) holds 8 consecutive K values of row wm*32 + tm*16 + fr).  Opaque
  // loads issued BEFORE the ring prologue, then one counted wait that leaves the prologue
  // DMAs in flight (an ordinary load would make hipcc drain everything at its first use,
  // and -- loop-carried -- again at every tile: the conv3 MFMAs read these every tile)
  typedef unsigned int sm_u32x4 __attribute__((ext_vector_type(4)));
  sm_u32x4 araw[AREG ? NC3 : 1][2][2];
  const int fr = lane & 15, fh = lane >> 4;
  if constexpr (AREG) {
#pragma unroll
    for (int kc = 0; kc < NC3; ++kc)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) {
          const int m = m0 + wm * 32 + tm * 16 + fr;
          const int k = kc * 64 + ks * 32 + fh * 8;
          const int off = (m < p.M && k < p.Cin) ? (m * p.ldx + p.x_coff + k) * 2 : kSmOOB;
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"
                       : "=v"(araw[kc][ks][tm]) : "v"(off), "s"(rx) : "memory");
        }
  }
  if constexpr (!AREG) {
#pragma unroll
    for (int kc = 0; kc < NC3; ++kc)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        char* dst = lds + kc * (BM * 128) + (wv * 2 + i) * 1024;
        const int v = (arow_off[i] != kSmOOB && kc * 64 + lc8[i] < p.Cin) ? arow_off[i] + kc * 128 : kSmOOB;
        kv_lds_dma16_nt(rx, dst, v);  // A: read here for the last time (see the y store)
      }
  }
#pragma unroll
  for (int t = 0; t < RD - 1; ++t) issue_R(t);
  sm_static_for<D - 1>([&](auto JJ) __attribute__((always_inline)) {
    constexpr int s = decltype(JJ)::value;
    issue_B(s / SPT, SmIC<s % SPT>{});
  });
  bf16x8 areg[AREG ? NC3 : 1][2][2];
  if constexpr (AREG) {
    // A landed: every op issued after it is a ring-prologue DMA (R(0 .. RD-2), B(0 .. D-2))
    sm_wait_vm<(RD - 1) * S::kR + (D - 1) * S::kB>();
#pragma unroll
    for (int kc = 0; kc < NC3; ++kc)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) {
          asm volatile("" : "+v"(araw[kc][ks][tm]));  // no consumer above the wait
          areg[kc][ks][tm] = __builtin_bit_cast(bf16x8, araw[kc][ks][tm]);
        }
  }

  floatx4 acc[2][2];
  floatx4 accz[NZC][2][2];
#pragma unroll
  for (int zc = 0; zc < NZC; ++zc)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) accz[zc][a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  // one 64-deep K chunk: acc[tn][tm] += Bs[wn*32 + tn*16 ..] . As[wm*32 + tm*16 ..]^T
  auto mma64 = [&](const char* As, const char* Bs, floatx4 (&c)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int q = ks * 4 + fh;
      bf16x8 af[2], bfg[2];
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        const int row = wm * 32 + tm * 16 + fr;
        af[tm] = *reinterpret_cast<const bf16x8*>(As + row * 128 + ((q ^ sm_sw(row)) << 4));
      }
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        const int row = wn * 32 + tn * 16 + fr;
        bfg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + ((q ^ sm_sw(row)) << 4));
      }
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
          c[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[tn], af[tm], c[tn][tm], 0, 0, 0);
    }
  };

  // conv3 K chunk kc with A from registers: acc[tn][tm] += Bs[wn*32 + tn*16 ..] . A^T
  auto mma64r = [&](int kc_unused, const bf16x8 (&a)[2][2], const char* Bs, floatx4 (&c)[2][2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int q = ks * 4 + fh;
      bf16x8 bfg[2];
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        const int row = wn * 32 + tn * 16 + fr;
        bfg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + ((q ^ sm_sw(row)) << 4));
      }
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
          c[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[tn], a[ks][tm], c[tn][tm], 0, 0, 0);
    }
  };

  // XP: weight fragments of one ring stage, [c][ks][tn], two sets by step parity
  bf16x8 bset[XP ? 2 : 1][XP ? KS2 : 1][2][2];
  auto read_B = [&](bf16x8 (&dst)[XP ? KS2 : 1][2][2], const char* Bs) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < (XP ? KS2 : 1); ++c)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          const int row = wn * 32 + tn * 16 + fr, q = ks * 4 + fh;
          dst[c][ks][tn] =
              *reinterpret_cast<const bf16x8*>(Bs + c * B_CHUNK + row * 128 + ((q ^ sm_sw(row)) << 4));
        }
  };
  // one 64-deep K chunk with B from registers: A from VGPRs (conv3) or from LDS (conv1: y)
  auto mma_xr = [&](const bf16x8 (&b)[2][2], const bf16x8 (&a)[2][2], floatx4 (&c)[2][2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
          c[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][tn], a[ks][tm], c[tn][tm], 0, 0, 0);
  };
  auto mma_xl = [&](const bf16x8 (&b)[2][2], const char* As, floatx4 (&c)[2][2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int q = ks * 4 + fh;
      bf16x8 af[2];
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        const int row = wm * 32 + tm * 16 + fr;
        af[tm] = *reinterpret_cast<const bf16x8*>(As + row * 128 + ((q ^ sm_sw(row)) << 4));
      }
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
          c[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][tn], af[tm], c[tn][tm], 0, 0, 0);
    }
  };

  dispatch_act(p.act, true, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
    for (int t = 0; t < ntiles; ++t) {
      const bool warm = t < S::kSteady;
      char* Rs = lds + R_OFF + (t % RD) * R_SLOT;
      sm_static_for<SPT>([&](auto JC) __attribute__((always_inline)) {
        constexpr int j = decltype(JC)::value;
        const int s = t * SPT + j;
        if constexpr (j == SY) {
          // ---- y epilogue of tile t: residual slot t % RD holds R(t); y overwrites it
          if (warm) sm_wait_vm<S::safe_E()>();
          else sm_wait_vm<S::wE(S::kFar)>();
          sm_lds_barrier();
          const float* bias_t = reinterpret_cast<const float*>(lds + BIAS_OFF) + t * 64;
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) {
            const int c0 = wn * 32 + tn * 16 + fh * 4;
            const float4 bv = *reinterpret_cast<const float4*>(bias_t + c0);
#pragma unroll
            for (int tm = 0; tm < 2; ++tm) {
              const int row = wm * 32 + tm * 16 + fr;
              bf16x4* ptr = reinterpret_cast<bf16x4*>(Rs + row * 128 + (((c0 >> 3) ^ sm_sw(row)) << 4) +
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
          sm_lds_barrier();
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int idx = tid + NT * i;
            const int row = idx >> 3, c = idx & 7;
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(Rs + row * 128 + ((c ^ sm_sw(row)) << 4));
            const int m = m0 + row, n = t * 64 + c * 8;
            const int off = (m < p.M && n < Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kSmOOB;
            // y non-temporal: re-read only as the residual two launches later (by then out
            // of the Infinity Cache anyway); z, read by the very next launch, stays cached
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(kv_i32x4, v), ry, off, 0, 2);
          }
        }
        if constexpr (j == 0) {
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        if constexpr (XP) {
          if (warm) sm_wait_vm<S::safe_XB(j)>();
          else sm_wait_vm<S::wXB(S::kFar, j)>();
        } else {
          if (warm) sm_wait_vm<S::safe_B(j)>();
          else sm_wait_vm<S::wB(S::kFar, j)>();
        }
        sm_lds_barrier();  // WAR: every wave's reads of the slot about to be refilled retired
        constexpr int jn = (j + D - 1) % SPT, tadv = (j + D - 1) / SPT;
        issue_B(t + tadv, SmIC<jn>{});
        if constexpr (j == 0) issue_R(t + RD - 1);
        const char* Bs = lds + B_OFF + (s % D) * B_STAGE;
        if constexpr (XP) {
          constexpr int cur = j & 1, nxt = cur ^ 1;  // SPT even: parity of s == parity of j
          if constexpr (j == 0) {
            if (t == 0) read_B(bset[cur], Bs);  // the first step has no predecessor
          }
          read_B(bset[nxt], lds + B_OFF + ((s + 1) % D) * B_STAGE);  // stage s + 1 landed
#pragma unroll
          for (int c = 0; c < KS2; ++c) {
            if constexpr (j < SY) mma_xr(bset[cur][c], areg[j * KS2 + c], acc);
            else mma_xl(bset[cur][c], Rs, accz[(j - SY) * KS2 + c]);
          }
        } else {
#pragma unroll
          for (int c = 0; c < KS2; ++c) {
            if constexpr (j < SY && AREG) mma64r(0, areg[j * KS2 + c], Bs + c * B_CHUNK, acc);
            else if constexpr (j < SY) mma64(lds + (j * KS2 + c) * (BM * 128), Bs + c * B_CHUNK, acc);
            else mma64(Rs, Bs + c * B_CHUNK, accz[(j - SY) * KS2 + c]);
          }
        }
      });
    }
  });

  // ---- z epilogue: ReLU(z + b1) staged through the (drained) residual slots -----------
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float* b1 = reinterpret_cast<const float*>(lds + b1_off);
  const bool relu_z = p.act_t == 1;
  sm_static_for<NZC>([&](auto ZC) __attribute__((always_inline)) {
    constexpr int zc = decltype(ZC)::value;
    char* Zs = lds + R_OFF + (zc % RD) * R_SLOT;
    if constexpr (zc > 0 && zc % RD == 0) __syncthreads();  // previous group's stores read it
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int c0 = wn * 32 + tn * 16 + fh * 4;
      const float4 bv = *reinterpret_cast<const float4*>(b1 + zc * 64 + c0);
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        const int row = wm * 32 + tm * 16 + fr;
        float v0 = accz[zc][tn][tm][0] + bv.x, v1 = accz[zc][tn][tm][1] + bv.y;
        float v2 = accz[zc][tn][tm][2] + bv.z, v3 = accz[zc][tn][tm][3] + bv.w;
        if (relu_z) {
          v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
        }
        bf16x4 o;
        o[0] = f2bf(v0); o[1] = f2bf(v1); o[2] = f2bf(v2); o[3] = f2bf(v3);
        *reinterpret_cast<bf16x4*>(Zs + row * 128 + (((c0 >> 3) ^ sm_sw(row)) << 4) + (c0 & 7) * 2) = o;
      }
    }
    if constexpr (zc % RD == RD - 1 || zc == NZC - 1) {
      __syncthreads();
      constexpr int z0 = zc - zc % RD;
#pragma unroll
      for (int g = z0; g <= zc; ++g) {
        const char* Zg = lds + R_OFF + (g % RD) * R_SLOT;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int idx = tid + NT * i;
          const int row = idx >> 3, c = idx & 7;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(Zg + row * 128 + ((c ^ sm_sw(row)) << 4));
          const int m = m0 + row, n = g * 64 + c * 8;
          const int off = (m < p.M && n < N1) ? (m * p.ldz + p.z_coff + n) * 2 : kSmOOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(kv_i32x4, v), rz, off, 0, 0);
        }
      }
    }
  });
}

typedef void (*SmFn)(const KvConvParams, int);

struct SmTile {
  int nc3, nzc, d, rd, nw, ks2, areg;
  SmFn fn;
};

template <int NC3, int NZC, int D, int RD, int NW = 8, int KS2 = 1, bool AREG = false,
          bool XP = false>
constexpr SmTile sm_tile() {
  return SmTile{NC3, NZC, D, RD, NW, KS2, AREG ? 1 : 0,
                &conv_seam_kernel<NC3, NZC, D, RD, NW, KS2, AREG, XP>};
}

// LDS = A (K3 x BM x 2) + d x ks2 x 8 KB ring + rd x BM x 128 B residual ring + bias tables.
// Batch 640, same box (profiles/r4_seam_probe.md): the 8-wave 8-KB-stage forms
// run ~0.44 us per ring step, latency-bound on the one shared weight ring; the 4-wave forms
// put two workgroups on a CU, the KS2 = 2 forms halve the waits and barriers per MFMA.
static const SmTile kSmTiles[] = {
    // stage 2 (K3 128, Cout 512 -> N1 128): 4 waves, two workgroups per CU first
    // (profiles/r4_v2_seam_probe_b640.md: 305 us vs 337 for the 8-wave form, 358 unfused)
    sm_tile<2, 2, 4, 3, 4>(),
    sm_tile<2, 2, 6, 3>(),
    sm_tile<2, 2, 4, 3, 8, 2>(),
    sm_tile<2, 2, 6, 3, 4, 1, true>(),   // A in VGPRs (4 waves: 80 KB)
    sm_tile<2, 2, 6, 3, 8, 2, true>(),   // A in VGPRs, 16-KB stages
    // stage 2 -> 3 (N1 256): A in VGPRs, 16-KB stages first (388 vs 408 us, 414 unfused)
    sm_tile<2, 4, 6, 3, 8, 2, true>(),
    sm_tile<2, 4, 6, 3>(),
    // stage 3 (K3 256, Cout 1024 -> N1 256): A in VGPRs with a 4-slot residual ring (3 tiles,
    // 48 KB, of residual in flight per CU) and the cross-step weight-fragment prefetch first:
    // 193.4 us vs 198.6 without the prefetch, 224 unfused (profiles/r4_v4_seam_probe_b640.md).
    // The prefetch lost on the stage-2 forms (327 vs 321 us, 401 vs 385 at 2 -> 3) and was
    // dropped there; the deeper residual ring lost on stage 2 too (r4_v3 probe)
    sm_tile<4, 4, 4, 4, 8, 2, true, true>(),
    sm_tile<4, 4, 4, 4, 8, 2, true>(),
    sm_tile<4, 4, 3, 2, 8, 2>(),
    sm_tile<4, 4, 5, 2>(),
    sm_tile<4, 4, 3, 2, 4>(),
    sm_tile<4, 4, 6, 2, 8, 2, true>(),   // A in VGPRs, 5 x 16 KB of weights in flight
    sm_tile<4, 4, 8, 3, 8, 1, true>(),
    sm_tile<4, 4, 3, 5, 8, 2, true>(),
    // stage 3 -> 4 (N1 512): not taken by the model (level with unfused at b640)
    sm_tile<4, 8, 4, 3>(),
};

int sm_lds_bytes(const SmTile& e, int cout, int n1) {
  const int bm = 16 * e.nw, round = e.nw * 1024;
  return (e.areg ? 0 : e.nc3 * bm * 128) + e.d * e.ks2 * 64 * 128 + e.rd * bm * 128 +
         ((cout * 4 + round - 1) / round) * round + ((n1 * 4 + round - 1) / round) * round;
}

}  // namespace

int seam_num_tiles() { return (int)(sizeof(kSmTiles) / sizeof(kSmTiles[0])); }

// the first tile (table order) that takes the shape; -1 if none does
int seam_pick_tile(const KvConvParams* p) {
  for (int i = 0; i < seam_num_tiles(); ++i) {
    const SmTile& e = kSmTiles[i];
    if (p->Kpad == e.nc3 * 64 && p->n_t == e.nzc * 64 && sm_lds_bytes(e, p->Cout, p->n_t) <= kSmLdsMax)
      return i;
  }
  return -1;
}

int seam_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= seam_num_tiles()) return -6;
  const SmTile& e = kSmTiles[tile];
  // plain conv3 + residual only (the dual conv3 + downsample form keeps too much A resident)
  if (p->mode != 1 || !p->res || p->x2 || !p->w_t || !p->z || p->in_u8 || p->pair_1x1) return -8;
  if (p->Kpad != e.nc3 * 64 || p->Cin > p->Kpad || p->n_t != e.nzc * 64 || p->Cout % 64) return -8;
  if (p->ldx % 8 || p->x_coff % 8 || p->ldy % 8 || p->y_coff % 8 || p->ldr % 8 || p->r_coff % 8 ||
      p->ldz % 8 || p->z_coff % 8 || p->x_coff + p->Cin > p->ldx || p->y_coff + p->Cout > p->ldy ||
      p->r_coff + p->Cout > p->ldr || p->z_coff + p->n_t > p->ldz)
    return -8;
  if ((long long)p->M * p->ldy * 2 >= kSmOOB || (long long)p->M * p->ldr * 2 >= kSmOOB ||
      (long long)p->M * p->ldx * 2 >= kSmOOB || (long long)p->M * p->ldz * 2 >= kSmOOB ||
      (long long)p->Cout * p->Kpad * 2 >= kSmOOB || (long long)p->n_t * p->Cout * 2 >= kSmOOB)
    return -9;
  const int lds = sm_lds_bytes(e, p->Cout, p->n_t);
  if (lds > kSmLdsMax) return -11;
  const int nbm = (p->M + 16 * e.nw - 1) / (16 * e.nw), ntiles = p->Cout / 64;
  if (nbm <= 0 || ntiles <= 0) return 0;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(e.fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(e.fn, dim3((unsigned)nbm), dim3(64 * e.nw), (unsigned)lds, stream, *p, ntiles);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
