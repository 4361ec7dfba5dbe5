// K1/K2/K3 v2 — implicit-GEMM conv with LDS-DMA (buffer_load ... lds) staging, gfx950.
//
// Second-generation main loop (the v1 register-staged kernel is conv_igemm.hip; the
// autotuner picks per layer between both families).  What changes, and why (rocprof
// PMC on v1: 2-3 VALU per MFMA on the 3x3 layers = VALU-issue-bound beside the
// MFMAs, and 33-70 % of wave cycles parked on waits):
//  * Operands go global -> LDS with buffer_load_dwordx4 ... lds: no staging VGPRs,
//    no ds_write instructions, and the buffer descriptor's range check turns every
//    out-of-image tap (conv padding, M/N/K tails) into zeros for free: an invalid lane
//    just gets an offset past num_records.
//  * Address work per K step is one scalar soffset (weights, 1x1 activations) or, for
//    KxK convs with Cin % 64 == 0, a wave-uniform tap offset plus a per-row tap-valid
//    bit (precomputed once): ~3 VALU per staged row instead of ~10.
//  * v_mfma_f32_32x32x16_bf16: 32 cycles per MFMA leave 24 issue cycles for VALU/LDS
//    (16x16x32 leaves 8), and half the LDS fragment bytes per FLOP.
//  * LDS image [row][64] bf16, 16-B chunk c of row r stored at c ^ ((r >> 1) & 7):
//    the DMA writes are lane-linear (swizzle applied on the SOURCE address, guide rule
//    21) and both the 32x32x16 and 16x16x32 fragment reads are conflict-free under the
//    ds_read_b128 lane grouping (derivation: docs/kernels.md).
//  * D-slot ring (D = 2..4): K step k+D-1 is issued before the MFMAs of step k.  Every
//    step issues the same number of DMA ops (steps past the end are all out of range),
//    so "step k landed" is an exact s_waitcnt vmcnt((D-2) * ops_per_step) that leaves
//    the younger steps in flight; one barrier per step.  D = 2 is the classic 2-phase
//    loop (guide §5.5 T3+T4); deeper rings trade LDS (occupancy) for latency hiding,
//    and the autotuner picks per layer.
//  * Fused epilogue (bias, residual before/after act, ReLU/SiLU) staged through LDS for
//    full-row 16-B stores, as in v1.
#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MF>
struct AccOf { typedef floatx16 type; static constexpr int n = 16; };
template <>
struct AccOf<16> { typedef floatx4 type; static constexpr int n = 4; };

namespace kvedge {
namespace {

constexpr int BK = 64;
constexpr int kOOB = 0x7ffffff0;  // byte offset beyond every tensor: buffer load returns 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t rs, bf16* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// MODE 0: KxK (or strided 1x1) conv with Cin % 64 == 0 -> tap uniform per K step
// MODE 1: 1x1 / stride 1 / pad 0 GEMM (A rows contiguous)
// MODE 3: generic gather, Cin % 8 == 0 (per-lane tap tracking)
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}

// BKT = K elements per ring stage.  64: 128-B rows, 8 rows per DMA instruction.  32: 64-B
// rows, 16 rows per instruction -- half the bytes per stage, so twice the stages fit the
// same LDS (a 128x128 tile can keep 4 K steps in flight at 2 workgroups per CU, D = 5).
//
// WM x WN waves: 4 (256 threads, up to 2 workgroups per CU) or 8 (512 threads, one
// workgroup per CU = 2 waves per SIMD).  The 8-wave 256x256 tile gives every wave a
// 128x64 (or 64x128) sub-tile -- 0.75 fragment reads per MFMA -- while keeping two waves
// per SIMD for latency hiding, which no 4-wave tile combines (a 4-wave 256x128 tile has
// the sub-tile but one wave per SIMD).
//
// MF = MFMA shape: 32 = v_mfma_f32_32x32x16_bf16, 16 = v_mfma_f32_16x16x32_bf16.  Same LDS
// image and the same fragment bytes per FLOP (a 16x16x32 fragment is 16 rows x 32 k, a
// 32x32x16 one 32 rows x 16 k: both one ds_read_b128); the 16x16x32 loop holds a higher
// clock under load (MI355X_MICROARCH.md, DVFS item 7) at twice the MFMA count.
//
// XP = true: the cross-stage pipelined main loop (v7 tiles, below the ring description).
template <int BM, int BN, int WM, int WN, int MODE, int D, int BKT = 64, int MF = 32,
          bool XP = false, bool DE = false, bool SK = false>
__global__ __launch_bounds__(64 * WM * WN, WM * WN == 4 ? 2 : 1) void conv_glds_kernel(
    const KvConvParams p) {
  constexpr int NW = WM * WN;     // waves per workgroup
  constexpr int NT = 64 * NW;     // threads per workgroup
  constexpr int BK = BKT;         // shadows the file-scope 64
  constexpr int CH = BK / 8;      // 16-B chunks per LDS row
  constexpr int RPI = 64 / CH;    // rows per DMA instruction (64 lanes x 16 B)
  constexpr int KS = BK / (MF == 32 ? 16 : 32);  // MFMA K steps per stage
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  static_assert(MF == 32 || MF == 16, "MFMA shape");
  using Acc = typename AccOf<MF>::type;
  constexpr int NACC = AccOf<MF>::n;
  constexpr int A_INS = BM / (NW * RPI);  // DMA instructions per wave per stage
  constexpr int B_INS = BN / (NW * RPI);
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(BK == 64 || BK == 32, "BK");
  static_assert(A_INS >= 1 && B_INS >= 1, "tile too small for BK");
  static_assert((NW == 4 || NW == 8) && TM >= 1 && TN >= 1 && D >= 2 && D <= 6, "tile");
  // chunk swizzle of row r: ds_read_b128 of 16 rows x one logical chunk is conflict-free
  // BK = 32 rows are 64 B (4 chunks): MF = 16 reads take rows 0-15 with chunk quarter
  // lane >> 4, so a ds_read_b128 lane group mixes rows {0-3, 12-15} of one quarter with
  // rows {4-11} of the next; XOR (row >> 2) & 2 makes the 16 (row & 3, chunk) slots of
  // every group distinct (the (row >> 2) & 3 form is 2-way conflicted there: PMC
  // SQ_LDS_BANK_CONFLICT 19x, profiles/r3_v2_pmc_s3c2_b256)
  auto sw = [](int r) __attribute__((always_inline)) {
    return BK == 64 ? ((r >> 1) & 7) : (MF == 16 ? ((r >> 2) & 2) : ((r >> 2) & 3));
  };
  __shared__ __attribute__((aligned(16))) bf16 smem[D * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.Cout + BN - 1) / BN;
  // split-K (SK): the p.ksplit consecutive blocks of a tile take equal shares of its K steps
  const int kz = SK ? (int)(blockIdx.x % p.ksplit) : 0;
  const int t = SK ? (int)(blockIdx.x / p.ksplit) : xcd_remap(blockIdx.x, nbm * nbn);
  const int m0 = (t / nbn) * BM, n0 = (t % nbn) * BN;
  const int nk_all = p.Kpad / BKT;
  const int kb = SK ? kz * nk_all / p.ksplit : 0;                  // first K step (absolute)
  const int ke = SK ? (kz + 1) * nk_all / p.ksplit : nk_all;      // one past the last

  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, p.N * p.H * p.W * p.ldx * 2);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w, p.Cout * p.Kpad * 2);
  const __amdgpu_buffer_rsrc_t rx2 =
      make_rsrc(MODE == 4 ? p.x2 : p.x, MODE == 4 ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);

  // ---- residual prefetch: issued before the K loop, consumed by the epilogue, so its
  // latency hides under the GEMM instead of serialising after it (memory-bound layers).
  // The epilogue stages the C tile through LDS in NSPLIT column halves when the whole
  // (padded) tile does not fit the ring (256x256); chunk j of half h -> rpre[h * PERH + j].
  constexpr int NSPLIT = BM * (BN + 8) <= D * STAGE ? 1 : 2;
  constexpr int BNH = BN / NSPLIT;  // columns per epilogue pass
  static_assert(WTN <= BNH && BNH % WTN == 0, "a wave's columns lie in one epilogue pass");
  static_assert(BM * (BNH + 8) <= D * STAGE, "C tile (pass) fits");
  constexpr int CPR = BNH / 8;
  constexpr int PERH = BM * CPR / NT;
  constexpr int PER = PERH * NSPLIT;
  constexpr bool kPrefetchRes = !DE && PER <= 8;
  bf16x8 rpre[kPrefetchRes ? PER : 1];
  if (kPrefetchRes && p.res) {
    const bf16* R = reinterpret_cast<const bf16*>(p.res);
#pragma unroll
    for (int h = 0; h < NSPLIT; ++h)
#pragma unroll
      for (int j = 0; j < PERH; ++j) {
        const int idx = threadIdx.x + NT * j;
        const int m = m0 + idx / CPR, n = n0 + h * BNH + (idx % CPR) * 8;
        if (m < p.M && n < p.Cout)
          rpre[h * PERH + j] = *reinterpret_cast<const bf16x8*>(R + (size_t)m * p.ldr + p.r_coff + n);
      }
  }

  // ---- per-lane source descriptors (constant over the K loop) -------------
  const int lrow = lane / CH, pch = lane % CH;
  int a_off[A_INS];   // MODE 0: pixel-row base offset (elements); MODE 1/4: full byte offset
  int a_off2[A_INS];  // MODE 4: byte offset of the strided second source
  unsigned a_msk[A_INS];
  int a_lc[A_INS];
  int a_h0[A_INS], a_w0[A_INS];  // MODE 3
  const int HoWo = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int row = (wv * A_INS + i) * RPI + lrow;
    const int lc = pch ^ sw(row);
    a_lc[i] = lc;
    const int m = m0 + row;
    a_msk[i] = 0u;
    a_h0[i] = -(1 << 28);
    a_w0[i] = -(1 << 28);
    a_off2[i] = kOOB;
    if (MODE == 1 || MODE == 4) {
      a_off[i] = m < p.M ? (m * p.ldx + p.x_coff + lc * 8) * 2 : kOOB;
      if (MODE == 4 && m < p.M) {
        const int img = m / HoWo;
        const int rem = m - img * HoWo;
        const int ho = rem / p.Wo, wo = rem - (rem / p.Wo) * p.Wo;
        a_off2[i] = (((img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2) * p.ldx2 + lc * 8) * 2;
      }
    } else {
      a_off[i] = 0;
      if (m < p.M) {
        const int img = m / HoWo;
        const int rem = m - img * HoWo;
        const int ho = rem / p.Wo, wo = rem - (rem / p.Wo) * p.Wo;
        const int h0 = ho * p.stride - p.pad, w0 = wo * p.stride - p.pad;
        a_h0[i] = h0;
        a_w0[i] = w0;
        a_off[i] = ((img * p.H + h0) * p.W + w0) * p.ldx + p.x_coff + lc * 8;  // may be < 0
        if (MODE == 0) {
          unsigned msk = 0;
          for (int r = 0; r < p.KH; ++r)
            for (int s = 0; s < p.KW; ++s)
              if ((unsigned)(h0 + r) < (unsigned)p.H && (unsigned)(w0 + s) < (unsigned)p.W)
                msk |= 1u << (r * p.KW + s);
          a_msk[i] = msk;
        }
      }
    }
  }
  int b_off[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int row = (wv * B_INS + i) * RPI + lrow;
    const int lc = pch ^ sw(row);
    const int n = n0 + row;
    b_off[i] = n < p.Cout ? (n * p.Kpad + lc * 8) * 2 : kOOB;
  }
  // MODE 3 per-lane incremental tap state, one per A instruction (lc differs per row)
  int g_tap[A_INS], g_c[A_INS];
  if (MODE == 3) {
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      int c = a_lc[i] * 8 + kb * BK, tap = 0;
      while (c >= p.Cin) { c -= p.Cin; ++tap; }
      g_tap[i] = tap;
      g_c[i] = c;
    }
  }

  // MODE 0 K-step position (tap row r, tap col s, channel base c0), advanced once per
  // issue(): the issue order is kt = 0, 1, 2, ... on both pipelines, so the per-step
  // k0 / Cin and tap / KW divisions (a ~20-instruction VALU expansion each: there is no
  // scalar divide) become a compare-and-bump on wave-uniform values
  int k_c0 = 0, k_r = 0, k_s = 0;
  if (SK && MODE == 0 && kb > 0) {  // split-K: start the tap walk at this slice's first step
    const int kbase = kb * BK, tap = kbase / p.Cin;
    k_c0 = kbase - tap * p.Cin;
    k_r = tap / p.KW;
    k_s = tap - k_r * p.KW;
  }
  auto issue = [&](int stage, int kt_rel) {
    const int kt = kt_rel + kb;  // absolute K step
    bf16* As = smem + stage * STAGE;
    bf16* Bs = As + BM * BK;
    if (MODE == 1) {
      const int kbase = kt * BK;
      if (kbase + BK <= p.Cin) {  // wave-uniform: no K tail in this step, no per-lane select
#pragma unroll
        for (int i = 0; i < A_INS; ++i) glds16(rx, As + (wv * A_INS + i) * 512, a_off[i], kbase * 2);
      } else {
#pragma unroll
        for (int i = 0; i < A_INS; ++i) {
          const int v = (kbase + a_lc[i] * 8 < p.Cin) ? a_off[i] : kOOB;
          glds16(rx, As + (wv * A_INS + i) * 512, v, kbase * 2);
        }
      }
    } else if (MODE == 4) {
      const int kbase = kt * BK;  // K1 and K - K1 are multiples of 64: no tails
      if (kbase < p.K1) {
#pragma unroll
        for (int i = 0; i < A_INS; ++i)
          glds16(rx, As + (wv * A_INS + i) * 512, a_off[i], kbase * 2);
      } else {
#pragma unroll
        for (int i = 0; i < A_INS; ++i)
          glds16(rx2, As + (wv * A_INS + i) * 512, a_off2[i], (kbase - p.K1) * 2);
      }
    } else if (MODE == 0) {
      const int c0 = k_c0, r = k_r, s = k_s;  // wave-uniform
      const int tap = r * p.KW + s;
      const int toff = (r * p.W + s) * p.ldx + c0;  // elements, wave-uniform
      k_c0 += BK;  // Cin % 64 == 0 in MODE 0: a K step never straddles two taps
      if (k_c0 >= p.Cin) {
        k_c0 = 0;
        if (++k_s == p.KW) { k_s = 0; ++k_r; }
      }
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        // a_off may be negative (top/left padding rows); only valid taps form an address
        const bool ok = tap < p.KH * p.KW && ((a_msk[i] >> tap) & 1u);
        const int v = ok ? (a_off[i] + toff) * 2 : kOOB;
        glds16(rx, As + (wv * A_INS + i) * 512, v, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int tap = g_tap[i];
        const int r = tap / p.KW, s = tap - (tap / p.KW) * p.KW;
        const int hi = a_h0[i] + r, wi = a_w0[i] + s;
        const bool ok = tap < p.KH * p.KW && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        const int v = ok ? (a_off[i] - a_lc[i] * 8 + (r * p.W + s) * p.ldx + g_c[i]) * 2 : kOOB;
        glds16(rx, As + (wv * A_INS + i) * 512, v, 0);
        int c = g_c[i] + BK;
        while (c >= p.Cin) { c -= p.Cin; ++g_tap[i]; }
        g_c[i] = c;
      }
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) glds16(rw, Bs + (wv * B_INS + i) * 512, b_off[i], kt * BK * 2);
  };

  Acc acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b)
#pragma unroll
      for (int e = 0; e < NACC; ++e) acc[a][b][e] = 0.f;

  // fragment lane roles: 32x32x16 -> row lane & 31, k half lane >> 5 (8 of 16);
  // 16x16x32 -> row lane & 15, k quarter lane >> 4 (8 of 32)
  const int fr = lane & (MF - 1), fh = lane / MF;
  auto compute = [&](int stage) {
    const bf16* As = smem + stage * STAGE;
    const bf16* Bs = As + BM * BK;
    // fragments double-buffered in registers: the ds_reads of step ks+1 are issued
    // before the MFMAs of step ks, so LDS latency hides under the MFMA pipe instead of
    // an lgkmcnt(0) stall in front of every group of MFMAs
    bf16x8 af[2][TM], bfg[2][TN];
    auto load = [&](int buf, int ks) __attribute__((always_inline)) {
      const int q = ks * (64 / MF) + fh;  // logical 16-B chunk of the row
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * MF + fr;
        af[buf][tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((q ^ sw(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * MF + fr;
        bfg[buf][tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((q ^ sw(row)) << 3));
      }
    };
    load(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks < KS - 1) load((ks + 1) & 1, ks + 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          if constexpr (MF == 32)
            acc[tn][tm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfg[ks & 1][tn], af[ks & 1][tm],
                                                                  acc[tn][tm], 0, 0, 0);
          else
            acc[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[ks & 1][tn], af[ks & 1][tm],
                                                                  acc[tn][tm], 0, 0, 0);
        }
    }
    // pin the order for the scheduler (it otherwise re-coalesces both register sets):
    // reads(0) | reads(1) MFMAs(0) | reads(2) MFMAs(1) | reads(3) MFMAs(2) | MFMAs(3)
    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks < KS - 1) __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
    }
  };

  const int nk = ke - kb;
  if constexpr (XP) {
    // v7 cross-stage pipeline.  The ring loop above opens every stage with its own
    // fragment reads AFTER the stage barrier, so each stage starts with an LDS-latency
    // bubble in which no wave of the workgroup has an MFMA to issue (8 waves x 12 reads
    // = 96 KB queue at 256 B/clk).  Here a phase (one stage = one MFMA k-step) issues
    // the fragment reads of the NEXT stage into the other register set before its own
    // MFMAs, so the MFMA stream never waits for LDS:
    //   phase kt:  DMA stage kt+D-1 -> slot of stage kt-1      (WAR: its reads fed the
    //              MFMAs of phase kt-1, which every wave issued before the last barrier)
    //              ds_read stage kt+1 -> register set (kt+1)&1  (RAW: stage kt+1 was
    //              waited for (own vmcnt) and published (barrier) at the end of kt-1)
    //              MFMAs of stage kt from register set kt&1
    //              vmcnt: stage kt+2 landed (D-3 younger stages in flight); s_barrier
    // One raw barrier per stage, never a vmcnt(0) inside the loop.
    static_assert(KS == 1 && D >= 4, "XP: one MFMA k-step per stage and >= 4 ring slots");
    constexpr int OPS = A_INS + B_INS;
    bf16x8 af0[TM], bg0[TN], af1[TM], bg1[TN];
    auto ld = [&](bf16x8 (&af)[TM], bf16x8 (&bg)[TN], int slot) __attribute__((always_inline)) {
      const bf16* As = smem + slot * STAGE;
      const bf16* Bs = As + BM * BK;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * MF + fr;
        af[tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((fh ^ sw(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * MF + fr;
        bg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((fh ^ sw(row)) << 3));
      }
    };
    auto mm = [&](bf16x8 (&af)[TM], bf16x8 (&bg)[TN]) __attribute__((always_inline)) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          if constexpr (MF == 32)
            acc[tn][tm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bg[tn], af[tm], acc[tn][tm], 0, 0, 0);
          else
            acc[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bg[tn], af[tm], acc[tn][tm], 0, 0, 0);
        }
    };
    // interleave: this phase's DMA issue and next-stage reads between the first MFMAs
    auto order = [&]() __attribute__((always_inline)) {
      constexpr int NR = TM + TN, NM = TM * TN;
      static_assert(NM >= 2 * NR, "enough MFMAs to cover the reads");
#pragma unroll
      for (int i = 0; i < OPS; ++i) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NM - 2 * NR, 0);
    };
#pragma unroll
    for (int s = 0; s < D - 1; ++s) issue(s, s);
    wait_vm<(D - 2) * OPS>();  // stage 0 landed (this wave's part)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    ld(af0, bg0, 0);
    wait_vm<(D - 3) * OPS>();  // stage 1
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    auto phase = [&](int kt, bf16x8 (&ca)[TM], bf16x8 (&cb)[TN], bf16x8 (&na)[TM],
                     bf16x8 (&nb)[TN]) __attribute__((always_inline)) {
      issue((kt + D - 1) % D, kt + D - 1);
      if (kt + 1 < nk) ld(na, nb, (kt + 1) % D);
      mm(ca, cb);
      order();
      wait_vm<(D - 3) * OPS>();  // stage kt+2 landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      phase(kt, af0, bg0, af1, bg1);
      phase(kt + 1, af1, bg1, af0, bg0);
    }
    if (kt < nk) phase(kt, af0, bg0, af1, bg1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land on the C tile
  } else if (D == 2) {
    issue(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // stage `cur` landed for every wave; stage cur^1 no longer read
      if (kt + 1 < nk) issue(cur ^ 1, kt + 1);
      compute(cur);
    }
  } else {
    // steps >= nk are issued too (all lanes out of range or never read) so that every
    // step is exactly A_INS + B_INS VMEM ops per wave and the wait below is exact
#pragma unroll
    for (int s = 0; s < D - 1; ++s) issue(s, s);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      wait_vm<(D - 2) * (A_INS + B_INS)>();  // step kt landed (this wave's part)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();           // ... for every wave; slot kt-1 free
      asm volatile("" ::: "memory");
      issue(cur == 0 ? D - 1 : cur - 1, kt + D - 1);
      compute(cur);
      cur = cur == D - 1 ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land on the C tile
  }
  if constexpr (SK) {
    // ---- split-K: fp32 partial sums of this K slice into ws (no bias / act / residual:
    // the finalize kernel applies them once).  A lane holds, per MFMA block, channels
    // (MF 32) 8g + 4fh + j / (MF 16) 4fh + j of pixel fr.
    float* __restrict__ ws = p.ws;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int m = m0 + wm * WTM + tm * MF + fr;
#pragma unroll
        for (int e = 0; e < NACC; ++e) {
          const int n = n0 + wn * WTN + tn * MF + (MF == 32 ? (e >> 2) * 8 : 0) + fh * 4 + (e & 3);
          if (m < p.M && n < p.Cout) unsafeAtomicAdd(ws + (size_t)m * p.Cout + n, acc[tn][tm][e]);
        }
      }
    return;
  }
  if constexpr (DE) {
    // ---- direct epilogue (no LDS C tile, no barrier): each lane holds 4 consecutive
    // channels of one pixel per 16x16 block; v_permlane16_swap between the blocks tn and
    // tn+1 (row 1 of one register <-> row 0 of the other, rows 3 <-> 2) leaves every lane
    // with 8 consecutive channels of its pixel -> one 16-B store per block pair (64 B per
    // pixel per wave instruction).  Rows 0..3 of the wave (lane >> 4) end up holding
    // channels [16 tn, +8), [16 (tn+1), +8), [16 tn + 8, +8), [16 (tn+1) + 8, +8).
    static_assert(MF == 16 && TN % 2 == 0, "DE: 16x16x32 accumulators, block pairs");
    const bool has_res = p.res != nullptr;
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y, p.M * p.ldy * 2);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.res, has_res ? p.M * p.ldr * 2 : 0);
    const int rho = lane >> 4;
    const int csel = 16 * (rho & 1) + 8 * (rho >> 1);  // channel offset within a block pair
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    dispatch_act(p.act, has_res, [&](auto A1, auto A2) __attribute__((always_inline)) {
      constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
#pragma unroll
      for (int tn = 0; tn < TN; tn += 2) {
        const int nb = n0 + wn * WTN + tn * 16;  // first channel of the block pair
        float4 bv0 = make_float4(0.f, 0.f, 0.f, 0.f), bv1 = bv0;
        if (p.bias) {
          if (nb + fh * 4 < p.Cout) bv0 = *reinterpret_cast<const float4*>(p.bias + nb + fh * 4);
          if (nb + 16 + fh * 4 < p.Cout) bv1 = *reinterpret_cast<const float4*>(p.bias + nb + 16 + fh * 4);
        }
        const int n = nb + csel;
        u32x4 rv[TM];
        if (has_res) {
#pragma unroll
          for (int tm = 0; tm < TM; ++tm) {
            const int m = m0 + wm * WTM + tm * 16 + fr;
            const int off = (m < p.M && n < p.Cout) ? (m * p.ldr + p.r_coff + n) * 2 : kOOB;
            rv[tm] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
          }
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          bf16x4 a, b;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[j] = f2bf(act_c<act1>(acc[tn][tm][j] + (&bv0.x)[j]));
            b[j] = f2bf(act_c<act1>(acc[tn + 1][tm][j] + (&bv1.x)[j]));
          }
          uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
          {
            const auto r0 = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
            const auto r1 = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
            ua.x = r0[0]; ub.x = r0[1];
            ua.y = r1[0]; ub.y = r1[1];
          }
          bf16x8 v = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
          if (has_res) {
            const bf16x8 r = __builtin_bit_cast(bf16x8, rv[tm]);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = f2bf(act_c<act2>((float)v[e] + (float)r[e]));
          }
          const int m = m0 + wm * WTM + tm * 16 + fr;
          const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kOOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, off, 0, 0);
        }
      }
    });
    return;
  }
  __syncthreads();

  // ---- fused epilogue through LDS (see conv_igemm.hip) ----------------------
  constexpr int CS = BNH + 8;
  const bool has_res = p.res != nullptr;
  bf16* __restrict__ Y = reinterpret_cast<bf16*>(p.y);
  const bf16* __restrict__ R = reinterpret_cast<const bf16*>(p.res);
  dispatch_act(p.act, has_res, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
#pragma unroll
    for (int h = 0; h < NSPLIT; ++h) {
      if (h > 0) __syncthreads();  // previous pass's C tile fully read
      if (wn * WTN / BNH == h) {   // this wave's columns belong to pass h
        // accumulator register r of a lane: 32x32 -> channel g*8 + fh*4 + j (g = r / 4,
        // j = r % 4), pixel lane & 31;  16x16 -> channel fh*4 + j, pixel lane & 15
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
          for (int g = 0; g < NACC / 4; ++g) {
            const int nl = wn * WTN + tn * MF + g * 8 + fh * 4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (p.bias && n0 + nl < p.Cout) bv = *reinterpret_cast<const float4*>(p.bias + n0 + nl);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
              const int ml = wm * WTM + tm * MF + fr;
              bf16x4 o;
              o[0] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 0] + bv.x));
              o[1] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 1] + bv.y));
              o[2] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 2] + bv.z));
              o[3] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 3] + bv.w));
              *reinterpret_cast<bf16x4*>(smem + ml * CS + nl - h * BNH) = o;
            }
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PERH; ++j) {
        const int idx = tid + NT * j;
        const int ml = idx / CPR, ch = idx % CPR;
        const int m = m0 + ml, n = n0 + h * BNH + ch * 8;
        if (m >= p.M || n >= p.Cout) continue;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + ml * CS + ch * 8);
        if (has_res) {
          const bf16x8 rv = kPrefetchRes ? rpre[kPrefetchRes ? h * PERH + j : 0]
                                         : *reinterpret_cast<const bf16x8*>(R + (size_t)m * p.ldr + p.r_coff + n);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(act_c<act2>((float)v[e] + (float)rv[e]));
        }
        *reinterpret_cast<bf16x8*>(Y + (size_t)m * p.ldy + p.y_coff + n) = v;
      }
    }
  });
}

}  // namespace

typedef void (*ConvKernelFn)(const KvConvParams);

template <int BM, int BN, int WM, int WN, int D = 2, int BKT = 64, int MF = 32, bool XP = false,
          bool DE = false, bool SK = false>
ConvKernelFn glds_get(int mode) {
  switch (mode) {
    case 0: return conv_glds_kernel<BM, BN, WM, WN, 0, D, BKT, MF, XP, DE, SK>;
    case 1: return conv_glds_kernel<BM, BN, WM, WN, 1, D, BKT, MF, XP, DE, SK>;
    case 4: return conv_glds_kernel<BM, BN, WM, WN, 4, D, BKT, MF, XP, DE, SK>;
    default: return conv_glds_kernel<BM, BN, WM, WN, 3, D, BKT, MF, XP, DE, SK>;
  }
}

// split-K finalize: y = act2(act1(ws + bias) (+ res)) -> bf16, and ws = 0 for the next layer
__global__ __launch_bounds__(256) void splitk_finalize_kernel(
    float* __restrict__ ws, const float* __restrict__ bias, const bf16* __restrict__ res,
    bf16* __restrict__ y, int M, int Cout, int ldy, int y_coff, int ldr, int r_coff, int act) {
  const int cpr = Cout >> 3;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)M * cpr) return;
  const int m = (int)(idx / cpr), c = (int)(idx - (long long)m * cpr) * 8;
  float4* src = reinterpret_cast<float4*>(ws + (size_t)m * Cout + c);
  const float4 a0 = src[0], a1 = src[1];
  src[0] = make_float4(0.f, 0.f, 0.f, 0.f);
  src[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  if (bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  bf16x8 o;
  dispatch_act(act, res != nullptr, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
    bf16x8 r;
    if (res) r = *reinterpret_cast<const bf16x8*>(res + (size_t)m * ldr + r_coff + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float u = act_c<act1>(v[e]);
      if (res) u = act_c<act2>((float)f2bf(u) + (float)r[e]);
      o[e] = f2bf(u);
    }
  });
  *reinterpret_cast<bf16x8*>(y + (size_t)m * ldy + y_coff + c) = o;
}

struct GldsTile {
  int bm, bn;
  ConvKernelFn (*get)(int);
  int nt = 256;  // threads per workgroup (64 x waves)
};

static const GldsTile kGldsTiles[] = {
    {128, 128, &glds_get<128, 128, 2, 2>},
    {128, 64, &glds_get<128, 64, 2, 2>},
    {64, 64, &glds_get<64, 64, 2, 2>},
    {256, 64, &glds_get<256, 64, 4, 1>},
    {64, 128, &glds_get<64, 128, 2, 2>},
    {256, 128, &glds_get<256, 128, 2, 2>},
    {128, 256, &glds_get<128, 256, 2, 2>},
    // deeper rings (3-4 K steps in flight); indices above are kept stable
    {128, 128, &glds_get<128, 128, 2, 2, 3>},
    {128, 64, &glds_get<128, 64, 2, 2, 3>},
    {64, 128, &glds_get<64, 128, 2, 2, 3>},
    {64, 64, &glds_get<64, 64, 2, 2, 4>},
    {128, 64, &glds_get<128, 64, 2, 2, 4>},
    // 128x64 / 64x128 per wave (0.75 fragment reads per MFMA instead of 1.0: the 3x3
    // layers are LDS-bandwidth-bound at 64x64 per wave), one workgroup per CU, 3 slots
    {256, 128, &glds_get<256, 128, 2, 2, 3>},
    {128, 256, &glds_get<128, 256, 2, 2, 3>},
    // narrow N (YOLO's 16/32-channel layers at 160^2 / 320^2): BN = 32, 4 waves along M
    {128, 32, &glds_get<128, 32, 4, 1>},
    {256, 32, &glds_get<256, 32, 4, 1>},
    // BN = 96 (3 x 32-wide MFMA blocks per wave, 4 waves along M): YOLO's 80-channel Detect
    // cls convs waste 17 % of the MFMA columns here instead of 37.5 % on a BN = 128 tile
    {128, 96, &glds_get<128, 96, 4, 1>},
    {256, 96, &glds_get<256, 96, 4, 1>},
    // 8 waves (512 threads), one workgroup per CU, two waves per SIMD: 256x256 with a
    // 128x64 / 64x128 sub-tile per wave (epilogue in two column passes), and 256x128 /
    // 128x256 with 64x64 per wave but the B / A tile shared by twice the waves
    {256, 256, &glds_get<256, 256, 2, 4>, 512},
    {256, 256, &glds_get<256, 256, 4, 2>, 512},
    {256, 128, &glds_get<256, 128, 4, 2>, 512},
    {128, 256, &glds_get<128, 256, 2, 4>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 3>, 512},
    // the same loops on v_mfma_f32_16x16x32_bf16 (MF = 16)
    {128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16>},
    {256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 2, 64, 16>, 512},
    // (BK = 32 rings -- glds_get<128, 128, 2, 2, 5, 32> etc., 4-5 K steps in flight at 2
    // workgroups per CU -- measured 10-40 % SLOWER than {128, 128} D = 2 on every 3x3 and
    // 1x1 layer of ResNet-50 at batch 640 (profiles/r1_v10_tile_probe_bk32.md): the 3x3
    // layers are not L2-latency-bound, so they are not instantiated)
};

int glds_num_tiles() { return (int)(sizeof(kGldsTiles) / sizeof(kGldsTiles[0])); }

// v7: the XP (cross-stage pipelined) main loop on BK = 32 rings, v_mfma_f32_16x16x32.
// Own index range after v6 so the older families keep their indices.
static const GldsTile kXpTiles[] = {
    {256, 256, &glds_get<256, 256, 2, 4, 4, 32, 16, true>, 512},  // 128 px x 64 ch per wave
    {256, 256, &glds_get<256, 256, 4, 2, 4, 32, 16, true>, 512},  // 64 px x 128 ch per wave
    {256, 256, &glds_get<256, 256, 2, 4, 5, 32, 16, true>, 512},  // 4 stages in flight
    {256, 256, &glds_get<256, 256, 4, 2, 5, 32, 16, true>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 6, 32, 16, true>, 512},  // N = 128 layers, 64 x 64
    {128, 256, &glds_get<128, 256, 2, 4, 6, 32, 16, true>, 512},
    // the plain ring loop on BK = 32 with the MF = 16 conflict-free swizzle (the round-1/2
    // BK = 32 rings were measured with a 2-way conflicted one); 4-wave forms fit <= 80 KB of
    // LDS, so two workgroups -- of this launch or of the other stream's -- share a CU and
    // one's epilogue overlaps the other's main loop
    {256, 256, &glds_get<256, 256, 4, 2, 4, 32, 16>, 512},        // 128 KB
    {256, 128, &glds_get<256, 128, 2, 2, 3, 32, 16>},             // 72 KB, 128 x 64 per wave
    {128, 256, &glds_get<128, 256, 2, 2, 3, 32, 16>},             // 72 KB, 64 x 128 per wave
    {128, 128, &glds_get<128, 128, 2, 2, 4, 32, 16>},             // 64 KB
    {128, 128, &glds_get<128, 128, 2, 2, 5, 32, 16>},             // 80 KB
    {256, 128, &glds_get<256, 128, 4, 2, 4, 32, 16>, 512},        // 96 KB
    // direct register epilogue (DE: v_permlane16_swap -> 16-B stores, no LDS C tile, no
    // epilogue barrier) on the best 8-wave forms and the 2-per-CU 256 x 128
    {256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, true>, 512},
    {256, 256, &glds_get<256, 256, 2, 4, 5, 32, 16, true, true>, 512},
    {256, 128, &glds_get<256, 128, 2, 2, 3, 32, 16, false, true>},
    {128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, true>},
};

int xp_num_tiles() { return (int)(sizeof(kXpTiles) / sizeof(kXpTiles[0])); }

// v8: split-K (edge batches: few output tiles, long K).  (instantiation, K slices)
struct SkTile {
  GldsTile t;
  int split;
};
static const SkTile kSkTiles[] = {
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 16},
    {{128, 64, &glds_get<128, 64, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{128, 64, &glds_get<128, 64, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{64, 128, &glds_get<64, 128, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{64, 128, &glds_get<64, 128, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 2},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 4},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 8},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 2},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 4},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 8},
};

int sk_num_tiles() { return (int)(sizeof(kSkTiles) / sizeof(kSkTiles[0])); }

// mode here is the caller's (0 general, 1 gemm); picks MODE 0 vs 3 by Cin and taps.
static int glds_launch_entry(const KvConvParams* p, const struct GldsTile& e, hipStream_t stream,
                             int split = 1);

int glds_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= glds_num_tiles()) return -6;
  return glds_launch_entry(p, kGldsTiles[tile], stream);
}

int xp_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= xp_num_tiles()) return -6;
  return glds_launch_entry(p, kXpTiles[tile], stream);
}

int sk_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= sk_num_tiles()) return -6;
  const SkTile& e = kSkTiles[tile];
  const int nk = p->Kpad / BK;
  if (!p->ws || e.split > nk) return -11;  // no workspace, or more slices than K steps
  KvConvParams q = *p;
  q.ksplit = e.split;
  if (const int rc = glds_launch_entry(&q, e.t, stream, e.split)) return rc;
  const long long thr = (long long)p->M * (p->Cout / 8);
  if (thr <= 0) return 0;
  hipLaunchKernelGGL(splitk_finalize_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0,
                     stream, p->ws, p->bias, (const bf16*)p->res, (bf16*)p->y, p->M, p->Cout,
                     p->ldy, p->y_coff, p->ldr, p->r_coff, p->act);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

static int glds_launch_entry(const KvConvParams* p, const GldsTile& e, hipStream_t stream,
                             int split) {
  int mode = p->mode;
  if (mode == 2) return -8;  // legacy stem layout: v1 only
  if (mode == 0 && (p->Cin % 64 != 0 || p->KH * p->KW > 32)) mode = 3;
  const long long xb = (long long)p->N * p->H * p->W * p->ldx * 2;
  const long long wb = (long long)p->Cout * p->Kpad * 2;
  if (xb >= kOOB || wb >= kOOB) return -9;
  if (mode == 4) {
    const long long x2b = (long long)p->N * p->H2 * p->W2 * p->ldx2 * 2;
    if (!p->x2 || x2b >= kOOB || p->K1 % BK || (p->Kpad - p->K1) % BK || p->ldx2 % 8) return -10;
  }
  const long long nwg =
      (long long)((p->M + e.bm - 1) / e.bm) * ((p->Cout + e.bn - 1) / e.bn) * split;
  if (nwg <= 0) return 0;
  hipLaunchKernelGGL(e.get(mode), dim3((unsigned)nwg), dim3(e.nt), 0, stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

int glds_tile_bm(int tile) { return kGldsTiles[tile].bm; }
int glds_tile_bn(int tile) { return kGldsTiles[tile].bn; }

}  // namespace kvedge
