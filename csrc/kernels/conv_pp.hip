// K1/K2/K3 v14: 256x256 implicit-GEMM conv on the 8-phase ping-pong schedule (gfx950).
//
// Why (profiles/r6_v1_hipblaslt_same_box_b640.md): the workhorse tile
// "de:80" (conv_glds_kernel<256, 256, 4, 2, *, 2, 64, 16, false, true>, 15 of the 42
// ResNet-50 layers, a quarter of the step) runs the classic 2-phase loop -- vmcnt(0),
// barrier, issue the next stage, read every fragment, 64 MFMAs -- and keeps the MFMA pipe
// busy 47 % of the time (PMC on s3.c2): after each barrier all eight waves queue their 24
// fragment reads at once and wait on them together, and both waves of a SIMD stall at the
// same barrier.
//
// This loop follows the 256^2 8-phase template of cdna_hip_programming.md §5 (T3+T4+T5):
//  * A K-tile (BK = 64) is four PHASES; phase q computes one quadrant of every wave's
//    128 x 64 output (16 v_mfma_f32_16x16x32_bf16) between two raw s_barriers.
//  * The eight waves form two groups of four (along M; one wave of each group per SIMD).  Group 1 runs ONE BARRIER BEHIND group 0, so while one group issues its MFMAs
//    the other does its fragment reads and DMA issue: the two waves of a SIMD take turns on
//    the MFMA pipe instead of stalling together.
//  * Each wave's 128 x 64 output is split over the four HALF-TILES of the LDS stage (A rows
//    [0, BM/2) / [BM/2, BM), B channels [0, BN/2) / [BN/2, BN)): rows wm*64 + [0, 64) of each
//    A half, channels wn*32 + [0, 32) of each B half.  Quadrant (qm, qn) reads only A half qm and B
//    half qn, in the order (0,0) (0,1) (1,1) (1,0), so the halves of a stage are consumed
//    one by one (A0 at phase 0, B1 at 1, A1 at 2, B0 at 3) and each is restaged with the
//    K-tile two ahead ONE phase after its last read.  With only two stages of LDS (64 KB
//    each at 256 x 256), three half-tiles (6 LDS-DMA ops per wave at 256 x 256) stay in
//    flight across every barrier; the only vmcnt wait is one counted wait per K-tile.
//  * Every phase retires its fragment reads (lgkmcnt(0)) BEFORE its first barrier: that is
//    what makes a one-phase restage distance safe for the other (staggered) group.
//  * Direct epilogue from registers (v_permlane16_swap pairs -> 16-B stores), bias from
//    LDS, residual prefetched before the first store: the de:80 epilogue.
// Hazard bookkeeping, per wave (P = 4 kt + q is the global phase):
//   phase q stages: q=0 B-half0 of tile kt+1; q=1 A-half0, q=2 B-half1, q=3 A-half1 of kt+2
//   phase q reads:  q=0 A0+B0, q=1 B1, q=2 A1, q=3 B0 of tile kt (buffer kt & 1)
//   RAW: tile kt+1's halves were staged at P <= 4 kt; the counted wait of phase 4 kt + 3 (before
//        its first barrier) retires every stage op up to P = 4 kt, and every wave of both
//        groups passes that barrier before its first read of tile kt+1.
//   WAR: a half is restaged one phase after its last read; that read was retired by the
//        reading wave's lgkmcnt(0) before a barrier the restaging wave passes first.
// Steps past the last K-tile are staged out of range (zero fill, into halves already
// consumed), so every phase issues the same two DMA ops and the counted waits stay exact.
#include <stdlib.h>

#include "conv_glds_kernel.inc"

#ifndef KV_PP_DMA
#define KV_PP_DMA 1
#endif
#ifndef KV_PP_PRIO
#define KV_PP_PRIO 1
#endif
#ifndef KV_PP_KEEPB
#define KV_PP_KEEPB 1
#endif

namespace kvedge {
namespace {

// BM x BN tile, 8 waves of 128 x 64 outputs each: (BM, BN) = (256, 256) -- waves 2 (M) x 4
// (N) -- or (512, 128) -- 4 x 2, for the 128-channel layers, whose two 80 KB stages fill the
// whole 160 KB of LDS (the bias then comes from global memory in the epilogue).
// MODE 0: KxK / strided conv with Cin % 64 == 0; MODE 1: 1x1 GEMM; MODE 4: dual 1x1
//
// PT (persistent): gridDim.x <= the tile count (one workgroup per CU) and workgroup g walks
// the logical tiles i * gridDim + slot(g).  The K-steps of all its tiles form ONE staging
// stream, so the first half-tiles of tile i+1 are in flight (and the pipeline full) while
// tile i finishes and runs its epilogue inside the loop: no prologue latency, no workgroup
// launch per tile.  The A and B staging descriptors switch tiles at the first A / B half
// staged for the new tile (every later stage of the old tile precedes it).  Bias: two LDS
// slots by tile parity (kLdsBias forms), the next tile's written at the end of an epilogue.
// ABL (ablation instantiations, timing only -- outputs are wrong; KVEDGE_PP_ABL, tile 117,
// MODE 0 and 1): bit 0 drops the MFMA clusters, bit 1 the fragment reads, bit 2 the LDS-DMA
// staging, bit 3 the lgkmcnt(0) before each phase's first barrier, bit 4 both barriers of
// every phase.  What is left of the phase period says what bounds it (tools/pp_abl.sh).
// Bits 5 / 6: drop only the B (weight) / only the A (activation) staging DMAs.
template <int BM, int BN, int MODE, bool PT, int ABL = 0>
__global__ __launch_bounds__(512, 1) void conv_pp_kernel(const KvConvParams p) {
  constexpr int kHA = BM / 2 * 64, kHB = BN / 2 * 64;  // bf16 elements per A / B half-tile
  constexpr int kStage = (BM + BN) * 64;               // one K-tile: A0 A1 B0 B1
  constexpr bool kLdsBias = (2 * kStage + BN * 4) * 2 <= 160 * 1024;
  constexpr int WM = BM / 128, WN = BN / 64;           // waves along M / N
  constexpr int AO = BM / 128, BO = BN / 128;          // DMA ops per wave per A / B half
  static_assert(WM * WN == 8 && BO >= 1, "8 waves of 128 x 64");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * kStage + (kLdsBias ? BN * 4 : 0)];
  float* const sbias = reinterpret_cast<float*>(smem + 2 * kStage);
  auto half_off = [](int h) __attribute__((always_inline)) {  // 0 A0, 1 A1, 2 B0, 3 B1
    return h < 2 ? h * kHA : BM * 64 + (h - 2) * kHB;
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;  // the wave's M sub-rows / N sub-columns
  const int grp = wm / (WM / 2);           // stagger group: one wave of each per SIMD
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.Cout + BN - 1) / BN;
  const int ntiles = nbm * nbn;
  const int G = PT ? (int)gridDim.x : ntiles;
  const int slot = xcd_remap(blockIdx.x, G);
  const int ntl = PT ? (ntiles - slot + G - 1) / G : 1;  // tiles of this workgroup
  auto tile_m0 = [&](int i) __attribute__((always_inline)) { return ((i * G + slot) / nbn) * BM; };
  auto tile_n0 = [&](int i) __attribute__((always_inline)) { return ((i * G + slot) % nbn) * BN; };
  const int nk = p.Kpad / 64;
  const int nsteps = ntl * nk;

  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, p.N * p.H * p.W * p.ldx * 2);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w, p.Cout * p.Kpad * 2);
  const __amdgpu_buffer_rsrc_t rx2 =
      make_rsrc(MODE == 4 ? p.x2 : p.x, MODE == 4 ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);

  // bias of the first tile's channels -> LDS slot 0 (published by the prologue barrier)
  if (kLdsBias && tid < BN) {
    const int n0 = tile_n0(0);
    sbias[tid] = (p.bias && n0 + tid < p.Cout) ? p.bias[n0 + tid] : 0.f;
  }

  // ---- staging descriptors: DMA op j of an A half covers rows (wid * AO + j) * 8 + lrow of
  // that half (B: BO ops); logical 16-B chunk lc = pch ^ swizzle(row) (lane-linear LDS image)
  const int lrow = lane >> 3, pch = lane & 7;
  auto sw = [](int r) __attribute__((always_inline)) { return (r >> 1) & 7; };
  int a_off[2][AO], a_off2[2][AO], a_lc[2][AO];
  unsigned a_msk[2][AO];
  int b_off[2][BO];
  const int HoWo = p.Ho * p.Wo;
  auto set_a = [&](int m0) __attribute__((always_inline)) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < AO; ++j) {
      const int row = (wid * AO + j) * 8 + lrow;  // within the half
      const int lc = pch ^ sw(row);
      a_lc[h][j] = lc;
      const int m = m0 + h * (BM / 2) + row;
      a_msk[h][j] = 0u;
      a_off2[h][j] = kOOB;
      if (MODE == 1 || MODE == 4) {
        a_off[h][j] = m < p.M ? (m * p.ldx + p.x_coff + lc * 8) * 2 : kOOB;
        if (MODE == 4 && m < p.M) {
          const int img = m / HoWo, rem = m - img * HoWo;
          const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
          const int h2 = p.up2 ? (ho >> 1) : ho * p.stride2, w2 = p.up2 ? (wo >> 1) : wo * p.stride2;
          a_off2[h][j] = (((img * p.H2 + h2) * p.W2 + w2) * p.ldx2 + p.x2_coff + lc * 8) * 2;
        }
      } else {
        a_off[h][j] = 0;
        if (m < p.M) {
          const int img = m / HoWo, rem = m - img * HoWo;
          const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
          const int h0 = ho * p.stride - p.pad, w0 = wo * p.stride - p.pad;
          a_off[h][j] = ((img * p.H + h0) * p.W + w0) * p.ldx + p.x_coff + lc * 8;  // may be < 0
          unsigned msk = 0;
          for (int r = 0; r < p.KH; ++r)
            for (int s = 0; s < p.KW; ++s)
              if ((unsigned)(h0 + r) < (unsigned)p.H && (unsigned)(w0 + s) < (unsigned)p.W)
                msk |= 1u << (r * p.KW + s);
          a_msk[h][j] = msk;
        }
      }
    }
  };
  auto set_b = [&](int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < BO; ++j) {
        const int row = (wid * BO + j) * 8 + lrow;
        const int n = n0 + h * (BN / 2) + row;
        b_off[h][j] = n < p.Cout ? (n * p.Kpad + (pch ^ sw(row)) * 8) * 2 : kOOB;
      }
  };

  // Staging cursors.  Over the workgroup's K-steps T = 0, 1, ... the A half 0 stages come
  // in order of T (A half 1 of T right after A half 0 of T) and so do the B half 1 stages
  // (B half 0 of T right after B half 1 of T): each cursor steps once per K-step and switches
  // its descriptors (and, for A, the MODE 0 tap walk) at a new tile's first K-step.
  int a_kt = nk - 1, a_i = -1, b_kt = nk - 1, b_i = -1;
  int k_c0 = 0, k_r = 0, k_s = 0;
  auto a_next = [&]() __attribute__((always_inline)) {
    if (++a_kt == nk) {
      a_kt = 0;
      ++a_i;
      if (a_i < ntl) set_a(tile_m0(a_i));
      k_c0 = 0; k_r = 0; k_s = 0;
    } else if (MODE == 0) {
      k_c0 += 64;  // Cin % 64 == 0: a K-step never straddles two taps
      if (k_c0 >= p.Cin) {
        k_c0 = 0;
        if (++k_s == p.KW) { k_s = 0; ++k_r; }
      }
    }
  };
  auto b_next = [&]() __attribute__((always_inline)) {
    if (++b_kt == nk) {
      b_kt = 0;
      ++b_i;
      if (b_i < ntl) set_b(tile_n0(b_i));
    }
  };
  // stage half h (0 A0, 1 A1, 2 B0, 3 B1) of K-step T: AO or BO DMA ops per wave, always
  // issued (out of range past the last K-step)
  auto stage = [&](int h, int T) __attribute__((always_inline)) {
    if constexpr ((ABL & 4) != 0) return;
    if ((ABL & 32) != 0 && h >= 2) return;
    if ((ABL & 64) != 0 && h < 2) return;
    bf16* dst = smem + (T & 1) * kStage + half_off(h) + wid * (h < 2 ? AO : BO) * 512;
    const bool live = T < nsteps;  // wave-uniform
    if (h == 0) a_next();
    if (h == 3) b_next();
    const int kbase = (h < 2 ? a_kt : b_kt) * 64;
    if (h >= 2) {
#pragma unroll
      for (int j = 0; j < BO; ++j)
        glds16(rw, dst + j * 512, live ? b_off[h - 2][j] : kOOB, live ? kbase * 2 : 0);
      return;
    }
    if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < AO; ++j) {
        const int v = (live && kbase + a_lc[h][j] * 8 < p.Cin) ? a_off[h][j] : kOOB;
        glds16(rx, dst + j * 512, v, live ? kbase * 2 : 0);
      }
    } else if (MODE == 4) {
      // both sources are read here for the last time: non-temporal (de:80 policy)
      if (kbase < p.K1) {
#pragma unroll
        for (int j = 0; j < AO; ++j) glds16<2>(rx, dst + j * 512, live ? a_off[h][j] : kOOB, kbase * 2);
      } else {
#pragma unroll
        for (int j = 0; j < AO; ++j)
          glds16<2>(rx2, dst + j * 512, live ? a_off2[h][j] : kOOB, live ? (kbase - p.K1) * 2 : 0);
      }
    } else {
      const int tap = k_r * p.KW + k_s;
      const int toff = (k_r * p.W + k_s) * p.ldx + k_c0;  // elements, wave-uniform
#pragma unroll
      for (int j = 0; j < AO; ++j) {
        const bool ok = live && tap < p.KH * p.KW && ((a_msk[h][j] >> tap) & 1u);
        glds16(rx, dst + j * 512, ok ? (a_off[h][j] + toff) * 2 : kOOB, 0);
      }
    }
  };

  // ---- fragments: 16x16x32 roles (row lane & 15, k quarter lane >> 4)
  const int fr = lane & 15, fh = lane >> 4;
  floatx4 acc[2][2][2][4];  // [qn][tnb][qm][tmb]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[a][b][c][d] = floatx4{0.f, 0.f, 0.f, 0.f};
  // B fragments per N half (KV_PP_KEEPB: B0's stay in registers from phase 0 to phase 3, so
  // the K-step reads 24 fragments instead of 28 -- the ablation puts the cost of the staging
  // in its contention with these LDS reads, profiles/r6_v10_pp_ablation_pmc.md)
  bf16x8 afr[2][4], bfrq[2][2][2];  // [ks][block] / [qn][ks][block]
  auto read_a = [&](const bf16* st, int qm) __attribute__((always_inline)) {
    const bf16* As = st + half_off(qm);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int row = wm * 64 + b * 16 + fr;
        afr[ks][b] = *reinterpret_cast<const bf16x8*>(As + row * 64 + (((ks * 4 + fh) ^ sw(row)) << 3));
      }
  };
  auto read_b = [&](const bf16* st, int qn) __attribute__((always_inline)) {
    const bf16* Bs = st + half_off(2 + qn);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int row = wn * 32 + b * 16 + fr;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(Bs + row * 64 + (((ks * 4 + fh) ^ sw(row)) << 3));
        if (KV_PP_KEEPB && qn == 1) bfrq[1][ks][b] = v;
        else bfrq[0][ks][b] = v;
      }
  };
  auto bfr_of = [&](int qn, int ks, int b) __attribute__((always_inline)) -> const bf16x8& {
    return (KV_PP_KEEPB && qn == 1) ? bfrq[1][ks][b] : bfrq[0][ks][b];
  };
  auto mma = [&](int qm, int qn) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
          acc[qn][tn][qm][tm] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr_of(qn, ks, tn), afr[ks][tm], acc[qn][tn][qm][tm], 0, 0, 0);
  };
  // one phase: reads + staging (+ the per-tile counted wait), barrier, MFMAs, barrier.
  // KV_PP_DMA (A/B knob): 1 = the two DMA ops after the fragment reads (default), 0 = before
  // them, 2 = inside the MFMA cluster (after 8 of its 16 MFMAs: the read section is then
  // reads only; the tile-end wait counts one phase less in flight)
  auto mma_half = [&](int qm, int qn, int ks) __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
        acc[qn][tn][qm][tm] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr_of(qn, ks, tn), afr[ks][tm], acc[qn][tn][qm][tm], 0, 0, 0);
  };
  auto phase = [&](const bf16* st, int qm, int qn, auto RA, auto RB, int sh, int sT, bool tile_end)
      __attribute__((always_inline)) {
    if (KV_PP_DMA == 0) stage(sh, sT);
    if constexpr (decltype(RA)::value && (ABL & 2) == 0) read_a(st, qm);
    if constexpr (decltype(RB)::value && (ABL & 2) == 0) read_b(st, qn);
    if (KV_PP_DMA == 1) stage(sh, sT);
    // tile kt+1 landed (this wave's part): 3 half-tiles stay in flight (2 when this phase's
    // DMA is issued later, inside its MFMA cluster)
    if (tile_end) wait_vm<KV_PP_DMA == 2 ? AO + BO : 2 * AO + BO>();
    if constexpr ((ABL & 8) == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((ABL & 16) == 0) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (KV_PP_PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr ((ABL & 1) != 0) {
    } else if (KV_PP_DMA == 2) {
      mma_half(qm, qn, 0);
      __builtin_amdgcn_sched_barrier(0);
      stage(sh, sT);
      __builtin_amdgcn_sched_barrier(0);
      mma_half(qm, qn, 1);
    } else {
      mma(qm, qn);
    }
    if (KV_PP_PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((ABL & 16) == 0) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- prologue: tile 0 whole, tile 1 minus its B half 0 (the steady-state lookahead)
  stage(0, 0); stage(3, 0); stage(1, 0); stage(2, 0);
  stage(0, 1); stage(3, 1); stage(1, 1);
  wait_vm<2 * AO + BO>();  // tile 0 landed (tile 1's three half-tiles in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // tile 0 and the bias published
  asm volatile("" ::: "memory");
  if (grp == 1) {  // group 1 runs one barrier behind group 0
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  // ---- direct epilogue (as de:80) of tile i: block pair (tnb 0, 1) of each (qn, qm, tmb) ->
  // one 16-B store per lane of 8 consecutive channels after v_permlane16_swap
  const bool has_res = p.res != nullptr;
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y, p.M * p.ldy * 2);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.res, has_res ? p.M * p.ldr * 2 : 0);
  const int rho = lane >> 4;
  const int csel = 16 * (rho & 1) + 8 * (rho >> 1);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto epilogue = [&](int i) __attribute__((always_inline)) {
    const int m0 = tile_m0(i), n0 = tile_n0(i);
    const float* sb = sbias + (PT ? (i & 1) * BN : 0);
    dispatch_act(p.act, has_res, [&](auto A1, auto A2) __attribute__((always_inline)) {
      constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        // the residual of this channel half, all 8 loads before its first store (32 VGPRs:
        // the whole tile's 64 would not fit beside the accumulators in the persistent loop)
        u32x4 rv[2][4];
        if (has_res) {
#pragma unroll
          for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int tm = 0; tm < 4; ++tm) {
              const int n = n0 + qn * (BN / 2) + wn * 32 + csel;
              const int m = m0 + qm * (BM / 2) + wm * 64 + tm * 16 + fr;
              const int off = (m < p.M && n < p.Cout) ? (m * p.ldr + p.r_coff + n) * 2 : kOOB;
              rv[qm][tm] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
            }
        }
        const int nl = qn * (BN / 2) + wn * 32;  // first channel of the pair, tile-local
        float4 bv0 = make_float4(0.f, 0.f, 0.f, 0.f), bv1 = bv0;
        if constexpr (kLdsBias) {
          bv0 = *reinterpret_cast<const float4*>(sb + nl + fh * 4);
          bv1 = *reinterpret_cast<const float4*>(sb + nl + 16 + fh * 4);
        } else if (p.bias) {  // Cout % 8 == 0: a 4-channel group is all in range or all out
          if (n0 + nl + fh * 4 < p.Cout) bv0 = *reinterpret_cast<const float4*>(p.bias + n0 + nl + fh * 4);
          if (n0 + nl + 16 + fh * 4 < p.Cout)
            bv1 = *reinterpret_cast<const float4*>(p.bias + n0 + nl + 16 + fh * 4);
        }
        const int n = n0 + nl + csel;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int tm = 0; tm < 4; ++tm) {
            bf16x4 a, b;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              a[j] = f2bf(act_c<act1>(acc[qn][0][qm][tm][j] + (&bv0.x)[j]));
              b[j] = f2bf(act_c<act1>(acc[qn][1][qm][tm][j] + (&bv1.x)[j]));
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
              const bf16x8 r = __builtin_bit_cast(bf16x8, rv[qm][tm]);
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = f2bf(act_c<act2>((float)v[e] + (float)r[e]));
            }
            const int m = m0 + qm * (BM / 2) + wm * 64 + tm * 16 + fr;
            const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kOOB;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, off, 0, 0);
          }
      }
    });
    if (PT && kLdsBias && i + 1 < ntl && tid < BN) {
      // the next tile's bias into the other slot (last read by tile i-1's epilogue, at least
      // one K-step of barriers ago); its tile's epilogue is at least four phases away
      const int nn = tile_n0(i + 1);
      sbias[((i + 1) & 1) * BN + tid] = (p.bias && nn + tid < p.Cout) ? p.bias[nn + tid] : 0.f;
    }
  };

  using T1 = IC<1>;
  using T0 = IC<0>;
  int c_kt = 0, c_i = 0;  // compute cursor: K-step within the tile, tile
  for (int T = 0; T < nsteps; ++T) {
    const bf16* st = smem + (T & 1) * kStage;
    phase(st, 0, 0, T1{}, T1{}, 2, T + 1, false);  // B0 of K-step T+1
    phase(st, 0, 1, T0{}, T1{}, 0, T + 2, false);  // A0 of K-step T+2
    phase(st, 1, 1, T1{}, T0{}, 3, T + 2, false);  // B1 of K-step T+2
    // (KV_PP_KEEPB: B0 is still in registers from phase 0, no reads in this phase)
    if constexpr (KV_PP_KEEPB) phase(st, 1, 0, T0{}, T0{}, 1, T + 2, true);
    else phase(st, 1, 0, T0{}, T1{}, 1, T + 2, true);   // A1 of K-step T+2; wait: K-step T+1
    if (PT && ++c_kt == nk) {  // the tile's last K-step: epilogue, fresh accumulators
      epilogue(c_i);
      c_kt = 0;
      ++c_i;
      if (PT && c_i < ntl) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int d = 0; d < 4; ++d) acc[a][b][c][d] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  if (grp == 0) {  // balance the stagger: every wave passes the same number of barriers
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup
  if (!PT) epilogue(0);
}

}  // namespace

int pp_num_tiles() { return 4; }  // 256 x 256, 512 x 128, and their persistent forms

int pp_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= pp_num_tiles()) return -6;
  const bool wide = (tile & 1) == 0, pt = tile >= 2;
  const int BM = wide ? 256 : 512, BN = wide ? 256 : 128;
  int mode = p->mode;
  if (mode == 0 && (p->Cin % 64 != 0 || p->KH * p->KW > 32)) return -8;  // no generic gather
  if (mode != 0 && mode != 1 && mode != 4) return -8;
  if (p->Kpad % 64 != 0 || p->Cout % 8 != 0) return -1;
  const long long xb = (long long)p->N * p->H * p->W * p->ldx * 2;
  const long long wb = (long long)p->Cout * p->Kpad * 2;
  if (xb >= kOOB || wb >= kOOB) return -9;
  if (mode == 4) {
    const long long x2b = (long long)p->N * p->H2 * p->W2 * p->ldx2 * 2;
    if (!p->x2 || x2b >= kOOB || p->K1 % 64 || (p->Kpad - p->K1) % 64 || p->ldx2 % 8) return -10;
    if (p->x2_coff % 8 || p->x2_coff + (p->Kpad - p->K1) > p->ldx2) return -10;
    if (p->up2 && (p->Ho != 2 * p->H2 || p->Wo != 2 * p->W2)) return -10;
  }
  const long long nwg = (long long)((p->M + BM - 1) / BM) * ((p->Cout + BN - 1) / BN);
  if (nwg <= 0) return 0;
  long long grid = nwg;
  if (pt) {  // one workgroup per CU (128 / 160 KB of LDS), each walks several tiles
    static int ncu = 0;
    if (ncu <= 0) {
      int dev = 0;
      ncu = 256;
      if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    }
    grid = nwg < ncu ? nwg : ncu;
  }
#define KV_PP_FN(bm, bn, P)                                                              \
  (mode == 0 ? conv_pp_kernel<bm, bn, 0, P> : mode == 1 ? conv_pp_kernel<bm, bn, 1, P>   \
             : conv_pp_kernel<bm, bn, 4, P>)
  ConvKernelFn fn = wide ? (pt ? KV_PP_FN(256, 256, true) : KV_PP_FN(256, 256, false))
                         : (pt ? KV_PP_FN(512, 128, true) : KV_PP_FN(512, 128, false));
#undef KV_PP_FN
  static const int abl = getenv("KVEDGE_PP_ABL") ? atoi(getenv("KVEDGE_PP_ABL")) : 0;
  if (abl && wide && !pt && (mode == 0 || mode == 1)) {
#define KV_PP_ABL(a) (mode == 0 ? conv_pp_kernel<256, 256, 0, false, a> : conv_pp_kernel<256, 256, 1, false, a>)
    switch (abl) {
      case 1: fn = KV_PP_ABL(1); break;
      case 2: fn = KV_PP_ABL(2); break;
      case 4: fn = KV_PP_ABL(4); break;
      case 6: fn = KV_PP_ABL(6); break;
      case 8: fn = KV_PP_ABL(8); break;
      case 16: fn = KV_PP_ABL(16); break;
      case 22: fn = KV_PP_ABL(22); break;
      case 32: fn = KV_PP_ABL(32); break;
      case 64: fn = KV_PP_ABL(64); break;
      case 34: fn = KV_PP_ABL(34); break;
      case 66: fn = KV_PP_ABL(66); break;
      default: return -6;
    }
#undef KV_PP_ABL
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), 0, stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
