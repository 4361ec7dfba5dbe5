// K3 v3 — persistent streaming 1x1 conv / GEMM for the HBM-bound layers (gfx950).
//
// Forward profile (profiles/r1_v2_*, batch 256): ~50 % of a ResNet-50 step is 1x1
// convs with K <= 512 that move far more bytes than they compute (bottleneck conv1
// "reduce" and conv3 "expand + residual").  A one-tile-per-workgroup kernel serialises
// load A,B -> MFMA -> epilogue inside every workgroup and leaves the overlap to
// occupancy; it reached 3.8-4.5 TB/s.  The bound is bytes in flight per CU (Little's
// law: ~6 TB/s x ~2-3 us loaded latency / 256 CUs ~ 48-72 KB per CU).
//
// Here a grid of 1-3 workgroups per CU walks a flat stream of (M tile, K step) stages:
//  * a D-slot LDS-DMA ring (buffer_load ... lds) is fed D-1 stages ahead, ACROSS tile
//    boundaries, so the next tiles' operands stream while this tile computes/stores;
//  * the residual tile is loaded into a D-deep REGISTER ring with the tile's last K
//    step (the loop is unrolled by D so every ring slot is a fixed register set); the
//    register file (512 KB/CU) holds far more in-flight residual bytes than spare LDS;
//  * BRES variants keep the workgroup's whole weight slice [BN x Kpad] resident in LDS
//    (loaded once) and stream only activations;
//  * every stage issues the same number of VMEM ops (out-of-range lanes/stages use an
//    offset past num_records -> zero fill), so the wait for stage j is an exact
//    vmcnt(n) computed from (D, #epilogues in the window): older stores stay in flight;
//  * the nbn workgroups that share an M tile are adjacent after the bijective XCD
//    remap, i.e. on the same XCD: the activation tile is fetched into one L2 once.
// Modes: 1 = plain 1x1 (stride 1) GEMM, 4 = dual-source (conv3 + fused downsample).
#include "common.h"
#include "kvedge_kernels.h"

#include <cstdlib>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MF>
struct SAccOf { typedef floatx16 type; static constexpr int n = 16; };
template <>
struct SAccOf<16> { typedef floatx4 type; static constexpr int n = 4; };

namespace kvedge {
namespace {

constexpr int BK = 64;
constexpr int kOOB = 0x7ffffff0;
constexpr int kLdsMax = 160 * 1024;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

template <int AUX = 0>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, bf16* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, AUX);
}

template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}

// LDS bytes of one variant (host + device agree on the layout)
__host__ __device__ constexpr int stream_lds_bytes(int bm, int bn, int d, bool res, bool bres,
                                                   int kpad, int nt1 = 0) {
  return 2 * (d * (bm * BK + (bres ? 0 : bn * BK)) + (bres ? bn * kpad : 0) + bm * (bn + 8) +
              nt1 * bn);
}

// NT1 > 0: fused bottleneck tail -- after the y tile is written, z = ReLU(y . Wt^T + bt)
// (the next block's 1x1 reduce, NT1 output channels) is computed from the y tile in LDS.
// MF: main-GEMM MFMA shape (32 = 32x32x16, 16 = 16x16x32; see conv_glds.hip); the fused
// tail GEMM always runs on 32x32x16.
template <int BM, int BN, int D, int MODE, bool RES, bool BRES, int POL, int NT1 = 0, int MF = 32>
// 128x128 resident-weight tiles (and the tail tiles) hold >100 KB of weights: one
// workgroup per CU, so they may use the whole 512-entry register file
__global__ __launch_bounds__(256, (NT1 || (BM * BN >= 128 * 128 && BRES)) ? 1 : 2)
void conv_stream_kernel(const KvConvParams p) {
  constexpr int WM = 2, WN = 2;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  using Acc = typename SAccOf<MF>::type;
  constexpr int NACC = SAccOf<MF>::n;
  constexpr int A_INS = BM / 32, B_INS = BN / 32;
  constexpr int CS = BN + 8;
  constexpr int CPR = BN / 8;
  constexpr int PER = BM * CPR / 256;  // 16-B output (and residual) chunks per thread
  constexpr int SA = BM * BK, SB = BRES ? 0 : BN * BK;
  constexpr int SLOT = SA + SB;
  // VMEM ops per stage per wave, and per epilogue (stores)
  constexpr int SI = A_INS + (BRES ? 0 : B_INS) + (RES ? PER : 0);
  constexpr int PERZ = NT1 ? BM * NT1 / 8 / 256 : 0;  // 16-B z chunks per thread (tail)
  constexpr int EPI = PER + PERZ;
  static_assert(NT1 == 0 || (BM == 64 && BRES && NT1 % 64 == 0 && PERZ >= 1), "tail tile");
  // cache policy of the streamed (read-once / write-once) bytes: 0 default, 2 = nt
  constexpr int SP = POL;
  // fused bottleneck tails (NT1 > 0): y (this block's output, re-read only two launches later
  // as the next residual, by then long out of the 256 MB Infinity Cache) is stored, and the
  // activations read here for the last time (A, the downsample source, the residual) are
  // loaded non-temporal, so z -- read by the very next launch (the 3x3) -- stays there
  constexpr int YP = NT1 > 0 ? 2 : SP;
  static_assert(TM >= 1 && TN >= 1 && PER >= 1 && D >= 2 && D <= 6, "tile");
  // one LDS array (guide §5 trap (a)): [D ring slots: A | B] [resident B] [C tile]
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  const int nk = p.Kpad / BK;
  bf16* const Bres = smem + D * SLOT;
  bf16* const Cs = Bres + (BRES ? BN * p.Kpad : 0);
  bf16* const W1s = Cs + BM * CS;  // tail: resident [BN/64][NT1][64] swizzled blocks

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.Cout + BN - 1) / BN;
  // grid = mgroups * nbn; the nbn slices of one M group are adjacent logical ids, and
  // xcd_remap puts adjacent logical ids on the same XCD (shared L2 for the A tile)
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = logical % nbn;
  const int n0 = nb * BN;
  const int mstep = gridDim.x / nbn;
  const int mfirst = logical / nbn;
  const int ntiles = mfirst < nbm ? (nbm - 1 - mfirst) / mstep + 1 : 0;
  const int nstages = ntiles * nk;
  if (nstages == 0) return;

  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(p.x, p.N * p.H * p.W * p.ldx * 2);
  const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.Cout * p.Kpad * 2);
  const __amdgpu_buffer_rsrc_t rx2 =
      mk_rsrc(MODE == 4 ? p.x2 : p.x, MODE == 4 ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);
  const __amdgpu_buffer_rsrc_t rr = mk_rsrc(RES ? p.res : p.x, RES ? p.M * p.ldr * 2 : 0);
  const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, p.M * p.ldy * 2);

  const int lrow = lane >> 3, pch = lane & 7;
  int b_off[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int row = (wv * B_INS + i) * 8 + lrow;
    const int n = n0 + row;
    b_off[i] = n < p.Cout ? (n * p.Kpad + (pch ^ ((row >> 1) & 7)) * 8) * 2 : kOOB;
  }
  int a_lc[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int row = (wv * A_INS + i) * 8 + lrow;
    a_lc[i] = pch ^ ((row >> 1) & 7);
  }
  const int HoWo = p.Ho * p.Wo;

  typedef u32x4 ResRegs[RES ? PER : 1];
  // one (tile, kt) stage into ring slot `slot`: always SI VMEM ops per wave
  auto issue = [&](int s, int slot, ResRegs& rdst) __attribute__((always_inline)) {
    const int ti = s / nk, kt = s - ti * nk;
    const bool tv = ti < ntiles;
    const int m0 = (mfirst + ti * mstep) * BM;
    bf16* As = smem + slot * SLOT;
    const int kbase = kt * BK;
    if (MODE == 4 && kbase >= p.K1) {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int m = m0 + (wv * A_INS + i) * 8 + lrow;
        int v = kOOB;
        if (tv && m < p.M) {
          const int img = m / HoWo, rem = m - img * HoWo;
          const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
          v = (((img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2) * p.ldx2 + a_lc[i] * 8) * 2;
        }
        dma16<YP>(rx2, As + (wv * A_INS + i) * 512, v, (kbase - p.K1) * 2);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int m = m0 + (wv * A_INS + i) * 8 + lrow;
        const bool ok = tv && m < p.M && (MODE == 4 || kbase + a_lc[i] * 8 < p.Cin);
        const int v = ok ? (m * p.ldx + p.x_coff + a_lc[i] * 8) * 2 : kOOB;
        dma16<YP>(rx, As + (wv * A_INS + i) * 512, v, kbase * 2);
      }
    }
    if (!BRES) {
      bf16* Bs = As + SA;
#pragma unroll
      for (int i = 0; i < B_INS; ++i)
        dma16(rw, Bs + (wv * B_INS + i) * 512, tv ? b_off[i] : kOOB, kbase * 2);
    }
    if (RES) {  // this thread's epilogue chunks idx = tid + 256 j of the residual tile
      const bool last = kt == nk - 1 && tv;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int idx = tid + 256 * j;
        const int m = m0 + idx / CPR, n = n0 + (idx % CPR) * 8;
        const int off = (last && m < p.M && n < p.Cout) ? (m * p.ldr + p.r_coff + n) * 2 : kOOB;
        rdst[j] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, YP);
      }
    }
  };

  Acc acc[TN][TM];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b)
#pragma unroll
        for (int e = 0; e < NACC; ++e) acc[a][b][e] = 0.f;
  };

  // main-GEMM fragment roles (MF); the tail GEMM keeps the 32x32 roles fr32/fh32
  const int fr = lane & (MF - 1), fh = lane / MF;
  const int fr32 = lane & 31, fh32 = lane >> 5;
  auto compute = [&](int slot, int kt) __attribute__((always_inline)) {
    const bf16* As = smem + slot * SLOT;
    const bf16* Bs = BRES ? Bres + kt * BN * BK : As + SA;
    // fragments double-buffered in registers: the ds_reads of step ks+1 are issued
    // before the MFMAs of step ks, so LDS latency hides under the MFMA pipe instead of
    // an lgkmcnt(0) stall in front of every group of MFMAs
    bf16x8 af[2][TM], bfg[2][TN];
    constexpr int KS = BK / (MF == 32 ? 16 : 32);
    auto load = [&](int buf, int ks) __attribute__((always_inline)) {
      const int q = ks * (64 / MF) + fh;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * MF + fr;
        af[buf][tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((q ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * MF + fr;
        bfg[buf][tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((q ^ ((row >> 1) & 7)) << 3));
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


  // this lane's bias values for the whole run (the N slice is fixed): registers, not
  // LDS -- an LDS read in the epilogue would make hipcc drain the in-flight DMA.
  float4 bias_r[TN][NACC / 4];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int g = 0; g < NACC / 4; ++g) {
      const int n = n0 + wn * WTN + tn * MF + g * 8 + fh * 4;
      bias_r[tn][g] = (p.bias && n < p.Cout) ? *reinterpret_cast<const float4*>(p.bias + n)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }

  // tail GEMM: 2 x 2 waves, wave tile 32 pixels x NT1/2 channels, bias in registers
  constexpr int TN1 = NT1 ? NT1 / 64 : 1;
  float4 bias1_r[TN1][4];
  const __amdgpu_buffer_rsrc_t rz = mk_rsrc(NT1 ? p.z : p.y, NT1 ? p.M * p.ldz * 2 : 0);
  if constexpr (NT1 > 0) {
#pragma unroll
    for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = (wv & 1) * (NT1 / 2) + tn * 32 + g * 8 + fh32 * 4;
        bias1_r[tn][g] = p.bias_t ? *reinterpret_cast<const float4*>(p.bias_t + n)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  }

  // ---- tail: z = ReLU(y_tile . Wt^T + bt) from the y tile (post residual + act) in Cs
  auto tail = [&](int m0) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // y tile complete in Cs
    asm volatile("" ::: "memory");
    const int wm2 = wv >> 1, wn2 = wv & 1;
    floatx16 acc2[TN1];
#pragma unroll
    for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc2[tn][4 * g + 0] = bias1_r[tn][g].x;
        acc2[tn][4 * g + 1] = bias1_r[tn][g].y;
        acc2[tn][4 * g + 2] = bias1_r[tn][g].z;
        acc2[tn][4 * g + 3] = bias1_r[tn][g].w;
      }
#pragma unroll
    for (int kk = 0; kk < BN / 16; ++kk) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(Cs + (wm2 * 32 + fr32) * CS + kk * 16 + fh32 * 8);
      const int kt = kk >> 2, q = (kk & 3) * 2 + fh32;
#pragma unroll
      for (int tn = 0; tn < TN1; ++tn) {
        const int row = wn2 * (NT1 / 2) + tn * 32 + fr32;
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(
            W1s + kt * NT1 * BK + row * BK + ((q ^ ((row >> 1) & 7)) << 3));
        acc2[tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc2[tn], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave done reading the y tile: reuse Cs for z
    asm volatile("" ::: "memory");
    constexpr int CZ = NT1 + 8;
#pragma unroll
    for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn2 * (NT1 / 2) + tn * 32 + g * 8 + fh32 * 4;
        bf16x4 o;
        o[0] = f2bf(fmaxf(acc2[tn][4 * g + 0], 0.f));
        o[1] = f2bf(fmaxf(acc2[tn][4 * g + 1], 0.f));
        o[2] = f2bf(fmaxf(acc2[tn][4 * g + 2], 0.f));
        o[3] = f2bf(fmaxf(acc2[tn][4 * g + 3], 0.f));
        *reinterpret_cast<bf16x4*>(Cs + (wm2 * 32 + fr32) * CZ + nl) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    constexpr int ZPR = NT1 ? NT1 / 8 : 1;
#pragma unroll
    for (int j = 0; j < PERZ; ++j) {
      const int idx = tid + 256 * j;
      const int ml = idx / ZPR, ch = idx % ZPR;
      const int m = m0 + ml;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + ml * CZ + ch * 8);
      const int off = m < p.M ? (m * p.ldz + p.z_coff + ch * 8) * 2 : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rz, off, 0, SP);
    }
  };

  // act1/act2 compile-time: instantiated per activation pair by dispatch_act() below
  auto epilogue = [&](int ti, const ResRegs& rres, auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
    const int m0 = (mfirst + ti * mstep) * BM;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int g = 0; g < NACC / 4; ++g) {
        const int nl = wn * WTN + tn * MF + g * 8 + fh * 4;
        const float4 bv = bias_r[tn][g];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int ml = wm * WTM + tm * MF + fr;
          bf16x4 o;
          o[0] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 0] + bv.x));
          o[1] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 1] + bv.y));
          o[2] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 2] + bv.z));
          o[3] = f2bf(act_c<act1>(acc[tn][tm][4 * g + 3] + bv.w));
          *reinterpret_cast<bf16x4*>(Cs + ml * CS + nl) = o;
        }
      }
    }
    // C tile complete: LDS writes drained + raw barrier (no vmcnt: the DMA ring and
    // the previous stores stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = tid + 256 * j;
      const int ml = idx / CPR, ch = idx % CPR;
      const int m = m0 + ml, n = n0 + ch * 8;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + ml * CS + ch * 8);
      if (RES) {
        const bf16x8 rv = __builtin_bit_cast(bf16x8, rres[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(act_c<act2>((float)v[e] + (float)rv[e]));
      }
      const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, off, 0, YP);
      if constexpr (NT1 > 0) *reinterpret_cast<bf16x8*>(Cs + ml * CS + ch * 8) = v;
    }
    if constexpr (NT1 > 0) tail(m0);
  };

  if (BRES) {  // the weight slice, once: nk x [BN][BK] swizzled blocks
    for (int kt = 0; kt < nk; ++kt)
#pragma unroll
      for (int i = 0; i < B_INS; ++i)
        dma16(rw, Bres + kt * BN * BK + (wv * B_INS + i) * 512, b_off[i], kt * BK * 2);
  }
  if constexpr (NT1 > 0) {  // tail weights [n_t][Cout = BN], once, swizzled like Bres
    const __amdgpu_buffer_rsrc_t rw1 = mk_rsrc(p.w_t, p.n_t * p.Cout * 2);
    constexpr int B1 = NT1 / 32;
#pragma unroll
    for (int kt = 0; kt < BN / BK; ++kt)
#pragma unroll
      for (int i = 0; i < B1; ++i) {
        const int row = (wv * B1 + i) * 8 + lrow;
        const int off = row < p.n_t ? (row * p.Cout + (pch ^ ((row >> 1) & 7)) * 8) * 2 : kOOB;
        dma16(rw1, W1s + kt * NT1 * BK + (wv * B1 + i) * 512, off, kt * BK * 2);
      }
  }
  ResRegs rres[D];
  static_for<D - 1>([&](auto S) __attribute__((always_inline)) {
    constexpr int i = decltype(S)::value;
    issue(i, i, rres[i]);
  });
  zero_acc();
  // Stage j with j % D == u: ring slot u, residual registers rres[u].  The stage count
  // is rounded up to a multiple of D; the extra stages are all out of range (zero DMA,
  // no stores), which keeps every iteration's VMEM count -- and so the waits -- exact.
  const int nround = (nstages + D - 1) / D * D;
  dispatch_act(p.act, RES, [&](auto A1, auto A2) __attribute__((always_inline)) {
  for (int j0 = 0; j0 < nround; j0 += D) {
    static_for<D>([&](auto U) __attribute__((always_inline)) {
      constexpr int u = decltype(U)::value;
      const int j = j0 + u;
      const int ti = j / nk, kt = j - ti * nk;
      // Stage j landed.  Issued after it: stages j+1..j+D-2 (SI ops each) and the stores
      // of every epilogue in iterations [max(0, j-D+1), j-1].
      const int lo = j - D + 1 > 0 ? j - D + 1 : 0;
      const int e = j / nk - lo / nk;
      if (e <= 0) wait_vm<(D - 2) * SI>();
      else if (e == 1) wait_vm<(D - 2) * SI + EPI>();
      else if (e == 2) wait_vm<(D - 2) * SI + 2 * EPI>();
      else if (e == 3) wait_vm<(D - 2) * SI + 3 * EPI>();
      else if (e == 4) wait_vm<(D - 2) * SI + 4 * EPI>();
      else wait_vm<(D - 2) * SI + 5 * EPI>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // all waves: stage j visible, slot j-1 and C tile free
      asm volatile("" ::: "memory");
      constexpr int un = (u + D - 1) % D;
      issue(j + D - 1, un, rres[un]);
      compute(u, kt);
      if (kt == nk - 1) {
        epilogue(ti, rres[u], A1, A2);
        zero_acc();
      }
    });
  }
  });
}

}  // namespace

typedef void (*StreamFn)(const KvConvParams);

template <int BM, int BN, int D, bool BRES, int POL = 0, int MF = 32>
StreamFn stream_get(int mode, bool res, int nt) {
  if (nt) return nullptr;
  if (mode == 4) return conv_stream_kernel<BM, BN, D, 4, false, BRES, POL, 0, MF>;
  return res ? conv_stream_kernel<BM, BN, D, 1, true, BRES, POL, 0, MF>
             : conv_stream_kernel<BM, BN, D, 1, false, BRES, POL, 0, MF>;
}

// tail-capable tile: plain BRES tile for nt == 0, fused bottleneck tail for nt = 64 / 128
// (conv3 + residual -> next conv1, or the fused-downsample dual GEMM -> next conv1)
template <int BM, int BN, int D, int MF = 32>
StreamFn stream_get_tail(int mode, bool res, int nt) {
  if (nt == 0) return stream_get<BM, BN, D, true, 0, MF>(mode, res, 0);
  if constexpr (D == 3) if (nt == 64) {
    if (mode == 4) return conv_stream_kernel<BM, BN, D, 4, false, true, 0, 64, MF>;
    return res ? conv_stream_kernel<BM, BN, D, 1, true, true, 0, 64, MF> : nullptr;
  }
  if constexpr (D == 2) if (nt == 128) {
    if (mode == 4) return conv_stream_kernel<BM, BN, D, 4, false, true, 0, 128, MF>;
    return res ? conv_stream_kernel<BM, BN, D, 1, true, true, 0, 128, MF> : nullptr;
  }
  return nullptr;
}

struct StreamTile {
  int bm, bn, d;
  bool bres;
  StreamFn (*get)(int, bool, int);
};

static const StreamTile kStreamTiles[] = {
    // resident weight slice (BRES): only activations stream through the ring
    {64, 64, 4, true, &stream_get<64, 64, 4, true>},
    {64, 128, 4, true, &stream_get<64, 128, 4, true>},
    {128, 64, 4, true, &stream_get<128, 64, 4, true>},
    {64, 64, 6, true, &stream_get<64, 64, 6, true>},
    {64, 128, 3, true, &stream_get<64, 128, 3, true>},
    // weights streamed with every K step (large K)
    {64, 64, 4, false, &stream_get<64, 64, 4, false>},
    {128, 64, 4, false, &stream_get<128, 64, 4, false>},
    {128, 128, 3, false, &stream_get<128, 128, 3, false>},
    {64, 128, 4, false, &stream_get<64, 128, 4, false>},
    // nt (streaming) cache policy on activations / residual / output
    {64, 128, 3, true, &stream_get<64, 128, 3, true, 2>},
    {64, 64, 4, true, &stream_get<64, 64, 4, true, 2>},
    {128, 128, 3, false, &stream_get<128, 128, 3, false, 2>},
    // 128x128 with the weight slice resident (stage-3/4 expand: K = 256..512, N = 1024+):
    // half the A re-reads of BN = 64 across the N slices
    {128, 128, 3, true, &stream_get<128, 128, 3, true>},
    {128, 128, 2, true, &stream_get<128, 128, 2, true>},
    {128, 128, 3, true, &stream_get<128, 128, 3, true, 2>},
    // v_mfma_f32_16x16x32 main GEMM (MF = 16) of the tiles the autotuner picks for
    // ResNet-50 (stage-3 expand, stage-2 expand / reduce) and of both tail tiles
    {64, 64, 4, true, &stream_get<64, 64, 4, true, 0, 16>},
    {64, 128, 3, true, &stream_get<64, 128, 3, true, 0, 16>},
    {128, 128, 3, false, &stream_get<128, 128, 3, false, 2, 16>},
    {64, 256, 3, true, &stream_get_tail<64, 256, 3, 16>},
    {64, 256, 2, true, &stream_get_tail<64, 256, 2, 16>},
    // 64 x 256 resident slice; also the fused bottleneck-tail tiles (stream_tail_tile):
    // D = 3 for a 64-channel tail, D = 2 for a 128-channel one (register budget)
    {64, 256, 3, true, &stream_get_tail<64, 256, 3>},
    {64, 256, 2, true, &stream_get_tail<64, 256, 2>},
};

}  // namespace kvedge

namespace kvedge {

int stream_num_tiles() { return (int)(sizeof(kStreamTiles) / sizeof(kStreamTiles[0])); }
// default fused-tail tile: the 32x32x16 forms (last two entries); KVEDGE_TAIL_MF16=1 picks
// the 16x16x32 forms (the two entries before them) -- an A/B knob, as tails are not autotuned;
// measured neutral within box noise (profiles/r2_v22_ab_tail_mf16.jsonl)
int stream_tail_tile(int n_t) {
  static const int mf16 = [] {
    const char* s = getenv("KVEDGE_TAIL_MF16");
    return s && s[0] == '1' ? 2 : 0;
  }();
  return stream_num_tiles() - (n_t > 64 ? 1 : 2) - mf16;
}

int stream_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= stream_num_tiles()) return -6;
  if (p->mode != 1 && p->mode != 4) return -8;  // 1x1 stride-1 GEMM or fused dual only
  if (p->mode == 4 && (p->res || p->up2 || p->x2_coff)) return -8;  // plain dual sources only
  if ((long long)p->M * p->ldy * 2 >= kOOB || (p->res && (long long)p->M * p->ldr * 2 >= kOOB))
    return -9;
  const long long xb = (long long)p->N * p->H * p->W * p->ldx * 2;
  const long long wb = (long long)p->Cout * p->Kpad * 2;
  if (xb >= kOOB || wb >= kOOB) return -9;
  if (p->mode == 4) {
    const long long x2b = (long long)p->N * p->H2 * p->W2 * p->ldx2 * 2;
    if (!p->x2 || x2b >= kOOB || p->K1 % BK || (p->Kpad - p->K1) % BK) return -10;
  }
  const StreamTile& e = kStreamTiles[tile];
  const bool res = p->res != nullptr;
  if (p->n_t) {  // fused tail: the whole y row (all Cout channels) in one workgroup
    if ((p->n_t != 64 && p->n_t != 128) || e.bn != p->Cout || !p->z || !p->w_t ||
        p->act_t != 1 || p->ldz % 8 || p->z_coff % 8 || p->ldz < p->z_coff + p->n_t)
      return -8;
    if ((long long)p->M * p->ldz * 2 >= kOOB) return -9;
  }
  const int lds = stream_lds_bytes(e.bm, e.bn, e.d, res, e.bres, p->Kpad, p->n_t);
  if (lds > kLdsMax) return -11;  // resident weight slice does not fit
  const int nbm = (p->M + e.bm - 1) / e.bm, nbn = (p->Cout + e.bn - 1) / e.bn;
  if (nbm <= 0 || nbn <= 0) return 0;
  int per_cu = kLdsMax / lds;
  if (per_cu > 4) per_cu = 4;
  static const int per_cu_env = [] {  // tuning knob: cap resident workgroups per CU
    const char* s = getenv("KVEDGE_STREAM_PER_CU");
    return s ? atoi(s) : 0;
  }();
  if (per_cu_env > 0 && per_cu_env < per_cu) per_cu = per_cu_env;
  int mgroups = (256 * per_cu + nbn - 1) / nbn;  // ~per_cu workgroups on every CU
  if (mgroups > nbm) mgroups = nbm;
  if (mgroups < 1) mgroups = 1;
  StreamFn fn = e.get(p->mode, res, p->n_t);
  if (!fn) return -8;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(fn, dim3((unsigned)(mgroups * nbn)), dim3(256), (unsigned)lds, stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
