// v10 -- persistent LDS-DMA implicit GEMM with the epilogue overlapped by the next tile.
//
// The compute-bound layers of ResNet-50 stages 3-4 (3x3 256/512, the fused-downsample dual
// GEMMs, the 1x1 reduce convs) run the v2/v7 8-wave 256 x 256 tiles at one workgroup per CU.
// PMC put MFMA busy at 44 %; a two-shape fit put ~12 us per tile ROUND into each tile's
// prologue (first K step's DMA latency, every CU at once) and epilogue (every CU storing its
// 128 KB C tile at once): docs/kernels.md "Round 3: measured and rejected" (XP row).  In-loop
// the same tiles reach ~1.3 PF/s.
//
// Here one workgroup per CU stays resident and walks tiles t = b, b + G, b + 2G ... (G =
// grid size; the XCD remap keeps consecutive tiles, which share A rows, on one XCD's L2).
// The last K step of tile i issues tile i+1's bias load and its first K stage (LDS DMA into
// the ring slot the last step does not read), THEN runs its MFMAs, and the epilogue of
// tile i -- bias + ReLU in registers, v_permlane16_swap to 8 consecutive channels per lane,
// 16-B buffer stores straight from the accumulators (the v7 "DE" form) -- runs while that
// stage lands.  The stores are younger than the stage in the in-order vmcnt, so tile i+1's
// first wait is vmcnt(#stores) and they drain under its main loop.  After the first round the
// CUs are out of phase, so store bursts and prologue fetches no longer hit HBM all at once.
//
// Scope: MODE 0 (KxK conv, Cin % 64 == 0), 1 (1x1 GEMM, Cin % 64 == 0), 4 (dual-source conv3
// + downsample); no residual (the residual layers are v6 / v9 seams); BK = 64, 2-slot ring,
// v_mfma_f32_16x16x32_bf16, 8 waves.  Every VMEM op of the main loop is an opaque LDS DMA
// (kv_lds_dma16) or a buffer store issued by every lane, so each wave's op sequence is fixed
// and every wait is an exact counted s_waitcnt.
#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int kPdOOB = 0x7ffffff0;

template <int N>
__device__ __forceinline__ void pd_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void pd_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int pd_sw(int r) { return (r >> 1) & 7; }

typedef unsigned int pd_u32x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(512, 1) void conv_pde_kernel(const KvConvParams p, int ntiles) {
  constexpr int NW = WM * WN, NT = 64 * NW, BK = 64;
  static_assert(NW == 8, "8 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  static_assert(TM >= 1 && TN >= 2 && TN % 2 == 0, "16x16 blocks, block pairs for the DE stores");
  constexpr int A_INS = BM / (NW * 8), B_INS = BN / (NW * 8), OPS = A_INS + B_INS;
  static_assert(A_INS >= 1 && B_INS >= 1, "tile");
  constexpr int STAGE = (BM + BN) * BK;          // bf16 elements per ring slot
  constexpr int NST = (TN / 2) * TM;             // 16-B stores per lane per epilogue
  static_assert(NST <= 63, "vmcnt");
  // ring + the bias table of the current and the next tile (1 KB DMA each: BN <= 256)
  static_assert(BN <= 256, "one 1-KB bias DMA per tile");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE + 2 * 256 * 2];
  float* const lbias = reinterpret_cast<float*>(smem + 2 * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.Cout + BN - 1) / BN;
  const int G = gridDim.x;
  const int nk = p.Kpad / BK;

  const kv_i32x4 rx = kv_rsrc4(p.x, p.N * p.H * p.W * p.ldx * 2);
  const kv_i32x4 rw = kv_rsrc4(p.w, p.Cout * p.Kpad * 2);
  const kv_i32x4 rx2 = kv_rsrc4(MODE == 4 ? p.x2 : p.x, MODE == 4 ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);
  const kv_i32x4 rb = kv_rsrc4(p.bias, p.bias ? p.Cout * 4 : 0);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.M * p.ldy * 2, 0x00020000);

  // ---- per-tile DMA descriptors (set up for the NEXT tile during the current one's last
  // K step: the current tile issues no more DMA after that point)
  const int lrow = lane >> 3, pch = lane & 7;
  int a_off[A_INS], a_off2[A_INS], b_off[B_INS];
  unsigned a_msk[A_INS];
  int k_c0 = 0, k_r = 0, k_s = 0;  // MODE 0 K walk (tap row, tap col, channel base)
  const int HoWo = p.Ho * p.Wo;
  // tile t's descriptors + its bias table DMA into lbias[par] (issued before its first K
  // stage, so that stage's wait covers it; every wave issues the same 1-KB DMA: identical
  // bytes, uniform per-wave op counts)
  auto setup = [&](int t, int par) __attribute__((always_inline)) {
    const int m0 = (t / nbn) * BM, n0 = (t % nbn) * BN;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int row = (wv * A_INS + i) * 8 + lrow;
      const int lc = pch ^ pd_sw(row);
      const int m = m0 + row;
      a_msk[i] = 0u;
      a_off2[i] = kPdOOB;
      if constexpr (MODE == 1 || MODE == 4) {
        a_off[i] = m < p.M ? (m * p.ldx + p.x_coff + lc * 8) * 2 : kPdOOB;
        if (MODE == 4 && m < p.M) {
          const int img = m / HoWo, rem = m - img * HoWo;
          const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
          a_off2[i] = (((img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2) * p.ldx2 + lc * 8) * 2;
        }
      } else {
        a_off[i] = 0;
        if (m < p.M) {
          const int img = m / HoWo, rem = m - img * HoWo;
          const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
          const int h0 = ho * p.stride - p.pad, w0 = wo * p.stride - p.pad;
          a_off[i] = ((img * p.H + h0) * p.W + w0) * p.ldx + p.x_coff + lc * 8;  // may be < 0
          unsigned msk = 0;
          for (int r = 0; r < p.KH; ++r)
            for (int s = 0; s < p.KW; ++s)
              if ((unsigned)(h0 + r) < (unsigned)p.H && (unsigned)(w0 + s) < (unsigned)p.W)
                msk |= 1u << (r * p.KW + s);
          a_msk[i] = msk;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int row = (wv * B_INS + i) * 8 + lrow;
      const int n = n0 + row;
      b_off[i] = n < p.Cout ? (n * p.Kpad + (pch ^ pd_sw(row)) * 8) * 2 : kPdOOB;
    }
    k_c0 = k_r = k_s = 0;
    kv_lds_dma16(rb, lbias + par * 256, n0 * 4 + lane * 16);  // past Cout: zero-filled
  };

  auto issue = [&](int slot, int kt) __attribute__((always_inline)) {
    bf16* As = smem + slot * STAGE;
    bf16* Bs = As + BM * BK;
    if constexpr (MODE == 1) {
      const int kb2 = kt * BK * 2;
#pragma unroll
      for (int i = 0; i < A_INS; ++i)
        kv_lds_dma16(rx, As + (wv * A_INS + i) * 512, a_off[i] != kPdOOB ? a_off[i] + kb2 : kPdOOB);
    } else if constexpr (MODE == 4) {
      const int kbase = kt * BK;  // K1 and K - K1 are multiples of 64
      if (kbase < p.K1) {
#pragma unroll
        for (int i = 0; i < A_INS; ++i)
          kv_lds_dma16(rx, As + (wv * A_INS + i) * 512, a_off[i] != kPdOOB ? a_off[i] + kbase * 2 : kPdOOB);
      } else {
#pragma unroll
        for (int i = 0; i < A_INS; ++i)
          kv_lds_dma16(rx2, As + (wv * A_INS + i) * 512,
                       a_off2[i] != kPdOOB ? a_off2[i] + (kbase - p.K1) * 2 : kPdOOB);
      }
    } else {
      const int tap = k_r * p.KW + k_s;
      const int toff = (k_r * p.W + k_s) * p.ldx + k_c0;
      k_c0 += BK;
      if (k_c0 >= p.Cin) {
        k_c0 = 0;
        if (++k_s == p.KW) { k_s = 0; ++k_r; }
      }
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const bool ok = tap < p.KH * p.KW && ((a_msk[i] >> tap) & 1u);
        kv_lds_dma16(rx, As + (wv * A_INS + i) * 512, ok ? (a_off[i] + toff) * 2 : kPdOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i)
      kv_lds_dma16(rw, Bs + (wv * B_INS + i) * 512, b_off[i] != kPdOOB ? b_off[i] + kt * BK * 2 : kPdOOB);
  };

  floatx4 acc[TN][TM];
  const int fr = lane & 15, fh = lane >> 4;
  auto compute = [&](int slot) __attribute__((always_inline)) {
    const bf16* As = smem + slot * STAGE;
    const bf16* Bs = As + BM * BK;
    bf16x8 af[2][TM], bfg[2][TN];
    auto load = [&](int buf, int ks) __attribute__((always_inline)) {
      const int q = ks * 4 + fh;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * 16 + fr;
        af[buf][tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((q ^ pd_sw(row)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * 16 + fr;
        bfg[buf][tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((q ^ pd_sw(row)) << 3));
      }
    };
    load(0, 0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) load(1, 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[ks][tn], af[ks][tm], acc[tn][tm], 0, 0, 0);
    }
    // reads(0) | reads(1) MFMAs(0) | MFMAs(1)
    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
  };

  // tile walk: physical index b + i G -> logical tile via the bijective XCD remap
  const int total = nbm * nbn;
  int tp = blockIdx.x;
  if (tp >= total) return;
  int t = xcd_remap(tp, total);
  setup(t, 0);
  issue(0, 0);
  int slot = 0;
  const int rho = lane >> 4;
  const int csel = 16 * (rho & 1) + 8 * (rho >> 1);  // channel offset within a block pair
  for (int it = 0;; ++it) {
    const int m0 = (t / nbn) * BM, n0 = (t % nbn) * BN;
    const int tpn = tp + G;
    const bool more = tpn < total;
    const int tn_next = more ? xcd_remap(tpn, total) : 0;
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    // stage 0 (and, older, the tile's bias table) landed; from the second tile on, the
    // previous tile's epilogue stores (NST per wave, younger) may stay in flight
    if (it == 0) pd_wait_vm<0>();
    else pd_wait_vm<NST>();
    pd_barrier();  // ... for every wave; the other slot is no longer read
    for (int kt = 0; kt + 1 < nk; ++kt) {
      issue(slot ^ 1, kt + 1);
      compute(slot);
      slot ^= 1;
      pd_wait_vm<0>();  // stage kt + 1: the only op issued since
      pd_barrier();
    }
    if (more) {
      // the last K step: this tile issues no more DMA, so its descriptors are free.
      // lbias[(it + 1) & 1] was last read by tile it-1's epilogue, before this tile's first
      // barrier; the next tile's first stage lands during this tile's epilogue
      setup(tn_next, (it + 1) & 1);
      issue(slot ^ 1, 0);
    }
    compute(slot);
    slot ^= 1;
    // ---- direct epilogue (the bias table landed with stage 0, published by its barrier): bias + act on the accumulators, 8 channels per lane via
    // v_permlane16_swap, one 16-B store per block pair and 16-pixel row (conv_glds_kernel.inc DE)
    const float* bt = lbias + (it & 1) * 256;
    dispatch_act(p.act, false, [&](auto A1, auto) __attribute__((always_inline)) {
      constexpr int act1 = decltype(A1)::value;
#pragma unroll
      for (int tn = 0; tn < TN; tn += 2) {
        const int nl = wn * WTN + tn * 16;  // first channel of the block pair, tile-local
        const float4 bv0 = *reinterpret_cast<const float4*>(bt + nl + fh * 4);
        const float4 bv1 = *reinterpret_cast<const float4*>(bt + nl + 16 + fh * 4);
        const int n = n0 + nl + csel;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          bf16x4 a, b;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[j] = f2bf(act_c<act1>(acc[tn][tm][j] + (&bv0.x)[j]));
            b[j] = f2bf(act_c<act1>(acc[tn + 1][tm][j] + (&bv1.x)[j]));
          }
          uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
          const auto r0 = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
          ua.x = r0[0]; ub.x = r0[1];
          ua.y = r1[0]; ub.y = r1[1];
          const int m = m0 + wm * WTM + tm * 16 + fr;
          const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kPdOOB;
          const pd_u32x4 v = {ua.x, ua.y, ub.x, ub.y};
          __builtin_amdgcn_raw_buffer_store_b128(v, ry, off, 0, 0);
        }
      }
    });
    if (!more) break;
    tp = tpn;
    t = tn_next;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

typedef void (*PdFn)(const KvConvParams, int);

struct PdTile {
  int bm, bn;
  PdFn f0, f1, f4;
};

template <int BM, int BN, int WM, int WN>
constexpr PdTile pd_tile() {
  return PdTile{BM, BN, &conv_pde_kernel<BM, BN, WM, WN, 0>, &conv_pde_kernel<BM, BN, WM, WN, 1>,
                &conv_pde_kernel<BM, BN, WM, WN, 4>};
}

static const PdTile kPdTiles[] = {
    pd_tile<256, 256, 4, 2>(),  // 64 px x 128 ch per wave (the v7 DE tile's layout)
    pd_tile<256, 256, 2, 4>(),  // 128 px x 64 ch per wave
    pd_tile<256, 128, 4, 2>(),  // N = 128 / 512 layers, 64 x 64 per wave
};

}  // namespace

int pde_num_tiles() { return (int)(sizeof(kPdTiles) / sizeof(kPdTiles[0])); }

int pde_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= pde_num_tiles()) return -6;
  const PdTile& e = kPdTiles[tile];
  if (p->res || p->n_t || p->in_u8 || p->pair_1x1) return -8;  // no residual / fused tails
  if (p->Kpad % 64 || p->Cout % 8 || p->ldy % 8 || p->y_coff % 8) return -8;
  PdFn fn = nullptr;
  if (p->mode == 0) {
    if (p->Cin % 64 || p->KH * p->KW > 32 || p->ldx % 8 || p->x_coff % 8) return -8;
    fn = e.f0;
  } else if (p->mode == 1) {
    if (p->Cin % 64 || p->Kpad != p->Cin || p->ldx % 8 || p->x_coff % 8) return -8;
    fn = e.f1;
  } else if (p->mode == 4) {
    if (!p->x2 || p->K1 % 64 || (p->Kpad - p->K1) % 64 || p->ldx2 % 8 || p->ldx % 8) return -8;
    if ((long long)p->N * p->H2 * p->W2 * p->ldx2 * 2 >= kPdOOB) return -9;
    fn = e.f4;
  } else {
    return -8;
  }
  if ((long long)p->N * p->H * p->W * p->ldx * 2 >= kPdOOB || (long long)p->Cout * p->Kpad * 2 >= kPdOOB ||
      (long long)p->M * p->ldy * 2 >= kPdOOB || (long long)p->M >= (1 << 26))
    return -9;
  const long long total = (long long)((p->M + e.bm - 1) / e.bm) * ((p->Cout + e.bn - 1) / e.bn);
  if (total <= 0) return 0;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const unsigned g = (unsigned)(total < ncu ? total : ncu);
  hipLaunchKernelGGL(fn, dim3(g), dim3(512), 0, stream, *p, (int)total);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
