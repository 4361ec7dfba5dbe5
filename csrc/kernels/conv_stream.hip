// K3 v3 — persistent streaming 1x1 conv / GEMM for the HBM-bound layers (gfx950).
//
// Forward profile (tools/profile_forward.py, batch 256): ~50 % of a ResNet-50 step is
// 1x1 convs with K <= 512 that move far more bytes than they compute (bottleneck
// conv1 "reduce" and conv3 "expand + residual").  A one-tile-per-workgroup kernel
// serialises  load A,B -> MFMA -> epilogue (residual read + store)  inside every
// workgroup and leaves the overlap to occupancy alone; it reached 3.8-4.5 TB/s.
//
// Here a grid of ~3 workgroups per CU walks a flat stream of (M tile, K step) stages:
//  * a 2-slot LDS-DMA ring (buffer_load ... lds, as in conv_glds.hip) is fed ACROSS
//    tile boundaries: the first K step of tile i+1 is in flight while tile i finishes
//    its MFMAs and its epilogue;
//  * the residual of tile i+1 is prefetched into registers during tile i;
//  * the epilogue stages C through its own LDS region (not the ring) and issues
//    full-row 16-B stores that are never waited on;
//  * each workgroup keeps one N slice for all its tiles (grid % n-slices == 0), so the
//    weight slice stays hot in the CU's L1/L2.
// Modes: 1 = plain 1x1 (stride 1) GEMM, 4 = dual-source (conv3 + fused downsample).
#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace kvedge {
namespace {

constexpr int BK = 64;
constexpr int kOOB = 0x7ffffff0;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, bf16* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

template <int BM, int BN, int WM, int WN, int MODE, bool RES>
__global__ __launch_bounds__(256, 2) void conv_stream_kernel(const KvConvParams p) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_INS = BM / 32, B_INS = BN / 32;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int CS = BN + 8;
  constexpr int CPR = BN / 8;
  constexpr int PER = BM * CPR / 256;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1 && PER >= 1, "tile");
  // one LDS array (guide §5 trap (a)): [ring slot 0 | ring slot 1 | C tile]
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * STAGE + BM * CS];
  bf16* const Cs = smem + 2 * STAGE;
  // VMEM ops a wave issues after the next stage's DMA in an epilogue iteration:
  // PER output stores (+ PER residual prefetch loads).  Exact: every one of them is
  // always issued (out-of-range lanes get an offset past num_records instead).
  constexpr int EPI = PER + (RES ? PER : 0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.Cout + BN - 1) / BN;
  // grid is a multiple of nbn: this workgroup owns N slice nb for all its tiles
  const int nb = blockIdx.x % nbn;
  const int n0 = nb * BN;
  const int mstep = gridDim.x / nbn;
  const int mfirst = blockIdx.x / nbn;
  const int ntiles = mfirst < nbm ? (nbm - 1 - mfirst) / mstep + 1 : 0;
  const int nk = p.Kpad / BK;
  const int nstages = ntiles * nk;

  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(p.x, p.N * p.H * p.W * p.ldx * 2);
  const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.Cout * p.Kpad * 2);
  const __amdgpu_buffer_rsrc_t rx2 =
      mk_rsrc(MODE == 4 ? p.x2 : p.x, MODE == 4 ? p.N * p.H2 * p.W2 * p.ldx2 * 2 : 0);

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

  // issue one (tile, kt) stage into ring slot `slot`
  auto issue = [&](int s, int slot) {
    const int ti = s / nk, kt = s - ti * nk;
    const int m0 = (mfirst + ti * mstep) * BM;
    bf16* As = smem + slot * STAGE;
    bf16* Bs = As + BM * BK;
    const int kbase = kt * BK;
    if (MODE == 4 && kbase >= p.K1) {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int m = m0 + (wv * A_INS + i) * 8 + lrow;
        int v = kOOB;
        if (m < p.M) {
          const int img = m / HoWo, rem = m - (m / HoWo) * HoWo;
          const int ho = rem / p.Wo, wo = rem - (rem / p.Wo) * p.Wo;
          v = (((img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2) * p.ldx2 + a_lc[i] * 8) * 2;
        }
        dma16(rx2, As + (wv * A_INS + i) * 512, v, (kbase - p.K1) * 2);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int m = m0 + (wv * A_INS + i) * 8 + lrow;
        const bool ok = m < p.M && (MODE == 4 || kbase + a_lc[i] * 8 < p.Cin);
        const int v = ok ? (m * p.ldx + p.x_coff + a_lc[i] * 8) * 2 : kOOB;
        dma16(rx, As + (wv * A_INS + i) * 512, v, kbase * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) dma16(rw, Bs + (wv * B_INS + i) * 512, b_off[i], kbase * 2);
  };

  const __amdgpu_buffer_rsrc_t rr = mk_rsrc(RES ? p.res : p.x, RES ? p.M * p.ldr * 2 : 0);
  const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, p.M * p.ldy * 2);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 rpre[PER];
  auto prefetch_res = [&](int ti) {  // always issues PER loads (counted waits rely on it)
    if (!RES) return;
    const int m0 = (mfirst + ti * mstep) * BM;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = tid + 256 * j;
      const int m = m0 + idx / CPR, n = n0 + (idx % CPR) * 8;
      const int off = (ti < ntiles && m < p.M && n < p.Cout) ? (m * p.ldr + p.r_coff + n) * 2 : kOOB;
      rpre[j] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    }
  };

  floatx16 acc[TN][TM];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  };

  const int fr = lane & 31, fh = lane >> 5;
  auto compute = [&](int slot) {
    const bf16* As = smem + slot * STAGE;
    const bf16* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int q = ks * 2 + fh;
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * 32 + fr;
        af[tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((q ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * 32 + fr;
        bfg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((q ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tn][tm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfg[tn], af[tm], acc[tn][tm], 0, 0, 0);
    }
  };

  const int act_fn = p.act & 3;
  const bool res_post = (p.act & 4) != 0;
  const int act1 = (RES && !res_post) ? kActNone : act_fn;
  const int act2 = res_post ? kActNone : act_fn;
  bf16* __restrict__ Y = reinterpret_cast<bf16*>(p.y);

  // this lane's bias values for the whole run (the N slice is fixed): registers, not
  // LDS -- an LDS read here would make hipcc drain the in-flight LDS-DMA (vmcnt(0)).
  float4 bias_r[TN][4];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = n0 + wn * WTN + tn * 32 + g * 8 + fh * 4;
      bias_r[tn][g] = (p.bias && n < p.Cout) ? *reinterpret_cast<const float4*>(p.bias + n)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  auto epilogue = [&](int ti) {
    const int m0 = (mfirst + ti * mstep) * BM;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * WTN + tn * 32 + g * 8 + fh * 4;
        const float4 bv = bias_r[tn][g];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int ml = wm * WTM + tm * 32 + fr;
          bf16x4 o;
          o[0] = f2bf(apply_act_bf(acc[tn][tm][4 * g + 0] + bv.x, act1));
          o[1] = f2bf(apply_act_bf(acc[tn][tm][4 * g + 1] + bv.y, act1));
          o[2] = f2bf(apply_act_bf(acc[tn][tm][4 * g + 2] + bv.z, act1));
          o[3] = f2bf(apply_act_bf(acc[tn][tm][4 * g + 3] + bv.w, act1));
          *reinterpret_cast<bf16x4*>(Cs + ml * CS + nl) = o;
        }
      }
    }
    // C tile complete: LDS writes drained + raw barrier (no vmcnt: the next stage's
    // DMA and the previous stores stay in flight)
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
        const bf16x8 rv = __builtin_bit_cast(bf16x8, rpre[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(apply_act_bf((float)v[e] + (float)rv[e], act2));
      }
      const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry, off, 0, 0);
    }
  };

  if (nstages == 0) return;
  prefetch_res(0);
  issue(0, 0);
  zero_acc();
  bool after_epi = false;
  for (int s = 0; s < nstages; ++s) {
    const int slot = s & 1;
    const int ti = s / nk, kt = s - ti * nk;
    // stage s landed: after an epilogue its EPI stores/prefetches are younger than this
    // stage's DMA and may stay in flight; otherwise drain everything.
    if (after_epi)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EPI) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all waves: stage s visible, slot^1 and C tile free
    asm volatile("" ::: "memory");
    // unconditional: past the last stage this fetches zeros/weights into the free slot.
    // A conditional issue makes hipcc's waitcnt merge assume the residual prefetch may
    // be the youngest VMEM op and emit vmcnt(1) in the epilogue (drains the ring).
    issue(s + 1, slot ^ 1);
    compute(slot);
    after_epi = false;
    if (kt == nk - 1) {
      epilogue(ti);
      prefetch_res(ti + 1);  // rides behind the stores; consumed one tile later
      zero_acc();
      after_epi = true;
    }
  }
}

}  // namespace

typedef void (*StreamFn)(const KvConvParams);

template <int BM, int BN, int WM, int WN>
StreamFn stream_get(int mode, bool res) {
  if (mode == 4) return conv_stream_kernel<BM, BN, WM, WN, 4, false>;
  return res ? conv_stream_kernel<BM, BN, WM, WN, 1, true> : conv_stream_kernel<BM, BN, WM, WN, 1, false>;
}

struct StreamTile {
  int bm, bn, per_cu;
  StreamFn (*get)(int, bool);
};

static const StreamTile kStreamTiles[] = {
    // per_cu = workgroups the LDS footprint lets one CU hold (2 ring slots + C tile)
    {64, 64, 3, &stream_get<64, 64, 2, 2>},     //  41 KB
    {64, 128, 2, &stream_get<64, 128, 2, 2>},   //  65 KB
    {128, 64, 2, &stream_get<128, 64, 2, 2>},   //  65 KB
    {128, 128, 1, &stream_get<128, 128, 2, 2>}, //  99 KB
};

int stream_num_tiles() { return (int)(sizeof(kStreamTiles) / sizeof(kStreamTiles[0])); }

int stream_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= stream_num_tiles()) return -6;
  if (p->mode != 1 && p->mode != 4) return -8;  // 1x1 stride-1 GEMM or fused dual only
  if (p->mode == 4 && p->res) return -8;
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
  const int nbm = (p->M + e.bm - 1) / e.bm, nbn = (p->Cout + e.bn - 1) / e.bn;
  if (nbm <= 0 || nbn <= 0) return 0;
  int mgroups = (256 * e.per_cu + nbn - 1) / nbn;  // ~per_cu workgroups per CU
  if (mgroups > nbm) mgroups = nbm;
  if (mgroups < 1) mgroups = 1;
  hipLaunchKernelGGL(e.get(p->mode, p->res != nullptr), dim3((unsigned)(mgroups * nbn)), dim3(256),
                     0, stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
