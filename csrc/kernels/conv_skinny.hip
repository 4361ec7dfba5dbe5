// v12: skinny implicit-GEMM convolution for edge batches (batch 1-8).
//
// At the module's small batches the ResNet-50 layers of stages 2-4 and the head have a few
// hundred output rows (M = 196 per image in stage 3, 49 in stage 4, 1 for the FC).  The
// 64 x 64+ tiles of the other families then launch a few dozen workgroups, each walking the
// whole reduction serially: the in-graph table of the batch-1 step
// (profiles/r5_v6_graph_layers_rn_b1.md) has a 1x1 1024 > 256 @14x14 at 6.6 us on 16
// workgroups and every 3x3 of stages 3 / 4 at 13-14 us as split-K GEMM + finalize launch,
// against well under 1 us of compulsory traffic.  The per-workgroup byte count of a tile is
// 2 K (BM + BN), so the cure is a small tile and many workgroups, with the reduction split
// inside the workgroup instead of across launches:
//
//   - a workgroup owns a (16 MB) x (16 NB) output tile; its WAVES waves split K in 64-wide
//     chunks (chunk c goes to wave c % WAVES);
//   - every wave streams its chunks through a private ring of R LDS slots (R chunks in
//     flight per wave, WAVES x R per workgroup: a layer of at most that many chunks costs one
//     memory latency, not one per K step) as LDS DMA (buffer_load ... lds, lane-linear: eight
//     lanes per 128-B row segment).  The first form loaded the MFMA fragments straight into
//     VGPRs: every 16-lane group of a load then touched 16 rows, and a 3x3 of stage 4 ran at
//     about a quarter of the L2 -> CU rate (profiles/r5_v7_skinny_tiles_b1.md vs
//     r5_v8_skinny_tiles_b1.md);
//   - padding taps, rows past M, channels past Cout and chunks past K read an offset beyond
//     the buffer descriptor and land as zeros, so every ring step issues the same DMA count
//     and one counted s_waitcnt vmcnt per chunk suffices (no barrier: each wave reads only
//     its own slots);
//   - the waves' fp32 partial tiles are summed through LDS by the epilogue threads, which
//     add bias and residual, apply the activation and store bf16 -- no split-K workspace and
//     no finalize launch.
//
// MFMA: v_mfma_f32_16x16x32_bf16 with the weights as the first operand (D = W . A^T), so a
// lane's four accumulators are four consecutive output channels of one pixel, as in
// conv_nloop.hip.  Within a 64-wide chunk, MFMA step s and lane quarter q cover reduction
// indices s*32 + q*8 .. +8 of BOTH operands (16-B piece 4s + q of the row's 128 B), read
// from the slot with an XOR swizzle (piece ^ row % 8) that the DMA source addresses apply.
// The blockIdx -> tile map is n-major through xcd_remap, so the m-tiles that share a weight
// panel run on one XCD and share its L2.
#include <algorithm>

#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

typedef unsigned int skn_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int skn_u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kSknOOB = 0x80000000u;  // >= every descriptor's byte count (< 2 GiB)

__device__ __forceinline__ int skn_bytes(long long bytes) {
  return (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t skn_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes),
                                           0x00020000);
}

// FastDiv (common.h) cannot encode d = 1 (its multiplier would be 2^32); used once per lane
__device__ __forceinline__ int skn_div(int n, FastDiv f) { return f.d == 1 ? n : fdiv(n, f); }
// quotient of a small wave-uniform index (chunk -> tap -> kernel row: n < 2^12, d <= 64) by
// its float reciprocal, branch-free: (n + 0.5) / d stays >= 1 / (2d) away from every integer
__device__ __forceinline__ int skn_qdiv(int n, float inv) {
  return (int)(((float)n + 0.5f) * inv);
}

// MODE: 0 general (KH x KW window, stride, padding), 1 1x1 / stride 1 GEMM, 4 dual 1x1 source
// (bottleneck conv3 + the downsample folded in as extra K: kvedge_kernels.h, mode 4)
template <int MODE, int WAVES, int R, int MB, int NB>
__global__ __launch_bounds__(WAVES * 64) void conv_skinny_kernel(const KvConvParams p, int mt,
                                                                 int ntiles, float inv_cpt,
                                                                 float inv_kw, FastDiv hw_d,
                                                                 FastDiv wo_d) {
  extern __shared__ __attribute__((aligned(16))) char skn_lds[];
  constexpr int kChunk = (MB + NB) * 2048;  // one 64-wide chunk: 16 rows x 128 B per block
  constexpr int kDma = 2 * (MB + NB);       // LDS-DMA instructions per chunk
  static_assert(R * kDma <= 63, "vmcnt field");
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if (L >= ntiles) return;
  const int ntile = L / mt, mtile = L - ntile * mt;  // n-major: one weight panel per XCD run
  const int m0 = mtile * 16 * MB, n0 = ntile * 16 * NB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr bool dual = MODE == 4;
  constexpr bool gemm = MODE != 0;  // 1x1 / stride 1 sources: pixel index = output row
  char* const wlds = skn_lds + w * R * kChunk;  // this wave's ring of chunk slots

  const kv_i32x4 rx = kv_rsrc4(p.x, skn_bytes((long long)p.N * p.H * p.W * p.ldx * 2));
  const kv_i32x4 rx2 =
      kv_rsrc4(dual ? p.x2 : p.x, dual ? skn_bytes((long long)p.N * p.H2 * p.W2 * p.ldx2 * 2) : 0);
  const kv_i32x4 rw = kv_rsrc4(p.w, skn_bytes((long long)p.Cout * p.Kpad * 2));

  // ---- epilogue operands first (the oldest loads: back long before the epilogue).  Item =
  // one lane's four output channels of one 16 x 16 block; a thread owns kIter of them
  constexpr int kItems = 64 * MB * NB;
  constexpr int kIter = (kItems + WAVES * 64 - 1) / (WAVES * 64);
  int e_m[kIter], e_n[kIter];
  bool e_ok[kIter];
  floatx4 bias4[kIter];
  skn_u32x2 res2[kIter];
#pragma unroll
  for (int it = 0; it < kIter; ++it) {
    const int item = threadIdx.x + it * WAVES * 64;
    const int ej = item >> 6, el = item & 63;
    const int e_nb = ej / MB, e_mb = ej - e_nb * MB;
    e_n[it] = n0 + e_nb * 16 + (el >> 4) * 4;
    e_m[it] = m0 + e_mb * 16 + (el & 15);
    e_ok[it] = item < kItems && e_m[it] < p.M && e_n[it] < p.Cout;
    bias4[it] = floatx4{0.f, 0.f, 0.f, 0.f};
    res2[it] = skn_u32x2{0u, 0u};
    if (p.bias) {
      const __amdgpu_buffer_rsrc_t rb = skn_rsrc(p.bias, (long long)p.Cout * 4);
      bias4[it] = __builtin_bit_cast(
          floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                       rb, e_ok[it] ? (unsigned)e_n[it] * 4u : kSknOOB, 0, 0));
    }
    if (p.res) {
      const __amdgpu_buffer_rsrc_t rr = skn_rsrc(p.res, (long long)p.M * p.ldr * 2);
      res2[it] = __builtin_amdgcn_raw_buffer_load_b64(
          rr, e_ok[it] ? (unsigned)(e_m[it] * p.ldr + p.r_coff + e_n[it]) * 2u : kSknOOB, 0, 0);
    }
  }

  // ---- DMA geometry: DMA j (0, 1) of a 16-row block brings rows 8j + (lane >> 3); lane
  // l & 7 fetches 16-B piece g = (l & 7) ^ (row & 7) of the row's 128-B chunk, which lands in
  // LDS slot l & 7 (lane-linear DMA): the XOR swizzle keeps the fragment reads conflict-free
  const int g = (lane & 7) ^ (lane >> 3);
  int pixb[MB][2], hi0[MB][2], wi0[MB][2], pix2[MB][2];
  bool mval[MB][2];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + mb * 16 + 8 * j + (lane >> 3);
      mval[mb][j] = m < p.M;
      const int img = skn_div(m, hw_d), rem = m - img * hw_d.d;
      const int ho = skn_div(rem, wo_d), wo = rem - ho * wo_d.d;
      hi0[mb][j] = ho * p.stride - p.pad;
      wi0[mb][j] = wo * p.stride - p.pad;
      pixb[mb][j] = gemm ? m : (img * p.H + hi0[mb][j]) * p.W + wi0[mb][j];
      pix2[mb][j] = dual ? (img * p.H2 + ho * p.stride2) * p.W2 + wo * p.stride2 : 0;
    }
  unsigned wrow[NB][2];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + nb * 16 + 8 * j + (lane >> 3);
      wrow[nb][j] = n < p.Cout ? (unsigned)n * (unsigned)p.Kpad * 2u + (unsigned)g * 16u : kSknOOB;
    }

  const int nch = p.K >> 6;
  const int nloc = (nch - w + WAVES - 1) / WAVES;  // this wave's chunks: c = w + WAVES * i
  floatx4 acc[NB][MB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = floatx4{0.f, 0.f, 0.f, 0.f};
  // fragment read offsets: lane (r16, q), MFMA step s reads piece 4s + q of row r16
  const int r16 = lane & 15, q = lane >> 4;
  const int frag0 = r16 * 128 + ((q ^ (r16 & 7)) << 4);
  const int frag1 = r16 * 128 + (((4 + q) ^ (r16 & 7)) << 4);

  // the kDma DMAs of local chunk i into a slot; past the wave's last chunk every offset is
  // out of range (zero-fill, no memory traffic), so each ring step issues the same count
  auto issue = [&](int i, char* slot) __attribute__((always_inline)) {
    const int c = w + WAVES * i;  // wave-uniform
    const bool cin = i < nloc;
    const int k0 = c * 64;
    bool second = false;
    int tap_off = 0, cin0 = k0, r = 0, s = 0;
    if constexpr (dual) {
      second = k0 >= p.K1;
      cin0 = second ? k0 - p.K1 : k0;
    } else if constexpr (!gemm) {
      const int t = skn_qdiv(c, inv_cpt);
      cin0 = k0 - t * p.Cin;
      r = skn_qdiv(t, inv_kw);
      s = t - r * p.KW;
      tap_off = r * p.W + s;
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bool ok = cin && mval[mb][j];
        int pix = pixb[mb][j] + tap_off;
        int ld = p.ldx, coff = p.x_coff;
        if constexpr (!gemm)
          ok = ok && (unsigned)(hi0[mb][j] + r) < (unsigned)p.H &&
               (unsigned)(wi0[mb][j] + s) < (unsigned)p.W;
        if (dual && second) {
          pix = pix2[mb][j];
          ld = p.ldx2;
          coff = 0;
        }
        const unsigned off =
            ok ? (unsigned)(pix * ld + coff + cin0) * 2u + (unsigned)g * 16u : kSknOOB;
        kv_lds_dma16(dual && second ? rx2 : rx, slot + mb * 2048 + j * 1024, (int)off);
      }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned off = cin ? wrow[nb][j] + (unsigned)k0 * 2u : kSknOOB;
        kv_lds_dma16(rw, slot + MB * 2048 + nb * 2048 + j * 1024, (int)off);
      }
  };

  // ring of R chunk slots per wave: R chunks in flight, chunk i consumed once its DMAs have
  // landed (the (R - 1) x kDma younger ones may still be in flight; this wave's own slots, so
  // no barrier), its slot refilled with chunk i + R as soon as the fragments are in VGPRs
  static_range<0, R>([&](auto ic) { issue(decltype(ic)::value, wlds + decltype(ic)::value * kChunk); });
  int si = 0;
  for (int i = 0; i < nloc; ++i) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDma * (R - 1)) : "memory");
    char* slot = wlds + si * kChunk;
    bf16x8 af[2][MB], bfr[2][NB];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int fo = st ? frag1 : frag0;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        af[st][mb] = *reinterpret_cast<const bf16x8*>(slot + mb * 2048 + fo);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        bfr[st][nb] = *reinterpret_cast<const bf16x8*>(slot + MB * 2048 + nb * 2048 + fo);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is read out: refill it
    issue(i + R, slot);
    si = si + 1 == R ? 0 : si + 1;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[st][nb], af[st][mb], acc[nb][mb], 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing zero-fills land first

  // ---- sum the waves' partial tiles (over the chunk slots), then bias / residual /
  // activation -> bf16
  __syncthreads();
  floatx4* red = reinterpret_cast<floatx4*>(skn_lds);  // [WAVES][MB * NB][64]
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) red[(w * MB * NB + nb * MB + mb) * 64 + lane] = acc[nb][mb];
  __syncthreads();
  const int act = p.act & 3;
  const bool after = (p.act & 4) != 0;
  const __amdgpu_buffer_rsrc_t ry = skn_rsrc(p.y, (long long)p.M * p.ldy * 2);
#pragma unroll
  for (int it = 0; it < kIter; ++it) {
    const int item = threadIdx.x + it * WAVES * 64;
    if (item >= kItems) break;
    const int ej = item >> 6, el = item & 63;
    floatx4 v = red[ej * 64 + el];
#pragma unroll
    for (int ww = 1; ww < WAVES; ++ww) v += red[(ww * MB * NB + ej) * 64 + el];
    const bf16x4 r4 = __builtin_bit_cast(bf16x4, res2[it]);
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e] + bias4[it][e];
      const float rr = p.res ? (float)r4[e] : 0.f;
      if (!after) x += rr;
      x = apply_act(x, act);
      if (after) x += rr;
      o[e] = f2bf(x);
    }
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(skn_u32x2, o), ry,
        e_ok[it] ? (unsigned)(e_m[it] * p.ldy + p.y_coff + e_n[it]) * 2u : kSknOOB, 0, 0);
  }
}

typedef void (*SknFn)(const KvConvParams, int, int, float, float, FastDiv, FastDiv);
struct SknTile {
  SknFn fn[3];  // general, 1x1 GEMM, dual
  int waves, ring, mb, nb;
};
#define KV_SKN(W, R, M, N)                                                             \
  {{&conv_skinny_kernel<0, W, R, M, N>, &conv_skinny_kernel<1, W, R, M, N>,            \
    &conv_skinny_kernel<4, W, R, M, N>},                                               \
   W, R, M, N}
// (waves, ring slots per wave, 16-row blocks, 16-channel blocks); LDS = waves x slots x
// (MB + NB) x 2 KB.  16 x 16 tiles for batch 1-2, 32 x 32 / 64 x 32 / 64 x 64 for batch ~8
const SknTile kSknTiles[] = {
    KV_SKN(4, 4, 1, 1), KV_SKN(8, 4, 1, 1), KV_SKN(16, 2, 1, 1), KV_SKN(8, 2, 2, 1),
    KV_SKN(8, 2, 2, 2), KV_SKN(4, 4, 2, 2), KV_SKN(4, 2, 4, 2), KV_SKN(4, 2, 2, 4),
    KV_SKN(4, 2, 4, 4),
};
#undef KV_SKN

}  // namespace

int skinny_num_tiles() { return (int)(sizeof(kSknTiles) / sizeof(kSknTiles[0])); }

int skinny_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= skinny_num_tiles()) return -6;
  if (p->n_t || p->in_u8 || p->pair_1x1) return -8;
  if (p->mode != 0 && p->mode != 1 && p->mode != 4) return -8;
  if (p->K % 64 || p->Cout % 4 || p->Kpad % 64) return -8;
  if (p->mode == 0 && (p->Cin % 64 || p->K != p->KH * p->KW * p->Cin)) return -8;
  if (p->mode == 1 && (p->Cin % 64 || p->K != p->Cin)) return -8;
  if (p->mode == 4 && (p->K1 % 64 || (p->K - p->K1) % 64 || p->ldx2 % 8 || p->K - p->K1 > p->ldx2 ||
                       p->up2 || p->x2_coff))
    return -8;
  if (p->M >= (1 << 16)) return -8;  // FastDiv is exact below 2^16 (edge batches only)
  const SknTile& e = kSknTiles[tile];
  const int mt = (p->M + 16 * e.mb - 1) / (16 * e.mb);
  const int nt = (p->Cout + 16 * e.nb - 1) / (16 * e.nb);
  const int ntiles = mt * nt;
  if (ntiles <= 0) return 0;
  if (p->K / 64 >= 4096 || p->Cin / 64 > 64 || p->KW > 64 || p->KW < 1) return -8;  // skn_qdiv range
  const float inv_cpt = 1.0f / (float)(p->mode == 0 ? p->Cin / 64 : 1);
  const float inv_kw = 1.0f / (float)p->KW;
  const FastDiv hw = make_fastdiv(p->Ho * p->Wo);
  const FastDiv wo = make_fastdiv(p->Wo);
  const SknFn fn = e.fn[p->mode == 0 ? 0 : p->mode == 1 ? 1 : 2];
  const int lds = std::max(e.waves * e.ring * (e.mb + e.nb) * 2048, e.waves * e.mb * e.nb * 1024);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(fn, dim3((unsigned)ntiles), dim3(e.waves * 64), (unsigned)lds, stream, *p, mt,
                     ntiles, inv_cpt, inv_kw, hw, wo);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
