// K2+K5 fused: ResNet stem (7x7/2 conv as a stride-1 4x4 conv over the space-to-depth
// image, BN folded, ReLU) + 3x3/2 max pool, in one kernel (gfx950).
//
// Unfused, the stem writes a [N,112,112,64] bf16 tensor (411 MB at batch 256) that the
// max pool reads back to write a 4x smaller one: 280 + 119 us per batch-256 step
// (profiles/r1_v4_resnet50_b256_forward.md), the stem itself at 0.37 PF/s because its
// implicit GEMM (N = 64, K = 256) re-fetches each input pixel for all 16 taps.
//
// Persistent: one workgroup per CU walks bands of RB = 2 pooled output rows (image-major):
//  * the 64 x 256 weight matrix is loaded into VGPRs ONCE per workgroup (32 fragments
//    per lane), the next band's input patch is prefetched into registers while this
//    band computes (a one-band-per-workgroup first version was latency-bound: 17 us
//    per band, slower than the unfused pair);
//  * the s2d input rows the band needs (8 rows of 16-ch pixels) are loaded ONCE into
//    LDS (zero padding included); every tap's A fragment is then a shifted
//    ds_read_b128 of that patch -- no re-fetch from L2 per tap;
//  * the 2*RB+1 = 5 stem rows the pool windows touch are computed with
//    v_mfma_f32_32x32x16_bf16 (D = W * A^T as in conv_glds.hip), the accumulators
//    seeded with the folded-BN bias;
//  * ReLU, bf16, into an LDS stem tile; then the 3x3/2 pool reads the tile and writes
//    the pooled [RB, W/2, 64] band with 16-B stores.
// A band's pool windows touch 5 stem rows, the first shared with the previous band.  Each
// workgroup walks a contiguous range of bands and keeps the stem tile as a 5-row ring, so
// the shared row is computed once (only the first band of a range recomputes it): the
// 112x112x64 intermediate is never written to HBM, and no conv row is computed twice.
//
// VALU diet (PMC of the previous version, profiles/r1_v7_stem_pmc.md: 17 VALU per MFMA,
// i.e. VALU-issue-bound at ~2x the MFMA time):
//  * patch pixels at a fixed 48-B pitch (16 ch + 16 B pad) and a fixed row pitch of
//    kPW = 128 pixels: 16 consecutive pixels' 16-B reads hit banks 12p mod 64, all 64
//    exactly once (conflict-free with a LINEAR layout), so a tap's fragment address is
//    the block base plus a compile-time constant = the ds_read immediate offset;
//  * the bias seeds the accumulators (no per-element add) and out-of-image stem rows
//    are never read (the pool clamps its padding taps in-image) instead of being zeroed;
//  * the pool runs packed 16-bit unsigned max (v_pk_max_u16) on the bf16 bit patterns:
//    post-ReLU values are >= 0 and non-negative IEEE values order like their bits;
//  * 512 threads (2 waves per SIMD): one wave's LDS reads / epilogue / pool overlap the
//    other's MFMAs (256 threads: 691 us -> 558 us at batch 640 on its own).
#include <stdlib.h>

#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace kvedge {
namespace {

constexpr int kCo = 64;        // stem output channels
constexpr int kCin = 16;       // s2d channels
constexpr int kTaps = 16;      // 4x4
constexpr int kK = kTaps * kCin;
constexpr int kRB = 2;         // pooled rows per workgroup
constexpr int kSR = 2 * kRB + 1;  // stem rows per band
constexpr int kPR = kSR + 3;      // patch (input) rows per band
constexpr int kTS = kCo + 8;      // stem-tile pixel stride (elements)
constexpr int kPW = 128;          // patch row pitch in pixels (W + 3 <= kPW)
constexpr int kPB = 48;           // patch bytes per pixel: 16 ch (32 B) + 16 B pad

__device__ __forceinline__ int patch_off(int p, int h) { return p * kPB + h * 16; }

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk_max_u16(unsigned a, unsigned b) {
  const u16x2 r = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                            __builtin_bit_cast(u16x2, b));
  return __builtin_bit_cast(unsigned, r);
}

// frames-in mode: per-channel normalisation of raw bytes, v = byte * a[c] + b[c]
struct StemNorm {
  float a[3], b[3];
};

// U8 = false: x is the bf16 s2d image [N,H,W,16] (ops.preprocess(s2d=True)).
// U8 = true : x is the raw uint8 frame [N,2H,2W,3]; the patch fetch reads 12 contiguous
//             bytes (two s2d pixels of one source row, 4-B aligned: one buffer_load_dwordx3)
//             and normalises + space-to-depths them in registers at commit time, so the
//             preprocess kernel and its 32 B/px bf16 image disappear from the step.
template <int NT, bool U8>  // threads per workgroup: 256 (1 wave/SIMD) or 512 (2 waves/SIMD)
__global__ __launch_bounds__(NT, 1) void stem_pool_kernel(
    const void* __restrict__ xv, const bf16* __restrict__ w, const float* __restrict__ bias,
    bf16* __restrict__ y, int N, int H, int W, int Hp, int Wp, int ldy, int y_coff,
    StemNorm nrm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int kPatchBytes = kPR * kPW * kPB;
  unsigned char* patch = lds;                                // kPR x kPW pixels
  bf16* tile = reinterpret_cast<bf16*>(lds + kPatchBytes);    // kSR*W px, stride kTS

  const int nbands = (Hp + kRB - 1) / kRB;
  const int total = N * nbands;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  constexpr int kNW = NT / 64;

  // ---- weights -> VGPRs, once: fragment (cb, t) rows n = cb*32 + fr, k = t*16 + fh*8 ..
  bf16x8 wreg[2][kTaps];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
      wreg[cb][t] = *reinterpret_cast<const bf16x8*>(w + (cb * 32 + fr) * kK + t * 16 + fh * 8);
  // bias for this lane's accumulator channels n = cb*32 + g*8 + fh*4 + j
  float4 bv[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      bv[cb][g] = *reinterpret_cast<const float4*>(bias + cb * 32 + g * 8 + fh * 4);

  // ---- patch prefetch: 16-B chunks q = tid + NT*i of a band's (kPR x kPW) patch.  Every
  // chunk is loaded: columns past the image and out-of-image rows read zeros through the
  // buffer range check (no branch; no zero-init of `pre`: a v_mov into a register whose
  // last writer was a VMEM load made hipcc wait vmcnt(0) at the top of every band)
  constexpr int kChunks = kPR * kPW * 2;
  constexpr int kPre = kChunks / NT;
  static_assert(kChunks % NT == 0, "patch chunks per thread");
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
  constexpr int kPreU = U8 ? kPre / 2 : 1;
  uint4 pre[U8 ? 1 : kPre];
  u32x3 preu[kPreU];  // U8: 12 raw bytes = s2d pixels (p, p+1), one source row h
  unsigned okm = 0;   // U8: bit i = pair i inside the image (padding must be 0, not -mean)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(xv), (short)0, U8 ? N * H * W * 12 : N * H * W * kCin * 2, 0x00020000);
  auto fetch = [&](int item) __attribute__((always_inline)) {
    const int n = item / nbands, band = item - n * nbands;
    const int iy0 = 2 * band * kRB - 3;
    const bool live = item < total;
    if constexpr (U8) {
      okm = 0;
#pragma unroll
      for (int i = 0; i < kPreU; ++i) {
        const int q = tid + NT * i;          // pair index: (pixel pair, source row h)
        const int p = (q >> 1) * 2, h = q & 1;
        const int pr = p / kPW, pc = p % kPW;
        const int iy = iy0 + pr, ix = pc - 2;  // ix even, W even: both pixels in or out
        const bool ok = live && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const int off = ok ? ((n * 2 * H + 2 * iy + h) * 2 * W + 2 * ix) * 3 : 0x7ffffff0;
        preu[i] = __builtin_amdgcn_raw_buffer_load_b96(rx, off, 0, 0);
        okm |= ok ? 1u << i : 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kPre; ++i) {
        const int q = tid + NT * i;
        const int p = q >> 1, h = q & 1;
        const int pr = p / kPW, pc = p % kPW;
        const int iy = iy0 + pr, ix = pc - 2;
        const bool ok = live && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const int off = ok ? (((n * H + iy) * W + ix) * kCin + h * 8) * 2 : 0x7ffffff0;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        pre[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  // U8: 6 bytes (2 source pixels x rgb) -> one 16-B s2d chunk [r g b 0 r g b 0] in bf16
  auto norm_chunk = [&](unsigned lo, unsigned hi, int sh, bool ok) __attribute__((always_inline)) {
    // bytes sh..sh+5 of the 8-byte word (lo | hi << 32), sh in {0, 2}
    const unsigned long long v = ((unsigned long long)hi << 32 | lo) >> (8 * sh);
    float f[6];
#pragma unroll
    for (int j = 0; j < 6; ++j)
      f[j] = ok ? (float)((unsigned)(v >> (8 * j)) & 0xffu) * nrm.a[j % 3] + nrm.b[j % 3] : 0.f;
    bf16x8 o;
    o[0] = f2bf(f[0]); o[1] = f2bf(f[1]); o[2] = f2bf(f[2]); o[3] = f2bf(0.f);
    o[4] = f2bf(f[3]); o[5] = f2bf(f[4]); o[6] = f2bf(f[5]); o[7] = f2bf(0.f);
    return __builtin_bit_cast(uint4, o);
  };
  auto commit = [&]() __attribute__((always_inline)) {
    if constexpr (U8) {
#pragma unroll
      for (int i = 0; i < kPreU; ++i) {
        const int q = tid + NT * i;
        const int p = (q >> 1) * 2, h = q & 1;
        const bool ok = (okm >> i) & 1u;
        *reinterpret_cast<uint4*>(patch + patch_off(p, h)) = norm_chunk(preu[i][0], preu[i][1], 0, ok);
        *reinterpret_cast<uint4*>(patch + patch_off(p + 1, h)) = norm_chunk(preu[i][1], preu[i][2], 2, ok);
      }
    } else {
#pragma unroll
      for (int i = 0; i < kPre; ++i) {
        const int q = tid + NT * i;
        *reinterpret_cast<uint4*>(patch + patch_off(q >> 1, q & 1)) = pre[i];
      }
    }
  };

  const FastDiv fW = make_fastdiv(W);  // once per thread; j / W per row block below
  // each workgroup walks a CONTIGUOUS range of bands, so consecutive bands of one image
  // run back to back here: a band's first stem row (y0) is the previous band's last one,
  // still in the stem tile, and only 4 of the 5 rows are computed (the tile's rows are a
  // ring: stem row y lives in slot (y + kSR) % kSR).  Band 0's row -1 is padding the pool
  // never reads, so it is never computed either.  20 % fewer MFMAs than recomputing the shared row;
  // measured time barely moves (376-407 -> 381 us at batch 640): the kernel is bound by its
  // fetch / commit / pool phases, not the MFMAs (profiles/r2_v12_stem_ring.md)
  const int per = (total + gridDim.x - 1) / gridDim.x;
  const int item0 = blockIdx.x * per, item1 = min(item0 + per, total);
  int item = item0;
  fetch(item);
  commit();
  __syncthreads();
  for (; item < item1; ++item) {
    const int n = item / nbands, band = item - n * nbands;
    const int P0 = band * kRB;  // first pooled row
    const int y0 = 2 * P0 - 1;  // first stem row (may be -1)
    fetch(item + 1 < item1 ? item + 1 : total);  // next band's patch, during these MFMAs
    const int skip = (band == 0 || item > item0) ? 1 : 0;  // row y0 padding or already in the tile

    // ---- stem rows of the band: 32-pixel row blocks round-robin over the kNW waves
    const int npix = (kSR - skip) * W;
    const int nrb = (npix + 31) / 32;
    for (int rb = wv; rb < nrb; rb += kNW) {
      const int j = min(rb * 32 + fr, npix - 1) + skip * W;  // clamp: rows past npix discarded
      const int yl = fdiv(j, fW), xc = j - yl * W;
      const int slot = (y0 + yl + kSR) % kSR;
      const unsigned char* pa = patch + patch_off(yl * kPW + xc, fh);
      floatx16 acc[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          acc[cb][4 * g + 0] = bv[cb][g].x;
          acc[cb][4 * g + 1] = bv[cb][g].y;
          acc[cb][4 * g + 2] = bv[cb][g].z;
          acc[cb][4 * g + 3] = bv[cb][g].w;
        }
      bf16x8 af[2];
      auto load = [&](int buf, int t) __attribute__((always_inline)) {
        af[buf] = *reinterpret_cast<const bf16x8*>(pa + ((t >> 2) * kPW + (t & 3)) * kPB);
      };
      load(0, 0);
#pragma unroll
      for (int t = 0; t < kTaps; ++t) {
        if (t + 1 < kTaps) load((t + 1) & 1, t + 1);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[0][t], af[t & 1], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[1][t], af[t & 1], acc[1], 0, 0, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int t = 0; t < kTaps; ++t) {
        if (t + 1 < kTaps) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      // ReLU -> bf16 stem tile.  Stem rows outside the image (above the first band, below
      // an odd-H image) are written but never read: the pool clamps padding taps in-image.
      if (rb * 32 + fr < npix) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            bf16x4 o;
            o[0] = f2bf(fmaxf(acc[cb][4 * g + 0], 0.f));
            o[1] = f2bf(fmaxf(acc[cb][4 * g + 1], 0.f));
            o[2] = f2bf(fmaxf(acc[cb][4 * g + 2], 0.f));
            o[3] = f2bf(fmaxf(acc[cb][4 * g + 3], 0.f));
            *reinterpret_cast<bf16x4*>(tile + (slot * W + xc) * kTS + cb * 32 + g * 8 + fh * 4) = o;
          }
      }
    }
    __syncthreads();  // stem tile complete; patch no longer read
    // next band's patch BEFORE the pool's stores (vmcnt counts stores on gfx9: a commit
    // after them waited for this band's stores to land)
    commit();

    // ---- 3x3/2 max pool (pad 1) of the band -> global, 16 B per thread-iteration.  Window
    // taps outside the image are clamped onto the nearest in-image tap of the SAME window
    // (x -1 -> 0, x W -> W-1, row -1 -> 0, row H -> H-1; the centre tap 2P / 2px is always
    // inside): a duplicate never changes a max, so the nine tile reads issue back to back
    // with no divergent branch.  The branchy form (skip padding taps) waited on each read in
    // turn: 9 serialised LDS round trips per output, ~1/3 of the kernel's time
    // (profiles/r2_v15_stem_pool_pmc.md)
#pragma unroll
    for (int pr = 0; pr < kRB; ++pr) {
      const int P = P0 + pr;
      if (P >= Hp) break;
      bf16* yrow = y + (long long)(n * Hp + P) * Wp * ldy + y_coff;
      int rbase[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
        rbase[dy] = (min(max(2 * P - 1 + dy, 0), H - 1) % kSR) * W;  // ring slot of the row
      for (int q = tid; q < Wp * (kCo / 8); q += NT) {
        const int px = q >> 3, c8 = q & 7;
        const int xs[3] = {max(2 * px - 1, 0), 2 * px, min(2 * px + 1, W - 1)};
        uint4 v[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            v[dy * 3 + dx] =
                *reinterpret_cast<const uint4*>(tile + (rbase[dy] + xs[dx]) * kTS + c8 * 8);
        uint4 m = v[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) {
          m.x = pk_max_u16(m.x, v[k].x);
          m.y = pk_max_u16(m.y, v[k].y);
          m.z = pk_max_u16(m.z, v[k].z);
          m.w = pk_max_u16(m.w, v[k].w);
        }
        *reinterpret_cast<uint4*>(yrow + px * ldy + c8 * 8) = m;
      }
    }
    __syncthreads();  // tile free, patch ready
  }
}

}  // namespace
}  // namespace kvedge

using namespace kvedge;

extern "C" int kv_stem_pool_lds_bytes(int W) { return kPR * kPW * kPB + kSR * W * kTS * 2; }

namespace {
template <bool U8>
int stem_launch(const void* x, const void* w, const float* bias, void* y, int N, int H, int W,
                int ldy, int y_coff, const StemNorm& nrm, hipStream_t s) {
  if (N <= 0) return 0;
  if (H <= 0 || W <= 0 || ldy % 8 || y_coff % 8 || ldy < y_coff + kCo || !bias) return -1;
  const int lds = kv_stem_pool_lds_bytes(W);
  if (lds > 160 * 1024 || W + 3 > kPW) return -2;                // patch row pitch: W <= 125
  if ((long long)N * H * W * 16 * 2 >= 0x7ffffff0LL) return -4;   // buffer range (2 GiB)
  if (U8 && W % 2) return -5;                                     // pixel-pair fetch
  const int Hp = (H - 1) / 2 + 1, Wp = (W - 1) / 2 + 1;  // 3x3 / 2, pad 1
  const long long items = (long long)N * ((Hp + kRB - 1) / kRB);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long long g = items < ncu ? items : ncu;  // persistent: one workgroup per CU
  // KVEDGE_STEM_THREADS=256|512 (probe knob; default 512: two waves per SIMD)
  static const int nt = [] {
    const char* e = getenv("KVEDGE_STEM_THREADS");
    return (e && atoi(e) == 256) ? 256 : 512;
  }();
  const void* fn = nt == 256 ? reinterpret_cast<const void*>(stem_pool_kernel<256, U8>)
                             : reinterpret_cast<const void*>(stem_pool_kernel<512, U8>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -3;
  if (nt == 256)
    hipLaunchKernelGGL((stem_pool_kernel<256, U8>), dim3((unsigned)g), dim3(256), (unsigned)lds, s,
                       x, (const bf16*)w, bias, (bf16*)y, N, H, W, Hp, Wp, ldy, y_coff, nrm);
  else
    hipLaunchKernelGGL((stem_pool_kernel<512, U8>), dim3((unsigned)g), dim3(512), (unsigned)lds, s,
                       x, (const bf16*)w, bias, (bf16*)y, N, H, W, Hp, Wp, ldy, y_coff, nrm);
  return hipGetLastError() == hipSuccess ? 0 : -100;
}
}  // namespace

extern "C" int kv_stem_pool(const void* x, const void* w, const float* bias, void* y, int N, int H,
                            int W, int ldy, int y_coff, hipStream_t s) {
  return stem_launch<false>(x, w, bias, y, N, H, W, ldy, y_coff, StemNorm{}, s);
}

// frames: uint8 [N, H0, W0, 3] (H0, W0 even); v = (byte/255 - mean) * inv_std per channel
extern "C" int kv_stem_pool_frames(const void* frames, const void* w, const float* bias, void* y,
                                   int N, int H0, int W0, const float* mean3,
                                   const float* inv_std3, int ldy, int y_coff, hipStream_t s) {
  if (H0 % 2 || W0 % 2) return -5;
  StemNorm nrm;
  for (int c = 0; c < 3; ++c) {
    nrm.a[c] = inv_std3[c] / 255.f;
    nrm.b[c] = -mean3[c] * inv_std3[c];
  }
  return stem_launch<true>(frames, w, bias, y, N, H0 / 2, W0 / 2, ldy, y_coff, nrm, s);
}
