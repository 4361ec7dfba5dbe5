// K2 v4: direct 3x3 convolution (stride 1 or 2, pad 1) for narrow channel counts,
// NHWC bf16, fp32 accumulate (gfx950).
//
// Why a fourth conv family.  For 3x3 convs with few channels the implicit-GEMM families
// re-stage the SAME input pixels once per tap (9x the A bytes through L2 -> LDS) while
// the narrow N gives each staged byte few MACs:
//   ResNet-50 stage 1, 64 -> 64 @56x56: 285 us per conv at batch 640 (0.52 PF/s) on the
//     best v1/v2 tile against a ~0.1 ms HBM floor;
//   YOLOv8n 16/32-channel convs @160x160 and @80x80: 4-6x their HBM floor
//     (profiles/r1_v6_yolov8n_b256_forward.md, conv_glds<128,32,4,1,3,2>).
// Here every input pixel is staged ONCE per band and all taps read it in place:
//
//  * Persistent, one 512-thread workgroup per CU (2 waves per SIMD) walking bands of kR
//    output rows of one image.  The band's input patch (halo rows/cols and zero padding
//    included, the padding via the buffer range check) is prefetched into VGPRs during
//    the previous band's MFMAs and committed to LDS between bands.
//  * Each wave owns one 32-channel block of Cout and holds that block's packed weights
//    for the whole kernel (9*CIN/16 MFMA fragments: 36 VGPRs at CIN 16 .. 144 at CIN 64).
//    Weights are read from HBM once per CU, never re-staged.
//  * A 32-pixel output block is 9*CIN/16 v_mfma_f32_32x32x16_bf16, each fed by one
//    ds_read_b128 of the patch.  Patch pixels sit at a pitch of CIN*2 + 16 bytes (48, 80,
//    144 B): 16 consecutive pixels' 16-B reads then hit all 64 banks exactly once, so the
//    LINEAR layout is conflict-free.  The three tap-row base pointers are formed once per
//    block; every tap/k-step offset is then a compile-time constant (the ds_read
//    immediate): no VALU per MFMA.
//  * Accumulators are seeded with the folded-BN bias; the epilogue is act + cvt into an
//    LDS output tile; the store pass adds the residual (YOLO Bottleneck: x + SiLU(conv))
//    and writes full 16-B channel chunks, with channel-slice (ldy / y_coff) support.
//  * Bands are dealt XCD-aware: concurrently running neighbour bands of one image sit on
//    one XCD, so their shared halo rows come from one L2.
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace kvedge {
namespace {

constexpr int kNT = 512;
constexpr int kOOB = 0x7ffffff0;
constexpr int kLds = 160 * 1024;
constexpr int kBiasBytes = 4 * 128;  // bias slot at the top of the LDS allocation

// s_waitcnt vmcnt(k) for the largest k <= n in {0, 4, ..., 60}: at most n of the wave's
// youngest vector-memory ops stay outstanding (rounding down only waits for more).  n must
// be wave-uniform (an SGPR): the cascade is scalar branches around immediates.
template <int K>
__device__ __forceinline__ void direct_wait_vm_le_(int n) {
  if constexpr (K == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= K) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
    else direct_wait_vm_le_<K - 4>(n);
  }
}
__device__ __forceinline__ void direct_wait_vm_le(int n) { direct_wait_vm_le_<60>(n); }

template <int CIN, int KK>
struct DirectCfg {
  static constexpr int PB = CIN * 2 + 16;         // patch bytes per pixel
  static constexpr int CPP = CIN / 8;             // 16-B chunks per pixel
  static constexpr int KPT = CIN / 16;            // 16-wide k-steps per tap
  static constexpr int KS = KK * KK * KPT;        // k-steps per output block
  // prefetch uint4 per thread (VGPR budget: CIN 80 holds 180 weight VGPRs)
  static constexpr int PRE = CIN >= 80 ? 6 : CIN >= 64 ? 7 : 10;
  static constexpr int MAX_PATCH = PRE * kNT * 16;
};

// KK = 3: 3x3, pad 1, stride S.  KK = 2: the space-to-depth form of a stride-2 3x3 stem
// (DeployedConv.stem_s2d): 2x2, stride 1, top/left pad 1, bottom/right pad 0.
// U8: x is uint8 RGB frames [N, 2H, 2W, 3]; the s2d patch (CIN = 16, channel
// (dy*2+dx)*4 + c, channel 3 zero) is built on the fly from raw bytes (exact in bf16; the
// 1/255 scale is folded into the weights), fusing the preprocess pass away.
#ifndef KV_DIRECT_PD
#define KV_DIRECT_PD 8
#endif
constexpr int KPD = KV_DIRECT_PD;

// bytes of one patch buffer: the DMA form rounds up to whole 1-KB DMA instructions (the
// last one may run past the patch) and keeps two buffers
__host__ __device__ constexpr int direct_patch_alloc(int patch_bytes, bool dma) {
  return dma ? (patch_bytes + 1023) / 1024 * 1024 : (patch_bytes + 15) / 16 * 16;
}  // LDS fragment reads in flight ahead of the MFMA

// DMA: the next band's patch goes global -> LDS with buffer_load ... lds into a second
// patch buffer (no VGPR staging, so no PRE cap on the band height: the CIN = 80 form holds
// 180 weight VGPRs and had room for a single 80-pixel output row per band otherwise).
// Lane-linear DMA slots of 16 B; slot q = (pixel q / SL, chunk q % SL) with SL = PB / 16,
// the pitch-padding chunk (q % SL == CPP) gets an out-of-range offset (zero fill).
// C2 > 0: fused 1x1 pair (YOLO Detect branch: 3x3 + SiLU, then a 1x1 with bias and no
// activation, C2 output channels).  The band's 3x3 output t stays in the LDS output tile
// (bf16, as the unfused layer would have stored it) and the 1x1 runs on it from there:
// z = t . W2^T + b2 goes to p.z [M][ldz] at z_coff and t never reaches HBM -- one launch and
// one tensor round trip less per Detect branch.  W2 [C2][COUT] and b2 sit in LDS.
// DE (direct epilogue, v10 tiles): each 32-pixel block's accumulators go straight to HBM (8-B
// buffer stores, out-of-range lanes dropped by the descriptor) instead of through the LDS
// output tile and a store pass behind a second barrier.  The band's stores then overlap the
// next blocks' MFMAs, the output tile's LDS goes to taller bands (less halo re-staging), and
// a band ends with ONE barrier after a counted vmcnt that waits for the next patch's DMAs
// only -- never for this band's stores (vmcnt retires in issue order, the DMAs are older).
// The plain-tile form spent ~64 % of wave cycles waiting at 31 % MFMA busy on the Detect P3
// stem (profiles/r3_v10_yolo_detect_p3_direct_tiles_b192.txt): MFMA phase, store pass and
// patch wait ran back to back on the only workgroup of the CU.
template <int CIN, int COUT, int S, int KK, int ACT, bool RES, bool U8 = false, bool DMA = false,
          bool PAIRS = false, int OCC = 1, int NT = kNT, int C2 = 0, bool DE = false,
          bool SB = false>
// SB (single patch buffer, DE forms at NT = 256 and two workgroups per CU): each band DMAs
// its own patch, waits, computes.  No prefetch within a workgroup; the CU's other workgroup
// runs its MFMA phase meanwhile, so the two band pipelines are not in lockstep (one
// workgroup of 8 waves syncs every wave of the CU at each band end).
// OCC = workgroups per CU the launch plans for (1 or 2); the second launch-bounds argument
// is HIP's minimum waves per SIMD (512 threads = 2 per SIMD per workgroup).  The narrow
// (16/32-channel) layers are latency-bound at one workgroup per CU -- one band in flight,
// 55-67 % of wave cycles waiting (profiles/r2_v5_yolov8n_b256_pmc.md) -- so their OCC = 2
// forms take shorter bands (LDS <= 80 KB) and <= 128 VGPRs, and two independent band
// pipelines share every CU.  Only the DMA forms fit 128 VGPRs without spilling.
// NT = 256 (4 waves, one workgroup per CU, one wave per SIMD): the whole 512-entry register
// file per lane, for weight blocks that do not fit 256 (CIN = 128: 288 weight VGPRs)
__global__ __launch_bounds__(NT, (NT / 256) * OCC) void conv3x3_direct_kernel(const KvConvParams p, int kR,
                                                                int PW, int patch_rows,
                                                                FastDiv fPW, FastDiv fWo,
                                                                int diag) {
  static_assert(!U8 || (CIN == 16 && KK == 2 && S == 1), "frames-in form: the 2x2 s2d stem");
  static_assert(!PAIRS || U8, "paired raw-row loads: frames-in form only");
  // KK = 1: a 1x1 conv through the same band machinery (pad 0): YOLO's narrow C2f / Detect
  // 1x1 convs at 160^2 / 80^2 are pure streaming, and the GEMM tiles' per-tile epilogue
  // overhead (K = 32..192, one or three K steps per tile) held them at 2.4-3.5 TB/s
  static_assert(KK != 1 || S == 1, "1x1 form: stride 1");
  constexpr int PADK = KK == 1 ? 0 : 1;
  using C = DirectCfg<CIN, KK>;
  constexpr int NCB = (COUT + 31) / 32;  // 32-channel blocks
  static_assert(NCB >= 1 && NCB <= 4 && NCB <= NT / 64, "channel blocks");
  // pixel-block phases; with NCB = 3 (YOLO's 80-channel Detect cls branch) waves 6 and 7
  // sit out the MFMA phase and only help with the patch fetch and the store pass
  constexpr int NPH = (NT / 64) / NCB;
  constexpr int OS = COUT + 8;           // output tile pixel stride (elements)
  static_assert(C2 == 0 || (!RES && !U8 && KK == 3 && COUT % 16 == 0), "pair form");
  constexpr int NCB2 = (C2 + 31) / 32;   // pair: 32-channel blocks of the 1x1's output
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  static_assert(!(DMA && U8), "DMA patch fetch: bf16 NHWC inputs only");
  static_assert(!DE || (DMA && C2 == 0 && !U8 && !(RES && SB)), "direct epilogue: plain DMA forms");
  static_assert(!SB || DE, "single patch buffer: direct-epilogue forms");
  static_assert(!DE || COUT % 16 == 0, "direct epilogue: 16-channel store pairs");
  const int psz = direct_patch_alloc(patch_rows * PW * C::PB, DMA);
  unsigned char* patch = lds;
  bf16* otile = reinterpret_cast<bf16*>(lds + (DMA && !SB ? 2 * psz : psz));

  const int H = p.H, W = p.W, Ho = p.Ho, Wo = p.Wo;
  const int nbands = (Ho + kR - 1) / kR;
  const int total = p.N * nbands;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loops
  const int fr = lane & 31, fh = lane >> 5;
  const int cb = wv % NCB, ph = wv / NCB;

  // ---- this wave's weight block -> VGPRs, once (rows past Cout are zero)
  const bf16* wp = reinterpret_cast<const bf16*>(p.w);
  const int wrow = cb * 32 + fr;
  bf16x8 wreg[C::KS];
#pragma unroll
  for (int kk = 0; kk < C::KS; ++kk) {
    bf16x8 v = {};
    if (wrow < COUT) v = *reinterpret_cast<const bf16x8*>(wp + wrow * p.Kpad + kk * 16 + fh * 8);
    wreg[kk] = v;
  }
  // bias staged once in LDS; the DMA forms (no prefetch registers) then hold their 16 bias
  // values in VGPRs for the whole kernel (the VGPR-prefetch forms sit at the 256 cap)
  float* lbias = reinterpret_cast<float*>(
      reinterpret_cast<unsigned char*>(otile) + (DE ? 0 : ((kR * p.Wo * OS * 2 + 15) & ~15)));
  if (tid < NCB * 32) lbias[tid] = (p.bias && tid < COUT) ? p.bias[tid] : 0.f;
  constexpr bool BREG = DMA && OCC == 1;  // bias in VGPRs (OCC = 2 forms: 128-VGPR cap)
  floatx16 breg = {};
  if constexpr (BREG) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = cb * 32 + g * 8 + fh * 4 + e;
        breg[4 * g + e] = (p.bias && c < COUT) ? p.bias[c] : 0.f;
      }
  }
  // pair: b2 [NCB2 * 32] then W2 [C2][OS] above the bias slot (the MFMA rows past C2 read
  // row C2 - 1 again and are discarded: with 96 rows the C2 = 80 pair missed a 2-row band by
  // 1.6 KB of LDS); the W2 row pitch equals the output tile's (conflict-free ds_read_b128)
  float* lbias2 = lbias + 128;
  bf16* w2s = reinterpret_cast<bf16*>(lbias2 + 128);
  if constexpr (C2 > 0) {
    static_assert(NCB2 * 32 <= 128 && NCB * 32 <= 128, "pair bias slots");
    if (tid < NCB2 * 32) lbias2[tid] = (p.bias_t && tid < C2) ? p.bias_t[tid] : 0.f;
    const bf16* w2 = reinterpret_cast<const bf16*>(p.w_t);
    for (int q = tid; q < C2 * (COUT / 8); q += NT) {
      const int r = q / (COUT / 8), c = (q - r * (COUT / 8)) * 8;
      *reinterpret_cast<bf16x8*>(w2s + r * OS + c) =
          *reinterpret_cast<const bf16x8*>(w2 + (size_t)r * COUT + c);
    }
  }

  // ---- band patch prefetch: 16-B chunk q -> patch pixel q / CPP (row-major, pitch PW)
  const int nchunks = patch_rows * PW * C::CPP;
  uint4 pre[C::PRE];
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, U8 ? p.N * H * W * 12 : p.N * H * W * p.ldx * 2,
      0x00020000);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  // Stride 2: patch row positions hold the EVEN input columns first, then the odd ones
  // (column pc at pc / 2, or HALF + pc / 2).  Neighbouring output pixels then read
  // neighbouring positions for every tap, at a pitch of PB = 16 x odd bytes: a ds_read_b128
  // lane group's 16 reads hit 16 distinct 16-B bank slots.  In column order the pitch was
  // 2 x PB (an even number of slots): every MFMA operand read 2-way conflicted
  // (SQ_LDS_BANK_CONFLICT 17-33 M per stride-2 launch, profiles/r2_v2_yolov8n_b384_pmc.md).
  const int HALF = (PW + 1) >> 1;
  auto col_of = [&](int pos) __attribute__((always_inline)) {
    if constexpr (S == 2) return pos < HALF ? 2 * pos : 2 * (pos - HALF) + 1;
    return pos;
  };
  // chunk q -> (patch pixel pp, 16-B chunk c).  U8: q = (pr*2 + c)*PW + pc, so consecutive
  // lanes walk one raw frame row (coalesced 6-B groups); otherwise pixel-major.
  auto chunk_of = [&](int q, int& pp, int& c) __attribute__((always_inline)) {
    if constexpr (U8) {
      const int rc = fdiv(q, fPW), pc = q - rc * PW;
      c = rc & 1;
      pp = (rc >> 1) * PW + pc;
    } else {
      pp = q / C::CPP;
      c = q - pp * C::CPP;
    }
  };
  // U8 with even W: one 12-B buffer_load_dwordx3 = two neighbouring s2d pixels (ix even,
  // 4-B aligned) of one raw row; patch column 0 (the left padding, ix = -1) is zeroed once
  // and never fetched.  Item u -> (rc = u / NPR, pair k = u % NPR): patch row rc >> 1, raw
  // row parity rc & 1, patch columns 2k+1, 2k+2.  (Odd W: the 3 x 16-bit loads per chunk.)
  // (PAIRS is instantiated for even W only: direct_plan picks the form by W's parity)
  const int NPR = W >> 1;
  constexpr bool pairs = PAIRS;
  const FastDiv fNPR = make_fastdiv(NPR > 0 ? NPR : 1);
  static_assert(!U8 || C::PRE % 2 == 0, "pairs: two chunks per prefetch pair");
  // pairs: the RAW 12 bytes stay in registers until commit (after the band's MFMAs), so
  // the loads' latency hides under the MFMA phase; bit i of okp = pair i's row in range
  typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
  u32x3 raw[PAIRS ? C::PRE / 2 : 1];
  unsigned okp = 0;
  auto fetch = [&](int item) __attribute__((always_inline)) {
    const int n = item / nbands, band = item - n * nbands;
    const int iy0 = band * kR * S - PADK;
    const bool live = item < total;
    if constexpr (PAIRS) {
      {
        okp = 0;
        const int nitems = patch_rows * 2 * NPR;
#pragma unroll
        for (int i = 0; i < C::PRE / 2; ++i) {
          const int u = tid + NT * i;
          const int rc = fdiv(u, fNPR), k = u - rc * NPR;
          const int iy = iy0 + (rc >> 1), ix = 2 * k;
          const bool rowok = live && u < nitems && (unsigned)iy < (unsigned)H;
          const int off = rowok ? ((n * 2 * H + 2 * iy + (rc & 1)) * 2 * W + 2 * ix) * 3 : kOOB;
          raw[i] = __builtin_amdgcn_raw_buffer_load_b96(rx, off, 0, 0);
          okp |= rowok ? 1u << i : 0u;
        }
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < C::PRE; ++i) {
      const int q = tid + NT * i;
      int pp, c;
      chunk_of(q, pp, c);
      const int pr = fdiv(pp, fPW), pc = col_of(pp - pr * PW);
      const int iy = iy0 + pr, ix = pc - PADK;
      const bool ok = live && q < nchunks && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      if constexpr (U8) {
        // s2d chunk c of pixel (iy, ix) = raw row 2*iy + c, raw cols 2*ix, 2*ix + 1, RGB:
        // 6 bytes -> [r g b 0 r' g' b' 0] as bf16 (integers 0..255 are exact)
        const int off = ok ? ((n * 2 * H + 2 * iy + c) * 2 * W + 2 * ix) * 3 : kOOB;
        const unsigned a = __builtin_amdgcn_raw_buffer_load_b16(rx, off, 0, 0);
        const unsigned b = __builtin_amdgcn_raw_buffer_load_b16(rx, off + 2, 0, 0);
        const unsigned d = __builtin_amdgcn_raw_buffer_load_b16(rx, off + 4, 0, 0);
        auto bfb = [](unsigned byte) { return __float_as_uint((float)byte) >> 16; };
        pre[i] = make_uint4(bfb(a & 0xff) | (bfb(a >> 8) << 16), bfb(b & 0xff),
                            bfb(b >> 8) | (bfb(d & 0xff) << 16), bfb(d >> 8));
      } else {
        const int off = ok ? (((n * H + iy) * W + ix) * p.ldx + p.x_coff + c * 8) * 2 : kOOB;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        pre[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto commit = [&]() __attribute__((always_inline)) {
    if constexpr (PAIRS) {
      {
        const int nitems = patch_rows * 2 * NPR;
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < C::PRE / 2; ++i) {
          const int u = tid + NT * i;
          if (u >= nitems) continue;
          const int rc = fdiv(u, fNPR), k = u - rc * NPR;
          const int pp = (rc >> 1) * PW + 2 * k + 1;
          unsigned char* dst = patch + pp * C::PB + (rc & 1) * 16;
          // bytes 0-5: pixel ix (raw cols 2ix, 2ix+1), bytes 6-11: pixel ix+1 -> two s2d
          // chunks [r g b 0 r' g' b' 0] in bf16 (0..255 exact); out-of-image rows: zeros
          const u32x3 v = raw[i];
          auto bf = [](unsigned w, int b) { return __float_as_uint((float)((w >> (8 * b)) & 0xffu)) >> 16; };
          const bool ok = (okp >> i) & 1u;
          *reinterpret_cast<uint4*>(dst) =
              ok ? make_uint4(bf(v[0], 0) | (bf(v[0], 1) << 16), bf(v[0], 2),
                              bf(v[0], 3) | (bf(v[1], 0) << 16), bf(v[1], 1)) : z;
          *reinterpret_cast<uint4*>(dst + C::PB) =
              ok ? make_uint4(bf(v[1], 2) | (bf(v[1], 3) << 16), bf(v[2], 0),
                              bf(v[2], 1) | (bf(v[2], 2) << 16), bf(v[2], 3)) : z;
        }
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < C::PRE; ++i) {
      const int q = tid + NT * i;
      int pp, c;
      chunk_of(q, pp, c);
      if (q < nchunks) *reinterpret_cast<uint4*>(patch + pp * C::PB + c * 16) = pre[i];
    }
  };

  constexpr int SL = C::PB / 16;  // 16-B slots per patch pixel (CPP data + 1 padding)
  const int nslots = patch_rows * PW * SL;
  const kv_i32x4 rx4 = kv_rsrc4(p.x, U8 ? 0 : p.N * H * W * p.ldx * 2);
  // DMA forms without a residual split the waves by role: the first half issues every patch
  // DMA, the second half every output store.  On gfx9 vmcnt counts stores too, so a wave
  // that stored the band and then waited for its next-patch DMA (vmcnt(0)) also waited for
  // its stores to be acknowledged -- one HBM write latency per band on every CU.  Split, the
  // DMA waves have no stores outstanding and the store waves never wait on vmcnt.
  constexpr int NWV = NT / 64;
  constexpr bool SPLIT = DMA && !RES && NWV >= 4 && C2 == 0 && !DE;
  constexpr int NWD = SPLIT ? NWV / 2 : NWV;  // waves issuing the patch DMA
  auto dma_fetch = [&](int item, unsigned char* dst) __attribute__((always_inline)) {
    const int n = item / nbands, band = item - n * nbands;
    const int iy0 = band * kR * S - PADK;
    const bool live = item < total;
    if (SPLIT && wv >= NWD) return;
    for (int j = wv; j * 64 < nslots; j += NWD) {  // one 1-KB DMA per wave per j
      const int q = j * 64 + lane;
      const int pp = q / SL, c = q - pp * SL;
      const int pr = fdiv(pp, fPW), pc = col_of(pp - pr * PW);
      const int iy = iy0 + pr, ix = pc - PADK;
      const bool ok = live && q < nslots && c < C::CPP && (unsigned)iy < (unsigned)H &&
                      (unsigned)ix < (unsigned)W;
      const int off = ok ? (((n * H + iy) * W + ix) * p.ldx + p.x_coff + c * 8) * 2 : kOOB;
      // opaque to the compiler (common.h): the builtin made hipcc drain this prefetch with a
      // vmcnt(0) in front of the current band's fragment reads
      kv_lds_dma16(rx4, dst + j * 1024, off);
    }
  };

  bf16* __restrict__ Y = reinterpret_cast<bf16*>(p.y);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      p.y, (short)0, DE ? p.N * Ho * Wo * p.ldy * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
      C2 > 0 ? p.z : p.y, (short)0, C2 > 0 ? p.N * Ho * Wo * p.ldz * 2 : 0, 0x00020000);
  const bf16* __restrict__ R = reinterpret_cast<const bf16*>(p.res);
  const kv_i32x4 rr4 = kv_rsrc4(p.res, DE && RES ? p.N * Ho * Wo * p.ldr * 2 : 0);
  const int npix = kR * Wo;
  const int nblk = (npix + 31) / 32;
  const int rowb = PW * C::PB;
  int item = xcd_remap(blockIdx.x, gridDim.x);  // neighbour bands share an XCD
  int cur = 0;
  if constexpr (PAIRS) {
    // patch column 0 = left padding of every patch row, both parities: zero
      for (int q = tid; q < patch_rows * 2; q += NT)
        *reinterpret_cast<uint4*>(patch + (q >> 1) * PW * C::PB + (q & 1) * 16) =
            make_uint4(0u, 0u, 0u, 0u);
  }
  if constexpr (SB) {
    // per band, below
  } else if constexpr (DMA) {
    dma_fetch(item, patch);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    fetch(item);
    commit();
  }
  __syncthreads();
  for (; item < total; item += gridDim.x) {
    const int n = item / nbands, band = item - n * nbands;
    const int oy0 = band * kR;
    // next band: in flight during this band's MFMAs (DMA: into the other patch buffer,
    // last read in the previous band, before the barrier that ended it)
    if constexpr (SB) {
      dma_fetch(item, patch);  // this band's patch (the last band's readers passed the barrier)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else if constexpr (DMA) {
      // diag bit 1 (KVEDGE_DIRECT_DIAG, timing experiments only: wrong results): no prefetch
      if (!(DE && (diag & 2))) dma_fetch(item + gridDim.x, patch + (cur ^ 1) * psz);
    } else {
      fetch(item + gridDim.x);
    }
    const unsigned char* pbase = patch + cur * psz;
    // residual of THIS band, loaded now so its HBM latency hides under the MFMA phase
    // (a load in the store pass stalled every band: 69 % of wave cycles waiting on the
    // 16-channel YOLO bottleneck conv, profiles/r2_v2_yolov8n_b384_pmc.md)
    constexpr int OCH = COUT / 8;
    // VGPR budget: narrow forms only; the VGPR-prefetch form also holds the next patch
    constexpr int RPF = RES && !DE && CIN <= 32 ? (DMA ? 12 : CIN <= 16 ? 6 : 0) : 0;
    uint4 rpf[RPF > 0 ? RPF : 1];
    const bool rpre = RPF > 0 && npix * OCH <= RPF * NT;
    if constexpr (RPF > 0) {
      if (rpre) {
#pragma unroll
        for (int i = 0; i < RPF; ++i) {
          const int q = tid + NT * i;
          const int px = q / OCH, c = q - (q / OCH) * OCH;
          const int yl = fdiv(px, fWo), xc = px - yl * Wo;
          const int oy = oy0 + yl;
          rpf[i] = make_uint4(0u, 0u, 0u, 0u);
          if (q < npix * OCH && oy < Ho) {
            const long long m = (long long)(n * Ho + oy) * Wo + xc;
            rpf[i] = *reinterpret_cast<const uint4*>(R + m * p.ldr + p.r_coff + c * 8);
          }
        }
      }
    }

    for (int b = ph < NPH ? ph : nblk; b < nblk; b += NPH) {
      const int j = min(b * 32 + fr, npix - 1);  // clamp: pixels past npix are discarded
      const int yl = fdiv(j, fWo), xc = j - yl * Wo;
      // stride 2: tap column s of output column xc sits at position xc + s / 2 (even s) or
      // HALF + xc (s = 1)
      const unsigned char* pa0 = pbase + (yl * S * PW + xc * (S == 2 ? 1 : S)) * C::PB + fh * 16;
      const unsigned char* pa[KK];
      const unsigned char* po[KK];
#pragma unroll
      for (int r = 0; r < KK; ++r) {
        pa[r] = pa0 + r * rowb;
        po[r] = pa[r] + (S == 2 ? HALF * C::PB : 0);
      }
      // DE + residual: this block's residual, in the store layout (lane fr: channels
      // [q*16 + fh*8, +8) of pixel j), issued before the MFMA phase so its latency hides
      // there; asm loads (common.h), so hipcc can neither sink them nor wait early
      u32x4 rv[2] = {};
      if constexpr (DE && RES) {
        const int oy = oy0 + yl;
        const bool ok = b * 32 + fr < npix && oy < Ho;
        const int rp = (((n * Ho + oy) * Wo + xc) * p.ldr + p.r_coff + cb * 32) * 2;
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (cb * 32 + q * 16 < COUT) vm_load16(rv[q], rr4, ok ? rp + (q * 16 + fh * 8) * 2 : kOOB);
      }
      floatx16 acc;
      if constexpr (BREG) {
        acc = breg;
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = *reinterpret_cast<const float4*>(lbias + cb * 32 + g * 8 + fh * 4);
          acc[4 * g + 0] = bv.x;
          acc[4 * g + 1] = bv.y;
          acc[4 * g + 2] = bv.z;
          acc[4 * g + 3] = bv.w;
        }
        // the bias reads retire here, before the counted fragment ring below starts
        asm volatile("" : "+v"(acc));
      }
      // fragment ring (asm reads, common.h): the read for step kk + PD is issued before the
      // MFMA of step kk and each MFMA waits for its own read only -- PD reads stay in flight
      // behind the MFMA pipe.  Tap offsets are ds_read immediates off KK (stride 2: 2 KK) row
      // bases; no VALU per MFMA.
      constexpr int PD = NT == kNT ? (OCC == 2 ? 2 : CIN >= 80 ? 3 : DMA ? KPD : 4) : 6;
      bf16x8 af[PD + 1];
      unsigned ba[KK], bo[KK];
#pragma unroll
      for (int r = 0; r < KK; ++r) {
        ba[r] = lds_addr(pa[r]);
        bo[r] = lds_addr(po[r]);
      }
      auto rd = [&](auto kc) __attribute__((always_inline)) {
        constexpr int kk = decltype(kc)::value;
        constexpr int tap = kk / C::KPT, s4 = kk % C::KPT;
        constexpr int r = tap / KK, s = tap % KK;
        if constexpr (S == 2 && s == 1)
          lds_read16<s4 * 32>(af[kk % (PD + 1)], bo[r]);
        else
          lds_read16<(S == 2 ? s / 2 : s) * C::PB + s4 * 32>(af[kk % (PD + 1)], ba[r]);
      };
      static_range<0, (PD < C::KS ? PD : C::KS)>(rd);
      static_range<0, C::KS>([&](auto kc) __attribute__((always_inline)) {
        constexpr int kk = decltype(kc)::value;
        if constexpr (kk + PD < C::KS) rd(IC<kk + PD>{});
        constexpr int younger = (C::KS - 1 - kk) < PD ? (C::KS - 1 - kk) : PD;
        lds_wait<younger>(af[kk % (PD + 1)]);
        if (!(DE && (diag & 4)))  // diag bit 2: no MFMAs
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[kk], af[kk % (PD + 1)], acc, 0, 0, 0);
      });
      const int jr = b * 32 + fr;
      if constexpr (DE) {
        const int oy = oy0 + yl;
        const bool ok = jr < npix && oy < Ho;
        if (diag & 1) continue;  // diag bit 0: no stores (the band-end wait then under-waits)
        const int pix = (((n * Ho + oy) * Wo + xc) * p.ldy + p.y_coff + cb * 32) * 2;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        if (!RES && (diag & 8)) {
          // diag bit 3: the first DE store form, 4 x 8 B per lane (lanes fr / fr + 32: channels
          // [g*8, g*8+4) / [g*8+4, g*8+8)), 32 16-B segments per instruction
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (cb * 32 + g * 8 >= COUT) continue;
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(act_c<ACT>(acc[4 * g + e]));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ry,
                                                  ok ? pix + (g * 8 + fh * 4) * 2 : kOOB, 0, 0);
          }
          continue;
        }
        // Half-wave exchange, then 16 B per lane: for the group pair (2q, 2q+1) lane fr ends
        // with channels [16q, 16q+8) of pixel jr and lane fr + 32 with [16q+8, 16q+16).  One
        // store instruction writes 32 pixels x 32 contiguous bytes (the 4 x 8-B form: 32 x 16 B).
        // Same box, 2-5 % faster than the 8-B form; the stores still cost ~80 of 250 us on the
        // Detect P3 stem slice (profiles/r4_v3_direct_diag.txt).
        // Residual: the block's loads are this wave's youngest vector-memory ops -> vmcnt(0)
        // (older: the previous block's stores, issued a whole MFMA phase ago, and the patch DMA).
        if constexpr (RES) vm_wait<0>(rv[0], rv[1]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (cb * 32 + q * 16 >= COUT) continue;  // wave-uniform (COUT % 16 == 0); counted below
          float rlo[4] = {}, rhi[4] = {};
          if constexpr (RES) {
            // the store exchange below is an involution: applied to the residual (store
            // layout) it yields the accumulator layout, so x + act(conv) rounds once, in fp32
            const auto t0 = __builtin_amdgcn_permlane32_swap(rv[q][0], rv[q][2], false, false);
            const auto t1 = __builtin_amdgcn_permlane32_swap(rv[q][1], rv[q][3], false, false);
            const unsigned wl[2] = {t0[0], t1[0]}, wh[2] = {t0[1], t1[1]};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              rlo[e] = __uint_as_float(e & 1 ? wl[e >> 1] & 0xffff0000u : wl[e >> 1] << 16);
              rhi[e] = __uint_as_float(e & 1 ? wh[e >> 1] & 0xffff0000u : wh[e >> 1] << 16);
            }
          }
          bf16x4 lo, hi;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lo[e] = f2bf(act_c<ACT>(acc[8 * q + e]) + rlo[e]);      // group 2q: 16q + fh*4 + e
            hi[e] = f2bf(act_c<ACT>(acc[8 * q + 4 + e]) + rhi[e]);  // group 2q+1: 16q + 8 + fh*4 + e
          }
          // v_permlane32_swap(a, b): a's lanes 32-63 <-> b's lanes 0-31.  Lane fr then holds
          // (a: own [16q, +4), b: partner's [16q+4, +4)), lane fr + 32 (a: partner's
          // [16q+8, +4), b: own [16q+12, +4)) -- 8 consecutive channels each, no LDS trip
          const u32x2 a0 = __builtin_bit_cast(u32x2, lo), a1 = __builtin_bit_cast(u32x2, hi);
          const auto s0 = __builtin_amdgcn_permlane32_swap(a0[0], a1[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(a0[1], a1[1], false, false);
          const u32x4 v = u32x4{s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v, ry, ok ? pix + (q * 16 + fh * 8) * 2 : kOOB, 0,
                                                 0);
        }
        continue;
      }
      if (jr < npix) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (cb * 32 + g * 8 >= COUT) continue;  // compile-time for COUT % 32 == 0
          bf16x4 o;
          o[0] = f2bf(act_c<ACT>(acc[4 * g + 0]));
          o[1] = f2bf(act_c<ACT>(acc[4 * g + 1]));
          o[2] = f2bf(act_c<ACT>(acc[4 * g + 2]));
          o[3] = f2bf(act_c<ACT>(acc[4 * g + 3]));
          *reinterpret_cast<bf16x4*>(otile + jr * OS + cb * 32 + g * 8 + fh * 4) = o;
        }
      }
    }
    if constexpr (SB) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave done reading the patch: the next DMA may land
      asm volatile("" ::: "memory");
      continue;
    } else if constexpr (DE) {
      // this wave's stores of the band (nbw blocks x ng groups) are its youngest vector-memory
      // ops: wait for everything older -- the next band's patch DMAs -- and leave them in flight
      const int nbw = ph < NPH ? (nblk - ph + NPH - 1) / NPH : 0;
      const int ng = (!RES && (diag & 8)) ? min(4,(COUT - cb * 32 + 7) / 8) : min(2, (COUT - cb * 32 + 15) / 16);
      direct_wait_vm_le(__builtin_amdgcn_readfirstlane(nbw * ng));
      cur ^= 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // next patch visible; this patch's reads all retired
      asm volatile("" ::: "memory");
      continue;
    }
    __syncthreads();  // output tile complete; patch no longer read
    // next band's patch BEFORE this band's stores: on gfx9 vmcnt counts stores too, so a
    // commit after the store pass made its vmcnt(0) wait for this band's stores to land
    if constexpr (!DMA) commit();

    // ---- store the band (+ residual after the activation): 16-B channel chunks
    if constexpr (RPF > 0) {
      if (rpre) {
#pragma unroll
        for (int i = 0; i < RPF; ++i) {
          const int q = tid + NT * i;
          if (q >= npix * OCH) break;
          const int px = q / OCH, c = q - (q / OCH) * OCH;
          const int yl = fdiv(px, fWo), xc = px - yl * Wo;
          const int oy = oy0 + yl;
          if (oy >= Ho) continue;
          const long long m = (long long)(n * Ho + oy) * Wo + xc;
          bf16x8 o8 = *reinterpret_cast<const bf16x8*>(otile + px * OS + c * 8);
          const bf16x8 r8 = __builtin_bit_cast(bf16x8, rpf[i]);
#pragma unroll
          for (int e = 0; e < 8; ++e) o8[e] = f2bf((float)o8[e] + (float)r8[e]);
          *reinterpret_cast<uint4*>(Y + m * p.ldy + p.y_coff + c * 8) = __builtin_bit_cast(uint4, o8);
        }
      }
    }
    if constexpr (C2 > 0) {
      // ---- pair: z = t . W2^T + b2 from the output tile, 32 pixels x 32 channels per unit,
      // stored straight from the accumulators (a lane: 4 consecutive channels of a pixel)
      for (int u = wv; u < nblk * NCB2; u += NWV) {
        const int b = u / NCB2, cb2 = u - b * NCB2;
        floatx16 acc2;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = *reinterpret_cast<const float4*>(lbias2 + cb2 * 32 + g * 8 + fh * 4);
          acc2[4 * g + 0] = bv.x;
          acc2[4 * g + 1] = bv.y;
          acc2[4 * g + 2] = bv.z;
          acc2[4 * g + 3] = bv.w;
        }
        const bf16* tp = otile + (b * 32 + fr) * OS + fh * 8;  // rows past npix: discarded
        const bf16* wp2 = w2s + min(cb2 * 32 + fr, C2 - 1) * OS + fh * 8;
#pragma unroll
        for (int ks = 0; ks < COUT / 16; ++ks)
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              *reinterpret_cast<const bf16x8*>(wp2 + ks * 16),
              *reinterpret_cast<const bf16x8*>(tp + ks * 16), acc2, 0, 0, 0);
        // buffer stores, out-of-range lanes dropped by the descriptor: every wave issues
        // exactly ng2(cb2) stores per unit, so the band end can count them (below)
        const int jr = b * 32 + fr;
        const int jc = min(jr, npix - 1);
        const int yl = fdiv(jc, fWo), xc = jc - yl * Wo;
        const int oy = oy0 + yl;
        const bool ok = jr < npix && oy < Ho;
        const int base = (((n * Ho + oy) * Wo + xc) * p.ldz + p.z_coff + cb2 * 32 + fh * 4) * 2;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (cb2 * 32 + g * 8 >= C2) continue;  // wave-uniform
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(acc2[4 * g + e]);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), rz,
                                                ok ? base + g * 16 : kOOB, 0, 0);
        }
      }
      if constexpr (DMA) {
        // the z stores are this wave's youngest vector-memory ops: wait for the next patch's
        // DMAs only, then an LDS-only barrier (__syncthreads' fence would drain the stores)
        int nz = 0;
        for (int u = wv; u < nblk * NCB2; u += NWV) {
          const int cb2 = u - (u / NCB2) * NCB2;
          nz += min(4, (C2 - cb2 * 32 + 7) / 8);
        }
        direct_wait_vm_le(__builtin_amdgcn_readfirstlane(nz));
        cur ^= 1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // next patch visible; output tile and patch free
        asm volatile("" ::: "memory");
        continue;
      }
    }
    constexpr int ST0 = SPLIT ? NWD * 64 : 0;  // first storing thread
    for (int q = C2 > 0 ? npix * OCH : RPF > 0 && rpre ? npix * OCH : tid - ST0; q < npix * OCH;
         q += NT - ST0) {
      if (SPLIT && q < 0) break;  // a DMA wave
      const int px = q / OCH, c = q - (q / OCH) * OCH;
      const int yl = fdiv(px, fWo), xc = px - yl * Wo;
      const int oy = oy0 + yl;
      if (oy >= Ho) continue;
      const long long m = (long long)(n * Ho + oy) * Wo + xc;
      uint4 v = *reinterpret_cast<const uint4*>(otile + px * OS + c * 8);
      if constexpr (RES) {
        const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(R + m * p.ldr + p.r_coff + c * 8);
        bf16x8 o8 = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) o8[e] = f2bf((float)o8[e] + (float)r8[e]);
        v = __builtin_bit_cast(uint4, o8);
      }
      *reinterpret_cast<uint4*>(Y + m * p.ldy + p.y_coff + c * 8) = v;
    }
    if constexpr (DMA) {
      if (!SPLIT || wv < NWD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMAs landed
      cur ^= 1;
    }
    __syncthreads();  // patch ready, output tile free
  }
}

typedef void (*DirectFn)(const KvConvParams, int, int, int, FastDiv, FastDiv, int);

struct DirectEntry {
  int cin, cout, stride, kk, act;
  bool res;
  DirectFn fn;
  bool u8 = false;
  bool dma = false;
  bool pairs = false;  // frames-in with even W: 12-B paired raw-row loads
  int occ = 1;         // workgroups per CU (launch bounds, LDS budget, grid)
  int nt = kNT;        // threads per workgroup
  int c2 = 0;          // fused 1x1 pair: its output channels (0 = plain conv)
  bool de = false;     // direct epilogue (v10 tiles; DMA forms only)
  bool sb = false;     // single patch buffer, 4 waves, two workgroups per CU (v10 tile 2)
};

#define KV_DIRECT(CI, CO, S, A, R) {CI, CO, S, 3, A, R, conv3x3_direct_kernel<CI, CO, S, 3, A, R>}
// the same shape with the DMA patch fetch (direct tile 1; the autotuner picks per layer)
#define KV_DIRECT_DMA(CI, CO, S, A, R) \
  {CI, CO, S, 3, A, R, conv3x3_direct_kernel<CI, CO, S, 3, A, R, false, true>, false, true}
#define KV_DIRECT2(CI, CO, S, A, R) KV_DIRECT(CI, CO, S, A, R), KV_DIRECT_DMA(CI, CO, S, A, R)
// two workgroups per CU (direct tiles 2 / 3)
#define KV_DIRECT_OCC2(CI, CO, S, KK, A, R)                                                       \
  {CI, CO, S, KK, A, R, conv3x3_direct_kernel<CI, CO, S, KK, A, R, false, true, false, 2>, false, \
   true, false, 2}
// v10: the direct-epilogue forms (one or two workgroups per CU)
#define KV_DIRECT_DE(CI, CO, S, KK, A)                                                          \
  {CI, CO, S, KK, A, false,                                                                    \
   conv3x3_direct_kernel<CI, CO, S, KK, A, false, false, true, false, 1, kNT, 0, true>, false,  \
   true, false, 1, kNT, 0, true}
// ... with the residual added after the activation (YOLO C2f bottleneck cv2: x + silu(conv))
#define KV_DIRECT_DER(CI, CO, OCC)                                                               \
  {CI, CO, 1, 3, kActSilu, true,                                                                 \
   conv3x3_direct_kernel<CI, CO, 1, 3, kActSilu, true, false, true, false, OCC, kNT, 0, true>,   \
   false, true, false, OCC, kNT, 0, true}
#define KV_DIRECT_DE2(CI, CO, S, KK, A)                                                         \
  {CI, CO, S, KK, A, false,                                                                    \
   conv3x3_direct_kernel<CI, CO, S, KK, A, false, false, true, false, 2, kNT, 0, true>, false,  \
   true, false, 2, kNT, 0, true}
#define KV_DIRECT_SB(CI, CO, S, KK, A)                                                          \
  {CI, CO, S, KK, A, false,                                                                    \
   conv3x3_direct_kernel<CI, CO, S, KK, A, false, false, true, false, 2, 256, 0, true, true>,   \
   false, true, false, 2, 256, 0, true, true}
#define KV_DIRECT_DE4(CI, CO, S, KK, A)                                                         \
  {CI, CO, S, KK, A, false,                                                                    \
   conv3x3_direct_kernel<CI, CO, S, KK, A, false, false, true, false, 1, 256, 0, true>, false,  \
   true, false, 1, 256, 0, true}
#define KV_DIRECT1(CI, CO, A)                                                        \
  {CI, CO, 1, 1, A, false, conv3x3_direct_kernel<CI, CO, 1, 1, A, false>},           \
  {CI, CO, 1, 1, A, false, conv3x3_direct_kernel<CI, CO, 1, 1, A, false, false, true>, false, true}
// the 3x3 shapes of ResNet-50 stage 1 and YOLOv8n's narrow layers (backbone, C2f
// bottlenecks, PAN downsamplers, Detect 64-channel branches)
static const DirectEntry kDirect[] = {
    KV_DIRECT2(64, 64, 1, kActRelu, false),   // ResNet-50 layer1 conv2 x3
    KV_DIRECT2(64, 64, 1, kActNone, false),
    KV_DIRECT2(16, 32, 2, kActSilu, false),   // YOLO b1
    KV_DIRECT2(16, 16, 1, kActSilu, false),   // b2 bottleneck cv1
    KV_DIRECT2(16, 16, 1, kActSilu, true),    // b2 bottleneck cv2 (+x)
    KV_DIRECT2(32, 64, 2, kActSilu, false),   // b3
    KV_DIRECT2(32, 32, 1, kActSilu, false),   // b4 / h15 bottlenecks
    KV_DIRECT2(32, 32, 1, kActSilu, true),
    KV_DIRECT2(64, 128, 2, kActSilu, false),  // b5
    KV_DIRECT2(64, 64, 1, kActSilu, false),   // b6 / h12 / h18 bottlenecks, Detect a1
    KV_DIRECT2(64, 64, 1, kActSilu, true),
    KV_DIRECT2(64, 64, 2, kActSilu, false),   // h16
    KV_DIRECT2(64, 128, 1, kActSilu, false),  // Detect P3 merged branch stem 64 -> 144 =
    KV_DIRECT2(64, 16, 1, kActSilu, false),   //   128 + 16 (Cout split, direct_launch)
    // 1x1 (KK = 1, pad 0): YOLO C2f cv1 / cv2 at 160^2 and 80^2, the neck's 80^2 C2f, and the
    // Detect heads' final 1x1 convs (no activation, written into the 144-channel head map)
    KV_DIRECT1(32, 32, kActSilu), KV_DIRECT1(48, 32, kActSilu), KV_DIRECT1(64, 64, kActSilu),
    KV_DIRECT1(128, 64, kActSilu), KV_DIRECT1(192, 64, kActSilu), KV_DIRECT1(96, 64, kActSilu),
    KV_DIRECT1(64, 64, kActNone), KV_DIRECT1(80, 80, kActNone),
    // two-workgroups-per-CU forms of the narrow, latency-bound YOLO layers
    KV_DIRECT_OCC2(16, 32, 2, 3, kActSilu, false), KV_DIRECT_OCC2(16, 16, 1, 3, kActSilu, false),
    KV_DIRECT_OCC2(32, 64, 2, 3, kActSilu, false), KV_DIRECT_OCC2(32, 32, 1, 3, kActSilu, false),
    KV_DIRECT_OCC2(32, 32, 1, 1, kActSilu, false), KV_DIRECT_OCC2(48, 32, 1, 1, kActSilu, false),
    // ResNet-50 stage-2 conv2 (128 -> 128 @28^2, stride 1): 4 waves, each holding one 32-channel
    // block's 288 weight VGPRs, one workgroup per CU; the band patch is staged once per band
    // instead of once per tap (the implicit GEMM re-reads every input pixel 9x through L2)
    {128, 128, 1, 3, kActRelu, false,
     conv3x3_direct_kernel<128, 128, 1, 3, kActRelu, false, false, true, false, 1, 256>, false, true,
     false, 1, 256},
    // Detect cls branch 3x3 (c3 = 80), NCB = 3: DMA form only (the VGPR-prefetch form
    // spills with 180 weight VGPRs and fits one output row per band)
    KV_DIRECT_DMA(80, 80, 1, kActSilu, false),
    // YOLO b0 stem in space-to-depth form: 2x2 over [N,320,320,16]
    {16, 16, 1, 2, kActSilu, false, conv3x3_direct_kernel<16, 16, 1, 2, kActSilu, false>},
    // ... and its frames-in form (preprocess fused): even W (paired loads) / odd W
    {16, 16, 1, 2, kActSilu, false,
     conv3x3_direct_kernel<16, 16, 1, 2, kActSilu, false, true, false, true>, true, false, true},
    {16, 16, 1, 2, kActSilu, false, conv3x3_direct_kernel<16, 16, 1, 2, kActSilu, false, true>,
     true},
    // YOLO Detect branch pairs, 3x3 + SiLU then 1x1 (no act) into the head map: box branch
    // 64 -> 64 -> 64, cls branch 80 -> 80 -> 80 (DMA patch fetch)
    {64, 64, 1, 3, kActSilu, false,
     conv3x3_direct_kernel<64, 64, 1, 3, kActSilu, false, false, true, false, 1, kNT, 64>, false,
     true, false, 1, kNT, 64},
    {80, 80, 1, 3, kActSilu, false,
     conv3x3_direct_kernel<80, 80, 1, 3, kActSilu, false, false, true, false, 1, kNT, 80>, false,
     true, false, 1, kNT, 80},
    // v10 direct-epilogue forms (listed last: the v4 tiles' any-form fallback never lands here)
    KV_DIRECT_DE(64, 64, 1, 3, kActRelu),     // ResNet-50 layer1 conv2
    KV_DIRECT_DE(64, 128, 1, 3, kActSilu),    // Detect P3 merged stem 64 -> 144 = 128 + 16
    KV_DIRECT_DE(64, 16, 1, 3, kActSilu),
    KV_DIRECT_DE(64, 80, 1, 3, kActSilu),     // ... or 80 + 64 (KVEDGE_DIRECT_SPLIT=balanced)
    KV_DIRECT_DE(64, 64, 1, 3, kActSilu),     // bottleneck cv1 / Detect a1
    KV_DIRECT_DE(80, 80, 1, 3, kActSilu),
    KV_DIRECT_DE(64, 128, 2, 3, kActSilu),    // b5
    KV_DIRECT_DE(64, 64, 2, 3, kActSilu),     // h16
    KV_DIRECT_DE(32, 64, 2, 3, kActSilu),     // b3
    KV_DIRECT_DE(16, 32, 2, 3, kActSilu),     // b1
    KV_DIRECT_DE(32, 32, 1, 3, kActSilu),
    KV_DIRECT_DE(16, 16, 1, 3, kActSilu),
    KV_DIRECT_DE(32, 32, 1, 1, kActSilu), KV_DIRECT_DE(48, 32, 1, 1, kActSilu),
    KV_DIRECT_DE(64, 64, 1, 1, kActSilu), KV_DIRECT_DE(128, 64, 1, 1, kActSilu),
    KV_DIRECT_DE(192, 64, 1, 1, kActSilu), KV_DIRECT_DE(96, 64, 1, 1, kActSilu),
    KV_DIRECT_DE(64, 64, 1, 1, kActNone), KV_DIRECT_DE(80, 80, 1, 1, kActNone),
    KV_DIRECT_DE2(16, 32, 2, 3, kActSilu), KV_DIRECT_DE2(16, 16, 1, 3, kActSilu),
    KV_DIRECT_DE2(32, 64, 2, 3, kActSilu), KV_DIRECT_DE2(32, 32, 1, 3, kActSilu),
    KV_DIRECT_DE2(32, 32, 1, 1, kActSilu), KV_DIRECT_DE2(48, 32, 1, 1, kActSilu),
    KV_DIRECT_DER(16, 16, 1), KV_DIRECT_DER(32, 32, 1), KV_DIRECT_DER(64, 64, 1),
    KV_DIRECT_DER(16, 16, 2), KV_DIRECT_DER(32, 32, 2),
    KV_DIRECT_SB(64, 64, 1, 3, kActRelu), KV_DIRECT_SB(64, 128, 1, 3, kActSilu),
    KV_DIRECT_SB(64, 16, 1, 3, kActSilu), KV_DIRECT_SB(64, 64, 1, 3, kActSilu),
    KV_DIRECT_SB(64, 80, 1, 3, kActSilu),
    KV_DIRECT_SB(64, 128, 2, 3, kActSilu), KV_DIRECT_SB(64, 64, 2, 3, kActSilu),
    KV_DIRECT_SB(32, 64, 2, 3, kActSilu), KV_DIRECT_SB(32, 32, 1, 3, kActSilu),
    KV_DIRECT_SB(80, 80, 1, 3, kActSilu),
    // CIN = 128 at 4 waves, one workgroup per CU (288 weight VGPRs per wave): ResNet-50
    // stage-2 conv2 and YOLO's 128-channel 3x3s, as v10 tile 0
    KV_DIRECT_DE4(128, 128, 1, 3, kActRelu), KV_DIRECT_DE4(128, 128, 1, 3, kActSilu),
    KV_DIRECT_DE4(128, 128, 2, 3, kActSilu),
};
#undef KV_DIRECT2
#undef KV_DIRECT_DE
#undef KV_DIRECT_DE2
#undef KV_DIRECT_DER
#undef KV_DIRECT_SB
#undef KV_DIRECT_DE4
#undef KV_DIRECT1
#undef KV_DIRECT_OCC2
#undef KV_DIRECT_DMA
#undef KV_DIRECT

int direct_pb(int cin) { return cin * 2 + 16; }
int direct_max_patch(int cin) { return (cin >= 80 ? 6 : cin >= 64 ? 7 : 10) * kNT * 16; }

}  // namespace

// tile 0: the VGPR-prefetch form where one exists; tile 1: the DMA form where one exists
// tile bit 0: DMA patch fetch; bit 1: two workgroups per CU (the OCC = 2 forms).
// Internal codes 4..7 (bit 2) are the direct-epilogue forms, exposed as the v10 tiles
// (direct_de_launch): they take only their own instantiations, no fallback.
int direct_num_tiles() { return 4; }
int direct_de_num_tiles() { return 3; }

// Returns the instantiation index for p (or < 0), and the band geometry it would use.
static int direct_plan(const KvConvParams* p, int tile, int* kR, int* PW, int* rows, int* lds) {
  const int kk = p->KH;
  if (p->KW != kk || kk < 1 || kk > 3) return -8;
  if (kk == 1 ? (p->pad != 0 || p->stride != 1 || p->Ho != p->H || p->Wo != p->W ||
                 (p->mode != 0 && p->mode != 1))
              : (p->mode != 0 || p->pad != 1))
    return -8;
  if (p->stride != 1 && p->stride != 2) return -8;
  if (kk == 2 && (p->stride != 1 || p->Ho != p->H || p->Wo != p->W)) return -8;  // s2d stem
  const int act = p->act & 3;
  const bool res = p->res != nullptr;
  if (res && !(p->act & 4) && act != kActNone) return -8;  // only x + act(conv)
  int idx = -1;
  for (int pass = 0; pass < ((tile & 4) ? 1 : 2) && idx < 0; ++pass) {  // the tile's form, then any
    for (int i = 0; i < (int)(sizeof(kDirect) / sizeof(kDirect[0])); ++i) {
      const DirectEntry& e = kDirect[i];
      if (e.cin == p->Cin && e.cout == p->Cout && e.stride == p->stride && e.kk == kk &&
          e.act == act && e.res == res && e.u8 == (p->in_u8 != 0) &&
          (!e.u8 || e.pairs == (p->W % 2 == 0)) &&
          e.c2 == (p->pair_1x1 ? p->n_t : 0) && e.de == ((tile & 4) != 0) &&
          e.sb == ((tile & 8) != 0) &&
          (pass == 1 || (e.dma == ((tile & 1) != 0) && e.occ == 1 + ((tile >> 1) & 1)))) {
        idx = i;
        break;
      }
    }
  }
  if (idx < 0) return -8;
  if (p->Kpad != (kk * kk * p->Cin + 63) / 64 * 64 || p->ldx % 8 || p->x_coff % 8) return -8;
  if (p->in_u8 && (long long)p->N * p->H * p->W * 12 >= kOOB) return -9;
  if (kk == 3 && (p->Ho != (p->H - 1) / p->stride + 1 || p->Wo != (p->W - 1) / p->stride + 1))
    return -8;
  if (!p->in_u8 && (long long)p->N * p->H * p->W * p->ldx * 2 >= kOOB) return -9;
  if ((long long)p->N * p->Ho * p->Wo * p->ldy * 2 >= kOOB) return -9;
  if (p->pair_1x1 && (long long)p->N * p->Ho * p->Wo * p->ldz * 2 >= kOOB) return -9;
  if (res && (long long)p->N * p->Ho * p->Wo * p->ldr * 2 >= kOOB) return -9;
  const int S = p->stride;
  *PW = (p->Wo - 1) * S + kk;
  const int pb = direct_pb(p->Cin);
  const int os = p->Cout + 8;
  // rows per band: as many as fit (<= 8) in the prefetch budget and LDS
  // (DMA form: two patch buffers in LDS, no VGPR prefetch budget)
  const bool dma = kDirect[idx].dma;
  auto lds_of = [&](int prows, int r) {
    const int np = dma && !kDirect[idx].sb ? 2 : 1;
    const int c2p = kDirect[idx].c2;  // pair: b2 slot + W2 [c2][os]
    const int ot = kDirect[idx].de ? 0 : ((r * p->Wo * os * 2 + 15) & ~15);  // output tile
    return np * direct_patch_alloc(prows * *PW * pb, dma) + ot + kBiasBytes +
           (c2p ? kBiasBytes + c2p * os * 2 : 0);
  };
  // band height: the tallest that fits (<= 8).  (A "fewest pixel-block rounds" rule was
  // measured slower on YOLO's 32-channel layers at 160^2: the extra halo rows and per-band
  // overhead of shorter bands outweigh the better MFMA-phase balance.)
  int r = 8;
  for (; r >= 1; --r) {
    const int prows = (r - 1) * S + kk;
    const int patch = prows * *PW * pb;
    if ((dma || patch <= direct_max_patch(p->Cin)) && lds_of(prows, r) <= kLds / kDirect[idx].occ)
      break;
  }
  if (r < 1) return -11;
  if (r > p->Ho) r = p->Ho;
  *kR = r;
  *rows = (r - 1) * S + kk;
  *lds = lds_of(*rows, r);
  return idx;
}

// KVEDGE_DIRECT_DIAG (timing experiments on the direct-epilogue forms only; bits 0-2 make
// the outputs wrong): bit 0 drops the stores, bit 1 the next-band patch prefetch, bit 2 the
// MFMAs; bit 3 selects the first (4 x 8-B) store form, for same-box A/B.
static int direct_diag() {
  const char* e = getenv("KVEDGE_DIRECT_DIAG");
  return e ? atoi(e) : 0;
}

static int direct_launch_one(const KvConvParams* p, int tile, hipStream_t stream) {
  int kR, PW, rows, lds;
  const int idx = direct_plan(p, tile, &kR, &PW, &rows, &lds);
  if (idx < 0) return idx;
  const long long items = (long long)p->N * ((p->Ho + kR - 1) / kR);
  if (items <= 0) return 0;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long long slots = (long long)ncu * kDirect[idx].occ;  // persistent: occ per CU
  const unsigned g = (unsigned)(items < slots ? items : slots);
  const DirectFn fn = kDirect[idx].fn;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(fn, dim3(g), dim3(kDirect[idx].nt), (unsigned)lds, stream, *p, kR, PW, rows,
                     make_fastdiv(PW), make_fastdiv(p->Wo), direct_diag());
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

// A Cout with no instantiation of its own is covered by consecutive output-channel slices
// that have one, e.g. YOLO's merged Detect stem 64 -> 144: each slice re-reads the input and
// writes its y_coff range, largest first (144 = 128 + 16).  KVEDGE_DIRECT_SPLIT=balanced
// takes the most balanced two-slice split instead (144 = 80 + 64 with the 64 -> 80 forms):
// the 16-wide slice does a ninth of the work at a fifth of the MFMA rate
// (profiles/r5_v10_graph_layers_yolo_b512_c2f.md: 137 vs 206 us per b256 slice), but the
// balanced pair measured level on the bench (profiles/r5_v15_direct_split_ab.txt).
int direct_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= 16) return -6;
  int kR, PW, rows, lds;
  if (direct_plan(p, tile, &kR, &PW, &rows, &lds) >= 0) return direct_launch_one(p, tile, stream);
  if (p->res || p->Cout % 16 || p->pair_1x1) return -8;
  static const bool greedy =
      !(getenv("KVEDGE_DIRECT_SPLIT") && strcmp(getenv("KVEDGE_DIRECT_SPLIT"), "balanced") == 0);
  // validate the whole split before launching anything
  int cuts[8], ncut = 0, done = 0;
  auto fits = [&](int cout) {
    KvConvParams q = *p;
    q.Cout = cout;
    return direct_plan(&q, tile, &kR, &PW, &rows, &lds) >= 0;
  };
  if (!greedy) {
    int best = 0;
    for (const DirectEntry& e : kDirect) {
      const int a = e.cout, b = p->Cout - e.cout;
      if (a >= b && b > 0 && (best == 0 || a < best) && fits(a) && fits(b)) best = a;
    }
    if (best) {
      cuts[ncut++] = best;
      cuts[ncut++] = p->Cout - best;
      done = p->Cout;
    }
  }
  while (done < p->Cout && ncut < 8) {
    int best = 0;
    for (const DirectEntry& e : kDirect) {
      KvConvParams q = *p;
      q.Cout = e.cout;
      if (e.cout <= p->Cout - done && e.cout > best && direct_plan(&q, tile, &kR, &PW, &rows, &lds) >= 0)
        best = e.cout;
    }
    if (best == 0) return -8;
    cuts[ncut++] = best;
    done += best;
  }
  if (done != p->Cout) return -8;
  int off = 0;
  for (int i = 0; i < ncut; ++i) {
    KvConvParams q = *p;
    q.Cout = cuts[i];
    q.w = static_cast<const bf16*>(p->w) + (size_t)off * p->Kpad;
    q.bias = p->bias ? p->bias + off : nullptr;
    q.y_coff = p->y_coff + off;
    const int rc = direct_launch_one(&q, tile, stream);
    if (rc != 0) return rc;
    off += cuts[i];
  }
  return 0;
}

// v10 tile 0 / 1: the DMA direct-epilogue form at 1 / 2 workgroups per CU (8 waves);
// tile 2: its single-buffer 4-wave form, two workgroups per CU
int direct_de_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= direct_de_num_tiles() || p->pair_1x1) return -8;
  // KVEDGE_DE_RES=0: the residual forms refuse (same-box A/B against the v1 / v4 picks)
  static const bool de_res = !getenv("KVEDGE_DE_RES") || atoi(getenv("KVEDGE_DE_RES")) != 0;
  if (p->res && !de_res) return -8;
  static const int code[3] = {4 | 1, 4 | 2 | 1, 4 | 8 | 2 | 1};
  return direct_launch(p, code[tile], stream);
}

}  // namespace kvedge

extern "C" int kv_conv_pair(const KvConvParams* p, int tile, hipStream_t stream) {
  if (!p->pair_1x1 || p->n_t <= 0 || !p->w_t || !p->z) return -8;
  return kvedge::direct_launch(p, tile, stream);
}
extern "C" int kv_conv_pair_num_tiles(void) { return kvedge::direct_num_tiles(); }
