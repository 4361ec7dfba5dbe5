// K2+K5+K12 fused, second generation: ResNet stem 7x7/2 conv (BN folded) + ReLU + 3x3/2
// max pool straight from raw uint8 frames, as a stride-1 4x4 conv over a 12-CHANNEL
// space-to-depth image (gfx950).
//
// Why a new formulation (stem+pool at 0.19 of its floor).  stem_pool.hip runs
// the 7x7x3 taps as a 4x4 conv over a 16-channel s2d image (3 colours padded to 4): K = 256
// for 147 real MACs, 1.74x the model work.  Here an s2d pixel is 2x2 input pixels x 3
// colours = 12 channels with no pad channel, so one s2d tap ROW (4 taps) is 48 contiguous
// K values and K = 4 x 48 = 192 (1.31x): 24 v_mfma_f32_32x32x16 per 32 pixels x 64
// channels instead of 32.  The weight of tap (r, s, dy, dx, c) is w[2r-1+dy][2s-1+dx][c]
// (zero where that falls outside 0..6: the 8x8 window covers the 7x7 kernel).
//
// A lane's 8-element K chunk of pixel x, tap row r, k-step j (3 per row) starts at byte
// 24x + 32j + 16h of the s2d row: 8-B aligned, read as two ds_read_b64 (lanes 0-31 hit
// banks 6x + {0,1} mod 64 -- all 64 once: conflict-free).  Addresses are one VGPR per tap
// row + immediates.
//
// Structure (2 workgroups of 4 waves per CU, ~68 KB LDS each, persistent over a contiguous
// range of (image, pooled row) bands -- one pooled row per band):
//  * s2d ring: 6 rows of (W + 4) s2d pixels (2 zero columns each side, written once).  A
//    band's NEW s2d rows (2 when the previous band was the row above, 5 at an image start)
//    are loaded as raw bytes into VGPRs at the START of the previous band (one 12-B
//    buffer_load per two s2d pixels of one input row) and normalised + committed after
//    its MFMA phase, so the fetch latency hides under the MFMAs;
//  * stem ring: 3 rows x W pixels x 64 channels (72-element pitch), bf16 WITHOUT the ReLU;
//    each band computes its 2 new stem rows (3 for the first band of a range) as 32-pixel
//    blocks of the flattened row pair, round-robin over the 4 waves, accumulators seeded
//    with the folded-BN bias, weights resident in 96 VGPRs;
//  * pool: max over the 3x3 window on the bf16 bit patterns as signed 16-bit integers
//    (v_pk_max_i16), then max with 0: relu(max(v)) == max(relu(v)), and whenever the max
//    is positive signed-int16 order agrees with float order (negatives, which int16 orders
//    backwards, only ever lose to a positive or are clamped to 0) -- the ReLU runs on the
//    pooled 1/4 of the pixels only.  Window taps outside the image are clamped onto the
//    window's in-image taps (a duplicate never changes a max).
// Two workgroups per CU are what hides each one's commit / pool phase under the other's
// MFMAs: the previous kernel (one 8-wave workgroup per CU, 129 KB LDS) ran them in series
// (PMC: 9 VALU per MFMA, 40 % of wave cycles waiting).
#include <stdlib.h>

#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace kvedge {
namespace {

constexpr int kC = 64;         // stem output channels
constexpr int kK = 192;        // 4 tap rows x 4 taps x 12 s2d channels
constexpr int kKs = kK / 16;   // 12 k-steps of v_mfma_f32_32x32x16
constexpr int kNT = 256;       // 4 waves
constexpr int kRing = 6;       // s2d rows resident
constexpr int kSR = 3;         // stem rows resident
constexpr int kTP = 72;        // stem tile pixel pitch (elements): 64 + 8
constexpr int kMaxLoads = 2;   // raw 12-B loads per thread per band (<= 3 s2d rows, W <= 256)

struct StemNorm12 {
  float a[3], b[3];
};

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk_max_i16(unsigned a, unsigned b) {
  const i16x2 r = __builtin_elementwise_max(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, b));
  return __builtin_bit_cast(unsigned, r);
}

__device__ __forceinline__ int ring6(int Y) { return (Y + 6 * 4) % kRing; }  // Y >= -24

// two floats -> one dword of two bf16 (one v_cvt_pk_bf16_f32; a in the low half)
typedef __bf16 stem_bf16x2 __attribute__((ext_vector_type(2)));
typedef float stem_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned stem_pk2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((stem_f2){a, b}, stem_bf16x2));
}
// byte B (compile-time, 0..11) of a 12-B raw load as float: one v_cvt_f32_ubyteN
template <int B>
__device__ __forceinline__ float stem_ub(const u32x3& r) {
  return (float)((r[B >> 2] >> (8 * (B & 3))) & 0xffu);
}

__global__ __launch_bounds__(kNT, 2) void stem12_pool_kernel(
    const unsigned char* __restrict__ frames, const bf16* __restrict__ w,
    const float* __restrict__ bias, bf16* __restrict__ y, int N, int Hs, int Ws, int Hp, int Wp,
    int ldy, int y_coff, StemNorm12 nrm, int RP) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* ring = lds;                                         // kRing x RP bytes
  unsigned char* stem = lds + kRing * RP;                            // kSR x Ws x kTP bf16
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int W0 = 2 * Ws;  // input width (pixels)

  // ---- weights -> VGPRs once: fragment (cb, t): rows cb*32 + fr, k = t*16 + fh*8 .. +8
  bf16x8 wreg[2][kKs];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int t = 0; t < kKs; ++t)
      wreg[cb][t] = *reinterpret_cast<const bf16x8*>(w + (cb * 32 + fr) * kK + t * 16 + fh * 8);
  // the folded-BN bias as the C operand of each block's first MFMA (accumulator layout:
  // element 4g + e = channel g * 8 + fh * 4 + e): no per-block seeding moves
  floatx16 bias16[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 v = *reinterpret_cast<const float4*>(bias + cb * 32 + g * 8 + fh * 4);
      kv_settle(v);  // loaded once: no waits for it inside the band loop
      bias16[cb][4 * g + 0] = v.x;
      bias16[cb][4 * g + 1] = v.y;
      bias16[cb][4 * g + 2] = v.z;
      bias16[cb][4 * g + 3] = v.w;
    }
  // loaded once: no waits for them inside the band loop (which has the raw prefetch in flight)
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
    for (int t = 0; t < kKs; ++t) kv_settle(wreg[cb][t]);
  }

  // ---- zero columns of every ring row (s2d X = -2, -1 and Ws, Ws + 1): written once
  for (int i = tid; i < kRing * 6; i += kNT) {
    const int r = i / 6, q = i % 6;  // 3 x 16 B on each side
    const int off = q < 3 ? q * 16 : (Ws + 2) * 24 + (q - 3) * 16;
    *reinterpret_cast<uint4*>(ring + r * RP + off) = make_uint4(0, 0, 0, 0);
  }

  const int total = N * Hp;
  const int per = (total + gridDim.x - 1) / gridDim.x;
  const int b0 = blockIdx.x * per, b1 = min(b0 + per, total);
  if (b0 >= b1) return;

  const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(frames), (short)0, N * Hs * 2 * W0 * 3, 0x00020000);
  const int pairs = Ws / 2;     // 12-B loads per input row
  const int per_row = 2 * pairs;  // loads per s2d row (two input rows)

  // Band-invariant load geometry (computed once, not per band): load i of this thread
  // covers s2d row ld_j of a fetch, input-row parity ld_dy, s2d pixel pair k of that row --
  // global byte offset ld_g within the s2d row, LDS byte offset ld_l within the ring row
  int ld_j[kMaxLoads], ld_g[kMaxLoads], ld_l[kMaxLoads];
  bool ld_dy[kMaxLoads];
#pragma unroll
  for (int i = 0; i < kMaxLoads; ++i) {
    const int q = tid + kNT * i;
    const int j = q / per_row, rem = q - j * per_row;
    const int dy = rem / pairs, k = rem - dy * pairs;
    ld_j[i] = j;
    ld_dy[i] = dy != 0;
    ld_g[i] = (dy * W0 + 4 * k) * 3;
    ld_l[i] = (2 * k + 2) * 24 + dy * 12;
  }
  const int srow_bytes = 2 * W0 * 3;  // one s2d row = two input rows

  // Raw prefetch of s2d rows [Ylo, Ylo + nrows) of image n (rows outside the image and
  // loads past the row count read nothing: the out-of-range offset returns zeros).
  u32x3 raw[kMaxLoads];
  unsigned okm = 0;
  auto fetch = [&](int n, int Ylo, int nrows) __attribute__((always_inline)) {
    okm = 0;
    const int base = (n * Hs + Ylo) * srow_bytes;
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      const int Y = Ylo + ld_j[i];
      const bool ok = ld_j[i] < nrows && (unsigned)Y < (unsigned)Hs;
      raw[i] = __builtin_amdgcn_raw_buffer_load_b96(rf, ok ? base + ld_j[i] * srow_bytes + ld_g[i]
                                                             : 0x7ffffff0, 0, 0);
      okm |= ok ? 1u << i : 0u;
    }
  };
  // write the fetched rows (and zeros for the rows that are outside the image).  Byte b of
  // the 12 is colour b % 3 of input pixel 4k + b / 3: v = byte * a[c] + b[c], with b[c]
  // zeroed for a load that read nothing (its bytes are 0), so out-of-image pixels are 0, not
  // -mean / std (the conv padding stays exact) -- no per-element select
  auto commit = [&](int Ylo, int nrows) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      if (ld_j[i] >= nrows) continue;
      const bool ok = (okm >> i) & 1u;
      const float a0 = nrm.a[0], a1 = nrm.a[1], a2 = nrm.a[2];
      const float c0 = ok ? nrm.b[0] : 0.f, c1 = ok ? nrm.b[1] : 0.f, c2 = ok ? nrm.b[2] : 0.f;
      const u32x3 r = raw[i];
      unsigned char* p0 = ring + ring6(Ylo + ld_j[i]) * RP + ld_l[i];  // s2d pixel 2k
      unsigned char* p1 = p0 + 24;                                       // s2d pixel 2k + 1
      const unsigned d0 = stem_pk2(stem_ub<0>(r) * a0 + c0, stem_ub<1>(r) * a1 + c1);
      const unsigned d1 = stem_pk2(stem_ub<2>(r) * a2 + c2, stem_ub<3>(r) * a0 + c0);
      const unsigned d2 = stem_pk2(stem_ub<4>(r) * a1 + c1, stem_ub<5>(r) * a2 + c2);
      const unsigned e0 = stem_pk2(stem_ub<6>(r) * a0 + c0, stem_ub<7>(r) * a1 + c1);
      const unsigned e1 = stem_pk2(stem_ub<8>(r) * a2 + c2, stem_ub<9>(r) * a0 + c0);
      const unsigned e2 = stem_pk2(stem_ub<10>(r) * a1 + c1, stem_ub<11>(r) * a2 + c2);
      if (!ld_dy[i]) {
        *reinterpret_cast<uint2*>(p0) = make_uint2(d0, d1);
        *reinterpret_cast<unsigned*>(p0 + 8) = d2;
        *reinterpret_cast<uint2*>(p1) = make_uint2(e0, e1);
        *reinterpret_cast<unsigned*>(p1 + 8) = e2;
      } else {
        *reinterpret_cast<unsigned*>(p0) = d0;
        *reinterpret_cast<uint2*>(p0 + 4) = make_uint2(d1, d2);
        *reinterpret_cast<unsigned*>(p1) = e0;
        *reinterpret_cast<uint2*>(p1 + 4) = make_uint2(e1, e2);
      }
    }
  };

  const FastDiv fW = make_fastdiv(Ws);
  // ---- one band: stem rows [ys, ye) -> stem ring (MFMA), all 4 waves
  auto stem_rows = [&](int ys, int ye) __attribute__((always_inline)) {
    const int npix = (ye - ys) * Ws;
    const int nblk = (npix + 31) / 32;
    for (int blk = wv; blk < nblk; blk += 4) {
      const int j = min(blk * 32 + fr, npix - 1);
      const int yl = fdiv(j, fW), x = j - yl * Ws;
      const int yr = ys + yl;  // stem row of this lane's pixel
      int ra[4];               // byte address of tap row r's 48-element window (+ k half)
#pragma unroll
      for (int r = 0; r < 4; ++r) ra[r] = ring6(yr - 2 + r) * RP + x * 24 + fh * 16;
      floatx16 acc[2];
      bf16x8 af[3];
      auto load = [&](int buf, int t) __attribute__((always_inline)) {
        const unsigned char* pa = ring + ra[t / 3] + (t % 3) * 32;
        const uint2 lo = *reinterpret_cast<const uint2*>(pa);
        const uint2 hi = *reinterpret_cast<const uint2*>(pa + 8);
        af[buf] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      };
      load(0, 0);
      load(1, 1);
#pragma unroll
      for (int t = 0; t < kKs; ++t) {
        if (t + 2 < kKs) load((t + 2) % 3, t + 2);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[0][t], af[t % 3],
                                                         t == 0 ? bias16[0] : acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[1][t], af[t % 3],
                                                         t == 0 ? bias16[1] : acc[1], 0, 0, 0);
      }
      // keep the reads two k-steps ahead of the MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int t = 0; t < kKs; ++t) {
        if (t + 2 < kKs) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      if (blk * 32 + fr < npix) {
        unsigned char* dst = stem + ((yr % kSR) * Ws + x) * (kTP * 2);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<uint2*>(dst + (cb * 32 + g * 8 + fh * 4) * 2) =
                make_uint2(stem_pk2(acc[cb][4 * g + 0], acc[cb][4 * g + 1]),
                           stem_pk2(acc[cb][4 * g + 2], acc[cb][4 * g + 3]));
      }
    }
  };

  // ---- prologue: the first band's s2d rows, synchronously (up to 6 rows: 3 per fetch)
  int n = b0 / Hp, P = b0 - (b0 / Hp) * Hp;
  int ys = P > 0 ? 2 * P - 1 : 0;  // first band of the range: the shared row too
  {
    const int lo = ys - 2, hi = min(2 * P + 1, Hs - 1) + 1;  // s2d rows [lo, hi]
    for (int Y = lo; Y <= hi; Y += 3) {
      const int cnt = min(3, hi - Y + 1);
      fetch(n, Y, cnt);
      commit(Y, cnt);
    }
  }
  __syncthreads();

  for (int b = b0; b < b1; ++b) {
    const int ye = min(2 * P + 2, Hs);
    // next band's new s2d rows, into registers while this band's MFMAs run
    const int bn = b + 1;
    int nn = n, nP = P + 1, nlo = 2 * P + 3, ncnt = 2;
    if (nP == Hp) {  // next band starts an image: s2d rows -2 .. 2 (-2, -1 are zero)
      nn = n + 1;
      nP = 0;
      nlo = -2;
      ncnt = 5;
    }
    const bool more = bn < b1;
    // raw loads: data rows only (nlo = -2: rows 0..2 -> fetch (0, 3), zero rows committed
    // from the same call through the range check)
    if (more) fetch(nn, nlo < 0 ? 0 : nlo, nlo < 0 ? 3 : ncnt);
    stem_rows(ys, ye);
    __syncthreads();  // stem rows done; this band's s2d rows no longer read
    if (more) {
      if (nlo < 0) {
        commit(0, 3);
        // zero rows -2, -1: 2 x Ws s2d pixels x 24 B
        for (int i = tid; i < 2 * Ws * 3; i += kNT) {
          const int r = i / (Ws * 3), q = i - r * (Ws * 3);
          *reinterpret_cast<uint2*>(ring + ring6(-2 + r) * RP + 48 + q * 8) = make_uint2(0, 0);
        }
      } else {
        commit(nlo, ncnt);
      }
    }
    // ---- 3x3/2 max pool of pooled row P (stem rows 2P-1 .. 2P+1, clamped) -> global
    {
      const int r0 = max(2 * P - 1, 0) % kSR, r1 = (2 * P) % kSR, r2 = min(2 * P + 1, Hs - 1) % kSR;
      bf16* yrow = y + (long long)(n * Hp + P) * Wp * ldy + y_coff;
      // lane -> (pixel, 16-B chunk): the two 8-lane halves of each 16-lane ds_read_b128 group
      // take pooled pixels p and p + 4, whose window columns are 8 stem pixels apart (1152 B =
      // 32 banks mod 64): the halves hit disjoint banks.  With neighbouring pixels (2 stem
      // pixels = 288 B apart) every pool read was 2-way bank-conflicted.
      for (int q = tid; q < (Wp + 7) / 8 * 64; q += kNT) {
        const int g16 = q >> 4, c8 = q & 7;
        const int px = 8 * (g16 >> 2) + (g16 & 3) + 4 * ((q >> 3) & 1);
        if (px >= Wp) continue;
        const int xs[3] = {max(2 * px - 1, 0), 2 * px, min(2 * px + 1, Ws - 1)};
        const int rs[3] = {r0, r1, r2};
        uint4 v[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            v[dy * 3 + dx] = *reinterpret_cast<const uint4*>(
                stem + ((rs[dy] * Ws + xs[dx]) * kTP + c8 * 8) * 2);
        uint4 m = v[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) {
          m.x = pk_max_i16(m.x, v[k].x);
          m.y = pk_max_i16(m.y, v[k].y);
          m.z = pk_max_i16(m.z, v[k].z);
          m.w = pk_max_i16(m.w, v[k].w);
        }
        m.x = pk_max_i16(m.x, 0u);
        m.y = pk_max_i16(m.y, 0u);
        m.z = pk_max_i16(m.z, 0u);
        m.w = pk_max_i16(m.w, 0u);
        *reinterpret_cast<uint4*>(yrow + px * ldy + c8 * 8) = m;
      }
    }
    __syncthreads();  // pool reads done (stem slots reusable); committed rows visible
    n = nn;
    P = nP;
    ys = 2 * P;
  }
}

}  // namespace
}  // namespace kvedge

using namespace kvedge;

static int stem12_row_pitch(int Ws) { return ((Ws + 4) * 24 + 15) / 16 * 16; }

extern "C" int kv_stem12_lds_bytes(int Ws) {
  return kRing * stem12_row_pitch(Ws) + kSR * Ws * kTP * 2;
}

// frames: uint8 [N, H0, W0, 3] (H0 even, W0 % 4 == 0); w: [64][192] (ops.pack_stem12);
// v = (byte/255 - mean) * inv_std per channel.  y: [N, Hp, Wp, ldy] at channel y_coff.
extern "C" int kv_stem12_pool_frames(const void* frames, const void* w, const float* bias, void* y,
                                     int N, int H0, int W0, const float* mean3,
                                     const float* inv_std3, int ldy, int y_coff, hipStream_t s) {
  if (N <= 0) return 0;
  if (H0 % 2 || W0 % 4 || H0 <= 0 || W0 <= 0 || !bias) return -1;
  if (ldy % 8 || y_coff % 8 || ldy < y_coff + kC) return -1;
  const int Hs = H0 / 2, Ws = W0 / 2;
  const int Hp = (Hs - 1) / 2 + 1, Wp = (Ws - 1) / 2 + 1;
  if (3 * Ws > kNT * kMaxLoads) return -2;  // 3 s2d rows of raw loads per band
  const int lds = kv_stem12_lds_bytes(Ws);
  if (lds > 160 * 1024) return -2;
  if ((long long)N * H0 * W0 * 3 >= 0x7ffffff0LL) return -4;  // 32-bit buffer offsets
  StemNorm12 nrm;
  for (int c = 0; c < 3; ++c) {
    nrm.a[c] = inv_std3[c] / 255.f;
    nrm.b[c] = -mean3[c] * inv_std3[c];
  }
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long long bands = (long long)N * Hp;
  const int per_cu = lds <= 80 * 1024 ? 2 : 1;
  const long long g = bands < (long long)ncu * per_cu ? bands : (long long)ncu * per_cu;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(stem12_pool_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -3;
  hipLaunchKernelGGL(stem12_pool_kernel, dim3((unsigned)g), dim3(kNT), (unsigned)lds, s,
                     (const unsigned char*)frames, (const bf16*)w, bias, (bf16*)y, N, Hs, Ws, Hp,
                     Wp, ldy, y_coff, nrm, stem12_row_pitch(Ws));
  return hipGetLastError() == hipSuccess ? 0 : -100;
}
