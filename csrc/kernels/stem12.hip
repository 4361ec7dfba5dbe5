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
  float4 bv[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      bv[cb][g] = *reinterpret_cast<const float4*>(bias + cb * 32 + g * 8 + fh * 4);
  // loaded once: no waits for them inside the band loop (which has the raw prefetch in flight)
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
    for (int t = 0; t < kKs; ++t) kv_settle(wreg[cb][t]);
#pragma unroll
    for (int g = 0; g < 4; ++g) kv_settle(bv[cb][g]);
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

  // Raw prefetch of s2d rows [Ylo, Ylo + nrows) of image n (rows outside the image and
  // loads past the row count read nothing and commit zeros).
  u32x3 raw[kMaxLoads];
  unsigned okm = 0;
  auto fetch = [&](int n, int Ylo, int nrows) __attribute__((always_inline)) {
    okm = 0;
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      const int q = tid + kNT * i;
      const int j = q / per_row, rem = q - j * per_row;
      const int dy = rem / pairs, k = rem - dy * pairs;
      const int Y = Ylo + j;
      const bool ok = j < nrows && (unsigned)Y < (unsigned)Hs;
      const int off = ok ? (((n * Hs + Y) * 2 + dy) * W0 + 4 * k) * 3 : 0x7ffffff0;
      raw[i] = __builtin_amdgcn_raw_buffer_load_b96(rf, off, 0, 0);
      okm |= ok ? 1u << i : 0u;
    }
  };
  // normalised bf16 of 6 bytes (2 input pixels x rgb) starting at byte `sh` of (lo | hi<<32)
  auto six = [&](unsigned lo, unsigned hi, int sh, bool ok, unsigned out[3]) __attribute__((always_inline)) {
    const unsigned long long v = ((unsigned long long)hi << 32 | lo) >> (8 * sh);
    float f[6];
#pragma unroll
    for (int e = 0; e < 6; ++e)
      f[e] = ok ? (float)((unsigned)(v >> (8 * e)) & 0xffu) * nrm.a[e % 3] + nrm.b[e % 3] : 0.f;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      bf16 p[2] = {f2bf(f[2 * e]), f2bf(f[2 * e + 1])};
      out[e] = __builtin_bit_cast(unsigned, p);
    }
  };
  // write the fetched rows (and zeros for the rows that are outside the image)
  auto commit = [&](int Ylo, int nrows) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      const int q = tid + kNT * i;
      const int j = q / per_row, rem = q - j * per_row;
      if (j >= nrows) continue;
      const int dy = rem / pairs, k = rem - dy * pairs;
      const bool ok = (okm >> i) & 1u;
      unsigned char* row = ring + ring6(Ylo + j) * RP;
      unsigned px0[3], px1[3];
      six(raw[i][0], raw[i][1], 0, ok, px0);  // s2d pixel 2k   (input pixels 4k, 4k+1)
      six(raw[i][1], raw[i][2], 2, ok, px1);  // s2d pixel 2k+1 (input pixels 4k+2, 4k+3)
      unsigned char* p0 = row + (2 * k + 2) * 24 + dy * 12;
      unsigned char* p1 = p0 + 24;
      if (dy == 0) {
        *reinterpret_cast<uint2*>(p0) = make_uint2(px0[0], px0[1]);
        *reinterpret_cast<unsigned*>(p0 + 8) = px0[2];
        *reinterpret_cast<uint2*>(p1) = make_uint2(px1[0], px1[1]);
        *reinterpret_cast<unsigned*>(p1 + 8) = px1[2];
      } else {
        *reinterpret_cast<unsigned*>(p0) = px0[0];
        *reinterpret_cast<uint2*>(p0 + 4) = make_uint2(px0[1], px0[2]);
        *reinterpret_cast<unsigned*>(p1) = px1[0];
        *reinterpret_cast<uint2*>(p1 + 4) = make_uint2(px1[1], px1[2]);
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
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          acc[cb][4 * g + 0] = bv[cb][g].x;
          acc[cb][4 * g + 1] = bv[cb][g].y;
          acc[cb][4 * g + 2] = bv[cb][g].z;
          acc[cb][4 * g + 3] = bv[cb][g].w;
        }
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
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[0][t], af[t % 3], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[1][t], af[t % 3], acc[1], 0, 0, 0);
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
          for (int g = 0; g < 4; ++g) {
            bf16x4 o;
            o[0] = f2bf(acc[cb][4 * g + 0]);
            o[1] = f2bf(acc[cb][4 * g + 1]);
            o[2] = f2bf(acc[cb][4 * g + 2]);
            o[3] = f2bf(acc[cb][4 * g + 3]);
            *reinterpret_cast<bf16x4*>(dst + (cb * 32 + g * 8 + fh * 4) * 2) = o;
          }
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
