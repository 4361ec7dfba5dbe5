// FIXTURE (tests/test_isa_lint.py): csrc/kernels/yolo_stem2.hip as of commit ad7a357, the round-4
// fragment prefetch that produced NaNs at 640x640.  Never built into the library; the ISA lint
// must flag its in-flight register copies.
// YOLOv8n b0 + b1 fused, straight from raw uint8 frames (gfx950):
//   b0: conv 3x3/2 3 -> 16 + SiLU   (run as its 2x2 stride-1 form over the 16-channel
//       space-to-depth image, DeployedConv.stem_s2d(in_scale = 1/255): raw bytes are exact
//       in bf16 and the 1/255 lives in the weights)
//   b1: conv 3x3/2 16 -> 32 + SiLU on b0's output, which never leaves LDS.
//
// Why (profiles/r3_v7_yolov8n_b192_op_roofline.md rows 0-1): b0 wrote a [N, 320, 320, 16]
// bf16 tensor (0.63 GB at batch 192) that b1 read straight back -- 1.26 GB of the two
// layers' 1.8 GB of HBM traffic, 477 us of the 5.7 ms forward.  Fused, the layer pair
// reads the frames once and writes b1's [N, 160, 160, 32] once (0.55 GB).
//
// Structure: persistent, 2 workgroups of 4 waves per CU (<= 80 KB LDS each), each walking a
// contiguous range of (image, b1 output row) bands.  Band yo of image n:
//  * s2d ring (3 rows, 32 B per s2d pixel, one zero column on the left): s2d rows 2yo-1 ..
//    2yo+1.  The next band's two new s2d rows (= 4 frame rows) are loaded as raw bytes into
//    VGPRs at the start of the band and committed after the b0 phase, so the HBM latency
//    hides under the band's MFMAs.
//  * b0 phase: stem rows 2yo, 2yo+1 = 2 x Ws pixels in 16-pixel blocks, two
//    v_mfma_f32_16x16x32_bf16 per block (K = 4 taps x 16 = 64; a lane's 8 K values are 16
//    contiguous bytes: taps (a, 0) and (a, 1) are neighbouring s2d pixels).  16 output
//    channels = the MFMA's 16 columns exactly.  SiLU, bf16 -> stem ring.
//  * stem ring (3 rows): even columns first, then a zero pad slot, then the odd columns,
//    at a 48-B pitch.  b1's stride-2 taps then read neighbouring slots for neighbouring
//    output pixels (conflict-free ds_read_b128, as in conv_direct's stride-2 patches).
//  * b1 phase: one output row = Ws / 2 pixels in 32-pixel blocks, nine
//    v_mfma_f32_32x32x16_bf16 per block (one per tap, 16 channels); SiLU; stores straight
//    from the accumulators (per pixel 4 x 16 B: the four stores fill each 64-B pixel row).
#include <stdlib.h>

#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace kvedge {
namespace {

constexpr int kNT = 256;      // 4 waves
constexpr int kSP = 32;       // s2d ring bytes per pixel (16 bf16 channels)
constexpr int kTP = 48;       // stem ring bytes per slot (16 bf16 + 16 B pad: conflict-free)
constexpr int kMaxLoads = 3;  // raw 12-B loads per thread per band (W0 <= 768)

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ int mod3(int y) { return (y + 3) % 3; }  // y >= -3

__global__ __launch_bounds__(kNT, 2) void yolo_stem2_kernel(
    const unsigned char* __restrict__ frames, const bf16* __restrict__ w0,
    const float* __restrict__ bias0, const bf16* __restrict__ w1, int w1_ld,
    const float* __restrict__ bias1, bf16* __restrict__ y, int N, int Hs, int Ws) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int SR = (Ws + 1) * kSP;        // s2d ring row pitch (pixel -1 = zero column)
  const int half = Ws / 2;              // even (= odd) stem columns per row
  const int TR = (Ws + 1) * kTP;        // stem ring row pitch: E[0..half) | pad | O[0..half)
  unsigned char* sring = lds;
  unsigned char* tring = lds + 3 * SR;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H1 = Hs / 2, W1 = Ws / 2;
  const int W0 = 2 * Ws;

  // ---- weights -> VGPRs once
  // b0 (16x16x32): B fragment lane = (cout lane & 15, k quarter lane >> 4), 2 k-steps
  const int q16 = lane & 15, kq = lane >> 4;
  bf16x8 w0r[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    w0r[t] = *reinterpret_cast<const bf16x8*>(w0 + q16 * 64 + t * 32 + kq * 8);
  float4 b0v = *reinterpret_cast<const float4*>(bias0 + kq * 4);
  // b1 (32x32x16): lane = (cout lane & 31, k half lane >> 5), 9 taps of 16 channels
  const int fr = lane & 31, fh = lane >> 5;
  bf16x8 w1r[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
    w1r[t] = *reinterpret_cast<const bf16x8*>(w1 + fr * w1_ld + t * 16 + fh * 8);
  float4 b1v[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) b1v[g] = *reinterpret_cast<const float4*>(bias1 + g * 8 + fh * 4);
  // loaded once: no waits for them inside the band loop (which has the raw prefetch in flight)
  kv_settle(w0r[0]);
  kv_settle(w0r[1]);
  kv_settle(b0v);
#pragma unroll
  for (int t = 0; t < 9; ++t) kv_settle(w1r[t]);
#pragma unroll
  for (int g = 0; g < 4; ++g) kv_settle(b1v[g]);

  // ---- zero column (s2d pixel -1) of every s2d ring row; stem pad slot of every stem row
  for (int i = tid; i < 3 * 2; i += kNT)
    *reinterpret_cast<uint4*>(sring + (i >> 1) * SR + (i & 1) * 16) = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < 3 * 3; i += kNT)
    *reinterpret_cast<uint4*>(tring + (i / 3) * TR + half * kTP + (i % 3) * 16) =
        make_uint4(0, 0, 0, 0);

  const int total = N * H1;
  const int per = (total + gridDim.x - 1) / gridDim.x;
  const int bb = blockIdx.x * per, be = min(bb + per, total);
  if (bb >= be) return;  // uniform per workgroup

  const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(frames), (short)0, N * Hs * 2 * W0 * 3, 0x00020000);
  const int upr = W0 / 4;        // 12-B units per frame row (4 frame pixels = 2 s2d pixels)
  const int ups = 2 * upr;       // units per s2d row (two frame rows)

  // raw fetch of s2d rows [Y0, Y0 + nrows) of image n (rows outside [0, Hs) load nothing)
  u32x3 raw[kMaxLoads];
  unsigned okm = 0;
  auto fetch = [&](int n, int Y0, int nrows) __attribute__((always_inline)) {
    okm = 0;
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      const int u = tid + kNT * i;
      const int j = u / ups, rem = u - j * ups;
      const int dy = rem / upr, k = rem - dy * upr;
      const int Y = Y0 + j;
      const bool ok = j < nrows && (unsigned)Y < (unsigned)Hs;
      const int off = ok ? (((n * Hs + Y) * 2 + dy) * W0 + 4 * k) * 3 : 0x7ffffff0;
      raw[i] = __builtin_amdgcn_raw_buffer_load_b96(rf, off, 0, 0);
      okm |= ok ? 1u << i : 0u;
    }
  };
  // s2d pixel (dy row part): channels dy*8 + dx*4 + c = byte (dx*3 + c) of the 6-byte group
  auto commit = [&](int Y0, int nrows) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kMaxLoads; ++i) {
      const int u = tid + kNT * i;
      const int j = u / ups, rem = u - j * ups;
      if (j >= nrows) continue;
      const int dy = rem / upr, k = rem - dy * upr;
      const bool ok = (okm >> i) & 1u;
      const unsigned long long lo = ((unsigned long long)raw[i][1] << 32) | raw[i][0];
      const unsigned hi = raw[i][2];
      auto bf = [](unsigned byte) { return __float_as_uint((float)byte) >> 16; };
      unsigned char* row = sring + mod3(Y0 + j) * SR;
#pragma unroll
      for (int p = 0; p < 2; ++p) {  // s2d pixels 2k, 2k+1: bytes 6p .. 6p+5
        unsigned b[6];
#pragma unroll
        for (int e = 0; e < 6; ++e) {
          const int at = 6 * p + e;
          b[e] = at < 8 ? (unsigned)(lo >> (8 * at)) & 0xffu : (hi >> (8 * (at - 8))) & 0xffu;
        }
        const uint4 v = ok ? make_uint4(bf(b[0]) | (bf(b[1]) << 16), bf(b[2]),
                                        bf(b[3]) | (bf(b[4]) << 16), bf(b[5]))
                           : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(row + (2 * k + p + 1) * kSP + dy * 16) = v;
      }
    }
  };

  // ---- b0: stem rows [s0, s0 + nr) from the s2d ring -> stem ring (all 4 waves)
  // Per row, blocks b = wv, wv + 4, ... (Ws / 16 per row): the row, its ring slots and the
  // block's column base are wave-uniform (scalar), the lane parts are constants -- no
  // per-block integer divide (it was a third of the phase's VALU, PMC:
  // profiles/r3_v10_pmc_yolo_stem2_b192.txt).
  const int bpr = Ws / 16;
  const int lslot = (q16 & 1) ? half + 1 + (q16 >> 1) : (q16 >> 1);  // stem slot of column q16
  auto stem_rows = [&](int s0, int nr) __attribute__((always_inline)) {
    for (int rl = 0; rl < nr; ++rl) {
      const int sy = s0 + rl;
      const unsigned char* sa0 = sring + mod3(sy - 1) * SR + q16 * kSP + kq * 16;  // pixel sx-1
      const unsigned char* sa1 = sring + mod3(sy) * SR + q16 * kSP + kq * 16;
      unsigned char* td = tring + mod3(sy) * TR + lslot * kTP + kq * 8;
      // the next block's two fragments are read (asm, common.h) before this block's MFMAs:
      // one block of latency ahead instead of an lgkmcnt(0) in front of every MFMA pair
      // (tools/isa_lint.py: 80 % of this kernel's MFMAs)
      const unsigned la0 = lds_addr(sa0), la1 = lds_addr(sa1);
      bf16x8 n0, n1;
      if (wv < bpr) {
        lds_read16<0>(n0, la0 + wv * 16 * kSP);
        lds_read16<0>(n1, la1 + wv * 16 * kSP);
      }
      for (int b = wv; b < bpr; b += 4) {
        floatx4 acc = {b0v.x, b0v.y, b0v.z, b0v.w};
        bf16x8 a0 = n0, a1 = n1;
        if (b + 4 < bpr) {
          lds_read16<0>(n0, la0 + (b + 4) * 16 * kSP);
          lds_read16<0>(n1, la1 + (b + 4) * 16 * kSP);
          lds_wait<2>(a0);  // this block's pair landed; the next pair stays in flight
        } else {
          lds_wait<0>(a0);
        }
        asm volatile("" : "+v"(a1));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0r[0], a0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0r[1], a1, acc, 0, 0, 0);
        // lane holds channels kq*4 .. +3 of stem pixel (sy, 16 b + q16)
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(act_c<kActSilu>(acc[e]));
        *reinterpret_cast<bf16x4*>(td + b * 8 * kTP) = o;
      }
    }
  };

  // ---- b1: output row yo of image n from stem rows 2yo-1 .. 2yo+1 -> global
  auto b1_row = [&](int n, int yo) __attribute__((always_inline)) {
    const int nblk = (W1 + 31) / 32;
    unsigned rowl[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) rowl[r] = lds_addr(tring + mod3(2 * yo - 1 + r) * TR + fh * 16);
    // the 9 tap fragments of a block, read (asm) one block ahead of its MFMAs
    // tap s: stem column 2xo - 1 + s -> s = 0: odd xo-1 (pad slot when xo = 0), s = 1: even
    // xo, s = 2: odd xo
    auto rd9 = [&](bf16x8 (&f)[9], int blk) __attribute__((always_inline)) {
      const int xo = min(blk * 32 + fr, W1 - 1);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        lds_read16<0>(f[3 * r + 0], rowl[r] + (half + xo) * kTP);
        lds_read16<0>(f[3 * r + 1], rowl[r] + xo * kTP);
        lds_read16<0>(f[3 * r + 2], rowl[r] + (half + 1 + xo) * kTP);
      }
    };
    bf16x8 nf[9];
    if (wv < nblk) rd9(nf, wv);
    for (int blk = wv; blk < nblk; blk += 4) {
      const int xo = min(blk * 32 + fr, W1 - 1);
      floatx16 acc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc[4 * g + 0] = b1v[g].x;
        acc[4 * g + 1] = b1v[g].y;
        acc[4 * g + 2] = b1v[g].z;
        acc[4 * g + 3] = b1v[g].w;
      }
      bf16x8 af[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) af[t] = nf[t];
      if (blk + 4 < nblk) {
        rd9(nf, blk + 4);
        lds_wait<9>(af[0]);  // this block's 9 landed; the next block's 9 stay in flight
      } else {
        lds_wait<0>(af[0]);
      }
#pragma unroll
      for (int t = 1; t < 9; ++t) asm volatile("" : "+v"(af[t]));
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1r[t], af[t], acc, 0, 0, 0);
      if (blk * 32 + fr < W1) {
        bf16* dst = y + ((long long)(n * H1 + yo) * W1 + xo) * 32 + fh * 4;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(act_c<kActSilu>(acc[4 * g + e]));
          *reinterpret_cast<bf16x4*>(dst + g * 8) = o;
        }
      }
    }
  };

  auto zero_row = [&](unsigned char* base, int bytes) __attribute__((always_inline)) {
    for (int i = tid; i < bytes / 16; i += kNT)
      *reinterpret_cast<uint4*>(base + i * 16) = make_uint4(0, 0, 0, 0);
  };

  // ---- prologue: ring state for the first band (image n, row yo)
  int n = bb / H1, yo = bb - (bb / H1) * H1;
  if (yo == 0) {
    zero_row(sring + mod3(-1) * SR + kSP, Ws * kSP);  // s2d row -1
    fetch(n, 0, 2);
    commit(0, 2);
  } else {
    // stem row 2yo-1 needs s2d rows 2yo-2, 2yo-1; the band's own stem rows need 2yo-1..2yo+1
    fetch(n, 2 * yo - 2, 2);
    commit(2 * yo - 2, 2);
    __syncthreads();
    stem_rows(2 * yo - 1, 1);
    __syncthreads();  // s2d row 2yo-2 no longer read: its slot takes row 2yo+1
    fetch(n, 2 * yo, 2);
    commit(2 * yo, 2);
  }
  __syncthreads();

  for (int b = bb; b < be; ++b) {
    // stem row 2yo-1 = zero at an image start (its slot is not written by this band)
    if (yo == 0) zero_row(tring + mod3(-1) * TR, TR);
    const bool more = b + 1 < be;
    const int nn = yo + 1 < H1 ? n : n + 1;
    const int nyo = yo + 1 < H1 ? yo + 1 : 0;
    // next band's new s2d rows (2 nyo, 2 nyo + 1): raw bytes in flight during this band
    if (more) fetch(nn, 2 * nyo, 2);
    stem_rows(2 * yo, 2);
    __syncthreads();  // stem rows written; s2d rows of this band no longer read
    if (more) {
      if (nyo == 0) zero_row(sring + mod3(-1) * SR + kSP, Ws * kSP);
      commit(2 * nyo, 2);
    }
    b1_row(n, yo);
    __syncthreads();  // stem ring free for the next band; committed s2d rows visible
    n = nn;
    yo = nyo;
  }
}

}  // namespace
}  // namespace kvedge

using namespace kvedge;

extern "C" int kv_yolo_stem2_lds_bytes(int Ws) { return 3 * (Ws + 1) * (kSP + kTP); }

// frames uint8 [N, H0, W0, 3] (H0 % 4 == 0, W0 % 32 == 0, W0 <= 640); w0 [16][64] (the
// frames-in s2d stem, in_scale 1/255 folded); w1 [32][w1_ld] (3x3 16 -> 32, k-order r, s, c);
// y [N, H0/4, W0/4, 32].
extern "C" int kv_yolo_stem2(const void* frames, const void* w0, const float* bias0, const void* w1,
                             int w1_ld, const float* bias1, void* y, int N, int H0, int W0,
                             hipStream_t s) {
  if (N <= 0) return 0;
  if (H0 % 4 || W0 % 32 || W0 > 640 || H0 <= 0 || !bias0 || !bias1 || w1_ld < 144) return -1;
  const int Hs = H0 / 2, Ws = W0 / 2;
  if ((long long)N * H0 * W0 * 3 >= 0x7ffffff0ll) return -9;
  const int lds = kv_yolo_stem2_lds_bytes(Ws);
  if (lds > 80 * 1024) return -11;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long long bands = (long long)N * (Hs / 2);
  const long long slots = 2ll * ncu;
  const unsigned g = (unsigned)(bands < slots ? bands : slots);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(yolo_stem2_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(yolo_stem2_kernel, dim3(g), dim3(kNT), (unsigned)lds, s,
                     (const unsigned char*)frames, (const bf16*)w0, bias0, (const bf16*)w1, w1_ld,
                     bias1, (bf16*)y, N, Hs, Ws);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
