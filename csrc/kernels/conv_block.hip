// Fused ResNet bottleneck body for the 64-wide stage (gfx950): 3x3 conv2 -> 1x1 conv3
// (+ residual, or + the fused 1x1 downsample) -> the NEXT block's 1x1 conv1, one kernel.
//
// Where it sits.  After the v3 fused tail (conv_stream.hip: conv3 + residual -> next conv1,
// y written once) a layer-1 bottleneck at batch 640 is two kernels: the v4 direct 3x3
// (176 us, conv_direct.hip) writes its 64-channel output c2 (257 MB) and the tail reads it
// back (profiles/r2_v6_resnet50_b640_forward.md).  That round trip is the HBM write and
// re-read of the 64-channel intermediate that VERDICT r1 item 4 asks to kill.  Here c2
// never leaves the chip: each 64-pixel tile's 3x3 output goes from the accumulators into
// LDS, and the conv3 GEMM reads it from there.
//
// Per image row (tile = one row of W <= 64 pixels; a persistent workgroup of 4 waves, one
// per CU, walks a contiguous range of rows):
//  * a rolling window of three input rows of t (the conv1 output) sits in LDS at a 144-B
//    pixel pitch (conflict-free 16-B fragment reads, as v4); each tile brings ONE new row,
//    prefetched into VGPRs a whole tile ahead (an image's first row brings two);
//  * 3x3: 9 taps x 4 k-steps of v_mfma_f32_32x32x16_bf16 per 32 x 32 block, the weights of a
//    wave's 32 output channels held in 144 VGPRs for the whole kernel;
//  * c2 = ReLU(. + b2) -> bf16 tile in LDS; conv3 (| the downsample source row, also in LDS)
//    against the resident conv3 weights; then the v3 tail epilogue: bias + residual + ReLU, y
//    stored in 16-B chunks and kept in LDS, z = ReLU(y . W1^T + b1) from LDS, z stored;
//  * the next row's residual is loaded right after this row's stores, so it has the whole
//    next tile to land; every wait is an exact s_waitcnt vmcnt over (prefetch loads, stores,
//    residual loads).
// Bytes per pixel: t 128 + residual 512 + y 512 + z 128..256.  Measured (batch 640,
// profiles/r2_v8_block_probe.md): level with or slower than direct + tail -- with one
// workgroup per CU (LDS 123-157 KB) the 3x3 phase and the memory phase of a row cannot
// overlap.  Opt-in: KvResNet50.fuse_block.
#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace kvedge {
namespace {

constexpr int kBM = 64;            // pixels per tile
constexpr int kBN = 256;           // conv3 output channels (= y row)
constexpr int kBK = 64;            // K per resident weight block
constexpr int kC2 = 64;            // bottleneck width (3x3 in/out channels)
constexpr int kNT = 256;           // 4 waves, 2 x 2
constexpr int kCS = kBN + 8;       // y tile pitch (elements)
constexpr int kCS2 = kC2 + 8;      // c2 tile pitch (elements): 144 B
constexpr int kPER = kBM * (kBN / 8) / kNT;  // 16-B y / residual chunks per thread (8)
constexpr int kOOB = 0x7ffffff0;
constexpr int kLdsMax = 160 * 1024;
// s_waitcnt immediate (gfx9 encoding): vmcnt 0, expcnt 7 and lgkmcnt 15 (no wait on those)
constexpr int kVmcnt0 = 0x0F70;

constexpr int kRowPx = 66;          // input row buffer: 64 output px + 2 halo columns (W <= 64)
constexpr int kPB = kC2 * 2 + 16;    // 144-B pixel pitch: 16 consecutive pixels' 16-B reads hit
                                     // all 64 banks once (conflict-free, as conv_direct.hip)
constexpr int kRowB = kRowPx * kPB;  // bytes per row buffer
constexpr int kRowCh = 2;            // 16-B chunks of one input row per thread (64 px x 8 / 256)

__host__ __device__ constexpr int block_lds_bytes(bool dual, int nt1) {
  return 3 * kRowB + 2 * ((dual ? 2 : 1) * kBN * kBK + kBM * kCS + nt1 * kBN);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t rs, bf16* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void bwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}

// chunk swizzle of resident-weight rows (as v2/v3): 16-B chunk c of row r at c ^ sw(r)
__device__ __forceinline__ int bsw(int r) { return (r >> 1) & 7; }

template <int NT1, bool DUAL>
__global__ __launch_bounds__(kNT, 1) void conv_block_kernel(const KvBlockParams p, int rows_per_wg) {
  constexpr int KM = DUAL ? 2 : 1;          // resident conv3 K blocks: c2 [| downsample]
  constexpr int PERZ = kBM * NT1 / 8 / kNT; // 16-B z chunks per thread
  constexpr int NPF = 2 * kRowCh + (DUAL ? kRowCh : 0);  // prefetch loads per thread per tile
  constexpr int RI = DUAL ? 0 : kPER;       // residual loads per thread per tile
  constexpr int EPI = kPER + PERZ;          // stores per thread per tile
  constexpr int TN = 4;                     // conv3: 32 px x 128 ch per wave
  constexpr int TN1 = NT1 / 64;             // tail: 32 px x NT1/2 ch per wave
  static_assert(NT1 == 64 || NT1 == 128, "tail width");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* const rows = lds;                                   // 3 x kRowB
  bf16* const Bres = reinterpret_cast<bf16*>(lds + 3 * kRowB);       // [KM][kBN][kBK] swizzled
  bf16* const Cs = Bres + KM * kBN * kBK;   // y tile [kBM][kCS]; c2 tile + x2 row alias it
  bf16* const W1s = Cs + kBM * kCS;         // [kBN / 64][NT1][64] swizzled blocks
  bf16* const X2s = Cs + kBM * kCS2;        // dual: this row's downsample source [64][kCS2]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv >> 1, wn = wv & 1;
  const int fr = lane & 31, fh = lane >> 5;
  const int H = p.H, W = p.W;
  const int NR = p.N * H;                   // tiles = image rows
  const int M = NR * W;
  const int q0 = blockIdx.x * rows_per_wg;
  const int q1 = min(q0 + rows_per_wg, NR);
  if (q0 >= q1) return;

  const __amdgpu_buffer_rsrc_t rt = brsrc(p.t, M * kC2 * 2);
  const __amdgpu_buffer_rsrc_t rx2 = brsrc(DUAL ? p.x2 : p.t, DUAL ? M * kC2 * 2 : 0);
  const __amdgpu_buffer_rsrc_t rr = brsrc(DUAL ? p.t : p.res, DUAL ? 0 : M * kBN * 2);
  const __amdgpu_buffer_rsrc_t ry = brsrc(p.y, M * kBN * 2);
  const __amdgpu_buffer_rsrc_t rz = brsrc(p.z, M * NT1 * 2);

  // ---- resident data, once: 3x3 weights (VGPRs), conv3 | downsample and tail weights (LDS)
  const bf16* w2 = reinterpret_cast<const bf16*>(p.w2);
  bf16x8 w2reg[36];  // rows wn*32 + fr, k = kk*16 + fh*8 (k = tap * 64 + c)
#pragma unroll
  for (int kk = 0; kk < 36; ++kk)
    w2reg[kk] = *reinterpret_cast<const bf16x8*>(w2 + (wn * 32 + fr) * 576 + kk * 16 + fh * 8);
  const int lrow = lane >> 3, pch = lane & 7;
  {
    const __amdgpu_buffer_rsrc_t rw3 = brsrc(p.w3, kBN * KM * kBK * 2);
#pragma unroll
    for (int kb = 0; kb < KM; ++kb)
#pragma unroll
      for (int i = 0; i < kBN / 32; ++i) {  // 8 rows per DMA, 4 waves
        const int row = (wv * (kBN / 32) + i) * 8 + lrow;
        bdma16(rw3, Bres + kb * kBN * kBK + (wv * (kBN / 32) + i) * 512,
               (row * KM * kBK + kb * kBK + (pch ^ bsw(row)) * 8) * 2);
      }
    const __amdgpu_buffer_rsrc_t rw1 = brsrc(p.w1, NT1 * kBN * 2);
#pragma unroll
    for (int kt = 0; kt < kBN / kBK; ++kt)
#pragma unroll
      for (int i = 0; i < NT1 / 32; ++i) {
        const int row = (wv * (NT1 / 32) + i) * 8 + lrow;
        bdma16(rw1, W1s + kt * NT1 * kBK + (wv * (NT1 / 32) + i) * 512,
               (row * kBN + kt * kBK + (pch ^ bsw(row)) * 8) * 2);
      }
  }
  // biases in registers (an LDS read in the epilogue would wait on the in-flight DMA)
  float4 b2r[4], b3r[TN][4], b1r[TN1][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) b2r[g] = *reinterpret_cast<const float4*>(p.b2 + wn * 32 + g * 8 + fh * 4);
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      b3r[tn][g] = *reinterpret_cast<const float4*>(p.b3 + wn * 128 + tn * 32 + g * 8 + fh * 4);
#pragma unroll
  for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      b1r[tn][g] = *reinterpret_cast<const float4*>(p.b1 + wn * (NT1 / 2) + tn * 32 + g * 8 + fh * 4);
  // zero padding columns of the three row buffers: column 0 (left pad) and W+1 .. 65
  {
    const int ncol = 1 + (kRowPx - 1 - W);
    for (int c = tid; c < 3 * ncol * (kPB / 16); c += kNT) {
      const int b = c / (ncol * (kPB / 16)), rem = c % (ncol * (kPB / 16));
      const int ci = rem / (kPB / 16), ch = rem % (kPB / 16);
      const int col = ci == 0 ? 0 : W + ci;
      *reinterpret_cast<uint4*>(rows + b * kRowB + col * kPB + ch * 16) = make_uint4(0u, 0u, 0u, 0u);
    }
  }

  // ---- input rows: row r of image img -> buffer (r + 3) % 3, columns 1 .. W --------------
  // prefetch of tile q's new rows into VGPRs (kRowCh 16-B chunks per thread per row): a
  // continuing tile needs row h+1, an image's first row needs rows 0 and 1 (row -1 = zeros)
  uint4 pre[2 * kRowCh], prex[DUAL ? kRowCh : 1];
  auto load_row = [&](int img, int r, uint4* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kRowCh; ++j) {
      const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
      const int off = (px < W && (unsigned)r < (unsigned)H) ? (((img * H + r) * W + px) * kC2 + ch * 8) * 2 : kOOB;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rt, off, 0, 0);
      dst[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto prefetch = [&](int q) __attribute__((always_inline)) {  // always NPF loads
    const bool live = q < q1;
    const int img = live ? q / H : 0, h = live ? q - img * H : 0;
    load_row(live ? img : 0, live ? (h == 0 ? 0 : h + 1) : -1, pre);
    load_row(live ? img : 0, live && h == 0 ? 1 : -1, pre + kRowCh);
    if constexpr (DUAL) {
#pragma unroll
      for (int j = 0; j < kRowCh; ++j) {
        const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
        const int off = (live && px < W) ? ((q * W + px) * kC2 + ch * 8) * 2 : kOOB;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx2, off, 0, 0);
        prex[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto put_row = [&](int buf, const uint4* src) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kRowCh; ++j) {
      const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
      if (px < W) *reinterpret_cast<uint4*>(rows + buf * kRowB + (px + 1) * kPB + ch * 16) = src[j];
    }
  };
  auto commit = [&](int q) __attribute__((always_inline)) {
    const int img = q / H, h = q - img * H;
    if (h == 0) {
      const uint4 zz = make_uint4(0u, 0u, 0u, 0u);
      const uint4 zr[kRowCh] = {};
      (void)zz;
      put_row(0, pre);
      put_row(1, pre + kRowCh);
      put_row(2, zr);  // row -1
    } else {
      put_row((h + 1) % 3, pre);
    }
    if constexpr (DUAL) {
#pragma unroll
      for (int j = 0; j < kRowCh; ++j) {
        const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
        if (px < W) *reinterpret_cast<uint4*>(X2s + px * kCS2 + ch * 8) = prex[j];
      }
    }
  };
  u32x4 rres[DUAL ? 1 : kPER];
  auto load_res = [&](int q) __attribute__((always_inline)) {
    if constexpr (!DUAL) {
#pragma unroll
      for (int j = 0; j < kPER; ++j) {
        const int idx = tid + kNT * j;
        const int px = idx / (kBN / 8), n = (idx % (kBN / 8)) * 8;
        const int off = (q < q1 && px < W) ? ((q * W + px) * kBN + n) * 2 : kOOB;
        rres[j] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
      }
    }
  };

  // the first tile's window, synchronously: rows h-1, h, h+1 (and its x2 row)
  {
    const int img = q0 / H, h = q0 - img * H;
    load_row(img, h - 1, pre);
    load_row(img, h, pre + kRowCh);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    put_row((h + 2) % 3, pre);
    put_row(h % 3, pre + kRowCh);
    load_row(img, h + 1, pre);
    if constexpr (DUAL) {
#pragma unroll
      for (int j = 0; j < kRowCh; ++j) {
        const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
        const int off = px < W ? ((q0 * W + px) * kC2 + ch * 8) * 2 : kOOB;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx2, off, 0, 0);
        prex[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    put_row((h + 1) % 3, pre);
    if constexpr (DUAL) {
#pragma unroll
      for (int j = 0; j < kRowCh; ++j) {
        const int c = tid + kNT * j, px = c >> 3, ch = c & 7;
        if (px < W) *reinterpret_cast<uint4*>(X2s + px * kCS2 + ch * 8) = prex[j];
      }
    }
  }
  // resident weights, biases and the first window landed (this wave).  The builtin, not
  // inline asm: the compiler's wait-count pass must SEE this wait, or it keeps the
  // pre-loop weight/bias loads "pending" and re-inserts a near-full vmcnt wait before
  // their uses inside the loop
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
  load_res(q0);

  floatx16 acc2;      // 3x3: 32 px x 32 ch per wave
  floatx16 acc[TN];   // conv3: 32 px x 128 ch per wave
  auto bres_frag = [&](int kb, int tn, int ks) __attribute__((always_inline)) {
    const int row = wn * 128 + tn * 32 + fr, q = ks * 2 + fh;
    return *reinterpret_cast<const bf16x8*>(Bres + kb * kBN * kBK + row * kBK + ((q ^ bsw(row)) << 3));
  };

  for (int q = q0; q < q1; ++q) {
    const int img = q / H, h = q - img * H;
    if (q > q0) {
      // tile q's rows were prefetched at the top of tile q-1; issued after them: tile q-1's
      // stores and tile q's residual loads
      bwait_vm<EPI + RI>();
      commit(q);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // window (and x2 row) visible to every wave
    asm volatile("" ::: "memory");
    prefetch(q + 1);

    // ---- 3x3: 9 taps x 4 k16 steps, A from the three row buffers (144-B pixel pitch)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc2[e] = 0.f;
    const unsigned char* rb[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) rb[r] = rows + ((h + r + 2) % 3) * kRowB + (wm * 32 + fr) * kPB + fh * 16;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      bf16x8 af[12];
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          af[s * 4 + ks] = *reinterpret_cast<const bf16x8*>(rb[r] + s * kPB + ks * 32);
#pragma unroll
      for (int k = 0; k < 12; ++k)
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2reg[r * 12 + k], af[k], acc2, 0, 0, 0);
    }
    // ---- c2 = ReLU(acc2 + b2) -> Cs as [64 px][kCS2]
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 o;
      o[0] = f2bf(fmaxf(acc2[4 * g + 0] + b2r[g].x, 0.f));
      o[1] = f2bf(fmaxf(acc2[4 * g + 1] + b2r[g].y, 0.f));
      o[2] = f2bf(fmaxf(acc2[4 * g + 2] + b2r[g].z, 0.f));
      o[3] = f2bf(fmaxf(acc2[4 * g + 3] + b2r[g].w, 0.f));
      *reinterpret_cast<bf16x4*>(Cs + (wm * 32 + fr) * kCS2 + wn * 32 + g * 8 + fh * 4) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // ---- conv3 over c2 (| the downsample source), A from LDS (144-B pitch), B resident
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[tn][e] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KM; ++kb)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16* src = kb == 0 ? Cs : X2s;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(src + (wm * 32 + fr) * kCS2 + ks * 16 + fh * 8);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bres_frag(kb, tn, ks), af, acc[tn], 0, 0, 0);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave done with c2 / x2: Cs takes the y tile
    asm volatile("" ::: "memory");
    // ---- y = ReLU(acc + b3 [+ res]) staged through Cs for full-row 16-B stores
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * 128 + tn * 32 + g * 8 + fh * 4;
        const float4 bv = b3r[tn][g];
        bf16x4 o;
        if constexpr (DUAL) {  // ReLU now (no residual)
          o[0] = f2bf(fmaxf(acc[tn][4 * g + 0] + bv.x, 0.f));
          o[1] = f2bf(fmaxf(acc[tn][4 * g + 1] + bv.y, 0.f));
          o[2] = f2bf(fmaxf(acc[tn][4 * g + 2] + bv.z, 0.f));
          o[3] = f2bf(fmaxf(acc[tn][4 * g + 3] + bv.w, 0.f));
        } else {  // ReLU after the residual add
          o[0] = f2bf(acc[tn][4 * g + 0] + bv.x);
          o[1] = f2bf(acc[tn][4 * g + 1] + bv.y);
          o[2] = f2bf(acc[tn][4 * g + 2] + bv.z);
          o[3] = f2bf(acc[tn][4 * g + 3] + bv.w);
        }
        *reinterpret_cast<bf16x4*>(Cs + (wm * 32 + fr) * kCS + nl) = o;
      }
    // the residual was loaded at the end of the previous tile (before the loop for the
    // first); issued after it: this tile's NPF prefetch loads
    if constexpr (!DUAL) bwait_vm<NPF>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int m0 = q * W;
#pragma unroll
    for (int j = 0; j < kPER; ++j) {
      const int idx = tid + kNT * j;
      const int ml = idx / (kBN / 8), ch = idx % (kBN / 8);
      bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + ml * kCS + ch * 8);
      if constexpr (!DUAL) {
        const bf16x8 rv = __builtin_bit_cast(bf16x8, rres[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e] + (float)rv[e], 0.f));
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry,
                                             ml < W ? ((m0 + ml) * kBN + ch * 8) * 2 : kOOB, 0, 0);
      if constexpr (!DUAL) *reinterpret_cast<bf16x8*>(Cs + ml * kCS + ch * 8) = v;
    }
    // ---- next block's conv1: z = ReLU(y . W1^T + b1), 32 px x NT1/2 ch per wave
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // y tile complete in Cs
    asm volatile("" ::: "memory");
    floatx16 accz[TN1];
#pragma unroll
    for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        accz[tn][4 * g + 0] = b1r[tn][g].x;
        accz[tn][4 * g + 1] = b1r[tn][g].y;
        accz[tn][4 * g + 2] = b1r[tn][g].z;
        accz[tn][4 * g + 3] = b1r[tn][g].w;
      }
#pragma unroll
    for (int kk = 0; kk < kBN / 16; ++kk) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(Cs + (wm * 32 + fr) * kCS + kk * 16 + fh * 8);
      const int kt = kk >> 2, qq = (kk & 3) * 2 + fh;
#pragma unroll
      for (int tn = 0; tn < TN1; ++tn) {
        const int row = wn * (NT1 / 2) + tn * 32 + fr;
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(W1s + kt * NT1 * kBK + row * kBK + ((qq ^ bsw(row)) << 3));
        accz[tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, accz[tn], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave done reading the y tile: Cs takes z
    asm volatile("" ::: "memory");
    constexpr int CZ = NT1 + 8;
#pragma unroll
    for (int tn = 0; tn < TN1; ++tn)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * (NT1 / 2) + tn * 32 + g * 8 + fh * 4;
        bf16x4 o;
        o[0] = f2bf(fmaxf(accz[tn][4 * g + 0], 0.f));
        o[1] = f2bf(fmaxf(accz[tn][4 * g + 1], 0.f));
        o[2] = f2bf(fmaxf(accz[tn][4 * g + 2], 0.f));
        o[3] = f2bf(fmaxf(accz[tn][4 * g + 3], 0.f));
        *reinterpret_cast<bf16x4*>(Cs + (wm * 32 + fr) * CZ + nl) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < PERZ; ++j) {
      const int idx = tid + kNT * j;
      const int ml = idx / (NT1 / 8), ch = idx % (NT1 / 8);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + ml * CZ + ch * 8);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rz,
                                             ml < W ? ((m0 + ml) * NT1 + ch * 8) * 2 : kOOB, 0, 0);
    }
    // every wave done reading Cs (the next tile's commit writes its x2 row there) and the
    // next tile's residual, issued behind this tile's stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    load_res(q + 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

typedef void (*BlockFn)(const KvBlockParams, int);

}  // namespace
}  // namespace kvedge

using namespace kvedge;

extern "C" int kv_conv_block(const KvBlockParams* p, hipStream_t stream) {
  if (!p || !p->t || !p->w2 || !p->b2 || !p->w3 || !p->b3 || !p->y || !p->w1 || !p->b1 || !p->z)
    return -1;
  const bool dual = p->x2 != nullptr;
  if (dual == (p->res != nullptr)) return -2;  // exactly one of residual / downsample source
  if (p->nt != 64 && p->nt != 128) return -3;
  if (p->W < 1 || p->W > 64 || p->H < 1) return -4;  // one image row per 64-pixel tile
  const long long M = (long long)p->N * p->H * p->W;
  if (M <= 0) return 0;
  if (M * kBN * 2 >= kOOB) return -9;  // 32-bit buffer offsets
  const int lds = block_lds_bytes(dual, p->nt);
  if (lds > kLdsMax) return -11;
  BlockFn fn = p->nt == 64 ? (dual ? conv_block_kernel<64, true> : conv_block_kernel<64, false>)
                           : (dual ? conv_block_kernel<128, true> : conv_block_kernel<128, false>);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // persistent: one workgroup per CU walks a contiguous range of image rows (the 3-row
  // window then slides by one row per tile)
  const long long nrows = (long long)p->N * p->H;
  const long long g = nrows < ncu ? nrows : ncu;
  const int per = (int)((nrows + g - 1) / g);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return -7;
  hipLaunchKernelGGL(fn, dim3((unsigned)((nrows + per - 1) / per)), dim3(kNT), (unsigned)lds,
                     stream, *p, per);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

extern "C" int kv_conv_block_lds_bytes(int dual, int nt) { return block_lds_bytes(dual != 0, nt); }
