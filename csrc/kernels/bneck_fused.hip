// v11 -- fused identity bottleneck: y = ReLU(W3 . ReLU(conv3x3(ReLU(W1 . x + b1)) + b2) + b3 + x)
// in ONE launch, the two intermediate activations kept in LDS (gfx950).
//
// Why (round 5, profiles/r5_*_graph_layers*.md): ResNet-50 stages 2 and 3 ran every identity
// block as a 3x3 launch plus a seam launch (conv3 + residual -> next conv1).  Per block and
// 640-image slice that moved z1 + z2 + z2 + x + y + z1' through HBM (stage 3: 3072 channel-
// bytes per pixel) at 0.3-0.5 of the per-kernel floors (3x3 160-230 us, seam 230-390 us),
// while the block's MFMA work is only ~280 GFLOP (113 us at the 2.5 PF dense peak).  Here a
// workgroup owns an image's row band end to end: x is read once (plus its residual re-read,
// mostly from the MALL), y is written once, nothing else touches HBM.
//
// Work split: one 4-wave workgroup (one wave per SIMD, 512-VGPR budget) per band of R output
// rows of one image (stage 3, 14x14x256: the whole image; stage 2, 28x28x128: 7 rows).
//   phase 1  z1 = ReLU(W1 . x^T + b1) over the band's rows AND its 1-row halo (recomputed:
//            +2/R of conv1): x streams through a 6-slot LDS ring of 32-channel chunks (LDS
//            DMA, 5 chunks ahead; piece-swizzled so the fragment reads are conflict-free);
//            z1 lands in LDS as a zero-padded (R+2) x (W+2) pixel image, 16-B pad per pixel;
//   phase 2  z2 = ReLU(conv3x3(z1) + b2): the im2col operand is read straight from the z1
//            image (tap offsets are ds_read immediates); z2 replaces z1 in LDS;
//   phase 3  y = ReLU(W3 . z2^T + b3 + x): 32 output channels per pass per wave, residual
//            for the NEXT pass loaded during this one, 16-B stores.
// MFMA v_mfma_f32_32x32x16_bf16 with the operand swap (A = weights, B = activations): a lane's
// accumulators are 16 channels of ONE pixel, so every epilogue is per pixel and the z1/z2
// writes and the y stores are 16 B after a v_permlane32_swap half-wave exchange.
// Weights come straight from L2 into VGPRs (every workgroup streams the same W1/W2/W3), three
// 32-deep K chunks ahead of their MFMAs, in FRAGMENT-MAJOR order (ops.mfma_frag_major: each
// 32-row x 16-deep A fragment is 1 KB contiguous, lane-linear), so one load instruction reads
// 1 KB of whole cache lines instead of 32 rows x 32 B.
//
// Waits.  Every vector-memory op of the kernel is an asm op (kv_lds_dma16, bn_load16) or a
// buffer store at a fixed place, issued by every wave in the same order: per 32-deep K chunk
// one "point" with a fixed op count (phase 1: 4 DMA + 2*CS weight loads; phase 2: 2*CS weight
// loads; phase 3: 2 weight loads + NR residual loads, plus 2*PS2 stores after each pass).
// Points past the end of a phase issue the same number of ops as out-of-range LDS DMAs into
// a scratch kilobyte (a dummy load into VGPRs would leave a dead asm destination that the
// register allocator may reuse while the load is still in flight); prologue ops before the
// first three points are not counted by any wait.  The op count between a load and its use
// is therefore a compile-time constant and every wait is an exact
// `s_waitcnt vmcnt(n)` (bn_sched below).  LDS fragment reads are asm too (common.h
// lds_read16), one K step ahead of their MFMAs, with counted lgkmcnt waits.
// tools/isa_lint.py --inflight checks that no instruction touches an in-flight destination.
#include "common.h"
#include "kvedge_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace kvedge {
namespace {

constexpr int kBnOOB = 0x7ffff000;  // past every operand (launcher checks): zero-fill / drop
typedef unsigned int bn_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int bn_u32x4 __attribute__((ext_vector_type(4)));

// 16-B buffer load into VGPRs with an immediate offset; the common.h vm_load16 contract
template <int OFF, class T>
__device__ __forceinline__ void bn_load16(T& dst, kv_i32x4 rs, int voff) {
  static_assert(sizeof(T) == 16 && OFF >= 0 && OFF < 4096, "buffer_load_dwordx4 offset");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
               : "=v"(dst) : "v"(voff), "s"(rs), "n"(OFF) : "memory");
}
// 16-B store through the compiler builtin, NOT inline asm: a dwordx4 store reads its data
// VGPRs after issue, and only a compiler-visible store gets the wait state the hazard
// recognizer inserts before the next write of those registers (an asm store here lost the
// third dword to the following instruction on ~0.1 % of the stores)
__device__ __forceinline__ void bn_store16(bn_u32x4 v, __amdgpu_buffer_rsrc_t rs, int voff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, 0, 0);
  asm volatile("" ::: "memory");  // keep the store in the counted op order
}
template <int N>
__device__ __forceinline__ void bn_vm_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void bn_lgkm_wait() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt field");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
template <class T>
__device__ __forceinline__ void bn_tie(T& v) {
  asm volatile("" : "+v"(v));
}
// s_barrier without __syncthreads()' fence (which would drain the in-flight weight and DMA
// rings behind it); callers retire what the hand-off needs first
__device__ __forceinline__ void bn_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void bn_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bn_barrier();
}

// Geometry of one instantiation.  C: bottleneck width (z1/z2 channels), C4 = 4C in/out.
template <int C_, int H_, int W_, int R_>
struct BnCfg {
  static constexpr int C = C_, H = H_, W = W_, R = R_, C4 = 4 * C_;
  static constexpr int NCS = C / 32;              // 32-channel subtiles of z1 / z2
  static constexpr int CS = NCS / 4;              // ... per wave (phases 1, 2)
  static constexpr int NB = H / R;                // workgroups per image
  static constexpr int M1MAX = (R + 2 < H ? R + 2 : H) * W;  // conv1 pixels incl. halo
  static constexpr int PS1 = (M1MAX + 31) / 32;   // 32-pixel subtiles, phase 1
  static constexpr int MO = R * W;                // output pixels per workgroup
  static constexpr int PS2 = (MO + 31) / 32;      // ... phases 2, 3
  static constexpr int SP = 2 * C + 16;           // LDS bytes per z1/z2 pixel (16-B pad)
  static constexpr int ZR = R + 2, ZC = W + 2;    // zero-padded z1 image
  static constexpr int SLOT = 256 * 64;           // one 32-channel x chunk of <= 256 pixels
  static constexpr int NSLOT = 6;                 // x ring (DMA 5 chunks ahead)
  static constexpr int NKC1 = C4 / 32;            // phase-1 chunks (2 K steps each)
  static constexpr int NKC2 = 9 * C / 32;         // phase-2 chunks
  static constexpr int NKC3 = C / 32;             // phase-3 chunks per pass
  static constexpr int NP3 = C4 / 32 / 4;         // phase-3 passes per wave (one subtile each)
  static constexpr int NR = 4;                    // residual loads per phase-3 position ...
  static constexpr int JR = (2 * PS2 + NR - 1) / NR;  // ... at the first JR positions of a pass
  static constexpr int BIAS = 6 * C * 4;          // b1, b2, b3 in LDS (fp32)
  static constexpr int ZBYTES = ZR * ZC * SP;
  static constexpr int SCR = (ZBYTES > NSLOT * SLOT ? ZBYTES : NSLOT * SLOT) + BIAS;  // 1 KB
  static constexpr int LDS = SCR + 1024;  // scratch: target of the count-keeping dummy DMAs
  static_assert(C % 128 == 0 && H % R == 0 && PS1 <= 8, "bneck geometry");
  static_assert(JR <= NKC3, "residual loads of a pass fit its positions");
  static_assert(NKC1 % 4 == 0 && NKC2 % 4 == 0 && NKC3 % 4 == 0 && NP3 % 2 == 0, "ring unroll");
  static_assert(MO <= PS2 * 32 && LDS <= 160 * 1024, "LDS");
};

// exact vmcnt of each wait (see the header): ops issued after the awaited one
template <class G>
struct BnSched {
  static constexpr int P1 = 4 + 2 * G::CS;                // ops per phase-1 point
  static constexpr int W1 = 2 * P1;                       // wait for W(kc): points kc-2, kc-1
  static constexpr int W2 = 2 * (2 * G::CS);
  // phase 3: ops of the point at pass position j; the wait for W(kc) at position j counts the
  // residual pieces issued after it in point kc - 3, points kc - 2 and kc - 1, and the 2 PS2
  // stores of the previous pass's epilogue when the pass edge lies in between (j < 3)
  static constexpr int r3(int j) { return j < G::JR ? G::NR : 0; }
  static constexpr int p3(int j) { return 2 + r3(j); }
  static constexpr int pos(int j) { return (j % G::NKC3 + G::NKC3) % G::NKC3; }
  static constexpr int w3(int j) {
    return r3(pos(j - 3)) + p3(pos(j - 2)) + p3(pos(j - 1)) + (j < 3 ? 2 * G::PS2 : 0);
  }
  // epilogue: ops issued after the pass's last residual piece (positions JR .. NKC3 - 1)
  static constexpr int res() {
    int n = 0;
    for (int j = G::JR; j < G::NKC3; ++j) n += p3(j);
    return n;
  }
  static constexpr int RES = res();
  static_assert(W1 <= 63 && w3(0) <= 63 && w3(1) <= 63 && w3(2) <= 63, "vmcnt field");
};

__device__ __forceinline__ floatx16 bn_mfma(const bf16x8& a, const bf16x8& b, const floatx16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// acc (lane: pixel, 16 channels 8g + 4h + e) + bias, ReLU -> bf16, exchanged so lane h holds
// channels [16q + 8h, +8) for q = 0, 1 (16 B each)
__device__ __forceinline__ void bn_pack(const floatx16& acc, const float* bl, bn_u32x4 out[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    bf16x4 lo, hi;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      lo[e] = f2bf(fmaxf(acc[8 * q + e] + bl[8 * q + e], 0.0f));
      hi[e] = f2bf(fmaxf(acc[8 * q + 4 + e] + bl[8 * q + 4 + e], 0.0f));
    }
    const bn_u32x2 a0 = __builtin_bit_cast(bn_u32x2, lo), a1 = __builtin_bit_cast(bn_u32x2, hi);
    const auto s0 = __builtin_amdgcn_permlane32_swap(a0[0], a1[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(a0[1], a1[1], false, false);
    out[q] = bn_u32x4{s0[0], s1[0], s0[1], s1[1]};
  }
}

// the 16 bias values of a lane's accumulators for channel subtile base c0 (from LDS)
__device__ __forceinline__ void bn_bias(const float* bsh, int c0, int h, float bl[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(bsh + c0 + 8 * g + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) bl[4 * g + e] = v[e];
  }
}

// debug (p.dbg = 1 / 2): copy the LDS image z1 (padded) or z2 (compact) of the band's output
// pixels into y[..., :C] (plain stores, other channels untouched)
template <class G>
__device__ void bn_debug_dump(const KvBneckParams& p, const unsigned char* lds, int n, int r0,
                              bool padded) {
  for (int i = threadIdx.x; i < G::MO * (G::C / 8); i += 256) {
    const int q = i / (G::C / 8), c8 = i % (G::C / 8);
    const int row = q / G::W, col = q % G::W;
    const int slot = padded ? (row + 1) * G::ZC + col + 1 : q;
    const bn_u32x4 v = *reinterpret_cast<const bn_u32x4*>(lds + slot * G::SP + c8 * 16);
    bn_u32x4* dst = reinterpret_cast<bn_u32x4*>(static_cast<bf16*>(p.y) +
                                                ((long)((n * G::H + r0 + row) * G::W + col)) * G::C4 + c8 * 8);
    *dst = v;
  }
}

template <class G>
__global__ __launch_bounds__(256, 1) void bneck_fused_kernel(KvBneckParams p) {
  using S = BnSched<G>;
  constexpr int C = G::C, W = G::W, CS = G::CS, PS1 = G::PS1, PS2 = G::PS2, SP = G::SP;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  float* bsh = reinterpret_cast<float*>(lds + (G::SCR - G::BIAS));  // b1 | b2 | b3
  unsigned char* scr = lds + G::SCR;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = blockIdx.x;
  const int n = wg / G::NB, r0 = (wg % G::NB) * G::R;
  const int g_lo = r0 > 0 ? r0 - 1 : 0;
  const int g_hi = r0 + G::R + 1 < G::H ? r0 + G::R + 1 : G::H;
  const int m1 = (g_hi - g_lo) * W;  // conv1 pixels of this band (rows g_lo .. g_hi - 1)
  const kv_i32x4 rx = kv_rsrc4(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.x_bytes, 0x00020000);
  const kv_i32x4 rw1 = kv_rsrc4(p.w1, C * G::C4 * 2);
  const kv_i32x4 rw2 = kv_rsrc4(p.w2, C * 9 * C * 2);
  const kv_i32x4 rw3 = kv_rsrc4(p.w3, G::C4 * C * 2);
  const bool wdbg = (p.dbg & 4) != 0;  // debug probe: every weight load out of range (zeros)
  const unsigned lbase = lds_addr(lds);

  // biases -> LDS (plain loads: any compiler VMEM op only makes the counted waits stricter)
  for (int i = tid; i < 6 * C; i += 256)
    bsh[i] = i < C ? p.b1[i] : (i < 2 * C ? p.b2[i - C] : p.b3[i - 2 * C]);

  // ------------------------------------------------------------------ phase 1: conv1
  {
    // DMA pieces: wave instruction j covers pixels 16 i .. 16 i + 15 (i = 4 wv + j), 4 pieces
    // of 16 B each; the piece at LDS position q holds channel piece q ^ ((p >> 2) & 3)
    int dsrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pp = (4 * wv + j) * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((pp >> 2) & 3);
      dsrc[j] = pp < m1 ? (((n * G::H + g_lo) * W + pp) * G::C4) * 2 + c * 16 : kBnOOB;
    }
    // weight fragment of subtile cs: row 32 (wv CS + cs) + r, k half h
    int wofs[CS];
#pragma unroll
    for (int cs = 0; cs < CS; ++cs) wofs[cs] = (((wv * CS + cs) * (G::C4 / 16)) * 64 + lane) * 16;
    // fragment read offsets within a slot for K step j of a chunk
    const int rsw = (r >> 2) & 3;
    const unsigned fo0 = lbase + r * 64 + ((0 + h) ^ rsw) * 16;
    const unsigned fo1 = lbase + r * 64 + ((2 + h) ^ rsw) * 16;

    floatx16 acc[CS][PS1];
#pragma unroll
    for (int cs = 0; cs < CS; ++cs)
#pragma unroll
      for (int ps = 0; ps < PS1; ++ps) acc[cs][ps] = floatx16{};
    bf16x8 wr[4][2][CS];  // weight ring: chunk kc % 4, step, subtile
    bf16x8 fb[2][PS1];    // fragment ring: step parity

    auto point = [&](int kc, auto slot) __attribute__((always_inline)) {
      // DMA chunk kc + 5 into slot (kc + 5) % 6; W chunk kc + 3 into ring slot (kc + 3) % 4
      const int dk = kc + 5;
      void* dst = lds + ((dk % G::NSLOT + G::NSLOT) % G::NSLOT) * G::SLOT;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        kv_lds_dma16(rx, static_cast<unsigned char*>(dst) + (4 * wv + j) * 1024,
                     dk < G::NKC1 && dk >= 0 ? dsrc[j] + dk * 64 : kBnOOB);
      // (past the end: out-of-range loads -> zeros, retired and tied after the loop, so no
      // in-flight destination is ever dead; the op sequence stays branch-free)
      const int wk = kc + 3;
      constexpr int ws = decltype(slot)::value;
#pragma unroll
      for (int cs = 0; cs < CS; ++cs) {
        const int o = wk < G::NKC1 && !wdbg ? wofs[cs] + wk * 2048 : kBnOOB;
        bn_load16<0>(wr[ws][0][cs], rw1, o);
        bn_load16<1024>(wr[ws][1][cs], rw1, o);
      }
    };
    auto reads = [&](int kc, auto step, bf16x8(&f)[PS1]) __attribute__((always_inline)) {
      const unsigned b = (decltype(step)::value ? fo1 : fo0) + (kc % G::NSLOT) * G::SLOT;
      static_range<0, PS1>([&](auto ps) __attribute__((always_inline)) {
        lds_read16<decltype(ps)::value * 2048>(f[decltype(ps)::value], b);
      });
    };
    // prologue: DMA chunks 0, 1, then points -3 .. -1 (DMA chunks 2..4, W chunks 0..2) -- the
    // first three points are the only prologue ops a wait counts
#pragma unroll
    for (int dk = 0; dk < 2; ++dk)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        kv_lds_dma16(rx, lds + dk * G::SLOT + (4 * wv + j) * 1024, dsrc[j] + dk * 64);
    point(-3, IC<0>{});
    point(-2, IC<1>{});
    point(-1, IC<2>{});
    bn_vm_wait<S::W1>();  // W(0), and the older DMA(0), landed
    bn_lds_barrier();     // every wave's DMA(0), and the biases
    reads(0, IC<0>{}, fb[0]);
    for (int kb = 0; kb < G::NKC1; kb += 4) {
      static_range<0, 4>([&](auto u) __attribute__((always_inline)) {
        constexpr int ws = decltype(u)::value;
        const int kc = kb + ws;
        // step 0: next step's fragments, then this step's weights + fragments
        reads(kc, IC<1>{}, fb[1]);
        bn_vm_wait<S::W1>();
#pragma unroll
        for (int cs = 0; cs < CS; ++cs) {
          bn_tie(wr[ws][0][cs]);
          bn_tie(wr[ws][1][cs]);
        }
        bn_lgkm_wait<PS1>();
#pragma unroll
        for (int ps = 0; ps < PS1; ++ps) bn_tie(fb[0][ps]);
#pragma unroll
        for (int ps = 0; ps < PS1; ++ps)
#pragma unroll
          for (int cs = 0; cs < CS; ++cs) acc[cs][ps] = bn_mfma(wr[ws][0][cs], fb[0][ps], acc[cs][ps]);
        // step 1: chunk kc + 1 landed everywhere (its DMA is older than W(kc)); the barrier
        // also frees slot (kc - 1) % 6 for DMA(kc + 5)
        bn_barrier();
        point(kc, IC<(ws + 3) % 4>{});
        // the next chunk's first fragments (after the last chunk: a harmless re-read of a
        // ring slot, retired below -- the op sequence stays branch-free)
        reads(kc + 1, IC<0>{}, fb[0]);
        bn_lgkm_wait<PS1>();  // this step's reads retired, the next step's in flight
#pragma unroll
        for (int ps = 0; ps < PS1; ++ps) bn_tie(fb[1][ps]);
#pragma unroll
        for (int ps = 0; ps < PS1; ++ps)
#pragma unroll
          for (int cs = 0; cs < CS; ++cs) acc[cs][ps] = bn_mfma(wr[ws][1][cs], fb[1][ps], acc[cs][ps]);
      });
    }
    bn_vm_wait<0>();  // the tail points' zero-fill DMAs land before the ring becomes z1
    bn_lgkm_wait<0>();
#pragma unroll
    for (int ps = 0; ps < PS1; ++ps) bn_tie(fb[0][ps]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int cs = 0; cs < CS; ++cs) {
        bn_tie(wr[i][0][cs]);
        bn_tie(wr[i][1][cs]);
      }
    bn_lds_barrier();
    // z1 image: clear (pads and out-of-image halo rows must be zero), then the band's pixels
    for (int i = tid * 16; i < G::ZBYTES; i += 256 * 16)
      *reinterpret_cast<bn_u32x4*>(lds + i) = bn_u32x4{0, 0, 0, 0};
    bn_lds_barrier();
#pragma unroll
    for (int cs = 0; cs < CS; ++cs) {
      const int c0 = 32 * (wv * CS + cs);
      float bl[16];
      bn_bias(bsh, c0, h, bl);
#pragma unroll
      for (int ps = 0; ps < PS1; ++ps) {
        const int q = ps * 32 + r;
        bn_u32x4 v[2];
        bn_pack(acc[cs][ps], bl, v);
        if (q < m1) {
          const int lr = q / W, col = q - lr * W;
          const int slot = (g_lo + lr - (r0 - 1)) * G::ZC + col + 1;
          unsigned char* d = lds + slot * SP + (c0 + 8 * h) * 2;
          *reinterpret_cast<bn_u32x4*>(d) = v[0];
          *reinterpret_cast<bn_u32x4*>(d + 32) = v[1];
        }
      }
    }
    bn_lds_barrier();
  }

  if ((p.dbg & 3) == 1) {
    bn_debug_dump<G>(p, lds, n, r0, true);
    return;
  }
  // ------------------------------------------------------------------ phase 2: 3x3
  {
    floatx16 acc2[CS][PS2];
#pragma unroll
    for (int cs = 0; cs < CS; ++cs)
#pragma unroll
      for (int ps = 0; ps < PS2; ++ps) acc2[cs][ps] = floatx16{};
    int wofs[CS];
    constexpr int K2 = 9 * C, CPT = C / 32;  // chunks per tap (CPT % 4 == 0)
#pragma unroll
    for (int cs = 0; cs < CS; ++cs) wofs[cs] = (((wv * CS + cs) * (K2 / 16)) * 64 + lane) * 16;
    // top-left window slot of output pixel q (clamped into the band for the padding lanes)
    unsigned pb[PS2];
#pragma unroll
    for (int ps = 0; ps < PS2; ++ps) {
      const int q = min(ps * 32 + r, G::MO - 1);
      const int i = q / W, j = q - i * W;
      pb[ps] = lbase + (i * G::ZC + j) * SP + 16 * h;
    }
    bf16x8 wr[4][2][CS];
    bf16x8 fb[2][PS2];
    auto point = [&](int kc, auto slot) __attribute__((always_inline)) {
      const int wk = kc + 3;
      constexpr int ws = decltype(slot)::value;
#pragma unroll
      for (int cs = 0; cs < CS; ++cs) {
        const int o = wk < G::NKC2 && !wdbg ? wofs[cs] + wk * 2048 : kBnOOB;
        bn_load16<0>(wr[ws][0][cs], rw2, o);
        bn_load16<1024>(wr[ws][1][cs], rw2, o);
      }
    };
    // tap t's byte offset in the z1 image (dy, dx = t / 3, t % 3)
    auto tapoff = [&](int t) __attribute__((always_inline)) {
      return ((t / 3) * G::ZC + t % 3) * SP;
    };
    // the fragments of K step `kk` (0 .. C/16 - 1, an immediate) of the tap at offset `to`
    auto reads = [&](int to, auto kk, bf16x8(&f)[PS2]) __attribute__((always_inline)) {
      static_range<0, PS2>([&](auto ps) __attribute__((always_inline)) {
        lds_read16<decltype(kk)::value * 32>(f[decltype(ps)::value], pb[decltype(ps)::value] + to);
      });
    };
    point(-3, IC<0>{});
    point(-2, IC<1>{});
    point(-1, IC<2>{});
    reads(0, IC<0>{}, fb[0]);
    for (int t = 0; t < 9; ++t) {
      const int to = tapoff(t), tn = tapoff(t < 8 ? t + 1 : 8);
      static_range<0, CPT>([&](auto u) __attribute__((always_inline)) {
        constexpr int j = decltype(u)::value;
        constexpr int ws = j % 4;  // chunk kc = t CPT + j, CPT % 4 == 0
        const int kc = t * CPT + j;
        reads(to, IC<2 * j + 1>{}, fb[1]);
        bn_vm_wait<S::W2>();
#pragma unroll
        for (int cs = 0; cs < CS; ++cs) {
          bn_tie(wr[ws][0][cs]);
          bn_tie(wr[ws][1][cs]);
        }
        bn_lgkm_wait<PS2>();
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[0][ps]);
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps)
#pragma unroll
          for (int cs = 0; cs < CS; ++cs) acc2[cs][ps] = bn_mfma(wr[ws][0][cs], fb[0][ps], acc2[cs][ps]);
        point(kc, IC<(ws + 3) % 4>{});
        // next step: this tap's step 2j + 2, or the next tap's step 0 (after the last tap: a
        // re-read, retired below)
        if constexpr (j + 1 < CPT) reads(to, IC<2 * j + 2>{}, fb[0]);
        else reads(tn, IC<0>{}, fb[0]);
        bn_lgkm_wait<PS2>();
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[1][ps]);
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps)
#pragma unroll
          for (int cs = 0; cs < CS; ++cs) acc2[cs][ps] = bn_mfma(wr[ws][1][cs], fb[1][ps], acc2[cs][ps]);
      });
    }
    bn_vm_wait<0>();
    bn_lgkm_wait<0>();
#pragma unroll
    for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[0][ps]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int cs = 0; cs < CS; ++cs) {
        bn_tie(wr[i][0][cs]);
        bn_tie(wr[i][1][cs]);
      }
    bn_lds_barrier();  // every wave is done reading z1: z2 replaces it
#pragma unroll
    for (int cs = 0; cs < CS; ++cs) {
      const int c0 = 32 * (wv * CS + cs);
      float bl[16];
      bn_bias(bsh + C, c0, h, bl);
#pragma unroll
      for (int ps = 0; ps < PS2; ++ps) {
        const int q = ps * 32 + r;
        bn_u32x4 v[2];
        bn_pack(acc2[cs][ps], bl, v);
        if (q < G::MO) {
          unsigned char* d = lds + q * SP + (c0 + 8 * h) * 2;
          *reinterpret_cast<bn_u32x4*>(d) = v[0];
          *reinterpret_cast<bn_u32x4*>(d + 32) = v[1];
        }
      }
    }
    bn_lds_barrier();
  }

  if ((p.dbg & 3) == 2) {
    bn_debug_dump<G>(p, lds, n, r0, false);
    return;
  }
  // ------------------------------------------------------------------ phase 3: conv3 + res
  {
    // pass P: output channels 32 (wv + 4 P) .. + 32; K = C from z2
    unsigned zb[PS2];
    int xo[PS2];  // byte offset of output pixel q's row in x / y (+ lane half), or OOB
#pragma unroll
    for (int ps = 0; ps < PS2; ++ps) {
      const int q = ps * 32 + r;
      zb[ps] = lbase + min(q, G::MO - 1) * SP + 16 * h;
      xo[ps] = q < G::MO ? (((n * G::H + r0) * W + q) * G::C4 + 8 * h) * 2 : kBnOOB;
    }
    const int wofs = ((wv * (C / 16)) * 64 + lane) * 16;  // + pass: 4 subtiles further
    constexpr int NKC = G::NP3 * G::NKC3;                // weight chunks over all passes
    floatx16 acc[PS2];
    bf16x8 wr[4][2];
    bf16x8 fb[2][PS2];
    bn_u32x4 rv[PS2][2];  // this pass's residual, store layout (pixel subtile, 16-ch group)
    // point at position po of pass `pass` (global chunk kc): W(kc + 3), then -- at the first
    // JR positions -- residual pieces [po NR, po NR + NR) of the SAME pass (piece = 2 ps + qq)
    auto point = [&](int kc, int pass, auto slot, auto pos, auto real) __attribute__((always_inline)) {
      constexpr int ws = decltype(slot)::value, po = decltype(pos)::value;
      constexpr bool rl = decltype(real)::value;  // false: the prologue's "pass -1"
      const int wk = kc + 3;  // >= 0: the prologue starts at point -3
      const int o = wk < NKC && !wdbg ? wofs + (wk / G::NKC3) * 4 * (C / 16) * 1024 +
                                            (wk % G::NKC3) * 2048
                                      : kBnOOB;
      bn_load16<0>(wr[ws][0], rw3, o);
      bn_load16<1024>(wr[ws][1], rw3, o);
      if constexpr (po < G::JR) {
        const int cofs = (32 * (wv + 4 * pass)) * 2;
        static_range<0, G::NR>([&](auto e) __attribute__((always_inline)) {
          constexpr int pc = po * G::NR + decltype(e)::value;
          constexpr int ps = pc / 2 < PS2 ? pc / 2 : PS2 - 1, qq = pc % 2;
          if constexpr (rl && pc < 2 * PS2)
            bn_load16<0>(rv[ps][qq], rx, xo[ps] != kBnOOB ? xo[ps] + cofs + qq * 32 : kBnOOB);
          else
            kv_lds_dma16(rx, scr, kBnOOB);  // keeps the op count of the position fixed
        });
      }
    };
    auto reads = [&](int kk, bf16x8(&f)[PS2]) __attribute__((always_inline)) {
      static_range<0, PS2>([&](auto ps) __attribute__((always_inline)) {
        lds_read16<0>(f[decltype(ps)::value], zb[decltype(ps)::value] + kk * 32);
      });
    };
    // prologue: the last three positions of a "pass -1" (W chunks 0..2; its residual pieces,
    // if any, are dummies), then that pass's 2 PS2 stores as out-of-range no-ops
    point(-3, -1, IC<0>{}, IC<G::NKC3 - 3>{}, IC<0>{});
    point(-2, -1, IC<1>{}, IC<G::NKC3 - 2>{}, IC<0>{});
    point(-1, -1, IC<2>{}, IC<G::NKC3 - 1>{}, IC<0>{});
    static_range<0, 2 * PS2>([&](auto e) __attribute__((always_inline)) {
      bn_store16(bn_u32x4{0, 0, 0, 0}, ry, kBnOOB);
      (void)e;
    });
    reads(0, fb[0]);
    for (int pass = 0; pass < G::NP3; ++pass) {
#pragma unroll
      for (int ps = 0; ps < PS2; ++ps) acc[ps] = floatx16{};
      static_range<0, G::NKC3>([&](auto u) __attribute__((always_inline)) {
        constexpr int j = decltype(u)::value;
        constexpr int ws = j % 4;  // NKC3 % 4 == 0: the ring slot of chunk kc is kc % 4 == j % 4
        const int kc = pass * G::NKC3 + j;
        reads(2 * j + 1, fb[1]);
        bn_vm_wait<BnSched<G>::w3(j)>();
        bn_tie(wr[ws][0]);
        bn_tie(wr[ws][1]);
        bn_lgkm_wait<PS2>();
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[0][ps]);
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) acc[ps] = bn_mfma(wr[ws][0], fb[0][ps], acc[ps]);
        point(kc, pass, IC<(ws + 3) % 4>{}, IC<j>{}, IC<1>{});
        // next step: after the pass's last step the same z2 fragments restart at K 0
        reads(j + 1 < G::NKC3 ? 2 * j + 2 : 0, fb[0]);
        bn_lgkm_wait<PS2>();
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[1][ps]);
#pragma unroll
        for (int ps = 0; ps < PS2; ++ps) acc[ps] = bn_mfma(wr[ws][1], fb[1][ps], acc[ps]);
      });
      // epilogue: + b3 + residual, ReLU, store.  The residual pieces are the ops of the first
      // JR positions; only the later positions' weight loads may still be in flight
      bn_vm_wait<BnSched<G>::RES>();
      const int c0 = 32 * (wv + 4 * pass);
      float bl[16];
      bn_bias(bsh + 2 * C, c0, h, bl);
#pragma unroll
      for (int ps = 0; ps < PS2; ++ps) {
        bn_tie(rv[ps][0]);
        bn_tie(rv[ps][1]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bn_u32x4 rr = rv[ps][q];
          const auto t0 = __builtin_amdgcn_permlane32_swap(rr[0], rr[2], false, false);
          const auto t1 = __builtin_amdgcn_permlane32_swap(rr[1], rr[3], false, false);
          const unsigned wl[2] = {t0[0], t1[0]}, wh[2] = {t0[1], t1[1]};
          bf16x4 lo, hi;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float rlo = __uint_as_float(e & 1 ? wl[e >> 1] & 0xffff0000u : wl[e >> 1] << 16);
            const float rhi = __uint_as_float(e & 1 ? wh[e >> 1] & 0xffff0000u : wh[e >> 1] << 16);
            lo[e] = f2bf(fmaxf(acc[ps][8 * q + e] + bl[8 * q + e] + rlo, 0.0f));
            hi[e] = f2bf(fmaxf(acc[ps][8 * q + 4 + e] + bl[8 * q + 4 + e] + rhi, 0.0f));
          }
          const bn_u32x2 a0 = __builtin_bit_cast(bn_u32x2, lo), a1 = __builtin_bit_cast(bn_u32x2, hi);
          const auto s0 = __builtin_amdgcn_permlane32_swap(a0[0], a1[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(a0[1], a1[1], false, false);
          bn_store16(bn_u32x4{s0[0], s1[0], s0[1], s1[1]}, ry,
                     xo[ps] != kBnOOB ? xo[ps] + c0 * 2 + q * 32 : kBnOOB);
        }
      }
    }
    // the last step prefetched a next pass's first fragments: retire them (no dead
    // destinations in flight), and every dummy DMA before this workgroup's LDS is released
    bn_lgkm_wait<0>();
#pragma unroll
    for (int ps = 0; ps < PS2; ++ps) bn_tie(fb[0][ps]);
    bn_vm_wait<0>();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bn_tie(wr[i][0]);
      bn_tie(wr[i][1]);
    }
  }
}

struct BnEntry {
  int C, H, W, R;
  void (*fn)(KvBneckParams);
  int lds;
};

template <int C, int H, int W, int R>
constexpr BnEntry bn_entry() {
  return BnEntry{C, H, W, R, bneck_fused_kernel<BnCfg<C, H, W, R>>, BnCfg<C, H, W, R>::LDS};
}

const BnEntry kBnTable[] = {
    bn_entry<256, 14, 14, 7>(),   // ResNet-50 stage 3 (half images: 128 accumulators per lane)
    bn_entry<128, 28, 28, 7>(),   // ResNet-50 stage 2
};

}  // namespace

}  // namespace kvedge

extern "C" int kv_bneck_fused_supported(int C, int H, int W) {
  using namespace kvedge;
  for (const BnEntry& e : kBnTable)
    if (e.C == C && e.H == H && e.W == W) return 1;
  return 0;
}

extern "C" int kv_bneck_fused(const KvBneckParams* p, hipStream_t stream) {
  using namespace kvedge;
  for (const BnEntry& e : kBnTable) {
    if (e.C != p->C || e.H != p->H || e.W != p->W) continue;
    if (p->N <= 0) return 0;
    if (p->x_bytes <= 0 || p->x_bytes >= kBnOOB - 4096) return -9;
    if ((long long)p->N * p->H * p->W * 4 * p->C * 2 != p->x_bytes) return -8;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(e.fn),
                            hipFuncAttributeMaxDynamicSharedMemorySize, e.lds) != hipSuccess)
      return -7;
    const unsigned grid = (unsigned)(p->N * (p->H / e.R));
    hipLaunchKernelGGL(e.fn, dim3(grid), dim3(256), (unsigned)e.lds, stream, *p);
    return hipGetLastError() == hipSuccess ? 0 : -7;
  }
  return -6;
}
