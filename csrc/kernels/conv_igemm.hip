// K1/K2/K3 — implicit-GEMM convolution and GEMM on CDNA4 MFMA (gfx950).
//
// One kernel family covers every conv in ResNet-50 and YOLOv8n plus the FC layer:
//   M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin (NHWC, k-order (r, s, c)).
// The im2col gather is fused into the global->register staging of the A tile:
// no im2col buffer ever exists.  BatchNorm is folded into W/bias on the host,
// and bias + residual + ReLU/SiLU + bf16 cast are fused into the epilogue.
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md):
//  * 256-thread workgroups (4 wave64s), tile BM x BN x 64, v_mfma_f32_16x16x32_bf16.
//  * Operands swapped: D = W * A^T, so the accumulator of a lane holds FOUR
//    CONSECUTIVE OUTPUT CHANNELS of one pixel -> 8-byte NHWC stores.
//  * LDS image [row][64] bf16 (128-B rows) with chunk ^= (row & 7) XOR swizzle:
//    ds_write_b128 (8-lane contiguous groups) and the ds_read_b128 fragment reads
//    (4 x 16-lane groups) are both bank-conflict-free (derivation in SURVEY.md
//    notes / docs/kernels.md).
//  * Register-staged double buffer (T14 async-STAGE split): tile k+1 is issued to
//    VGPRs before the MFMAs of tile k and written to the other LDS buffer after,
//    one barrier per K step.
//  * XCD-aware bijective block remap so the N-tiles of one M panel share an L2.
//
// The reference has no kernels; the kernel inventory this
// implements is SURVEY.md §2.5 K1-K3.
#include <algorithm>

#include "common.h"
#include "kvedge_kernels.h"

namespace kvedge {
namespace {

constexpr int BK = 64;

struct TileCfg {
  int bm, bn, wm, wn;
};

template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(const KvConvParams p) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int AR = BM / 32;  // A rows staged per thread
  constexpr int BR = BN / 32;  // B rows staged per thread
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 16x16");

  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * BK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int wm = wv / WN, wn = wv % WN;

  const int nbm = (p.M + BM - 1) / BM;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, nbm * nbn);
  const int m0 = (t / nbn) * BM;
  const int n0 = (t % nbn) * BN;
  // the tile's bias slice, one value per thread, loaded before the K loop and staged through
  // LDS for the epilogue (per-lane global bias loads there each waited with a vmcnt(0))
  static_assert(BN <= 256, "one bias value per thread");
  const float bias_r = (tid < BN && p.bias && n0 + tid < p.Cout) ? p.bias[n0 + tid] : 0.f;

  const bf16* __restrict__ X = reinterpret_cast<const bf16*>(p.x);
  const bf16* __restrict__ Wt = reinterpret_cast<const bf16*>(p.w);

  const int cc = tid & 7;   // 16-B chunk column this thread stages
  const int rr = tid >> 3;  // first staged row (then +32, +64 ...)

  // ---- per-row gather info (fixed for the whole K loop) -------------------
  int a_base[AR], a_h0[AR], a_w0[AR];
  const int HoWo = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + rr + 32 * i;
    if (m < p.M) {
      if (MODE == 1) {
        a_base[i] = m * p.ldx + p.x_coff;
        a_h0[i] = 0;
        a_w0[i] = 0;
      } else {
        const int img = m / HoWo;
        const int rem = m - img * HoWo;
        const int ho = rem / p.Wo;
        const int wo = rem - ho * p.Wo;
        a_base[i] = img * p.H * p.W * p.ldx + p.x_coff;
        a_h0[i] = ho * p.stride - p.pad;
        a_w0[i] = wo * p.stride - p.pad;
      }
    } else {
      a_base[i] = 0;
      a_h0[i] = -(1 << 28);  // never in range
      a_w0[i] = -(1 << 28);
    }
  }

  // ---- incremental (r, s, c) state of this thread's chunk column (MODE 0) --
  int kr = 0, ksx = 0, kc = cc * 8;
  if (MODE == 0) {
    while (kc >= p.Cin) {
      kc -= p.Cin;
      if (++ksx == p.KW) { ksx = 0; ++kr; }
    }
  }
  const int kwp = (p.KW + 1) & ~1;  // stem: KW padded to even
  const int kpr = kwp * 4;          // stem: K elements per filter row

  uint4 ra[AR], rb[BR];

  auto load_a = [&](int kt) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (MODE == 1) {
        const int k = kt * BK + cc * 8;
        if (a_h0[i] >= 0 && k < p.Cin)
          v = *reinterpret_cast<const uint4*>(X + a_base[i] + k);
      } else if (MODE == 0) {
        const int hi = a_h0[i] + kr, wi = a_w0[i] + ksx;
        if (kr < p.KH && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
          v = *reinterpret_cast<const uint4*>(X + a_base[i] + (hi * p.W + wi) * p.ldx + kc);
      } else {  // MODE 2 stem: chunk = pixels (s, s+1) x 4 channels of filter row r
        const int k = kt * BK + cc * 8;
        const int r = k / kpr;
        const int s = ((k - r * kpr) >> 3) * 2;
        const int hi = a_h0[i] + r, wi = a_w0[i] + s;
        if (r < p.KH && (unsigned)hi < (unsigned)p.H) {
          const bf16* rowp = X + a_base[i] + hi * p.W * 4;
          uint2 lo = make_uint2(0, 0), hi2 = make_uint2(0, 0);
          if ((unsigned)wi < (unsigned)p.W) lo = *reinterpret_cast<const uint2*>(rowp + wi * 4);
          if ((unsigned)(wi + 1) < (unsigned)p.W)
            hi2 = *reinterpret_cast<const uint2*>(rowp + (wi + 1) * 4);
          v = make_uint4(lo.x, lo.y, hi2.x, hi2.y);
        }
      }
      ra[i] = v;
    }
  };
  auto advance_k = [&]() {
    if (MODE == 0) {
      kc += BK;
      while (kc >= p.Cin) {
        kc -= p.Cin;
        if (++ksx == p.KW) { ksx = 0; ++kr; }
      }
    }
  };
  auto load_b = [&](int kt) {
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + rr + 32 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < p.Cout)
        v = *reinterpret_cast<const uint4*>(Wt + (size_t)n * p.Kpad + kt * BK + cc * 8);
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
    bf16* As = smem + buf * (BM + BN) * BK;
    bf16* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int row = rr + 32 * i;
      *reinterpret_cast<uint4*>(As + row * BK + ((cc ^ (row & 7)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rr + 32 * i;
      *reinterpret_cast<uint4*>(Bs + row * BK + ((cc ^ (row & 7)) << 3)) = rb[i];
    }
  };

  floatx4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16* As = smem + buf * (BM + BN) * BK;
    const bf16* Bs = As + BM * BK;
    const int fr = lane & 15;
    const int sw = lane & 7;  // == row & 7 for every fragment row
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int q = ks * 4 + (lane >> 4);
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = wm * WTM + tm * 16 + fr;
        af[tm] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((q ^ sw) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = wn * WTN + tn * 16 + fr;
        bfg[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((q ^ sw) << 3));
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tn][tm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[tn], af[tm], acc[tn][tm], 0, 0, 0);
    }
  };

  const int nk = p.Kpad / BK;
  load_a(0);
  load_b(0);
  store_tiles(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      advance_k();
      load_a(kt + 1);
      load_b(kt + 1);
    }
    compute(cur);
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue, staged through LDS for full-line 16-B stores ----------
  // Phase 1: acc (+bias, +act when there is no residual) -> bf16 C tile in LDS,
  //          row stride BN*2+16 B (ds_write_b64 at most 2-way, rows 16-B aligned).
  // Phase 2: each lane moves 16 B (8 channels) of a row: residual read, act,
  //          store — consecutive lanes cover consecutive bytes of a row, so a wave
  //          writes whole 128-256 B row segments instead of 32-B pieces.
  constexpr int CS = BN + 8;  // C-tile row stride in elements
  static_assert(BM * CS * 2 + BN * 4 <= 2 * (BM + BN) * BK * 2, "C tile + bias slot must fit");
  const bool has_res = p.res != nullptr;
  float* const lbias = reinterpret_cast<float*>(smem + 2 * (BM + BN) * BK) - BN;  // past the C tile
  if (tid < BN) lbias[tid] = bias_r;
  __syncthreads();
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, p.M * p.ldy * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.res), (short)0, has_res ? p.M * p.ldr * 2 : 0, 0x00020000);
  constexpr int kOOB1 = 0x7ffffff0;
  constexpr int CPR = BN / 8;               // 16-B chunks per tile row
  constexpr int PER = BM * CPR / 256;       // chunks per thread
  dispatch_act(p.act, has_res, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int nl = wn * WTN + tn * 16 + (lane >> 4) * 4;
      const float4 bv = *reinterpret_cast<const float4*>(lbias + nl);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int ml = wm * WTM + tm * 16 + (lane & 15);
        bf16x4 o;
        o[0] = f2bf(act_c<act1>(acc[tn][tm][0] + bv.x));
        o[1] = f2bf(act_c<act1>(acc[tn][tm][1] + bv.y));
        o[2] = f2bf(act_c<act1>(acc[tn][tm][2] + bv.z));
        o[3] = f2bf(act_c<act1>(acc[tn][tm][3] + bv.w));
        *reinterpret_cast<bf16x4*>(smem + ml * CS + nl) = o;
      }
    }
    // the residual chunks are all loaded before the first store; range-checked buffer
    // loads / stores (out-of-tile: offset past the end), so the loop has no branches
    u32x4v rv[PER];
    if (has_res) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int idx = tid + 256 * j;
        const int m = m0 + idx / CPR, n = n0 + (idx % CPR) * 8;
        const int off = (m < p.M && n < p.Cout) ? (m * p.ldr + p.r_coff + n) * 2 : kOOB1;
        rv[j] = __builtin_amdgcn_raw_buffer_load_b128(rres, off, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int idx = tid + 256 * j;
      const int ml = idx / CPR, ch = idx % CPR;
      const int m = m0 + ml, n = n0 + ch * 8;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + ml * CS + ch * 8);
      if (has_res) {
        const bf16x8 r8 = __builtin_bit_cast(bf16x8, rv[j]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(act_c<act2>((float)v[e] + (float)r8[e]));
      }
      const int off = (m < p.M && n < p.Cout) ? (m * p.ldy + p.y_coff + n) * 2 : kOOB1;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), ry, off, 0, 0);
    }
  });
}

typedef void (*ConvKernelFn)(const KvConvParams);

template <int BM, int BN, int WM, int WN>
struct TileInst {
  static ConvKernelFn get(int mode) {
    switch (mode) {
      case 0: return conv_igemm_kernel<BM, BN, WM, WN, 0>;
      case 1: return conv_igemm_kernel<BM, BN, WM, WN, 1>;
      default: return conv_igemm_kernel<BM, BN, WM, WN, 2>;
    }
  }
};

struct TileEntry {
  TileCfg cfg;
  ConvKernelFn (*get)(int);
};

const TileEntry kTiles[] = {
    {{128, 128, 2, 2}, &TileInst<128, 128, 2, 2>::get},
    {{128, 64, 2, 2}, &TileInst<128, 64, 2, 2>::get},
    {{64, 64, 2, 2}, &TileInst<64, 64, 2, 2>::get},
    {{256, 64, 4, 1}, &TileInst<256, 64, 4, 1>::get},
    {{64, 128, 2, 2}, &TileInst<64, 128, 2, 2>::get},
    {{256, 128, 2, 2}, &TileInst<256, 128, 2, 2>::get},
};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

}  // namespace
}  // namespace kvedge

using namespace kvedge;

namespace kvedge {
// v2 family (conv_glds.hip): tile indices kNumTiles .. kNumTiles + glds_num_tiles() - 1
int glds_num_tiles();
int glds_launch(const KvConvParams* p, int tile, hipStream_t stream);
int glds_tile_bm(int tile);
int glds_tile_bn(int tile);
// v3 persistent streaming family (conv_stream.hip, 1x1 GEMM / dual only): indices after v2
int stream_num_tiles();
int stream_launch(const KvConvParams* p, int tile, hipStream_t stream);
int stream_tail_tile(int n_t);
// v4 family (conv_direct.hip): persistent direct 3x3 conv for narrow channel counts
int direct_num_tiles();
int direct_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v6 A-resident N-loop 1x1 GEMM (conv_nloop.hip): indices after v4
int nloop_num_tiles();
int nloop_launch(const KvConvParams* p, int tile, hipStream_t stream);
int nloop_sched_check();
// v7 cross-stage pipelined LDS-DMA GEMM (conv_glds.hip XP loop): indices after v6
int xp_num_tiles();
int xp_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v8 split-K (conv_glds.hip SK kernels + finalize): indices after v7
int sk_num_tiles();
int sk_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v10 direct-epilogue forms of the v4 family (conv_direct.hip): indices after v8
int direct_de_num_tiles();
int direct_de_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v12 skinny implicit GEMM for edge batches (conv_skinny.hip): indices after v10
int skinny_num_tiles();
int skinny_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v14 256x256 8-phase ping-pong implicit GEMM (conv_pp.hip): indices after v12
int pp_num_tiles();
int pp_launch(const KvConvParams* p, int tile, hipStream_t stream);
// v9 bottleneck seam, conv3 + residual -> next conv1 (conv_seam.hip): tail calls only, tile
// indices after the whole table above (kv_conv_num_tiles() + i)
int seam_num_tiles();
int seam_pick_tile(const KvConvParams* p);
int seam_launch(const KvConvParams* p, int tile, hipStream_t stream);
}  // namespace kvedge

extern "C" int kv_conv_seam_num_tiles(void) { return kvedge::seam_num_tiles(); }

extern "C" int kv_nloop_sched_check(void) { return kvedge::nloop_sched_check(); }

extern "C" int kv_conv_num_tiles(void) {
  return kNumTiles + glds_num_tiles() + stream_num_tiles() + direct_num_tiles() +
         nloop_num_tiles() + xp_num_tiles() + sk_num_tiles() + direct_de_num_tiles() +
         skinny_num_tiles() + pp_num_tiles();
}

// first split-K (v8) tile index: ops.is_splitk() sizes a workspace for exactly these, so it
// is read from here rather than re-derived from family sizes in Python (adding the v14 family
// after the split-K one once shifted a derived base by four)
extern "C" int kv_conv_splitk_base(void) {
  return kNumTiles + glds_num_tiles() + stream_num_tiles() + direct_num_tiles() +
         nloop_num_tiles() + xp_num_tiles();
}
extern "C" int kv_conv_splitk_num_tiles(void) { return sk_num_tiles(); }

extern "C" int kv_conv_pick_tile(const KvConvParams* p) {
  // Heuristic: enough workgroups to cover 256 CUs x 2, largest tile otherwise.
  const long long M = p->M, N = p->Cout;
  auto nwg = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (N <= 64) {
    if (nwg(256, 64) >= 1024) return 3;
    if (nwg(128, 64) >= 512) return 1;
    return 2;
  }
  if (nwg(256, 128) >= 2048) return 5;
  if (nwg(128, 128) >= 512) return 0;
  if (nwg(64, 128) >= 256) return 4;
  return 2;
}

#ifdef KVEDGE_CHECKS
// Bounds-check build (`python -m kvedge_amd._build --checks`): before a
// launch, every operand extent the kernel may touch must lie inside the device
// allocation that contains its base pointer.  GPU ASan / xnack+ are unavailable on the
// MI355X pool, so this host-side check is what guards the raw C ABI (native tools and
// tests that bypass the torch bindings, which always check tensor extents).
static bool kv_in_alloc(const void* ptr, long long bytes) {
  if (!ptr || bytes <= 0) return true;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const char* b = static_cast<const char*>(base);
  const char* q = static_cast<const char*>(ptr);
  return q >= b && q + bytes <= b + size;
}

static int kv_conv_check_extents(const KvConvParams* p) {
  const long long M = (long long)p->N * p->Ho * p->Wo;
  if (!kv_in_alloc(p->x, p->in_u8 ? (long long)p->N * p->H * p->W * 12
                                    : (long long)p->N * p->H * p->W * p->ldx * 2)) return -20;
  if (!kv_in_alloc(p->w, (long long)p->Cout * p->Kpad * 2)) return -21;
  if (!kv_in_alloc(p->bias, (long long)p->Cout * 4)) return -22;
  if (!kv_in_alloc(p->y, M * p->ldy * 2)) return -23;
  if (p->res && !kv_in_alloc(p->res, M * p->ldr * 2)) return -24;
  if (p->n_t && (!kv_in_alloc(p->z, M * p->ldz * 2) ||
                 !kv_in_alloc(p->w_t, (long long)p->n_t * p->Cout * 2) ||
                 !kv_in_alloc(p->bias_t, (long long)p->n_t * 4)))
    return -28;
  if (p->mode == 4 && !kv_in_alloc(p->x2, (long long)p->N * p->H2 * p->W2 * p->ldx2 * 2)) return -25;
  if (p->x_coff + p->Cin > p->ldx || p->y_coff + p->Cout > p->ldy) return -26;
  if (p->res && p->r_coff + p->Cout > p->ldr) return -27;
  return 0;
}
#endif

static int kv_conv2d_one(const KvConvParams* p, int tile, hipStream_t stream);

// Byte span of one image of every NHWC operand a conv touches.  The kernels address
// operands through 32-bit buffer-resource offsets (out-of-range offsets are the zero-fill
// padding trick), so one launch must keep every operand below 2 GiB.
static long long kv_conv_max_image_bytes(const KvConvParams* p) {
  const long long hw = (long long)p->H * p->W, ohw = (long long)p->Ho * p->Wo;
  long long m = p->in_u8 ? hw * 12 : hw * p->ldx * 2;
  m = std::max(m, ohw * p->ldy * 2);
  if (p->res) m = std::max(m, ohw * p->ldr * 2);
  if (p->mode == 4) m = std::max(m, (long long)p->H2 * p->W2 * p->ldx2 * 2);
  if (p->n_t) m = std::max(m, ohw * p->ldz * 2);
  return m;
}

// Batches whose activations exceed 2 GiB per tensor (ResNet-50 past ~1200 images, YOLOv8n
// past ~650: the 288 GB of HBM holds far more) run as a sequence of image-chunk launches
// on the same stream; each chunk's base pointers are 64-bit offsets from the host, so
// the in-kernel 32-bit offsets stay in range.  Small batches take the single launch.
static long long g_chunk_bytes = 0x7f000000LL;  // < kOOB: OOB offsets stay past the end

// Tests shrink the chunk size to exercise the chunked path with small tensors
// (0 restores the default).  Returns the value in effect.
extern "C" long long kv_set_conv_chunk_bytes(long long bytes) {
  g_chunk_bytes = bytes > 0 ? std::min(bytes, 0x7f000000LL) : 0x7f000000LL;
  return g_chunk_bytes;
}

extern "C" int kv_conv2d(const KvConvParams* p, int tile, hipStream_t stream) {
#ifdef KVEDGE_CHECKS
  if (const int rc = kv_conv_check_extents(p)) return rc;
#endif
  const long long kChunkBytes = g_chunk_bytes;
  const long long per = kv_conv_max_image_bytes(p);
  if (per <= 0 || per >= kChunkBytes) return per <= 0 ? -1 : -9;
  const long long cap = kChunkBytes / per;
  if (p->N <= cap) return kv_conv2d_one(p, tile, stream);
  const long long hw = (long long)p->H * p->W, ohw = (long long)p->Ho * p->Wo;
  for (int n0 = 0; n0 < p->N; n0 += (int)cap) {
    KvConvParams q = *p;
    q.N = (int)std::min<long long>(cap, p->N - n0);
    q.M = (int)(q.N * ohw);
    auto adv = [&](const void* b, long long bytes_per_image) -> const char* {
      return b ? static_cast<const char*>(b) + (long long)n0 * bytes_per_image : nullptr;
    };
    q.x = adv(p->x, p->in_u8 ? hw * 12 : hw * p->ldx * 2);
    q.y = const_cast<char*>(adv(p->y, ohw * p->ldy * 2));
    if (p->res) q.res = adv(p->res, ohw * p->ldr * 2);
    if (p->mode == 4) q.x2 = adv(p->x2, (long long)p->H2 * p->W2 * p->ldx2 * 2);
    if (p->n_t) q.z = const_cast<char*>(adv(p->z, ohw * p->ldz * 2));
    if (const int rc = kv_conv2d_one(&q, tile, stream)) return rc;
  }
  return 0;
}

static int kv_conv2d_one(const KvConvParams* p, int tile, hipStream_t stream) {
  if (p->Kpad % BK != 0 || p->Cout % 8 != 0) return -1;
  if (p->n_t) {  // fused bottleneck tail: v3 tail tiles (Cout 256) or v9 seam tiles
    const int v3 = kNumTiles + glds_num_tiles();
    const int v9 = kv_conv_num_tiles();
    if (tile < 0) {
      if (p->Cout == 256) {
        tile = v3 + stream_tail_tile(p->n_t);
      } else {
        const int s = seam_pick_tile(p);
        if (s < 0) return -8;
        tile = v9 + s;
      }
    }
    if (tile >= v9) return seam_launch(p, tile - v9, stream);
    if (tile < v3 || tile >= v3 + stream_num_tiles()) return -8;
    return stream_launch(p, tile - v3, stream);
  }
  if (p->in_u8) {  // frames-in s2d stem: the direct family only
    const int v4 = kNumTiles + glds_num_tiles() + stream_num_tiles();
    if (tile >= 0 && tile < v4) return -8;
    return direct_launch(p, tile < 0 ? 0 : tile - v4, stream);
  }
  if (p->mode == 2 && (p->Cin != 4 || p->ldx != 4)) return -2;
  if (p->mode != 2 && (p->Cin % 8 != 0 || p->ldx % 8 != 0 || p->x_coff % 8 != 0)) return -3;
  if (p->mode == 1 && (p->KH != 1 || p->KW != 1 || p->stride != 1 || p->pad != 0)) return -4;
  if ((p->ldy % 8) || (p->y_coff % 8) || (p->res && ((p->ldr % 8) || (p->r_coff % 8)))) return -5;
  if (p->mode == 4) {  // dual-source (fused downsample): v2 LDS-DMA family only
    if (tile < 0) {
      const long long nwg128 = ((p->M + 127) / 128) * ((p->Cout + 127) / 128);
      tile = kNumTiles + (nwg128 >= 512 ? 0 : 4);
    }
    if (tile < kNumTiles) return -8;
  }
  if (tile < 0) tile = kv_conv_pick_tile(p);
  const int v3 = kNumTiles + glds_num_tiles();
  const int v4 = v3 + stream_num_tiles();
  const int v6 = v4 + direct_num_tiles();
  const int v7 = v6 + nloop_num_tiles();
  const int v8 = v7 + xp_num_tiles();
  const int v10 = v8 + sk_num_tiles();
  const int v12 = v10 + direct_de_num_tiles();
  const int v14 = v12 + skinny_num_tiles();
  if (tile >= v14 + pp_num_tiles()) return -6;
  if (tile >= v14) return pp_launch(p, tile - v14, stream);
  if (tile >= v12) return skinny_launch(p, tile - v12, stream);
  if (tile >= v10) return direct_de_launch(p, tile - v10, stream);
  if (tile >= v8) return sk_launch(p, tile - v8, stream);
  if (tile >= v7) return xp_launch(p, tile - v7, stream);
  if (tile >= v6) return nloop_launch(p, tile - v6, stream);
  if (tile >= v4) return direct_launch(p, tile - v4, stream);
  if (tile >= v3) return stream_launch(p, tile - v3, stream);
  if (tile >= kNumTiles) return glds_launch(p, tile - kNumTiles, stream);
  const TileEntry& e = kTiles[tile];
  const long long nwg = (long long)((p->M + e.cfg.bm - 1) / e.cfg.bm) *
                        ((p->Cout + e.cfg.bn - 1) / e.cfg.bn);
  if (nwg <= 0) return 0;
  ConvKernelFn fn = e.get(p->mode);
  hipLaunchKernelGGL(fn, dim3((unsigned)nwg), dim3(256), 0, stream, *p);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}
