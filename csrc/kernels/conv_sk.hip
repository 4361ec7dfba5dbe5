// v8: split-K (edge batches: few output tiles, long K).  (instantiation, K slices)
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {

// split-K finalize: y = act2(act1(ws + bias) (+ res)) -> bf16, and ws = 0 for the next layer
__global__ __launch_bounds__(256) void splitk_finalize_kernel(
    float* __restrict__ ws, const float* __restrict__ bias, const bf16* __restrict__ res,
    bf16* __restrict__ y, int M, int Cout, int ldy, int y_coff, int ldr, int r_coff, int act) {
  const int cpr = Cout >> 3;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)M * cpr) return;
  const int m = (int)(idx / cpr), c = (int)(idx - (long long)m * cpr) * 8;
  float4* src = reinterpret_cast<float4*>(ws + (size_t)m * Cout + c);
  const float4 a0 = src[0], a1 = src[1];
  src[0] = make_float4(0.f, 0.f, 0.f, 0.f);
  src[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  if (bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  bf16x8 o;
  dispatch_act(act, res != nullptr, [&](auto A1, auto A2) __attribute__((always_inline)) {
    constexpr int act1 = decltype(A1)::value, act2 = decltype(A2)::value;
    bf16x8 r;
    if (res) r = *reinterpret_cast<const bf16x8*>(res + (size_t)m * ldr + r_coff + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float u = act_c<act1>(v[e]);
      if (res) u = act_c<act2>((float)f2bf(u) + (float)r[e]);
      o[e] = f2bf(u);
    }
  });
  *reinterpret_cast<bf16x8*>(y + (size_t)m * ldy + y_coff + c) = o;
}

struct SkTile {
  GldsTile t;
  int split;
};
const SkTile kSkTiles[] = {
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{64, 64, &glds_get<64, 64, 2, 2, 2, 64, 32, false, false, true>}, 16},
    {{128, 64, &glds_get<128, 64, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{128, 64, &glds_get<128, 64, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{64, 128, &glds_get<64, 128, 2, 2, 2, 64, 32, false, false, true>}, 4},
    {{64, 128, &glds_get<64, 128, 2, 2, 2, 64, 32, false, false, true>}, 8},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 2},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 4},
    {{128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, false, true>}, 8},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 2},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 4},
    {{256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, false, true>, 512}, 8},
};

}  // namespace

int sk_num_tiles() { return (int)(sizeof(kSkTiles) / sizeof(kSkTiles[0])); }

int sk_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= sk_num_tiles()) return -6;
  const SkTile& e = kSkTiles[tile];
  const int nk = p->Kpad / BK;
  if (!p->ws) return -11;  // split-K needs the caller's zeroed fp32 workspace
  KvConvParams q = *p;
  q.ksplit = e.split < nk ? e.split : nk;  // never more slices than K steps
  if (const int rc = glds_launch_entry(&q, e.t, stream, q.ksplit)) return rc;
  const long long thr = (long long)p->M * (p->Cout / 8);
  if (thr <= 0) return 0;
  hipLaunchKernelGGL(splitk_finalize_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0,
                     stream, p->ws, p->bias, (const bf16*)p->res, (bf16*)p->y, p->M, p->Cout,
                     p->ldy, p->y_coff, p->ldr, p->r_coff, p->act);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
