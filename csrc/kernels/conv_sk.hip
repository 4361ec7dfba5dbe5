// v8: split-K (edge batches: few output tiles, long K).  (instantiation, K slices)
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {

// split-K finalize (sk_cnt == NULL): y = act2(act1(ws + bias) (+ res)) -> bf16, ws = 0 again
__global__ __launch_bounds__(256) void splitk_finalize_kernel(const KvConvParams p) {
  const int cpr = p.Cout >> 3;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)p.M * cpr) return;
  const int m = (int)(idx / cpr), c = (int)(idx - (long long)m * cpr) * 8;
  float4* src = reinterpret_cast<float4*>(p.ws + (size_t)m * p.Cout + c);
  const float4 a0 = src[0], a1 = src[1];
  src[0] = make_float4(0.f, 0.f, 0.f, 0.f);
  src[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  sk_finish8(p, m, c, v);
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
  const long long tiles = (long long)((p->M + e.t.bm - 1) / e.t.bm) * ((p->Cout + e.t.bn - 1) / e.t.bn);
  if (q.sk_cnt && tiles > KV_SK_COUNTERS) return -12;  // one arrival counter per output tile
  if (const int rc = glds_launch_entry(&q, e.t, stream, q.ksplit)) return rc;
  if (q.sk_cnt) return 0;  // the last slice of each tile finished it in-kernel
  const long long thr = (long long)p->M * (p->Cout / 8);
  if (thr <= 0) return 0;
  hipLaunchKernelGGL(splitk_finalize_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0,
                     stream, q);
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
