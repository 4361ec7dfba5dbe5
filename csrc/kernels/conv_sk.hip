// v8: split-K (edge batches: few output tiles, long K).  (instantiation, K slices)
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {

// split-K finalize: y = act2(act1(sum over the KS slabs + bias) (+ res)) -> bf16.  KS is a
// template argument so every slab load of a thread is issued before the first add: the
// runtime-count loop kept one slab pair in flight, i.e. KS dependent memory latencies per
// launch (~5 us at batch 1 for the 16-slice layers)
template <int KS>
__global__ __launch_bounds__(256) void splitk_finalize_kernel(const KvConvParams p) {
  const int cpr = p.Cout >> 3;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)p.M * cpr) return;
  const int m = (int)(idx / cpr), c = (int)(idx - (long long)m * cpr) * 8;
  const size_t slab = (size_t)p.M * p.Cout;
  const float* src = p.ws + (size_t)m * p.Cout + c;
  float4 a[KS][2];
#pragma unroll
  for (int z = 0; z < KS; ++z) {
    a[z][0] = *reinterpret_cast<const float4*>(src + z * slab);
    a[z][1] = *reinterpret_cast<const float4*>(src + z * slab + 4);
  }
#pragma unroll
  for (int w = 1; w < KS; w <<= 1)  // pairwise tree
#pragma unroll
    for (int z = 0; z + w < KS; z += 2 * w)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        a[z][h].x += a[z + w][h].x;
        a[z][h].y += a[z + w][h].y;
        a[z][h].z += a[z + w][h].z;
        a[z][h].w += a[z + w][h].w;
      }
  float v[8] = {a[0][0].x, a[0][0].y, a[0][0].z, a[0][0].w,
                a[0][1].x, a[0][1].y, a[0][1].z, a[0][1].w};
  sk_finish8(p, m, c, v);
}

struct SkTile {
  GldsTile t;
  int split;
};
// D = 2 forms first (indices of earlier rounds' tuning caches stay valid), then the D = 4
// rings (three K steps in flight: a slice of a batch-1 layer is latency-bound on its few
// K steps) and 32-way splits for the 72-step stage-4 3x3
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
    {{64, 64, &glds_get<64, 64, 2, 2, 4, 64, 32, false, false, true>}, 8},
    {{64, 64, &glds_get<64, 64, 2, 2, 4, 64, 32, false, false, true>}, 16},
    {{64, 64, &glds_get<64, 64, 2, 2, 4, 64, 32, false, false, true>}, 32},
    {{128, 64, &glds_get<128, 64, 2, 2, 4, 64, 32, false, false, true>}, 8},
    {{64, 128, &glds_get<64, 128, 2, 2, 4, 64, 32, false, false, true>}, 8},
    {{64, 128, &glds_get<64, 128, 2, 2, 4, 64, 32, false, false, true>}, 16},
};

}  // namespace

int sk_num_tiles() { return (int)(sizeof(kSkTiles) / sizeof(kSkTiles[0])); }
int sk_tile_split(int tile) { return tile >= 0 && tile < sk_num_tiles() ? kSkTiles[tile].split : 0; }

int sk_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= sk_num_tiles()) return -6;
  const SkTile& e = kSkTiles[tile];
  const int nk = p->Kpad / BK;
  if (!p->ws) return -11;  // split-K needs the caller's fp32 slab workspace
  KvConvParams q = *p;
  q.ksplit = e.split;  // never more slices than K steps (halved: the finalize is templated
  while (q.ksplit > nk) q.ksplit >>= 1;  // on power-of-two slice counts)
  if ((long long)q.ksplit * p->M * p->Cout > p->ws_elems || p->Cout % 8) return -12;
  if (const int rc = glds_launch_entry(&q, e.t, stream, q.ksplit)) return rc;
  const long long thr = (long long)p->M * (p->Cout / 8);
  if (thr <= 0) return 0;
  const dim3 g((unsigned)((thr + 255) / 256));
  switch (q.ksplit) {
    case 1: hipLaunchKernelGGL(splitk_finalize_kernel<1>, g, dim3(256), 0, stream, q); break;
    case 2: hipLaunchKernelGGL(splitk_finalize_kernel<2>, g, dim3(256), 0, stream, q); break;
    case 4: hipLaunchKernelGGL(splitk_finalize_kernel<4>, g, dim3(256), 0, stream, q); break;
    case 8: hipLaunchKernelGGL(splitk_finalize_kernel<8>, g, dim3(256), 0, stream, q); break;
    case 16: hipLaunchKernelGGL(splitk_finalize_kernel<16>, g, dim3(256), 0, stream, q); break;
    case 32: hipLaunchKernelGGL(splitk_finalize_kernel<32>, g, dim3(256), 0, stream, q); break;
    default: return -13;  // a split clamped to a K-step count that is no power of two
  }
  return hipGetLastError() == hipSuccess ? 0 : -7;
}

}  // namespace kvedge
