// K1/K2/K3 v2 tile table, first half (kernel body: conv_glds_kernel.inc; second half of
// the table: conv_glds_b.hip).
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {


const GldsTile kGldsTiles[] = {
    {128, 128, &glds_get<128, 128, 2, 2>},
    {128, 64, &glds_get<128, 64, 2, 2>},
    {64, 64, &glds_get<64, 64, 2, 2>},
    {256, 64, &glds_get<256, 64, 4, 1>},
    {64, 128, &glds_get<64, 128, 2, 2>},
    {256, 128, &glds_get<256, 128, 2, 2>},
    {128, 256, &glds_get<128, 256, 2, 2>},
    // deeper rings (3-4 K steps in flight); indices above are kept stable
    {128, 128, &glds_get<128, 128, 2, 2, 3>},
    {128, 64, &glds_get<128, 64, 2, 2, 3>},
    {64, 128, &glds_get<64, 128, 2, 2, 3>},
    {64, 64, &glds_get<64, 64, 2, 2, 4>},
    {128, 64, &glds_get<128, 64, 2, 2, 4>},
    // 128x64 / 64x128 per wave (0.75 fragment reads per MFMA instead of 1.0: the 3x3
    // layers are LDS-bandwidth-bound at 64x64 per wave), one workgroup per CU, 3 slots
    {256, 128, &glds_get<256, 128, 2, 2, 3>},
    {128, 256, &glds_get<128, 256, 2, 2, 3>},
};

}  // namespace

int glds_b_num_tiles();
int glds_b_launch(const KvConvParams* p, int tile, hipStream_t stream);
int glds_b_tile_bm(int tile);
int glds_b_tile_bn(int tile);

static constexpr int kNa = (int)(sizeof(kGldsTiles) / sizeof(kGldsTiles[0]));
int glds_num_tiles() { return kNa + glds_b_num_tiles(); }

int glds_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= glds_num_tiles()) return -6;
  if (tile >= kNa) return glds_b_launch(p, tile - kNa, stream);
  return glds_launch_entry(p, kGldsTiles[tile], stream);
}

int glds_tile_bm(int tile) { return tile < kNa ? kGldsTiles[tile].bm : glds_b_tile_bm(tile - kNa); }
int glds_tile_bn(int tile) { return tile < kNa ? kGldsTiles[tile].bn : glds_b_tile_bn(tile - kNa); }

}  // namespace kvedge
