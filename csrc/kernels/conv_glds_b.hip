// v2 tile table, second half (narrow-N, BN 96, 8-wave and MF 16 forms): its own translation
// unit so it compiles beside conv_glds.hip.
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {


const GldsTile kGldsTilesB[] = {
    // narrow N (YOLO's 16/32-channel layers at 160^2 / 320^2): BN = 32, 4 waves along M
    {128, 32, &glds_get<128, 32, 4, 1>},
    {256, 32, &glds_get<256, 32, 4, 1>},
    // BN = 96 (3 x 32-wide MFMA blocks per wave, 4 waves along M): YOLO's 80-channel Detect
    // cls convs waste 17 % of the MFMA columns here instead of 37.5 % on a BN = 128 tile
    {128, 96, &glds_get<128, 96, 4, 1>},
    {256, 96, &glds_get<256, 96, 4, 1>},
    // 8 waves (512 threads), one workgroup per CU, two waves per SIMD: 256x256 with a
    // 128x64 / 64x128 sub-tile per wave (epilogue in two column passes), and 256x128 /
    // 128x256 with 64x64 per wave but the B / A tile shared by twice the waves
    {256, 256, &glds_get<256, 256, 2, 4>, 512},
    {256, 256, &glds_get<256, 256, 4, 2>, 512},
    {256, 128, &glds_get<256, 128, 4, 2>, 512},
    {128, 256, &glds_get<128, 256, 2, 4>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 3>, 512},
    // the same loops on v_mfma_f32_16x16x32_bf16 (MF = 16)
    {128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16>},
    {256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 2, 64, 16>, 512},
    // (BK = 32 rings -- glds_get<128, 128, 2, 2, 5, 32> etc., 4-5 K steps in flight at 2
    // workgroups per CU -- measured 10-40 % SLOWER than {128, 128} D = 2 on every 3x3 and
    // 1x1 layer of ResNet-50 at batch 640 (profiles/r1_v10_tile_probe_bk32.md): the 3x3
    // layers are not L2-latency-bound, so they are not instantiated)
};

}  // namespace

int glds_b_num_tiles() { return (int)(sizeof(kGldsTilesB) / sizeof(kGldsTilesB[0])); }
int glds_b_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= glds_b_num_tiles()) return -6;
  return glds_launch_entry(p, kGldsTilesB[tile], stream);
}
int glds_b_tile_bm(int tile) { return kGldsTilesB[tile].bm; }
int glds_b_tile_bn(int tile) { return kGldsTilesB[tile].bn; }

}  // namespace kvedge
