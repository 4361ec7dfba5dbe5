// v7: the XP (cross-stage pipelined) main loop on BK = 32 rings, v_mfma_f32_16x16x32.
// Own index range after v6 so the older families keep their indices.
#include "conv_glds_kernel.inc"

namespace kvedge {
namespace {


const GldsTile kXpTiles[] = {
    {256, 256, &glds_get<256, 256, 2, 4, 4, 32, 16, true>, 512},  // 128 px x 64 ch per wave
    {256, 256, &glds_get<256, 256, 4, 2, 4, 32, 16, true>, 512},  // 64 px x 128 ch per wave
    {256, 256, &glds_get<256, 256, 2, 4, 5, 32, 16, true>, 512},  // 4 stages in flight
    {256, 256, &glds_get<256, 256, 4, 2, 5, 32, 16, true>, 512},
    {256, 128, &glds_get<256, 128, 4, 2, 6, 32, 16, true>, 512},  // N = 128 layers, 64 x 64
    {128, 256, &glds_get<128, 256, 2, 4, 6, 32, 16, true>, 512},
    // the plain ring loop on BK = 32 with the MF = 16 conflict-free swizzle (the round-1/2
    // BK = 32 rings were measured with a 2-way conflicted one); 4-wave forms fit <= 80 KB of
    // LDS, so two workgroups -- of this launch or of the other stream's -- share a CU and
    // one's epilogue overlaps the other's main loop
    {256, 256, &glds_get<256, 256, 4, 2, 4, 32, 16>, 512},        // 128 KB
    {256, 128, &glds_get<256, 128, 2, 2, 3, 32, 16>},             // 72 KB, 128 x 64 per wave
    {128, 256, &glds_get<128, 256, 2, 2, 3, 32, 16>},             // 72 KB, 64 x 128 per wave
    {128, 128, &glds_get<128, 128, 2, 2, 4, 32, 16>},             // 64 KB
    {128, 128, &glds_get<128, 128, 2, 2, 5, 32, 16>},             // 80 KB
    {256, 128, &glds_get<256, 128, 4, 2, 4, 32, 16>, 512},        // 96 KB
    // direct register epilogue (DE: v_permlane16_swap -> 16-B stores, no LDS C tile, no
    // epilogue barrier) on the best 8-wave forms and the 2-per-CU 256 x 128
    {256, 256, &glds_get<256, 256, 4, 2, 2, 64, 16, false, true>, 512},
    {256, 256, &glds_get<256, 256, 2, 4, 5, 32, 16, true, true>, 512},
    {256, 128, &glds_get<256, 128, 2, 2, 3, 32, 16, false, true>},
    {128, 128, &glds_get<128, 128, 2, 2, 2, 64, 16, false, true>},
    // N = 144 (YOLO Detect branch stems, box 64 + cls 80): a 160-wide N tile (ten 16x16
    // blocks per wave, 4 x 1 waves of 32 px) computes 10 % padding channels where 128- and
    // 256-wide tiles computed 44 %; B rows past Cout are zero-filled by the range check
    {128, 160, &glds_get<128, 160, 4, 1, 2, 64, 16, false, true>},
    {128, 160, &glds_get<128, 160, 4, 1, 3, 64, 16, false, true>},
};

}  // namespace

int xp_num_tiles() { return (int)(sizeof(kXpTiles) / sizeof(kXpTiles[0])); }

int xp_launch(const KvConvParams* p, int tile, hipStream_t stream) {
  if (tile < 0 || tile >= xp_num_tiles()) return -6;
  return glds_launch_entry(p, kXpTiles[tile], stream);
}

}  // namespace kvedge
