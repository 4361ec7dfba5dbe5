// Host-visible launcher ABI of libkvedge kernels (gfx950 only).
//
// The kernels take raw device pointers and a hipStream_t so they can be driven
// from the torch binding (csrc/bindings/ops.cpp), from native C++ tools and from
// hipGraph capture alike.  Every launcher is capture-safe: no allocation, no
// synchronisation, no host<->device copies (cdna_hip_programming.md G9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---------------------------------------------------------------------------
// K1/K2/K3: implicit-GEMM convolution / GEMM on MFMA, NHWC bf16, fp32 accumulate
//   y[m, y_coff + n] = act( sum_k A[m,k] * W[n,k] + bias[n] + res[m, n] )
//   m = (img, ho, wo), k = (r, s, c).  BN is folded into W/bias at load time.
// ---------------------------------------------------------------------------
typedef struct KvConvParams {
  const void* x;      // bf16 input, pixel stride ldx elements, channel offset x_coff
  const void* w;      // bf16 packed weights [Cout][Kpad]
  const float* bias;  // fp32 [Cout] or NULL
  const void* res;    // bf16 residual [M][ldr] or NULL
  void* y;            // bf16 output, row stride ldy, channel offset y_coff
  int N, H, W, Cin;   // input geometry (Cin = logical channels read)
  int ldx, x_coff;
  int Ho, Wo, Cout;
  int KH, KW, stride, pad;
  int K, Kpad;        // logical and padded (multiple of 64) reduction length
  int M;              // N*Ho*Wo
  int ldy, y_coff, ldr, r_coff;
  int act;            // bits[1:0]: 0 none, 1 relu, 2 silu; bit 2: residual after act
  int mode;           // 0 general, 1 1x1/s1/p0 GEMM, 2 stem (Cin=4, KW padded even),
                      // 4 dual 1x1 (bottleneck conv3 + fused downsample, v2 tiles only)
  // mode 4 second source: k in [K1, K) reads x2 [N, H2, W2, ldx2] at stride stride2
  // (the bottleneck's input, i.e. the downsample branch folded in as extra K).
  const void* x2;
  int K1, H2, W2, ldx2, stride2;
  // in_u8 = 1: x is uint8 RGB frames [N, 2H, 2W, 3] and the conv reads their
  // space-to-depth image [N, H, W, 16] (channel (dy*2+dx)*4 + c, channel 3 zero) built on
  // the fly -- the preprocess pass is fused away (v4 direct tile, 2x2 s2d stem only).
  int in_u8;
  // Fused bottleneck tail (v3 streaming tail tile, BN == Cout): after y is written,
  // z = ReLU(y . w_t^T + bias_t) -- the NEXT block's 1x1 reduce conv -- is computed from
  // the y tile still in LDS (w_t: bf16 [n_t][Cout], resident) and written to
  // z[m * ldz + z_coff + n]: y is never re-read from HBM.  n_t = 0: no tail.
  // pair_1x1 = 1 (v4 direct tiles, 3x3 stride 1): the same fields describe a 1x1 conv
  // (w_t [n_t][Cout], bias_t, no activation) applied to the 3x3's activated output, whose
  // result goes to z; y is not written (YOLO Detect branch pairs).
  const void* w_t;
  const float* bias_t;
  void* z;
  int n_t, ldz, z_coff, act_t;
  int pair_1x1;
  // Split-K (v8 tiles, small-M layers: edge batches): K slice z of the launch writes its fp32
  // partial sums to slab z of ws [ksplit][M][Cout] with plain 16-B stores, and a finalize
  // kernel sums the slabs, applies bias, residual and activation and writes y.  ws = NULL:
  // v8 tiles refuse.  (ksplit is set by the tile; ws must hold ksplit x M x Cout floats.)
  float* ws;
  int ksplit;
  long long ws_elems;  // floats in ws
  // mode 4, second source extras (YOLO neck): channel offset of x2's slice, and up2 = 1: x2
  // is a half-resolution map read at (ho / 2, wo / 2) -- the nearest 2x upsample of the
  // concat folded into the GEMM (H2 = Ho / 2).  v2 LDS-DMA tiles (and their v7 / v8 forms)
  // only; every other family refuses.
  int x2_coff;
  int up2;
} KvConvParams;

// tile: -1 = heuristic; otherwise an index into the tile table (kv_conv_num_tiles()).
int kv_conv2d(const KvConvParams* p, int tile, hipStream_t stream);
// image-chunk size of kv_conv2d launches (bytes per operand per launch); 0 = default
long long kv_set_conv_chunk_bytes(long long bytes);
int kv_conv_num_tiles(void);
int kv_conv_splitk_base(void);       // split-K tiles: [base, base + splitk_num_tiles)
int kv_conv_splitk_num_tiles(void);
// host replay of the v6 (conv_nloop.hip) counted-wait schedules: 0 = every tile is safe
int kv_nloop_sched_check(void);
int kv_conv_pick_tile(const KvConvParams* p);
// v9 seam tiles (conv3 + residual -> next conv1, p->n_t set): valid tile arguments of a tail
// call are kv_conv_num_tiles() + i, i < kv_conv_seam_num_tiles()
int kv_conv_seam_num_tiles(void);
// Fused 3x3 + 1x1 pair on the v4 direct family (p->pair_1x1 = 1, see KvConvParams): tile =
// direct tile 0-3; < 0 when no instantiation covers the shape.
int kv_conv_pair(const KvConvParams* p, int tile, hipStream_t stream);
int kv_conv_pair_num_tiles(void);

// K5: max pool NHWC (k x k, stride, pad); C % 8 == 0.  ldx/ldy allow channel slices.
// Fused ResNet stem (4x4 stride-1 conv over the s2d image [N,H,W,16], Cout 64, weights
// [64][256] packed, bias, ReLU) + 3x3/2 max pool -> y [N,(H+1)/2,(W+1)/2,ldy] at y_coff.
int kv_stem_pool(const void* x, const void* w, const float* bias, void* y, int N, int H, int W,
                 int ldy, int y_coff, hipStream_t s);
int kv_stem_pool_lds_bytes(int W);
int kv_stem_pool_frames(const void* frames, const void* w, const float* bias, void* y, int N,
                        int H0, int W0, const float* mean3, const float* inv_std3, int ldy,
                        int y_coff, hipStream_t s);
// second-generation frames-in stem + pool (stem12.hip): 12-channel s2d, K = 192, w [64][192]
int kv_stem12_pool_frames(const void* frames, const void* w, const float* bias, void* y, int N,
                          int H0, int W0, const float* mean3, const float* inv_std3, int ldy,
                          int y_coff, hipStream_t s);
int kv_stem12_lds_bytes(int Ws);
// YOLOv8n b0 + b1 fused from raw frames (yolo_stem2.hip): w0 [16][64] frames-in s2d stem,
// w1 [32][w1_ld] 3x3/2 16 -> 32; y [N, H0/4, W0/4, 32]
int kv_yolo_stem2(const void* frames, const void* w0, const float* bias0, const void* w1,
                  int w1_ld, const float* bias1, void* y, int N, int H0, int W0, hipStream_t s);
int kv_yolo_stem2_lds_bytes(int Ws);

int kv_maxpool2d(const void* x, void* y, int N, int H, int W, int C, int ldx, int x_coff,
                 int ldy, int y_coff, int k, int stride, int pad, int Ho, int Wo, hipStream_t s);
// K5b: YOLOv8 SPPF: buf holds [x | y1 | y2 | y3] channel slices (4*C wide); x is
// already written in slice 0; writes y1=mp5(x), y2=mp5(y1), y3=mp5(y2) in one pass.
int kv_sppf_pool(void* buf, int N, int H, int W, int C, hipStream_t s);
// K6: global average pool NHWC -> [N, C] bf16.
int kv_global_avgpool(const void* x, void* y, int N, int HW, int C, hipStream_t s);
// K6+K1 at edge batches: y[n, :ncls] = bf16(fc(bf16(mean over HW of x[n]))), x [N, HW, C] bf16,
// w [ncls][ldw] bf16 (packed 1x1 conv weight), bias fp32 [ncls] or NULL.
int kv_pooled_fc(const void* x, int N, int HW, int C, const void* w, int ldw, const float* bias,
                 void* y, int ncls, hipStream_t s);
// K7: row softmax, bf16 [rows, cols] -> fp32 probabilities; also writes argmax.
int kv_softmax_rows(const void* x, float* y, int64_t* argmax, int rows, int cols, hipStream_t s);
// K8: nearest 2x upsample of x [N,H,W,C] written into channel slice of y [N,2H,2W,ldy].
int kv_upsample2x(const void* x, void* y, int N, int H, int W, int C, int ldx, int x_coff,
                  int ldy, int y_coff, hipStream_t s);
// K9: YOLOv8 decode (DFL softmax + expectation + dist2bbox + class sigmoid/max).
//   feats: per level bf16 [N, HW_l, 64 + nc]; out boxes fp32 [N, A, 4] xyxy,
//   scores fp32 [N, A], cls int32 [N, A].  A = sum HW_l.
int kv_yolo_decode(const void* f0, const void* f1, const void* f2, int h0, int w0, int h1,
                   int w1, int h2, int w2, int s0, int s1, int s2, int N, int nc,
                   float* boxes, float* scores, int* cls, hipStream_t s);
// K10: class-aware NMS per image: score threshold, sort, greedy IoU suppression,
//   keep <= max_det.  out fp32 [N, max_det, 6] (x1,y1,x2,y2,score,cls); count int32 [N].
int kv_nms(const float* boxes, const float* scores, const int* cls, int N, int A,
           float conf_thres, float iou_thres, int max_det, float* out, int* count,
           hipStream_t s);
// K11: on-device synthetic camera frames, uint8 NHWC3, deterministic in (seed, step).
int kv_synth_frames(uint8_t* y, int N, int H, int W, uint64_t seed, uint64_t step,
                    hipStream_t s);
// K11b: same but the step counter is read from device memory and incremented, so a
// captured hipGraph produces fresh frames on every replay.  bump_done = 1: step[1] is a
// zeroed finished-block count and the kernel's last block advances step[0] (one launch);
// 0: a one-thread kernel after it does.
int kv_synth_frames_dev(uint8_t* y, int N, int H, int W, uint64_t seed, uint64_t* step,
                        int bump_done, hipStream_t s);
// K12: uint8 NHWC3 -> bf16 NHWC4 normalized ((x/255 - mean)/std), channel 3 = 0.
int kv_preprocess(const uint8_t* x, void* y, int N, int H, int W, const float* mean3,
                  const float* inv_std3, hipStream_t s);
// K12b: uint8 NHWC3 -> bf16 space-to-depth [N, H/2, W/2, 16] normalized
//   (channel (dy*2+dx)*4 + c, c == 3 zero) for the stride-1 s2d stem conv.
int kv_preprocess_s2d(const uint8_t* x, void* y, int N, int H, int W, const float* mean3,
                      const float* inv_std3, hipStream_t s);
// K4 fallback: y = x*scale[c] + shift[c] (+relu) on NHWC bf16.
int kv_batchnorm_nhwc(const void* x, void* y, const float* scale, const float* shift,
                      int64_t rows, int C, int relu, hipStream_t s);

// ---------------------------------------------------------------------------
// v13 fused YOLOv8 C2f(32, 32, n=1, shortcut) (c2f_fused.hip): t = SiLU(W1 . x + b1) (a =
// t[:16], s = t[16:]), u = SiLU(conv3x3(s) + bm1), v = s + SiLU(conv3x3(u) + bm2),
// y = SiLU(W2 . [a, s, v] + b2); NHWC bf16, x [N, H, W, ldx] at x_coff (32 channels), y at
// y_coff (32); packed weights w1 [32][ldw1], wm1 / wm2 [16][ldwm] (tap-major, cin minor),
// w2 [32][ldw2]; fp32 biases.  S: output rows per workgroup (a multiple of 4 dividing H).
// ---------------------------------------------------------------------------
typedef struct KvC2fParams {
  const void* x;
  void* y;
  const void* w1;
  const float* b1;
  const void* wm1;
  const float* bm1;
  const void* wm2;
  const float* bm2;
  const void* w2;
  const float* b2;
  int N, H, W, ldx, x_coff, ldy, y_coff;
  int ldw1, ldwm, ldw2;
  int S;
} KvC2fParams;
int kv_c2f16_supported(int H, int W, int S);
int kv_c2f16_fused(const KvC2fParams* p, hipStream_t stream);

#ifdef __cplusplus
}
#endif
