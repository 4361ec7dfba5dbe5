// N14: torch custom-op bindings for the gfx950 kernel library (TORCH_LIBRARY "kvedge").
//
// Every op writes into caller-provided output tensors (schema `Tensor(a!)`), runs
// on torch's current HIP stream, allocates nothing and never synchronises, so a
// whole forward built from these ops can be captured into one hipGraph
// (kvedge_amd/engine).  Shapes/strides are computed by the Python wrappers in
// kvedge_amd/ops/__init__.py; this layer only validates and launches.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../kernels/kvedge_kernels.h"

namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "kvedge: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "kvedge: ", name, " must be contiguous");
}

void check_bf16(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "kvedge: ", name, " must be bf16");
}

// Split-K workspace: fp32 slabs, one per K slice of the tile ([ksplit][M][Cout]); the
// launcher refuses a tile whose slabs do not fit (ops.splitk_workspace sizes it per tile).
void set_splitk_ws(KvConvParams& p, const at::Tensor& ws) {
  p.ws = ws.data_ptr<float>();
  p.ws_elems = ws.numel();
}

void conv(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
          const c10::optional<at::Tensor>& res, at::Tensor& y, int64_t N, int64_t H, int64_t W,
          int64_t Cin, int64_t ldx, int64_t x_coff, int64_t Ho, int64_t Wo, int64_t Cout,
          int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t K, int64_t ldy,
          int64_t y_coff, int64_t ldr, int64_t r_coff, int64_t act, int64_t mode,
          int64_t tile, const c10::optional<at::Tensor>& ws) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  const c10::DeviceGuard g(x.device());
  KvConvParams p{};
  if (ws.has_value() && ws->defined()) {  // split-K workspace (v8 tiles): fp32, zero, >= M*Cout
    check_dev(*ws, "ws");
    TORCH_CHECK(ws->scalar_type() == at::kFloat, "kvedge: split-K workspace fp32");
    set_splitk_ws(p, *ws);
  }
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "kvedge: bias fp32[Cout]");
    p.bias = bias->data_ptr<float>();
  }
  p.res = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16(*res, "res");
    p.res = res->data_ptr();
  }
  p.y = y.data_ptr();
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.Cin = (int)Cin;
  p.ldx = (int)ldx; p.x_coff = (int)x_coff;
  p.Ho = (int)Ho; p.Wo = (int)Wo; p.Cout = (int)Cout;
  p.KH = (int)KH; p.KW = (int)KW; p.stride = (int)stride; p.pad = (int)pad;
  p.K = (int)K;
  TORCH_CHECK(w.dim() == 2 && w.size(0) == Cout, "kvedge: packed weight must be [Cout, Kpad]");
  p.Kpad = (int)w.size(1);
  p.M = (int)(N * Ho * Wo);
  p.ldy = (int)ldy; p.y_coff = (int)y_coff; p.ldr = (int)ldr; p.r_coff = (int)r_coff;
  p.act = (int)act; p.mode = (int)mode;
  // bounds: every operand inside its tensor.  No whole-tensor size cap: kv_conv2d splits
  // batches whose operands exceed 2 GiB into image chunks (32-bit in-kernel offsets)
  TORCH_CHECK(N > 0 && H * W * ldx * 2 < (1ll << 31) && Ho * Wo * ldy * 2 < (1ll << 31),
              "kvedge: one image's activations exceed 2 GiB");
  TORCH_CHECK(x.numel() >= N * H * W * ldx, "kvedge: x smaller than N*H*W*ldx");
  TORCH_CHECK(x_coff >= 0 && x_coff + Cin <= ldx, "kvedge: x channel slice out of range");
  TORCH_CHECK(y.numel() >= (int64_t)p.M * ldy && y_coff + Cout <= ldy, "kvedge: y too small");
  if (p.res) TORCH_CHECK(res->numel() >= (int64_t)p.M * ldr && r_coff + Cout <= ldr, "kvedge: residual too small");
  const int rc = kv_conv2d(&p, (int)tile, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: kv_conv2d failed rc=", rc);
}

// Fused Detect-branch pair (v4 direct tiles): z[.., z_coff : z_coff + C2] =
//   act(conv3x3/1(x[.., x_coff : x_coff + Cin]) + bias) . W2^T + b2
// t = the 3x3's activated output stays in LDS (never written); tile = v4 direct tile 0-3.
void conv_pair(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias,
               const at::Tensor& w2, const at::Tensor& b2, at::Tensor& z, int64_t Cin,
               int64_t x_coff, int64_t z_coff, int64_t act, int64_t tile) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(w2, "w2");
  check_bf16(z, "z");
  check_dev(bias, "bias");
  check_dev(b2, "b2");
  TORCH_CHECK(x.dim() == 4 && z.dim() == 4 && w.dim() == 2 && w2.dim() == 2, "kvedge: conv_pair shapes");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), ldx = x.size(3);
  const int64_t Cout = w.size(0), C2 = w2.size(0);
  TORCH_CHECK(w2.size(1) == Cout, "kvedge: conv_pair w2 must be [C2, Cout]");
  TORCH_CHECK(z.size(0) == N && z.size(1) == H && z.size(2) == W && z_coff + C2 <= z.size(3),
              "kvedge: conv_pair z [N, H, W, >= z_coff + C2]");
  TORCH_CHECK(x_coff + Cin <= ldx && w.size(1) == (9 * Cin + 63) / 64 * 64, "kvedge: conv_pair x / w");
  // the C2 store path writes 8-B bf16x4 chunks at z + pixel * ldz + z_coff + 4j
  TORCH_CHECK(x_coff >= 0 && z_coff >= 0, "kvedge: conv_pair channel offsets must be >= 0");
  TORCH_CHECK(z_coff % 4 == 0 && z.size(3) % 4 == 0,
              "kvedge: conv_pair z_coff and the z row pitch must be multiples of 4 channels");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() >= Cout && b2.scalar_type() == at::kFloat &&
              b2.numel() >= C2, "kvedge: conv_pair biases fp32");
  TORCH_CHECK(N * H * W * ldx * 2 < (1ll << 31) && N * H * W * z.size(3) * 2 < (1ll << 31),
              "kvedge: conv_pair operands exceed 2 GiB");
  const c10::DeviceGuard g(x.device());
  KvConvParams p{};
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.bias = bias.data_ptr<float>();
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.Cin = (int)Cin;
  p.ldx = (int)ldx; p.x_coff = (int)x_coff;
  p.Ho = (int)H; p.Wo = (int)W; p.Cout = (int)Cout;
  p.KH = 3; p.KW = 3; p.stride = 1; p.pad = 1;
  p.K = (int)(9 * Cin); p.Kpad = (int)w.size(1);
  p.M = (int)(N * H * W);
  p.act = (int)act; p.mode = 0;
  p.w_t = w2.data_ptr(); p.bias_t = b2.data_ptr<float>(); p.z = z.data_ptr();
  p.n_t = (int)C2; p.ldz = (int)z.size(3); p.z_coff = (int)z_coff;
  p.pair_1x1 = 1;
  const int rc = kv_conv_pair(&p, (int)tile, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: conv_pair failed rc=", rc);
}

// Bottleneck conv3 with the downsample branch folded in as extra K (mode 4):
//   y = act( x1 (1x1) . W[:, :K1]  +  x2 (1x1, stride s2) . W[:, K1:]  + bias )
void conv_dual(const at::Tensor& x1, const at::Tensor& x2, const at::Tensor& w,
               const c10::optional<at::Tensor>& bias, at::Tensor& y, int64_t stride2,
               int64_t act, int64_t tile, const c10::optional<at::Tensor>& ws) {
  check_bf16(x1, "x1");
  check_bf16(x2, "x2");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x1.dim() == 4 && x2.dim() == 4 && y.dim() == 4, "kvedge: NHWC tensors");
  const int64_t N = x1.size(0), Ho = x1.size(1), Wo = x1.size(2), K1 = x1.size(3);
  const int64_t K2 = x2.size(3), Cout = y.size(3);
  TORCH_CHECK(x2.size(0) == N && (x2.size(1) + stride2 - 1) / stride2 == Ho &&
                  (x2.size(2) + stride2 - 1) / stride2 == Wo, "kvedge: x2 geometry vs stride");
  TORCH_CHECK(y.size(0) == N && y.size(1) == Ho && y.size(2) == Wo, "kvedge: y shape");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == Cout && w.size(1) == K1 + K2, "kvedge: w [Cout, K1+K2]");
  TORCH_CHECK(K1 % 64 == 0 && K2 % 64 == 0, "kvedge: K1, K2 multiples of 64");
  const c10::DeviceGuard g(x1.device());
  KvConvParams p{};
  p.x = x1.data_ptr();
  p.w = w.data_ptr();
  p.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "kvedge: bias fp32[Cout]");
    p.bias = bias->data_ptr<float>();
  }
  p.res = nullptr;
  p.y = y.data_ptr();
  p.N = (int)N; p.H = (int)Ho; p.W = (int)Wo; p.Cin = (int)K1; p.ldx = (int)K1; p.x_coff = 0;
  p.Ho = (int)Ho; p.Wo = (int)Wo; p.Cout = (int)Cout;
  p.KH = 1; p.KW = 1; p.stride = 1; p.pad = 0;
  p.K = (int)(K1 + K2); p.Kpad = (int)(K1 + K2);
  p.M = (int)(N * Ho * Wo);
  p.ldy = (int)Cout; p.y_coff = 0; p.ldr = 0; p.r_coff = 0;
  p.act = (int)act; p.mode = 4;
  p.x2 = x2.data_ptr(); p.K1 = (int)K1; p.H2 = (int)x2.size(1); p.W2 = (int)x2.size(2);
  p.ldx2 = (int)K2; p.stride2 = (int)stride2;
  if (ws.has_value() && ws->defined()) {
    check_dev(*ws, "ws");
    TORCH_CHECK(ws->scalar_type() == at::kFloat, "kvedge: split-K workspace fp32");
    set_splitk_ws(p, *ws);
  }
  const int rc = kv_conv2d(&p, (int)tile, cur_stream(x1));
  TORCH_CHECK(rc == 0, "kvedge: conv_dual failed rc=", rc);
}

// Dual-source 1x1 GEMM over channel slices (YOLO neck): y[.., y_coff : y_coff + Cout] =
//   act( x[.., x_coff : x_coff + K1] . W[:, :K1] + x2'[.., x2_coff : x2_coff + K2] . W[:, K1:] + b )
// with x2' = x2 at stride s2 (up2 = 0) or x2 upsampled 2x nearest (up2 = 1: x2 is [N, Ho/2,
// Wo/2, ..]; the concat of an upsampled map and a skip tensor never materialises).
void conv_dual2(const at::Tensor& x, int64_t x_coff, int64_t K1, const at::Tensor& x2,
                int64_t x2_coff, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                at::Tensor& y, int64_t y_coff, int64_t stride2, int64_t up2, int64_t act,
                int64_t tile, const c10::optional<at::Tensor>& ws) {
  check_bf16(x, "x");
  check_bf16(x2, "x2");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 4 && x2.dim() == 4 && y.dim() == 4 && w.dim() == 2, "kvedge: NHWC tensors");
  const int64_t N = x.size(0), Ho = x.size(1), Wo = x.size(2);
  const int64_t Cout = w.size(0), K2 = w.size(1) - K1;
  TORCH_CHECK(K1 > 0 && K2 > 0 && K1 % 64 == 0 && K2 % 64 == 0, "kvedge: K1, K2 multiples of 64");
  TORCH_CHECK(x_coff >= 0 && x_coff % 8 == 0 && x_coff + K1 <= x.size(3), "kvedge: x slice");
  TORCH_CHECK(x2_coff >= 0 && x2_coff % 8 == 0 && x2_coff + K2 <= x2.size(3), "kvedge: x2 slice");
  TORCH_CHECK(y_coff >= 0 && y_coff % 8 == 0 && y_coff + Cout <= y.size(3), "kvedge: y slice");
  TORCH_CHECK(x.size(3) % 8 == 0 && x2.size(3) % 8 == 0 && y.size(3) % 8 == 0, "kvedge: pitches");
  TORCH_CHECK(y.size(0) == N && y.size(1) == Ho && y.size(2) == Wo && x2.size(0) == N, "kvedge: y shape");
  if (up2) {
    TORCH_CHECK(x2.size(1) * 2 == Ho && x2.size(2) * 2 == Wo, "kvedge: up2 needs x2 at half size");
  } else {
    TORCH_CHECK(stride2 >= 1 && (x2.size(1) + stride2 - 1) / stride2 == Ho &&
                    (x2.size(2) + stride2 - 1) / stride2 == Wo,
                "kvedge: x2 geometry vs stride");
  }
  // no whole-tensor cap: kv_conv2d splits a batch whose per-image operands fit a launch
  // into image chunks (x2 advanced per image, up2 included) and refuses (rc -9) only an
  // IMAGE too large for 32-bit offsets -- the same contract as conv2d
  const c10::DeviceGuard g(x.device());
  KvConvParams p{};
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "kvedge: bias fp32[Cout]");
    p.bias = bias->data_ptr<float>();
  }
  p.y = y.data_ptr();
  p.N = (int)N; p.H = (int)Ho; p.W = (int)Wo; p.Cin = (int)K1; p.ldx = (int)x.size(3);
  p.x_coff = (int)x_coff;
  p.Ho = (int)Ho; p.Wo = (int)Wo; p.Cout = (int)Cout;
  p.KH = 1; p.KW = 1; p.stride = 1; p.pad = 0;
  p.K = (int)(K1 + K2); p.Kpad = (int)(K1 + K2);
  p.M = (int)(N * Ho * Wo);
  p.ldy = (int)y.size(3); p.y_coff = (int)y_coff; p.ldr = 0; p.r_coff = 0;
  p.act = (int)act; p.mode = 4;
  p.x2 = x2.data_ptr(); p.K1 = (int)K1; p.H2 = (int)x2.size(1); p.W2 = (int)x2.size(2);
  p.ldx2 = (int)x2.size(3); p.stride2 = (int)stride2; p.x2_coff = (int)x2_coff; p.up2 = (int)up2;
  if (ws.has_value() && ws->defined()) {
    check_dev(*ws, "ws");
    TORCH_CHECK(ws->scalar_type() == at::kFloat, "kvedge: split-K workspace fp32");
    set_splitk_ws(p, *ws);
  }
  const int rc = kv_conv2d(&p, (int)tile, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: conv_dual2 failed rc=", rc);
}

// Fused bottleneck tail: y = act(x . W^T [+ x2 . W2^T] + bias [+ res]) (conv3, optionally
// with the fused downsample), then z = ReLU(y . w1^T + b1) -- the next block's 1x1 reduce --
// from the y tile still in LDS, so y is written once and never re-read.
void conv_tail(const at::Tensor& x, const c10::optional<at::Tensor>& x2, const at::Tensor& w,
               const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
               at::Tensor& y, const at::Tensor& w1, const c10::optional<at::Tensor>& b1,
               at::Tensor& z, int64_t stride2, int64_t act, int64_t tile) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  check_bf16(w1, "w1");
  check_bf16(z, "z");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && z.dim() == 4, "kvedge: NHWC tensors");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), K1 = x.size(3);
  const int64_t Cout = y.size(3), Nt = w1.size(0);
  TORCH_CHECK(y.size(0) == N && y.size(1) == H && y.size(2) == W, "kvedge: y shape");
  TORCH_CHECK(z.size(0) == N && z.size(1) == H && z.size(2) == W && z.size(3) == Nt,
              "kvedge: z shape");
  TORCH_CHECK(w1.dim() == 2 && w1.size(1) == Cout, "kvedge: w1 must be [n_t, Cout]");
  TORCH_CHECK(K1 % 64 == 0, "kvedge: conv_tail K1 multiple of 64");
  const c10::DeviceGuard g(x.device());
  KvConvParams p{};
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "kvedge: bias fp32[Cout]");
    p.bias = bias->data_ptr<float>();
  }
  p.y = y.data_ptr();
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.Cin = (int)K1; p.ldx = (int)K1; p.x_coff = 0;
  p.Ho = (int)H; p.Wo = (int)W; p.Cout = (int)Cout;
  p.KH = 1; p.KW = 1; p.stride = 1; p.pad = 0;
  p.M = (int)(N * H * W);
  p.ldy = (int)Cout; p.y_coff = 0; p.r_coff = 0;
  p.act = (int)act;
  if (x2.has_value() && x2->defined()) {
    check_bf16(*x2, "x2");
    TORCH_CHECK(!(res.has_value() && res->defined()), "kvedge: conv_tail dual form takes no res");
    const int64_t K2 = x2->size(3);
    TORCH_CHECK(x2->dim() == 4 && x2->size(0) == N && (x2->size(1) + stride2 - 1) / stride2 == H &&
                    (x2->size(2) + stride2 - 1) / stride2 == W && K2 % 64 == 0,
                "kvedge: x2 geometry vs stride");
    TORCH_CHECK(w.dim() == 2 && w.size(0) == Cout && w.size(1) == K1 + K2, "kvedge: w [Cout, K1+K2]");
    p.mode = 4; p.K = (int)(K1 + K2); p.Kpad = (int)(K1 + K2);
    p.x2 = x2->data_ptr(); p.K1 = (int)K1; p.H2 = (int)x2->size(1); p.W2 = (int)x2->size(2);
    p.ldx2 = (int)K2; p.stride2 = (int)stride2;
    p.res = nullptr; p.ldr = 0;
  } else {
    TORCH_CHECK(res.has_value() && res->defined(), "kvedge: conv_tail plain form needs res");
    check_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == y.sizes(), "kvedge: res shape");
    TORCH_CHECK(w.dim() == 2 && w.size(0) == Cout && w.size(1) == K1, "kvedge: w [Cout, K1]");
    p.mode = 1; p.K = (int)K1; p.Kpad = (int)K1;
    p.res = res->data_ptr(); p.ldr = (int)Cout;
  }
  p.w_t = w1.data_ptr();
  p.bias_t = nullptr;
  if (b1.has_value() && b1->defined()) {
    check_dev(*b1, "b1");
    TORCH_CHECK(b1->scalar_type() == at::kFloat && b1->numel() >= Nt, "kvedge: b1 fp32[n_t]");
    p.bias_t = b1->data_ptr<float>();
  }
  p.z = z.data_ptr(); p.n_t = (int)Nt; p.ldz = (int)Nt; p.z_coff = 0; p.act_t = 1;
  const int rc = kv_conv2d(&p, (int)tile, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: conv_tail failed rc=", rc);
}

// Frames-in space-to-depth stem (preprocess fused): y = act(conv2x2_s2d(frames) + bias)
// with frames uint8 [N, 2H, 2W, 3] and w the packed [Cout, 64] s2d stem weights, already
// scaled for raw 0..255 inputs (kvedge_amd.ops.stem_from_frames).
void conv_frames_s2d(const at::Tensor& frames, const at::Tensor& w,
                     const c10::optional<at::Tensor>& bias, at::Tensor& y, int64_t act,
                     int64_t tile) {
  check_dev(frames, "frames");
  TORCH_CHECK(frames.scalar_type() == at::kByte && frames.dim() == 4 && frames.size(3) == 3 &&
                  frames.size(1) % 2 == 0 && frames.size(2) % 2 == 0,
              "kvedge: frames must be uint8 [N, H, W, 3] with even H, W");
  check_bf16(w, "w");
  check_bf16(y, "y");
  const int64_t N = frames.size(0), H = frames.size(1) / 2, W = frames.size(2) / 2;
  const int64_t Cout = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == 64, "kvedge: s2d stem weight must be [Cout, 64]");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == H && y.size(2) == W &&
                  y.size(3) == Cout, "kvedge: y must be [N, H/2, W/2, Cout]");
  const c10::DeviceGuard g(frames.device());
  KvConvParams p{};
  p.x = frames.data_ptr();
  p.w = w.data_ptr();
  p.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "kvedge: bias fp32[Cout]");
    p.bias = bias->data_ptr<float>();
  }
  p.res = nullptr;
  p.y = y.data_ptr();
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.Cin = 16; p.ldx = 16; p.x_coff = 0;
  p.Ho = (int)H; p.Wo = (int)W; p.Cout = (int)Cout;
  p.KH = 2; p.KW = 2; p.stride = 1; p.pad = 1; p.K = 64; p.Kpad = 64;
  p.M = (int)(N * H * W);
  p.ldy = (int)Cout; p.y_coff = 0; p.ldr = 0; p.r_coff = 0;
  p.act = (int)act; p.mode = 0; p.in_u8 = 1;
  const int rc = kv_conv2d(&p, (int)tile, cur_stream(frames));
  TORCH_CHECK(rc == 0, "kvedge: conv_frames_s2d failed rc=", rc);
}

void maxpool2d(const at::Tensor& x, at::Tensor& y, int64_t N, int64_t H, int64_t W, int64_t C,
               int64_t ldx, int64_t x_coff, int64_t ldy, int64_t y_coff, int64_t k, int64_t stride, int64_t pad,
               int64_t Ho, int64_t Wo) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.numel() >= N * H * W * ldx && y.numel() >= N * Ho * Wo * ldy, "kvedge: maxpool sizes");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_maxpool2d(x.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)ldx,
                              (int)x_coff, (int)ldy, (int)y_coff, (int)k, (int)stride, (int)pad, (int)Ho,
                              (int)Wo, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: maxpool2d failed rc=", rc);
}

void stem_pool(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, at::Tensor& y,
               int64_t y_coff) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 16, "kvedge: stem_pool x must be [N,H,W,16] (s2d)");
  TORCH_CHECK(w.numel() == 64 * 256, "kvedge: stem_pool w must be [64][256]");
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == 64 &&
                  bias.is_contiguous(), "kvedge: stem_pool bias");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == (H - 1) / 2 + 1 &&
                  y.size(2) == (W - 1) / 2 + 1 && y.size(3) >= y_coff + 64,
              "kvedge: stem_pool y shape");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_stem_pool(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), y.data_ptr(),
                              (int)N, (int)H, (int)W, (int)y.size(3), (int)y_coff, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: stem_pool failed rc=", rc);
}

void sppf_pool(at::Tensor& buf, int64_t N, int64_t H, int64_t W, int64_t C) {
  check_bf16(buf, "buf");
  TORCH_CHECK(buf.numel() == N * H * W * 4 * C, "kvedge: sppf buffer must be [N,H,W,4C]");
  const c10::DeviceGuard g(buf.device());
  const int rc = kv_sppf_pool(buf.data_ptr(), (int)N, (int)H, (int)W, (int)C, cur_stream(buf));
  TORCH_CHECK(rc == 0, "kvedge: sppf failed rc=", rc);
}

void global_avgpool(const at::Tensor& x, at::Tensor& y, int64_t N, int64_t HW, int64_t C) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.numel() == N * HW * C && y.numel() == N * C, "kvedge: avgpool sizes");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_global_avgpool(x.data_ptr(), y.data_ptr(), (int)N, (int)HW, (int)C, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: avgpool failed rc=", rc);
}

// Edge-batch classifier head: y [N, ncls] bf16 = fc(global_avgpool(x)), x [N, H, W, C]
void pooled_fc(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
               at::Tensor& y) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2 && y.dim() == 2, "kvedge: pooled_fc shapes");
  const int64_t N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3), ncls = w.size(0);
  TORCH_CHECK(w.size(1) >= C && y.size(0) == N && y.size(1) == ncls, "kvedge: pooled_fc w / y");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= ncls, "kvedge: pooled_fc bias");
    bp = bias->data_ptr<float>();
  }
  const c10::DeviceGuard g(x.device());
  const int rc = kv_pooled_fc(x.data_ptr(), (int)N, (int)HW, (int)C, w.data_ptr(), (int)w.size(1),
                              bp, y.data_ptr(), (int)ncls, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: pooled_fc failed rc=", rc);
}

void softmax_rows(const at::Tensor& x, at::Tensor& y, at::Tensor& argmax) {
  check_bf16(x, "x");
  check_dev(y, "y");
  check_dev(argmax, "argmax");
  TORCH_CHECK(x.dim() == 2 && y.sizes() == x.sizes() && y.scalar_type() == at::kFloat, "kvedge: softmax y");
  TORCH_CHECK(argmax.scalar_type() == at::kLong && argmax.numel() == x.size(0), "kvedge: argmax");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_softmax_rows(x.data_ptr(), y.data_ptr<float>(), argmax.data_ptr<int64_t>(),
                                 (int)x.size(0), (int)x.size(1), cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: softmax failed rc=", rc);
}

void upsample2x(const at::Tensor& x, at::Tensor& y, int64_t N, int64_t H, int64_t W, int64_t C,
                int64_t ldx, int64_t x_coff, int64_t ldy, int64_t y_coff) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.numel() >= N * H * W * ldx && y.numel() >= N * 4 * H * W * ldy, "kvedge: upsample sizes");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_upsample2x(x.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)ldx,
                               (int)x_coff, (int)ldy, (int)y_coff, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: upsample2x failed rc=", rc);
}

void yolo_decode(const at::Tensor& f0, const at::Tensor& f1, const at::Tensor& f2, int64_t h0,
                 int64_t w0, int64_t h1, int64_t w1, int64_t h2, int64_t w2, int64_t s0,
                 int64_t s1, int64_t s2, int64_t nc, at::Tensor& boxes, at::Tensor& scores,
                 at::Tensor& cls) {
  check_bf16(f0, "f0");
  check_bf16(f1, "f1");
  check_bf16(f2, "f2");
  const int64_t N = f0.size(0);
  const int64_t A = h0 * w0 + h1 * w1 + h2 * w2;
  const int64_t ch = 64 + nc;
  TORCH_CHECK(f0.numel() == N * h0 * w0 * ch && f1.numel() == N * h1 * w1 * ch &&
                  f2.numel() == N * h2 * w2 * ch, "kvedge: decode feature sizes");
  TORCH_CHECK(boxes.numel() == N * A * 4 && boxes.scalar_type() == at::kFloat, "kvedge: boxes");
  TORCH_CHECK(scores.numel() == N * A && scores.scalar_type() == at::kFloat, "kvedge: scores");
  TORCH_CHECK(cls.numel() == N * A && cls.scalar_type() == at::kInt, "kvedge: cls");
  const c10::DeviceGuard g(f0.device());
  const int rc = kv_yolo_decode(f0.data_ptr(), f1.data_ptr(), f2.data_ptr(), (int)h0, (int)w0,
                                (int)h1, (int)w1, (int)h2, (int)w2, (int)s0, (int)s1, (int)s2,
                                (int)N, (int)nc, boxes.data_ptr<float>(), scores.data_ptr<float>(),
                                cls.data_ptr<int>(), cur_stream(f0));
  TORCH_CHECK(rc == 0, "kvedge: yolo_decode failed rc=", rc);
}

void nms(const at::Tensor& boxes, const at::Tensor& scores, const at::Tensor& cls, double conf,
         double iou, int64_t max_det, at::Tensor& out, at::Tensor& count) {
  check_dev(boxes, "boxes");
  check_dev(scores, "scores");
  check_dev(cls, "cls");
  TORCH_CHECK(scores.dim() == 2, "kvedge: scores [N, A]");
  const int64_t N = scores.size(0), A = scores.size(1);
  TORCH_CHECK(boxes.numel() == N * A * 4 && cls.numel() == N * A, "kvedge: nms inputs");
  TORCH_CHECK(out.numel() == N * max_det * 6 && out.scalar_type() == at::kFloat, "kvedge: nms out");
  TORCH_CHECK(count.numel() == N && count.scalar_type() == at::kInt, "kvedge: nms count");
  const c10::DeviceGuard g(scores.device());
  const int rc = kv_nms(boxes.data_ptr<float>(), scores.data_ptr<float>(), cls.data_ptr<int>(),
                        (int)N, (int)A, (float)conf, (float)iou, (int)max_det,
                        out.data_ptr<float>(), count.data_ptr<int>(), cur_stream(scores));
  TORCH_CHECK(rc == 0, "kvedge: nms failed rc=", rc);
}

void synth_frames(at::Tensor& y, int64_t seed, int64_t step) {
  check_dev(y, "y");
  TORCH_CHECK(y.scalar_type() == at::kByte && y.dim() == 4 && y.size(3) == 3, "kvedge: frames u8 [N,H,W,3]");
  const c10::DeviceGuard g(y.device());
  const int rc = kv_synth_frames(y.data_ptr<uint8_t>(), (int)y.size(0), (int)y.size(1),
                                 (int)y.size(2), (uint64_t)seed, (uint64_t)step, cur_stream(y));
  TORCH_CHECK(rc == 0, "kvedge: synth_frames failed rc=", rc);
}

void synth_frames_dev(at::Tensor& y, at::Tensor& step, int64_t seed) {
  check_dev(y, "y");
  check_dev(step, "step");
  TORCH_CHECK(y.scalar_type() == at::kByte && y.dim() == 4 && y.size(3) == 3, "kvedge: frames u8 [N,H,W,3]");
  // int64[1]: counter, bumped by a second launch; int64[2]: counter + finished-block
  // count (zero), bumped in-kernel by the last block to finish
  TORCH_CHECK(step.scalar_type() == at::kLong && (step.numel() == 1 || step.numel() == 2),
              "kvedge: step int64[1] or int64[2]");
  const c10::DeviceGuard g(y.device());
  const int rc = kv_synth_frames_dev(y.data_ptr<uint8_t>(), (int)y.size(0), (int)y.size(1),
                                     (int)y.size(2), (uint64_t)seed,
                                     reinterpret_cast<uint64_t*>(step.data_ptr<int64_t>()),
                                     step.numel() == 2 ? 1 : 0, cur_stream(y));
  TORCH_CHECK(rc == 0, "kvedge: synth_frames_dev failed rc=", rc);
}

// Frames-in ResNet stem + pool: preprocess (normalise + s2d) fused into stem_pool's fetch
// Frames-in ResNet stem + pool, 12-channel s2d formulation (stem12.hip: K = 192, not 256)
void stem12_pool_frames(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias,
                        at::Tensor& y, at::ArrayRef<double> mean, at::ArrayRef<double> stdv,
                        int64_t y_coff) {
  check_dev(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(),
              "kvedge: stem12_pool_frames x must be contiguous u8 [N,H,W,3]");
  TORCH_CHECK(x.size(1) % 2 == 0 && x.size(2) % 4 == 0, "kvedge: stem12_pool_frames H even, W % 4");
  TORCH_CHECK(w.numel() == 64 * 192 && w.is_contiguous(), "kvedge: stem12 w must be [64][192]");
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == 64 &&
                  bias.is_contiguous(), "kvedge: stem12 bias");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "kvedge: mean/std of 3");
  const int64_t N = x.size(0), H = x.size(1) / 2, W = x.size(2) / 2;
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == (H - 1) / 2 + 1 &&
                  y.size(2) == (W - 1) / 2 + 1 && y.size(3) >= y_coff + 64 && y.is_contiguous(),
              "kvedge: stem12_pool_frames y shape");
  float m[3], is[3];
  for (int i = 0; i < 3; ++i) {
    m[i] = (float)mean[i];
    is[i] = (float)(1.0 / stdv[i]);
  }
  const c10::DeviceGuard g(x.device());
  const int rc = kv_stem12_pool_frames(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(),
                                       y.data_ptr(), (int)N, (int)x.size(1), (int)x.size(2), m, is,
                                       (int)y.size(3), (int)y_coff, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: stem12_pool_frames failed rc=", rc);
}

// YOLOv8n b0 (frames-in s2d stem) + b1 (3x3/2 16 -> 32) in one kernel (yolo_stem2.hip)
void yolo_stem2(const at::Tensor& x, const at::Tensor& w0, const at::Tensor& b0,
                const at::Tensor& w1, const at::Tensor& b1, at::Tensor& y) {
  check_dev(x, "x");
  check_bf16(w0, "w0");
  check_bf16(w1, "w1");
  check_bf16(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(),
              "kvedge: yolo_stem2 x must be contiguous u8 [N,H,W,3]");
  TORCH_CHECK(x.size(1) % 4 == 0 && x.size(2) % 32 == 0 && x.size(2) <= 640,
              "kvedge: yolo_stem2 needs H % 4 == 0, W % 32 == 0, W <= 640");
  TORCH_CHECK(w0.dim() == 2 && w0.size(0) == 16 && w0.size(1) == 64 && w0.is_contiguous(),
              "kvedge: yolo_stem2 w0 must be [16][64]");
  TORCH_CHECK(w1.dim() == 2 && w1.size(0) == 32 && w1.size(1) >= 144 && w1.size(1) % 8 == 0 &&
                  w1.is_contiguous(), "kvedge: yolo_stem2 w1 must be [32][>= 144]");
  for (const at::Tensor* b : {&b0, &b1}) {
    check_dev(*b, "bias");
    TORCH_CHECK(b->scalar_type() == at::kFloat && b->is_contiguous(), "kvedge: fp32 biases");
  }
  TORCH_CHECK(b0.numel() >= 16 && b1.numel() >= 32, "kvedge: bias sizes");
  const int64_t N = x.size(0), H0 = x.size(1), W0 = x.size(2);
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == H0 / 4 && y.size(2) == W0 / 4 &&
                  y.size(3) == 32 && y.is_contiguous(), "kvedge: yolo_stem2 y must be [N,H/4,W/4,32]");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_yolo_stem2(x.data_ptr(), w0.data_ptr(), b0.data_ptr<float>(), w1.data_ptr(),
                               (int)w1.size(1), b1.data_ptr<float>(), y.data_ptr(), (int)N,
                               (int)H0, (int)W0, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: yolo_stem2 failed rc=", rc);
}

void stem_pool_frames(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias,
                      at::Tensor& y, at::ArrayRef<double> mean, at::ArrayRef<double> stdv,
                      int64_t y_coff) {
  check_dev(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(),
              "kvedge: stem_pool_frames x must be contiguous u8 [N,H,W,3]");
  TORCH_CHECK(x.size(1) % 2 == 0 && x.size(2) % 4 == 0, "kvedge: stem_pool_frames H even, W % 4");
  TORCH_CHECK(w.numel() == 64 * 256, "kvedge: stem_pool w must be [64][256]");
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == 64 &&
                  bias.is_contiguous(), "kvedge: stem_pool bias");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "kvedge: mean/std of 3");
  const int64_t N = x.size(0), H = x.size(1) / 2, W = x.size(2) / 2;
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == (H - 1) / 2 + 1 &&
                  y.size(2) == (W - 1) / 2 + 1 && y.size(3) >= y_coff + 64,
              "kvedge: stem_pool_frames y shape");
  float m[3], is[3];
  for (int i = 0; i < 3; ++i) {
    m[i] = (float)mean[i];
    is[i] = (float)(1.0 / stdv[i]);
  }
  const c10::DeviceGuard g(x.device());
  const int rc = kv_stem_pool_frames(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(),
                                     y.data_ptr(), (int)N, (int)x.size(1), (int)x.size(2), m, is,
                                     (int)y.size(3), (int)y_coff, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: stem_pool_frames failed rc=", rc);
}

void preprocess(const at::Tensor& x, at::Tensor& y, at::ArrayRef<double> mean,
                at::ArrayRef<double> stdv) {
  check_dev(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) == 3, "kvedge: x u8 [N,H,W,3]");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == x.size(0), "kvedge: y batch");
  const bool s2d = y.size(3) == 16;
  if (s2d) {
    TORCH_CHECK(y.size(1) * 2 == x.size(1) && y.size(2) * 2 == x.size(2), "kvedge: y bf16 [N,H/2,W/2,16]");
  } else {
    TORCH_CHECK(y.size(1) == x.size(1) && y.size(2) == x.size(2) && y.size(3) == 4,
                "kvedge: y bf16 [N,H,W,4] or [N,H/2,W/2,16]");
  }
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "kvedge: mean/std of 3");
  float m[3], is[3];
  for (int i = 0; i < 3; ++i) {
    m[i] = (float)mean[i];
    is[i] = (float)(1.0 / stdv[i]);
  }
  const c10::DeviceGuard g(x.device());
  const int rc = s2d ? kv_preprocess_s2d(x.data_ptr<uint8_t>(), y.data_ptr(), (int)x.size(0),
                                         (int)x.size(1), (int)x.size(2), m, is, cur_stream(x))
                     : kv_preprocess(x.data_ptr<uint8_t>(), y.data_ptr(), (int)x.size(0),
                                     (int)x.size(1), (int)x.size(2), m, is, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: preprocess failed rc=", rc);
}

void batchnorm_nhwc(const at::Tensor& x, at::Tensor& y, const at::Tensor& scale,
                    const at::Tensor& shift, bool relu) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  check_dev(scale, "scale");
  check_dev(shift, "shift");
  const int64_t C = x.size(-1);
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat &&
                  shift.scalar_type() == at::kFloat, "kvedge: bn scale/shift fp32[C]");
  TORCH_CHECK(y.sizes() == x.sizes(), "kvedge: bn y shape");
  const c10::DeviceGuard g(x.device());
  const int rc = kv_batchnorm_nhwc(x.data_ptr(), y.data_ptr(), scale.data_ptr<float>(),
                                   shift.data_ptr<float>(), x.numel() / C, (int)C, relu ? 1 : 0,
                                   cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: batchnorm failed rc=", rc);
}

int64_t conv_num_tiles() { return kv_conv_num_tiles(); }
int64_t conv_splitk_base() { return kv_conv_splitk_base(); }
int64_t conv_splitk_num_tiles() { return kv_conv_splitk_num_tiles(); }
int64_t nloop_sched_check() { return kv_nloop_sched_check(); }
int64_t conv_seam_num_tiles() { return kv_conv_seam_num_tiles(); }
int64_t set_conv_chunk_bytes(int64_t b) { return kv_set_conv_chunk_bytes(b); }

// v13 fused YOLOv8 C2f(32, 32, n=1, shortcut) (csrc/kernels/c2f_fused.hip): x [N, H, W, ldx]
// channels x_coff .. x_coff + 31 -> y [N, H, W, ldy] channels y_coff .. y_coff + 31
void c2f16_fused(const at::Tensor& x, int64_t x_coff, const at::Tensor& w1, const at::Tensor& b1,
                 const at::Tensor& wm1, const at::Tensor& bm1, const at::Tensor& wm2,
                 const at::Tensor& bm2, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& y,
                 int64_t y_coff, int64_t S) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  for (const at::Tensor* w : {&w1, &wm1, &wm2, &w2}) check_bf16(*w, "w");
  for (const at::Tensor* b : {&b1, &bm1, &bm2, &b2}) {
    check_dev(*b, "bias");
    TORCH_CHECK(b->scalar_type() == at::kFloat && b->is_contiguous(), "kvedge: c2f16 biases fp32");
  }
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(1) == y.size(1) &&
                  x.size(2) == y.size(2), "kvedge: c2f16 x / y [N, H, W, C]");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(x_coff >= 0 && x_coff + 32 <= x.size(3) && y_coff >= 0 && y_coff + 32 <= y.size(3),
              "kvedge: c2f16 channel slices");
  TORCH_CHECK(w1.dim() == 2 && w1.size(0) == 32 && w1.size(1) >= 32 && wm1.dim() == 2 &&
                  wm1.size(0) == 16 && wm1.size(1) >= 144 && wm2.sizes() == wm1.sizes() &&
                  w2.dim() == 2 && w2.size(0) == 32 && w2.size(1) >= 48,
              "kvedge: c2f16 weights w1 [32, >=32], wm [16, >=144], w2 [32, >=48]");
  TORCH_CHECK(b1.numel() == 32 && bm1.numel() == 16 && bm2.numel() == 16 && b2.numel() == 32,
              "kvedge: c2f16 bias sizes");
  TORCH_CHECK(kv_c2f16_supported((int)H, (int)W, (int)S), "kvedge: c2f16 has no form for H=", H,
              " W=", W, " S=", S);
  TORCH_CHECK(x.numel() * 2 < (1ll << 31) - (1 << 20) && y.numel() * 2 < (1ll << 31) - (1 << 20),
              "kvedge: c2f16 operands exceed 2 GiB");
  TORCH_CHECK(x.data_ptr() != y.data_ptr(), "kvedge: c2f16 cannot run in place");
  const c10::DeviceGuard g(x.device());
  KvC2fParams p{};
  p.x = x.data_ptr();
  p.y = y.data_ptr();
  p.w1 = w1.data_ptr();
  p.b1 = b1.data_ptr<float>();
  p.wm1 = wm1.data_ptr();
  p.bm1 = bm1.data_ptr<float>();
  p.wm2 = wm2.data_ptr();
  p.bm2 = bm2.data_ptr<float>();
  p.w2 = w2.data_ptr();
  p.b2 = b2.data_ptr<float>();
  p.N = (int)N; p.H = (int)H; p.W = (int)W;
  p.ldx = (int)x.size(3); p.x_coff = (int)x_coff;
  p.ldy = (int)y.size(3); p.y_coff = (int)y_coff;
  p.ldw1 = (int)w1.size(1); p.ldwm = (int)wm1.size(1); p.ldw2 = (int)w2.size(1);
  p.S = (int)S;
  const int rc = kv_c2f16_fused(&p, cur_stream(x));
  TORCH_CHECK(rc == 0, "kvedge: c2f16_fused failed rc=", rc);
}

int64_t c2f16_supported(int64_t H, int64_t W, int64_t S) {
  return kv_c2f16_supported((int)H, (int)W, (int)S);
}

}  // namespace

TORCH_LIBRARY(kvedge, m) {
  m.def("conv(Tensor x, Tensor w, Tensor? bias, Tensor? res, Tensor(a!) y, int N, int H, int W, "
        "int Cin, int ldx, int x_coff, int Ho, int Wo, int Cout, int KH, int KW, int stride, "
        "int pad, int K, int ldy, int y_coff, int ldr, int r_coff, int act, int mode, int tile, "
        "Tensor(b!)? ws=None) -> ()");
  m.def("conv_pair(Tensor x, Tensor w, Tensor bias, Tensor w2, Tensor b2, Tensor(a!) z, int Cin, "
        "int x_coff, int z_coff, int act, int tile) -> ()");
  m.def("conv_dual(Tensor x1, Tensor x2, Tensor w, Tensor? bias, Tensor(a!) y, int stride2, int act, "
        "int tile, Tensor(b!)? ws=None) -> ()");
  m.def("conv_tail(Tensor x, Tensor? x2, Tensor w, Tensor? bias, Tensor? res, Tensor(a!) y, "
        "Tensor w1, Tensor? b1, Tensor(b!) z, int stride2, int act, int tile) -> ()");
  m.def("conv_frames_s2d(Tensor frames, Tensor w, Tensor? bias, Tensor(a!) y, int act, "
        "int tile) -> ()");
  m.def("stem_pool(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, int y_coff) -> ()");
  m.def("maxpool2d(Tensor x, Tensor(a!) y, int N, int H, int W, int C, int ldx, int x_coff, int ldy, "
        "int y_coff, int k, int stride, int pad, int Ho, int Wo) -> ()");
  m.def("sppf_pool(Tensor(a!) buf, int N, int H, int W, int C) -> ()");
  m.def("global_avgpool(Tensor x, Tensor(a!) y, int N, int HW, int C) -> ()");
  m.def("softmax_rows(Tensor x, Tensor(a!) y, Tensor(b!) argmax) -> ()");
  m.def("pooled_fc(Tensor x, Tensor w, Tensor? bias, Tensor(a!) y) -> ()");
  m.def("upsample2x(Tensor x, Tensor(a!) y, int N, int H, int W, int C, int ldx, int x_coff, int ldy, "
        "int y_coff) -> ()");
  m.def("yolo_decode(Tensor f0, Tensor f1, Tensor f2, int h0, int w0, int h1, int w1, int h2, "
        "int w2, int s0, int s1, int s2, int nc, Tensor(a!) boxes, Tensor(b!) scores, "
        "Tensor(c!) cls) -> ()");
  m.def("nms(Tensor boxes, Tensor scores, Tensor cls, float conf, float iou, int max_det, "
        "Tensor(a!) out, Tensor(b!) count) -> ()");
  m.def("synth_frames(Tensor(a!) y, int seed, int step) -> ()");
  m.def("synth_frames_dev(Tensor(a!) y, Tensor(b!) step, int seed) -> ()");
  m.def("stem_pool_frames(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, float[] mean, float[] std, int y_coff) -> ()");
  m.def("stem12_pool_frames(Tensor x, Tensor w, Tensor bias, Tensor(a!) y, float[] mean, float[] std, int y_coff) -> ()");
  m.def("yolo_stem2(Tensor x, Tensor w0, Tensor b0, Tensor w1, Tensor b1, Tensor(a!) y) -> ()");
  m.def("preprocess(Tensor x, Tensor(a!) y, float[] mean, float[] std) -> ()");
  m.def("batchnorm_nhwc(Tensor x, Tensor(a!) y, Tensor scale, Tensor shift, bool relu) -> ()");
  m.def("conv_num_tiles() -> int", conv_num_tiles);
  m.def("conv_splitk_base() -> int", conv_splitk_base);
  m.def("conv_splitk_num_tiles() -> int", conv_splitk_num_tiles);
  m.def("nloop_sched_check() -> int", nloop_sched_check);
  m.def("conv_seam_num_tiles() -> int", conv_seam_num_tiles);
  m.def("c2f16_fused(Tensor x, int x_coff, Tensor w1, Tensor b1, Tensor wm1, Tensor bm1, "
        "Tensor wm2, Tensor bm2, Tensor w2, Tensor b2, Tensor(a!) y, int y_coff, int S) -> ()");
  m.def("c2f16_supported(int H, int W, int S) -> int", c2f16_supported);
  m.def("conv_dual2(Tensor x, int x_coff, int K1, Tensor x2, int x2_coff, Tensor w, Tensor? bias, "
        "Tensor(a!) y, int y_coff, int stride2, int up2, int act, int tile, Tensor(b!)? ws=None) -> ()");
  m.def("set_conv_chunk_bytes(int bytes) -> int", set_conv_chunk_bytes);
}

TORCH_LIBRARY_IMPL(kvedge, CUDA, m) {
  m.impl("conv", conv);
  m.impl("conv_dual", conv_dual);
  m.impl("maxpool2d", maxpool2d);
  m.impl("stem_pool", stem_pool);
  m.impl("conv_frames_s2d", conv_frames_s2d);
  m.impl("conv_tail", conv_tail);
  m.impl("conv_pair", conv_pair);
  m.impl("c2f16_fused", c2f16_fused);
  m.impl("conv_dual2", conv_dual2);
  m.impl("sppf_pool", sppf_pool);
  m.impl("global_avgpool", global_avgpool);
  m.impl("softmax_rows", softmax_rows);
  m.impl("pooled_fc", pooled_fc);
  m.impl("upsample2x", upsample2x);
  m.impl("yolo_decode", yolo_decode);
  m.impl("nms", nms);
  m.impl("synth_frames", synth_frames);
  m.impl("synth_frames_dev", synth_frames_dev);
  m.impl("preprocess", preprocess);
  m.impl("stem_pool_frames", stem_pool_frames);
  m.impl("stem12_pool_frames", stem12_pool_frames);
  m.impl("yolo_stem2", yolo_stem2);
  m.impl("batchnorm_nhwc", batchnorm_nhwc);
}

