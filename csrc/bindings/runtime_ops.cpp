// Torch bindings of the native serving runtime (csrc/runtime/kv_runtime.h):
//   kvedge::hist_len / hist_add / hist_quantiles / hist_mean   (CPU int64 tensors)
//   kvedge::arena_plan / arena_live_peak                      (int lists)
//   kvedge::serve_loop                                        (hipGraphExec_t replay)
//   torch.classes.kvedge.FrameRing                            (pinned frame ring)
// These are catch-all ops (no tensor-device dispatch): they run on the build box's CPU
// too, so the CPU test tier exercises the same native code the GPU box runs.
#include <ATen/ATen.h>
#include <Python.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include "kv_runtime.h"

namespace {

using kvrt::LatencyHist;

// Drop the GIL around blocking native loops so Python producer threads can keep
// filling the frame ring; a no-op when called without the GIL (C++ callers).
struct NoGil {
  PyThreadState* st = nullptr;
  NoGil() {
    if (Py_IsInitialized() && PyGILState_Check()) st = PyEval_SaveThread();
  }
  ~NoGil() {
    if (st) PyEval_RestoreThread(st);
  }
};

int64_t* hist_ptr(const at::Tensor& h) {
  TORCH_CHECK(h.device().is_cpu() && h.scalar_type() == at::kLong && h.is_contiguous() &&
                  h.numel() == LatencyHist::kLen,
              "kvedge: latency histogram must be a contiguous CPU int64[", LatencyHist::kLen, "]");
  return h.data_ptr<int64_t>();
}

int64_t hist_len() { return LatencyHist::kLen; }

void hist_add(at::Tensor& hist, double us) { LatencyHist::add(hist_ptr(hist), us); }

void hist_add_many(at::Tensor& hist, const at::Tensor& us) {
  auto v = us.to(at::kDouble).contiguous();
  int64_t* h = hist_ptr(hist);
  const double* p = v.data_ptr<double>();
  for (int64_t i = 0; i < v.numel(); ++i) LatencyHist::add(h, p[i]);
}

std::vector<double> hist_quantiles(const at::Tensor& hist, std::vector<double> q) {
  const int64_t* h = hist_ptr(hist);
  for (auto& x : q) x = LatencyHist::quantile(h, x);
  return q;
}

double hist_mean(const at::Tensor& hist) { return LatencyHist::mean(hist_ptr(hist)); }

std::vector<int64_t> arena_plan(std::vector<int64_t> sizes, std::vector<int64_t> first,
                                std::vector<int64_t> last, int64_t align) {
  std::vector<int64_t> off;
  const int64_t total = kvrt::arena_plan(sizes, first, last, align, &off);
  TORCH_CHECK(total >= 0, "kvedge: arena_plan: inconsistent sizes/lifetimes");
  off.push_back(total);  // offsets..., slab size
  return off;
}

int64_t arena_live_peak(std::vector<int64_t> sizes, std::vector<int64_t> first,
                        std::vector<int64_t> last) {
  TORCH_CHECK(sizes.size() == first.size() && sizes.size() == last.size(), "kvedge: arena sizes");
  return kvrt::arena_live_peak(sizes, first, last);
}

std::vector<double> stats_vec(const kvrt::ServeStats& st) {
  return {(double)st.steps, st.wall_s, st.device_ms, (double)st.frames_in};
}

hipStream_t stream_of(int64_t device) {
  return c10::hip::getCurrentHIPStream(device).stream();
}

// serve_loop(exec, n, depth, hist?, device) without a frame ring (synthetic-frame graphs)
std::vector<double> serve_loop(int64_t exec, int64_t n_steps, int64_t depth,
                               const c10::optional<at::Tensor>& hist, int64_t device) {
  TORCH_CHECK(exec != 0, "kvedge: serve_loop needs an instantiated graph exec");
  int64_t* h = hist.has_value() && hist->defined() ? hist_ptr(*hist) : nullptr;
  kvrt::ServeStats st;
  int rc;
  {
    NoGil ng;
    rc = kvrt::serve_loop(reinterpret_cast<hipGraphExec_t>(exec), stream_of(device), n_steps,
                          (int)depth, h, nullptr, nullptr, 0, &st);
  }
  TORCH_CHECK(rc == 0, "kvedge: serve_loop failed (hipError ", -rc, ")");
  return stats_vec(st);
}

struct FrameRingHolder : torch::CustomClassHolder {
  std::unique_ptr<kvrt::FrameRing> ring;
  FrameRingHolder(int64_t slots, int64_t slot_bytes)
      : ring(std::make_unique<kvrt::FrameRing>((int)slots, (size_t)slot_bytes)) {}

  int64_t acquire_write(int64_t timeout_ms, bool drop_oldest) {
    NoGil ng;
    return ring->acquire_write((int)timeout_ms, drop_oldest);
  }
  // uint8 CPU view of slot i (pinned on a GPU host); valid while the ring lives
  at::Tensor slot(int64_t i) {
    TORCH_CHECK(i >= 0 && i < ring->slots(), "kvedge: FrameRing slot index");
    return at::from_blob(ring->slot_ptr((int)i), {(int64_t)ring->slot_bytes()},
                         at::TensorOptions().dtype(at::kByte));
  }
  void publish(int64_t i, int64_t seq) { ring->publish((int)i, seq); }
  std::vector<int64_t> acquire_read(int64_t timeout_ms) {
    int64_t seq = -1;
    int s;
    {
      NoGil ng;
      s = ring->acquire_read((int)timeout_ms, &seq);
    }
    return {s, seq};
  }
  void release(int64_t i) { ring->release((int)i); }
  void close() { ring->close(); }
  int64_t dropped() { return ring->dropped(); }
  int64_t ready() { return ring->ready(); }
  int64_t slots() { return ring->slots(); }
  int64_t slot_bytes() { return (int64_t)ring->slot_bytes(); }
  bool pinned() { return ring->pinned(); }

  // native serve loop fed from this ring into the graph's fixed input buffer
  std::vector<double> serve(int64_t exec, int64_t n_steps, int64_t depth,
                            const c10::optional<at::Tensor>& hist, at::Tensor dev_input,
                            int64_t timeout_ms) {
    TORCH_CHECK(exec != 0, "kvedge: serve needs an instantiated graph exec");
    TORCH_CHECK(dev_input.is_cuda() && dev_input.is_contiguous() &&
                    dev_input.nbytes() == ring->slot_bytes(),
                "kvedge: serve: dev_input must be a contiguous GPU tensor of slot_bytes");
    int64_t* h = hist.has_value() && hist->defined() ? hist_ptr(*hist) : nullptr;
    kvrt::ServeStats st;
    int rc;
    {
      NoGil ng;
      rc = kvrt::serve_loop(reinterpret_cast<hipGraphExec_t>(exec),
                            stream_of(dev_input.device().index()), n_steps, (int)depth, h,
                            ring.get(), dev_input.data_ptr(), (int)timeout_ms, &st);
    }
    TORCH_CHECK(rc == 0, "kvedge: serve failed (hipError ", -rc, ")");
    return stats_vec(st);
  }
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(kvedge, m) {
  m.def("hist_len() -> int", hist_len);
  m.def("hist_add(Tensor(a!) hist, float us) -> ()", hist_add);
  m.def("hist_add_many(Tensor(a!) hist, Tensor us) -> ()", hist_add_many);
  m.def("hist_quantiles(Tensor hist, float[] q) -> float[]", hist_quantiles);
  m.def("hist_mean(Tensor hist) -> float", hist_mean);
  m.def("arena_plan(int[] sizes, int[] first, int[] last, int align) -> int[]", arena_plan);
  m.def("arena_live_peak(int[] sizes, int[] first, int[] last) -> int", arena_live_peak);
  m.def("serve_loop(int exec, int n_steps, int depth, Tensor? hist, int device) -> float[]",
        serve_loop);
  m.class_<FrameRingHolder>("FrameRing")
      .def(torch::init<int64_t, int64_t>())
      .def("acquire_write", &FrameRingHolder::acquire_write)
      .def("slot", &FrameRingHolder::slot)
      .def("publish", &FrameRingHolder::publish)
      .def("acquire_read", &FrameRingHolder::acquire_read)
      .def("release", &FrameRingHolder::release)
      .def("close", &FrameRingHolder::close)
      .def("dropped", &FrameRingHolder::dropped)
      .def("ready", &FrameRingHolder::ready)
      .def("slots", &FrameRingHolder::slots)
      .def("slot_bytes", &FrameRingHolder::slot_bytes)
      .def("pinned", &FrameRingHolder::pinned)
      .def("serve", &FrameRingHolder::serve);
}
