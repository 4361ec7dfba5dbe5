// Shared device helpers for the kvedge_amd gfx950 (CDNA4) kernel library.
//
// Everything here is written for wave64 / MFMA / 160 KiB LDS; there is no
// other target.  The reference (levi106/kvedge) has no kernels at all
// (SURVEY.md §2.2); these exist for the north-star inference hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace kvedge {

constexpr int kWave = 64;   // CDNA wavefront; never 32
constexpr int kNumXcd = 8;  // MI355X: 8 XCDs x 32 CUs, private 4 MiB L2 each

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective").  Blocks b, b+8, b+16 ... are dealt to the same XCD, so we hand
// them CONSECUTIVE logical tiles: neighbouring tiles share operand panels and
// hit the same L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / kNumXcd, r = nwg % kNumXcd;
  const int xcd = bid % kNumXcd, idx = bid / kNumXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Division by a runtime-uniform divisor d without the ~20-instruction VALU expansion of
// an integer divide (there is no hardware divider): q = umulhi(n, ceil(2^32 / d)), exact
// for 0 <= n, d < 2^16 (error term n * (m*d - 2^32) / (d * 2^32) < 1/d).  The direct-conv
// and stem kernels divide pixel indices by row pitches per fetched chunk and per output
// block; with this the divide is one v_mul_hi_u32.
struct FastDiv {
  unsigned m;
  int d;
};
__host__ __device__ __forceinline__ FastDiv make_fastdiv(int d) {
  return FastDiv{(unsigned)((0x100000000ull + (unsigned long long)d - 1) / (unsigned long long)d), d};
}
__device__ __forceinline__ int fdiv(int n, FastDiv f) { return (int)__umulhi((unsigned)n, f.m); }
__device__ __forceinline__ int fmod_(int n, int q, FastDiv f) { return n - q * f.d; }

// 16-B-per-lane global -> LDS DMA (buffer_load_dwordx4 ... lds) that the compiler does NOT
// see as an LDS write.  With the builtin (__builtin_amdgcn_raw_ptr_buffer_load_lds) hipcc
// assumes the pending DMA may alias every later LDS read and puts an s_waitcnt vmcnt(0) in
// front of them: a next-tile prefetch into a SECOND buffer then drains before the current
// tile's fragment reads, i.e. the double buffer does nothing (seen in conv_direct.hip's
// pixel-block loop).  Callers of this form own the synchronisation: an explicit
// s_waitcnt vmcnt(...) + barrier before the destination buffer is read.  An out-of-range
// voff (>= the descriptor's byte count) zero-fills the 16 B, as with the builtin.
typedef int kv_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ kv_i32x4 kv_rsrc4(const void* base, int bytes) {
  const unsigned long long a = (unsigned long long)base;
  kv_i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                                  // num_records
  r[3] = 0x00020000;                                                             // as make_buffer_rsrc
  return r;
}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is set here and never assumed preserved
__device__ __forceinline__ void kv_lds_dma16(kv_i32x4 rs, void* lds, int voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long long)(__attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(m0), "v"(voff), "s"(rs) : "memory", "m0");
}
// ... non-temporal: a once-read stream (a fused tail's residual) that should not displace the
// next launch's input from the Infinity Cache
__device__ __forceinline__ void kv_lds_dma16_nt(kv_i32x4 rs, void* lds, int voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long long)(__attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds"
               :: "s"(m0), "v"(voff), "s"(rs) : "memory", "m0");
}
#pragma clang diagnostic pop

// Registers loaded once per kernel (weights, biases) and read inside a loop that also has
// loads in flight (a band prefetch): pass them through an empty asm after loading.  hipcc's
// wait-count pass then waits for them once, before the asm, and afterwards sees asm-defined
// values instead of pending loads.  Without it the pass re-waited for them inside the loop
// with a vmcnt(0) -- which also drained the next band's in-flight prefetch on every block
// (stem12.hip, yolo_stem2.hip: PMC 30-40 % of wave cycles waiting).
template <class T>
__device__ __forceinline__ void kv_settle(T& v) {
  static_assert(sizeof(T) == 16, "16-byte register groups");
  typedef unsigned int u32x4s __attribute__((ext_vector_type(4)));
  u32x4s u = __builtin_bit_cast(u32x4s, v);
  asm volatile("" : "+v"(u));
  v = __builtin_bit_cast(T, u);
}

// Compile-time loop: f(IC<I>{}) for I in [B, E) (IC below), so a body can use its index as an
// immediate (asm "n"/"i" operands, constexpr ring slots).
template <int I>
struct IC;
template <int B, int E, class F>
__device__ __forceinline__ void static_range(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    static_range<B + 1, E>(f);
  }
}

// ds_read_b128 that hipcc can neither sink nor merge: the caller owns the wait (a counted
// s_waitcnt lgkmcnt tied to the destination, lds_wait below).  The destination register is
// written when the data returns, after the asm statement hipcc sees: keep it out of
// loop-carried values (a back-edge copy may read it before the wait -- the YOLO stem2
// prefetch produced NaNs that way) and consume it only after its lds_wait.  hipcc's scheduler sank every
// fragment read of conv_direct.hip's ring to just before its MFMA under register pressure,
// so each MFMA waited out a full LDS round trip (an lgkmcnt(0) in front of 100 % of them).
template <int OFF, class T>
__device__ __forceinline__ void lds_read16(T& dst, unsigned addr) {
  static_assert(sizeof(T) == 16 && OFF >= 0 && OFF < 65536, "ds_read_b128 immediate offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "n"(OFF) : "memory");
}
// wait until at most N LDS ops are outstanding; dst is threaded through so that its consumer
// cannot be scheduled above the wait
template <int N, class T>
__device__ __forceinline__ void lds_wait(T& dst) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt field");
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(dst) : "n"(N) : "memory");
}
// 16-B buffer load that hipcc neither sinks nor waits for: the same contract as lds_read16
// (not loop-carried, consumed only after vm_wait).  vmcnt counts every vector-memory op of
// the wave in issue order (loads, stores, LDS DMAs): vm_wait<N> leaves the N youngest in flight.
template <class T>
__device__ __forceinline__ void vm_load16(T& dst, kv_i32x4 rs, int voff) {
  static_assert(sizeof(T) == 16, "buffer_load_dwordx4");
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(dst) : "v"(voff), "s"(rs) : "memory");
}
template <int N, class T>
__device__ __forceinline__ void vm_wait(T& a, T& b) {
  static_assert(N >= 0 && N <= 63, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
template <class T>
__device__ __forceinline__ unsigned lds_addr(const T* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }  // v_cvt_pk_bf16_f32, NaN-safe

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

enum Act : int { kActNone = 0, kActRelu = 1, kActSilu = 2 };

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == kActRelu) return fmaxf(v, 0.0f);
  if (act == kActSilu) return silu(v);
  return v;
}

// Compile-time activation for fused epilogues.  A runtime `act` inside a fully unrolled
// epilogue costs a scalar branch per element (and an IEEE divide per SiLU); the kernels
// instead instantiate the epilogue once per activation pair via dispatch_act().
template <int I>
struct IC {
  static constexpr int value = I;
};

template <int ACT>
__device__ __forceinline__ float act_c(float v) {
  if constexpr (ACT == kActRelu) return fmaxf(v, 0.0f);
  else if constexpr (ACT == kActSilu) return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
  else return v;
}

// act bits: [1:0] activation, bit 2 = residual added AFTER the activation (YOLO
// Bottleneck x + SiLU(conv)); otherwise act(conv + res) (ResNet).  Calls
// f(IC<act1>, IC<act2>): act1 applies to acc + bias, act2 after the residual add.
template <class F>
__device__ __forceinline__ void dispatch_act(int act_bits, bool has_res, F&& f) {
  const int a = act_bits & 3;
  if (!has_res || (act_bits & 4)) {
    if (a == kActRelu) f(IC<kActRelu>{}, IC<kActNone>{});
    else if (a == kActSilu) f(IC<kActSilu>{}, IC<kActNone>{});
    else f(IC<kActNone>{}, IC<kActNone>{});
  } else {
    if (a == kActRelu) f(IC<kActNone>{}, IC<kActRelu>{});
    else if (a == kActSilu) f(IC<kActNone>{}, IC<kActSilu>{});
    else f(IC<kActNone>{}, IC<kActNone>{});
  }
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

}  // namespace kvedge
