// Shared helpers for the libdlamd HIP sources (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/dlamd.h"

namespace dl {

void set_error(const char* fmt, ...);

#define DL_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      ::dl::set_error(__VA_ARGS__);    \
      return 22; /* EINVAL */          \
    }                                  \
  } while (0)

#define DL_RETURN_LAUNCH(name)                                                  \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::dl::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));    \
      return 1000 + (int)e_;                                                    \
    }                                                                           \
    return 0;                                                                   \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One atomic per block for per-step regulariser sums (every thread of the block calls it):
// device-scope atomics on one address serialise across the XCDs (~12 ns each measured — a
// per-wave atomic over a 26 M-row sweep cost ~100 us, over 1.7 M wide rows ~300 us), so
// kernels that use it also cap their grid (kSumGrid blocks, grid-stride loops).
// The block's partial (a fixed-order wave and block sum) is added as 64-bit fixed point
// (units 1/DL_REG_SUM_SCALE, include/dlamd.h): integer adds are associative, so the total is
// the same bits whichever order the blocks land in (a float atomic made the printed loss vary
// from run to run in its last bits).
constexpr unsigned kSumGrid = 1024;
__device__ __forceinline__ void block_fixed_add(float x, int64_t* out) {
  __shared__ float part[16];
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    if (t != 0.f)
      atomicAdd(reinterpret_cast<unsigned long long*>(out),
                (unsigned long long)__double2ll_rn((double)t * DL_REG_SUM_SCALE));
  }
}
// a fixed-point regulariser sum as a double
__device__ __forceinline__ double reg_sum_value(const int64_t* q) { return (double)*q * (1.0 / DL_REG_SUM_SCALE); }

// Reads id and validates it against [0, n); out-of-range -> row -1 + error word.
__device__ __forceinline__ int64_t checked_row(int64_t id, int64_t off, int64_t n, int32_t* err) {
  int64_t r = id + off;
  if (r < 0 || r >= n) {
    if (err) atomicOr(err, 1);
    return -1;
  }
  return r;
}

// Optimizer state block (include/dlamd.h, DL_OPT_*): [0..7] Adam scalars, [8..15] per-step
// regulariser sums, [16] the sticky status word (int32 bits, the host's report), [17] the
// step's skip word.  A set skip word poisons the step: every kernel that writes parameters or
// optimizer state returns without doing so (the gradients it would have consumed are still
// reset), so a batch with an out-of-range id changes nothing — as TF's failing sess.run
// applies nothing before raising — and the next batch applies normally.
__device__ __forceinline__ bool step_poisoned(const float* opt) {
  return __float_as_int(opt[DL_OPT_SKIP]) != 0;
}
// An internal fault (DL_STATUS_LAG / DL_STATUS_INDEX) seen mid-step: reported to the host
// (status) and poisoning the rest of this step and every later one (skip, re-derived from the
// status at each step begin).  `status` points at opt[DL_OPT_STATUS]; the skip word follows it.
__device__ __forceinline__ void raise_fault(int* status, int bits) {
  atomicOr(status, bits);
  atomicOr(status + (DL_OPT_SKIP - DL_OPT_STATUS), bits);
}
// The status bits that poison every later step until the host clears them (internal faults,
// and the sharded step's overflow / desynchronisation, decided identically on every rank).
constexpr int kStickyFaults = DL_STATUS_LAG | DL_STATUS_INDEX | DL_STATUS_OVERFLOW | DL_STATUS_DESYNC;
__device__ __forceinline__ int* opt_status(const float* opt) {
  return const_cast<int*>(reinterpret_cast<const int*>(opt + DL_OPT_STATUS));
}

// One TF1 ApplyAdam element update (training_ops.cc ApplyAdam, non-Nesterov):
//   m += (g - m)(1 - b1);  v += (g^2 - v)(1 - b2);  p -= m * alpha / (sqrt(v) + eps)
// Shared by the dense sweep (optim.hip) and the lazy row-record path (rec.hip) so the
// two compile to the same float operations: a zero-gradient step replayed later by
// rec.hip's catch-up is bit-identical to the step the dense sweep would have taken.
//
// The square root and the reciprocal are the hardware's single instructions
// (v_sqrt_f32, v_rcp_f32: <= 1 ulp each) rather than the correctly rounded sequences of
// Eigen / numpy (~28 instructions): an update differs from TF's by a few ulp of the update
// itself (relative ~2e-7 of |delta p| <= ~1e-3), far inside the 1e-5 parity tolerance, and
// the catch-up replay — the zero-gradient steps of every row a batch touches, ~8 per row
// per step at C2's steady state — runs ~4x faster (it bound the lazy step: DESIGN.md §5).
// DL_ADAM_IEEE=1 builds the correctly rounded form for diagnostics.
#ifndef DL_ADAM_IEEE
#define DL_ADAM_IEEE 0
#endif
__device__ __forceinline__ float adam_step_size(float m, float v, float alpha, float eps) {
#pragma clang fp contract(off)
#if DL_ADAM_IEEE
  return (m * alpha) / (sqrtf(v) + eps);
#else
  return (m * alpha) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) + eps);
#endif
}

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float alpha,
                                          float omb1, float omb2, float eps) {
#pragma clang fp contract(off)
  m = m + (g - m) * omb1;
  v = v + (g * g - v) * omb2;
  p = p - adam_step_size(m, v, alpha, eps);
}

// TF1 Adam._apply_sparse_shared (adam.py), the update of a Variable whose gradient arrives
// as IndexedSlices — one read by tf.nn.embedding_lookup directly, with no concat in between:
// wdl.py:44-47,132 weight_mat, deepfm.py:57-60,78,85,98 feats_emb / feats, dnn.py:49-54
// weight_mat.  m = m*b1 for every row, then scatter_add(g*(1-b1)) on the batch's (deduplicated,
// summed) rows; v likewise with (g*g)*(1-b2); every row then moves by lr*m/(sqrt(v)+eps).  A
// row outside the batch is the g = 0 case of the same formula (x + 0 = x), so one function
// serves the touched rows, the dense sweep and the lazy catch-up alike.
__device__ __forceinline__ void adam_elem_sparse(float& p, float& m, float& v, float g, float alpha, float b1,
                                                 float b2, float omb1, float omb2, float eps) {
#pragma clang fp contract(off)
  m = m * b1 + g * omb1;
  v = v * b2 + (g * g) * omb2;
  p = p - adam_step_size(m, v, alpha, eps);
}

// ---------------------------------------------------------------------------
// Embedding-table Adam state in the root form: the table keeps s = sqrt(v) in place of v
// (records, the dense table sweep, the gather's moment stash; the host converts at the
// boundary: adam_state() exports fl(s*s), set_adam_state() imports fl(sqrt(v))).
//
// Why: a row the batch does not touch takes g = 0 steps — every replayed catch-up step and
// almost every element of the dense sweep.  With g = 0, v' = v * b2 exactly in real
// arithmetic, so s' = s * sqrt(b2): the step needs one reciprocal instead of a square root and
// a reciprocal (the two quarter-rate transcendentals bounded the lazy replay).  sqrt(b2) is
// applied as a two-term product fma(s, c_hi, s * c_lo) (c_hi + c_lo = sqrt(b2) to ~2^-48),
// so an idle row's s drifts by rounding only (random, ~0.5 ulp a step), not by a constant
// ~0.4 ulp a step that a single rounded c would compound over long idle runs.
// A g != 0 step forms v = s * s, applies TF's v update and takes s' = sqrt(v'): the same
// operations as before plus one multiply.  TF parity: v differs from TF's by a few ulp, p by
// a few ulp of its update — far inside the 1e-5 bar.  Lazy / dense bit-identity holds by
// construction: every path applies this one function of (p, m, s, g), and g == 0 selects
// the zero form wherever it arises (a replayed step, an untouched row of the sweep, a touched
// row whose summed gradient is exactly 0).
// s3 weight planes (gemm_s3.hip NT kernels; written by dl_split3 and dl_adam_dense_split3):
// with DL_S3_KPERM the k index of every whole 32-deep chunk is stored permuted, so that lane
// group kq's eight bf16 (positions 8kq .. 8kq+7) hold k = 4kq .. 4kq+3 and 16+4kq .. 16+4kq+3:
// the NT kernel then reads A as two contiguous 64-B half lines per row per chunk (four lane
// groups x 16 B) instead of one whole line in four 16-B pieces per instruction.  A trailing
// partial chunk (K % 32 != 0) stays in natural order.  K = the planes' row length.
#ifndef DL_S3_KPERM
#define DL_S3_KPERM 0
#endif
__host__ __device__ __forceinline__ int s3_kpos(int k, int K) {
  if (!DL_S3_KPERM || (k | 31) >= K) return k;
  const int kk = k & 31;
  return (k & ~31) | (kk < 16 ? 8 * (kk >> 2) + (kk & 3) : 8 * ((kk - 16) >> 2) + 4 + (kk & 3));
}

// The row-offset table of the fused predict front (dl_embed_fwd_gtab writes it,
// dl_gemm_s3_nt_gather_tab stages it in LDS as it stands): per 256-sample tile of the batch,
// per deep field, kGtabPitch u32 — sample b's entry at [b / 256][f][b % 256] holds the byte
// offset of its row in the plane, or kGtabMasked (past any plane: reads as zeros) for a masked
// or invalid id.  The pitch keeps a wave's reads of two fields in disjoint LDS banks.
constexpr int kGtabRows = 256, kGtabPitch = 272;
constexpr uint32_t kGtabMasked = 0xFFFFFF00u;

// DL_ROOT_STATE=0 (A/B builds only: the host's adam_state conversions assume the root form)
// keeps TF's v in the tables as before.
#ifndef DL_ROOT_STATE
#define DL_ROOT_STATE 1
#endif
struct RootDecay {   // c_hi + c_lo = sqrt(b2)
  float hi, lo;
};
__device__ __forceinline__ RootDecay root_decay(float b2) {
  const double c = sqrt((double)b2);   // 1 - (1 - b2) == b2 exactly for b2 in [0.5, 1]
  RootDecay r;
  r.hi = (float)c;
  r.lo = (float)(c - (double)r.hi);
  return r;
}

__device__ __forceinline__ float root_step_size(float m, float s, float alpha, float eps) {
#pragma clang fp contract(off)
#if DL_ADAM_IEEE
  return (m * alpha) / (s + eps);
#else
  return (m * alpha) * __builtin_amdgcn_rcpf(s + eps);
#endif
}

__device__ __forceinline__ float root_sqrt(float v) {
#if DL_ADAM_IEEE
  return sqrtf(v);
#else
  return __builtin_amdgcn_sqrtf(v);
#endif
}

// the g = 0 step of both forms' s
__device__ __forceinline__ float root_decay_step(float s, RootDecay c) { return __builtin_fmaf(s, c.hi, s * c.lo); }

// TF1 ApplyAdam (dense form, adam_elem) on the root state
__device__ __forceinline__ void adam_elem_root(float& p, float& m, float& s, float g, float alpha, float omb1,
                                               float omb2, RootDecay c, float eps) {
#pragma clang fp contract(off)
  if (g == 0.f) {
    m = m + m * (-omb1);
    s = root_decay_step(s, c);
  } else {
    m = m + (g - m) * omb1;
    float v = s * s;
    v = v + (g * g - v) * omb2;
    s = root_sqrt(v);
  }
  p = p - root_step_size(m, s, alpha, eps);
}

// TF1 sparse-apply form (adam_elem_sparse) on the root state
__device__ __forceinline__ void adam_elem_sparse_root(float& p, float& m, float& s, float g, float alpha, float b1,
                                                      float b2, float omb1, float omb2, RootDecay c, float eps) {
#pragma clang fp contract(off)
  if (g == 0.f) {
    m = m * b1;
    s = root_decay_step(s, c);
  } else {
    m = m * b1 + g * omb1;
    const float v = (s * s) * b2 + (g * g) * omb2;
    s = root_sqrt(v);
  }
  p = p - root_step_size(m, s, alpha, eps);
}

#define DL_DISPATCH_E(E, ...)                    \
  switch (E) {                                   \
    case 4: { constexpr int kE = 4; __VA_ARGS__; break; }   \
    case 8: { constexpr int kE = 8; __VA_ARGS__; break; }   \
    case 16: { constexpr int kE = 16; __VA_ARGS__; break; } \
    case 32: { constexpr int kE = 32; __VA_ARGS__; break; } \
    case 64: { constexpr int kE = 64; __VA_ARGS__; break; } \
  }

// References per sample in the batch index: FM slots (use_fm), deep slots, multi-hot slots.
__host__ __device__ __forceinline__ int index_slots(const dl_emb_layout& L) {
  return (L.use_fm ? L.cate_fields : 0) + L.cate_fields + L.multi_width;
}
// first multi-hot reference of a sample
__host__ __device__ __forceinline__ int index_multi_base(const dl_emb_layout& L) {
  return (L.use_fm ? L.cate_fields : 0) + L.cate_fields;
}

// Batch-index key (index.hip): (owner << 27) | local; owner == world marks a replicated row.
__device__ __forceinline__ int64_t decode_key(uint32_t k, int world) {
  const uint32_t owner = k >> 27, local = k & ((1u << 27) - 1);
  return owner >= (uint32_t)world ? (int64_t)local : (int64_t)local * world + owner;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// The wdl wide-weight gradient as 64-bit fixed point (include/dlamd.h DL_WIDE_GRAD_SCALE):
// deterministic integer accumulation of the per-sample dz terms, read back as f32 by the
// wide Adam sweep (DL_ROWS_GRAD_FIXED).
__device__ __forceinline__ long long wide_fixed(float g) { return __double2ll_rn((double)g * DL_WIDE_GRAD_SCALE); }
__device__ __forceinline__ float wide_float(long long q) { return (float)((double)q * (1.0 / DL_WIDE_GRAD_SCALE)); }

// bf16 <-> f32 (bf16 tower): round-to-nearest-even; NaN kept NaN
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(((unsigned)h) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

}  // namespace dl
