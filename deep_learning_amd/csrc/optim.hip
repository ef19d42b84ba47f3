// TF1-faithful Adam (training_ops.cc ApplyAdam, non-Nesterov) and parameter init.
//
// Reference: models/deepfm_pipeline.py:184-188 — exponential_decay(staircase) +
// tf.train.AdamOptimizer(...).minimize(loss, global_step).  The embedding
// gradient reaches its Variable densified (concat + strided-slice, :83-86), so
// TF applies the DENSE update: every element's m and v decay every step and
// every row with m != 0 moves (SURVEY.md ledger item 6).  Here that dense sweep
// is one streaming pass over p, m, v; the gradient table is only read (and
// reset) for rows the step touched, which a uint8 flag per row records — an
// untouched row's gradient is exactly zero, so the result is the dense one.
#include "common.h"

namespace dl {

// opt: [0] b1p [1] b2p [2] lr [3] alpha [4] b1 [5] b2 [6] eps [7] step
__device__ __forceinline__ void adam_begin_body(float* opt, float decay_rate, float decay_steps) {
  if (step_poisoned(opt)) return;   // a failed batch: the step does not begin (common.h)
  const float step = opt[7];
  const float pw = floorf(step / decay_steps);                   // staircase=True
  const float lr_t = opt[2] * powf(decay_rate, pw);
  const float b1p = opt[0], b2p = opt[1];
  opt[3] = lr_t * sqrtf(1.f - b2p) / (1.f - b1p);                // ApplyAdamNonCuda alpha
  opt[0] = b1p * opt[4];                                         // Adam._finish
  opt[1] = b2p * opt[5];
  opt[7] = step + 1.f;                                           // global_step += 1
  for (int i = 8; i < 16; ++i) opt[i] = 0.f;                     // per-step L2 accumulators (all-zero bits)
}

__global__ void adam_begin_kernel(float* opt, float decay_rate, float decay_steps) {
  adam_begin_body(opt, decay_rate, decay_steps);
}

// The batch's id validation (dl_index_build / the forward's err word) poisons the step it
// belongs to: opt's sticky status word gets the batch's error bits before the step begins.
__device__ __forceinline__ void step_guard_kernel_body(const int32_t* batch_err, float* opt) {
  const int e = batch_err[0];
  int* st = opt_status(opt);
  const int bad = e ? ((e & DL_STATUS_BAD_ID) ? DL_STATUS_BAD_ID : e) : 0;
  // this step's skip word: the batch's own bits + any sticky internal fault
  st[DL_OPT_SKIP - DL_OPT_STATUS] = bad | (st[0] & kStickyFaults);
  if (bad) {
    st[0] |= bad;
    opt[DL_OPT_BAD_STEP] = opt[7];            // global_step the bad batch would have advanced from
    opt[DL_OPT_BAD_COUNT] += 1.f;
  }
}

__global__ void step_guard_kernel(const int32_t* batch_err, float* opt) { step_guard_kernel_body(batch_err, opt); }

// The running loss of a training loop — the load-style fit's epoch mean of the per-step loss
// (wdl.py:305-313, deepfm.py:172-190, dnn.py:111-127 sum loss_t * batch_size over the epoch):
// acc[0] += the step's data term (the head slab's loss column summed in a fixed order, in
// double, times inv_b); acc[1] += reg_coef * the step's regulariser sum (the int64 fixed-point
// accumulator at opt[DL_OPT_REG], added to by the Adam kernels); acc[2] += 1.  A skipped step (bad batch) adds nothing.  One block, so the
// step needs no host read; the host reads acc once per epoch.
// ring (may be NULL): the step's status report into pinned host memory, in place of a
// device-to-host copy after the step — every step (skipped ones too) advances the sequence
// opt[DL_OPT_SEQ] to k and writes slot k & 3: [2s] = k and [2s + 1] = the status word in one
// 8-byte store, so a host that reads k there reads this step's status.
__global__ __launch_bounds__(256) void loss_accumulate_kernel(const float* __restrict__ slab, int rows, int pitch,
                                                              int col, double inv_b, float* __restrict__ opt,
                                                              float reg_coef, double* __restrict__ acc,
                                                              int32_t* __restrict__ ring) {
  __shared__ double part[256];
  if (ring && threadIdx.x == 0) {
    // (k, status) as one 8-byte store: the host never sees a slot's k without its status; it
    // lands with this kernel's end-of-kernel release (no system-scope fence, which would write
    // back the L2)
    const int k = __float_as_int(opt[DL_OPT_SEQ]) + 1;
    opt[DL_OPT_SEQ] = __int_as_float(k);
    // the status word: the sticky status bits (low half) and this step's own skip bits (high half)
    const int* st = opt_status(opt);
    const uint32_t word = ((uint32_t)st[0] & 0xffffu) | ((uint32_t)st[DL_OPT_SKIP - DL_OPT_STATUS] << 16);
    *reinterpret_cast<volatile unsigned long long*>(ring + 2 * (k & 3)) =
        (unsigned long long)(uint32_t)k | ((unsigned long long)word << 32);
  }
  if (step_poisoned(opt)) return;
  double s = 0.0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) s += (double)slab[(long long)r * pitch + col];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    acc[0] += part[0] * inv_b;
    acc[1] += (double)reg_coef * reg_sum_value(reinterpret_cast<const int64_t*>(opt + DL_OPT_REG));
    acc[2] += 1.0;
  }
}

// The three scalar updates that open a training step, in one launch (one graph node instead
// of three): the guard (dl_step_guard), the Adam step begin (dl_adam_begin_step) and, for the
// lazy tables, the alpha ring entry (dl_adam_hist_record) — the same operations in the same order.
__global__ void step_begin_kernel(const int32_t* batch_err, float* opt, float decay_rate, float decay_steps,
                                  float* hist, int mask) {
  step_guard_kernel_body(batch_err, opt);
  adam_begin_body(opt, decay_rate, decay_steps);
  if (hist) hist[(int)opt[7] & mask] = opt[3];
}

// The sharded step's opening node, after the request exchange: one decision every rank takes
// from the same data — the headers every rank sent this one (block p from rank p: its count,
// its batch's validation bit, its overflow and sticky fault bits, its global step).  A bad id on
// any rank skips the step everywhere (the batch's bit, not sticky); an overflowing block, an
// internal fault on any rank or ranks at different steps poison this and every later step
// everywhere until the host clears the status (it then replays the skipped steps).
__global__ void shard_step_begin_kernel(const int32_t* __restrict__ hdr, const int32_t* __restrict__ hdr2, int world,
                                        long long cap, long long cap2, float* opt, float decay_rate, float decay_steps,
                                        float* hist, int mask) {
  int fl = 0, bad_ranks = 0;
  const int step = (int)opt[7];
  for (int p = 0; p < world; ++p) {
    const int* h = hdr + 4 * p;
    if (h[0] < 0 || h[0] > cap) fl |= DL_STATUS_INDEX;
    if (h[3] != step) fl |= DL_STATUS_DESYNC;
    fl |= h[1];
    if (h[1] & DL_STATUS_BAD_ID) bad_ranks |= 1 << p;
    if (hdr2) {   // the second id set's blocks (wdl's wide ids): their counts and flags
      const int* h2 = hdr2 + 4 * p;
      if (h2[0] < 0 || h2[0] > cap2) fl |= DL_STATUS_INDEX;
      fl |= h2[1];
      if (h2[1] & DL_STATUS_BAD_ID) bad_ranks |= 1 << p;
    }
  }
  int* st = opt_status(opt);
  const int bad = fl & DL_STATUS_BAD_ID;
  const int sticky = (fl | st[0]) & kStickyFaults;
  st[DL_OPT_SKIP - DL_OPT_STATUS] = bad | sticky;
  st[0] |= bad | sticky;
  if (bad) {
    opt[DL_OPT_BAD_STEP] = opt[7];
    opt[DL_OPT_BAD_COUNT] += 1.f;
    opt[DL_OPT_BAD_RANKS] = __int_as_float(__float_as_int(opt[DL_OPT_BAD_RANKS]) | bad_ranks);
  }
  adam_begin_body(opt, decay_rate, decay_steps);
  if (hist) hist[(int)opt[7] & mask] = opt[3];
}


// One f32 -> its three exact bf16 planes, as gemm_s3.hip's split (v_cvt_pk_bf16_f32, round to
// nearest even): x = hi + mid + lo.
typedef __bf16 dl_optim_bf16x2 __attribute__((ext_vector_type(2)));
typedef float dl_optim_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned short bf16_rne_hw(float x) {
  return (unsigned short)(__builtin_bit_cast(uint32_t, __builtin_convertvector((dl_optim_f32x2){x, 0.f}, dl_optim_bf16x2)) &
                          0xffffu);
}
__device__ __forceinline__ void split3_one(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
#pragma clang fp contract(off)
  h = bf16_rne_hw(x);
  const float r = x - __uint_as_float((uint32_t)h << 16);
  m = bf16_rne_hw(r);
  const float t = r - __uint_as_float((uint32_t)m << 16);
  l = bf16_rne_hw(t);
}

// The s3 tower's operand planes of an updated weight W [rows][cols] (dl_split3's two layouts):
// wp[q][r][c] and wtp[q][c][r], q = hi, mid, lo; plane stride rows * cols.
struct Split3Out {
  unsigned short* wp;
  unsigned short* wtp;
  int rows, cols;
};

// Dense parameter, gradient = sum of partial slabs (+ l2 * p for i < l2_count).
// REG: 0 = L2 (g += l2 * p, sq_out += p^2: tf.contrib.layers.l2_regularizer), 1 = L1
// (g += l1 * sign(p), sq_out += |p|: l1_regularizer, models/dnn.py:88-90).
// NPL: also writes the updated element's operand copies (in place of separate launches after
// the update): 3 = the s3 planes (dl_split3's rounding), 1 = the bf16 copy (dl_cast_bf16 /
// dl_transpose_bf16's rounding, f2bf), 0 = none.
template <int REG, int NPL = 0>
__global__ __launch_bounds__(256) void adam_dense_thread_kernel(float* __restrict__ p, float* __restrict__ m,
                                                                float* __restrict__ v,
                                                                const float* __restrict__ slab, int nslab,
                                                                long long stride, long long n, float l2,
                                                                long long l2_count, const float* __restrict__ opt,
                                                                float* __restrict__ p_prev, int64_t* __restrict__ sq_out,
                                                                Split3Out so = {}) {
  if (step_poisoned(opt)) return;
  const float alpha = opt[3], omb1 = 1.f - opt[4], omb2 = 1.f - opt[5], eps = opt[6];
  const long long plane = NPL ? (long long)so.rows * so.cols : 0;
  float sq = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    // the slab column: 32 (then 16) loads in flight per round trip, added in slab order (the
    // same sum for any grouping)
    float g = 0.f;
    int s = 0;
    for (; s + 32 <= nslab; s += 32) {
      float a[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) a[j] = slab[(s + j) * stride + i];
#pragma unroll
      for (int j = 0; j < 32; ++j) g += a[j];
    }
    for (; s < nslab; s += 16) {   // the rest 16 at a time, loads past the last slab masked
      float a[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = s + j < nslab ? slab[(s + j) * stride + i] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (s + j < nslab) g += a[j];
    }
    float pi = p[i], mi = m[i], vi = v[i];
    if (p_prev) p_prev[i] = pi;
    if (i < l2_count) {
      if (REG == 0) { g += l2 * pi; sq += pi * pi; }
      else { g += l2 * (pi > 0.f ? 1.f : pi < 0.f ? -1.f : 0.f); sq += fabsf(pi); }
    }
    adam_elem(pi, mi, vi, g, alpha, omb1, omb2, eps);
    p[i] = pi; m[i] = mi; v[i] = vi;
    if (NPL == 3) {
      unsigned short h, mm, l;
      split3_one(pi, h, mm, l);
      const int r = (int)(i / so.cols), c = (int)(i - (long long)r * so.cols);
      const long long w = (long long)r * so.cols + s3_kpos(c, so.cols);   // dl_split3's layouts
      so.wp[w] = h; so.wp[plane + w] = mm; so.wp[2 * plane + w] = l;
      const long long t = (long long)c * so.rows + s3_kpos(r, so.rows);
      so.wtp[t] = h; so.wtp[plane + t] = mm; so.wtp[2 * plane + t] = l;
    } else if (NPL == 1) {
      const unsigned short h = f2bf(pi);
      const int r = (int)(i / so.cols), c = (int)(i - (long long)r * so.cols);
      so.wp[i] = h;
      so.wtp[(long long)c * so.rows + r] = h;
    }
  }
  if (sq_out) block_fixed_add(sq, sq_out);
}

// Several tower weights in one launch (dl_adam_dense_layers): thread i of the concatenated
// element ranges runs adam_dense_thread_kernel's per-element code for its layer.
struct AdamLayersArg {
  dl_adam_layer l[DL_ADAM_MAX_LAYERS];
  long long start[DL_ADAM_MAX_LAYERS + 1];   // element offsets of the layers in the concatenation
  int nl;
};

template <int NPL>
__global__ __launch_bounds__(256) void adam_dense_layers_kernel(AdamLayersArg a, const float* __restrict__ opt) {
  if (step_poisoned(opt)) return;
  const float alpha = opt[3], omb1 = 1.f - opt[4], omb2 = 1.f - opt[5], eps = opt[6];
  float sq[DL_ADAM_MAX_LAYERS] = {0.f, 0.f, 0.f, 0.f};
  const long long total = a.start[a.nl];
  for (long long gi = (long long)blockIdx.x * blockDim.x + threadIdx.x; gi < total;
       gi += (long long)gridDim.x * blockDim.x) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < DL_ADAM_MAX_LAYERS; ++j) k += (j < a.nl && gi >= a.start[j]) ? 1 : 0;
    const dl_adam_layer& L = a.l[k];
    const long long i = gi - a.start[k];
    const float* __restrict__ slab = L.slab;
    const long long stride = L.slab_stride;
    const int nslab = L.nslab;
    float g = 0.f;
    int s = 0;
    for (; s + 32 <= nslab; s += 32) {
      float t[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) t[j] = slab[(s + j) * stride + i];
#pragma unroll
      for (int j = 0; j < 32; ++j) g += t[j];
    }
    for (; s < nslab; s += 16) {   // the rest 16 at a time, loads past the last slab masked
      float t[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) t[j] = s + j < nslab ? slab[(s + j) * stride + i] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (s + j < nslab) g += t[j];
    }
    float pi = L.p[i], mi = L.m[i], vi = L.v[i];
    if (i < L.reg_count) {
      if (L.reg_kind == 0) { g += L.reg * pi; sq[k] += pi * pi; }
      else { g += L.reg * (pi > 0.f ? 1.f : pi < 0.f ? -1.f : 0.f); sq[k] += fabsf(pi); }
    }
    adam_elem(pi, mi, vi, g, alpha, omb1, omb2, eps);
    L.p[i] = pi; L.m[i] = mi; L.v[i] = vi;
    unsigned short* wp = reinterpret_cast<unsigned short*>(L.wp);
    unsigned short* wtp = reinterpret_cast<unsigned short*>(L.wtp);
    const int r = (int)(i / L.cols), c = (int)(i - (long long)r * L.cols);
    if (NPL == 3) {
      const long long plane = (long long)L.rows * L.cols;
      unsigned short h, mm, l;
      split3_one(pi, h, mm, l);
      const long long w = (long long)r * L.cols + s3_kpos(c, L.cols);   // dl_split3's layouts
      wp[w] = h; wp[plane + w] = mm; wp[2 * plane + w] = l;
      const long long t = (long long)c * L.rows + s3_kpos(r, L.rows);
      wtp[t] = h; wtp[plane + t] = mm; wtp[2 * plane + t] = l;
    } else if (NPL == 1) {
      const unsigned short h = f2bf(pi);
      wp[i] = h;
      wtp[(long long)c * L.rows + r] = h;
    }
  }
  for (int k = 0; k < a.nl; ++k)   // the regulariser terms (uniform branch: every thread joins)
    if (a.l[k].acc_out) {
      block_fixed_add(sq[k], a.l[k].acc_out);
      __syncthreads();             // block_atomic_add's partials are reused by the next layer
    }
}

// Few elements, many slabs (head weights): one wave per element.
template <int REG>
__global__ __launch_bounds__(256) void adam_dense_wave_kernel(float* __restrict__ p, float* __restrict__ m,
                                                              float* __restrict__ v,
                                                              const float* __restrict__ slab, int nslab,
                                                              long long stride, long long n, float l2,
                                                              long long l2_count, const float* __restrict__ opt,
                                                              float* __restrict__ p_prev, int64_t* __restrict__ sq_out) {
  if (step_poisoned(opt)) return;
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  float sq = 0.f;
  if (i < n) {   // no early return: the whole block meets in block_atomic_add
    float g = 0.f;
    for (int s = lane; s < nslab; s += 64) g += slab[s * stride + i];
    g = wave_sum(g);
    if (lane == 0) {
      float pi = p[i], mi = m[i], vi = v[i];
      if (p_prev) p_prev[i] = pi;
      if (i < l2_count) {
        if (REG == 0) { g += l2 * pi; sq = pi * pi; }
        else { g += l2 * (pi > 0.f ? 1.f : pi < 0.f ? -1.f : 0.f); sq = fabsf(pi); }
      }
      adam_elem(pi, mi, vi, g, opt[3], 1.f - opt[4], 1.f - opt[5], opt[6]);
      p[i] = pi; m[i] = mi; v[i] = vi;
    }
  }
  if (sq_out) block_fixed_add(sq, sq_out);
}

// Table element update in the reference's form for the table: ApplyAdam (dense) or the
// sparse-apply form of Variables read by embedding_lookup directly (common.h).  ROOT: the
// embedding tables' root state (v holds s = sqrt(v): common.h adam_elem_root, the form the
// lazy records replay); the wdl wide weights (fixed-point gradients) keep v.
template <bool SPARSE, bool ROOT>
__device__ __forceinline__ void table_adam(float& p, float& m, float& v, float g, float alpha, float b1, float b2,
                                           float omb1, float omb2, RootDecay rd, float eps) {
  if (ROOT && DL_ROOT_STATE) {
    if (SPARSE) adam_elem_sparse_root(p, m, v, g, alpha, b1, b2, omb1, omb2, rd, eps);
    else adam_elem_root(p, m, v, g, alpha, omb1, omb2, rd, eps);
  } else {
    if (SPARSE) adam_elem_sparse(p, m, v, g, alpha, b1, b2, omb1, omb2, eps);
    else adam_elem(p, m, v, g, alpha, omb1, omb2, eps);
  }
}

// Embedding table rows of width W (multiple of 4): one thread per float4.
template <bool SPARSE>
__global__ __launch_bounds__(256) void adam_rows4_kernel(float4* __restrict__ p, float4* __restrict__ m,
                                                         float4* __restrict__ v, float4* __restrict__ g,
                                                         const uint8_t* __restrict__ touched, long long n4,
                                                         int lpr, float l2, const float* __restrict__ opt,
                                                         int64_t* __restrict__ sq_out) {
  const float alpha = opt[3], b1 = opt[4], b2 = opt[5], omb1 = 1.f - opt[4], omb2 = 1.f - opt[5], eps = opt[6];
  const RootDecay rd = root_decay(b2);
  const bool skip = step_poisoned(opt);   // consume the gradients, apply nothing
  float sq = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / lpr;
    float4 pi = p[i], mi = m[i], vi = v[i];   // issued before the touched test: one round trip
    float4 gi = make_float4(0.f, 0.f, 0.f, 0.f);
    if (touched[row]) {
      gi = g[i];
      g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (skip) continue;
    if (l2 != 0.f) { gi.x += l2 * pi.x; gi.y += l2 * pi.y; gi.z += l2 * pi.z; gi.w += l2 * pi.w; }
    if (sq_out) sq += pi.x * pi.x + pi.y * pi.y + pi.z * pi.z + pi.w * pi.w;
    table_adam<SPARSE, true>(pi.x, mi.x, vi.x, gi.x, alpha, b1, b2, omb1, omb2, rd, eps);
    table_adam<SPARSE, true>(pi.y, mi.y, vi.y, gi.y, alpha, b1, b2, omb1, omb2, rd, eps);
    table_adam<SPARSE, true>(pi.z, mi.z, vi.z, gi.z, alpha, b1, b2, omb1, omb2, rd, eps);
    table_adam<SPARSE, true>(pi.w, mi.w, vi.w, gi.w, alpha, b1, b2, omb1, omb2, rd, eps);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
  if (sq_out) block_fixed_add(sq, sq_out);
}

// Width-1 tables (first-order weights): one thread per 4 rows.
template <bool SPARSE, bool FIXED>
__global__ __launch_bounds__(256) void adam_rows1_kernel(float* __restrict__ p, float* __restrict__ m,
                                                         float* __restrict__ v, void* __restrict__ g_,
                                                         uint8_t* __restrict__ touched, long long n,
                                                         float l2, int clear, const float* __restrict__ opt,
                                                         int64_t* __restrict__ sq_out) {
  const float alpha = opt[3], b1 = opt[4], b2 = opt[5], omb1 = 1.f - opt[4], omb2 = 1.f - opt[5], eps = opt[6];
  const RootDecay rd = root_decay(b2);
  const bool skip = step_poisoned(opt);
  const long long n4 = n / 4;
  float sq = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n + 3) / 4;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < n4) {
      // p, m, v issued before the touched test: one round trip instead of two
      float4 pi = reinterpret_cast<float4*>(p)[i], mi = reinterpret_cast<float4*>(m)[i],
             vi = reinterpret_cast<float4*>(v)[i];
      const uchar4 t = reinterpret_cast<const uchar4*>(touched)[i];
      float4 gi = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t.x | t.y | t.z | t.w) {
        if (FIXED) {   // 64-bit fixed-point gradient (the wdl wide weights)
          long long* q = reinterpret_cast<long long*>(g_) + 4 * i;
          gi = make_float4(wide_float(q[0]), wide_float(q[1]), wide_float(q[2]), wide_float(q[3]));
          q[0] = 0; q[1] = 0; q[2] = 0; q[3] = 0;
        } else {
          float4* g4 = reinterpret_cast<float4*>(g_) + i;
          gi = *g4;
          *g4 = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (!t.x) gi.x = 0.f; if (!t.y) gi.y = 0.f; if (!t.z) gi.z = 0.f; if (!t.w) gi.w = 0.f;
        if (clear) reinterpret_cast<uchar4*>(touched)[i] = make_uchar4(0, 0, 0, 0);
      }
      if (skip) continue;
      // the L2 term as one fma (wide.hip's lazy replay uses the same expression: bit-identical)
      if (l2 != 0.f) { gi.x = fmaf(l2, pi.x, gi.x); gi.y = fmaf(l2, pi.y, gi.y); gi.z = fmaf(l2, pi.z, gi.z); gi.w = fmaf(l2, pi.w, gi.w); }
      sq += pi.x * pi.x + pi.y * pi.y + pi.z * pi.z + pi.w * pi.w;
      table_adam<SPARSE, !FIXED>(pi.x, mi.x, vi.x, gi.x, alpha, b1, b2, omb1, omb2, rd, eps);
      table_adam<SPARSE, !FIXED>(pi.y, mi.y, vi.y, gi.y, alpha, b1, b2, omb1, omb2, rd, eps);
      table_adam<SPARSE, !FIXED>(pi.z, mi.z, vi.z, gi.z, alpha, b1, b2, omb1, omb2, rd, eps);
      table_adam<SPARSE, !FIXED>(pi.w, mi.w, vi.w, gi.w, alpha, b1, b2, omb1, omb2, rd, eps);
      reinterpret_cast<float4*>(p)[i] = pi; reinterpret_cast<float4*>(m)[i] = mi;
      reinterpret_cast<float4*>(v)[i] = vi;
    } else {
      for (long long r = 4 * i; r < n; ++r) {
        float gi = 0.f;
        if (touched[r]) {
          if (FIXED) {
            gi = wide_float(reinterpret_cast<long long*>(g_)[r]);
            reinterpret_cast<long long*>(g_)[r] = 0;
          } else {
            gi = reinterpret_cast<float*>(g_)[r];
            reinterpret_cast<float*>(g_)[r] = 0.f;
          }
          if (clear) touched[r] = 0;
        }
        if (skip) continue;
        float pi = p[r], mi = m[r], vi = v[r];
        if (l2 != 0.f) gi = fmaf(l2, pi, gi);
        sq += pi * pi;
        table_adam<SPARSE, !FIXED>(pi, mi, vi, gi, alpha, b1, b2, omb1, omb2, rd, eps);
        p[r] = pi; m[r] = mi; v[r] = vi;
      }
    }
  }
  if (sq_out) block_fixed_add(sq, sq_out);
}

__global__ void clear_touched_kernel(uint8_t* touched, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n + 15) / 16;
       i += (long long)gridDim.x * blockDim.x) {
    if (16 * i + 16 <= n) reinterpret_cast<uint4*>(touched)[i] = make_uint4(0, 0, 0, 0);
    else for (long long r = 16 * i; r < n; ++r) touched[r] = 0;
  }
}

// ---------------------------------------------------------------------------
// Philox-4x32-10 counter-based RNG
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    c = make_uint4((unsigned)(p1 >> 32) ^ c.y ^ k.x, (unsigned)p1, (unsigned)(p0 >> 32) ^ c.w ^ k.y,
                   (unsigned)p0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ __launch_bounds__(256) void init_random_kernel(float* p, long long n, int dist, float mean,
                                                          float scale, unsigned long long seed,
                                                          unsigned long long offset) {
  const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; 4 * i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long ctr = offset / 4 + (unsigned long long)i;
    const uint4 r = philox(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), 0x5eedu, 0u), key);
    const float u0 = (r.x >> 8) * (1.f / 16777216.f), u1 = (r.y >> 8) * (1.f / 16777216.f);
    const float u2 = (r.z >> 8) * (1.f / 16777216.f), u3 = (r.w >> 8) * (1.f / 16777216.f);
    float o[4];
    if (dist == 0) {  // Box-Muller
      const float a = sqrtf(-2.f * logf(1.f - u0)), b = sqrtf(-2.f * logf(1.f - u2));
      o[0] = a * cospif(2.f * u1); o[1] = a * sinpif(2.f * u1);
      o[2] = b * cospif(2.f * u3); o[3] = b * sinpif(2.f * u3);
      for (int j = 0; j < 4; ++j) o[j] = mean + scale * o[j];
    } else {
      o[0] = mean + scale * u0; o[1] = mean + scale * u1; o[2] = mean + scale * u2; o[3] = mean + scale * u3;
    }
    for (int j = 0; j < 4; ++j)
      if (4 * i + j < n) p[4 * i + j] = o[j];
  }
}

static int grid_for(long long n, int per_thread = 1) {
  long long g = (n / per_thread + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  return g < 1 ? 1 : (int)g;
}

}  // namespace dl

using namespace dl;

extern "C" int dl_adam_begin_step(float* opt, float decay_rate, float decay_steps, void* stream) {
  DL_CHECK_ARG(opt != nullptr, "opt is NULL");
  hipLaunchKernelGGL(adam_begin_kernel, dim3(1), dim3(1), 0, as_stream(stream), opt, decay_rate, decay_steps);
  DL_RETURN_LAUNCH("dl_adam_begin_step");
}

extern "C" int dl_step_guard(const int32_t* batch_err, float* opt, void* stream) {
  DL_CHECK_ARG(batch_err && opt, "NULL pointer");
  hipLaunchKernelGGL(step_guard_kernel, dim3(1), dim3(1), 0, as_stream(stream), batch_err, opt);
  DL_RETURN_LAUNCH("dl_step_guard");
}

extern "C" int dl_loss_accumulate(const float* slab, int32_t rows, int32_t pitch, int32_t col, double inv_b,
                                  float* opt, float reg_coef, double* acc, int32_t* status_ring, void* stream) {
  DL_CHECK_ARG(slab && opt && acc, "NULL pointer");
  DL_CHECK_ARG(rows >= 0 && pitch > col && col >= 0, "bad slab shape");
  hipLaunchKernelGGL(loss_accumulate_kernel, dim3(1), dim3(256), 0, as_stream(stream), slab, rows, pitch, col, inv_b,
                     opt, reg_coef, acc, status_ring);
  DL_RETURN_LAUNCH("dl_loss_accumulate");
}

extern "C" int dl_shard_step_begin(const int32_t* hdr, const int32_t* hdr2, int32_t world, int64_t cap, int64_t cap2,
                                   float* opt, float decay_rate, float decay_steps, float* hist, int32_t hist_len,
                                   void* stream) {
  DL_CHECK_ARG(hdr && opt && world >= 1 && world <= 31 && cap >= 1 && (!hdr2 || cap2 >= 1), "bad args");
  DL_CHECK_ARG(!hist || (hist_len >= 2 && (hist_len & (hist_len - 1)) == 0), "bad hist");
  hipLaunchKernelGGL(shard_step_begin_kernel, dim3(1), dim3(1), 0, as_stream(stream), hdr, hdr2, world, (long long)cap,
                     (long long)cap2, opt, decay_rate, decay_steps, hist, hist ? hist_len - 1 : 0);
  DL_RETURN_LAUNCH("dl_shard_step_begin");
}

extern "C" int dl_step_begin(const int32_t* batch_err, float* opt, float decay_rate, float decay_steps, float* hist,
                             int32_t hist_len, void* stream) {
  DL_CHECK_ARG(batch_err && opt, "NULL pointer");
  DL_CHECK_ARG(!hist || (hist_len >= 2 && (hist_len & (hist_len - 1)) == 0), "bad hist");
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(1), 0, as_stream(stream), batch_err, opt, decay_rate,
                     decay_steps, hist, hist ? hist_len - 1 : 0);
  DL_RETURN_LAUNCH("dl_step_begin");
}

extern "C" int dl_adam_dense_reg(float* p, float* m, float* v, const float* slab, int32_t nslab,
                                 int64_t slab_stride, int64_t n, float reg, int64_t reg_count, int32_t reg_kind,
                                 const float* opt, float* p_prev, int64_t* acc_out, void* stream) {
  DL_CHECK_ARG(p && m && v && slab && opt, "NULL pointer");
  DL_CHECK_ARG(nslab >= 1 && slab_stride >= n, "bad slabs");
  DL_CHECK_ARG(reg_kind == 0 || reg_kind == 1, "reg_kind must be 0 (L2) or 1 (L1)");
  if (n == 0) return 0;
#define DL_ADAM_DENSE(R)                                                                                      \
  if (n < 16384 && nslab >= 32) {                                                                             \
    const long long blocks = (n * 64 + 255) / 256;                                                            \
    hipLaunchKernelGGL(adam_dense_wave_kernel<R>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, \
                       m, v, slab, nslab, (long long)slab_stride, (long long)n, reg, (long long)reg_count, opt, \
                       p_prev, acc_out);                                                                      \
  } else {                                                                                                    \
    hipLaunchKernelGGL(adam_dense_thread_kernel<R>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, m, \
                       v, slab, nslab, (long long)slab_stride, (long long)n, reg, (long long)reg_count, opt,    \
                       p_prev, acc_out, Split3Out{});                                                         \
  }
  if (reg_kind == 0) { DL_ADAM_DENSE(0) } else { DL_ADAM_DENSE(1) }
#undef DL_ADAM_DENSE
  DL_RETURN_LAUNCH("dl_adam_dense_reg");
}

template <int NPL>
static int adam_dense_copies(float* p, float* m, float* v, const float* slab, int32_t nslab, int64_t slab_stride,
                             int32_t rows, int32_t cols, float reg, int64_t reg_count, int32_t reg_kind,
                             const float* opt, int64_t* acc_out, uint16_t* wp, uint16_t* wtp, void* stream) {
  DL_CHECK_ARG(p && m && v && slab && opt && wp && wtp, "NULL pointer");
  const long long n = (long long)rows * cols;
  DL_CHECK_ARG(rows > 0 && cols > 0 && nslab >= 1 && slab_stride >= n, "bad shape / slabs");
  DL_CHECK_ARG(reg_kind == 0 || reg_kind == 1, "reg_kind must be 0 (L2) or 1 (L1)");
  const Split3Out so{reinterpret_cast<unsigned short*>(wp), reinterpret_cast<unsigned short*>(wtp), rows, cols};
  if (reg_kind == 0)
    hipLaunchKernelGGL((adam_dense_thread_kernel<0, NPL>), dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, m, v,
                       slab, nslab, (long long)slab_stride, n, reg, (long long)reg_count, opt, nullptr, acc_out, so);
  else
    hipLaunchKernelGGL((adam_dense_thread_kernel<1, NPL>), dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, m, v,
                       slab, nslab, (long long)slab_stride, n, reg, (long long)reg_count, opt, nullptr, acc_out, so);
  DL_RETURN_LAUNCH(NPL == 3 ? "dl_adam_dense_split3" : "dl_adam_dense_bf16");
}

extern "C" int dl_adam_dense_split3(float* p, float* m, float* v, const float* slab, int32_t nslab,
                                    int64_t slab_stride, int32_t rows, int32_t cols, float reg, int64_t reg_count,
                                    int32_t reg_kind, const float* opt, int64_t* acc_out, uint16_t* wp, uint16_t* wtp,
                                    void* stream) {
  return adam_dense_copies<3>(p, m, v, slab, nslab, slab_stride, rows, cols, reg, reg_count, reg_kind, opt, acc_out,
                              wp, wtp, stream);
}

extern "C" int dl_adam_dense_layers(int32_t n_layers, const dl_adam_layer* layers, int32_t copies, const float* opt,
                                    void* stream) {
  DL_CHECK_ARG(n_layers >= 1 && n_layers <= DL_ADAM_MAX_LAYERS && layers && opt,
               "n_layers %d: 1..%d and non-NULL arguments", n_layers, DL_ADAM_MAX_LAYERS);
  DL_CHECK_ARG(copies == 3 || copies == 1, "copies %d: 3 (s3 planes) or 1 (bf16)", copies);
  AdamLayersArg a{};
  a.nl = n_layers;
  long long off = 0;
  for (int k = 0; k < n_layers; ++k) {
    const dl_adam_layer& L = layers[k];
    const long long n = (long long)L.rows * L.cols;
    DL_CHECK_ARG(L.p && L.m && L.v && L.slab && L.wp && L.wtp, "layer %d: NULL pointer", k);
    DL_CHECK_ARG(L.rows > 0 && L.cols > 0 && L.nslab >= 1 && L.slab_stride >= n, "layer %d: bad shape / slabs", k);
    DL_CHECK_ARG(L.reg_kind == 0 || L.reg_kind == 1, "layer %d: reg_kind must be 0 (L2) or 1 (L1)", k);
    a.l[k] = L;
    a.start[k] = off;
    off += n;
  }
  for (int k = n_layers; k <= DL_ADAM_MAX_LAYERS; ++k) a.start[k] = off;
  if (copies == 3)
    hipLaunchKernelGGL(adam_dense_layers_kernel<3>, dim3(grid_for(off)), dim3(256), 0, as_stream(stream), a, opt);
  else
    hipLaunchKernelGGL(adam_dense_layers_kernel<1>, dim3(grid_for(off)), dim3(256), 0, as_stream(stream), a, opt);
  DL_RETURN_LAUNCH("dl_adam_dense_layers");
}

extern "C" int dl_adam_dense_bf16(float* p, float* m, float* v, const float* slab, int32_t nslab,
                                  int64_t slab_stride, int32_t rows, int32_t cols, float reg, int64_t reg_count,
                                  int32_t reg_kind, const float* opt, int64_t* acc_out, uint16_t* wb, uint16_t* wbt,
                                  void* stream) {
  return adam_dense_copies<1>(p, m, v, slab, nslab, slab_stride, rows, cols, reg, reg_count, reg_kind, opt, acc_out,
                              wb, wbt, stream);
}

extern "C" int dl_adam_dense(float* p, float* m, float* v, const float* slab, int32_t nslab,
                             int64_t slab_stride, int64_t n, float l2, int64_t l2_count,
                             const float* opt, float* p_prev, int64_t* sq_out, void* stream) {
  return dl_adam_dense_reg(p, m, v, slab, nslab, slab_stride, n, l2, l2_count, 0, opt, p_prev, sq_out, stream);
}

extern "C" int dl_adam_rows(float* p, float* m, float* v, void* g, uint8_t* touched, int64_t n_rows,
                            int32_t width, float l2, int32_t rows_flags, const float* opt, int64_t* sq_out,
                            void* stream) {
  const int clear_touched = rows_flags & DL_ROWS_CLEAR_TOUCHED;
  const bool sparse = (rows_flags & DL_ROWS_SPARSE_ADAM) != 0;
  const bool fixed = (rows_flags & DL_ROWS_GRAD_FIXED) != 0;
  DL_CHECK_ARG(!fixed || width == 1, "the fixed-point gradient form is for width-1 rows");
  DL_CHECK_ARG(p && m && v && g && touched && opt, "NULL pointer");
  DL_CHECK_ARG(width == 1 || width % 4 == 0, "width must be 1 or a multiple of 4");
  DL_CHECK_ARG(((uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g) % 16 == 0, "16-B alignment");
  if (n_rows == 0) return 0;
  hipStream_t s = as_stream(stream);
  if (width == 1) {
    DL_CHECK_ARG(((uintptr_t)touched % 4) == 0, "touched must be 4-B aligned");
    auto k = fixed ? (sparse ? adam_rows1_kernel<true, true> : adam_rows1_kernel<false, true>)
                   : (sparse ? adam_rows1_kernel<true, false> : adam_rows1_kernel<false, false>);
    hipLaunchKernelGGL(k, dim3(grid_for(n_rows, 4)), dim3(256), 0, s, p, m, v, g, touched, (long long)n_rows, l2,
                       clear_touched, opt, sq_out);
  } else {
    const long long n4 = n_rows * (width / 4);
    hipLaunchKernelGGL(sparse ? adam_rows4_kernel<true> : adam_rows4_kernel<false>, dim3(grid_for(n4)), dim3(256),
                       0, s, (float4*)p, (float4*)m, (float4*)v, (float4*)g, touched, n4, width / 4, l2, opt,
                       sq_out);
    if (clear_touched) {
      DL_CHECK_ARG(((uintptr_t)touched % 16) == 0, "touched must be 16-B aligned");
      hipLaunchKernelGGL(clear_touched_kernel, dim3(grid_for(n_rows, 16)), dim3(256), 0, s, touched,
                         (long long)n_rows);
    }
  }
  DL_RETURN_LAUNCH("dl_adam_rows");
}

extern "C" int dl_init_random(float* p, int64_t n, int32_t dist, float mean, float scale, uint64_t seed,
                              uint64_t offset, void* stream) {
  DL_CHECK_ARG(p && n >= 0 && offset % 4 == 0, "bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(init_random_kernel, dim3(grid_for(n, 4)), dim3(256), 0, as_stream(stream), p,
                     (long long)n, dist, mean, scale, (unsigned long long)seed, (unsigned long long)offset);
  DL_RETURN_LAUNCH("dl_init_random");
}
