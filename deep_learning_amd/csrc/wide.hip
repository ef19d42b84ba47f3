// Lazy-exact TF1 Adam for Wide&Deep's wide weights (models/wdl.py:241-285).
//
// wdl_weights [N + H, 1] carries an L2 penalty on every row (wdl.py:270-271), so TF's
// gradient is dense: each step every row r gets g_r = (batch term) + l2 * w_r and every row's
// w, m, v move — a 26 M-row sweep of p, m, v per step (the dense form, dl_adam_rows).  Here a
// row the batch does not reference is left alone and its skipped steps are replayed when it is
// next read: for each skipped step j, g = l2 * w (the dense sweep's gradient of an untouched
// row), then the same adam_elem — bit-identical to the sweep, only computed later.
//
// Record per row: float4 {w, m, v, stamp} (stamp = int32 bits of the last step applied).
// (128-B slots written whole, to spare the partial-line merges of the random updates, measured
// slower: update 70 -> 92 us, gather 58 -> 69 us at C5 — 8x the table's span for the random
// accesses; profiles/r03t/.)
// One step (single GPU, the batch's wide ids indexed by dl_index_build):
//   dl_wide_rec_gather   unique wide rows + the H deep-output rows caught up to t - lag, into
//                        the head's compact local table wloc = [— (Fw) | deep rows Fw..Fw+H |
//                        unique wide rows]; the unique rows' caught-up state stashed
//   (dl_wdl_head_fwd_bwd on local ids: int64 fixed-point gradients per local row in gloc)
//   dl_wide_rec_update   the TF1 Adam step t of every touched row (the batch's unique wide rows
//                        and the H deep-output rows; a row that is both gets both gradient
//                        parts summed exactly in fixed point first), written with stamp t; the
//                        L2 loss term of these rows (pre-update w^2) into sq_out
//   dl_wide_rec_flush    every row caught up to step t (the flush schedule, exports); the L2
//                        loss term of the rows the last step did not touch comes with it
#include "common.h"

namespace dl {

constexpr int kWideRecF4 = 1;   // float4s per record slot

// the whole slot: the record, then zeros
__device__ __forceinline__ void wide_rec_store(float4* __restrict__ rec, long long row, float4 r) {
  float4* q = rec + row * kWideRecF4;
  q[0] = r;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 1; i < kWideRecF4; ++i) q[i] = z;
}

// per-block partial sums of the L2 term (every thread of the block calls it): written, not
// added, so the update kernels need no grid cap for atomics; the host sums the partials
__device__ __forceinline__ void block_sum_store(float x, float* out) {
  __shared__ float part[16];
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    *out = t;
  }
}

// uncapped grid of a one-thread-per-row kernel (the chains of dependent loads want every row in flight)
static unsigned wide_rows_grid(long long n) {
  long long b = (n + 255) / 256;
  if (b > 65535) b = 65535;
  return (unsigned)(b < 1 ? 1 : b);
}

struct WideHyper {
  float b1, b2, omb1, omb2, eps, l2;
  int mask;
};

__device__ __forceinline__ WideHyper wide_hyper(const float* opt, float l2, int hist_len) {
  return WideHyper{opt[4], opt[5], 1.f - opt[4], 1.f - opt[5], opt[6], l2, hist_len - 1};
}

// the dense sweep's gradient of a row: batch term + l2 * w (adam_rows1_kernel, the same fma)
__device__ __forceinline__ float wide_l2_grad(float g, float l2, float w) { return fmaf(l2, w, g); }

// steps from+1 .. to with a zero batch term (rows the batch did not touch)
__device__ __forceinline__ void wide_catch_up(float& w, float& m, float& v, int from, int to, const float* __restrict__ hist,
                                              const WideHyper& h) {
  for (int j = from + 1; j <= to; ++j)
    adam_elem(w, m, v, wide_l2_grad(0.f, h.l2, w), hist[j & h.mask], h.omb1, h.omb2, h.eps);
}

// the same, summing w^2 of each replayed step's pre-update state (the loss's L2 term of that
// step for this row: wdl.py:270-271) into sq
__device__ __forceinline__ void wide_catch_up_sq(float& w, float& m, float& v, int from, int to,
                                                 const float* __restrict__ hist, const WideHyper& h, float& sq) {
  for (int j = from + 1; j <= to; ++j) {
    sq = fmaf(w, w, sq);
    adam_elem(w, m, v, wide_l2_grad(0.f, h.l2, w), hist[j & h.mask], h.omb1, h.omb2, h.eps);
  }
}

// A kernel's running-loss contribution: the block's sum added to its own slot of acc (double;
// slots are per block index, and the kernels that add to them run in stream order, so no
// atomics).  The host sums the slots when it reads the running loss (engine.loss_sum_end).
__device__ __forceinline__ void block_sum_accumulate(float x, double* acc) {
  __shared__ float part[16];
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    acc[blockIdx.x] += (double)t;
  }
  __syncthreads();
}

__device__ __forceinline__ int wide_from(float stamp_bits, int target, int hist_len, int* status) {
  const int st = __float_as_int(stamp_bits);
  if (target - st >= hist_len - 1) {   // lagged past the alpha ring: report, never truncate silently
    raise_fault(status, DL_STATUS_LAG);
    return target;
  }
  return st;
}

// Unique wide rows u < n_uniq (rows uniq[u]) and the H deep-output rows Fw + j, caught up to
// step opt[7] - lag: wloc[Fw + j] / wloc[Fw + H + u] = w; stash[u] = (w, m, v, row bits).
__global__ __launch_bounds__(256) void wide_rec_gather_kernel(const float4* __restrict__ rec, long long w_rows,
                                                              const uint32_t* __restrict__ uniq,
                                                              const int32_t* __restrict__ n_uniq, long long max_u,
                                                              int Fw, int H, const float* __restrict__ hist,
                                                              int hist_len, const float* __restrict__ opt, float l2,
                                                              int lag, float* __restrict__ wloc,
                                                              float4* __restrict__ stash, float* __restrict__ rep_sq) {
  const WideHyper h = wide_hyper(opt, l2, hist_len);
  int* status = opt_status(opt);
  const int target = (int)opt[7] - lag;
  const long long nu = n_uniq ? (long long)min((long long)max(n_uniq[0], 0), max_u) : max_u;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < H + nu;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i < H ? Fw + i : (long long)uniq[i - H];
    if (row < 0 || row >= w_rows) {
      raise_fault(status, DL_STATUS_INDEX);
      continue;
    }
    float4 r = rec[row * kWideRecF4];
    const int from = wide_from(r.w, target, hist_len, status);
    float sq = 0.f;
    if (from < target) {
      if (rep_sq && i >= H) wide_catch_up_sq(r.x, r.y, r.z, from, target, hist, h, sq);
      else wide_catch_up(r.x, r.y, r.z, from, target, hist, h);
    }
    wloc[Fw + i] = r.x;   // i < H: the deep-output row Fw + i; else local row Fw + H + u
    if (i >= H && stash) stash[i - H] = make_float4(r.x, r.y, r.z, __int_as_float((int)row));
    if (i >= H && rep_sq) rep_sq[i - H] = sq;   // the replayed steps' L2 terms, counted once the update lands
  }
}

// Pass A: the batch's unique wide rows.  g = (its wide terms + its deep-output term when the row
// is one of Fw..Fw+H: exact int64 sum) + l2 * w, TF1 Adam step t from the stashed caught-up
// state, record written with stamp t.  Deep-output rows it covered are marked for pass B.
__global__ __launch_bounds__(256) void wide_rec_update_kernel(float4* __restrict__ rec, const int32_t* __restrict__ n_uniq,
                                                              long long max_u, const float4* __restrict__ stash,
                                                              long long* __restrict__ gloc, int Fw, int H, float l2,
                                                              int hist_len, const float* __restrict__ opt,
                                                              uint8_t* __restrict__ dmark, float* __restrict__ sq_out,
                                                              const float* __restrict__ rep_sq, double* __restrict__ acc) {
  const WideHyper h = wide_hyper(opt, l2, hist_len);
  const bool skip = step_poisoned(opt);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const long long nu = (long long)min((long long)max(n_uniq[0], 0), max_u);
  float sq = 0.f, run = 0.f;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (long long)gridDim.x * blockDim.x) {
    const float4 s = stash[u];
    const long long row = (long long)__float_as_int(s.w);
    long long q = gloc[Fw + H + u];
    gloc[Fw + H + u] = 0;
    const bool deep = row >= Fw && row < Fw + H;
    if (deep) {
      q += gloc[row];   // the deep-output term of the same row (pass B resets it)
      dmark[row - Fw] = 1;
    }
    if (skip) continue;
    float w = s.x, m = s.y, v = s.z;
    sq += w * w;
    if (acc) run += (rep_sq ? rep_sq[u] : 0.f) + w * w;
    adam_elem(w, m, v, wide_l2_grad(wide_float(q), h.l2, w), alpha, h.omb1, h.omb2, h.eps);
    wide_rec_store(rec, row, make_float4(w, m, v, __int_as_float(t)));
  }
  if (sq_out) block_sum_store(sq, sq_out + blockIdx.x);
  if (acc) block_sum_accumulate(run, acc);
}

// Pass B: the H deep-output rows pass A did not cover (their gradient: the deep term alone).
__global__ __launch_bounds__(256) void wide_rec_update_deep_kernel(float4* __restrict__ rec, long long* __restrict__ gloc,
                                                                   int Fw, int H, float l2, const float* __restrict__ hist,
                                                                   int hist_len, const float* __restrict__ opt,
                                                                   uint8_t* __restrict__ dmark,
                                                                   float* __restrict__ sq_out, double* __restrict__ acc) {
  const WideHyper h = wide_hyper(opt, l2, hist_len);
  const bool skip = step_poisoned(opt);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  float sq = 0.f, run = 0.f;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < H; j += gridDim.x * blockDim.x) {
    const long long row = Fw + j;
    const long long q = gloc[row];
    gloc[row] = 0;
    if (dmark[j]) {   // updated in pass A with the batch's wide terms
      dmark[j] = 0;
      continue;
    }
    if (skip) continue;
    float4 r = rec[row * kWideRecF4];
    const int from = wide_from(r.w, t - 1, hist_len, opt_status(opt));
    if (from < t - 1) wide_catch_up_sq(r.x, r.y, r.z, from, t - 1, hist, h, run);
    sq += r.x * r.x;
    run += r.x * r.x;
    adam_elem(r.x, r.y, r.z, wide_l2_grad(wide_float(q), h.l2, r.x), alpha, h.omb1, h.omb2, h.eps);
    wide_rec_store(rec, row, make_float4(r.x, r.y, r.z, __int_as_float(t)));
  }
  if (sq_out) block_sum_store(sq, sq_out + blockIdx.x);
  if (acc) block_sum_accumulate(run, acc);
}

// Every row caught up to step opt[7].  Rows the last step did not touch (stamp < t) pass
// through their step t - 1 state on the way: its w^2 — the L2 loss term of step t's pre-update
// weights for those rows — is summed into sq_untouched.
__global__ __launch_bounds__(256) void wide_rec_flush_kernel(float4* __restrict__ rec, long long w_rows, float l2,
                                                             const float* __restrict__ hist, int hist_len,
                                                             const float* __restrict__ opt,
                                                             int64_t* __restrict__ sq_untouched, double* __restrict__ acc) {
  const WideHyper h = wide_hyper(opt, l2, hist_len);
  const int t = (int)opt[7];
  float sq = 0.f, run = 0.f;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < w_rows;
       row += (long long)gridDim.x * blockDim.x) {
    float4 r = rec[row * kWideRecF4];   // (the sweep reads every slot's line: the record alone is written back)
    const int from = wide_from(r.w, t, hist_len, opt_status(opt));
    if (from >= t) continue;
    if (from < t - 1) wide_catch_up_sq(r.x, r.y, r.z, from, t - 1, hist, h, run);
    sq += r.x * r.x;
    run += r.x * r.x;
    wide_catch_up(r.x, r.y, r.z, t - 1, t, hist, h);
    rec[row * kWideRecF4] = make_float4(r.x, r.y, r.z, __int_as_float(t));
  }
  if (sq_untouched) block_fixed_add(sq, sq_untouched);
  if (acc) block_sum_accumulate(run, acc);
}

// The batch's wide gradient per unique wide row, from the wide index instead of atomics:
// q[u] = sum over the row's references e (sorted positions off[u] .. off[u + 1]) of
// wide_fixed(dz[e / Fw]) — TF's UnsortedSegmentSum of the cross logit's gradient (wdl.py:
// 241-264).  Int64 fixed point adds associatively, so the sum is the same bits as the head's
// per-reference atomics it replaces, in any order.  Pass 1: one thread per unique row for
// segments up to kWideSegShort references, longer ones (hot ids) appended to a list; pass 2:
// one block per listed row, the block's threads striding the segment.
constexpr int kWideSegShort = 64;

__global__ __launch_bounds__(256) void wide_seg_sum_kernel(const float* __restrict__ dz, int Fw,
                                                           const int32_t* __restrict__ refs,
                                                           const int32_t* __restrict__ off,
                                                           const int32_t* __restrict__ n_uniq, long long max_u,
                                                           long long nrefs, long long* __restrict__ q,
                                                           int32_t* __restrict__ lng, const float* __restrict__ opt) {
  int* status = opt_status(opt);
  const long long nu = min((long long)max(n_uniq[0], 0), max_u);
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (long long)gridDim.x * blockDim.x) {
    const int e0 = off[u], e1 = off[u + 1];
    if (e0 < 0 || e1 > nrefs || e0 > e1) {
      raise_fault(status, DL_STATUS_INDEX);
      q[u] = 0;
      continue;
    }
    if (e1 - e0 > kWideSegShort) {
      lng[1 + atomicAdd(lng, 1)] = (int32_t)u;
      continue;
    }
    long long acc = 0;
    for (int e = e0; e < e1; ++e) acc += wide_fixed(dz[refs[e] / Fw]);
    q[u] = acc;
  }
}

__global__ void wide_seg_reset_kernel(int32_t* __restrict__ lng) {
  if (threadIdx.x == 0) lng[0] = 0;
}

__global__ __launch_bounds__(256) void wide_seg_long_kernel(const float* __restrict__ dz, int Fw,
                                                            const int32_t* __restrict__ refs,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ lng, long long* __restrict__ q) {
  __shared__ long long part[4];
  const int n = lng[0];
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int u = lng[1 + i];
    const int e0 = off[u], e1 = off[u + 1];
    long long acc = 0;
    for (int e = e0 + threadIdx.x; e < e1; e += blockDim.x) acc += wide_fixed(dz[refs[e] / Fw]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) q[u] = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
  }
}

static unsigned wide_grid(long long n) {   // grid-stride kernels, one regulariser atomic per block
  long long b = (n + 255) / 256;
  if (b > kSumGrid) b = kSumGrid;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace dl

using namespace dl;

extern "C" int dl_wide_rec_gather(const float* rec, int64_t w_rows, const uint32_t* uniq_rows, const int32_t* n_uniq,
                                  int64_t max_uniq, int32_t Fw, int32_t H, const float* hist, int32_t hist_len,
                                  const float* opt, float l2, int32_t lag, float* wloc, float* stash, float* rep_sq,
                                  void* stream) {
  DL_CHECK_ARG(rec && hist && opt && wloc && (max_uniq == 0 || uniq_rows), "NULL argument");
  DL_CHECK_ARG(hist_len >= 2 && (hist_len & (hist_len - 1)) == 0, "hist_len must be a power of two");
  DL_CHECK_ARG(Fw >= 0 && H >= 0 && (long long)Fw + H <= w_rows, "bad Fw / H");
  DL_CHECK_ARG(((uintptr_t)rec % 16) == 0 && ((uintptr_t)stash % 16) == 0, "rec / stash must be 16-B aligned");
  const long long n = H + (max_uniq > 0 ? max_uniq : 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(wide_rec_gather_kernel, dim3(wide_rows_grid(n)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(rec), (long long)w_rows, uniq_rows, n_uniq, (long long)max_uniq,
                     Fw, H, hist, hist_len, opt, l2, lag, wloc, reinterpret_cast<float4*>(stash), rep_sq);
  DL_RETURN_LAUNCH("dl_wide_rec_gather");
}

extern "C" int64_t dl_wide_update_blocks(int64_t max_uniq, int32_t H) {
  return (max_uniq > 0 ? wide_rows_grid(max_uniq) : 0) + (H > 0 ? wide_rows_grid(H) : 0);
}

extern "C" int dl_wide_seg_grad(const float* dz, int32_t Fw, const int32_t* refs, const int32_t* seg_off,
                                const int32_t* n_uniq, int64_t max_uniq, int64_t nrefs, int64_t* q, int32_t* long_ws,
                                const float* opt, void* stream) {
  DL_CHECK_ARG(dz && refs && seg_off && n_uniq && q && long_ws && opt, "NULL argument");
  DL_CHECK_ARG(Fw > 0, "Fw must be positive");
  if (max_uniq <= 0) return 0;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(wide_seg_reset_kernel, dim3(1), dim3(64), 0, s, long_ws);   // (no memset node in the graph)
  // one thread per unique row (no regulariser atomic here, so no grid cap: the chain
  // offsets -> references -> dz is latency-bound and wants every row in flight at once)
  hipLaunchKernelGGL(wide_seg_sum_kernel, dim3(wide_rows_grid(max_uniq)), dim3(256), 0, s, dz, Fw, refs, seg_off, n_uniq,
                     (long long)max_uniq, (long long)nrefs, reinterpret_cast<long long*>(q), long_ws, opt);
  hipLaunchKernelGGL(wide_seg_long_kernel, dim3(256), dim3(256), 0, s, dz, Fw, refs, seg_off, long_ws,
                     reinterpret_cast<long long*>(q));
  DL_RETURN_LAUNCH("dl_wide_seg_grad");
}

extern "C" int dl_wide_rec_update(float* rec, const int32_t* n_uniq, int64_t max_uniq, const float* stash, int64_t* gloc,
                                  int32_t Fw, int32_t H, float l2, const float* hist, int32_t hist_len,
                                  const float* opt, uint8_t* dmark, float* sq_out, const float* rep_sq, double* acc,
                                  void* stream) {
  DL_CHECK_ARG(rec && n_uniq && stash && gloc && hist && opt && dmark, "NULL argument");
  DL_CHECK_ARG(hist_len >= 2 && (hist_len & (hist_len - 1)) == 0, "hist_len must be a power of two");
  DL_CHECK_ARG(Fw >= 0 && H >= 0, "bad Fw / H");
  hipStream_t s = as_stream(stream);
  if (max_uniq > 0)
    hipLaunchKernelGGL(wide_rec_update_kernel, dim3(wide_rows_grid(max_uniq)), dim3(256), 0, s,
                       reinterpret_cast<float4*>(rec), n_uniq, (long long)max_uniq,
                       reinterpret_cast<const float4*>(stash), reinterpret_cast<long long*>(gloc), Fw, H, l2, hist_len,
                       opt, dmark, sq_out, rep_sq, acc);   // partials [0, wide_rows_grid(max_uniq))
  if (H > 0)
    hipLaunchKernelGGL(wide_rec_update_deep_kernel, dim3(wide_rows_grid(H)), dim3(256), 0, s, reinterpret_cast<float4*>(rec),
                       reinterpret_cast<long long*>(gloc), Fw, H, l2, hist, hist_len, opt, dmark,
                       sq_out ? sq_out + (max_uniq > 0 ? wide_rows_grid(max_uniq) : 0) : nullptr, acc);
  DL_RETURN_LAUNCH("dl_wide_rec_update");
}

extern "C" int dl_wide_rec_flush(float* rec, int64_t w_rows, float l2, const float* hist, int32_t hist_len,
                                 const float* opt, int64_t* sq_untouched, double* acc, void* stream) {
  DL_CHECK_ARG(rec && hist && opt, "NULL argument");
  DL_CHECK_ARG(hist_len >= 2 && (hist_len & (hist_len - 1)) == 0, "hist_len must be a power of two");
  if (w_rows <= 0) return 0;
  hipLaunchKernelGGL(wide_rec_flush_kernel, dim3(wide_grid(w_rows)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<float4*>(rec), (long long)w_rows, l2, hist, hist_len, opt, sq_untouched, acc);
  DL_RETURN_LAUNCH("dl_wide_rec_flush");
}
