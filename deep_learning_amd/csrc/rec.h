// Row-record helpers shared by rec.hip (gather / update / flush) and embed.hip (the
// forward that reads records directly): the device-side Adam hyper-parameters and the
// lazy-exact catch-up (replayed zero-gradient TF1 Adam steps, see rec.hip).
#pragma once
#include "common.h"

namespace dl {

struct RecCfg {
  int E, ld, has_first, hist_mask;
  int sparse;                          // TF's sparse-apply Adam form (DL_REC_SPARSE_ADAM)
  float b1, b2, omb1, omb2, eps;       // filled on the device from opt (rec_load_hyper)
  RootDecay rd;                        // sqrt(b2) for the root state's zero steps (common.h)
  int* status;                         // opt's status word (lag overflow is reported there)
};

// rec_flags of the C ABI (DL_REC_FIRST | DL_REC_SPARSE_ADAM) -> the kernel config
inline RecCfg make_rec_cfg(int E, int ld, int rec_flags, int hist_len) {
  RecCfg c{};
  c.E = E;
  c.ld = ld;
  c.has_first = (rec_flags & DL_REC_FIRST) ? 1 : 0;
  c.sparse = (rec_flags & DL_REC_SPARSE_ADAM) ? 1 : 0;
  c.hist_mask = hist_len - 1;
  return c;
}

__device__ __forceinline__ void rec_load_hyper(RecCfg& c, const float* opt) {
  c.b1 = opt[4];
  c.b2 = opt[5];
  c.omb1 = 1.f - opt[4];
  c.omb2 = 1.f - opt[5];
  c.eps = opt[6];
  c.rd = root_decay(opt[5]);
  c.status = opt_status(opt);
}

// The table's TF1 Adam element update in the form the reference applies to it, on the root
// state (s = sqrt(v): common.h adam_elem_root).  `v` below is that s throughout.
__device__ __forceinline__ void rec_adam(float& p, float& m, float& v, float g, float alpha, const RecCfg& c) {
#if DL_ROOT_STATE
  if (c.sparse) adam_elem_sparse_root(p, m, v, g, alpha, c.b1, c.b2, c.omb1, c.omb2, c.rd, c.eps);
  else adam_elem_root(p, m, v, g, alpha, c.omb1, c.omb2, c.rd, c.eps);
#else
  if (c.sparse) adam_elem_sparse(p, m, v, g, alpha, c.b1, c.b2, c.omb1, c.omb2, c.eps);
  else adam_elem(p, m, v, g, alpha, c.omb1, c.omb2, c.eps);
#endif
}

// A row lagging more steps than the alpha ring holds cannot be caught up exactly: the host
// flushes on schedule so this never happens; if it does, the status word says so (the host
// raises) and the replay covers the ring's steps only.
__device__ __forceinline__ int catch_up_from(int from, int to, const RecCfg& c) {
  if (to - from > c.hist_mask + 1) {
    raise_fault(c.status, DL_STATUS_LAG);
    return to - (c.hist_mask + 1);
  }
  return from;
}

// The per-step alphas of the zero-gradient steps a catch-up replays.  RingG reads the ring
// where it lies (global memory, or an LDS copy of the whole ring); RingW keeps the newest
// kHistWin steps before t0 in LDS (filled once per block by load_hist_window) and reads only
// older steps from the global ring: one replayed step used to wait a full global-load round
// trip for its alpha, which bound the catch-up loop by memory latency at realistic row lags.
constexpr int kHistWin = 256;

struct RingG {
  const float* h;
  int mask;
  __device__ __forceinline__ float operator()(int j) const { return h[j & mask]; }
};

struct RingW {
  const float* sh;   // sh[d] = alpha of step t0 - d, d < kHistWin
  const float* h;
  int mask, t0;
  __device__ __forceinline__ float operator()(int j) const {
    const int d = t0 - j;
    return d < kHistWin ? sh[d] : h[j & mask];
  }
};

// Whole block: the window of the kHistWin steps up to t0 (entries past the ring's length are
// never read: a row's lag never exceeds the ring).  Call before any divergent return.
__device__ __forceinline__ RingW load_hist_window(float* sh, const float* __restrict__ hist, int t0, const RecCfg& c) {
  for (int d = threadIdx.x; d < kHistWin; d += blockDim.x) sh[d] = hist ? hist[(t0 - d) & c.hist_mask] : 0.f;
  __syncthreads();
  return RingW{sh, hist, c.hist_mask, t0};
}

// Replays zero-gradient steps (from, to] on one float4 of p/m/v (and the
// first-order triple when `first` is set).
template <class Ring>
__device__ __forceinline__ void catch_up4_loop(float4& p, float4& m, float4& v, float& w, float& wm, float& wv,
                                               bool first, int from, int to, const Ring& ring, const RecCfg& c) {
  for (int j = from + 1; j <= to; ++j) {
    const float al = ring(j);
    rec_adam(p.x, m.x, v.x, 0.f, al, c);
    rec_adam(p.y, m.y, v.y, 0.f, al, c);
    rec_adam(p.z, m.z, v.z, 0.f, al, c);
    rec_adam(p.w, m.w, v.w, 0.f, al, c);
    if (first) rec_adam(w, wm, wv, 0.f, al, c);
  }
}

template <class Ring>
__device__ __forceinline__ void catch_up1_loop(float& p, float& m, float& v, float& w, float& wm, float& wv,
                                               bool first, int from, int to, const Ring& ring, const RecCfg& c) {
  for (int j = from + 1; j <= to; ++j) {
    const float al = ring(j);
    rec_adam(p, m, v, 0.f, al, c);
    if (first) rec_adam(w, wm, wv, 0.f, al, c);
  }
}

// One zero-gradient step of the catch-up replay: rec_adam(..., g = 0, ...) written out (the
// g == 0 branch of adam_elem_root / adam_elem_sparse_root), with its constants hoisted.
struct Zero0 {   // per-launch constants of the zero-gradient step
  float b1, nomb1, eps;
  RootDecay rd;
  float b2, nomb2, z1, z2;   // the v form (DL_ROOT_STATE=0)
  __device__ __forceinline__ explicit Zero0(const RecCfg& c) {
#pragma clang fp contract(off)
    b1 = c.b1; nomb1 = -c.omb1; eps = c.eps; rd = c.rd;
    b2 = c.b2; nomb2 = -c.omb2;
    const float g = 0.f;
    z1 = g * c.omb1;
    z2 = (g * g) * c.omb2;
  }
};

template <bool SPARSE>
__device__ __forceinline__ void rec_adam0_x1(float& p, float& m, float& s, float alpha, const Zero0& k) {
#pragma clang fp contract(off)
#if DL_ROOT_STATE
  if (SPARSE) m = m * k.b1;
  else m = m + m * k.nomb1;
  s = root_decay_step(s, k.rd);
  p = p - root_step_size(m, s, alpha, k.eps);
#else   // s is TF's v here: the round-3 zero step
  if (SPARSE) {
    m = m * k.b1 + k.z1;
    s = s * k.b2 + k.z2;
  } else {
    m = m + m * k.nomb1;
    s = s + s * k.nomb2;
  }
  p = p - adam_step_size(m, s, alpha, k.eps);
#endif
}

// Two elements of one row stepped together: the same float operations per half as
// rec_adam0_x1 (the packed multiplies, fmas and adds round each half exactly as the scalar
// ones do), so the halves stay bit-identical to the dense sweep; the packed form issues the
// decays, the alpha product and the update once for both elements.
typedef float rec_f2v __attribute__((ext_vector_type(2)));
template <bool SPARSE>
__device__ __forceinline__ void rec_adam0_x2(rec_f2v& p, rec_f2v& m, rec_f2v& s, float alpha, const Zero0& k) {
#pragma clang fp contract(off)
#if DL_ADAM_IEEE || !DL_ROOT_STATE
  rec_adam0_x1<SPARSE>(p.x, m.x, s.x, alpha, k);
  rec_adam0_x1<SPARSE>(p.y, m.y, s.y, alpha, k);
#else
  if (SPARSE) m = m * k.b1;
  else m = m + m * k.nomb1;
  s = __builtin_elementwise_fma(s, rec_f2v{k.rd.hi, k.rd.hi}, s * k.rd.lo);
  const rec_f2v d = s + k.eps;
  rec_f2v r;
  r.x = __builtin_amdgcn_rcpf(d.x);
  r.y = __builtin_amdgcn_rcpf(d.y);
  p = p - (m * alpha) * r;
#endif
}

// LDS-only reads of the alpha window
struct RingWin {
  const float* sh;
  int t0;
  __device__ __forceinline__ float operator()(int j) const { return sh[t0 - j]; }
};

template <class Ring>
__device__ __forceinline__ void catch_up4(float4& p, float4& m, float4& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const Ring& ring, const RecCfg& c) {
  from = catch_up_from(from, to, c);
  catch_up4_loop(p, m, v, w, wm, wv, first, from, to, ring, c);
}

// the window form: steps inside the LDS window are read from LDS only (a row lagging
// further first replays its older steps from the global ring)
__device__ __forceinline__ void catch_up4(float4& p, float4& m, float4& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const RingW& ring, const RecCfg& c) {
  from = catch_up_from(from, to, c);
  const int lo = ring.t0 - kHistWin;   // steps > lo are in the window
  if (from < lo) {
    catch_up4_loop(p, m, v, w, wm, wv, first, from, lo, RingG{ring.h, ring.mask}, c);
    from = lo;
  }
  catch_up4_loop(p, m, v, w, wm, wv, first, from, to, RingWin{ring.sh, ring.t0}, c);
}

template <class Ring>
__device__ __forceinline__ void catch_up1(float& p, float& m, float& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const Ring& ring, const RecCfg& c) {
  from = catch_up_from(from, to, c);
  catch_up1_loop(p, m, v, w, wm, wv, first, from, to, ring, c);
}

__device__ __forceinline__ void catch_up1(float& p, float& m, float& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const RingW& ring, const RecCfg& c) {
  from = catch_up_from(from, to, c);
  const int lo = ring.t0 - kHistWin;
  if (from < lo) {
    catch_up1_loop(p, m, v, w, wm, wv, first, from, lo, RingG{ring.h, ring.mask}, c);
    from = lo;
  }
  catch_up1_loop(p, m, v, w, wm, wv, first, from, to, RingWin{ring.sh, ring.t0}, c);
}

}  // namespace dl
