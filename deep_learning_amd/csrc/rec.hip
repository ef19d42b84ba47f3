// Lazy-exact TF1 Adam on interleaved embedding row records.
//
// The reference applies the DENSE Adam update to the embedding table every step
// (deepfm_pipeline.py:184-188; the gradient reaches the Variable densified, SURVEY.md
// ledger item 6): every row's m and v decay and every row with m != 0 moves, even
// when the batch never referenced it.  Sweeping p, m, v of a 26M x 16 table is
// ~10.4 GB of HBM traffic per step — the single largest cost of the step.
//
// Here a row that the batch does not reference is left alone and its pending
// zero-gradient steps are replayed ("caught up") the next time it is read:
//   for j = stamp+1 .. target:   adam_elem(p, m, v, g = 0, alpha_j)
// with alpha_j from a ring of per-step alphas written by dl_adam_hist_record.
// adam_elem is the same inline function the dense sweep uses (common.h), so the
// replayed steps are the same float operations in the same order: the result is
// bit-identical to the dense update, only the time at which it is computed moves.
// The host bounds every row's lag below the ring length by calling dl_rec_flush
// (catch every row up) at least once per hist_len steps, and before any export.
//
// Row record (rec_ld floats, rec_ld % 32 == 0 so a record starts a 128-B line):
//   [0, E)        p                   (the embedding row)
//   E .. E+2      w1, m(w1), s(w1)    (FM first-order weight of the row, if any)
//   E+3           stamp               (int32 bits: last step applied to the row)
//   [E+4, 2E+4)   m
//   [2E+4, 3E+4)  s = sqrt(v)         (the root state, common.h adam_elem_root: a replayed
//                                      zero-gradient step costs one reciprocal)
// p and w1 share the first 128-B line: the forward's useful bytes sit together,
// and one record is two lines for E = 16.
#include "common.h"
#include <climits>
#include "rec.h"
#include "segment.h"

#ifndef DL_REC_FULL_LINES
#define DL_REC_FULL_LINES 1   // record updates also write the pad (see rec_write_pad)
#endif

// The gather's moment stash (mv: what the backward updates from, so it never re-reads and
// replays a record).  DL_STASH_M = 0: [m (E) | s (E) | m1 s1 0 0] per unique row, 2E + 4 floats.
// DL_STASH_M = 1 (root state only): [m (E) | m1 s1 lag 0], E + 4 floats — the backward reads the
// row's stale s from the record line it rewrites anyway and applies the `lag` zero-gradient
// decays itself: with g = 0 a step's s' = fma(s, c_hi, s c_lo) does not depend on p, m or the
// step's alpha (common.h adam_elem_root), so the same operations give the same bits as the
// gather's replay.  64 B a row less written by the gather and read back by the backward, for
// one random 64-B read of the record's second line.
#ifndef DL_STASH_M
#define DL_STASH_M 0
#endif
#if DL_STASH_M && !DL_ROOT_STATE
#error "DL_STASH_M needs the root state (DL_ROOT_STATE=1)"
#endif
__host__ __device__ constexpr int rec_stash_floats(int E) { return DL_STASH_M ? E + 4 : 2 * E + 4; }

// The record / stash streams' float4 accesses (round 4 tried them non-temporal, so the random
// per-reference reads might stay cached: gather 328 -> 410 us, backward 439 -> 723 us at C2,
// profiles/r04f_nt/ — removed).
__device__ __forceinline__ float4 rec_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void rec_st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

namespace dl {

// ---------------------------------------------------------------------------
// Forward gather of the batch's rows, caught up to step opt[7] - lag:
//   out[i] = p(row_i), out1[i] = w1(row_i),   row_i = rep_base + i (i < n_rep), else uniq[i - n_rep]
// (rep_base = the layout's fm_cont_offset: the replicated FM cont-field rows)
// Records are only read: the backward's update writes (it takes the caught-up moments
// from `mv` when given, or replays the catch-up itself).  E/4 lanes per row, float4 each.
//
// Lag-balanced catch-up.  A wave holds RPW = 256/E rows, and row lags differ (geometric at
// steady state: C2 mean ~8, max of 16 rows ~25): with each row replayed by its own lanes the
// wave runs as long as its worst row while every lane carries E/4 + 1 element chains.
// Instead the wave stages its rows' p, m, v (and first-order triple) in LDS and splits the
// replay into single-element chains (E or E + 1 per row, each as long as its row's lag),
// dealt to the 64 lanes in descending-lag order, snake-wise (round i: chains 64i..64i+63,
// reversed on odd rounds): lanes that took a long chain take short ones after it.  Each
// chain is the same sequence of rec_adam calls as before, so the results are unchanged.
// 1: rank-dealt single elements, wave-uniform step loop; 2: the same with element pairs
// (packed math; measured no faster: profiles/r04f_rp/); 0: per-lane chains (round-2 v1)
#ifndef DL_GATHER_REPLAY
#define DL_GATHER_REPLAY 1
#endif

// The replay loop of rec_gather_kernel's staged rows: one wave-uniform loop over the steps
// k = top .. 1 (step target - k + 1), a lane stepping its unit (one element's p / m / v, or
// the first-order triple) while the unit's lag `mine` covers k.  The alphas of
// the last 64 steps sit one per lane in `alv` (lane l: step target - l, loaded once per
// kernel) and are read with v_readlane: no LDS round trip inside the loop; older steps (a lag
// beyond 64, rare) read the ring.
template <bool SPARSE>
__device__ __forceinline__ void replay_steps(float& p, float& m, float& v, int mine, int top, int target,
                                             const RingW& ring, const Zero0& z, float alv) {
  int k = top;
  for (; k > 64; --k) {
    const float al = ring(target - k + 1);
    if (mine >= k) rec_adam0_x1<SPARSE>(p, m, v, al, z);
  }
  for (; k >= 1; --k) {
    const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(alv), k - 1));
    if (mine >= k) rec_adam0_x1<SPARSE>(p, m, v, al, z);
  }
}

// The staged rows' replay: E element units + the first-order triple per row, dealt in rank
// order (most-lagging rows first) 64 to a round, so a round's uniform loop runs as long as its
// first row's lag and the later, less-lagging rounds stop early.
template <int E, bool SPARSE>
__device__ __forceinline__ void replay_elems(float* st, const int* from_s, const int* order, int pitch, int target,
                                             int nch, const RingW& ring, const RecCfg& c, float alv) {
  constexpr int LPR = E / 4, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const Zero0 z(c);
  const int T = RPW * nch;
  for (int r0 = 0; r0 < T; r0 += 64) {
    const int top = __builtin_amdgcn_readfirstlane(target - from_s[order[r0 / nch]]);
    if (top <= 0) break;                             // rank order: every later round is caught up too
    const int k = r0 + lane;
    const int r = order[min(k, T - 1) / nch], e = k % nch;
    float* sr = st + r * pitch;
    const int mine = k < T ? target - from_s[r] : 0;
    float* x = e < E ? sr + e : sr + 3 * E;
    const int s1 = e < E ? E : 1;
    float P = x[0], M = x[s1], V = x[2 * s1];
    replay_steps<SPARSE>(P, M, V, mine, top, target, ring, z, alv);
    if (k < T) { x[0] = P; x[s1] = M; x[2 * s1] = V; }
  }
}

// The paired form: a unit is two adjacent elements of a row (same lag, one rec_adam0_x2 chain)
// or the row's first-order triple (its second half idle: zeros in, nothing written back).
// E / 2 + 1 units per row instead of E + 1: half the rounds, and the packed decay / update.
template <bool SPARSE>
__device__ __forceinline__ void replay_steps2(rec_f2v& p, rec_f2v& m, rec_f2v& v, int mine, int top, int target,
                                              const RingW& ring, const Zero0& z, float alv) {
  int k = top;
  for (; k > 64; --k) {
    const float al = ring(target - k + 1);
    if (mine >= k) rec_adam0_x2<SPARSE>(p, m, v, al, z);
  }
  for (; k >= 1; --k) {
    const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(alv), k - 1));
    if (mine >= k) rec_adam0_x2<SPARSE>(p, m, v, al, z);
  }
}

template <int E, bool SPARSE>
__device__ __forceinline__ void replay_pairs(float* st, const int* from_s, const int* order, int pitch, int target,
                                             int has_first, const RingW& ring, const RecCfg& c, float alv) {
  constexpr int LPR = E / 4, RPW = 64 / LPR, NP = E / 2;
  const int lane = threadIdx.x & 63;
  const Zero0 z(c);
  const int nu = NP + has_first;
  const int T = RPW * nu;
  for (int r0 = 0; r0 < T; r0 += 64) {
    const int top = __builtin_amdgcn_readfirstlane(target - from_s[order[r0 / nu]]);
    if (top <= 0) break;                             // rank order: every later round is caught up too
    const int k = r0 + lane;
    const int r = order[min(k, T - 1) / nu], e = k % nu;
    float* sr = st + r * pitch;
    const int mine = k < T ? target - from_s[r] : 0;
    rec_f2v P, M, V;
    if (e < NP) {
      float* x = sr + 2 * e;
      P = rec_f2v{x[0], x[1]};
      M = rec_f2v{x[E], x[E + 1]};
      V = rec_f2v{x[2 * E], x[2 * E + 1]};
    } else {
      float* x = sr + 3 * E;
      P = rec_f2v{x[0], 0.f};
      M = rec_f2v{x[1], 0.f};
      V = rec_f2v{x[2], 0.f};
    }
    replay_steps2<SPARSE>(P, M, V, mine, top, target, ring, z, alv);
    if (k < T) {
      if (e < NP) {
        float* x = sr + 2 * e;
        x[0] = P.x; x[1] = P.y; x[E] = M.x; x[E + 1] = M.y; x[2 * E] = V.x; x[2 * E + 1] = V.y;
      } else {
        float* x = sr + 3 * E;
        x[0] = P.x; x[1] = M.x; x[2] = V.x;
      }
    }
  }
}

// Forward scatter (the lazy single-GPU forward, dl_rec_gather_scatter): each caught-up row is
// also written straight to the references that read it, through the batch index's sorted
// segments, instead of only compactly for embed_fwd to re-read at random through the inverse
// map — random 64-B writes run at the HBM write rate, random 64-B reads at about half of it
// (profiles/r03b/ubench_scatter.txt: 6.0 vs 3.3 TB/s):
//   FM reference (b, f)    -> fmst[n_rep + b*S + f] (the rows embed_fwd's staged mode sums per
//                             sample) and fm_out[b][Cf + f] = w1 (the first-order output)
//   deep reference (b, f)  -> x0[b][x0_cat_col + f*E] (f32, or bf16 for the bf16 tower)
// Multi-hot references are pooled from the compact rows as before; the replicated rows go to
// fmst[0, n_rep).  Rows with more than kSegLong references are left to gather_scatter_long.
struct GatherScatter {
  const int32_t* seg_off;
  const int32_t* refs;
  float* fmst;
  float* x0;
  float* fm_out;
  float* mst;      // multi-hot staging (may be NULL): position l of sample b -> mst[b*mw + l][E], mst1
  float* mst1;
  long long nrefs;
  int ns, S, mb, use_fm, Cf, x0_ld, x0_cat_col, x0_bf16, fm_ld, n_rep, mw;
  int* status;
};

template <int E>
__device__ __forceinline__ void scatter_ref(const GatherScatter& s, int k, int q, float4 p, float w, bool first) {
  if (k < 0 || k >= s.nrefs) {
    index_fault(s.status);
    return;
  }
  const int b = k / s.ns, sl = k - b * s.ns;
  if (sl >= s.mb) {   // multi-hot: into the staging rows the pooling reads per sample (or left)
    if (s.mst) {
      const long long o = (long long)b * s.mw + (sl - s.mb);
      *reinterpret_cast<float4*>(s.mst + o * E + 4 * q) = p;
      if (s.mst1 && q == 0) s.mst1[o] = w;
    }
    return;
  }
  if (s.use_fm && sl < s.S) {
    *reinterpret_cast<float4*>(s.fmst + ((long long)s.n_rep + (long long)b * s.S + sl) * E + 4 * q) = p;
    if (first && q == 0) s.fm_out[(long long)b * s.fm_ld + s.Cf + sl] = w * 1.f;
  } else {
    const int f = s.use_fm ? sl - s.S : sl;
    const long long o = (long long)b * s.x0_ld + s.x0_cat_col + f * E + 4 * q;
    if (s.x0_bf16)
      *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(s.x0) + o) =
          make_uint2(f2bf(p.x) | ((unsigned)f2bf(p.y) << 16), f2bf(p.z) | ((unsigned)f2bf(p.w) << 16));
    else
      *reinterpret_cast<float4*>(s.x0 + o) = p;
  }
}

template <int E, bool SPARSE, bool SCAT = false>
__global__ __launch_bounds__(256) void rec_gather_kernel(const float* __restrict__ rec, RecCfg c, int64_t n_rows,
                                                         int n_rep, int64_t rep_base,
                                                         const uint32_t* __restrict__ uniq,
                                                         const int32_t* __restrict__ n_uniq, long long max_u,
                                                         int world, const float* __restrict__ hist,
                                                         const float* __restrict__ opt, int lag,
                                                         float* __restrict__ out, float* __restrict__ out1,
                                                         float* __restrict__ mv, GatherScatter sc = {}) {
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4, RPW = 64 / LPR, PITCH = 3 * E + 3;
  __shared__ float st_all[4][RPW * PITCH];           // per wave: p | m | v | w wm wv of each row
  __shared__ int from_all[4][RPW], order_all[4][RPW];
  const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
  float* st = st_all[wv_];
  int* from_s = from_all[wv_];
  int* order = order_all[wv_];
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = lane % LPR, rw = lane / LPR;
  const long long wave_id = gt >> 6, nwaves = ((long long)gridDim.x * blockDim.x) >> 6;
  const long long total = n_rep + (n_uniq ? (long long)clamp_uniq(n_uniq, max_u, c.status) : max_u);
  const int target = (int)opt[7] - lag;
  const float alv = ring(target - lane);               // lane l: alpha of step target - l
  const int nch = E + (c.has_first ? 1 : 0);          // element chains per row
  const int T = RPW * nch;
  for (long long base = wave_id * RPW; base < total; base += nwaves * RPW) {
    const long long i = base + rw;
    const bool valid = i < total;
    const int64_t row = !valid ? -1 : i < n_rep ? rep_base + i : decode_key(uniq[i - n_rep], world);
    // the row's reference segment (scatter form), loaded beside the record
    int so0 = 0, so1 = 0, k0 = -1;
    if (SCAT && valid && i >= n_rep) {
      so0 = sc.seg_off[i - n_rep];
      so1 = sc.seg_off[i - n_rep + 1];
      if (so0 < 0 || so1 > sc.nrefs || so0 > so1) {
        index_fault(sc.status);
        so0 = so1 = 0;
      }
      k0 = so0 < so1 ? sc.refs[so0] : -1;
    }
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 p = z, m = z, v = z;
    float w = 0.f, wm = 0.f, wv = 0.f;
    int from = target;
    if (row >= 0 && row < n_rows) {
      const float* r = rec + row * c.ld;
      p = rec_ld4(r + 4 * q);
      m = rec_ld4(r + E + 4 + 4 * q);
      v = rec_ld4(r + 2 * E + 4 + 4 * q);
      const float4 tail = rec_ld4(r + E);
      w = tail.x; wm = tail.y; wv = tail.z;
      const int stamp = __float_as_int(tail.w);
      if (stamp < target) from = catch_up_from(stamp, target, c);
    }
    if (__any(from < target)) {
      // stage the rows
      float* sr = st + rw * PITCH;
      sr[4 * q + 0] = p.x; sr[4 * q + 1] = p.y; sr[4 * q + 2] = p.z; sr[4 * q + 3] = p.w;
      sr[E + 4 * q + 0] = m.x; sr[E + 4 * q + 1] = m.y; sr[E + 4 * q + 2] = m.z; sr[E + 4 * q + 3] = m.w;
      sr[2 * E + 4 * q + 0] = v.x; sr[2 * E + 4 * q + 1] = v.y; sr[2 * E + 4 * q + 2] = v.z;
      sr[2 * E + 4 * q + 3] = v.w;
      const int mylag = target - from;
      int rank = 0;   // rows with a longer lag (ties: lower row first)
#pragma unroll
      for (int o = 0; o < RPW; ++o) {
        const int lo = __shfl(mylag, o * LPR, 64);
        rank += (lo > mylag || (lo == mylag && o < rw)) ? 1 : 0;
      }
      if (q == 0) {
        sr[3 * E] = w; sr[3 * E + 1] = wm; sr[3 * E + 2] = wv;
        from_s[rw] = from;
        order[rank] = rw;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
#if DL_GATHER_REPLAY == 2
      replay_pairs<E, SPARSE>(st, from_s, order, PITCH, target, c.has_first, ring, c, alv);
#elif DL_GATHER_REPLAY
      replay_elems<E, SPARSE>(st, from_s, order, PITCH, target, nch, ring, c, alv);
#else
      for (int k0 = 0; k0 < T; k0 += 64) {
        const int k = k0 + (((k0 >> 6) & 1) ? 63 - lane : lane);
        if (k < T) {
          const int r = order[k / nch], e = k % nch;
          float* sr2 = st + r * PITCH;
          const int f = from_s[r];
          if (e < E) {
            float pe = sr2[e], me = sr2[E + e], ve = sr2[2 * E + e];
            float d0 = 0.f, d1 = 0.f, d2 = 0.f;
            catch_up1(pe, me, ve, d0, d1, d2, false, f, target, ring, c);
            sr2[e] = pe; sr2[E + e] = me; sr2[2 * E + e] = ve;
          } else {
            float pe = sr2[3 * E], me = sr2[3 * E + 1], ve = sr2[3 * E + 2];
            float d0 = 0.f, d1 = 0.f, d2 = 0.f;
            catch_up1(pe, me, ve, d0, d1, d2, false, f, target, ring, c);
            sr2[3 * E] = pe; sr2[3 * E + 1] = me; sr2[3 * E + 2] = ve;
          }
        }
      }
#endif
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      p = make_float4(sr[4 * q], sr[4 * q + 1], sr[4 * q + 2], sr[4 * q + 3]);
      m = make_float4(sr[E + 4 * q], sr[E + 4 * q + 1], sr[E + 4 * q + 2], sr[E + 4 * q + 3]);
      v = make_float4(sr[2 * E + 4 * q], sr[2 * E + 4 * q + 1], sr[2 * E + 4 * q + 2], sr[2 * E + 4 * q + 3]);
      w = sr[3 * E]; wm = sr[3 * E + 1]; wv = sr[3 * E + 2];
      __builtin_amdgcn_s_waitcnt(0xc07f);            // reads done before the next rows are staged
      __builtin_amdgcn_wave_barrier();
    }
    if (!valid) continue;
    if (SCAT) {
      if (i < n_rep) {
        *reinterpret_cast<float4*>(sc.fmst + i * E + 4 * q) = p;
      } else if (so1 - so0 <= kSegLong) {   // longer segments: gather_scatter_long_kernel
        if (so0 < so1) scatter_ref<E>(sc, k0, q, p, w, c.has_first);
        for (int e = so0 + 1; e < so1; ++e) scatter_ref<E>(sc, sc.refs[e], q, p, w, c.has_first);
      }
    }
    *reinterpret_cast<float4*>(out + i * E + 4 * q) = p;
    if (out1 && q == 0) out1[i] = w;
    if (mv) {   // caught-up moments for the backward's update (rec_stash_floats)
      float* o = mv + i * rec_stash_floats(E);
      rec_st4(o + 4 * q, m);
      if (DL_STASH_M) {
        if (q == 0) rec_st4(o + E, make_float4(wm, wv, __int_as_float(target - from), 0.f));
      } else {
        rec_st4(o + E + 4 * q, v);
        if (q == 0) rec_st4(o + 2 * E, make_float4(wm, wv, 0.f, 0.f));
      }
    }
  }
}

// The scatter form's second pass: the rows with more than kSegLong references (hot ids), one
// whole block each, from the compact rows the gather wrote (the write order is immaterial:
// every reference has its own destination).
template <int E>
__global__ __launch_bounds__(256) void gather_scatter_long_kernel(GatherScatter s, const int32_t* __restrict__ n_uniq,
                                                                  long long max_u, const float* __restrict__ rows,
                                                                  const float* __restrict__ rows1, int has_first) {
  __shared__ int n_long;
  __shared__ int long_u[256];
  constexpr int LPR = E / 4, NS = 256 / LPR;
  const int tid = threadIdx.x, q = tid % LPR;
  const long long nu = clamp_uniq(n_uniq, max_u, s.status);
  const long long per = (nu + gridDim.x - 1) / gridDim.x;
  const long long u0 = (long long)blockIdx.x * per, u1 = min(nu, u0 + per);
  for (long long base = u0; base < u1; base += 256) {
    const long long u = base + tid;
    int o0 = 0, o1 = 0;
    if (u < u1) {
      o0 = max(0, s.seg_off[u]);
      o1 = (int)min(s.nrefs, (long long)s.seg_off[u + 1]);
    }
    const bool lng = o1 - o0 > kSegLong;
    if (tid == 0) n_long = 0;
    if (!__syncthreads_or(lng)) continue;
    if (lng) long_u[atomicAdd(&n_long, 1)] = (int)(u - base);
    __syncthreads();
    const int n = n_long;
    for (int t = 0; t < n; ++t) {
      const long long uu = base + long_u[t];
      const int e0 = max(0, s.seg_off[uu]), e1 = (int)min(s.nrefs, (long long)s.seg_off[uu + 1]);
      const long long iu = s.n_rep + uu;
      const float4 p = *reinterpret_cast<const float4*>(rows + iu * E + 4 * q);
      const float w = has_first ? rows1[iu] : 0.f;
      for (int e = e0 + tid / LPR; e < e1; e += NS) scatter_ref<E>(s, s.refs[e], q, p, w, has_first);
    }
    __syncthreads();
  }
}

// One row's step-t update: catch up to t-1, then apply gradient (g, g1) with alpha_t.
// Lane d of an E-lane group owns dim d; lane 0 also owns the first-order triple and
// the stamp (every lane reads the stamp before lane 0 rewrites it: same wave).
__device__ __forceinline__ void rec_update(float* __restrict__ r, int E, int d, float g, float g1, int t,
                                           float alpha_t, const RingW& ring, const RecCfg& c) {
  const int stamp = __float_as_int(r[E + 3]);
  float p = r[d], m = r[E + 4 + d], v = r[2 * E + 4 + d];
  const bool first = c.has_first && d == 0;
  float w = 0.f, wm = 0.f, wv = 0.f;
  if (first) { w = r[E]; wm = r[E + 1]; wv = r[E + 2]; }
  if (stamp < t - 1) catch_up1(p, m, v, w, wm, wv, first, stamp, t - 1, ring, c);
  rec_adam(p, m, v, g, alpha_t, c);
  r[d] = p; r[E + 4 + d] = m; r[2 * E + 4 + d] = v;
  if (first) {
    rec_adam(w, wm, wv, g1, alpha_t, c);
    r[E] = w; r[E + 1] = wm; r[E + 2] = wv;
  }
  if (d == 0) r[E + 3] = __int_as_float(t);
}

// Backward + Adam fused: per unique row of the batch, the ordered segment sum of its
// references (segment.h) is applied at once — no gradient table, no atomics, no
// touched flags.  The row's caught-up state comes from the gather's compact outputs
// (p: rows_u, w1: rows_u1, m/v: mv), read in u order, so the record is only WRITTEN
// here (one random 208-B store per row instead of a read-modify-write).
// Replicated rows (fm_cont_offset <= row < fm_cont_offset + n_rep, hit by every sample
// through the FM cont fields)
// only deposit their cate-reference gradient into g_rep/g1_rep; dl_rec_apply_rows
// updates them after the cont part is added.  E/4 lanes per row, float4 each.
// Per (sample, pooled slot): the gradient every member row of the slot receives,
// (dx0[pool m] + dsec*(fm_sum - pooled_m)) / cnt  (div_no_nan; deepfm_multi_cate.py:71-111),
// and dz * w_head[fm_col + m] / cnt_first for the first-order weights.
template <int E>
__global__ __launch_bounds__(256) void pool_grad_kernel(dl_emb_layout L, dl_pool_desc p, const float* __restrict__ dz,
                                                        const float* __restrict__ w_head,
                                                        const float* __restrict__ fm_sum,
                                                        const float* __restrict__ dx0, bool g1) {
  constexpr int LPR = E / 4;
  const int S = L.cate_fields;
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + S + L.fm_extra;
  const long long n = (long long)L.batch * p.n_slots * LPR;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % LPR);
    const long long bm = i / LPR;
    const int b = (int)(bm / p.n_slots), m = (int)(bm % p.n_slots);
    const float c = p.cnt_emb[bm];
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
    const float dzb = L.use_fm ? dz[b] : 0.f;
    if (c > 0.f) {
      float4 dp = *reinterpret_cast<const float4*>(dx0 + (long long)b * L.dx0_ld + p.dx0_pool_col + m * E + 4 * q);
      if (L.use_fm) {
        const float* ws = w_head + F + 4 * q;
        const float4 fs = *reinterpret_cast<const float4*>(fm_sum + (long long)b * E + 4 * q);
        const float4 pv = *reinterpret_cast<const float4*>(p.x0 + (long long)b * L.x0_ld + L.x0_pool_col + m * E + 4 * q);
        dp.x = fmaf(dzb * ws[0], fs.x - pv.x, dp.x); dp.y = fmaf(dzb * ws[1], fs.y - pv.y, dp.y);
        dp.z = fmaf(dzb * ws[2], fs.z - pv.z, dp.z); dp.w = fmaf(dzb * ws[3], fs.w - pv.w, dp.w);
      }
      gv = make_float4(dp.x / c, dp.y / c, dp.z / c, dp.w / c);
    }
    const int gp = p.g_pitch > 0 ? p.g_pitch : E;
    *reinterpret_cast<float4*>(p.g_pool + bm * gp + 4 * q) = gv;
    if (g1 && q == 0) {
      const float c1 = p.cnt_first[bm];
      p.g1_pool[bm * (p.g_pitch > 0 ? p.g_pitch : 1)] = c1 > 0.f ? dzb * w_head[p.fm_col + m] / c1 : 0.f;
    }
  }
}

// A record update writes p, the tail, m and v — 208 of the 256 B at E = 16, so the record's
// second 128-B line would be left partly dirty and merged with its old bytes below the L2
// (a read of the line per update).  Writing the pad (zeros) too makes both lines whole:
// same-box C2, rec_bwd_adam 531 -> 452 us, step 2.49 -> 2.39 ms.
template <int E>
__device__ __forceinline__ void rec_write_pad(float* __restrict__ r, int q, int ld) {
#if DL_REC_FULL_LINES
  for (int o = 3 * E + 4 + 4 * q; o < ld; o += E) rec_st4(r + o, make_float4(0.f, 0.f, 0.f, 0.f));
#endif
}

// DL_STASH_M: the row's s caught up over `lag` zero-gradient steps — the replay's own s update
// (rec_adam0_x1 / _x2 on the root state), alone
__device__ __forceinline__ float4 stash_decay(float4 s, int lag, const RecCfg& c) {
#pragma clang fp contract(off)
  for (int j = 0; j < lag; ++j) {
    s.x = root_decay_step(s.x, c.rd);
    s.y = root_decay_step(s.y, c.rd);
    s.z = root_decay_step(s.z, c.rd);
    s.w = root_decay_step(s.w, c.rd);
  }
  return s;
}

// The backward's per-row state: the caught-up p, m, v (and first-order triple) of unique
// row u — from the gather's stash, or the record caught up again without one.
template <int E, bool STASH = false>   // STASH: the stash is known present (no catch-up code)
__device__ __forceinline__ void rec_bwd_state(int64_t row, long long iu, int q, bool first, bool row_ok,
                                              const float* __restrict__ rec, const float* __restrict__ rows_u,
                                              const float* __restrict__ rows_u1, const float* __restrict__ mv,
                                              const RecCfg& c, int t, const RingW& ring, float4& p, float4& m,
                                              float4& v, float& w, float& wm, float& wv) {
  if (STASH || mv) {
    if (DL_BWD_DIAG & 4) iu = 0;   // diagnostics: the stash and compact rows from one cached row
    p = rec_ld4(rows_u + iu * E + 4 * q);
    const float* o = mv + iu * rec_stash_floats(E);
    m = rec_ld4(o + 4 * q);
    if (DL_STASH_M) {
      const float4 tl = rec_ld4(o + E);
      // the stale s from the record (the caller checked the row: row_ok) and the gather's lag
      if (row_ok) v = rec_ld4(rec + row * c.ld + 2 * E + 4 + 4 * q);
      v = stash_decay(v, __float_as_int(tl.z), c);
      if (first) { w = rows_u1[iu]; wm = tl.x; wv = tl.y; }
    } else {
      v = rec_ld4(o + E + 4 * q);
      if (first) { w = rows_u1[iu]; wm = o[2 * E]; wv = o[2 * E + 1]; }
    }
  } else if (!STASH && row_ok) {   // no stash: re-read the record and replay its catch-up
    const float* r = rec + row * c.ld;
    p = *reinterpret_cast<const float4*>(r + 4 * q);
    m = *reinterpret_cast<const float4*>(r + E + 4 + 4 * q);
    v = *reinterpret_cast<const float4*>(r + 2 * E + 4 + 4 * q);
    const float4 tail = *reinterpret_cast<const float4*>(r + E);
    w = tail.x; wm = tail.y; wv = tail.z;
    const int stamp = __float_as_int(tail.w);
    if (stamp < t - 1) catch_up4(p, m, v, w, wm, wv, first, stamp, t - 1, ring, c);
  }
}

// The row's gradient from its segment sums, then the TF1 Adam step on the record (or the
// replicated rows' accumulation for the later dense update).
template <int E>
__device__ __forceinline__ void rec_bwd_apply(const SegGrad4& s, int64_t row, int q, bool first, float4 p, float4 m,
                                              float4 v, float w, float wm, float wv, float* __restrict__ rec,
                                              const RecCfg& c, const dl_emb_layout& L, int n_rep,
                                              float* __restrict__ g_rep, float* __restrict__ g1_rep, float alpha,
                                              int t) {
  float4 g;
  g.x = seg_row_grad(s.s.x, s.dsum.x, s.x.x, s.dsum.x != 0.f ? p.x : 0.f);
  g.y = seg_row_grad(s.s.y, s.dsum.y, s.x.y, s.dsum.y != 0.f ? p.y : 0.f);
  g.z = seg_row_grad(s.s.z, s.dsum.z, s.x.z, s.dsum.z != 0.f ? p.z : 0.f);
  g.w = seg_row_grad(s.s.w, s.dsum.w, s.x.w, s.dsum.w != 0.f ? p.w : 0.f);
  const int64_t rrow = row - L.fm_cont_offset;   // replicated rows: [fm_cont_offset, + n_rep)
  if (rrow >= 0 && rrow < n_rep) {
    float* gr = g_rep + rrow * E + 4 * q;
    gr[0] += g.x; gr[1] += g.y; gr[2] += g.z; gr[3] += g.w;
    if (g1_rep && q == 0) g1_rep[rrow] += s.g1;
    return;
  }
  rec_adam(p.x, m.x, v.x, g.x, alpha, c);
  rec_adam(p.y, m.y, v.y, g.y, alpha, c);
  rec_adam(p.z, m.z, v.z, g.z, alpha, c);
  rec_adam(p.w, m.w, v.w, g.w, alpha, c);
  if (DL_BWD_DIAG & 8) {   // diagnostics: no record writes (one lane keeps the result live)
    if (p.x == 1234.5f) rec[q] = p.y + m.x + v.x;
    return;
  }
  float* r = rec + row * c.ld;
  rec_st4(r + 4 * q, p);
  rec_st4(r + E + 4 + 4 * q, m);
  rec_st4(r + 2 * E + 4 + 4 * q, v);
  if (q == 0) {
    if (first) rec_adam(w, wm, wv, s.g1, alpha, c);
    rec_st4(r + E, make_float4(w, wm, wv, __int_as_float(t)));
  }
  rec_write_pad<E>(r, q, c.ld);
}

#define DL_REC_BWD_PARAMS                                                                                    \
  SegGradIn sg, float *__restrict__ rec, RecCfg c, int n_rep, const float *__restrict__ rows_u,              \
      const float *__restrict__ rows_u1, const float *__restrict__ mv, const uint32_t *__restrict__ uniq,   \
      const int32_t *__restrict__ n_uniq, int world, float *__restrict__ g_rep, float *__restrict__ g1_rep, \
      const float *__restrict__ hist, const float *__restrict__ opt, int32_t *__restrict__ hot

// The hot rows' workspace (dl_rec_bwd_workspace_bytes): int32 header [kHotN] the number of
// hot rows, [kHotT] their chunks; then the hot rows' unique indices (appended by pass 1 in any
// order), their first chunk (exclusive prefix over ceil(refs / kSegChunk), plus the total), the
// owner of every chunk, and one partial sum per chunk (E/4 x {s, x, dsum} float4 + g1).
constexpr int kHotN = 0, kHotT = 1, kHotDone = 2, kHotList = 4;
struct HotWs {
  int32_t* hdr;
  int32_t* list;
  int32_t* off;
  int32_t* map;
  float* part;
  long long cap_list, cap_chunks;
};
__host__ __device__ inline long long hot_cap_list(long long nrefs) { return nrefs / (kSegLong + 1) + 1; }
__host__ __device__ inline long long hot_cap_chunks(long long nrefs) { return nrefs / kSegChunk + hot_cap_list(nrefs); }
__host__ __device__ inline int hot_part_floats(int E) { return 3 * E + 4; }
__host__ __device__ inline HotWs hot_ws(void* ws, long long nrefs, int E) {
  HotWs h;
  const long long cl = hot_cap_list(nrefs), cc = hot_cap_chunks(nrefs);
  h.hdr = reinterpret_cast<int32_t*>(ws);
  h.list = h.hdr + kHotList;
  h.off = h.list + cl;
  h.map = h.off + cl + 1;
  long long o = (long long)kHotList + cl + (cl + 1) + cc;
  o = (o + 3) / 4 * 4;   // 16-B aligned partials
  h.part = reinterpret_cast<float*>(h.hdr + o);
  h.cap_list = cl;
  h.cap_chunks = cc;
  return h;
}
__host__ __device__ inline long long hot_ws_bytes(long long nrefs, int E) {
  const long long cl = hot_cap_list(nrefs), cc = hot_cap_chunks(nrefs);
  long long o = (long long)kHotList + cl + (cl + 1) + cc;
  o = (o + 3) / 4 * 4;
  return 4 * o + 4 * cc * (long long)hot_part_floats(E);
}

// The scan, by one block of any size (a multiple of 64, at most 1024 threads).  (Run instead
// by pass 1's last block to finish, it cost every block a device-scope release fence — an L2
// write-back each on this chip: C2 2.25 -> 4.26 ms, profiles/r04zg/.)
__device__ __forceinline__ void hot_scan_block(const SegGradIn& sg, const HotWs& h, int nu, long long nrefs) {
  __shared__ int ws[16];
  __shared__ int carry_s;
  const int n = (int)min((long long)h.hdr[kHotN], h.cap_list);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nt = blockDim.x;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n; i0 += nt) {
    const int i = i0 + tid;
    int nch = 0;
    if (i < n) {
      const SegRange r = seg_range(sg, h.list[i], nu, nrefs);
      nch = (r.e1 - r.e0 + kSegChunk - 1) / kSegChunk;
    }
    int inc = nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wv; ++w) wbase += ws[w];
    const int carry = carry_s;
    const int ex = carry + wbase + inc - nch;
    if (i < n) {
      h.off[i] = ex;
      for (int c = 0; c < nch && ex + c < h.cap_chunks; ++c) h.map[ex + c] = i;
    }
    __syncthreads();
    if (tid == nt - 1) carry_s = ex + nch;
    __syncthreads();
  }
  if (tid == 0) {
    const int total = (int)min((long long)carry_s, h.cap_chunks);
    h.off[n] = total;
    h.hdr[kHotT] = total;
  }
}

// Pass 1: every unique row but the hot ones (more than kSegLong references: pass 2), E/4
// lanes per row.  STASH (the gather's moment stash is given, the engine's default): the
// catch-up path and its alpha window are compiled out — 96 -> fewer VGPRs, no LDS window.
// MULTI (multi-hot references present, C3): the pooled slot of a position from an LDS table,
// and each row's references fetched four at a time (their loads in flight together: a
// multi-hot row has ~2-3 references, each a dependent refs -> g_pool round trip); same sums.
template <int E, bool STASH, bool MULTI = false>
#ifndef DL_BWD_MIN_WAVES
#define DL_BWD_MIN_WAVES 1
#endif
#ifndef DL_BWD_STASH_SPECIAL
#define DL_BWD_STASH_SPECIAL 1
#endif
__global__ __launch_bounds__(256, STASH ? DL_BWD_MIN_WAVES : 1) void rec_bwd_adam_kernel(DL_REC_BWD_PARAMS) {
  if (step_poisoned(opt)) return;   // the batch failed validation: no update (common.h)
  rec_load_hyper(c, opt);
  __shared__ unsigned char slot_lut[MULTI ? kSlotLutMax : 1];
  if (MULTI) build_slot_lut(sg, slot_lut, sg.L.multi_width);
  __shared__ float hw[STASH ? 1 : kHistWin];
  RingW ring{hw, hist, c.hist_mask, (int)opt[7]};
  if (!STASH) ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4;
  const dl_emb_layout& L = sg.L;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const long long group0 = gt / LPR, ngroups = (long long)gridDim.x * blockDim.x / LPR;
  const int S = L.cate_fields;
  const int ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + S + L.fm_extra;
  const long long nrefs = (long long)L.batch * ns;
  const int nu = clamp_uniq(n_uniq, nrefs, sg.status);
  // head weights of the FM second-order outputs (offset F: not 16-B aligned)
  const float* ws = sg.w_head + F + 4 * q;
  const float4 wsec = L.use_fm ? make_float4(ws[0], ws[1], ws[2], ws[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const bool first = c.has_first && q == 0;
  // Software pipelining across this group's rows (each row is a chain of dependent loads:
  // segment bounds -> first reference -> dz / fm_sum / dx0 rows): the bounds are loaded
  // two rows ahead and the first reference one row ahead, so a row's own chain starts at
  // its data loads.  The references are still summed in the same order.
  SegRange nx = seg_range(sg, group0, nu, nrefs);
  int kx = nx.e0 < nx.e1 ? sg.refs[nx.e0] : -1;
  SegRange nn = seg_range(sg, group0 + ngroups, nu, nrefs);
  uint32_t key_n = group0 < nu ? uniq[group0] : 0u;   // the row key too (the record load waits on it)
  for (long long u = group0; u < nu; u += ngroups) {
    const SegRange cr = nx;
    const int kc = kx;
    const uint32_t key = key_n;
    nx = nn;
    kx = nx.e0 < nx.e1 ? sg.refs[nx.e0] : -1;
    nn = seg_range(sg, u + 2 * ngroups, nu, nrefs);
    key_n = u + ngroups < nu ? uniq[u + ngroups] : 0u;
    if (cr.e1 - cr.e0 > kSegLong) {   // a hot row: pass 2 (rec_bwd_long_kernel, or the chunked passes)
      if (hot && q == 0) {
        // at most nrefs / (kSegLong + 1) rows can be hot; an index past that means a stale
        // header (a step whose apply never ran): report it instead of writing past the list
        const int k = atomicAdd(&hot[kHotN], 1);
        if (k < hot_cap_list(nrefs)) hot[kHotList + k] = (int32_t)u;
        else index_fault(sg.status);
      }
      continue;
    }
    const int64_t row = decode_key(key, world);
    const bool row_ok = row >= 0 && row < L.n_rows;
    // the row's caught-up state (independent of the segment walk: issued first)
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), m = p, v = p;
    float w = 0.f, wm = 0.f, wv = 0.f;
    rec_bwd_state<E, STASH>(row, n_rep + u, q, first, row_ok, rec, rows_u, rows_u1, mv, c, t, ring, p, m, v, w, wm,
                            wv);
    const SegGrad4 s = MULTI ? segment_grad4_range_pf<E>(sg, cr.e0, cr.e1, kc, q, nrefs, wsec)
                             : segment_grad4_range<E>(sg, cr.e0, cr.e1, kc, q, nrefs, wsec);
    if (!row_ok) continue;
    rec_bwd_apply<E>(s, row, q, first, p, m, v, w, wm, wv, rec, c, L, n_rep, g_rep, g1_rep, alpha, t);
  }
}

// Pass 2: the rows whose segments have more than kSegLong references, one whole block each.
template <int E>
__global__ __launch_bounds__(256) void rec_bwd_long_kernel(DL_REC_BWD_PARAMS) {
  if (step_poisoned(opt)) return;
  rec_load_hyper(c, opt);
  __shared__ unsigned char slot_lut[kSlotLutMax];
  build_slot_lut(sg, slot_lut, sg.L.multi_width);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  __shared__ SegLongLds sh;
  const dl_emb_layout& L = sg.L;
  const int q = threadIdx.x % (E / 4);
  const int S = L.cate_fields, ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + S + L.fm_extra;
  const long long nrefs = (long long)L.batch * ns;
  const int nu = clamp_uniq(n_uniq, nrefs, sg.status);
  const float* ws = sg.w_head + F + 4 * q;
  const float4 wsec = L.use_fm ? make_float4(ws[0], ws[1], ws[2], ws[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const bool first = c.has_first && q == 0;
  for_long_segments<E>(sg, nu, nrefs, wsec, sh, [&](long long u, const SegGrad4& s) {
    const int64_t row = decode_key(uniq[u], world);
    const bool row_ok = row >= 0 && row < L.n_rows;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), m = p, v = p;
    float w = 0.f, wm = 0.f, wv = 0.f;
    rec_bwd_state<E>(row, n_rep + u, q, first, row_ok, rec, rows_u, rows_u1, mv, c, t, ring, p, m, v, w, wm, wv);
    if (row_ok) rec_bwd_apply<E>(s, row, q, first, p, m, v, w, wm, wv, rec, c, L, n_rep, g_rep, g1_rep, alpha, t);
  });
}

// Hot rows over many blocks (Zipf: a C3 batch's hottest rows have ~10^5 references, which one
// block summed alone while the rest of the chip idled).  Pass 1 lists the hot rows; then
//   rec_hot_scan_kernel   (one block) each hot row's chunks of kSegChunk references: the
//                         exclusive prefix of their counts and every chunk's owner
//   rec_hot_chunk_kernel  one block per chunk (grid-stride): the chunk's block sum
//                         (segment_grad4_block), written as the chunk's partial
//   rec_hot_apply_kernel  E/4 lanes per hot row: its partials added in chunk order (the
//                         canonical long-segment sum, segment.h) and the row's Adam step
__global__ __launch_bounds__(1024) void rec_hot_scan_kernel(SegGradIn sg, HotWs h, const int32_t* __restrict__ n_uniq,
                                                           const float* __restrict__ opt) {
  if (step_poisoned(opt)) return;
  const long long nrefs = (long long)sg.L.batch * index_slots(sg.L);
  hot_scan_block(sg, h, clamp_uniq(n_uniq, nrefs, sg.status), nrefs);
}

template <int E>
__global__ __launch_bounds__(256) void rec_hot_chunk_kernel(SegGradIn sg, HotWs h, const int32_t* __restrict__ n_uniq,
                                                            const float* __restrict__ opt) {
  if (step_poisoned(opt)) return;
  const int T = h.hdr[kHotT];
  if ((int)blockIdx.x >= T) return;   // (uniform ids: no hot chunk, every block leaves here)
  __shared__ unsigned char slot_lut[kSlotLutMax];
  build_slot_lut(sg, slot_lut, sg.L.multi_width);
  __shared__ SegLongLds sh;
  const dl_emb_layout& L = sg.L;
  const int q = threadIdx.x % (E / 4);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + L.cate_fields + L.fm_extra;
  const long long nrefs = (long long)L.batch * index_slots(L);
  const int nu = clamp_uniq(n_uniq, nrefs, sg.status);
  const float* ws = sg.w_head + F + 4 * q;
  const float4 wsec = L.use_fm ? make_float4(ws[0], ws[1], ws[2], ws[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int PF = hot_part_floats(E);
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    const int i = h.map[t];
    const int c = t - h.off[i];
    const SegRange r = seg_range(sg, h.list[i], nu, nrefs);
    const int c0 = r.e0 + c * kSegChunk;
    const SegGrad4 p = segment_grad4_block<E>(sg, c0, min(r.e1, c0 + kSegChunk), nrefs, wsec, sh);
    if (threadIdx.x < E / 4) {
      float4* o = reinterpret_cast<float4*>(h.part + (long long)t * PF) + 3 * q;
      o[0] = p.s; o[1] = p.x; o[2] = p.dsum;
      if (q == 0) h.part[(long long)t * PF + 3 * E] = p.g1;
    }
  }
}

template <int E>
__global__ __launch_bounds__(256) void rec_hot_apply_kernel(SegGradIn sg, float* __restrict__ rec, RecCfg c, int n_rep,
                                                            const float* __restrict__ rows_u,
                                                            const float* __restrict__ rows_u1,
                                                            const float* __restrict__ mv,
                                                            const uint32_t* __restrict__ uniq, int world,
                                                            float* __restrict__ g_rep, float* __restrict__ g1_rep,
                                                            const float* __restrict__ hist,
                                                            const float* __restrict__ opt, HotWs h) {
  const bool live = !step_poisoned(opt);
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4;
  const dl_emb_layout& L = sg.L;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const long long g0 = gt / LPR, ng = (long long)gridDim.x * blockDim.x / LPR;
  const int n = live ? (int)min((long long)h.hdr[kHotN], h.cap_list) : 0;
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const bool first = c.has_first && q == 0;
  const int PF = hot_part_floats(E);
  for (long long i = g0; i < n; i += ng) {
    const long long u = h.list[i];
    const int t0 = h.off[i], t1 = h.off[i + 1];
    auto load = [&](int k) {
      const float4* o = reinterpret_cast<const float4*>(h.part + (long long)k * PF) + 3 * q;
      return SegGrad4{o[0], o[1], o[2], h.part[(long long)k * PF + 3 * E]};
    };
    SegGrad4 s = load(t0);
    for (int k = t0 + 1; k < t1; ++k) seg_add(s, load(k));
    const int64_t row = decode_key(uniq[u], world);
    const bool row_ok = row >= 0 && row < L.n_rows;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), m = p, v = p;
    float w = 0.f, wm = 0.f, wv = 0.f;
    rec_bwd_state<E>(row, n_rep + u, q, first, row_ok, rec, rows_u, rows_u1, mv, c, t, ring, p, m, v, w, wm, wv);
    if (row_ok) rec_bwd_apply<E>(s, row, q, first, p, m, v, w, wm, wv, rec, c, L, n_rep, g_rep, g1_rep, alpha, t);
  }
  // the last block to finish resets the header for the next step's pass 1 (in place of a
  // reset launch before it): every block has read it by then (its loop bound came from it).
  // No fences: the zeros reach the next kernel through this one's end-of-kernel release, and a
  // device-scope fence here would write back the XCD's L2 in every block.
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(&h.hdr[kHotDone], 1) == (int)gridDim.x - 1) {
    h.hdr[kHotN] = 0;
    h.hdr[kHotT] = 0;
    h.hdr[kHotDone] = 0;
  }
}

// Rows [row0, row0 + n) updated with dense gradients g [n][E], g1 [n] (then zeroed).
__global__ __launch_bounds__(256) void rec_apply_rows_kernel(float* __restrict__ rec, RecCfg c, long long row0,
                                                             long long n, float* __restrict__ g,
                                                             float* __restrict__ g1, const float* __restrict__ hist,
                                                             const float* __restrict__ opt) {
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  const int E = c.E;
  const int t = (int)opt[7];
  const float alpha_t = opt[3];
  const bool skip = step_poisoned(opt);   // consume the gradients, apply nothing
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n * E;
       k += (long long)gridDim.x * blockDim.x) {
    const long long i = k / E;
    const int d = (int)(k % E);
    const float gi = g[k];
    const float g1i = (g1 && d == 0) ? g1[i] : 0.f;
    if (!skip) rec_update(rec + (row0 + i) * c.ld, E, d, gi, g1i, t, alpha_t, ring, c);
    g[k] = 0.f;
    if (g1 && d == 0) g1[i] = 0.f;
  }
}

// Every row caught up to step opt[7] (zero-gradient steps only).
template <int E>
__global__ __launch_bounds__(256) void rec_flush_kernel(float* __restrict__ rec, RecCfg c, long long n_rows,
                                                        const float* __restrict__ hist,
                                                        const float* __restrict__ opt, float* __restrict__ p_plane,
                                                        float* __restrict__ w1_plane, int slots) {
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const int target = (int)opt[7];
  // planes: p at p_plane + row * pitch, the first-order weight at w1_plane[row * w1s] (slot plane:
  // pitch 2E, the weight in column E of the same slot)
  const int pitch = slots ? 2 * E : E;
  const long long w1s = slots ? 2 * E : 1;
  float* w1p = slots ? (p_plane && c.has_first ? p_plane + E : nullptr) : w1_plane;
  for (long long row = gt / LPR; row < n_rows; row += (long long)gridDim.x * blockDim.x / LPR) {
    float* r = rec + row * c.ld;
    const float4 tail = *reinterpret_cast<const float4*>(r + E);
    const int stamp = __float_as_int(tail.w);
    if (stamp >= target) {
      if (p_plane) {   // caught up already: its p (and first-order weight) into the planes
        *reinterpret_cast<float4*>(p_plane + row * pitch + 4 * q) = *reinterpret_cast<const float4*>(r + 4 * q);
        if (w1p && q == 0) w1p[row * w1s] = tail.x;
      }
      continue;
    }
    float4 p = *reinterpret_cast<const float4*>(r + 4 * q);
    float4 m = *reinterpret_cast<const float4*>(r + E + 4 + 4 * q);
    float4 v = *reinterpret_cast<const float4*>(r + 2 * E + 4 + 4 * q);
    float w = tail.x, wm = tail.y, wv = tail.z;
    const bool first = c.has_first && q == 0;
    catch_up4(p, m, v, w, wm, wv, first, stamp, target, ring, c);
    if (p_plane) {
      *reinterpret_cast<float4*>(p_plane + row * pitch + 4 * q) = p;
      if (w1p && q == 0) w1p[row * w1s] = w;
    }
    *reinterpret_cast<float4*>(r + 4 * q) = p;
    *reinterpret_cast<float4*>(r + E + 4 + 4 * q) = m;
    *reinterpret_cast<float4*>(r + 2 * E + 4 + 4 * q) = v;
    if (q == 0) *reinterpret_cast<float4*>(r + E) = make_float4(w, wm, wv, __int_as_float(target));
  }
}

// Owner side of the sharded step, deterministic form: the received gradients g [n][E],
// g1 [n] of one step, grouped by row by dl_sort_unique over the received ids, are summed
// per row in sorted (position) order and applied: catch-up + TF1 Adam step t.
// E/4 lanes per row, float4 each (as the gather).
template <int E>
__global__ __launch_bounds__(256) void rec_apply_segments_kernel(float* __restrict__ rec, RecCfg c,
                                                                 const int32_t* __restrict__ uniq,
                                                                 const int32_t* __restrict__ seg_off,
                                                                 const int32_t* __restrict__ n_uniq, long long cap,
                                                                 long long n, const int32_t* __restrict__ pos,
                                                                 const float* __restrict__ g,
                                                                 const float* __restrict__ g1,
                                                                 const float* __restrict__ rows,
                                                                 const float* __restrict__ rows1,
                                                                 const float* __restrict__ mv,
                                                                 const float* __restrict__ hist,
                                                                 const float* __restrict__ opt) {
  if (step_poisoned(opt)) return;
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const long long nu = n_uniq ? (long long)clamp_uniq(n_uniq, cap, c.status) : cap;
  const bool first = c.has_first && q == 0;
  for (long long u = gt / LPR; u < nu; u += (long long)gridDim.x * blockDim.x / LPR) {
    const long long row = uniq[u];
    float* r = rec + row * c.ld;
    const int e0 = max(0, seg_off[u]);
    const int e1 = (int)min(n, (long long)seg_off[u + 1]);
    float4 p, m, v;
    float w = 0.f, wm = 0.f, wv = 0.f;
    int stamp = t - 1;
    if (mv) {
      // the owner gather's caught-up state at the row's first arrival (every arrival of a row
      // was gathered from the same record to the same step): no record read, no replay
      const int k0 = e0 < e1 ? pos[e0] : -1;
      if (k0 < 0 || k0 >= n) {
        index_fault(c.status);
        continue;
      }
      p = *reinterpret_cast<const float4*>(rows + (long long)k0 * E + 4 * q);
      const float* o = mv + (long long)k0 * rec_stash_floats(E);
      m = *reinterpret_cast<const float4*>(o + 4 * q);
      if (DL_STASH_M) {   // the stale s from the record, decayed over the gather's lag
        const float4 tl = *reinterpret_cast<const float4*>(o + E);
        v = stash_decay(*reinterpret_cast<const float4*>(r + 2 * E + 4 + 4 * q), __float_as_int(tl.z), c);
        if (first) { w = rows1[k0]; wm = tl.x; wv = tl.y; }
      } else {
        v = *reinterpret_cast<const float4*>(o + E + 4 * q);
        if (first) { w = rows1[k0]; wm = o[2 * E]; wv = o[2 * E + 1]; }
      }
    } else {
      p = *reinterpret_cast<const float4*>(r + 4 * q);
      m = *reinterpret_cast<const float4*>(r + E + 4 + 4 * q);
      v = *reinterpret_cast<const float4*>(r + 2 * E + 4 + 4 * q);
      const float4 tail = *reinterpret_cast<const float4*>(r + E);
      w = tail.x; wm = tail.y; wv = tail.z;
      stamp = __float_as_int(tail.w);
    }
    float4 gs = make_float4(0.f, 0.f, 0.f, 0.f);
    float g1s = 0.f;
    for (int e = e0; e < e1; ++e) {
      const int k = pos[e];
      if (k < 0 || k >= n) continue;
      const float4 gk = *reinterpret_cast<const float4*>(g + (long long)k * E + 4 * q);
      gs.x += gk.x; gs.y += gk.y; gs.z += gk.z; gs.w += gk.w;
      if (first) g1s += g1[k];
    }
    if (stamp < t - 1) catch_up4(p, m, v, w, wm, wv, first, stamp, t - 1, ring, c);
    rec_adam(p.x, m.x, v.x, gs.x, alpha, c);
    rec_adam(p.y, m.y, v.y, gs.y, alpha, c);
    rec_adam(p.z, m.z, v.z, gs.z, alpha, c);
    rec_adam(p.w, m.w, v.w, gs.w, alpha, c);
    *reinterpret_cast<float4*>(r + 4 * q) = p;
    *reinterpret_cast<float4*>(r + E + 4 + 4 * q) = m;
    *reinterpret_cast<float4*>(r + 2 * E + 4 + 4 * q) = v;
    if (q == 0) {
      if (first) rec_adam(w, wm, wv, g1s, alpha, c);
      *reinterpret_cast<float4*>(r + E) = make_float4(w, wm, wv, __int_as_float(t));
    }
    rec_write_pad<E>(r, q, c.ld);
  }
}

// Owner-side arrivals without a sort.  Each sender's ids are unique, so a row arrives at
// most once per sender.  link: head[row] <- position (atomic exchange), next[pos] <- the
// previous head: a per-row chain of its arrivals.  apply: the group whose position is the
// row's head is its leader; it sums the chain's gradients in ascending position order
// (selection over the short chain — the same order as a stable sort by row, so the result
// does not depend on which arrival won the exchange), steps the record and resets head.
constexpr int kMaxChain = 64;

__global__ __launch_bounds__(256) void rec_chain_link_kernel(const int32_t* __restrict__ ids, long long n,
                                                             int32_t* __restrict__ head, int32_t* __restrict__ next) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    if (ids[i] >= 0) next[i] = atomicExch(head + ids[i], (int32_t)i);   // -1: an empty exchange slot
}

template <int E>
__global__ __launch_bounds__(256) void rec_apply_chain_kernel(float* __restrict__ rec, RecCfg c,
                                                              const int32_t* __restrict__ ids, long long n,
                                                              int32_t* __restrict__ head,
                                                              const int32_t* __restrict__ next,
                                                              const float* __restrict__ g,
                                                              const float* __restrict__ g1,
                                                              const float* __restrict__ hist,
                                                              const float* __restrict__ opt) {
  if (step_poisoned(opt)) return;
  rec_load_hyper(c, opt);
  __shared__ float hw[kHistWin];
  const RingW ring = load_hist_window(hw, hist, (int)opt[7], c);
  constexpr int LPR = E / 4;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const int t = (int)opt[7];
  const float alpha = opt[3];
  const bool first = c.has_first && q == 0;
  for (long long i = gt / LPR; i < n; i += (long long)gridDim.x * blockDim.x / LPR) {
    const long long row = ids[i];
    if (row < 0 || head[row] != (int32_t)i) continue;   // an empty slot, or not the row's leader
    float* r = rec + row * c.ld;
    float4 p = *reinterpret_cast<const float4*>(r + 4 * q);
    float4 m = *reinterpret_cast<const float4*>(r + E + 4 + 4 * q);
    float4 v = *reinterpret_cast<const float4*>(r + 2 * E + 4 + 4 * q);
    const float4 tail = *reinterpret_cast<const float4*>(r + E);
    float w = tail.x, wm = tail.y, wv = tail.z;
    float4 gs = make_float4(0.f, 0.f, 0.f, 0.f);
    float g1s = 0.f;
    if (next[i] < 0) {   // one arrival (the common case)
      gs = *reinterpret_cast<const float4*>(g + i * E + 4 * q);
      if (first) g1s = g1[i];
    } else {
      // chains hold at most one arrival per sender (< kMaxChain): the walks are bounded so a
      // corrupted chain can never spin a wave forever
      long long last = -1;
      for (int sel = 0; sel < kMaxChain; ++sel) {
        long long best = LLONG_MAX;
        int hops = 0;
        for (long long j = i; j >= 0 && j < n && hops < kMaxChain; j = next[j], ++hops)
          if (j > last && j < best) best = j;
        if (best == LLONG_MAX) break;
        const float4 gk = *reinterpret_cast<const float4*>(g + best * E + 4 * q);
        gs.x += gk.x; gs.y += gk.y; gs.z += gk.z; gs.w += gk.w;
        if (first) g1s += g1[best];
        last = best;
      }
    }
    const int stamp = __float_as_int(tail.w);
    if (stamp < t - 1) catch_up4(p, m, v, w, wm, wv, first, stamp, t - 1, ring, c);
    rec_adam(p.x, m.x, v.x, gs.x, alpha, c);
    rec_adam(p.y, m.y, v.y, gs.y, alpha, c);
    rec_adam(p.z, m.z, v.z, gs.z, alpha, c);
    rec_adam(p.w, m.w, v.w, gs.w, alpha, c);
    *reinterpret_cast<float4*>(r + 4 * q) = p;
    *reinterpret_cast<float4*>(r + E + 4 + 4 * q) = m;
    *reinterpret_cast<float4*>(r + 2 * E + 4 + 4 * q) = v;
    if (q == 0) {
      if (first) rec_adam(w, wm, wv, g1s, alpha, c);
      *reinterpret_cast<float4*>(r + E) = make_float4(w, wm, wv, __int_as_float(t));
    }
    rec_write_pad<E>(r, q, c.ld);
  }
}

// head reset after the apply, as a separate pass: the leader test reads a stable head.
__global__ __launch_bounds__(256) void rec_chain_reset_kernel(const int32_t* __restrict__ ids, long long n,
                                                              int32_t* __restrict__ head) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    if (ids[i] >= 0) head[ids[i]] = -1;
}

__global__ void hist_record_kernel(const float* opt, float* hist, int mask) {
  hist[(int)opt[7] & mask] = opt[3];
}

static int rec_check(int E, int ld, int hist_len) {
  DL_CHECK_ARG(E == 4 || E == 8 || E == 16 || E == 32 || E == 64, "emb_dim %d not in {4,8,16,32,64}", E);
  DL_CHECK_ARG(ld >= 3 * E + 4 && ld % 32 == 0, "rec_ld %d: need >= 3E+4 and a multiple of 32", ld);
  DL_CHECK_ARG(hist_len >= 2 && (hist_len & (hist_len - 1)) == 0, "hist_len %d must be a power of two", hist_len);
  return 0;
}

static unsigned grid_cap(long long threads) {
  long long b = (threads + 255) / 256;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace dl

using namespace dl;

extern "C" int dl_adam_hist_record(const float* opt, float* hist, int32_t hist_len, void* stream) {
  DL_CHECK_ARG(opt && hist && hist_len >= 2 && (hist_len & (hist_len - 1)) == 0, "bad hist");
  hipLaunchKernelGGL(hist_record_kernel, dim3(1), dim3(1), 0, as_stream(stream), opt, hist, hist_len - 1);
  DL_RETURN_LAUNCH("dl_adam_hist_record");
}

extern "C" int32_t dl_rec_stash_floats(int32_t emb_dim) { return rec_stash_floats(emb_dim); }

extern "C" int dl_rec_gather(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                             int32_t n_rep, const uint32_t* uniq_keys, const int32_t* n_uniq, int64_t max_uniq,
                             int32_t world, const float* hist, int32_t hist_len, const float* opt, int32_t lag,
                             float* rows_u, float* rows_u1, float* mv_u, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(L && rec && hist && opt && rows_u, "NULL argument");
  if (int rc = rec_check(L->emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(n_rep >= 0 && n_rep <= L->n_rows && world >= 1, "bad n_rep/world");
  DL_CHECK_ARG(max_uniq == 0 || uniq_keys, "uniq keys required");
  DL_CHECK_ARG(!has_first || rows_u1, "rows_u1 required with first-order weights");
  const long long total = n_rep + (max_uniq > 0 ? max_uniq : 0);
  if (total == 0) return 0;
  DL_DISPATCH_E(L->emb_dim, {
    const unsigned grid = grid_cap(total * (kE / 4));
    auto kern = (rec_flags & DL_REC_SPARSE_ADAM) ? rec_gather_kernel<kE, true> : rec_gather_kernel<kE, false>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, as_stream(stream), rec,
                       make_rec_cfg(kE, rec_ld, rec_flags, hist_len), (int64_t)L->n_rows, n_rep,
                       n_rep ? (int64_t)L->fm_cont_offset : (int64_t)0, uniq_keys, n_uniq, (long long)max_uniq,
                       world, hist, opt, lag, rows_u,
                       has_first ? rows_u1 : nullptr, mv_u, GatherScatter{});
  });
  DL_RETURN_LAUNCH("dl_rec_gather");
}

extern "C" int dl_rec_gather_scatter(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                                     int32_t n_rep, const uint32_t* uniq_keys, const int32_t* n_uniq,
                                     int64_t max_uniq, const int32_t* seg_off, const int32_t* sorted_refs,
                                     const float* hist, int32_t hist_len, const float* opt, int32_t lag,
                                     float* rows_u, float* rows_u1, float* mv_u, float* fmst, void* x0,
                                     float* fm_out, float* mst, float* mst1, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(L && rec && hist && opt && rows_u && uniq_keys && n_uniq && seg_off && sorted_refs && x0,
               "NULL argument");
  if (int rc = rec_check(L->emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(n_rep >= 0 && n_rep <= L->n_rows, "bad n_rep");
  DL_CHECK_ARG(!has_first || rows_u1, "rows_u1 required with first-order weights");
  DL_CHECK_ARG(!L->use_fm || (fmst && fm_out), "FM staging rows and fm_out required");
  DL_CHECK_ARG(L->x0_ld % 4 == 0 && L->x0_cat_col % 4 == 0, "x0 must be float4 aligned");
  const long long total = n_rep + (max_uniq > 0 ? max_uniq : 0);
  if (total == 0) return 0;
  GatherScatter sc{};
  sc.seg_off = seg_off;
  sc.refs = sorted_refs;
  sc.fmst = fmst;
  sc.x0 = reinterpret_cast<float*>(x0);
  sc.fm_out = fm_out;
  sc.nrefs = (long long)L->batch * index_slots(*L);
  sc.ns = index_slots(*L);
  sc.S = L->cate_fields;
  sc.mb = index_multi_base(*L);
  sc.use_fm = L->use_fm;
  sc.Cf = (L->use_fm && L->fm_cont) ? L->cont_fields : 0;
  sc.x0_ld = L->x0_ld;
  sc.x0_cat_col = L->x0_cat_col;
  sc.x0_bf16 = L->x0_bf16;
  sc.fm_ld = L->fm_ld;
  sc.n_rep = n_rep;
  sc.mst = L->multi_width > 0 ? mst : nullptr;
  sc.mst1 = (L->multi_width > 0 && mst && has_first) ? mst1 : nullptr;
  sc.mw = L->multi_width;
  sc.status = reinterpret_cast<int*>(const_cast<float*>(opt) + DL_OPT_STATUS);
  DL_DISPATCH_E(L->emb_dim, {
    const unsigned grid = grid_cap(total * (kE / 4));
    auto kern = (rec_flags & DL_REC_SPARSE_ADAM) ? rec_gather_kernel<kE, true, true> : rec_gather_kernel<kE, false, true>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, as_stream(stream), rec,
                       make_rec_cfg(kE, rec_ld, rec_flags, hist_len), (int64_t)L->n_rows, n_rep,
                       n_rep ? (int64_t)L->fm_cont_offset : (int64_t)0, uniq_keys, n_uniq, (long long)max_uniq, 1,
                       hist, opt, lag, rows_u, has_first ? rows_u1 : nullptr, mv_u, sc);
    if (max_uniq > 0)
      hipLaunchKernelGGL(gather_scatter_long_kernel<kE>, dim3(1024), dim3(256), 0, as_stream(stream), sc, n_uniq,
                         (long long)max_uniq, rows_u, has_first ? rows_u1 : nullptr, has_first);
  });
  DL_RETURN_LAUNCH("dl_rec_gather_scatter");
}

extern "C" int64_t dl_rec_bwd_workspace_bytes(int64_t nrefs, int32_t emb_dim) {
  return nrefs > 0 && emb_dim > 0 ? hot_ws_bytes(nrefs, emb_dim) : 0;
}

extern "C" int dl_rec_bwd_adam(const dl_emb_layout* L, float* rec, int32_t rec_ld, int32_t rec_flags, int32_t n_rep,
                               const float* rows_u, const float* rows_u1, const float* mv_u,
                               const uint32_t* uniq_keys, const int32_t* seg_off, const int32_t* n_uniq,
                               const int32_t* sorted_refs, int32_t world, int64_t max_uniq, const float* dz,
                               const float* w_head, const float* fm_sum, const float* dx0, float* g_rep,
                               float* g1_rep, const float* hist, int32_t hist_len, const float* opt,
                               const dl_pool_desc* pool, void* hot_ws_ptr, int64_t hot_ws_size, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(L && rec && rows_u && uniq_keys && seg_off && n_uniq && sorted_refs && dx0 && opt,
               "NULL argument");
  const long long nrefs_all = (long long)L->batch * index_slots(*L);
  DL_CHECK_ARG(!hot_ws_ptr || (hot_ws_size >= hot_ws_bytes(nrefs_all, L->emb_dim) && (uintptr_t)hot_ws_ptr % 16 == 0),
               "hot-row workspace: %lld bytes needed (dl_rec_bwd_workspace_bytes), 16-B aligned",
               (long long)hot_ws_bytes(nrefs_all, L->emb_dim));
  DL_CHECK_ARG(mv_u || hist, "without the moment stash the alpha ring is required");
  if (int rc = rec_check(L->emb_dim, rec_ld, mv_u ? 2 : hist_len)) return rc;
  DL_CHECK_ARG(!L->use_fm || (dz && w_head && fm_sum), "FM backward inputs required");
  DL_CHECK_ARG(!has_first || rows_u1, "rows_u1 required with first-order weights");
  DL_CHECK_ARG(n_rep == 0 || g_rep, "g_rep required with replicated rows");
  DL_CHECK_ARG(!(n_rep && has_first) || g1_rep, "g1_rep required");
  DL_CHECK_ARG(L->dx0_ld % 4 == 0 && L->dx0_cat_col % 4 == 0, "dx0 must be float4 aligned");
  if (max_uniq <= 0) return 0;
  const bool multi = L->multi_width > 0;
  DL_CHECK_ARG(!multi || (pool && pool->slot_start && pool->slot_end && pool->x0 && pool->cnt_emb &&
                          pool->g_pool && pool->n_slots > 0),
               "multi-hot references need the pool descriptor");
  DL_CHECK_ARG(!multi || !L->use_fm || !has_first || (pool->cnt_first && pool->g1_pool),
               "cnt_first / g1_pool required");
  DL_CHECK_ARG(!multi || (pool->dx0_pool_col % 4 == 0 && L->x0_pool_col % 4 == 0),
               "pool columns not float4 aligned");
  DL_CHECK_ARG(!multi || pool->g_pitch == 0 || (pool->g_pitch >= L->emb_dim + 1 && pool->g_pitch % 4 == 0),
               "g_pitch %d: 0 or >= E + 1 and a multiple of 4", multi ? pool->g_pitch : 0);
  SegGradIn sg{*L, seg_off, sorted_refs, dz, w_head, fm_sum, dx0};
  sg.status = reinterpret_cast<int*>(const_cast<float*>(opt) + DL_OPT_STATUS);   // opt_status(opt), host side
  const bool g1p = multi && L->use_fm && has_first;
  if (multi) {
    sg.slot_start = pool->slot_start; sg.slot_end = pool->slot_end; sg.n_slots = pool->n_slots;
    sg.g_pool = pool->g_pool; sg.g1_pool = g1p ? pool->g1_pool : nullptr;
    sg.g_pitch = pool->g_pitch > 0 ? pool->g_pitch : L->emb_dim;
    sg.g1_stride = pool->g_pitch > 0 ? pool->g_pitch : 1;
    if (L->batch > 0)
      DL_DISPATCH_E(L->emb_dim, {
        hipLaunchKernelGGL(pool_grad_kernel<kE>, dim3(grid_cap((long long)L->batch * pool->n_slots * (kE / 4))),
                           dim3(256), 0, as_stream(stream), *L, *pool, dz, w_head, fm_sum, dx0, g1p);
      });
  }
  DL_DISPATCH_E(L->emb_dim, {
    unsigned grid = grid_cap(max_uniq * (kE / 4));
#ifdef DL_BWD_GRID_CAP
    if (grid > DL_BWD_GRID_CAP) grid = DL_BWD_GRID_CAP;
#endif
    auto bwd = (DL_BWD_STASH_SPECIAL && mv_u) ? (multi ? rec_bwd_adam_kernel<kE, true, true> : rec_bwd_adam_kernel<kE, true>)
                                              : rec_bwd_adam_kernel<kE, false>;
    hipStream_t st = as_stream(stream);
    const RecCfg rc = make_rec_cfg(kE, rec_ld, rec_flags, (mv_u ? 2 : hist_len));
    if (hot_ws_ptr) {
      const HotWs h = hot_ws(hot_ws_ptr, nrefs_all, kE);
      // the header is zero here: zeroed at allocation, reset by the previous step's apply
      hipLaunchKernelGGL(bwd, dim3(grid), dim3(256), 0, st, sg, rec, rc, n_rep, rows_u, has_first ? rows_u1 : nullptr,
                         mv_u, uniq_keys, n_uniq, world, g_rep, has_first ? g1_rep : nullptr, hist, opt, h.hdr);
      // the hot rows (none at uniform ids): chunks over the whole grid, then their updates
      hipLaunchKernelGGL(rec_hot_scan_kernel, dim3(1), dim3(1024), 0, st, sg, h, n_uniq, opt);
      hipLaunchKernelGGL(rec_hot_chunk_kernel<kE>, dim3(1024), dim3(256), 0, st, sg, h, n_uniq, opt);
      hipLaunchKernelGGL(rec_hot_apply_kernel<kE>, dim3(64), dim3(256), 0, st, sg, rec, rc, n_rep, rows_u,
                         has_first ? rows_u1 : nullptr, mv_u, uniq_keys, world, g_rep, has_first ? g1_rep : nullptr,
                         hist, opt, h);
    } else {
      hipLaunchKernelGGL(bwd, dim3(grid), dim3(256), 0, st, sg, rec, rc, n_rep, rows_u, has_first ? rows_u1 : nullptr,
                         mv_u, uniq_keys, n_uniq, world, g_rep, has_first ? g1_rep : nullptr, hist, opt, nullptr);
      // the hot rows' long segments (none at uniform ids: one scan of the segment offsets)
      hipLaunchKernelGGL(rec_bwd_long_kernel<kE>, dim3(1024), dim3(256), 0, st, sg, rec, rc, n_rep, rows_u,
                         has_first ? rows_u1 : nullptr, mv_u, uniq_keys, n_uniq, world, g_rep,
                         has_first ? g1_rep : nullptr, hist, opt, nullptr);
    }
  });
  DL_RETURN_LAUNCH("dl_rec_bwd_adam");
}

extern "C" int dl_rec_apply_rows(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, int64_t row0,
                                 int64_t n, float* g, float* g1, const float* hist, int32_t hist_len,
                                 const float* opt, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(rec && g && hist && opt, "NULL argument");
  if (int rc = rec_check(emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(!has_first || g1, "g1 required with first-order weights");
  DL_CHECK_ARG(row0 >= 0 && n >= 0, "bad row range");
  if (n == 0) return 0;
  hipLaunchKernelGGL(rec_apply_rows_kernel, dim3(grid_cap(n * emb_dim)), dim3(256), 0, as_stream(stream), rec,
                     make_rec_cfg(emb_dim, rec_ld, rec_flags, hist_len), (long long)row0,
                     (long long)n, g, has_first ? g1 : nullptr, hist, opt);
  DL_RETURN_LAUNCH("dl_rec_apply_rows");
}

extern "C" int dl_rec_flush(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, int64_t n_rows,
                            const float* hist, int32_t hist_len, const float* opt, float* p_plane, float* w1_plane,
                            void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(rec && hist && opt, "NULL argument");
  if (int rc = rec_check(emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(!p_plane || (uintptr_t)p_plane % 16 == 0, "p_plane must be 16-B aligned");
  if (n_rows <= 0) return 0;
  DL_DISPATCH_E(emb_dim, {
    hipLaunchKernelGGL(rec_flush_kernel<kE>, dim3(grid_cap(n_rows * (kE / 4))), dim3(256), 0, as_stream(stream),
                       rec, make_rec_cfg(kE, rec_ld, rec_flags, hist_len), (long long)n_rows, hist,
                       opt, p_plane, has_first ? w1_plane : nullptr, (rec_flags & DL_REC_PLANE_SLOTS) ? 1 : 0);
  });
  DL_RETURN_LAUNCH("dl_rec_flush");
}

extern "C" int dl_rec_apply_segments(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags,
                                     const int32_t* uniq, const int32_t* seg_off, const int32_t* n_uniq,
                                     int64_t max_uniq, int64_t n, const int32_t* sorted_pos, const float* g,
                                     const float* g1, const float* rows, const float* rows1, const float* mv,
                                     const float* hist, int32_t hist_len, const float* opt, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(rec && uniq && seg_off && sorted_pos && g && hist && opt, "NULL argument");
  if (int rc = rec_check(emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(!has_first || g1, "g1 required with first-order weights");
  DL_CHECK_ARG(!mv || (rows && (!has_first || rows1)), "the stash needs the gathered rows (and rows1)");
  if (max_uniq <= 0 || n <= 0) return 0;
  DL_DISPATCH_E(emb_dim, {
    hipLaunchKernelGGL(rec_apply_segments_kernel<kE>, dim3(grid_cap(max_uniq * (kE / 4))), dim3(256), 0,
                       as_stream(stream), rec, make_rec_cfg(kE, rec_ld, rec_flags, hist_len), uniq,
                       seg_off, n_uniq, (long long)max_uniq, (long long)n, sorted_pos, g, has_first ? g1 : nullptr,
                       rows, has_first ? rows1 : nullptr, mv, hist, opt);
  });
  DL_RETURN_LAUNCH("dl_rec_apply_segments");
}

extern "C" int dl_rec_chain_link(const int32_t* ids, int64_t n, int32_t* head, int32_t* next, void* stream) {
  DL_CHECK_ARG(ids && head && next && n >= 0, "bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(rec_chain_link_kernel, dim3(grid_cap(n)), dim3(256), 0, as_stream(stream), ids, (long long)n,
                     head, next);
  DL_RETURN_LAUNCH("dl_rec_chain_link");
}

extern "C" int dl_rec_apply_chain(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, const int32_t* ids,
                                  int64_t n, int32_t* head, const int32_t* next, const float* g, const float* g1,
                                  const float* hist, int32_t hist_len, const float* opt, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  DL_CHECK_ARG(rec && ids && head && next && g && hist && opt, "NULL argument");
  if (int rc = rec_check(emb_dim, rec_ld, hist_len)) return rc;
  DL_CHECK_ARG(!has_first || g1, "g1 required with first-order weights");
  if (n <= 0) return 0;
  DL_DISPATCH_E(emb_dim, {
    hipLaunchKernelGGL(rec_apply_chain_kernel<kE>, dim3(grid_cap(n * (kE / 4))), dim3(256), 0, as_stream(stream), rec,
                       make_rec_cfg(kE, rec_ld, rec_flags, hist_len), ids, (long long)n, head, next, g,
                       has_first ? g1 : nullptr, hist, opt);
  });
  hipLaunchKernelGGL(rec_chain_reset_kernel, dim3(grid_cap(n)), dim3(256), 0, as_stream(stream), ids, (long long)n,
                     head);
  DL_RETURN_LAUNCH("dl_rec_apply_chain");
}
