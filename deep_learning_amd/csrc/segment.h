// Per-unique-row gradient from the sorted batch index (index.hip), shared by the
// table-gradient backward (embed.hip) and the fused backward + lazy Adam on row
// records (rec.hip).
//
// A row's references are summed in sorted (deterministic) order.  FM references
// (deepfm_pipeline.py:89-107) contribute  dsec_b * (fm_sum_b - V[row])  per dim
// (value 1 for a cate field) and dz_b * w_first[slot] to the first-order weight;
// deep references (:120) contribute the dx0 columns of their slot.  Lane d of an
// E-lane group owns dim d.
#pragma once

// Diagnostics builds only (wrong results): DL_BWD_DIAG bits redirect one of the backward's
// access streams to a cache-resident address, so PMC bytes and time split by stream —
// 1: the dx0 slices, 2: the fm_sum rows, 16: the pooled-slot gradients (segment_grad4_range,
// seg_fetch), 4: the stash rows, 8: the record writes (rec.hip rec_bwd_state / rec_bwd_apply).
#ifndef DL_BWD_DIAG
#define DL_BWD_DIAG 0
#endif
#include "common.h"

namespace dl {

struct SegGradIn {
  dl_emb_layout L;
  const int32_t* seg_off;
  const int32_t* refs;
  const float* dz;
  const float* w_head;
  const float* fm_sum;
  const float* dx0;
  // multi-hot references (index_multi_base(L) <= slot; records only): nonzero-mean pooling
  // (deepfm_multi_cate.py:71-111) — slot ranges within the multi block and the per-sample
  // pooled-slot gradients g_pool [B][n_slots][E], g1_pool [B][n_slots] (rec.hip pool_grad)
  const int32_t* slot_start;
  const int32_t* slot_end;
  int n_slots;
  const float* g_pool;
  const float* g1_pool;
  int g_pitch;    // floats between (sample, slot) rows of g_pool (E: packed)
  int g1_stride;  // ... and between their g1_pool entries (1: packed; g_pitch: interleaved)
  // opt's status word: an index entry out of range (a corrupt batch index) sets
  // DL_STATUS_INDEX there and the host raises, instead of the entry being skipped silently
  int* status;
  // optional: the pooled slot of every multi-hot position (slot_lut[l], n_slots = none), an LDS
  // table built by the kernel in place of the per-reference search over the slot ranges
  const unsigned char* slot_lut;
};

// The pooled slot of multi-hot position l (n_slots when l lies in no slot).
__device__ __forceinline__ int seg_slot_of(const SegGradIn& a, int l) {
  if (a.slot_lut) return a.slot_lut[l];
  int m = 0;
  while (m < a.n_slots && !(l >= a.slot_start[m] && l < a.slot_end[m])) ++m;
  return m;
}

// Fills an LDS slot table for positions [0, width) (every thread of the block calls it).
constexpr int kSlotLutMax = 2048;
__device__ __forceinline__ void build_slot_lut(SegGradIn& a, unsigned char* lut, int width) {
  if (a.n_slots <= 0 || width <= 0 || width > kSlotLutMax || a.n_slots > 255) return;
  for (int l = threadIdx.x; l < width; l += blockDim.x) {
    int m = 0;
    while (m < a.n_slots && !(l >= a.slot_start[m] && l < a.slot_end[m])) ++m;
    lut[l] = (unsigned char)m;
  }
  __syncthreads();
  a.slot_lut = lut;
}

__device__ __forceinline__ void index_fault(int* status) {
  if (status) raise_fault(status, DL_STATUS_INDEX);
}

struct SegGrad {
  float s, dsum, x, g1;   // sum dsec*fm_sum, sum dsec, sum dx0, first-order gradient
};

// Products are fused explicitly (fmaf) so the per-dim and the float4 forms below —
// and every kernel that inlines them — produce bit-identical sums.
template <int E>
__device__ __forceinline__ SegGrad segment_grad(const SegGradIn& a, long long u, int d, long long nrefs,
                                                float wsec) {
  const dl_emb_layout& L = a.L;
  const int S = L.cate_fields;
  const int ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int o0 = a.seg_off[u], o1 = a.seg_off[u + 1];
  if (o0 < 0 || o1 > nrefs || o0 > o1) index_fault(a.status);
  const int e0 = max(0, o0);
  const int e1 = (int)min(nrefs, (long long)o1);
  SegGrad r{0.f, 0.f, 0.f, 0.f};
  const int mb = index_multi_base(L);   // multi-hot refs exist only with records (segment_grad4)
  for (int e = e0; e < e1; ++e) {
    const int k = a.refs[e];
    if (k < 0 || k >= nrefs) {
      index_fault(a.status);
      continue;
    }
    const int b = k / ns, sl = k % ns;
    if (sl >= mb) continue;
    if (L.use_fm && sl < S) {
      const float dzb = a.dz[b];
      const float ds = dzb * wsec;
      r.s = fmaf(ds, a.fm_sum[(long long)b * E + d], r.s);
      r.dsum += ds;
      r.g1 = fmaf(dzb, a.w_head[Cf + sl], r.g1);
    } else {
      const int f = L.use_fm ? sl - S : sl;
      r.x += a.dx0[(long long)b * L.dx0_ld + L.dx0_cat_col + f * E + d];
    }
  }
  return r;
}

// Row gradient from the sums: FM part  s - V[row]*dsum, plus the deep part.
__device__ __forceinline__ float seg_row_grad(float s, float dsum, float x, float v) {
  return fmaf(-v, dsum, s) + x;
}

struct SegGrad4 {
  float4 s, x;
  float4 dsum;   // per-dim sum of dsec (wsec differs per dim)
  float g1;
};

// Same sums for dims 4q..4q+3 of one row (one lane, float4 loads).
// A unique row's reference range [e0, e1) in the sorted refs (empty past nu).
struct SegRange { int e0, e1; };
__device__ __forceinline__ SegRange seg_range(const SegGradIn& a, long long u, long long nu, long long nrefs) {
  if (u >= nu) return SegRange{0, 0};
  const int o0 = a.seg_off[u], o1 = a.seg_off[u + 1];
  if (o0 < 0 || o1 > nrefs || o0 > o1) index_fault(a.status);
  return SegRange{max(0, o0), (int)min(nrefs, (long long)o1)};
}

// Sums over the references e0..e1 of one row; k_first = refs[e0] when the caller has
// already loaded it (software pipelining across rows), -2 to load it here.
template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_range(const SegGradIn& a, int e0, int e1, int k_first, int q,
                                                        long long nrefs, float4 wsec, int stride = 1) {
  const dl_emb_layout& L = a.L;
  const int S = L.cate_fields;
  const int ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  SegGrad4 r{z, z, z, 0.f};
  const int mb = index_multi_base(L);
  for (int e = e0; e < e1; e += stride) {
    const int k = (e == e0 && k_first != -2) ? k_first : a.refs[e];
    if (k < 0 || k >= nrefs) {
      index_fault(a.status);
      continue;
    }
    const int b = k / ns, sl = k % ns;
    if (sl >= mb) {
      // pooled slot m of multi position l: every member row gets the slot's gradient
      const int m = seg_slot_of(a, sl - mb);
      if (m == a.n_slots) continue;
      const long long bm = (long long)b * a.n_slots + m;
      const long long bmd = (DL_BWD_DIAG & 16) ? 0 : bm;
      const float4 gp = *reinterpret_cast<const float4*>(a.g_pool + bmd * a.g_pitch + 4 * q);
      r.x.x += gp.x; r.x.y += gp.y; r.x.z += gp.z; r.x.w += gp.w;
      if (a.g1_pool) r.g1 += a.g1_pool[bmd * a.g1_stride];
    } else if (L.use_fm && sl < S) {
      const float dzb = a.dz[b];
      const float4 fs = *reinterpret_cast<const float4*>(a.fm_sum + (long long)((DL_BWD_DIAG & 2) ? 0 : b) * E + 4 * q);
      const float4 ds = make_float4(dzb * wsec.x, dzb * wsec.y, dzb * wsec.z, dzb * wsec.w);
      r.s.x = fmaf(ds.x, fs.x, r.s.x); r.s.y = fmaf(ds.y, fs.y, r.s.y);
      r.s.z = fmaf(ds.z, fs.z, r.s.z); r.s.w = fmaf(ds.w, fs.w, r.s.w);
      r.dsum.x += ds.x; r.dsum.y += ds.y; r.dsum.z += ds.z; r.dsum.w += ds.w;
      r.g1 = fmaf(dzb, a.w_head[Cf + sl], r.g1);
    } else {
      const int f = L.use_fm ? sl - S : sl;
      const float4 gx = *reinterpret_cast<const float4*>(a.dx0 + (long long)((DL_BWD_DIAG & 1) ? 0 : b) * L.dx0_ld +
                                                         L.dx0_cat_col + f * E + 4 * q);
      r.x.x += gx.x; r.x.y += gx.y; r.x.z += gx.z; r.x.w += gx.w;
    }
  }
  return r;
}

// One reference's contribution, loaded (fetch) apart from its accumulation (acc), so that
// several references' loads can be in flight before the first is added; acc in reference
// order performs exactly the operations of segment_grad4_range.
struct SegRef {
  int kind;     // 0 none, 1 pooled slot, 2 FM second order, 3 deep embedding
  float4 v;     // g_pool row / fm_sum row / dx0 row
  float dzb, w; // FM: dz[b], w_head[Cf + sl]; pooled: g1_pool (when present)
};

template <int E>
__device__ __forceinline__ SegRef seg_fetch(const SegGradIn& a, bool in, int k, int q, long long nrefs) {
  const dl_emb_layout& L = a.L;
  const int S = L.cate_fields, ns = index_slots(L), mb = index_multi_base(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  SegRef f{0, make_float4(0.f, 0.f, 0.f, 0.f), 0.f, 0.f};
  if (!in) return f;
  if (k < 0 || k >= nrefs) {
    index_fault(a.status);
    return f;
  }
  const int b = k / ns, sl = k % ns;
  if (sl >= mb) {
    const int m = seg_slot_of(a, sl - mb);
    if (m == a.n_slots) return f;
    const long long bm = (long long)b * a.n_slots + m;
    f.kind = 1;
    const long long bmd = (DL_BWD_DIAG & 16) ? 0 : bm;
    f.v = *reinterpret_cast<const float4*>(a.g_pool + bmd * a.g_pitch + 4 * q);
    f.w = a.g1_pool ? a.g1_pool[bmd * a.g1_stride] : 0.f;
  } else if (L.use_fm && sl < S) {
    f.kind = 2;
    f.dzb = a.dz[b];
    f.v = *reinterpret_cast<const float4*>(a.fm_sum + (long long)((DL_BWD_DIAG & 2) ? 0 : b) * E + 4 * q);
    f.w = a.w_head[Cf + sl];
  } else {
    const int fi = L.use_fm ? sl - S : sl;
    f.kind = 3;
    f.v = *reinterpret_cast<const float4*>(a.dx0 + (long long)((DL_BWD_DIAG & 1) ? 0 : b) * L.dx0_ld + L.dx0_cat_col +
                                           fi * E + 4 * q);
  }
  return f;
}

__device__ __forceinline__ void seg_acc(SegGrad4& r, const SegRef& f, float4 wsec, bool g1pool) {
  if (f.kind == 1 || f.kind == 3) {
    r.x.x += f.v.x; r.x.y += f.v.y; r.x.z += f.v.z; r.x.w += f.v.w;
    if (f.kind == 1 && g1pool) r.g1 += f.w;
  } else if (f.kind == 2) {
    const float4 ds = make_float4(f.dzb * wsec.x, f.dzb * wsec.y, f.dzb * wsec.z, f.dzb * wsec.w);
    r.s.x = fmaf(ds.x, f.v.x, r.s.x); r.s.y = fmaf(ds.y, f.v.y, r.s.y);
    r.s.z = fmaf(ds.z, f.v.z, r.s.z); r.s.w = fmaf(ds.w, f.v.w, r.s.w);
    r.dsum.x += ds.x; r.dsum.y += ds.y; r.dsum.z += ds.z; r.dsum.w += ds.w;
    r.g1 = fmaf(f.dzb, f.w, r.g1);
  }
}

// segment_grad4_range with four references' loads in flight at a time (same sums, same
// order): k_first = refs[e0] already loaded by the caller, or -2
template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_range_pf(const SegGradIn& a, int e0, int e1, int k_first, int q,
                                                           long long nrefs, float4 wsec) {
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  SegGrad4 r{z, z, z, 0.f};
  const bool g1pool = a.g1_pool != nullptr;
  for (int e = e0; e < e1; e += 4) {
    int k[4];
    bool in[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      in[i] = e + i < e1;
      k[i] = !in[i] ? -1 : (e + i == e0 && k_first != -2) ? k_first : a.refs[e + i];
    }
    SegRef f[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = seg_fetch<E>(a, in[i], k[i], q, nrefs);
#pragma unroll
    for (int i = 0; i < 4; ++i) seg_acc(r, f[i], wsec, g1pool);
  }
  return r;
}

// segment_grad4_range over e0, e0 + stride, ... < e1 (same sums, same order) for the long
// segments of hot rows (Zipf: a C3 batch's hottest multi-hot row has ~10^5 references, ~3 k per
// lane group): kSegUnroll references' data loads in flight at a time, and the next group's
// reference indices loaded while this group's data is in flight — one memory round trip per
// kSegUnroll references instead of two.  (16 in flight: 198 VGPRs, the long kernel's 1,024
// blocks in two rounds, and no faster on hot rows; 4 keeps 4 waves per SIMD: profiles/r03u4/.)
#ifndef DL_SEG_UNROLL
#define DL_SEG_UNROLL 4
#endif
constexpr int kSegUnroll = DL_SEG_UNROLL;

template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_strided(const SegGradIn& a, int e0, int e1, int stride, int q,
                                                          long long nrefs, float4 wsec) {
  constexpr int U = kSegUnroll;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  SegGrad4 r{z, z, z, 0.f};
  const bool g1pool = a.g1_pool != nullptr;
  int kn[U];
#pragma unroll
  for (int i = 0; i < U; ++i) kn[i] = e0 + i * stride < e1 ? a.refs[e0 + i * stride] : -1;
  for (int e = e0; e < e1; e += U * stride) {
    int k[U];
    bool in[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      in[i] = e + i * stride < e1;
      k[i] = kn[i];
    }
    SegRef f[U];
#pragma unroll
    for (int i = 0; i < U; ++i) f[i] = seg_fetch<E>(a, in[i], k[i], q, nrefs);
    const int en = e + U * stride;
#pragma unroll
    for (int i = 0; i < U; ++i) kn[i] = en + i * stride < e1 ? a.refs[en + i * stride] : -1;
#pragma unroll
    for (int i = 0; i < U; ++i) seg_acc(r, f[i], wsec, g1pool);
  }
  return r;
}

// Hot rows (Zipf ids; a Zipf batch's hottest rows have ~15 k references, where one lane
// group used to take ~15 k dependent loads).  A segment of more than kSegLong references is
// left out of the per-row pass and summed in a second pass by a whole 256-thread block:
// 256 / (E/4) slots of E/4 lanes each take the references slot, slot + NS, ... in order
// (four loads in flight); a wave's slot sums are combined by a fixed butterfly (lane xor E/4,
// 2E/4, ... 32), the block's four wave sums in wave order.  The order is fixed, so the sums
// are deterministic, and every kernel using it (the lazy record update, the dense sorted
// backward, the sharded senders) sums a row alike.  The per-row pass keeps its registers
// (and occupancy): a long segment costs it one length test.
constexpr int kSegLong = 32;

__device__ __forceinline__ float4 seg_xor4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64), __shfl_xor(v.z, m, 64), __shfl_xor(v.w, m, 64));
}
__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

template <int LPR>
__device__ __forceinline__ void seg_wave_butterfly(SegGrad4& r) {
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1) {
    r.s = f4add(r.s, seg_xor4(r.s, m));
    r.x = f4add(r.x, seg_xor4(r.x, m));
    r.dsum = f4add(r.dsum, seg_xor4(r.dsum, m));
    r.g1 += __shfl_xor(r.g1, m, 64);
  }
}

struct SegLongLds {   // per block
  int n;
  int u[256];
  float4 s[4][16], x[4][16], d[4][16];   // per wave, per q (E/4 <= 16)
  float g1[4];
};

// One long segment summed by the whole block (every thread calls it); the total lands in
// threads 0 .. E/4 - 1 (lane q = thread).
template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_block(const SegGradIn& a, int e0, int e1, long long nrefs,
                                                        float4 wsec, SegLongLds& sh) {
  constexpr int LPR = E / 4, NS = 256 / LPR;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = tid % LPR;
  SegGrad4 r = segment_grad4_strided<E>(a, e0 + tid / LPR, e1, NS, q, nrefs, wsec);
  seg_wave_butterfly<LPR>(r);
  if (lane < LPR) {
    sh.s[wv][lane] = r.s; sh.x[wv][lane] = r.x; sh.d[wv][lane] = r.dsum;
    if (lane == 0) sh.g1[wv] = r.g1;
  }
  __syncthreads();
  SegGrad4 t = {sh.s[0][q], sh.x[0][q], sh.d[0][q], sh.g1[0]};
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    t.s = f4add(t.s, sh.s[w][q]); t.x = f4add(t.x, sh.x[w][q]); t.dsum = f4add(t.dsum, sh.d[w][q]);
    t.g1 += sh.g1[w];
  }
  __syncthreads();   // the partials are re-used by the next segment
  return t;
}

// The canonical sum of a long segment: chunks of kSegChunk references, each summed by
// segment_grad4_block from its own start, and the chunk sums added in chunk order
// (total = c0; total += c1; ...).  One block computes it chunk after chunk here; the lazy
// record backward spreads the chunks of its hot rows over many blocks (rec.hip,
// rec_bwd_chunk_kernel) and adds their partials in the same order — the same sums either way.
constexpr int kSegChunk = 1024;

__device__ __forceinline__ void seg_add(SegGrad4& t, const SegGrad4& c) {
  t.s = f4add(t.s, c.s); t.x = f4add(t.x, c.x); t.dsum = f4add(t.dsum, c.dsum);
  t.g1 += c.g1;
}

template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_chunked(const SegGradIn& a, int e0, int e1, long long nrefs,
                                                          float4 wsec, SegLongLds& sh) {
  SegGrad4 t = segment_grad4_block<E>(a, e0, min(e1, e0 + kSegChunk), nrefs, wsec, sh);
  for (int c0 = e0 + kSegChunk; c0 < e1; c0 += kSegChunk)
    seg_add(t, segment_grad4_block<E>(a, c0, min(e1, c0 + kSegChunk), nrefs, wsec, sh));
  return t;
}

// Second pass over the long segments: block b scans its share of the unique rows for
// segments of more than kSegLong references and calls fn(u, sums) for each, in threads
// 0 .. E/4 - 1, after the whole block summed it.  Block-uniform; one barrier per 256 rows.
template <int E, class Fn>
__device__ __forceinline__ void for_long_segments(const SegGradIn& a, long long nu, long long nrefs, float4 wsec,
                                                  SegLongLds& sh, Fn&& fn) {
  const int tid = threadIdx.x;
  const long long per = (nu + gridDim.x - 1) / gridDim.x;
  const long long u0 = (long long)blockIdx.x * per, u1 = min(nu, u0 + per);
  for (long long base = u0; base < u1; base += 256) {
    const long long u = base + tid;
    const SegRange cr = seg_range(a, u < u1 ? u : nu, nu, nrefs);
    const bool lng = cr.e1 - cr.e0 > kSegLong;
    if (tid == 0) sh.n = 0;
    if (!__syncthreads_or(lng)) continue;
    if (lng) sh.u[atomicAdd(&sh.n, 1)] = (int)(u - base);
    __syncthreads();
    const int n = sh.n;
    for (int k = 0; k < n; ++k) {
      const long long uu = base + sh.u[k];
      const SegRange r = seg_range(a, uu, nu, nrefs);
      const SegGrad4 t = segment_grad4_chunked<E>(a, r.e0, r.e1, nrefs, wsec, sh);
      if (tid < E / 4) fn(uu, t);
    }
    __syncthreads();   // sh.n / sh.u before the next chunk
  }
}

template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4(const SegGradIn& a, long long u, int q, long long nrefs,
                                                  float4 wsec) {
  const int o0 = a.seg_off[u], o1 = a.seg_off[u + 1];
  if (o0 < 0 || o1 > nrefs || o0 > o1) index_fault(a.status);
  return segment_grad4_range<E>(a, max(0, o0), (int)min(nrefs, (long long)o1), -2, q, nrefs, wsec);
}

__device__ __forceinline__ int clamp_uniq(const int32_t* n_uniq, long long cap, int* status = nullptr) {
  const int nu = n_uniq[0];
  if (nu < 0 || nu > cap) index_fault(status);
  return nu < 0 ? 0 : (nu > cap ? (int)cap : nu);
}

}  // namespace dl
