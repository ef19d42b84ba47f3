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
  // opt's status word: an index entry out of range (a corrupt batch index) sets
  // DL_STATUS_INDEX there and the host raises, instead of the entry being skipped silently
  int* status;
};

__device__ __forceinline__ void index_fault(int* status) {
  if (status) atomicOr(status, DL_STATUS_INDEX);
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
      const int l = sl - mb;
      int m = 0;
      while (m < a.n_slots && !(l >= a.slot_start[m] && l < a.slot_end[m])) ++m;
      if (m == a.n_slots) continue;
      const long long bm = (long long)b * a.n_slots + m;
      const float4 gp = *reinterpret_cast<const float4*>(a.g_pool + bm * E + 4 * q);
      r.x.x += gp.x; r.x.y += gp.y; r.x.z += gp.z; r.x.w += gp.w;
      if (a.g1_pool) r.g1 += a.g1_pool[bm];
    } else if (L.use_fm && sl < S) {
      const float dzb = a.dz[b];
      const float4 fs = *reinterpret_cast<const float4*>(a.fm_sum + (long long)b * E + 4 * q);
      const float4 ds = make_float4(dzb * wsec.x, dzb * wsec.y, dzb * wsec.z, dzb * wsec.w);
      r.s.x = fmaf(ds.x, fs.x, r.s.x); r.s.y = fmaf(ds.y, fs.y, r.s.y);
      r.s.z = fmaf(ds.z, fs.z, r.s.z); r.s.w = fmaf(ds.w, fs.w, r.s.w);
      r.dsum.x += ds.x; r.dsum.y += ds.y; r.dsum.z += ds.z; r.dsum.w += ds.w;
      r.g1 = fmaf(dzb, a.w_head[Cf + sl], r.g1);
    } else {
      const int f = L.use_fm ? sl - S : sl;
      const float4 gx = *reinterpret_cast<const float4*>(a.dx0 + (long long)b * L.dx0_ld + L.dx0_cat_col + f * E + 4 * q);
      r.x.x += gx.x; r.x.y += gx.y; r.x.z += gx.z; r.x.w += gx.w;
    }
  }
  return r;
}

// Hot rows (Zipf ids): a segment longer than kSegLong references is not walked by its own
// lane group, one reference after another, but by the whole wave: 64 / (E/4) slots of E/4
// lanes each take the references slot, slot + NS, ... in order, and the slot sums are
// combined by a fixed butterfly (lane xor E/4, 2E/4, ... 32).  Every lane of the wave must
// call this, with the same (e0, e1); every lane gets the total for its dims 4q..4q+3.  The
// order is fixed, so the sums are deterministic, and every kernel using it (the lazy
// record update, the dense sorted backward, the sharded senders) sums a row alike.
constexpr int kSegLong = 32;

__device__ __forceinline__ float4 seg_xor4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64), __shfl_xor(v.z, m, 64), __shfl_xor(v.w, m, 64));
}

template <int E>
__device__ __forceinline__ SegGrad4 segment_grad4_wave(const SegGradIn& a, int e0, int e1, long long nrefs,
                                                       float4 wsec) {
  constexpr int LPR = E / 4, NS = 64 / LPR;
  const int lane = threadIdx.x & 63, q = lane % LPR, slot = lane / LPR;
  SegGrad4 r = segment_grad4_range<E>(a, e0 + slot, e1, -2, q, nrefs, wsec, NS);
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1) {
    const float4 s2 = seg_xor4(r.s, m), x2 = seg_xor4(r.x, m), d2 = seg_xor4(r.dsum, m);
    const float g2 = __shfl_xor(r.g1, m, 64);
    // lower slot first, so both partners form the same sum
    const bool lo = (lane & m) == 0;
    r.s = lo ? make_float4(r.s.x + s2.x, r.s.y + s2.y, r.s.z + s2.z, r.s.w + s2.w)
             : make_float4(s2.x + r.s.x, s2.y + r.s.y, s2.z + r.s.z, s2.w + r.s.w);
    r.x = lo ? make_float4(r.x.x + x2.x, r.x.y + x2.y, r.x.z + x2.z, r.x.w + x2.w)
             : make_float4(x2.x + r.x.x, x2.y + r.x.y, x2.z + r.x.z, x2.w + r.x.w);
    r.dsum = lo ? make_float4(r.dsum.x + d2.x, r.dsum.y + d2.y, r.dsum.z + d2.z, r.dsum.w + d2.w)
                : make_float4(d2.x + r.dsum.x, d2.y + r.dsum.y, d2.z + r.dsum.z, d2.w + r.dsum.w);
    r.g1 = lo ? r.g1 + g2 : g2 + r.g1;
  }
  return r;
}

// The wave's long segments, one after another (wave-uniform loop): a lane group whose
// segment [e0, e1) is longer than kSegLong gets its sums here; the others keep theirs.
// Every lane of the wave must call this.
template <int E>
__device__ __forceinline__ void segment_grad4_long(const SegGradIn& a, int e0, int e1, bool mine_long,
                                                   long long nrefs, float4 wsec, SegGrad4& out) {
  constexpr int LPR = E / 4;
  const int lane = threadIdx.x & 63;
  uint64_t todo = __ballot(mine_long && (lane % LPR) == 0);
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    todo &= todo - 1;
    const int le0 = __shfl(e0, leader, 64), le1 = __shfl(e1, leader, 64);
    const SegGrad4 t = segment_grad4_wave<E>(a, le0, le1, nrefs, wsec);
    if (lane / LPR == leader / LPR) out = t;
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
