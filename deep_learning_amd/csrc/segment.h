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
};

struct SegGrad {
  float s, dsum, x, g1;   // sum dsec*fm_sum, sum dsec, sum dx0, first-order gradient
};

// every index derived from another kernel's output is clamped: a stale or
// racing index can cost accuracy, never an out-of-bounds access
template <int E>
__device__ __forceinline__ SegGrad segment_grad(const SegGradIn& a, long long u, int d, long long nrefs,
                                                float wsec) {
  const dl_emb_layout& L = a.L;
  const int S = L.cate_fields;
  const int ns = (L.use_fm ? S : 0) + S;
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int e0 = max(0, a.seg_off[u]);
  const int e1 = (int)min(nrefs, (long long)a.seg_off[u + 1]);
  SegGrad r{0.f, 0.f, 0.f, 0.f};
  for (int e = e0; e < e1; ++e) {
    const int k = a.refs[e];
    if (k < 0 || k >= nrefs) continue;
    const int b = k / ns, sl = k % ns;
    if (L.use_fm && sl < S) {
      const float dzb = a.dz[b];
      const float ds = dzb * wsec;
      r.s += ds * a.fm_sum[(long long)b * E + d];
      r.dsum += ds;
      r.g1 += dzb * a.w_head[Cf + sl];
    } else {
      const int f = L.use_fm ? sl - S : sl;
      r.x += a.dx0[(long long)b * L.dx0_ld + L.dx0_cat_col + f * E + d];
    }
  }
  return r;
}

__device__ __forceinline__ int clamp_uniq(const int32_t* n_uniq, long long cap) {
  const int nu = n_uniq[0];
  return nu < 0 ? 0 : (nu > cap ? (int)cap : nu);
}

}  // namespace dl
