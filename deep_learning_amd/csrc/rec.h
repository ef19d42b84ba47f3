// Row-record helpers shared by rec.hip (gather / update / flush) and embed.hip (the
// forward that reads records directly): the device-side Adam hyper-parameters and the
// lazy-exact catch-up (replayed zero-gradient TF1 Adam steps, see rec.hip).
#pragma once
#include "common.h"

namespace dl {

struct RecCfg {
  int E, ld, has_first, hist_mask;
  float omb1, omb2, eps;   // filled on the device from opt (rec_load_hyper)
};

__device__ __forceinline__ void rec_load_hyper(RecCfg& c, const float* opt) {
  c.omb1 = 1.f - opt[4];
  c.omb2 = 1.f - opt[5];
  c.eps = opt[6];
}

// Replays zero-gradient steps (from, to] on one float4 of p/m/v (and the
// first-order triple when `first` is set).
__device__ __forceinline__ void catch_up4(float4& p, float4& m, float4& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const float* __restrict__ hist,
                                          const RecCfg& c) {
  if (to - from > c.hist_mask + 1) from = to - (c.hist_mask + 1);   // host bounds the lag; never read past the ring
  for (int j = from + 1; j <= to; ++j) {
    const float al = hist[j & c.hist_mask];
    adam_elem(p.x, m.x, v.x, 0.f, al, c.omb1, c.omb2, c.eps);
    adam_elem(p.y, m.y, v.y, 0.f, al, c.omb1, c.omb2, c.eps);
    adam_elem(p.z, m.z, v.z, 0.f, al, c.omb1, c.omb2, c.eps);
    adam_elem(p.w, m.w, v.w, 0.f, al, c.omb1, c.omb2, c.eps);
    if (first) adam_elem(w, wm, wv, 0.f, al, c.omb1, c.omb2, c.eps);
  }
}

__device__ __forceinline__ void catch_up1(float& p, float& m, float& v, float& w, float& wm, float& wv,
                                          bool first, int from, int to, const float* __restrict__ hist,
                                          const RecCfg& c) {
  if (to - from > c.hist_mask + 1) from = to - (c.hist_mask + 1);
  for (int j = from + 1; j <= to; ++j) {
    const float al = hist[j & c.hist_mask];
    adam_elem(p, m, v, 0.f, al, c.omb1, c.omb2, c.eps);
    if (first) adam_elem(w, wm, wv, 0.f, al, c.omb1, c.omb2, c.eps);
  }
}

}  // namespace dl
