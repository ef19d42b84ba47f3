// Output layer + sigmoid + eps-clipped log-loss, forward and backward in one pass.
//
// Reference: models/deepfm_pipeline.py:155-183 (z = concat([first, second, deep]) @ W + b,
// score = sigmoid(z), loss = tf.losses.log_loss(label, score) = mean_B of
// -y ln(p+1e-7) - (1-y) ln(1-p+1e-7)); models/dnn_pipeline.py:114-131 (no FM part).
//
// One wave per sample: the feature row (FM part + last hidden layer) is read
// once, z is a wave reduction, and the same registers then produce
//   dh = dz * w_h * (h > 0)   (ReluGrad of the last hidden layer, fused)
// and the per-lane partial sums of dW = sum_b dz_b * feat_b.  Blocks leave
// their partials in a slab that dl_adam_dense reduces (deterministic; no atomics).
#include "common.h"

namespace dl {

constexpr int kHeadMaxFm = 128;   // FM columns (F + E)
constexpr int kHeadMaxH4 = 4;     // hidden float4 chunks per lane: H <= 1024

__global__ __launch_bounds__(256) void head_kernel(int B, int fm_cols, int H, const float* __restrict__ fm_out,
                                                   int fm_ld, const float* __restrict__ h, int ldh,
                                                   const float* __restrict__ w, const float* __restrict__ label,
                                                   float eps, float inv_batch, float* __restrict__ score,
                                                   float* __restrict__ z_out, float* __restrict__ dz,
                                                   float* __restrict__ dh, float* __restrict__ slab) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int H4 = (H + 3) / 4;
  const float bias = w[fm_cols + H];
  // per-lane weights (held in registers across samples)
  float wf[kHeadMaxFm / 64];
  float4 wh[kHeadMaxH4];
#pragma unroll
  for (int k = 0; k < kHeadMaxFm / 64; ++k) {
    const int c = lane + 64 * k;
    wf[k] = c < fm_cols ? w[c] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < kHeadMaxH4; ++k) {
    const int c = 4 * (lane + 64 * k);
    wh[k].x = c + 0 < H ? w[fm_cols + c + 0] : 0.f;
    wh[k].y = c + 1 < H ? w[fm_cols + c + 1] : 0.f;
    wh[k].z = c + 2 < H ? w[fm_cols + c + 2] : 0.f;
    wh[k].w = c + 3 < H ? w[fm_cols + c + 3] : 0.f;
  }
  float gf[kHeadMaxFm / 64] = {};
  float4 gh[kHeadMaxH4];
#pragma unroll
  for (int k = 0; k < kHeadMaxH4; ++k) gh[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  float gb = 0.f, lsum = 0.f;

  // Four samples per round: their rows are loaded together (four round trips in flight
  // per wave instead of one), then reduced in the same sample order as a one-sample loop.
  constexpr int kAhead = 4;
  for (int b0 = wave; b0 < B; b0 += kAhead * nwaves) {
    float ff[kAhead][kHeadMaxFm / 64];
    float4 hh[kAhead][kHeadMaxH4];
    float yy[kAhead];
#pragma unroll
    for (int i = 0; i < kAhead; ++i) {
      const int b = b0 + i * nwaves;
      const bool ok = b < B;
#pragma unroll
      for (int k = 0; k < kHeadMaxFm / 64; ++k) {
        const int c = lane + 64 * k;
        ff[i][k] = ok && c < fm_cols ? fm_out[(long long)b * fm_ld + c] : 0.f;
      }
      const float* hb = h + (long long)b * ldh;
#pragma unroll
      for (int k = 0; k < kHeadMaxH4; ++k) {
        const int c4 = lane + 64 * k;
        hh[i][k] = ok && c4 < H4 ? *reinterpret_cast<const float4*>(hb + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      yy[i] = ok ? label[b] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kAhead; ++i) {
      const int b = b0 + i * nwaves;
      if (b >= B) break;   // wave-uniform
      float part = 0.f;
#pragma unroll
      for (int k = 0; k < kHeadMaxFm / 64; ++k) part += ff[i][k] * wf[k];
#pragma unroll
      for (int k = 0; k < kHeadMaxH4; ++k)
        part += hh[i][k].x * wh[k].x + hh[i][k].y * wh[k].y + hh[i][k].z * wh[k].z + hh[i][k].w * wh[k].w;
      const float z = wave_sum(part) + bias;
      const float p = 1.f / (1.f + expf(-z));
      const float y = yy[i];
      const float dp = (-y / (p + eps) + (1.f - y) / (1.f - p + eps)) * inv_batch;
      const float g = dp * p * (1.f - p);   // SigmoidGrad
      if (lane == 0) {
        score[b] = p;
        if (z_out) z_out[b] = z;
        dz[b] = g;
        gb += g;
        lsum += -y * logf(p + eps) - (1.f - y) * logf(1.f - p + eps);
      }
#pragma unroll
      for (int k = 0; k < kHeadMaxFm / 64; ++k) gf[k] += g * ff[i][k];
      float* dhb = dh + (long long)b * ldh;
#pragma unroll
      for (int k = 0; k < kHeadMaxH4; ++k) {
        const int c4 = lane + 64 * k;
        gh[k].x += g * hh[i][k].x; gh[k].y += g * hh[i][k].y;
        gh[k].z += g * hh[i][k].z; gh[k].w += g * hh[i][k].w;
        if (c4 < H4) {
          const int c = 4 * c4;
          float4 o;
          o.x = hh[i][k].x > 0.f ? g * wh[k].x : 0.f;
          o.y = hh[i][k].y > 0.f ? g * wh[k].y : 0.f;
          o.z = hh[i][k].z > 0.f ? g * wh[k].z : 0.f;
          o.w = hh[i][k].w > 0.f ? g * wh[k].w : 0.f;
          if (c + 3 < H) *reinterpret_cast<float4*>(dhb + c) = o;
          else {
            if (c + 0 < H) dhb[c + 0] = o.x;
            if (c + 1 < H) dhb[c + 1] = o.y;
            if (c + 2 < H) dhb[c + 2] = o.z;
          }
        }
      }
    }
  }
  // block reduction -> slab[block][fm_cols + H + 2]
  const int width = fm_cols + H + 2;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][width]
#pragma unroll
  for (int k = 0; k < kHeadMaxFm / 64; ++k) {
    const int c = lane + 64 * k;
    if (c < fm_cols) red[wid * width + c] = gf[k];
  }
#pragma unroll
  for (int k = 0; k < kHeadMaxH4; ++k) {
    const int c = 4 * (lane + 64 * k);
    float* o = red + wid * width + fm_cols;
    if (c + 0 < H) o[c + 0] = gh[k].x;
    if (c + 1 < H) o[c + 1] = gh[k].y;
    if (c + 2 < H) o[c + 2] = gh[k].z;
    if (c + 3 < H) o[c + 3] = gh[k].w;
  }
  if (lane == 0) {
    red[wid * width + fm_cols + H] = gb;
    red[wid * width + fm_cols + H + 1] = lsum;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < width; c += blockDim.x)
    slab[(long long)blockIdx.x * width + c] =
        red[c] + red[width + c] + red[2 * width + c] + red[3 * width + c];
}

// Wide&Deep cross logit (models/wdl.py:225-264):
//   z = sum_f w[wide_f] + sum_j w[Fw + j] * h_j + bias    (w = wdl_weights [N + H])
// The deep-output weights are rows Fw..Fw+H of the same vector, aliasing wide ids
// in that range.  Wide rows get dz added into g_w (+ touched flag) as 64-bit fixed point
// (units of 2^-48, DL_WIDE_GRAD_SCALE): integer atomics are associative, so the wide gradient
// — a segment sum over the batch's wide ids, TF's UnsortedSegmentSum — is the same bits
// whatever order the waves add in (f32 atomics were not: run-to-run ulp differences),
// and at |sum| << 2^15 every term keeps ~2^-48 absolute precision, finer than an f32 sum.
// The dense part leaves per-block partials slab[block][0..H) = sum dz*h_j,
// [H] = sum dz (bias), [H+1] = sum loss_b.
//
// One wave per sample, samples strided over the grid.  The wide lookups are two
// dependent round trips (ids, then weights), so they run ahead of the sample being
// reduced: ids two samples ahead, weights one ahead; only the h row load is left on
// a sample's critical path.  DHB: dh written as bf16 (the bf16 tower's dY operand,
// no separate cast pass).
// H4M: float4 chunks of a hidden row per lane (2: H <= 512, 4: H <= 1024).  With DL_WDL_HEAD_PF the
// next sample's h row is loaded while this one is reduced (a wave walks ~8 samples, each a dependent chain:
// row -> wave sum -> loss -> gradient stores), as the wide ids (two ahead) and weights (one).
#ifndef DL_WDL_HEAD_PF
#define DL_WDL_HEAD_PF 0   // 1: prefetch the next sample's h row (measured neutral, C5 head 64 us both: profiles/r06f)
#endif
template <bool DHB, int H4M = kHeadMaxH4>
__global__ __launch_bounds__(256) void wdl_head_kernel(int B, int Fw, int H, const int64_t* __restrict__ wide,
                                                       int wide_ld, const float* __restrict__ h, int ldh,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       long long w_rows, const float* __restrict__ label, float eps,
                                                       float inv_batch, float* __restrict__ score,
                                                       float* __restrict__ z_out, float* __restrict__ dz,
                                                       void* __restrict__ dh_out, long long* __restrict__ g_w,
                                                       uint8_t* __restrict__ touched, float* __restrict__ slab,
                                                       int32_t* err) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int H4 = (H + 3) / 4;
  const float b0 = bias[0];
  float4 wh[H4M], gh[H4M];
#pragma unroll
  for (int k = 0; k < H4M; ++k) {
    const int c = 4 * (lane + 64 * k);
    wh[k].x = c + 0 < H ? w[Fw + c + 0] : 0.f;
    wh[k].y = c + 1 < H ? w[Fw + c + 1] : 0.f;
    wh[k].z = c + 2 < H ? w[Fw + c + 2] : 0.f;
    wh[k].w = c + 3 < H ? w[Fw + c + 3] : 0.f;
    gh[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // this lane's wide id of sample bb, validated (-1: none or out of range)
  auto load_id = [&](int bb) -> long long {
    if (bb >= B || lane >= Fw) return -1;
    const long long r = wide[(long long)bb * wide_ld + lane];
    if (r < 0 || r >= w_rows) { if (err) atomicOr(err, 1); return -1; }
    return r;
  };
  long long id_n = load_id(wave);
  float wv_n = id_n >= 0 ? w[id_n] : 0.f;
  long long id_nn = load_id(wave + nwaves);
  float gb = 0.f, lsum = 0.f;
  // sample bb's h row (zeros past B or H)
  auto load_h = [&](int bb, float4 (&r)[H4M]) {
    const float* hb = h + (long long)min(bb, B - 1) * ldh;
#pragma unroll
    for (int k = 0; k < H4M; ++k) {
      const int c4 = lane + 64 * k;
      r[k] = (c4 < H4 && bb < B) ? *reinterpret_cast<const float4*>(hb + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float4 hn[H4M];
  if (DL_WDL_HEAD_PF) load_h(wave, hn);
  for (int b = wave; b < B; b += nwaves) {
    const long long wr = id_n;
    float part = wv_n;
    id_n = id_nn;
    wv_n = id_n >= 0 ? w[id_n] : 0.f;
    id_nn = load_id(b + 2 * nwaves);
    float4 hh[H4M];
    if (DL_WDL_HEAD_PF) {
#pragma unroll
      for (int k = 0; k < H4M; ++k) hh[k] = hn[k];
      load_h(b + nwaves, hn);   // the next sample's row, in flight during this one
    } else {
      load_h(b, hh);
    }
#pragma unroll
    for (int k = 0; k < H4M; ++k)
      part += hh[k].x * wh[k].x + hh[k].y * wh[k].y + hh[k].z * wh[k].z + hh[k].w * wh[k].w;
    const float z = wave_sum(part) + b0;
    const float p = 1.f / (1.f + expf(-z));
    const float y = label[b];
    const float g = (-y / (p + eps) + (1.f - y) / (1.f - p + eps)) * inv_batch * p * (1.f - p);
    if (lane == 0) {
      score[b] = p;
      if (z_out) z_out[b] = z;
      dz[b] = g;
      gb += g;
      lsum += -y * logf(p + eps) - (1.f - y) * logf(1.f - p + eps);
    }
    if (wr >= 0 && g_w) {
      atomicAdd(reinterpret_cast<unsigned long long*>(g_w + wr), (unsigned long long)wide_fixed(g));
      if (touched) touched[wr] = 1;
    }
#pragma unroll
    for (int k = 0; k < H4M; ++k) {
      const int c4 = lane + 64 * k;
      gh[k].x += g * hh[k].x; gh[k].y += g * hh[k].y; gh[k].z += g * hh[k].z; gh[k].w += g * hh[k].w;
      if (c4 < H4) {
        const int c = 4 * c4;
        float o[4] = {hh[k].x > 0.f ? g * wh[k].x : 0.f, hh[k].y > 0.f ? g * wh[k].y : 0.f,
                      hh[k].z > 0.f ? g * wh[k].z : 0.f, hh[k].w > 0.f ? g * wh[k].w : 0.f};
        if (DHB) {
          unsigned short* d = reinterpret_cast<unsigned short*>(dh_out) + (long long)b * ldh + c;
          if (c + 4 <= H) {
            *reinterpret_cast<uint2*>(d) = make_uint2(f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16),
                                                      f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16));
          } else {
            for (int e = 0; e < 4; ++e)
              if (c + e < H) d[e] = f2bf(o[e]);
          }
        } else {
          float* d = reinterpret_cast<float*>(dh_out) + (long long)b * ldh + c;
          if (c + 4 <= H) {
            *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
          } else {
            for (int e = 0; e < 4; ++e)
              if (c + e < H) d[e] = o[e];
          }
        }
      }
    }
  }
  const int width = H + 2;
  extern __shared__ __attribute__((aligned(16))) float red[];
#pragma unroll
  for (int k = 0; k < H4M; ++k) {
    const int c = 4 * (lane + 64 * k);
    float* o = red + wid * width;
    if (c + 0 < H) o[c + 0] = gh[k].x;
    if (c + 1 < H) o[c + 1] = gh[k].y;
    if (c + 2 < H) o[c + 2] = gh[k].z;
    if (c + 3 < H) o[c + 3] = gh[k].w;
  }
  if (lane == 0) {
    red[wid * width + H] = gb;
    red[wid * width + H + 1] = lsum;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < width; c += blockDim.x)
    slab[(long long)blockIdx.x * width + c] = red[c] + red[width + c] + red[2 * width + c] + red[3 * width + c];
}

// g[row0 + j] += sum_blocks slab[blk*width + col0 + j] (fixed point, as the head's wide
// gradient); touched[row0 + j] = 1
__global__ __launch_bounds__(256) void slab_fold_rows_kernel(const float* __restrict__ slab, int blocks, int width,
                                                             int col0, int n, long long* __restrict__ g,
                                                             long long row0, uint8_t* __restrict__ touched) {
  const int j = blockIdx.x;
  if (j >= n) return;
  float acc = 0.f;
  for (int t = threadIdx.x; t < blocks; t += blockDim.x) acc += slab[(long long)t * width + col0 + j];
  acc = wave_sum(acc);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    g[row0 + j] += wide_fixed(part[0] + part[1] + part[2] + part[3]);
    if (touched) touched[row0 + j] = 1;
  }
}

}  // namespace dl

using namespace dl;

template <bool DHB>
static int wdl_head(int32_t B, int32_t Fw, int32_t H, const int64_t* wide, int32_t wide_ld, const float* h,
                    int32_t ldh, const float* w, const float* bias, int64_t w_rows, const float* label, float eps,
                    float inv_batch, float* score, float* z_out, float* dz, void* dh, int64_t* g_w, uint8_t* touched,
                    float* slab, int32_t slab_blocks, int32_t* err, void* stream) {
  DL_CHECK_ARG(Fw >= 0 && Fw <= 64, "Fw %d not in [0, 64]", Fw);
  DL_CHECK_ARG(H > 0 && H <= 4 * 64 * kHeadMaxH4, "H %d too large", H);
  DL_CHECK_ARG(w_rows >= Fw + H, "wdl_weights must have >= Fw + H rows");
  DL_CHECK_ARG(ldh % 4 == 0 && ldh >= H && ((uintptr_t)h % 16) == 0, "h must be 16-B aligned, ldh %% 4 == 0");
  DL_CHECK_ARG(((uintptr_t)dh % (DHB ? 8 : 16)) == 0, "dh must be %d-B aligned", DHB ? 8 : 16);
  DL_CHECK_ARG(w && bias && label && score && dz && dh && slab, "NULL argument");
  const int grid = dl_wdl_head_grid(B);
  DL_CHECK_ARG(slab_blocks >= grid, "slab needs %d blocks", grid);
  if (B == 0) return 0;
  const size_t lds = 4 * (size_t)(H + 2) * sizeof(float);
  auto kern = H <= 4 * 64 * 2 ? wdl_head_kernel<DHB, 2> : wdl_head_kernel<DHB, kHeadMaxH4>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, as_stream(stream), B, Fw, H, wide, wide_ld,
                     h, ldh, w, bias, (long long)w_rows, label, eps, inv_batch, score, z_out, dz, dh,
                     reinterpret_cast<long long*>(g_w), touched,
                     slab, err);
  DL_RETURN_LAUNCH(DHB ? "dl_wdl_head_fwd_bwd_bf16" : "dl_wdl_head_fwd_bwd");
}

extern "C" int dl_wdl_head_fwd_bwd(int32_t B, int32_t Fw, int32_t H, const int64_t* wide, int32_t wide_ld,
                                   const float* h, int32_t ldh, const float* w, const float* bias, int64_t w_rows,
                                   const float* label, float eps, float inv_batch, float* score, float* z_out,
                                   float* dz, float* dh, int64_t* g_w, uint8_t* touched, float* slab,
                                   int32_t slab_blocks, int32_t* err, void* stream) {
  return wdl_head<false>(B, Fw, H, wide, wide_ld, h, ldh, w, bias, w_rows, label, eps, inv_batch, score, z_out, dz,
                         dh, g_w, touched, slab, slab_blocks, err, stream);
}

extern "C" int dl_wdl_head_fwd_bwd_bf16(int32_t B, int32_t Fw, int32_t H, const int64_t* wide, int32_t wide_ld,
                                        const float* h, int32_t ldh, const float* w, const float* bias,
                                        int64_t w_rows, const float* label, float eps, float inv_batch, float* score,
                                        float* z_out, float* dz, uint16_t* dh, int64_t* g_w, uint8_t* touched,
                                        float* slab, int32_t slab_blocks, int32_t* err, void* stream) {
  return wdl_head<true>(B, Fw, H, wide, wide_ld, h, ldh, w, bias, w_rows, label, eps, inv_batch, score, z_out, dz,
                        dh, g_w, touched, slab, slab_blocks, err, stream);
}

extern "C" int dl_slab_fold_rows(const float* slab, int32_t blocks, int32_t width, int32_t col0, int32_t n,
                                 int64_t* g, int64_t row0, uint8_t* touched, void* stream) {
  DL_CHECK_ARG(slab && g && blocks >= 1 && col0 + n <= width, "bad args");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(slab_fold_rows_kernel, dim3(n), dim3(256), 0, as_stream(stream), slab, blocks, width, col0, n,
                     reinterpret_cast<long long*>(g), (long long)row0, touched);
  DL_RETURN_LAUNCH("dl_slab_fold_rows");
}

extern "C" int dl_head_grid(int32_t B) {
  int g = (B + 63) / 64;   // ~16 samples per wave; the slab stays small for the dense Adam
  if (g > 512) g = 512;      // that reads it one element per wave
  return g < 1 ? 1 : g;
}

extern "C" int dl_wdl_head_grid(int32_t B) {
  // the wdl head is a latency-bound chain per sample (ids -> weights, row load -> wave
  // sum -> loss -> atomics): ~8 samples per wave at B = 65,536 (512 blocks: 155 us,
  // 2048: 130 us); its slab is folded column-wise (dl_slab_fold_rows), one block per column
  int g = (B + 31) / 32;
  if (g > 2048) g = 2048;
  return g < 1 ? 1 : g;
}

extern "C" int dl_head_fwd_bwd(int32_t B, int32_t fm_cols, int32_t H, const float* fm_out,
                               int32_t fm_ld, const float* h, int32_t ldh, const float* w,
                               const float* label, float eps, float inv_batch, float* score,
                               float* z_out, float* dz, float* dh, float* slab,
                               int32_t slab_blocks, void* stream) {
  DL_CHECK_ARG(fm_cols >= 0 && fm_cols <= kHeadMaxFm, "fm_cols %d > %d", fm_cols, kHeadMaxFm);
  DL_CHECK_ARG(H > 0 && H <= 4 * 64 * kHeadMaxH4, "H %d > %d", H, 4 * 64 * kHeadMaxH4);
  DL_CHECK_ARG(ldh % 4 == 0 && ldh >= H && ((uintptr_t)h % 16) == 0, "h must be 16-B aligned, ldh %% 4 == 0");
  DL_CHECK_ARG(!fm_cols || fm_out, "fm_out required");
  const int grid = dl_head_grid(B);
  DL_CHECK_ARG(slab_blocks >= grid, "slab needs %d blocks", grid);
  if (B == 0) return 0;
  const size_t lds = 4 * (size_t)(fm_cols + H + 2) * sizeof(float);
  hipLaunchKernelGGL(head_kernel, dim3(grid), dim3(256), lds, as_stream(stream), B, fm_cols, H,
                     fm_out, fm_ld, h, ldh, w, label, eps, inv_batch, score, z_out, dz, dh, slab);
  DL_RETURN_LAUNCH("dl_head_fwd_bwd");
}
