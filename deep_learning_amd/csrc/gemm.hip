// Dense-tower GEMMs on the CDNA4 matrix cores.
//
// fp32: v_mfma_f32_16x16x4_f32 (exact f32 in / f32 accumulate, a k-ordered fma
// chain — the fp32 reference numerics of deepfm_pipeline.py:150-152 and the
// MatMul gradients, at the f32 matrix peak of 157 TF).
// bf16: v_mfma_f32_16x16x32_bf16 for the Wide&Deep bf16 tower (config C5).
//
// One kernel template covers the three products of a layer:
//   forward  H  = X  . W        (A row-major [i][r], B row-major [r][j])
//   dX       dX = dY . W^T      (B read transposed)
//   dW       dW = X^T . dY      (A read transposed, split-K over the batch into
//                                partial slabs that the Adam kernel sums)
// Bias is folded in: every activation matrix carries a ones column and every
// weight matrix an extra bias row, so dW's extra row IS the bias gradient.
//
// Block: 256 threads = 4 waves; tile BM x BN, K-step 16, LDS double buffer with
// register-staged prefetch (issue-early / write-late).  LDS images are k-major
// ([k][i], [k][j]) with the row stride padded to 16 mod 32 words so the two
// 16-lane k-rows of an MFMA operand read land in disjoint banks.
// Block -> tile mapping is XCD-aware: tiles that share the A rows are dealt to
// blocks b, b+8, ... which the dispatcher places on one XCD (speed only).
#include "common.h"
#include <cstdlib>

namespace dl {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int dl_u32x4_t __attribute__((__vector_size__(4 * sizeof(unsigned int))));
typedef unsigned int dl_u32x2_t __attribute__((__vector_size__(2 * sizeof(unsigned int))));

#ifndef DL_GEMM_BK
#define DL_GEMM_BK 16   // k-slab per LDS stage of the f32 GEMM
#endif
#ifndef DL_GEMM_GLDS
#define DL_GEMM_GLDS 0  // LDS-DMA for the k-contiguous A tile (correct, measured neutral: DESIGN.md §4)
#endif

struct GemmParams {
  const void* A;
  const void* B;
  void* C;
  const void* mask;
  int M, N, K;
  int lda, ldb, ldc, ldm;
  int k_per_split;
  long long c_split_stride;
};

enum { EPI_STORE = 0, EPI_RELU = 1, EPI_MASK = 2, EPI_SPLIT = 3 };

__device__ __forceinline__ int xcd_tile(int bid, int T) {
  const int x = bid & 7;
  const int q = T >> 3, rm = T & 7;
  return (x < rm ? x * (q + 1) : rm * (q + 1) + (x - rm) * q) + (bid >> 3);
}

// LDS images follow the operand's layout in HBM, so every global float4 goes to
// LDS as one ds_write_b128 (no transposing scalar stores):
//   k-contiguous operand (A when !TA, B when TB): image [m][BK + 4] — written and
//     read as b128 fragments of 4 consecutive k (stride 20 words: 2-way conflicts
//     on the b128 reads, accepted so that 5 blocks of 128x80 fit a CU's LDS and the
//     2560 tiles of a 65536 x 400 product run in exactly two rounds);
//   m-contiguous operand (A when TA, B when !TB): image [k][BM + pad], read as
//     ds_read_b32 (pad keeps the two 32-lane groups on disjoint banks).
// With a k-contiguous operand the 16 k of a slab are handed to the 4 MFMA steps as
// k = 4*kr + s (lane group kr owns 4 consecutive k); otherwise k = 4*s + kr.  Each
// output is still one exact f32 fma chain over all K (in a permuted k order).
// Occupancy: the 128 x 80 tiles are held to <= 96 registers (40 accumulators in
// AGPRs) so 5 waves share a SIMD — 5 blocks per CU, and a 65536 x 400 product's
// 2560 tiles fill exactly two rounds of the 256 CUs (at 3 blocks/CU, 3.3 rounds
// left a 17 % tail).
template <int BM, int BN>
struct GemmOcc {
  static constexpr int waves = (BM == 128 && BN <= 80 && DL_GEMM_BK == 16) ? 5 : (BM > 128 ? 3 : 2);
};

// FAST: M % BM == 0, N % BN == 0 and every split's k range whole BK slabs (the tower's
// products: batch rows, 400-wide layers, zero-padded K = leading dims): no bounds checks,
// each thread's staging addresses computed once and advanced by a constant per slab.
template <int BM, int BN, int WM, int WN, bool TA, bool TB, int EPI, int BK, bool FAST>
__global__ __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(GemmOcc<BM, BN>::waves)))
void gemm_f32_kernel(GemmParams p) {
  constexpr int NT = 64 * WM * WN;   // threads: 4 waves, or 5 for the tall dW tiles (WM 1 x WN 5)
  constexpr bool AKC = !TA, BKC = TB, KPERM = AKC || BKC;
  constexpr int KCS = BK == 16 ? BK + 4 : BK + 8;  // BK=16: 2-way b128 read conflicts, but 5 blocks/CU fit
  constexpr int MCPAD_A = KPERM ? (4 - BM % 8 + 8) % 8 : (48 - BM % 32) % 32;
  constexpr int MCPAD_B = KPERM ? (4 - BN % 8 + 8) % 8 : (48 - BN % 32) % 32;
  constexpr int A_ROWS = AKC ? BM : BK, A_LD = AKC ? KCS : BM + MCPAD_A;
  constexpr int B_ROWS = BKC ? BN : BK, B_LD = BKC ? KCS : BN + MCPAD_B;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int QA = (BM * BK / 4 + NT - 1) / NT;  // float4 staged per thread
  constexpr int QB = (BN * BK / 4 + NT - 1) / NT;
  static_assert(WM * WN == 4 || (WM * WN == 5 && !(DL_GEMM_GLDS && !TA)), "4 waves (or 5 without LDS-DMA)");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0 && BK % 16 == 0, "tile shape");

  // GLDS: the k-contiguous A tile is filled by LDS-DMA (global_load_lds_dwordx4), which
  // writes lane-linear 1 KB pieces: the image is unpadded [row][16] and conflict-free
  // b128 reads come from an XOR swizzle of the 16-B chunks, applied on the SOURCE
  // address: slot(row, chunk) = 4*row + (chunk ^ ((row >> 1) & 3)).
  constexpr bool GLDS = DL_GEMM_GLDS && AKC && BK == 16;
  constexpr int A_LD_EFF = GLDS ? BK : A_LD;
  __shared__ __attribute__((aligned(16))) float As[2][A_ROWS][A_LD_EFF];
  __shared__ __attribute__((aligned(16))) float Bs[2][B_ROWS][B_LD];

  const float* __restrict__ A = reinterpret_cast<const float*>(p.A);
  const float* __restrict__ Bm = reinterpret_cast<const float*>(p.B);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_tile(blockIdx.x, ntm * ntn);
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * BN;
  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  floatx4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  float4 ra[QA], rb[QB];

  // FAST staging: buffer loads, SGPR resource + per-thread 32-bit byte offset (fixed) +
  // SGPR slab offset (advanced by a_step / b_step bytes per slab)
  unsigned a_off[QA], b_off[QB];
  const unsigned a_step = TA ? (unsigned)(BK * p.lda * 4) : (unsigned)(BK * 4);
  const unsigned b_step = TB ? (unsigned)(BK * 4) : (unsigned)(BK * p.ldb * 4);
  const float* a_base = A + (TA ? (long long)kbeg * p.lda + i0 : (long long)i0 * p.lda + kbeg);
  const float* b_base = Bm + (TB ? (long long)j0 * p.ldb + kbeg : (long long)kbeg * p.ldb + j0);
  const auto a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a_base, (short)0, 0x7fffffff, 0x00020000);
  const auto b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)b_base, (short)0, 0x7fffffff, 0x00020000);
  if (FAST) {
#pragma unroll
    for (int u = 0; u < QA; ++u) {
      const int qi = min(tid + u * NT, BM * BK / 4 - 1);
      if (TA) a_off[u] = 4u * (unsigned)((qi / (BM / 4)) * p.lda + 4 * (qi % (BM / 4)));
      else a_off[u] = 4u * (unsigned)((qi / (BK / 4)) * p.lda + 4 * (qi % (BK / 4)));
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int qi = min(tid + u * NT, BN * BK / 4 - 1);
      if (!TB) b_off[u] = 4u * (unsigned)((qi / (BN / 4)) * p.ldb + 4 * (qi % (BN / 4)));
      else b_off[u] = 4u * (unsigned)((qi / (BK / 4)) * p.ldb + 4 * (qi % (BK / 4)));
    }
  }
  auto glds_a = [&](int k0, int buf) {
    // 8 pieces of 16 rows for BM = 128: wave w issues pieces w, w + 4, ...
#pragma unroll
    for (int g = wid; g < BM / 16; g += 4) {
      const int row = g * 16 + (lane >> 2);
      const int chunk = (lane & 3) ^ ((row >> 1) & 3);
      int gi = i0 + row;
      gi = gi < p.M ? gi : p.M - 1;                    // rows past M: any valid row (outputs dropped)
      int gr = k0 + 4 * chunk;
      gr = gr < kend ? gr : kend - 4;                  // k past kend: B is zero there
      const float* src = A + (long long)gi * p.lda + gr;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)&As[buf][g * 16][0], 16, 0, 0);
    }
  };
  auto load_tile = [&](int k0) {
    if (FAST) {
      const unsigned ks = (unsigned)((k0 - kbeg) / BK);
      const int sa = (int)(ks * a_step), sb = (int)(ks * b_step);
#pragma unroll
      for (int u = 0; u < (GLDS ? 0 : QA); ++u) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)a_off[u], sa, 0);
        ra[u] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
      }
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(b_rsrc, (int)b_off[u], sb, 0);
        rb[u] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
      }
    } else {
#pragma unroll
    for (int u = 0; u < (GLDS ? 0 : QA); ++u) {
      const int qi = tid + u * NT;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (qi < BM * BK / 4) {
        if (TA) {  // A stored [r][i]
          const int r = qi / (BM / 4), i4 = qi % (BM / 4);
          const int gr = k0 + r, gi = i0 + 4 * i4;
          if (gr < kend && gi < p.M) v = *reinterpret_cast<const float4*>(A + (long long)gr * p.lda + gi);
        } else {   // A stored [i][r]
          const int i = qi / (BK / 4), r4 = qi % (BK / 4);
          const int gi = i0 + i, gr = k0 + 4 * r4;
          if (gi < p.M && gr < kend) v = *reinterpret_cast<const float4*>(A + (long long)gi * p.lda + gr);
        }
      }
      ra[u] = v;
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int qi = tid + u * NT;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (qi < BN * BK / 4) {
        if (!TB) {  // B stored [r][j]
          const int r = qi / (BN / 4), j4 = qi % (BN / 4);
          const int gr = k0 + r, gj = j0 + 4 * j4;
          if (gr < kend && gj < p.N) v = *reinterpret_cast<const float4*>(Bm + (long long)gr * p.ldb + gj);
        } else {    // B stored [j][r]
          const int j = qi / (BK / 4), r4 = qi % (BK / 4);
          const int gj = j0 + j, gr = k0 + 4 * r4;
          if (gj < p.N && gr < kend) v = *reinterpret_cast<const float4*>(Bm + (long long)gj * p.ldb + gr);
        }
      }
      rb[u] = v;
    }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < (GLDS ? 0 : QA); ++u) {
      const int qi = tid + u * NT;
      if (qi < BM * BK / 4) {
        if (TA) {
          const int r = qi / (BM / 4), i4 = qi % (BM / 4);
          *reinterpret_cast<float4*>(&As[buf][r][4 * i4]) = ra[u];
        } else {
          const int i = qi / (BK / 4), r4 = qi % (BK / 4);
          *reinterpret_cast<float4*>(&As[buf][i][4 * r4]) = ra[u];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int qi = tid + u * NT;
      if (qi < BN * BK / 4) {
        if (!TB) {
          const int r = qi / (BN / 4), j4 = qi % (BN / 4);
          *reinterpret_cast<float4*>(&Bs[buf][r][4 * j4]) = rb[u];
        } else {
          const int j = qi / (BK / 4), r4 = qi % (BK / 4);
          *reinterpret_cast<float4*>(&Bs[buf][j][4 * r4]) = rb[u];
        }
      }
    }
  };

  if (nk > 0) {
    if (GLDS) glds_a(kbeg, 0);
    load_tile(kbeg);
    store_tile(0);
    __syncthreads();
  }
  const int kr = lane >> 4, cl = lane & 15;
  // A wave whose rows (or columns) all lie past M (N) still stages and meets the barriers
  // but issues no LDS reads or MFMAs: the ragged last M tile of the dW products (M = 416 /
  // 432 in 128-row tiles) then costs its staging, not four waves of MFMA time.
  const bool live = FAST || (i0 + wm * WTM < p.M && j0 + wn * WTN < p.N);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (GLDS && kt + 1 < nk) glds_a(kbeg + (kt + 1) * BK, cur ^ 1);
    if (kt + 1 < nk) load_tile(kbeg + (kt + 1) * BK);
#pragma unroll
    for (int s16 = 0; s16 < (live ? BK / 16 : 0); ++s16) {
      float4 a4[AKC ? FM : 1], b4[BKC ? FN : 1];
      if (AKC) {
#pragma unroll
        for (int a = 0; a < FM; ++a) {
          if (GLDS)
            a4[a] = *reinterpret_cast<const float4*>(&As[cur][wm * WTM + a * 16 + cl][4 * (kr ^ ((cl >> 1) & 3))]);
          else
            a4[a] = *reinterpret_cast<const float4*>(&As[cur][AKC ? wm * WTM + a * 16 + cl : 0][s16 * 16 + 4 * kr]);
        }
      }
      if (BKC) {
#pragma unroll
        for (int b = 0; b < FN; ++b)
          b4[b] = *reinterpret_cast<const float4*>(&Bs[cur][BKC ? wn * WTN + b * 16 + cl : 0][s16 * 16 + 4 * kr]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = s16 * 16 + (KPERM ? 4 * kr + s : 4 * s + kr);
        float av[FM], bv[FN];
#pragma unroll
        for (int a = 0; a < FM; ++a) {
          if (AKC) av[a] = s == 0 ? a4[a].x : s == 1 ? a4[a].y : s == 2 ? a4[a].z : a4[a].w;
          else av[a] = As[cur][AKC ? 0 : k][wm * WTM + a * 16 + cl];
        }
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          if (BKC) bv[b] = s == 0 ? b4[b].x : s == 1 ? b4[b].y : s == 2 ? b4[b].z : b4[b].w;
          else bv[b] = Bs[cur][BKC ? 0 : k][wn * WTN + b * 16 + cl];
        }
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  float* __restrict__ C = reinterpret_cast<float*>(p.C);
  if (EPI == EPI_SPLIT) C += (long long)blockIdx.z * p.c_split_stride;
  const float* __restrict__ Mk = reinterpret_cast<const float*>(p.mask);
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const int col = j0 + wn * WTN + b * 16 + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = i0 + wm * WTM + a * 16 + kr * 4 + j;
        if (FAST || (row < p.M && col < p.N)) {
          float v = acc[a][b][j];
          if (EPI == EPI_RELU) v = fmaxf(v, 0.f);
          if (EPI == EPI_MASK) v = Mk[(long long)row * p.ldm + col] > 0.f ? v : 0.f;
          C[(long long)row * p.ldc + col] = v;
        }
      }
    }
}

// ---------------------------------------------------------------------------
// bf16 variant (Wide&Deep tower): 16x16x32 bf16 MFMA, K-step 32, fp32 accumulate.
typedef short shortx8 __attribute__((ext_vector_type(8)));


template <int BM, int BN, int WM, int WN, bool TA, bool TB, int EPI, bool CBF16>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmParams p) {
  constexpr int BK = 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  // LDS images: [i][k] and [j][k] with k contiguous (8 bf16 = 16 B per lane read)
  constexpr int SK = BK + 8;  // pad 16 B per row: rows shift banks by 4 words
  __shared__ __attribute__((aligned(16))) unsigned short As[2][BM][SK];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BN][SK];
  const unsigned short* __restrict__ A = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* __restrict__ Bm = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_tile(blockIdx.x, ntm * ntn);
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * BN;
  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;
  floatx4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  // element-wise staging (general transposes); bf16 tower is a secondary path
  auto stage = [&](int buf, int k0) {
    for (int e = tid; e < BM * BK; e += 256) {
      const int i = e / BK, k = e % BK;
      const int gi = i0 + i, gk = k0 + k;
      unsigned short v = 0;
      if (gi < p.M && gk < kend) v = TA ? A[(long long)gk * p.lda + gi] : A[(long long)gi * p.lda + gk];
      As[buf][i][k] = v;
    }
    for (int e = tid; e < BN * BK; e += 256) {
      const int j = e / BK, k = e % BK;
      const int gj = j0 + j, gk = k0 + k;
      unsigned short v = 0;
      if (gj < p.N && gk < kend) v = TB ? Bm[(long long)gj * p.ldb + gk] : Bm[(long long)gk * p.ldb + gj];
      Bs[buf][j][k] = v;
    }
  };
  if (nk > 0) { stage(0, kbeg); __syncthreads(); }
  const int cl = lane & 15, kq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    shortx8 av[FM], bv[FN];
#pragma unroll
    for (int a = 0; a < FM; ++a)
      av[a] = *reinterpret_cast<const shortx8*>(&As[cur][wm * WTM + a * 16 + cl][8 * kq]);
#pragma unroll
    for (int b = 0; b < FN; ++b)
      bv[b] = *reinterpret_cast<const shortx8*>(&Bs[cur][wn * WTN + b * 16 + cl][8 * kq]);
    if (kt + 1 < nk) stage(cur ^ 1, kbeg + (kt + 1) * BK);
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
    __syncthreads();
  }
  const int kr = lane >> 4;
  const long long zoff = (EPI == EPI_SPLIT) ? (long long)blockIdx.z * p.c_split_stride : 0;
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const int col = j0 + wn * WTN + b * 16 + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = i0 + wm * WTM + a * 16 + kr * 4 + j;
        if (row < p.M && col < p.N) {
          float v = acc[a][b][j];
          if (EPI == EPI_RELU) v = fmaxf(v, 0.f);
          if (EPI == EPI_MASK) {
            const unsigned short* mk = reinterpret_cast<const unsigned short*>(p.mask);
            v = bf2f(mk[(long long)row * p.ldm + col]) > 0.f ? v : 0.f;
          }
          const long long o = zoff + (long long)row * p.ldc + col;
          if (CBF16) reinterpret_cast<unsigned short*>(p.C)[o] = f2bf(v);
          else reinterpret_cast<float*>(p.C)[o] = v;
        }
      }
    }
}

// dst[r*ldd + c] = bf16(src[r*lds + c]) (round to nearest even), r < rows, c < cols.
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ src, int rows, int cols, int lds,
                                                        unsigned short* __restrict__ dst, int ldd) {
  const long long n = (long long)rows * cols;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const long long r = k / cols;
    const int c = (int)(k % cols);
    dst[r * ldd + c] = f2bf(src[r * lds + c]);
  }
}

// bf16 GEMM with both operands k-contiguous in HBM (A [i][k], B given as [j][k], i.e.
// ta = 0, tb = 1): the tower's forward (B = W^T copy), dX (B = W) and dW (A = X^T, B = dY^T
// copies) are all put in this form by the engine, so every LDS image is a straight b128
// copy and every MFMA fragment one ds_read_b128: lane (cl, kq) holds A[i = cl][k = 8kq..8kq+7]
// and B[k = 8kq..8kq+7][j = cl] of v_mfma_f32_16x16x32_bf16.  BK = 64 (two MFMA k-steps),
// LDS rows padded to 80 bf16 = 40 words (conflict-free for the b128 lane groups).
template <int BM, int BN, int WM, int WN, int EPI, bool CBF16>
__global__ __launch_bounds__(256) void gemm_bf16_kc_kernel(GemmParams p) {
  constexpr int BK = 64, SK = BK + 16;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int QA = (BM * BK / 8 + 255) / 256, QB = (BN * BK / 8 + 255) / 256;   // uint4 per thread
  static_assert(WM * WN == 4 && WTM % 16 == 0 && WTN % 16 == 0, "tile");
  __shared__ __attribute__((aligned(16))) unsigned short As[2][BM][SK];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BN][SK];
  const unsigned short* __restrict__ A = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* __restrict__ Bm = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_tile(blockIdx.x, ntm * ntn);
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * BN;
  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;
  floatx4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  uint4 ra[QA], rb[QB];
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int u = 0; u < QA; ++u) {
      const int q = tid + u * 256, i = q / (BK / 8), k8 = q % (BK / 8);
      const int gi = i0 + i, gk = k0 + 8 * k8;
      ra[u] = (q < BM * BK / 8 && gi < p.M && gk < kend)
                  ? *reinterpret_cast<const uint4*>(A + (long long)gi * p.lda + gk) : z4;
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int q = tid + u * 256, j = q / (BK / 8), k8 = q % (BK / 8);
      const int gj = j0 + j, gk = k0 + 8 * k8;
      rb[u] = (q < BN * BK / 8 && gj < p.N && gk < kend)
                  ? *reinterpret_cast<const uint4*>(Bm + (long long)gj * p.ldb + gk) : z4;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < QA; ++u) {
      const int q = tid + u * 256;
      if (q < BM * BK / 8) *reinterpret_cast<uint4*>(&As[buf][q / (BK / 8)][8 * (q % (BK / 8))]) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int q = tid + u * 256;
      if (q < BN * BK / 8) *reinterpret_cast<uint4*>(&Bs[buf][q / (BK / 8)][8 * (q % (BK / 8))]) = rb[u];
    }
  };
  if (nk > 0) {
    load_tile(kbeg);
    store_tile(0);
    __syncthreads();
  }
  const int cl = lane & 15, kq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kbeg + (kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      shortx8 av[FM], bv[FN];
#pragma unroll
      for (int a = 0; a < FM; ++a)
        av[a] = *reinterpret_cast<const shortx8*>(&As[cur][wm * WTM + a * 16 + cl][32 * s + 8 * kq]);
#pragma unroll
      for (int b = 0; b < FN; ++b)
        bv[b] = *reinterpret_cast<const shortx8*>(&Bs[cur][wn * WTN + b * 16 + cl][32 * s + 8 * kq]);
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }
  const int kr = lane >> 4;
  const long long zoff = (EPI == EPI_SPLIT) ? (long long)blockIdx.z * p.c_split_stride : 0;
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const int col = j0 + wn * WTN + b * 16 + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = i0 + wm * WTM + a * 16 + kr * 4 + j;
        if (row < p.M && col < p.N) {
          float v = acc[a][b][j];
          if (EPI == EPI_RELU) v = fmaxf(v, 0.f);
          if (EPI == EPI_MASK) {
            const unsigned short* mk = reinterpret_cast<const unsigned short*>(p.mask);
            v = bf2f(mk[(long long)row * p.ldm + col]) > 0.f ? v : 0.f;
          }
          const long long o = zoff + (long long)row * p.ldc + col;
          if (CBF16) reinterpret_cast<unsigned short*>(p.C)[o] = f2bf(v);
          else reinterpret_cast<float*>(p.C)[o] = v;
        }
      }
    }
}

// Tall-skinny bf16 product with the B tile resident in LDS (the C5 tower's forward and dX:
// M = batch rows, N <= 416, K <= 448, both operands k-contiguous).  A block owns 256 rows x
// 80 columns: its whole B slab (80 x K bf16, <= 72 KB) is loaded into LDS once, and each
// of its 8 waves streams its own 32 rows of A straight into MFMA fragments (16 B per lane
// per 32-deep k-chunk; A is read once per column tile, the column tiles of a row tile
// placed on one XCD) with a KC-chunk fully unrolled loop whose loads run DEPTH chunks
// ahead.  The generic kc kernel re-staged both operands every 64-deep step and waited a
// full memory round trip per step (7 steps per tile): 139 us for the 65536 x 400 x 432
// forward; this one is bound by streaming A.
template <int KC, int EPI, bool CBF16>
__global__ __launch_bounds__(512) void gemm_bf16_bres_kernel(GemmParams p) {
  constexpr int BM = 256, BN = 80, NF = BN / 16, DEPTH = 3;
  constexpr int KP = KC * 32 + 8;                 // LDS row pitch (bf16): +16 B keeps b128 reads conflict-free
  extern __shared__ __attribute__((aligned(16))) unsigned short Bs[];   // [BN][KP]
  const unsigned short* __restrict__ A = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* __restrict__ Bm = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_tile(blockIdx.x, ntm * ntn);
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * BN;
  const int cl = lane & 15, kq = lane >> 4;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  // A fragments of this wave: rows r0 + cl and r0 + 16 + cl, k = 32c + 8kq .. +7
  const int r0 = i0 + wid * 32;
  // A through a buffer descriptor (the host checks M * lda * 2 < 2^31): a piece past M or K
  // gets an offset past the range and reads as zeros — no select on a loaded value, which
  // made hipcc wait for each load where it was issued
  const auto a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  const uint32_t o0 = 2u * (uint32_t)(min(r0 + cl, p.M - 1) * p.lda + 8 * kq);
  const uint32_t o1 = 2u * (uint32_t)(min(r0 + 16 + cl, p.M - 1) * p.lda + 8 * kq);
  const bool ok0 = r0 + cl < p.M, ok1 = r0 + 16 + cl < p.M;
  auto lda_ = [&](int c, uint4 (&r)[2]) {
    const bool kin = 32 * c + 8 * kq < p.K;
    r[0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)((ok0 & kin) ? o0 + 64u * c : 0x80000000u), 0, 0));
    r[1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)((ok1 & kin) ? o1 + 64u * c : 0x80000000u), 0, 0));
  };
  uint4 ra[KC][2];
#pragma unroll
  for (int c = 0; c < DEPTH && c < KC; ++c) lda_(c, ra[c]);
  // B slab -> LDS: row j (column j0 + j of the product), k contiguous, zero past N and K
  for (int q = tid; q < BN * KC * 4; q += 512) {
    const int j = q / (KC * 4), k8 = q % (KC * 4);
    const int gj = j0 + j, gk = 8 * k8;
    const uint4 v = (gj < p.N && gk < p.K) ? *reinterpret_cast<const uint4*>(Bm + (long long)gj * p.ldb + gk) : z4;
    *reinterpret_cast<uint4*>(&Bs[j * KP + gk]) = v;
  }
  __syncthreads();
  floatx4 acc[2][NF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[a][f] = floatx4{0.f, 0.f, 0.f, 0.f};
  // every fragment (the slab is zero past N): no per-fragment branch to stop the scheduler
  // from overlapping the next fragment's read with this one's MFMAs
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    if (c + DEPTH < KC) lda_(c + DEPTH, ra[c + DEPTH]);
    const shortx8 av0 = __builtin_bit_cast(shortx8, ra[c][0]);
    const shortx8 av1 = __builtin_bit_cast(shortx8, ra[c][1]);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const shortx8 bv = *reinterpret_cast<const shortx8*>(&Bs[(16 * f + cl) * KP + 32 * c + 8 * kq]);
      acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av0, bv, acc[0][f], 0, 0, 0);
      acc[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av1, bv, acc[1][f], 0, 0, 0);
    }
  }
  // Epilogue through LDS (the B slab is dead now): each wave writes its 32 x 80 tile row-major
  // (element stores from the MFMA layout), then every lane moves whole 16-B row pieces, so the
  // output (and the ReluGrad mask) go to HBM as full row segments instead of 2/4-byte
  // scatters.  f32 output goes in two 16-row halves (32 x 80 x 4 B would not fit beside the
  // other waves' tiles).
  __syncthreads();
  constexpr int ES = CBF16 ? 2 : 4;                 // output element bytes
  constexpr int HR = CBF16 ? 32 : 16;               // rows per pass
  constexpr int TP = BN + (CBF16 ? 8 : 4);          // tile pitch (elements): rows start 16-B aligned
  constexpr int EPP = 16 / ES;                      // elements per 16-B piece
  constexpr int VPR = BN / EPP;                     // pieces per row (10 or 20)
  unsigned char* tile = reinterpret_cast<unsigned char*>(Bs) + (size_t)wid * HR * TP * ES;
  constexpr int NIT = (HR * VPR + 63) / 64;         // pieces per lane per pass
#pragma unroll
  for (int h = 0; h < 32 / HR; ++h) {
    // the ReluGrad mask's pieces of this pass, loaded before the tile's LDS writes: all in
    // flight together instead of one dependent round trip per piece
    uint4 mkr[EPI == EPI_MASK ? NIT : 1];
    if (EPI == EPI_MASK) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = min(lane + 64 * it, HR * VPR - 1);
        const int rl = q / VPR, pc = q % VPR;
        const int row = min(r0 + HR * h + rl, p.M - 1), col = max(0, min(j0 + pc * EPP, p.N - EPP));
        const unsigned short* mk = reinterpret_cast<const unsigned short*>(p.mask) + (long long)row * p.ldm + col;
        if (CBF16) {
          mkr[it] = *reinterpret_cast<const uint4*>(mk);
        } else {
          const uint2 m2 = *reinterpret_cast<const uint2*>(mk);
          mkr[it] = make_uint4(m2.x, m2.y, 0u, 0u);
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (16 * a < HR * h || 16 * a >= HR * (h + 1)) continue;
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = 16 * a + 4 * kq + j - HR * h, cc = 16 * f + cl;
          float v = acc[a][f][j];
          if (EPI == EPI_RELU) v = fmaxf(v, 0.f);
          if (CBF16) reinterpret_cast<unsigned short*>(tile)[rl * TP + cc] = f2bf(v);
          else reinterpret_cast<float*>(tile)[rl * TP + cc] = v;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);             // lgkmcnt(0): this wave's tile writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = lane + 64 * it;
      const int rl = q / VPR, pc = q % VPR;
      const int row = r0 + HR * h + rl, col = j0 + pc * EPP;
      if (q >= HR * VPR || row >= p.M || col >= p.N) continue;
      uint4 v = *reinterpret_cast<const uint4*>(tile + ((size_t)rl * TP * ES + pc * 16));
      const int nv = min(EPP, p.N - col);           // elements of this piece inside N
      if (EPI == EPI_MASK) {
        const unsigned short* mk = reinterpret_cast<const unsigned short*>(p.mask) + (long long)row * p.ldm + col;
        unsigned short mv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (nv == EPP && (reinterpret_cast<uintptr_t>(mk) & (2 * EPP - 1)) == 0) {
          const uint4 m4 = mkr[EPI == EPI_MASK ? it : 0];
          memcpy(mv, &m4, CBF16 ? 16 : 8);
        } else {
          for (int e = 0; e < nv; ++e) mv[e] = mk[e];
        }
        if (CBF16) {
          unsigned short x[8];
          memcpy(x, &v, 16);
          for (int e = 0; e < 8; ++e) x[e] = bf2f(mv[e]) > 0.f ? x[e] : (unsigned short)0;
          memcpy(&v, x, 16);
        } else {
          float x[4];
          memcpy(x, &v, 16);
          for (int e = 0; e < 4; ++e) x[e] = bf2f(mv[e]) > 0.f ? x[e] : 0.f;
          memcpy(&v, x, 16);
        }
      }
      unsigned char* dst = reinterpret_cast<unsigned char*>(p.C) + ((long long)row * p.ldc + col) * ES;
      if (nv == EPP && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        *reinterpret_cast<uint4*>(dst) = v;
      } else {
        unsigned char src[16];
        memcpy(src, &v, 16);
        for (int e = 0; e < nv; ++e) {
          if (CBF16) { unsigned short w; memcpy(&w, src + 2 * e, 2); reinterpret_cast<unsigned short*>(dst)[e] = w; }
          else { float w; memcpy(&w, src + 4 * e, 4); reinterpret_cast<float*>(dst)[e] = w; }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int KC>
static void launch_bf16_bres_kc(const GemmParams& gp, int epi, bool cb, hipStream_t s) {
  const int tiles = (int)(ceil_div(gp.M, 256) * ceil_div(gp.N, 80));
  const size_t lds = (size_t)80 * (KC * 32 + 8) * sizeof(unsigned short);
  const dim3 grid(tiles), block(512);
#define DL_BRES(E_, C_) hipLaunchKernelGGL((gemm_bf16_bres_kernel<KC, E_, C_>), grid, block, lds, s, gp)
  if (epi == EPI_STORE) {
    if (cb) DL_BRES(EPI_STORE, true); else DL_BRES(EPI_STORE, false);
  } else if (epi == EPI_RELU) {
    if (cb) DL_BRES(EPI_RELU, true); else DL_BRES(EPI_RELU, false);
  } else {
    if (cb) DL_BRES(EPI_MASK, true); else DL_BRES(EPI_MASK, false);
  }
#undef DL_BRES
}

// true if the B-resident kernel takes the product (and launches it)
static bool launch_bf16_bres(const GemmParams& gp, int epi, bool cb, hipStream_t s) {
  if (epi == EPI_SPLIT || gp.K <= 0 || gp.K > 448 || gp.K % 8 || gp.lda % 8 || gp.ldb % 8 || gp.M < 256 ||
      (long long)gp.M * gp.lda * 2 >= (1LL << 31))
    return false;
  const int kc = (gp.K + 31) / 32;
  if (kc <= 13) launch_bf16_bres_kc<13>(gp, epi, cb, s);
  else launch_bf16_bres_kc<14>(gp, epi, cb, s);
  return true;
}

// ---------------------------------------------------------------------------
// Tall-skinny bf16 product with the weights streamed through an LDS ring (the C5 tower's
// forward and dX: M = batch rows, both operands k-contiguous bf16).  The structure of the
// s3 NT kernel (gemm_s3.hip) on one plane: block 256 x 208 (8 waves x 32 rows x 13 column
// fragments), A streamed from HBM straight into MFMA fragments (one 16-B load per lane and
// row fragment per 32-deep chunk), each chunk's [208][32] weight image (conflict-free slot
// swizzle) filled by LDS-DMA two chunks ahead into a ring of three.  Against the B-resident
// kernel above (256 x 80 blocks: A fetched once per 80 columns, five times for N = 400) a
// block covers 208 columns, so A is fetched twice; the weight chunks come from L2.
constexpr int kBnBM = 256, kBnBN = 208, kBnNF = 13;
constexpr int kBnPlane = kBnBN * 32;                         // bf16 elements of one chunk image (13,312 B)
constexpr int kBnDma = kBnBN / 16;                           // DMA instructions per chunk (13)
constexpr int kBnDmaW = (kBnDma + 7) / 8;                    // per wave (2; the last clamped)
constexpr int kBnEP = kBnBN + 4;                             // epilogue tile pitch (floats)
constexpr size_t kBnLds = 8 * 16 * kBnEP * sizeof(float);    // the epilogue tiles: 108,544 B
static_assert(3 * kBnPlane * sizeof(unsigned short) <= kBnLds, "the ring fits in the epilogue's LDS");
#ifndef DL_BN_PF
#define DL_BN_PF 4   // weight fragments read this many fragments ahead of their MFMAs
#endif
// DL_BN_ASMA: where each step takes its A chunk.  hipcc counts only its own loads in vmcnt (not
// the weight LDS-DMA, inline asm), and it hoisted the copy of the next step's A registers into
// the current step, where that load is the youngest it knows of: a vmcnt(0) drain in the middle
// of every chunk's MFMAs (the weights two chunks ahead included).  With the copy made by an asm
// statement it stays at its step's start, after the barrier (also asm), where hipcc's wait for
// the chunk's A is vmcnt(2): it lets the next chunk's A loads stay in flight.
#ifndef DL_BN_ASMA
#define DL_BN_ASMA 1
#endif
// DL_BN_WIDE: bf16 output stored as 16-B pieces (two fragments' lane rows exchanged by
// v_permlane16_swap, so a lane holds 8 consecutive columns) instead of 8-B pieces
#ifndef DL_BN_WIDE
#define DL_BN_WIDE 1
#endif
#ifndef DL_BN_NW
#define DL_BN_NW 8   // waves a block of the register-epilogue NT kernel (gemm_bf16_nt_kernel NWV)
#endif
typedef unsigned int bn_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bn_bf16x2 __attribute__((ext_vector_type(2)));
typedef float bn_f32x2 __attribute__((ext_vector_type(2)));
// two f32 -> packed bf16 (v_cvt_pk_bf16_f32: round to nearest even, the same bits as f2bf for
// every non-NaN value; a NaN stays a NaN)
__device__ __forceinline__ unsigned bn_pack2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((bn_f32x2){lo, hi}, bn_bf16x2));
}

__device__ __forceinline__ int bn_slot(int j, int kq) { return kq ^ ((j >> 2) & 2); }   // an involution in kq

// s_waitcnt vmcnt(n) (n < 64), other counters untouched
#define DL_BN_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

// DIRECT: the operands' roles swapped in each MFMA (the weight fragment as src A), so a lane's
// accumulator holds four consecutive columns of one output row, and the epilogue stores them
// straight from registers (8 B of bf16 or 16 B of f32 per lane and fragment; the ReluGrad mask's
// four bf16 read the same way) instead of transposing each wave's tile through LDS (gemm_s3.hip's
// register epilogue).  Needs N, ldc, ldm multiples of 4 (the host picks it then).
// NWV: waves a block (32 rows each; 8 = 256-row blocks, one a CU; 4 = 128-row blocks, three a
// CU at 155 VGPRs — the register epilogue only, its LDS being the 40-KB ring).
template <int EPI, bool CBF16, bool DIRECT = false, int NWV = 8>
__global__ __launch_bounds__(64 * NWV) void gemm_bf16_nt_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [3 bufs][BN][32], then the epilogue
  static_assert(NWV == 8 || DIRECT, "the LDS epilogue's tiles assume 8 waves");
  constexpr int NW = NWV, BM = 32 * NWV, DMAW = (kBnDma + NWV - 1) / NWV;
  const unsigned short* __restrict__ Bm = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + kBnBN - 1) / kBnBN;
  const int t = xcd_tile(blockIdx.x, ntm * ntn);     // the column tiles of a row tile on one XCD: A from L2
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * kBnBN;
  const int cl = lane & 15, kq = lane >> 4;
  const int r0 = i0 + wid * 32;
  const bool ok0 = r0 + cl < p.M, ok1 = r0 + 16 + cl < p.M;
  // A through a buffer descriptor (the host checks M * lda * 2 < 2^31): a piece past M or K
  // gets an offset past the range and reads as zeros (no fixup after a load)
  const uint32_t a_off0 = 2u * (uint32_t)(min(r0 + cl, p.M - 1) * p.lda + 8 * kq);
  const uint32_t a_off1 = 2u * (uint32_t)(min(r0 + 16 + cl, p.M - 1) * p.lda + 8 * kq);
  const auto a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 2, 0x00020000);
  const int KC = (p.K + 31) / 32;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned short*)lds;
  // LDS-DMA of chunk c into buffer `buf`: instruction g fills rows 16g .. 16g + 15; lane L writes
  // slot L & 3 of row L >> 2 and fetches the piece that belongs there.  Rows past N / k past K
  // read clamped in-range data (discarded by the epilogue / multiplied by A's zeros).  Inline
  // asm, as in gemm_s3.hip: a builtin LDS-DMA makes hipcc wait vmcnt(0) before the first use of
  // any A load; every wave issues exactly kBnDmaW instructions, so the counts below are
  // straight-line.
  auto dma_b = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < DMAW; ++i) {
      const int g = min(wid + NW * i, kBnDma - 1);
      const int rb = 16 * g;
      const int j = rb + (lane >> 2);
      const int kpc = bn_slot(j, lane & 3);
      const int gj = min(j0 + j, p.N - 1);
      const int gk = min(32 * c + 8 * kpc, p.K - 8);
      const unsigned short* src = Bm + (long long)gj * p.ldb + gk;
      const uint32_t dst = lds_base + 2u * (uint32_t)(buf * kBnPlane + rb * 32);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst)) : "memory");
    }
  };
  auto load_a = [&](int c, bn_u32x4 (&ra)[2]) {
    const bool kin = 32 * c + 8 * kq < p.K;
    const uint32_t o0 = (ok0 & kin) ? a_off0 + 64u * c : 0x80000000u;
    const uint32_t o1 = (ok1 & kin) ? a_off1 + 64u * c : 0x80000000u;
    ra[0] = __builtin_bit_cast(bn_u32x4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)o0, 0, 0));
    ra[1] = __builtin_bit_cast(bn_u32x4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)o1, 0, 0));
  };
  floatx4 acc[2][kBnNF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int f = 0; f < kBnNF; ++f) acc[a][f] = floatx4{0.f, 0.f, 0.f, 0.f};
  bn_u32x4 raA[2], raB[2];
  // every step issues chunk c + 2's weight DMA (DMAW instructions) and then its A loads (2): the
  // vector-memory queue of a wave is ... DMA(c+1) A(c+1) | DMA(c+2) A(c+2)
  dma_b(0, 0);
  load_a(0, raA);
  dma_b(1, 1);     // unconditional, like every prefetch below: chunks past KC read clamped
  load_a(1, raB);  // weights into a free buffer and zeros for A
  // chunk c + 1's weights -> every wave: wait for this wave's DMA(c+1) (younger: A(c+1),
  // DMA(c+2), A(c+2)), then a bare s_barrier (a __syncthreads would drain the prefetch: vmcnt(0))
  auto publish = [&](int c) {
    if (DL_BN_ASMA) {   // as asm: it keeps its place among the DMA and the A copies
      if (c + 1 < KC) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(DMAW + 4) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      return;
    }
    if (c + 1 < KC) DL_BN_VMCNT(DMAW + 2);
    else DL_BN_VMCNT(0);                  // nothing may still land after the loop
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();
  };
  publish(-1);
  auto step = [&](int c, bn_u32x4 (&ra)[2]) {
    shortx8 a0, a1;
    if (DL_BN_ASMA) {   // chunk c's A copied here (hipcc waits for its loads right before)
      bn_u32x4 x0, x1;
      asm volatile("" : "=v"(x0), "=v"(x1) : "0"(ra[0]), "1"(ra[1]));
      a0 = __builtin_bit_cast(shortx8, x0);
      a1 = __builtin_bit_cast(shortx8, x1);
    } else {
      a0 = __builtin_bit_cast(shortx8, ra[0]);
      a1 = __builtin_bit_cast(shortx8, ra[1]);
    }
    // chunk c's A in registers of their own before the next batch reuses ra
    asm volatile("" : "+v"(a0), "+v"(a1));
    dma_b(c + 2, (c + 2) % 3);
    load_a(c + 2, ra);
    const unsigned short* Bs = lds + (c % 3) * kBnPlane + cl * 32 + 8 * bn_slot(cl, kq);
    constexpr int PF = DL_BN_PF, NB = PF + 1;
    shortx8 bb[NB];
#pragma unroll
    for (int i = 0; i < PF; ++i) bb[i] = *reinterpret_cast<const shortx8*>(Bs + 512 * i);   // fragment rows 16i + cl
#pragma unroll
    for (int f = 0; f < kBnNF; ++f) {
      if (f + PF < kBnNF) bb[(f + PF) % NB] = *reinterpret_cast<const shortx8*>(Bs + 512 * (f + PF));
      const shortx8 bv = bb[f % NB];
      if (DIRECT) {
        acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, a0, acc[0][f], 0, 0, 0);
        acc[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, a1, acc[1][f], 0, 0, 0);
      } else {
        acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bv, acc[0][f], 0, 0, 0);
        acc[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bv, acc[1][f], 0, 0, 0);
      }
    }
    publish(c);
  };
  int c = 0;
  for (; c + 1 < KC; c += 2) {
    step(c, raA);
    step(c + 1, raB);
  }
  if (c < KC) step(c, raA);

  if constexpr (DIRECT) {
    // lane (kq, cl): acc[a][f][j] = C[r0 + 16a + cl][j0 + 16f + 4kq + j]; stores and mask loads
    // through buffer descriptors (pieces past M or N: offsets past the range, dropped / zeros)
    constexpr int EB = CBF16 ? 2 : 4;
    const auto c_rsrc = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, p.M * p.ldc * EB, 0x00020000);
    const auto m_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.mask, (short)0,
                                                          EPI == EPI_MASK ? p.M * p.ldm * 2 : 0, 0x00020000);
    // 16-B bf16 pieces need N, ldc multiples of 8 (the swapped lane holds 8 columns)
    const bool wide = CBF16 && DL_BN_WIDE && p.N % 8 == 0 && p.ldc % 8 == 0;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int row = r0 + 16 * a + cl;
      unsigned plo = 0u, phi = 0u;   // the even fragment's packed words, until its pair's swap
      // the ReluGrad mask's pieces of these 13 fragments first, all in flight together
      uint2 mk[EPI == EPI_MASK ? kBnNF : 1];
      if constexpr (EPI == EPI_MASK) {
#pragma unroll
        for (int f = 0; f < kBnNF; ++f) {
          const int col = j0 + 16 * f + 4 * kq;
          const uint32_t off = (row < p.M && col + 4 <= p.N) ? 2u * (uint32_t)(row * p.ldm + col) : 0x80000000u;
          mk[f] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(m_rsrc, (int)off, 0, 0));
        }
      }
#pragma unroll
      for (int f = 0; f < kBnNF; ++f) {
        const int col = j0 + 16 * f + 4 * kq;
        float x[4] = {acc[a][f][0], acc[a][f][1], acc[a][f][2], acc[a][f][3]};
        if (EPI == EPI_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
        }
        if constexpr (EPI == EPI_MASK) {
          const unsigned short mv[4] = {(unsigned short)(mk[f].x & 0xffffu), (unsigned short)(mk[f].x >> 16),
                                        (unsigned short)(mk[f].y & 0xffffu), (unsigned short)(mk[f].y >> 16)};
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = bf2f(mv[e]) > 0.f ? x[e] : 0.f;
        }
        if (CBF16 && wide) {
          // fragment pairs (f, f + 1): v_permlane16_swap exchanges lane rows kq = 1, 3 of f's
          // two packed words with rows kq = 0, 2 of f + 1's, so an even-kq lane holds f's columns
          // 4kq .. 4kq + 7 and an odd-kq lane f + 1's columns 4(kq - 1) .. 4kq + 3: one 16-B
          // store each (64 contiguous bytes of a row per lane-row quad) instead of two 8-B ones
          const unsigned lo = bn_pack2(x[0], x[1]), hi = bn_pack2(x[2], x[3]);
          if ((f & 1) == 0 && f + 1 < kBnNF) {
            plo = lo;
            phi = hi;
            continue;
          }
          if (f & 1) {
            const auto sl = __builtin_amdgcn_permlane16_swap(plo, lo, false, false);
            const auto sh = __builtin_amdgcn_permlane16_swap(phi, hi, false, false);
            const int c8 = (kq & 1) ? j0 + 16 * f + 4 * (kq - 1) : j0 + 16 * (f - 1) + 4 * kq;
            const bool ok = row < p.M && c8 + 8 <= p.N;
            const uint32_t off = ok ? 2u * (uint32_t)(row * p.ldc + c8) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dl_u32x4_t, make_uint4(sl[0], sh[0], sl[1], sh[1])),
                                                   c_rsrc, (int)off, 0, 0);
            continue;
          }
          // the odd fragment left over (kBnNF = 13): its 8-B pieces
          const bool ok = row < p.M && col + 4 <= p.N;
          const uint32_t off = ok ? 2u * (uint32_t)(row * p.ldc + col) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(dl_u32x2_t, make_uint2(lo, hi)), c_rsrc, (int)off, 0,
                                                0);
          continue;
        }
        const bool ok = row < p.M && col + 4 <= p.N;
        const uint32_t off = ok ? (uint32_t)EB * (uint32_t)(row * p.ldc + col) : 0x80000000u;
        if (CBF16)
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(dl_u32x2_t, make_uint2(bn_pack2(x[0], x[1]), bn_pack2(x[2], x[3]))), c_rsrc,
              (int)off, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dl_u32x4_t, make_float4(x[0], x[1], x[2], x[3])),
                                                 c_rsrc, (int)off, 0, 0);
      }
    }
    return;
  }
  // Epilogue through LDS (free after the last barrier): per wave and half (rows 16h .. 16h + 15
  // of its 32) the 16 x 208 f32 tile is written from the MFMA layout, then each lane moves
  // whole row pieces (8 bf16 or 4 f32 = 16 B), ReLU / ReluGrad mask applied there.
  float* tile = reinterpret_cast<float*>(lds) + wid * 16 * kBnEP;
  const unsigned short* __restrict__ Mk = reinterpret_cast<const unsigned short*>(p.mask);
  constexpr int EPP = CBF16 ? 8 : 4;                // output elements per 16-B piece
  constexpr int VPR = kBnBN / EPP;                  // pieces per row (26 or 52)
  constexpr int NIT = (16 * VPR + 63) / 64;         // pieces per lane per half
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // the mask's pieces of this half first (all in flight together, under the tile writes)
    uint4 mk4[EPI == EPI_MASK ? NIT : 1];
    if (EPI == EPI_MASK) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = min(lane + 64 * it, 16 * VPR - 1);
        const int rl = q / VPR, pc = q % VPR;
        const int row = min(r0 + 16 * h + rl, p.M - 1), col = max(0, min(j0 + EPP * pc, p.N - EPP));
        const unsigned short* mk = Mk + (long long)row * p.ldm + col;
        if (CBF16) {
          mk4[it] = *reinterpret_cast<const uint4*>(mk);
        } else {
          const uint2 m2 = *reinterpret_cast<const uint2*>(mk);
          mk4[it] = make_uint4(m2.x, m2.y, 0u, 0u);
        }
      }
    }
#pragma unroll
    for (int f = 0; f < kBnNF; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[(4 * kq + j) * kBnEP + 16 * f + cl] = acc[h][f][j];
    __builtin_amdgcn_s_waitcnt(0xc07f);             // lgkmcnt(0): this wave's tile writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = lane + 64 * it;
      const int rl = q / VPR, pc = q % VPR;
      const int row = r0 + 16 * h + rl, col = j0 + EPP * pc;
      if (q >= 16 * VPR || row >= p.M || col >= p.N) continue;
      float x[8];
      const float4 v0 = *reinterpret_cast<const float4*>(tile + rl * kBnEP + EPP * pc);
      x[0] = v0.x; x[1] = v0.y; x[2] = v0.z; x[3] = v0.w;
      if (CBF16) {
        const float4 v1 = *reinterpret_cast<const float4*>(tile + rl * kBnEP + EPP * pc + 4);
        x[4] = v1.x; x[5] = v1.y; x[6] = v1.z; x[7] = v1.w;
      }
      const int nv = min(EPP, p.N - col);
      const unsigned short* mk = Mk + (long long)row * p.ldm + col;
      const bool whole_mask = EPI == EPI_MASK && nv == EPP && (reinterpret_cast<uintptr_t>(mk) & (2 * EPP - 1)) == 0;
      unsigned short mv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (EPI == EPI_MASK) {
        if (whole_mask) memcpy(mv, &mk4[EPI == EPI_MASK ? it : 0], 2 * EPP);
        else for (int e = 0; e < nv; ++e) mv[e] = mk[e];
      }
#pragma unroll
      for (int e = 0; e < EPP; ++e) {
        if (EPI == EPI_RELU) x[e] = fmaxf(x[e], 0.f);
        if (EPI == EPI_MASK) x[e] = bf2f(mv[e]) > 0.f ? x[e] : 0.f;
      }
      unsigned char* dst = reinterpret_cast<unsigned char*>(p.C) + ((long long)row * p.ldc + col) * (CBF16 ? 2 : 4);
      if (nv == EPP && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        if (CBF16)
          *reinterpret_cast<uint4*>(dst) = make_uint4(f2bf(x[0]) | ((unsigned)f2bf(x[1]) << 16),
                                                      f2bf(x[2]) | ((unsigned)f2bf(x[3]) << 16),
                                                      f2bf(x[4]) | ((unsigned)f2bf(x[5]) << 16),
                                                      f2bf(x[6]) | ((unsigned)f2bf(x[7]) << 16));
        else
          *reinterpret_cast<float4*>(dst) = make_float4(x[0], x[1], x[2], x[3]);
      } else {
        for (int e = 0; e < nv; ++e) {
          if (CBF16) reinterpret_cast<unsigned short*>(dst)[e] = f2bf(x[e]);
          else reinterpret_cast<float*>(dst)[e] = x[e];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

#ifndef DL_BF16_NT
#define DL_BF16_NT 1   // forward / dX products on gemm_bf16_nt_kernel (0: the B-resident kernel)
#endif

// DL_BF16_DIRECT=0 in the environment: the LDS epilogue (A/B measurements)
static bool bf16_direct_enabled() {
  static const bool on = [] {
    const char* e = getenv("DL_BF16_DIRECT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// true if the streamed-weight kernel takes the product (and launches it)
static bool launch_bf16_nt(const GemmParams& gp, int epi, bool cb, hipStream_t s) {
  if (!DL_BF16_NT || epi == EPI_SPLIT || gp.K < 8 || gp.K % 8 || gp.lda % 8 || gp.ldb % 8 || gp.lda < gp.K ||
      gp.ldb < gp.K || (epi == EPI_MASK && gp.ldm % 8) || (reinterpret_cast<uintptr_t>(gp.A) & 15) ||
      (reinterpret_cast<uintptr_t>(gp.B) & 15) || (long long)gp.M * gp.lda * 2 >= (1LL << 31))
    return false;
  const bool direct = bf16_direct_enabled() && gp.N % 4 == 0 && gp.ldc % 4 == 0 &&
                      (epi != EPI_MASK || gp.ldm % 4 == 0) && (long long)gp.M * gp.ldc * 4 < (1LL << 31);
  constexpr int NWD = DL_BN_NW;   // waves a block of the register-epilogue kernel
  const dim3 grid((unsigned)(ceil_div(gp.M, direct ? 32 * NWD : kBnBM) * ceil_div(gp.N, kBnBN))),
      block(direct ? 64 * NWD : 512);
  // the register epilogue needs only the ring (39,936 B instead of the 108,544-B tiles), so other
  // kernels' blocks (the side stream's index build) can share the CU
  constexpr size_t ring = 3 * kBnPlane * sizeof(unsigned short);
#define DL_BNT(E_, C_)                                                                                     \
  do {                                                                                                     \
    if (direct) hipLaunchKernelGGL((gemm_bf16_nt_kernel<E_, C_, true, NWD>), grid, block, ring, s, gp);   \
    else hipLaunchKernelGGL((gemm_bf16_nt_kernel<E_, C_>), grid, block, kBnLds, s, gp);                    \
  } while (0)
  if (epi == EPI_STORE) {
    if (cb) DL_BNT(EPI_STORE, true); else DL_BNT(EPI_STORE, false);
  } else if (epi == EPI_RELU) {
    if (cb) DL_BNT(EPI_RELU, true); else DL_BNT(EPI_RELU, false);
  } else {
    if (cb) DL_BNT(EPI_MASK, true); else DL_BNT(EPI_MASK, false);
  }
#undef DL_BNT
  return true;
}

// Weight gradients of the bf16 tower without transposed operand copies (ta = 1, tb = 0,
// split-K slabs): slab z of C = sum over the batch rows k of split z of X[k][m] dY[k][n], with
// X [K][lda] bf16 (m contiguous: the activations as the forward wrote them) and dY [K][ldb]
// (n contiguous: the layer's output gradient).  32 batch rows of each are copied into LDS as
// plain rows and read as MFMA fragments with ds_read_b64_tr_b16 (CDNA4's transposing LDS
// read): lane group kq takes batch rows 4kq..4kq+3 and 16+4kq..16+4kq+3 of the step for both
// operands (the same k set, so the product is unchanged), and row pitches of 8 x odd words
// make every transposed read conflict-free.  Block: 5 waves, 64 rows (m) x 400 columns (n);
// wave w owns columns 80w..80w+79 (4 x 5 fragments).  The m tiles of one split are
// consecutive tiles of the XCD-aware order: dY's slice comes from HBM once, then from L2.
typedef __attribute__((__vector_size__(4 * sizeof(__fp16)))) __fp16 dl_fp16x4_t;

__device__ __forceinline__ uint2 lds_tr16(const unsigned short* ptr_) {
  auto lp = (__attribute__((address_space(3))) unsigned short*)(const_cast<unsigned short*>(ptr_));
  const dl_fp16x4_t v =
      __builtin_amdgcn_ds_read_tr16_b64_v4f16(reinterpret_cast<__attribute__((address_space(3))) dl_fp16x4_t*>(lp));
  return __builtin_bit_cast(uint2, v);
}

__global__ __launch_bounds__(320) void gemm_bf16_dw_kernel(GemmParams p) {
  constexpr int BM = 64, BN = 400, NT = 320, KS = 32;
  constexpr int PA = 80, PB = 400;                      // row pitches: 40 and 200 words = 8 x odd
  constexpr int A_EL = KS * PA, B_EL = KS * PB;         // elements per buffer
  constexpr int QA_N = KS * BM / 8, QB_N = KS * BN / 8; // 16-B pieces per step
  constexpr int Q = (QA_N + QB_N + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * (A_EL + B_EL)];
  const unsigned short* __restrict__ X = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* __restrict__ Y = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mtiles = (p.M + BM - 1) / BM;
  const int t = xcd_tile(blockIdx.x, gridDim.x);
  const int m0 = (t % mtiles) * BM, z = t / mtiles;
  const int kbeg = z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + KS - 1) / KS;
  // both operands through buffer descriptors (the host checks K * ld * 2 < 2^31): a piece
  // past K, M or N gets an offset past the range and reads as zeros, so every load is issued
  // unconditionally (a branch around each load made hipcc wait for it in place)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.K * p.lda * 2, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.K * p.ldb * 2, 0x00020000);
  uint4 rs[Q];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const int q = tid + u * NT;
      if (q < QA_N) {   // (u, tid) ranges: wave-uniform for this mapping except at the boundary
        const int r = q / (BM / 8), c8 = q % (BM / 8);
        const int gk = k0 + r, gm = m0 + 8 * c8;
        const uint32_t o = 2u * (uint32_t)(gk * p.lda + gm);
        rs[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                              xr, (int)(((gk < kend) & (gm < p.M)) ? o : 0x80000000u), 0, 0));
      } else {
        const int qq = q - QA_N, r = qq / (BN / 8), c8 = qq % (BN / 8);
        const int gk = k0 + r, gn = 8 * c8;
        const uint32_t o = 2u * (uint32_t)(gk * p.ldb + gn);
        const bool ok = (q < QA_N + QB_N) & (gk < kend) & (gn < p.N);
        rs[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, (int)(ok ? o : 0x80000000u), 0, 0));
      }
    }
  };
  auto store = [&](int buf) {
    unsigned short* As = lds + buf * (A_EL + B_EL);
    unsigned short* Bs = As + A_EL;
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const int q = tid + u * NT;
      if (q < QA_N) {
        const int r = q / (BM / 8), c8 = q % (BM / 8);
        *reinterpret_cast<uint4*>(&As[r * PA + 8 * c8]) = rs[u];
      } else if (q < QA_N + QB_N) {
        const int qq = q - QA_N, r = qq / (BN / 8), c8 = qq % (BN / 8);
        *reinterpret_cast<uint4*>(&Bs[r * PB + 8 * c8]) = rs[u];
      }
    }
  };
  floatx4 acc[4][5];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    load(kbeg);
    store(0);
    __syncthreads();
  }
  const int cl = lane & 15, kq = lane >> 4, rq = cl >> 2, cp = cl & 3;
  const int ra = 4 * kq + rq, rb = 16 + 4 * kq + rq;   // this lane's rows of the two transposed reads
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load(kbeg + (kt + 1) * KS);
    const unsigned short* As = lds + cur * (A_EL + B_EL);
    const unsigned short* Bs = As + A_EL;
    shortx8 af[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const uint2 lo = lds_tr16(&As[ra * PA + 16 * a + 4 * cp]);
      const uint2 hi = lds_tr16(&As[rb * PA + 16 * a + 4 * cp]);
      af[a] = __builtin_bit_cast(shortx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const int c0 = 80 * wid + 16 * b + 4 * cp;
      const uint2 lo = lds_tr16(&Bs[ra * PB + c0]);
      const uint2 hi = lds_tr16(&Bs[rb * PB + c0]);
      const shortx8 bf = __builtin_bit_cast(shortx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf, acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  float* __restrict__ C = reinterpret_cast<float*>(p.C) + (long long)z * p.c_split_stride;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const int col = 80 * wid + 16 * b + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + 16 * a + 4 * kq + j;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] = acc[a][b][j];
      }
    }
}

// The same weight gradients with a deeper pipeline and fewer operand re-reads: block 144 (m) x
// 400 (n) — three m tiles for the tower's M = 416 / 432, so each dY slice is read three times
// (from L2) instead of seven — and 15 waves (3 m groups of 48 rows x 5 n groups of 80 columns,
// 3 x 5 fragments each).  Per 32-deep batch step the X [32][144] and dY [32][400] bf16 rows land
// in LDS by LDS-DMA (global_load_lds_dwordx4, 34 one-KB instructions per step) into a ring of four
// stages issued three steps ahead, so a step waits on no memory round trip (the two-buffer kernel
// above, with its register-staged next step, paid one per 32 rows: 77 us for a C5 layer).  The
// images are the operands' plain rows (pitches 144 and 400 bf16 = 8 x odd words: conflict-free
// transposed reads, as above), so every DMA lane moves one 16-B piece of one row.  Needs whole
// 32-row steps in every split (K % 32 == 0; the split size is a multiple of 64); pieces past M
// or N read clamped in-range data whose products only reach discarded outputs.
constexpr int kD3BM = 144, kD3BN = 400, kD3KS = 32, kD3R = 4, kD3W = 15;
constexpr int kD3AB = kD3KS * kD3BM * 2, kD3BB = kD3KS * kD3BN * 2;   // image bytes per stage
constexpr int kD3SB = kD3AB + kD3BB;                                   // 34,816 B
constexpr int kD3DA = kD3AB / 1024, kD3D = kD3DA + kD3BB / 1024;      // 9 + 25 DMA instructions
constexpr size_t kD3Lds = (size_t)kD3R * kD3SB;                        // 139,264 B
static_assert(kD3AB % 1024 == 0 && kD3BB % 1024 == 0 && kD3D == 34, "whole DMA instructions per image");
static_assert(kD3D <= 3 * kD3W, "at most three DMA instructions per wave and step");
#ifndef DL_BF16_DW3
#define DL_BF16_DW3 1   // 0: the two-buffer kernel above for every weight gradient
#endif

__global__ __launch_bounds__(960) void gemm_bf16_dw3_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [R stages][A image | B image]
  const unsigned short* __restrict__ X = reinterpret_cast<const unsigned short*>(p.A);
  const unsigned short* __restrict__ Y = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (p.M + kD3BM - 1) / kD3BM;
  const int t = xcd_tile(blockIdx.x, gridDim.x);   // the m tiles of one split adjacent: dY's slice shared in L2
  const int m0 = (t % mtiles) * kD3BM, z = t / mtiles;
  const int kbeg = z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg) / kD3KS;            // whole steps (the host checks K % 32 == 0)
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned short*)lds;
  // This wave's DMA instructions (wave-uniform): waves 0-3 issue three per step, the others two
  // (34 = 4 x 3 + 11 x 2).  Instruction g < 9 fills A image bytes 1024 g .. +1023 (row o / 288,
  // piece (o % 288) / 16), g >= 9 the B image's (row o / 800, piece (o % 800) / 16).  The source
  // row and piece of this lane are fixed per instruction; a step adds 32 rows.
  const int ndma = wid < 4 ? 3 : 2;
  const unsigned short* src[3];
  uint32_t dst[3];
  int ld[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int g = wid < 4 ? 3 * wid + i : 12 + 2 * (wid - 4) + min(i, 1);
    if (g < kD3DA) {
      const int o = 1024 * g + 16 * lane, r = o / (2 * kD3BM), m = m0 + ((o % (2 * kD3BM)) >> 1);
      src[i] = X + (long long)(kbeg + r) * p.lda + (m < p.M ? m : 0);
      dst[i] = 1024u * g;
      ld[i] = p.lda;
    } else {
      const int o = 1024 * (g - kD3DA) + 16 * lane, r = o / (2 * kD3BN), n = (o % (2 * kD3BN)) >> 1;
      src[i] = Y + (long long)(kbeg + r) * p.ldb + (n < p.N ? n : 0);
      dst[i] = (uint32_t)kD3AB + 1024u * (g - kD3DA);
      ld[i] = p.ldb;
    }
  }
  // step c's rows into stage c % R; steps past this split's range re-read its last step (the
  // stage is never computed on), so every wave issues the same count every step
  auto dma = [&](int c) {
    const long long dk = (long long)min(c, nk - 1) * kD3KS;
    const uint32_t sb = lds_base + (uint32_t)((c % kD3R) * kD3SB);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < ndma) {
        const unsigned short* sp = src[i] + dk * ld[i];
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(sp), "s"(__builtin_amdgcn_readfirstlane(sb + dst[i])) : "memory");
      }
    }
  };
  floatx4 acc[3][5];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int wm = wid / 5, wn = wid % 5;
  const int cl = lane & 15, kq = lane >> 4, rq = cl >> 2, cp = cl & 3;
  const int ra = 4 * kq + rq, rb = 16 + 4 * kq + rq;   // this lane's rows of the two transposed reads
  if (nk > 0) {
#pragma unroll
    for (int c = 0; c < kD3R - 1; ++c) dma(c);
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMA of step kt has landed once only the younger R - 2 steps' are in flight;
      // then the barrier publishes every wave's (a bare s_barrier: __syncthreads' fence would
      // wait for the whole prefetch)
      if (ndma == 3) DL_BN_VMCNT(3 * (kD3R - 2));
      else DL_BN_VMCNT(2 * (kD3R - 2));
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's reads of step kt - 1 are done
      __builtin_amdgcn_s_barrier();
      dma(kt + kD3R - 1);                   // into the stage step kt - 1 used
      const unsigned short* As = lds + (kt % kD3R) * (kD3SB / 2);
      const unsigned short* Bs = As + kD3AB / 2;
      shortx8 af[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int col = 48 * wm + 16 * a + 4 * cp;
        const uint2 lo = lds_tr16(&As[ra * kD3BM + col]);
        const uint2 hi = lds_tr16(&As[rb * kD3BM + col]);
        af[a] = __builtin_bit_cast(shortx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
#pragma unroll
      for (int b = 0; b < 5; ++b) {
        const int col = 80 * wn + 16 * b + 4 * cp;
        const uint2 lo = lds_tr16(&Bs[ra * kD3BN + col]);
        const uint2 hi = lds_tr16(&Bs[rb * kD3BN + col]);
        const shortx8 bf = __builtin_bit_cast(shortx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
#pragma unroll
        for (int a = 0; a < 3; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf, acc[a][b], 0, 0, 0);
      }
    }
    DL_BN_VMCNT(0);   // the trailing DMAs land before the workgroup's LDS is released
  }
  float* __restrict__ C = reinterpret_cast<float*>(p.C) + (long long)z * p.c_split_stride;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const int col = 80 * wn + 16 * b + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + 48 * wm + 16 * a + 4 * kq + j;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] = acc[a][b][j];
      }
    }
}

// true if the transposed-read kernel takes the product (ta = 1, tb = 0, split slabs)
static bool launch_bf16_dw(const GemmParams& gp0, int splits_req, hipStream_t s) {
  if (gp0.N > 400 || gp0.N % 8 || gp0.M % 8 || gp0.lda % 8 || gp0.ldb % 8 || gp0.lda < gp0.M ||
      gp0.ldb < gp0.N || (reinterpret_cast<uintptr_t>(gp0.A) & 15) || (reinterpret_cast<uintptr_t>(gp0.B) & 15) ||
      (long long)gp0.K * gp0.lda * 2 >= (1LL << 31) || (long long)gp0.K * gp0.ldb * 2 >= (1LL << 31))
    return false;
  GemmParams gp = gp0;
  int kps = (int)ceil_div(gp.K > 0 ? gp.K : 1, splits_req);
  kps = (kps + 63) / 64 * 64;                 // the engine sums ceil(K / kps) slabs at this rounding
  gp.k_per_split = kps;
  const int splits = (int)ceil_div(gp.K > 0 ? gp.K : 1, kps);
  if (DL_BF16_DW3 && gp.K % kD3KS == 0) {
    const int mtiles = (int)ceil_div(gp.M, kD3BM);
    hipLaunchKernelGGL(gemm_bf16_dw3_kernel, dim3((unsigned)(mtiles * splits)), dim3(64 * kD3W), kD3Lds, s, gp);
    return true;
  }
  const int mtiles = (int)ceil_div(gp.M, 64);
  hipLaunchKernelGGL(gemm_bf16_dw_kernel, dim3((unsigned)(mtiles * splits)), dim3(320), 0, s, gp);
  return true;
}

// dst[c*ldd + r] = bf16(src[r*lds + c]) through a 32x33 LDS tile; src f32 or bf16.
template <bool SRC_F32>
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const void* __restrict__ src, int rows, int cols, int lds,
                                                             unsigned short* __restrict__ dst, int ldd) {
  __shared__ unsigned short t[32][34];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    unsigned short v = 0;
    if (r < rows && c < cols) {
      const long long o = (long long)r * lds + c;
      v = SRC_F32 ? f2bf(reinterpret_cast<const float*>(src)[o]) : reinterpret_cast<const unsigned short*>(src)[o];
    }
    t[y][tx] = v;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < cols && r < rows) dst[(long long)c * ldd + r] = t[tx][y];
  }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool FAST>
static void launch_f32_v(const GemmParams& gp, int epi, dim3 grid, hipStream_t s) {
  constexpr int BK = DL_GEMM_BK;
  constexpr int NT = 64 * WM * WN;
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, TA, TB, EPI_STORE, BK, FAST>), grid, dim3(NT), 0, s, gp); break;
    case EPI_RELU: hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, TA, TB, EPI_RELU, BK, FAST>), grid, dim3(NT), 0, s, gp); break;
    case EPI_MASK: hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, TA, TB, EPI_MASK, BK, FAST>), grid, dim3(NT), 0, s, gp); break;
    default: hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, TA, TB, EPI_SPLIT, BK, FAST>), grid, dim3(NT), 0, s, gp); break;
  }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB>
static void launch_f32(const GemmParams& gp, int epi, int splits, hipStream_t s) {
  constexpr int BK = DL_GEMM_BK;
  const int tiles = (int)(ceil_div(gp.M, BM) * ceil_div(gp.N, BN));
  dim3 grid(tiles, 1, splits);
  const bool fast = gp.M % BM == 0 && gp.N % BN == 0 && gp.K % BK == 0 && gp.k_per_split % BK == 0 && !DL_GEMM_GLDS;
  if (fast) launch_f32_v<BM, BN, WM, WN, TA, TB, true>(gp, epi, grid, s);
  else launch_f32_v<BM, BN, WM, WN, TA, TB, false>(gp, epi, grid, s);
}

template <bool TA, bool TB>
static void dispatch_bn_f32(const GemmParams& gp, int epi, int splits, hipStream_t s) {
  // Weight gradients (split-K slabs of x^T dh: M = K_in + bias row padded to 16, N = 400):
  // the 128-row tiles leave a ragged last tile (432 -> 512 rows).  Tall 144 x 80 tiles
  // (9 fragments, 5 waves of 16 columns) divide M = 432 exactly: C2's layer-0 dW 229 ->
  // 215 us.  (208-row tiles for M = 416 measured slower than the 128-row tiles with the
  // wave skip — 233-248 vs 229 us — and are not used.)
  if (epi == EPI_SPLIT && gp.N % 80 == 0 && gp.K >= 4096 && gp.M % 144 == 0 && gp.M % 128 != 0) {
    launch_f32<144, 80, 1, 5, TA, TB>(gp, epi, splits, s);
    return;
  }
  // pick the N tile with the least padding (ties -> wider tile)
  const int cand[4] = {208, 128, 80, 64};
  int best = 64;
  long long bestpad = 1LL << 60;
  for (int c : cand) {
    const long long pad = ceil_div(gp.N, c) * c;
    if (pad < bestpad) { bestpad = pad; best = c; }
  }
  switch (best) {
    case 208: launch_f32<128, 208, 4, 1, TA, TB>(gp, epi, splits, s); break;
    case 128: launch_f32<128, 128, 2, 2, TA, TB>(gp, epi, splits, s); break;
    case 80: launch_f32<128, 80, 4, 1, TA, TB>(gp, epi, splits, s); break;
    default: launch_f32<128, 64, 4, 1, TA, TB>(gp, epi, splits, s); break;
  }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool CB>
static void launch_bf16(const GemmParams& gp, int epi, int splits, hipStream_t s) {
  const int tiles = (int)(ceil_div(gp.M, BM) * ceil_div(gp.N, BN));
  dim3 grid(tiles, 1, splits);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, TA, TB, EPI_STORE, CB>), grid, dim3(256), 0, s, gp); break;
    case EPI_RELU: hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, TA, TB, EPI_RELU, CB>), grid, dim3(256), 0, s, gp); break;
    case EPI_MASK: hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, TA, TB, EPI_MASK, CB>), grid, dim3(256), 0, s, gp); break;
    default: hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, TA, TB, EPI_SPLIT, false>), grid, dim3(256), 0, s, gp); break;
  }
}

// dst[c][r] = src[r][c] through a 32x33 LDS tile.
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ src, int rows, int cols, int lds,
                                                        float* __restrict__ dst, int ldd) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    t[y][tx] = (r < rows && c < cols) ? src[(long long)r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < cols && r < rows) dst[(long long)c * ldd + r] = t[tx][y];
  }
}

template <int BN, int EPI, bool CB>
static void launch_bf16_kc(const GemmParams& gp, int splits, hipStream_t s) {
  const int tiles = (int)(ceil_div(gp.M, 128) * ceil_div(gp.N, BN));
  hipLaunchKernelGGL((gemm_bf16_kc_kernel<128, BN, 4, 1, EPI, CB>), dim3(tiles, 1, splits), dim3(256), 0, s, gp);
}

template <int BN>
static void dispatch_bf16_kc_bn(const GemmParams& gp, int epi, int splits, bool cb, hipStream_t s) {
  switch (epi) {
    case EPI_STORE: cb ? launch_bf16_kc<BN, EPI_STORE, true>(gp, splits, s) : launch_bf16_kc<BN, EPI_STORE, false>(gp, splits, s); break;
    case EPI_RELU: cb ? launch_bf16_kc<BN, EPI_RELU, true>(gp, splits, s) : launch_bf16_kc<BN, EPI_RELU, false>(gp, splits, s); break;
    case EPI_MASK: cb ? launch_bf16_kc<BN, EPI_MASK, true>(gp, splits, s) : launch_bf16_kc<BN, EPI_MASK, false>(gp, splits, s); break;
    default: launch_bf16_kc<BN, EPI_SPLIT, false>(gp, splits, s); break;
  }
}

static void dispatch_bf16_kc(const GemmParams& gp, int epi, int splits, bool cb, int bn, hipStream_t s) {
  if (bn == 208) dispatch_bf16_kc_bn<208>(gp, epi, splits, cb, s);
  else dispatch_bf16_kc_bn<80>(gp, epi, splits, cb, s);
}

}  // namespace dl

using namespace dl;

extern "C" int dl_transpose_bf16(const void* src, int32_t src_f32, int32_t rows, int32_t cols, int32_t lds,
                                 uint16_t* dst, int32_t ldd, void* stream) {
  DL_CHECK_ARG(src && dst && rows >= 0 && cols >= 0 && lds >= cols && ldd >= rows, "bad transpose args");
  if (rows == 0 || cols == 0) return 0;
  const dim3 grid((unsigned)ceil_div(cols, 32), (unsigned)ceil_div(rows, 32));
  if (src_f32)
    hipLaunchKernelGGL(transpose_bf16_kernel<true>, grid, dim3(256), 0, as_stream(stream), src, rows, cols, lds, dst, ldd);
  else
    hipLaunchKernelGGL(transpose_bf16_kernel<false>, grid, dim3(256), 0, as_stream(stream), src, rows, cols, lds, dst, ldd);
  DL_RETURN_LAUNCH("dl_transpose_bf16");
}

extern "C" int dl_transpose_f32(const float* src, int32_t rows, int32_t cols, int32_t lds, float* dst, int32_t ldd,
                                void* stream) {
  DL_CHECK_ARG(src && dst && rows >= 0 && cols >= 0 && lds >= cols && ldd >= rows, "bad transpose args");
  if (rows == 0 || cols == 0) return 0;
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)ceil_div(cols, 32), (unsigned)ceil_div(rows, 32)), dim3(256), 0,
                     as_stream(stream), src, rows, cols, lds, dst, ldd);
  DL_RETURN_LAUNCH("dl_transpose_f32");
}

extern "C" int dl_gemm_f32(int32_t ta, int32_t tb, int32_t M, int32_t N, int32_t K, const float* A,
                           int32_t lda, const float* B, int32_t ldb, float* C, int32_t ldc,
                           int32_t epi, const float* mask, int32_t ldm, int32_t splits,
                           int64_t c_split_stride, void* stream) {
  DL_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative dims");
  DL_CHECK_ARG(A && B && C, "NULL operand");
  DL_CHECK_ARG(lda % 4 == 0 && ldb % 4 == 0 && ldc >= N, "lda/ldb must be multiples of 4, ldc >= N");
  DL_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "A/B must be 16-byte aligned");
  // float4 staging reads whole 4-element groups of the contiguous dimension:
  // the rows must be allocated (and finite, normally zero) up to the next multiple of 4.
  DL_CHECK_ARG(lda >= (ta ? (M + 3) / 4 * 4 : (K + 3) / 4 * 4),
               "lda %d < padded contiguous extent of A (ta=%d M=%d K=%d)", lda, ta, M, K);
  DL_CHECK_ARG(ldb >= (tb ? (K + 3) / 4 * 4 : (N + 3) / 4 * 4),
               "ldb %d < padded contiguous extent of B (tb=%d N=%d K=%d)", ldb, tb, N, K);
  DL_CHECK_ARG(epi >= 0 && epi <= 3, "bad epilogue %d", epi);
  DL_CHECK_ARG(epi != EPI_MASK || mask, "mask epilogue needs mask");
  if (splits < 1) splits = 1;
  DL_CHECK_ARG(splits == 1 || epi == EPI_SPLIT, "splits > 1 requires the split epilogue");
  if (M == 0 || N == 0) return 0;
  GemmParams gp;
  gp.A = A; gp.B = B; gp.C = C; gp.mask = mask;
  gp.M = M; gp.N = N; gp.K = K; gp.lda = lda; gp.ldb = ldb; gp.ldc = ldc; gp.ldm = ldm;
  int kps = (int)ceil_div(K, splits);
  kps = (kps + 15) / 16 * 16;
  if (kps == 0) kps = 16;
  gp.k_per_split = kps;
  splits = (int)ceil_div(K > 0 ? K : 1, kps);
  gp.c_split_stride = c_split_stride;
  hipStream_t s = as_stream(stream);
  if (!ta && !tb) dispatch_bn_f32<false, false>(gp, epi, splits, s);
  else if (!ta && tb) dispatch_bn_f32<false, true>(gp, epi, splits, s);
  else if (ta && !tb) dispatch_bn_f32<true, false>(gp, epi, splits, s);
  else dispatch_bn_f32<true, true>(gp, epi, splits, s);
  DL_RETURN_LAUNCH("dl_gemm_f32");
}

extern "C" int dl_gemm_bf16(int32_t ta, int32_t tb, int32_t M, int32_t N, int32_t K,
                            const uint16_t* A, int32_t lda, const uint16_t* B, int32_t ldb, void* C,
                            int32_t ldc, int32_t c_bf16, int32_t epi, const void* mask, int32_t ldm,
                            int32_t splits, int64_t c_split_stride, void* stream) {
  DL_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative dims");
  DL_CHECK_ARG(A && B && C, "NULL operand");
  DL_CHECK_ARG(epi >= 0 && epi <= 3, "bad epilogue %d", epi);
  DL_CHECK_ARG(epi != EPI_MASK || mask, "mask epilogue needs mask");
  DL_CHECK_ARG(!(epi == EPI_SPLIT && c_bf16), "split slabs are fp32");
  if (splits < 1) splits = 1;
  const int splits_req = splits;
  DL_CHECK_ARG(splits == 1 || epi == EPI_SPLIT, "splits > 1 requires the split epilogue");
  if (M == 0 || N == 0) return 0;
  GemmParams gp;
  gp.A = A; gp.B = B; gp.C = C; gp.mask = mask;
  gp.M = M; gp.N = N; gp.K = K; gp.lda = lda; gp.ldb = ldb; gp.ldc = ldc; gp.ldm = ldm;
  int kps = (int)ceil_div(K, splits);
  kps = (kps + 31) / 32 * 32;
  if (kps == 0) kps = 32;
  gp.k_per_split = kps;
  splits = (int)ceil_div(K > 0 ? K : 1, kps);
  gp.c_split_stride = c_split_stride;
  hipStream_t s = as_stream(stream);
  if (ta && !tb && epi == EPI_SPLIT && launch_bf16_dw(gp, splits_req, s)) DL_RETURN_LAUNCH("dl_gemm_bf16");
  if (!ta && tb && lda % 8 == 0 && ldb % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0 &&
      lda >= (K + 7) / 8 * 8 && ldb >= (K + 7) / 8 * 8) {
    // k-contiguous fast path (the tower's products are arranged into this form)
    int kps2 = (int)ceil_div(K, splits);
    kps2 = (kps2 + 63) / 64 * 64;
    if (kps2 == 0) kps2 = 64;
    gp.k_per_split = kps2;
    const int sp2 = (int)ceil_div(K > 0 ? K : 1, kps2);
    if (sp2 == 1 && launch_bf16_nt(gp, epi, c_bf16 != 0, s)) DL_RETURN_LAUNCH("dl_gemm_bf16");
    if (sp2 == 1 && launch_bf16_bres(gp, epi, c_bf16 != 0, s)) DL_RETURN_LAUNCH("dl_gemm_bf16");
    const int bn = (N + 79) / 80 * 80 <= (N + 207) / 208 * 208 ? 80 : 208;
    dispatch_bf16_kc(gp, epi, sp2, c_bf16 != 0, bn, s);
    DL_RETURN_LAUNCH("dl_gemm_bf16");
  }
#define DL_BF(TA_, TB_)                                                              \
  if (c_bf16) launch_bf16<128, 64, 4, 1, TA_, TB_, true>(gp, epi, splits, s);        \
  else launch_bf16<128, 64, 4, 1, TA_, TB_, false>(gp, epi, splits, s);
  if (!ta && !tb) { DL_BF(false, false) }
  else if (!ta && tb) { DL_BF(false, true) }
  else if (ta && !tb) { DL_BF(true, false) }
  else { DL_BF(true, true) }
#undef DL_BF
  DL_RETURN_LAUNCH("dl_gemm_bf16");
}

extern "C" int dl_cast_bf16(const float* src, int32_t rows, int32_t cols, int32_t lds, uint16_t* dst, int32_t ldd,
                            void* stream) {
  DL_CHECK_ARG(src && dst && rows >= 0 && cols >= 0 && lds >= cols && ldd >= cols, "bad cast args");
  if (rows == 0 || cols == 0) return 0;
  long long blocks = ((long long)rows * cols + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), src, rows, cols, lds,
                     dst, ldd);
  DL_RETURN_LAUNCH("dl_cast_bf16");
}
