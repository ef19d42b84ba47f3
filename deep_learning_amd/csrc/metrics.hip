// Exact tie-aware ROC-AUC on the GPU — the evaluation metric of the reference
// (sklearn.metrics.roc_auc_score at models/deepfm_pipeline.py:311,344, wdl.py:343-358).
// No library kernels: the sort is the hand-written stable radix sort of rsort.hip (the one
// the batch index build uses), the scan below is this file's own.
//
// AUC = sum over tie groups g of pos_g * (neg_below_g + 0.5 * neg_g) / (P * N)
// (a positive counts every negative scored below it and half of each negative tied with it).
// Steps:
//   1. keys[i] = order-preserving bits of score i; rsort_pairs sorts (key, i) stably
//   2. per sorted position j: label bit of the sample it holds, head bit (first of a tie group)
//      packed as one int64 v[j] = label + (head << 32); exclusive scan of v gives, at every
//      position, the positives before it (low word) and the number of groups that started
//      before it (high word)
//   3. at every group head j (group g = high word): start[g] = j, cpos[g] = positives before j
//   4. per group: e = next group's start (or n), pos_g = cpos[g+1] - cpos[g], neg_g = e - s - pos_g,
//      neg_below = s - cpos[g]; 2 * numerator += pos_g * (2 * neg_below + neg_g) — an exact
//      int64 sum (order-free, deterministic), divided once in double at the end.
#include "common.h"
#include "rsort.h"

namespace dl {
namespace {

constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;                            // elements per thread
constexpr int kScanTile = kScanThreads * kScanPer;      // 4096

struct AucWs {
  uint32_t* keys;        // float keys (input order)
  uint32_t* skeys;       // sorted keys
  int32_t* sidx;         // sorted sample indices
  uint64_t* v;           // packed label / head bits, then their exclusive scan (in place)
  uint64_t* tsum;        // per-tile sums, then their exclusive scan
  int32_t* gstart;       // start position of group g
  int32_t* gcpos;        // positives before group g
  int32_t* n_valid;      // rsort's count (every key is valid)
  unsigned long long* acc;   // [0] = 2 * numerator, [1] = P, [2] = groups
  void* sort_ws;
  size_t sort_ws_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
int scan_tiles(int n) { return (n + kScanTile - 1) / kScanTile; }

AucWs carve(void* ws, int n) {
  char* p = static_cast<char*>(ws);
  AucWs w;
  const int T = scan_tiles(n);
  w.keys = reinterpret_cast<uint32_t*>(p); p += align256(4ull * n);
  w.skeys = reinterpret_cast<uint32_t*>(p); p += align256(4ull * n);
  w.sidx = reinterpret_cast<int32_t*>(p); p += align256(4ull * n);
  w.v = reinterpret_cast<uint64_t*>(p); p += align256(8ull * n);
  w.tsum = reinterpret_cast<uint64_t*>(p); p += align256(8ull * (T + 1));
  w.gstart = reinterpret_cast<int32_t*>(p); p += align256(4ull * (n + 1));
  w.gcpos = reinterpret_cast<int32_t*>(p); p += align256(4ull * (n + 1));
  w.n_valid = reinterpret_cast<int32_t*>(p); p += 256;
  w.acc = reinterpret_cast<unsigned long long*>(p); p += 256;
  w.sort_ws = p;
  w.sort_ws_bytes = rsort_workspace_bytes(n);
  return w;
}

size_t ws_bytes(int n) {
  const int T = scan_tiles(n);
  return 3 * align256(4ull * n) + align256(8ull * n) + align256(8ull * (T + 1)) + 2 * align256(4ull * (n + 1)) +
         512 + rsort_workspace_bytes(n);
}

// order-preserving map of a float to uint32 (-0.0 folded onto +0.0: they tie, as np.diff says)
__device__ __forceinline__ uint32_t float_key(float x) {
  uint32_t u = __float_as_uint(x == 0.f ? 0.f : x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void auc_keys_kernel(const float* __restrict__ scores, int64_t s_stride, int n,
                                                       uint32_t* __restrict__ keys, unsigned long long* acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 4) acc[threadIdx.x] = 0;
  if (i < n) keys[i] = float_key(scores[(int64_t)i * s_stride]);
}

// v[j] = label of the sample at sorted position j + (j starts a tie group) << 32
__global__ __launch_bounds__(256) void auc_flags_kernel(const uint32_t* __restrict__ sk, const int32_t* __restrict__ si,
                                                        const float* __restrict__ labels, int64_t l_stride, int n,
                                                        uint64_t* __restrict__ v) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t k = sk[j];
  const int idx = min(max(si[j], 0), n - 1);
  const uint64_t lab = labels[(int64_t)idx * l_stride] > 0.5f ? 1u : 0u;
  const uint64_t head = (j == 0 || sk[j - 1] != k) ? 1u : 0u;
  v[j] = lab | (head << 32);
}

// Block-wide exclusive scan of one uint64 per thread; *total = the block's sum.
__device__ __forceinline__ uint64_t block_exscan(uint64_t x, uint64_t* wsum, uint64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t base = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kScanThreads / 64; ++i) {
    base += i < w ? wsum[i] : 0;
    all += wsum[i];
  }
  *total = all;
  return base + inc - x;
}

// Pass 1: the sum of each 4096-element tile.
__global__ __launch_bounds__(kScanThreads) void scan_tile_sums(const uint64_t* __restrict__ v, int n,
                                                               uint64_t* __restrict__ tsum) {
  __shared__ uint64_t wsum[kScanThreads / 64];
  const long long t0 = (long long)blockIdx.x * kScanTile;
  uint64_t s = 0;
#pragma unroll
  for (int r = 0; r < kScanPer; ++r) {
    const long long e = t0 + r * kScanThreads + threadIdx.x;
    s += e < n ? v[e] : 0;
  }
  uint64_t all;
  block_exscan(s, wsum, &all);
  if (threadIdx.x == 0) tsum[blockIdx.x] = all;
}

// Pass 2 (one block): exclusive scan of the tile sums in place; tsum[T] = the grand total.
__global__ __launch_bounds__(kScanThreads) void scan_tile_prefix(uint64_t* __restrict__ tsum, int T) {
  __shared__ uint64_t wsum[kScanThreads / 64];
  const int per = (T + kScanThreads - 1) / kScanThreads;
  const int a = threadIdx.x * per, b = min(T, a + per);
  uint64_t s = 0;
  for (int i = a; i < b; ++i) s += tsum[i];
  uint64_t all;
  uint64_t run = block_exscan(s, wsum, &all);
  for (int i = a; i < b; ++i) {
    const uint64_t c = tsum[i];
    tsum[i] = run;
    run += c;
  }
  if (threadIdx.x == 0) tsum[T] = all;
}

// Pass 3: each tile's exclusive scan (thread-contiguous runs of kScanPer elements), offset by
// the tile's prefix; at every group head j: gstart[g] = j, gcpos[g] = positives before j.
__global__ __launch_bounds__(kScanThreads) void scan_tile_apply(uint64_t* __restrict__ v, int n,
                                                                const uint64_t* __restrict__ tsum,
                                                                int32_t* __restrict__ gstart,
                                                                int32_t* __restrict__ gcpos) {
  __shared__ uint64_t wsum[kScanThreads / 64];
  const long long e0 = (long long)blockIdx.x * kScanTile + (long long)threadIdx.x * kScanPer;
  uint64_t x[kScanPer];
  uint64_t s = 0;
#pragma unroll
  for (int r = 0; r < kScanPer; ++r) {
    x[r] = e0 + r < n ? v[e0 + r] : 0;
    s += x[r];
  }
  uint64_t all;
  uint64_t run = block_exscan(s, wsum, &all) + tsum[blockIdx.x];
#pragma unroll
  for (int r = 0; r < kScanPer; ++r) {
    const long long e = e0 + r;
    if (e < n) {
      v[e] = run;
      if (x[r] >> 32) {   // a group head: run's high word = groups before it = its group index
        const uint32_t g = (uint32_t)(run >> 32);
        gstart[g] = (int32_t)e;
        gcpos[g] = (int32_t)(run & 0xffffffffu);
      }
    }
    run += x[r];
  }
}

// Per group g: its positives times (2 x negatives below it + its own negatives).
__global__ __launch_bounds__(256) void auc_groups_kernel(const int32_t* __restrict__ gstart,
                                                         const int32_t* __restrict__ gcpos,
                                                         const uint64_t* __restrict__ tsum, int T, int n,
                                                         unsigned long long* acc) {
  const uint64_t tot = tsum[T];
  const long long G = (long long)(tot >> 32);
  const long long P = (long long)(tot & 0xffffffffu);
  unsigned long long num = 0;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (long long)gridDim.x * blockDim.x) {
    const long long s = gstart[g];
    const long long e = g + 1 < G ? gstart[g + 1] : n;
    const long long c0 = gcpos[g];
    const long long c1 = g + 1 < G ? gcpos[g + 1] : P;
    const long long pos = c1 - c0;
    const long long neg = (e - s) - pos;
    const long long below = s - c0;
    num += (unsigned long long)(pos * (2 * below + neg));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) num += __shfl_xor(num, o, 64);
  if ((threadIdx.x & 63) == 0 && num) atomicAdd(acc, num);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    acc[1] = (unsigned long long)P;
    acc[2] = (unsigned long long)G;
  }
}

__global__ void auc_final_kernel(const unsigned long long* acc, int n, double* out) {
  const double P = (double)acc[1], N = (double)n - P;
  out[0] = (P == 0.0 || N == 0.0) ? __builtin_nan("") : (double)acc[0] / (2.0 * P * N);
}

}  // namespace
}  // namespace dl

using namespace dl;

extern "C" int64_t dl_auc_workspace_bytes(int64_t n) {
  if (n <= 0 || n > 0x7fffffff) return -1;
  return (int64_t)ws_bytes((int)n);
}

extern "C" int dl_auc(const float* scores, int64_t s_stride, const float* labels, int64_t l_stride, int64_t n,
                      void* ws, int64_t ws_bytes_, double* out, void* stream) {
  DL_CHECK_ARG(scores && labels && out && ws, "NULL argument");
  DL_CHECK_ARG(n > 0 && n <= 0x7fffffff, "n = %lld out of range", (long long)n);
  DL_CHECK_ARG(ws_bytes_ >= dl_auc_workspace_bytes(n), "workspace too small (%lld < %lld)", (long long)ws_bytes_,
               (long long)dl_auc_workspace_bytes(n));
  const int m = (int)n;
  hipStream_t s = as_stream(stream);
  AucWs w = carve(ws, m);
  const int g = (m + 255) / 256;
  hipLaunchKernelGGL(auc_keys_kernel, dim3(g), dim3(256), 0, s, scores, s_stride, m, w.keys, w.acc);
  RsSource src{};
  src.kind = 0;
  src.keys = w.keys;
  if (int rc = rsort_pairs(src, m, 0, 32, w.sort_ws, w.sort_ws_bytes, w.skeys, w.sidx, w.n_valid, s)) {
    set_error("dl_auc: radix sort failed (%d)", rc);
    return rc;
  }
  hipLaunchKernelGGL(auc_flags_kernel, dim3(g), dim3(256), 0, s, w.skeys, w.sidx, labels, l_stride, m, w.v);
  const int T = scan_tiles(m);
  hipLaunchKernelGGL(scan_tile_sums, dim3(T), dim3(kScanThreads), 0, s, w.v, m, w.tsum);
  hipLaunchKernelGGL(scan_tile_prefix, dim3(1), dim3(kScanThreads), 0, s, w.tsum, T);
  hipLaunchKernelGGL(scan_tile_apply, dim3(T), dim3(kScanThreads), 0, s, w.v, m, w.tsum, w.gstart, w.gcpos);
  hipLaunchKernelGGL(auc_groups_kernel, dim3(std::min(g, 2048)), dim3(256), 0, s, w.gstart, w.gcpos, w.tsum, T, m,
                     w.acc);
  hipLaunchKernelGGL(auc_final_kernel, dim3(1), dim3(1), 0, s, w.acc, m, out);
  DL_RETURN_LAUNCH("dl_auc");
}

// ---------------------------------------------------------------------------
// The measured HBM yardstick (bench.py roofline.peak_measured): a streaming copy, each block one
// chunk of 8 x 256 16-B pieces, all eight non-temporal loads in flight before the non-temporal
// stores — the fastest of the copy forms scripts/ubench_copy.hip measured on this chip (5.56
// TB/s at 1 and 4 GiB; grid-stride plain copies 4.2-4.7, torch's copy_ 5.0-5.2,
// profiles/r06d/ubench_copy.txt): what a read-once / write-once stream reaches here, beside the
// 8 TB/s specification the roofline fractions are priced against.
typedef unsigned int hbm_u4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void hbm_copy_kernel(const hbm_u4* __restrict__ src, hbm_u4* __restrict__ dst,
                                                       long long n16) {
  const long long c0 = (long long)blockIdx.x * 2048;
  hbm_u4 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const long long i = c0 + u * 256 + threadIdx.x;
    if (i < n16) v[u] = __builtin_nontemporal_load(src + i);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const long long i = c0 + u * 256 + threadIdx.x;
    if (i < n16) __builtin_nontemporal_store(v[u], dst + i);
  }
}

extern "C" int dl_hbm_copy(const void* src, void* dst, int64_t bytes, void* stream) {
  DL_CHECK_ARG(src && dst && bytes >= 0 && bytes % 16 == 0, "dl_hbm_copy: bad arguments (bytes %lld)",
               (long long)bytes);
  DL_CHECK_ARG(((uintptr_t)src | (uintptr_t)dst) % 16 == 0, "dl_hbm_copy: 16-B alignment");
  if (bytes == 0) return 0;
  const long long n16 = bytes / 16;
  DL_CHECK_ARG((n16 + 2047) / 2048 < (1LL << 31), "dl_hbm_copy: too many bytes");
  hipLaunchKernelGGL(hbm_copy_kernel, dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const hbm_u4*>(src), reinterpret_cast<hbm_u4*>(dst), n16);
  DL_RETURN_LAUNCH("dl_hbm_copy");
}
