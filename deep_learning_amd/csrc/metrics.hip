// Exact tie-aware ROC-AUC on the GPU — the evaluation metric of the reference
// (sklearn.metrics.roc_auc_score at models/deepfm_pipeline.py:311,344, wdl.py:343-358).
//
// AUC = sum over positives of (#negatives scored below + 0.5 * #negatives tied) / (P * N).
// The scores are sorted as 33-bit keys (order-preserving float bits << 1 | label), so
// within a tie group the negatives come first.  For a positive at sorted position i in a
// tie group starting at s (cpos = exclusive count of positives):
//     negatives at positions < i  = i - cpos[i]   (= below + tied: all tied negatives precede it)
//     negatives below the group   = s - cpos[s]
// and twice its contribution is their sum — an integer.  The numerator is therefore an
// exact int64 sum (order-free, deterministic), divided once in double at the end.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace dl {
namespace {

struct AucWs {
  uint64_t* keys;
  uint64_t* keys_sorted;
  int32_t* cpos;         // exclusive count of positives before i
  int32_t* start;        // first position of i's tie group
  unsigned long long* acc;  // [0] = 2 * numerator, [1] = P
  void* temp;
  size_t temp_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// max-scan functor over group-head positions
struct MaxOp {
  __device__ __forceinline__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; }
};

size_t cub_bytes(int n) {
  size_t a = 0, b = 0, c = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr, n, 0, 33);
  hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, n);
  hipcub::DeviceScan::InclusiveScan(nullptr, c, (const int32_t*)nullptr, (int32_t*)nullptr, MaxOp(), n);
  return std::max(a, std::max(b, c));
}

AucWs carve(void* ws, int n) {
  char* p = static_cast<char*>(ws);
  AucWs w;
  w.keys = reinterpret_cast<uint64_t*>(p); p += align256(8ull * n);
  w.keys_sorted = reinterpret_cast<uint64_t*>(p); p += align256(8ull * n);
  w.cpos = reinterpret_cast<int32_t*>(p); p += align256(4ull * n);
  w.start = reinterpret_cast<int32_t*>(p); p += align256(4ull * n);
  w.acc = reinterpret_cast<unsigned long long*>(p); p += 256;
  w.temp = p;
  w.temp_bytes = cub_bytes(n);
  return w;
}

// order-preserving map of a float to uint32 (-0.0 folded onto +0.0: they tie, as np.diff says)
__device__ __forceinline__ uint32_t float_key(float x) {
  uint32_t u = __float_as_uint(x == 0.f ? 0.f : x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void auc_keys_kernel(const float* __restrict__ scores, int64_t s_stride,
                                                       const float* __restrict__ labels, int64_t l_stride,
                                                       int n, uint64_t* __restrict__ keys,
                                                       unsigned long long* acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2 && blockIdx.x == 0) acc[i] = 0;
  if (i >= n) return;
  const uint64_t lab = labels[(int64_t)i * l_stride] > 0.5f ? 1u : 0u;
  keys[i] = ((uint64_t)float_key(scores[(int64_t)i * s_stride]) << 1) | lab;
}

// label bits of the sorted keys (for the scan) and the group-head positions (for the max-scan)
__global__ __launch_bounds__(256) void auc_flags_kernel(const uint64_t* __restrict__ k, int n,
                                                        int32_t* __restrict__ lab, int32_t* __restrict__ head) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ki = k[i];
  lab[i] = (int32_t)(ki & 1u);
  head[i] = (i == 0 || (k[i - 1] >> 1) != (ki >> 1)) ? i : 0;
}

__global__ __launch_bounds__(256) void auc_sum_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ cpos,
                                                      const int32_t* __restrict__ start, int n,
                                                      unsigned long long* acc) {
  unsigned long long num = 0, pos = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (k[i] & 1u) {
      const int s = start[i];
      num += (unsigned long long)(i - cpos[i]) + (unsigned long long)(s - cpos[s]);
      pos += 1;
    }
  }
  // wave reduce, then one atomic per wave (integer: the order does not matter)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    num += __shfl_xor(num, o, 64);
    pos += __shfl_xor(pos, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && pos) {
    atomicAdd(acc, num);
    atomicAdd(acc + 1, pos);
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
  const int m = (int)n;
  return (int64_t)(2 * align256(8ull * m) + 2 * align256(4ull * m) + 256 + cub_bytes(m));
}

extern "C" int dl_auc(const float* scores, int64_t s_stride, const float* labels, int64_t l_stride, int64_t n,
                      void* ws, int64_t ws_bytes, double* out, void* stream) {
  DL_CHECK_ARG(scores && labels && out && ws, "NULL argument");
  DL_CHECK_ARG(n > 0 && n <= 0x7fffffff, "n = %lld out of range", (long long)n);
  DL_CHECK_ARG(ws_bytes >= dl_auc_workspace_bytes(n), "workspace too small (%lld < %lld)", (long long)ws_bytes,
               (long long)dl_auc_workspace_bytes(n));
  const int m = (int)n;
  hipStream_t s = as_stream(stream);
  AucWs w = carve(ws, m);
  const int g = (m + 255) / 256;
  hipLaunchKernelGGL(auc_keys_kernel, dim3(g), dim3(256), 0, s, scores, s_stride, labels, l_stride, m, w.keys,
                     w.acc);
  size_t tb = w.temp_bytes;
  if (hipcub::DeviceRadixSort::SortKeys(w.temp, tb, w.keys, w.keys_sorted, m, 0, 33, s) != hipSuccess) {
    set_error("dl_auc: radix sort failed");
    return 1001;
  }
  // the key buffer is free after the sort: reuse it for the label bits and head positions
  int32_t* lab = reinterpret_cast<int32_t*>(w.keys);
  int32_t* head = lab + m;
  hipLaunchKernelGGL(auc_flags_kernel, dim3(g), dim3(256), 0, s, w.keys_sorted, m, lab, head);
  tb = w.temp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(w.temp, tb, lab, w.cpos, m, s) != hipSuccess) {
    set_error("dl_auc: scan failed");
    return 1001;
  }
  tb = w.temp_bytes;
  if (hipcub::DeviceScan::InclusiveScan(w.temp, tb, head, w.start, MaxOp(), m, s) != hipSuccess) {
    set_error("dl_auc: max-scan failed");
    return 1001;
  }
  const int gs = std::min(g, 2048);
  hipLaunchKernelGGL(auc_sum_kernel, dim3(gs), dim3(256), 0, s, w.keys_sorted, w.cpos, w.start, m, w.acc);
  hipLaunchKernelGGL(auc_final_kernel, dim3(1), dim3(1), 0, s, w.acc, m, out);
  DL_RETURN_LAUNCH("dl_auc");
}
