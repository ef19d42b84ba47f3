// Micro-benchmark: random 64-B row gathers on MI355X (what bounds the embedding lookup).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/ubench_gather.hip -o /tmp/ubench_gather
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// variant 0: 4 lanes per row (float4 each), one row index per lane group
__global__ void g_f4(const float4* __restrict__ tab, const int* __restrict__ idx, float4* __restrict__ out, long n_rows_req) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (long i = t; i < n_rows_req * 4; i += stride) {
    const int r = idx[i >> 2];
    out[i] = tab[(long)r * 4 + (i & 3)];
  }
}
// variant 1: same, but each thread handles U row-quarters with all loads issued first
template <int U>
__global__ void g_f4u(const float4* __restrict__ tab, const int* __restrict__ idx, float4* __restrict__ out, long n) {
  long base = ((long)blockIdx.x * blockDim.x) * U + threadIdx.x;
  float4 v[U];
  int r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; r[u] = i < n * 4 ? idx[i >> 2] : 0; }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; v[u] = tab[(long)r[u] * 4 + (i & 3)]; }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n * 4) out[i] = v[u]; }
}
// variant 2: read-only (sum), no output stream
template <int U>
__global__ void g_sum(const float4* __restrict__ tab, const int* __restrict__ idx, float* __restrict__ out, long n) {
  long base = ((long)blockIdx.x * blockDim.x) * U + threadIdx.x;
  float4 v[U];
  int r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; r[u] = i < n * 4 ? idx[i >> 2] : 0; }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; v[u] = tab[(long)r[u] * 4 + (i & 3)]; }
  float s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
  if (s == 123.456f) out[0] = s;
}
// variant 3: scalar 4-B random loads (first-order weights)
template <int U>
__global__ void g_scalar(const float* __restrict__ tab, const int* __restrict__ idx, float* __restrict__ out, long n) {
  long base = ((long)blockIdx.x * blockDim.x) * U + threadIdx.x;
  float v[U];
  int r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; r[u] = i < n ? idx[i] : 0; }
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = tab[r[u]];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; if (i < n) out[i] = v[u]; }
}
// variant 4: 64-B row + its 4-B first-order weight, the weight in a separate [rows] array
// (the predict planes' layout) or at byte 64 of a 128-B slot (row, weight, pad): two loads per
// reference either way; do they cost two random requests or one?
template <int U, bool SAME>
__global__ void g_row_w1(const float4* __restrict__ tab, const float* __restrict__ w1, const int* __restrict__ idx,
                         float* __restrict__ out, long n) {
  long base = ((long)blockIdx.x * blockDim.x) * U + threadIdx.x;
  float4 v[U];
  float w[U];
  int r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + (long)u * blockDim.x; r[u] = i < n * 4 ? idx[i >> 2] : 0; }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    long i = base + (long)u * blockDim.x;
    v[u] = tab[(long)r[u] * (SAME ? 8 : 4) + (i & 3)];
    const bool q0 = (i & 3) == 0;
    w[u] = q0 ? (SAME ? reinterpret_cast<const float*>(tab)[(long)r[u] * 32 + 16] : w1[r[u]]) : 0.f;
  }
  float s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w + w[u];
  if (s == 123.456f) out[0] = s;
}
// streaming copy for reference
__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}

int main(int argc, char** argv) {
  const long rows = argc > 1 ? atol(argv[1]) : 26000013;
  const long nreq = argc > 2 ? atol(argv[2]) : 65536L * 52;
  float4* tab; int* idx; float4* out; float* outs;
  CK(hipMalloc(&tab, rows * 64));
  CK(hipMalloc(&idx, nreq * 4));
  CK(hipMalloc(&out, nreq * 64));
  CK(hipMalloc(&outs, nreq * 4));
  CK(hipMemset(tab, 0, rows * 64));
  float4* tab128; float* w1;
  CK(hipMalloc(&tab128, rows * 128));
  CK(hipMalloc(&w1, rows * 4));
  CK(hipMemset(tab128, 0, rows * 128));
  CK(hipMemset(w1, 0, rows * 4));
  std::vector<int> h(nreq);
  srand(1);
  for (long i = 0; i < nreq; ++i) h[i] = (int)(((unsigned long)rand() * 2654435761UL + rand()) % rows);
  std::vector<int> hs = h; std::sort(hs.begin(), hs.end());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double bytes) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int w = 0; w < it; ++w) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double us = ms * 1e3 / it;
    printf("%-40s %9.1f us  %8.1f GB/s (rows %.2f G/s)\n", name, us, bytes / us / 1e3, nreq / us / 1e3);
  };
  for (int sorted = 0; sorted < 2; ++sorted) {
    CK(hipMemcpy(idx, sorted ? hs.data() : h.data(), nreq * 4, hipMemcpyHostToDevice));
    printf("== table %ld rows (%.2f GB), %ld requests, %s\n", rows, rows * 64 / 1e9, nreq, sorted ? "sorted" : "random");
    const double rb = nreq * 64.0;
    timeit("f4 gridstride 2048x256 (+write)", [&] { hipLaunchKernelGGL(g_f4, dim3(2048), dim3(256), 0, 0, tab, idx, out, nreq); }, 2 * rb);
    timeit("f4 1-per-thread (+write)", [&] { hipLaunchKernelGGL(g_f4, dim3((nreq * 4 + 255) / 256), dim3(256), 0, 0, tab, idx, out, nreq); }, 2 * rb);
    timeit("f4u U=4 (+write)", [&] { hipLaunchKernelGGL(g_f4u<4>, dim3((nreq * 4 + 1023) / 1024), dim3(256), 0, 0, tab, idx, out, nreq); }, 2 * rb);
    timeit("f4u U=8 (+write)", [&] { hipLaunchKernelGGL(g_f4u<8>, dim3((nreq * 4 + 2047) / 2048), dim3(256), 0, 0, tab, idx, out, nreq); }, 2 * rb);
    timeit("sum U=4 (read only)", [&] { hipLaunchKernelGGL(g_sum<4>, dim3((nreq * 4 + 1023) / 1024), dim3(256), 0, 0, tab, idx, outs, nreq); }, rb);
    timeit("sum U=8 (read only)", [&] { hipLaunchKernelGGL(g_sum<8>, dim3((nreq * 4 + 2047) / 2048), dim3(256), 0, 0, tab, idx, outs, nreq); }, rb);
    timeit("row + w1 separate array U=4 (read only)", [&] { hipLaunchKernelGGL((g_row_w1<4, false>), dim3((nreq * 4 + 1023) / 1024), dim3(256), 0, 0, tab, w1, idx, outs, nreq); }, rb);
    timeit("row + w1 same 128-B slot U=4 (read only)", [&] { hipLaunchKernelGGL((g_row_w1<4, true>), dim3((nreq * 4 + 1023) / 1024), dim3(256), 0, 0, tab128, w1, idx, outs, nreq); }, rb);
    timeit("scalar 4B U=8 (+write)", [&] { hipLaunchKernelGGL(g_scalar<8>, dim3((nreq + 2047) / 2048), dim3(256), 0, 0, (const float*)tab, idx, outs, nreq); }, nreq * 8.0);
  }
  const long n4 = rows * 4;
  float4* cp; CK(hipMalloc(&cp, rows * 64));
  timeit("stream copy table (r+w)", [&] { hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, tab, cp, n4); }, 2.0 * rows * 64);
  return 0;
}
