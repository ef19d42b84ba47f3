// Micro-benchmark: streaming copy variants on MI355X (the HBM yardstick of bench.py).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/ubench_copy.hip -o /tmp/ubench_copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// A: grid-stride, 4 pieces in flight a thread, pieces a grid apart (the round-6 dl_hbm_copy)
__global__ __launch_bounds__(256) void copy_gs4(const uint4* __restrict__ s, uint4* __restrict__ d, long n) {
  const long st = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    uint4 a = s[i], b = s[i + st], c = s[i + 2 * st], e = s[i + 3 * st];
    d[i] = a; d[i + st] = b; d[i + 2 * st] = c; d[i + 3 * st] = e;
  }
  for (; i < n; i += st) d[i] = s[i];
}
// B: each block copies contiguous chunks of U x 256 pieces (all loads, then all stores)
template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const uint4* __restrict__ s, uint4* __restrict__ d, long n) {
  const long chunk = (long)U * 256;
  for (long c0 = (long)blockIdx.x * chunk; c0 < n; c0 += (long)gridDim.x * chunk) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { const long i = c0 + u * 256 + threadIdx.x; if (i < n) v[u] = s[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { const long i = c0 + u * 256 + threadIdx.x; if (i < n) d[i] = v[u]; }
  }
}
// C: B with non-temporal loads and stores
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void copy_chunk_nt(const uint4* __restrict__ s_, uint4* __restrict__ d_, long n) {
  const u4v* s = reinterpret_cast<const u4v*>(s_);
  u4v* d = reinterpret_cast<u4v*>(d_);
  const long chunk = (long)U * 256;
  for (long c0 = (long)blockIdx.x * chunk; c0 < n; c0 += (long)gridDim.x * chunk) {
    u4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { const long i = c0 + u * 256 + threadIdx.x; if (i < n) v[u] = __builtin_nontemporal_load(s + i); }
#pragma unroll
    for (int u = 0; u < U; ++u) { const long i = c0 + u * 256 + threadIdx.x; if (i < n) __builtin_nontemporal_store(v[u], d + i); }
  }
}

template <class F>
static void run(const char* name, F launch, long n) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < 10; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / 10;
  printf("%-28s %8.1f us  %7.1f GB/s\n", name, us, 2.0 * n * 16 / us / 1e3);
}

int main() {
  for (long gib : {1L, 4L}) {
    const long n = gib * (1L << 30) / 16;
    uint4 *a, *b;
    CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16));
    CK(hipMemset(a, 1, n * 16)); CK(hipMemset(b, 0, n * 16));
    printf("== %ld GiB\n", gib);
    for (int g : {1024, 2048, 4096}) {
      char nm[64];
      snprintf(nm, 64, "gs4 grid %d", g);
      run(nm, [&] { hipLaunchKernelGGL(copy_gs4, dim3(g), dim3(256), 0, 0, a, b, n); }, n);
    }
    for (int g : {512, 1024, 2048, 4096}) {
      char nm[64];
      snprintf(nm, 64, "chunk8 grid %d", g);
      run(nm, [&] { hipLaunchKernelGGL(copy_chunk<8>, dim3(g), dim3(256), 0, 0, a, b, n); }, n);
      snprintf(nm, 64, "chunk4 grid %d", g);
      run(nm, [&] { hipLaunchKernelGGL(copy_chunk<4>, dim3(g), dim3(256), 0, 0, a, b, n); }, n);
      snprintf(nm, 64, "chunk8 nt grid %d", g);
      run(nm, [&] { hipLaunchKernelGGL(copy_chunk_nt<8>, dim3(g), dim3(256), 0, 0, a, b, n); }, n);
    }
    const long blocks = (n + 2047) / 2048;   // one chunk of 8 x 256 pieces a block, no loop
    run("chunk8 one-shot", [&] { hipLaunchKernelGGL(copy_chunk<8>, dim3(blocks), dim3(256), 0, 0, a, b, n); }, n);
    run("chunk8 nt one-shot", [&] { hipLaunchKernelGGL(copy_chunk_nt<8>, dim3(blocks), dim3(256), 0, 0, a, b, n); }, n);
    CK(hipFree(a)); CK(hipFree(b));
  }
  return 0;
}
