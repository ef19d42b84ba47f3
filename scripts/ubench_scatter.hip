// Micro-benchmark: how fast are the access shapes the embedding path could use?
//   seq64     64-B pieces (4 lanes x float4) written / read in order
//   scat64    64-B pieces written / read through a random permutation (each piece once)
//   rec256    256-B records read / written at random rows of a 6.6 GB table (uniform ids)
// hipcc -O3 --offload-arch=gfx950 scripts/ubench_scatter.hip -o /tmp/ubs && /tmp/ubs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_write64(float4* __restrict__ dst, const int* __restrict__ perm, long long n, int use_perm) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n * 4; i += (long long)gridDim.x * blockDim.x) {
    const long long piece = i >> 2;
    const long long d = use_perm ? perm[piece] : piece;
    dst[d * 4 + (i & 3)] = make_float4((float)i, 1.f, 2.f, 3.f);
  }
}

__global__ void k_read64(const float4* __restrict__ src, const int* __restrict__ perm, long long n, int use_perm,
                         float* __restrict__ out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n * 4; i += (long long)gridDim.x * blockDim.x) {
    const long long piece = i >> 2;
    const long long d = use_perm ? perm[piece] : piece;
    const float4 v = src[d * 4 + (i & 3)];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

// 16 lanes per record (E=16 layout: 64 floats, 256 B), rows[] uniform random
__global__ void k_rec(float4* __restrict__ rec, const int* __restrict__ rows, long long n, int mode,
                      float* __restrict__ out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n * 16; i += (long long)gridDim.x * blockDim.x) {
    const long long r = rows[i >> 4];
    float4* p = rec + r * 16 + (i & 15);
    if (mode == 0) {
      const float4 v = *p;
      acc += v.x + v.w;
    } else if (mode == 1) {
      *p = make_float4(1.f, 2.f, (float)i, 4.f);
    } else {
      float4 v = *p;
      v.x += 1.f;
      *p = v;
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

template <typename F>
float timeit(F f, int reps = 5) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1000.f;   // us
}

int main() {
  const long long n = 3407872;   // pieces: C2's references (65536 x 52)
  float4* buf;
  int *perm, *iden;
  float* out;
  CK(hipMalloc(&buf, n * 64));
  CK(hipMalloc(&perm, n * 4));
  CK(hipMalloc(&iden, n * 4));
  CK(hipMalloc(&out, 64));
  std::vector<int> h(n);
  for (long long i = 0; i < n; ++i) h[i] = (int)i;
  CK(hipMemcpy(iden, h.data(), n * 4, hipMemcpyHostToDevice));
  std::mt19937_64 g(1);
  std::shuffle(h.begin(), h.end(), g);
  CK(hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice));
  const double mb = n * 64 / 1e6;
  const dim3 grid(8192), blk(256);
  float t;
  t = timeit([&] { k_write64<<<grid, blk>>>(buf, iden, n, 0); });
  printf("seq64  write %8.1f us  %7.1f GB/s  (%.0f MB)\n", t, mb / t * 1e3, mb);
  t = timeit([&] { k_write64<<<grid, blk>>>(buf, perm, n, 1); });
  printf("scat64 write %8.1f us  %7.1f GB/s\n", t, mb / t * 1e3);
  t = timeit([&] { k_read64<<<grid, blk>>>(buf, iden, n, 0, out); });
  printf("seq64  read  %8.1f us  %7.1f GB/s\n", t, mb / t * 1e3);
  t = timeit([&] { k_read64<<<grid, blk>>>(buf, perm, n, 1, out); });
  printf("scat64 read  %8.1f us  %7.1f GB/s\n", t, mb / t * 1e3);
  // records: 26M x 256 B table, 3.2M random rows (uniform)
  const long long rows = 26000016, U = 3200000;
  float4* rec;
  int* rix;
  CK(hipMalloc(&rec, rows * 256));
  CK(hipMemset(rec, 0, rows * 256));
  CK(hipMalloc(&rix, U * 4));
  std::vector<int> hr(U);
  std::uniform_int_distribution<int> ud(0, (int)rows - 1);
  for (long long i = 0; i < U; ++i) hr[i] = ud(g);
  std::sort(hr.begin(), hr.end());   // the gather walks unique rows in sorted order
  CK(hipMemcpy(rix, hr.data(), U * 4, hipMemcpyHostToDevice));
  const double rmb = U * 256 / 1e6;
  t = timeit([&] { k_rec<<<grid, blk>>>(rec, rix, U, 0, out); });
  printf("rec256 read  %8.1f us  %7.1f GB/s  (%.0f MB)\n", t, rmb / t * 1e3, rmb);
  t = timeit([&] { k_rec<<<grid, blk>>>(rec, rix, U, 1, out); });
  printf("rec256 write %8.1f us  %7.1f GB/s\n", t, rmb / t * 1e3);
  t = timeit([&] { k_rec<<<grid, blk>>>(rec, rix, U, 2, out); });
  printf("rec256 rmw   %8.1f us  %7.1f GB/s (counting R+W)\n", t, 2 * rmb / t * 1e3);
  CK(hipFree(rec));
  CK(hipFree(buf));
  return 0;
}
