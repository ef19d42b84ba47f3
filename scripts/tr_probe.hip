// Probe of ds_read_b64_tr_b16 lane semantics on gfx950: LDS tile [32 rows][32 cols] of
// u16 = row*100 + col; every lane supplies &T[4*kq + (cl>>2)][4*(cl&3)] (cl = lane&15,
// kq = lane>>4) and prints the 4 values it receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(4 * sizeof(__fp16)))) __fp16 f16x4;
__global__ void probe(unsigned* out) {
  __shared__ unsigned short T[32 * 32];
  for (int i = threadIdx.x; i < 32 * 32; i += 64) T[i] = (unsigned short)((i / 32) * 100 + (i % 32));
  __syncthreads();
  const int lane = threadIdx.x, cl = lane & 15, kq = lane >> 4;
  unsigned short* p = &T[(4 * kq + (cl >> 2)) * 32 + 4 * (cl & 3)];
  auto lp = (__attribute__((address_space(3))) unsigned short*)(p);
  f16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4f16(reinterpret_cast<__attribute__((address_space(3))) f16x4*>(lp));
  unsigned short s[4];
  __builtin_memcpy(s, &v, 8);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = s[e];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4u %4u %4u %4u\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  return 0;
}
