// Probe of ds_read_b64_tr_b16 lane semantics on gfx950: LDS holds a [16 rows][64 cols] u16 tile with
// value row * 100 + col; every lane of 16-lane group g supplies the address of row 4g + (l & 15) / 4,
// columns 4 ((l & 15) % 4) .. +3; prints the 4 values each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short t[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) t[i] = (short)((i / 64) * 100 + i % 64);
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int row = 4 * g + q, col = 4 * p;
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(t + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = v[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
