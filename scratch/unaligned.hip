#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
__global__ void k(const uint8_t* p, u32x4* out) {
  int t = threadIdx.x;
  out[t] = *(const u32x4_u*)(p + t);
}
__global__ void k2(const uint8_t* p, u32x4* out) {
  int t = threadIdx.x;
  out[t] = __builtin_nontemporal_load((const u32x4_u*)(p + t));
}
int main() {
  uint8_t h[4096]; for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
  uint8_t* d; u32x4* o; hipMalloc(&d, 4096); hipMalloc(&o, 64 * 16);
  hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
  int bad = 0;
  for (int kk = 0; kk < 2; ++kk) {
    if (kk == 0) k<<<1, 64>>>(d, o); else k2<<<1, 64>>>(d, o);
    hipError_t e = hipDeviceSynchronize();
    if (e) { printf("err %s\n", hipGetErrorString(e)); return 1; }
    uint8_t r[64 * 16]; hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    for (int t = 0; t < 64; ++t) for (int b = 0; b < 16; ++b) if (r[t * 16 + b] != h[t + b]) ++bad;
  }
  printf("unaligned dwordx4: %s (%d bad bytes)\n", bad ? "MISMATCH" : "ok", bad);
  return bad != 0;
}
