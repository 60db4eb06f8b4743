// Learns the lane mapping of ds_read_b64_tr_b8 on gfx950: LDS byte p holds
// p & 255 (pass 0) or p >> 8 (pass 1); lane l reads at byte l * 8.  Output:
// out[pass][lane][8] -> the source byte index of every received byte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void probe(uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[1024];
  const int l = threadIdx.x;
  for (int pass = 0; pass < 2; ++pass) {
    for (int p = l; p < 1024; p += 64) s[p] = pass ? (uint8_t)(p >> 8) : (uint8_t)(p & 255);
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)s + l * 8;
    v2i r;
    asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a));
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&r);
    for (int k = 0; k < 8; ++k) out[(pass * 64 + l) * 8 + k] = b[k];
    __syncthreads();
  }
}
int main() {
  uint8_t* d;
  hipMalloc(&d, 1024);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint8_t h[1024];
  hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int k = 0; k < 8; ++k) {
      const int p = h[l * 8 + k] | (h[(64 + l) * 8 + k] << 8);
      printf(" L%02d.b%d", p / 8, p % 8);
    }
    printf("\n");
  }
  return 0;
}
