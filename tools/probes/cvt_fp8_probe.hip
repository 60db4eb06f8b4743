// Probe: is v_cvt_pk_fp8_f32 exact round-to-nearest-even on arbitrary f32?
// Compares it with a software nearest-even (f32 bits) over values around
// every e4m3 midpoint (+-0..64 ulps) and random values; prints mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>
#include <cmath>

__device__ float rne_e4m3(float f) {
  const float a = fabsf(f);
  if (a < 0.015625f) return rintf(f * 512.f) * (1.f / 512.f);
  uint32_t b = __float_as_uint(f);
  b += 0x7ffffu + ((b >> 20) & 1u);
  return __uint_as_float(b & 0xfff00000u);
}

__global__ void probe(const float* x, int n, uint32_t* out_hw, uint32_t* out_sw) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float f = fminf(fmaxf(x[i], -448.f), 448.f);
  out_hw[i] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xffu;
  out_sw[i] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(rne_e4m3(f), rne_e4m3(f), 0, false) & 0xffu;
}

int main() {
  std::vector<float> xs;
  // e4m3 positive values: subnormals k*2^-9, normals (1+m/8)*2^e, e in [-6, 8]
  std::vector<double> vals;
  for (int k = 0; k < 8; ++k) vals.push_back(k / 512.0);
  for (int e = -6; e <= 8; ++e)
    for (int m = 0; m < 8; ++m) vals.push_back((1 + m / 8.0) * std::ldexp(1.0, e));
  for (size_t i = 0; i + 1 < vals.size(); ++i) {
    float mid = (float)((vals[i] + vals[i + 1]) / 2);
    uint32_t b;
    std::memcpy(&b, &mid, 4);
    for (int d = -64; d <= 64; ++d) {
      uint32_t c = b + d;
      float f;
      std::memcpy(&f, &c, 4);
      xs.push_back(f);
      xs.push_back(-f);
    }
  }
  uint32_t s = 12345;
  for (int i = 0; i < (1 << 20); ++i) {
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) / 16777216.0f - 0.5f) * 900.f;
    xs.push_back(f);
  }
  int n = xs.size();
  float* dx; uint32_t *dh, *ds;
  hipMalloc(&dx, n * 4); hipMalloc(&dh, n * 4); hipMalloc(&ds, n * 4);
  hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
  probe<<<(n + 255) / 256, 256>>>(dx, n, dh, ds);
  std::vector<uint32_t> h(n), w(n);
  hipMemcpy(h.data(), dh, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(w.data(), ds, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i)
    if (h[i] != w[i]) {
      if (bad < 12) printf("x=%.9g hw=%u sw=%u\n", xs[i], h[i], w[i]);
      ++bad;
    }
  printf("values %d mismatches %d\n", n, bad);
  hipFree(dx); hipFree(dh); hipFree(ds);
  return 0;
}
