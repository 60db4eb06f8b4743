// Cost of a device-wide barrier inside one persistent kernel vs one kernel
// launch per phase in a HIP graph (the decode step's launch chain), and a
// check that values stored by one workgroup before a barrier are seen by
// every other workgroup (other XCDs included) after it.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gridbar gridbar_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr long SPIN_LIMIT = 20000000;  // ~ seconds: a barrier that never opens ends the kernel

// bar[0] arrivals, bar[1] generation, bar[2] error flag
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned nblk, unsigned& gen, int mode) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned a = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (a == nblk - 1) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&bar[1], gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long n = 0;
      while (__hip_atomic_load(&bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (mode == 1) __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_LIMIT) { __hip_atomic_store(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
    }
  }
  ++gen;
  __syncthreads();
}

// relaxed form: no cache maintenance; the data exchanged across the barrier
// is stored / loaded with agent-scope relaxed atomics (L2 write-through /
// bypass), every store retired (s_waitcnt) before the arrival.  H > 1: the
// blocks arrive on one of H counters, the last of each group on the top one.
__device__ __forceinline__ void grid_barrier_relaxed(unsigned* bar, unsigned nblk, unsigned& gen, int H) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    bool last;
    if (H > 1) {
      const unsigned grp = blockIdx.x % H, gsz = (nblk - grp + H - 1) / H;
      const unsigned a = __hip_atomic_fetch_add(&bar[16 + 16 * grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = false;
      if (a == gsz - 1) {
        __hip_atomic_store(&bar[16 + 16 * grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)H - 1;
      }
    } else {
      last = __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
    }
    if (last) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      __hip_atomic_store(&bar[1], gen + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long n = 0;
      while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (++n > SPIN_LIMIT) { __hip_atomic_store(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
    }
  }
  ++gen;
  __syncthreads();
}

__global__ __launch_bounds__(512) void relaxed_kernel(unsigned* bar, int P, int H, float* buf,
                                                      unsigned* err, int check) {
  unsigned gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned nblk = gridDim.x;
  for (int p = 0; p < P; ++p) {
    if (check) {
      float* dst = buf + (long)(p & 1) * nblk * 512;
      __hip_atomic_store(&dst[blockIdx.x * 512 + threadIdx.x], (float)(blockIdx.x * 7 + p * 131 + threadIdx.x),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_barrier_relaxed(bar, nblk, gen, H);
    if (__hip_atomic_load(&bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    if (check) {
      const float* src = buf + (long)(p & 1) * nblk * 512;
      const unsigned other = (blockIdx.x + 37 + p) % nblk;
      const float v = __hip_atomic_load(&src[other * 512 + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v != (float)(other * 7 + p * 131 + threadIdx.x)) atomicAdd(err, 1u);
    }
  }
}

__global__ __launch_bounds__(512) void phases_kernel(unsigned* bar, int P, int mode, float* buf,
                                                     unsigned* err, int check) {
  unsigned gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned nblk = gridDim.x;
  for (int p = 0; p < P; ++p) {
    if (check) {
      float* dst = buf + (long)(p & 1) * nblk * 512;
      dst[blockIdx.x * 512 + threadIdx.x] = (float)(blockIdx.x * 7 + p * 131 + threadIdx.x);
    }
    grid_barrier(bar, nblk, gen, mode);
    if (bar[2]) return;
    if (check) {
      const float* src = buf + (long)(p & 1) * nblk * 512;
      const unsigned other = (blockIdx.x + 37 + p) % nblk;
      const float v = src[other * 512 + threadIdx.x];
      if (v != (float)(other * 7 + p * 131 + threadIdx.x)) atomicAdd(err, 1u);
    }
  }
}

__global__ __launch_bounds__(512) void empty_kernel(float* buf) {
  if (threadIdx.x == 0 && blockIdx.x == 100000) buf[0] = 1.f;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, phases_kernel, 512, 0));
  printf("CUs %d, resident phases_kernel blocks per CU %d\n", cus, occ);
  unsigned *bar, *err;
  float* buf;
  CK(hipMalloc(&bar, 1024));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&buf, 2L * 1024 * 512 * 4));
  CK(hipMemset(bar, 0, 1024));
  CK(hipMemset(err, 0, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int P = 42, REP = 50;
  for (int nb : {64, 128, 256}) {
    if (nb > cus * occ) continue;
    for (int mode = 0; mode < 2; ++mode)
      for (int check = 0; check < 2; ++check) {
        hipLaunchKernelGGL(phases_kernel, dim3(nb), dim3(512), 0, s, bar, P, mode, buf, err, check);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < REP; ++r)
          hipLaunchKernelGGL(phases_kernel, dim3(nb), dim3(512), 0, s, bar, P, mode, buf, err, check);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned hb[3], he = 0;
        CK(hipMemcpy(hb, bar, 12, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
        printf("blocks %3d sleep %d store/check %d: %.2f us per kernel of %d barriers, %.3f us per barrier; "
               "timeout flag %u, mismatches %u\n", nb, mode, check, 1000.f * ms / REP, P,
               1000.f * ms / REP / P, hb[2], he);
        if (hb[2]) return 1;
      }
  }
  for (int nb : {64, 128, 256})
    for (int H : {1, 8})
      for (int check = 0; check < 2; ++check) {
        hipLaunchKernelGGL(relaxed_kernel, dim3(nb), dim3(512), 0, s, bar, P, H, buf, err, check);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < REP; ++r)
          hipLaunchKernelGGL(relaxed_kernel, dim3(nb), dim3(512), 0, s, bar, P, H, buf, err, check);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned hb[3], he = 0;
        CK(hipMemcpy(hb, bar, 12, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
        printf("relaxed: blocks %3d groups %d store/check %d: %.3f us per barrier; timeout flag %u, mismatches %u\n",
               nb, H, check, 1000.f * ms / REP / P, hb[2], he);
        if (hb[2]) return 1;
      }
  // the same number of phases as separate launches captured in a graph
  for (int nb : {64, 256, 512}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int p = 0; p < P; ++p) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(512), 0, s, buf);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < REP; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph of %d empty launches (%d blocks): %.2f us per graph, %.3f us per launch\n", P, nb,
           1000.f * ms / REP, 1000.f * ms / REP / P);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
