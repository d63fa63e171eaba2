// Persistent-kernel primitive costs on one MI355X (round 6 calibration for gs_bfs_pers.hip):
// G workgroups of 1024 threads (one per CU, LDS-limited), 200 iterations of
//   [sc1 stores of a slot row by 256 threads] -> grid barrier -> [one sc1 load per thread
//   of another workgroup's row] -> [one plain random 64-B row load per thread from 128 MB]
//   -> [one returning agent atomicAdd by thread 0]
// Thread 0 of each workgroup sums each phase's wall clock (100 MHz) and the host prints the
// mean per iteration over workgroups (and the max over workgroups).
// usage: pbar [spread]   spread = 1: barrier words on separate 256-B lines (else packed 64 B)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ inline void grid_sync(uint32_t* bar, uint32_t e, uint32_t G, uint32_t str, uint32_t* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t sh = blockIdx.x & 7u, ns = min(G, 8u), cs = (G - sh + 7u) / 8u;
    const uint32_t r = __hip_atomic_fetch_add(&bar[str * sh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r + 1u == e * cs) {
      const uint32_t t = __hip_atomic_fetch_add(&bar[str * 8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == e * ns) __hip_atomic_store(&bar[str * 9], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (uint32_t it = 0; __hip_atomic_load(&bar[str * 9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e; ++it) {
      if (it > (1u << 22)) { atomicOr(err, 1u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024, 1) void k_prim(uint32_t* bar, uint32_t str, uint32_t* rows, const uint4* big,
                                                  uint32_t bigmask, uint32_t* ctr, unsigned long long* out,
                                                  uint32_t iters, uint32_t* err) {
  extern __shared__ uint32_t lds[];
  const uint32_t tid = threadIdx.x, g = blockIdx.x, G = gridDim.x;
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0}, mx = 0;
  uint32_t x = tid * 7919u + g;
  lds[tid] = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    unsigned long long t0 = wall_clock64();
    if (tid < 256) __hip_atomic_store(&rows[(size_t)tid * 1024 + (it & 1) * 512 + g], x + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    unsigned long long t1 = wall_clock64();
    grid_sync(bar, it + 1, G, str, err);
    unsigned long long t2 = wall_clock64();
    // another workgroup's word, sc1
    const uint32_t src = (g + 1 + it) % G;
    uint32_t v = 0;
    if (tid < 64) v = __hip_atomic_load(&rows[(size_t)tid * 1024 + (it & 1) * 512 + src], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds[tid] += v;
    __syncthreads();
    unsigned long long t3 = wall_clock64();
    // one random 16-B row load per thread (plain)
    x = x * 1664525u + 1013904223u;
    const uint4 r = big[(x >> 4) & bigmask];
    lds[tid] += r.x ^ r.w;
    __syncthreads();
    unsigned long long t4 = wall_clock64();
    // one returning agent atomic by thread 0
    if (tid == 0) lds[1] += atomicAdd(&ctr[it & 255], 1u);
    __syncthreads();
    unsigned long long t5 = wall_clock64();
    // empty barrier: syncthreads only
    __syncthreads();
    unsigned long long t6 = wall_clock64();
    acc[0] += t1 - t0; acc[1] += t2 - t1; acc[2] += t3 - t2; acc[3] += t4 - t3; acc[4] += t5 - t4; acc[5] += t6 - t5;
    mx = max(mx, t2 - t1);
  }
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) out[g * 8 + k] = acc[k];
    out[g * 8 + 6] = mx;
    out[g * 8 + 7] = lds[5];
  }
}

int main(int argc, char** argv) {
  const uint32_t spread = argc > 1 ? atoi(argv[1]) : 0;
  int cus = 0;
  HC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t G = cus >= 256 ? 256 : 128, iters = 200, str = spread ? 64 : 16;
  uint32_t *bar, *rows, *ctr, *err;
  uint4* big;
  unsigned long long* out;
  const size_t bigN = (128u << 20) / 16;
  HC(hipMalloc(&bar, 4096)); HC(hipMemset(bar, 0, 4096));
  HC(hipMalloc(&rows, 256 * 1024 * 4)); HC(hipMemset(rows, 0, 256 * 1024 * 4));
  HC(hipMalloc(&ctr, 1024)); HC(hipMemset(ctr, 0, 1024));
  HC(hipMalloc(&err, 4)); HC(hipMemset(err, 0, 4));
  HC(hipMalloc(&big, bigN * 16)); HC(hipMemset(big, 1, bigN * 16));
  HC(hipMalloc(&out, G * 64));
  const size_t lds = 144 * 1024;
  HC(hipFuncSetAttribute((const void*)k_prim, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int rep = 0; rep < 3; ++rep) {
    HC(hipMemset(bar, 0, 4096));
    hipLaunchKernelGGL(k_prim, dim3(G), dim3(1024), lds, 0, bar, str, rows, big, (uint32_t)(bigN - 1), ctr, out, iters, err);
    HC(hipDeviceSynchronize());
  }
  std::vector<unsigned long long> h(G * 8);
  uint32_t he = 0;
  HC(hipMemcpy(h.data(), out, G * 64, hipMemcpyDeviceToHost));
  HC(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
  const char* nm[6] = {"sc1 stores+sync", "grid barrier", "sc1 load after barrier", "plain random 16B load",
                       "returning atomic (t0)", "empty syncthreads"};
  printf("G=%u spread=%u err=%u (us per iteration, mean over workgroups / max)\n", G, spread, he);
  for (int k = 0; k < 6; ++k) {
    double s = 0, m = 0;
    for (uint32_t g = 0; g < G; ++g) { s += h[g * 8 + k]; m = std::max(m, (double)h[g * 8 + k]); }
    printf("  %-26s %7.3f  %7.3f\n", nm[k], s / G / iters / 100.0, m / iters / 100.0);
  }
  double mxb = 0;
  for (uint32_t g = 0; g < G; ++g) mxb = std::max(mxb, (double)h[g * 8 + 6]);
  printf("  max single barrier %.2f us\n", mxb / 100.0);
  return 0;
}
