// calib_fetch.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access widths the
// engine uses (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B/lane
// streaming reads). Each kernel moves a known number of bytes of a 1 GiB buffer
// (far beyond the 256 MiB Infinity Cache, so every line comes from HBM):
//   rd4     4 B per lane, coalesced (the cache-row and meta reads)
//   rd16    16 B per lane, coalesced (rows)
//   rd4s    4 B per lane, one lane per 128-B line (scattered single-word reads)
//   wr4     4 B per lane, coalesced stores
//   wr4s    4 B per lane, one lane per 128-B line (scattered single-word stores)
// rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) --kernel-trace -- ./calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
  if (s == 0x12345678u) out[0] = s;
}
__global__ void rd16(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}
__global__ void rd4s(const uint32_t* __restrict__ p, size_t lines, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
    s += p[i * 32];
  if (s == 0x12345678u) out[0] = s;
}
__global__ void wr4(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}
__global__ void wr4s(uint32_t* __restrict__ p, size_t lines) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
    p[i * 32] = (uint32_t)i;
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 4, lines = bytes / 128;
  uint32_t *buf = nullptr, *out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(buf, 1, bytes);
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(rd4, g, b, 0, 0, buf, n, out);
    hipLaunchKernelGGL(rd16, g, b, 0, 0, reinterpret_cast<const uint4*>(buf), n / 4, out);
    hipLaunchKernelGGL(rd4s, g, b, 0, 0, buf, lines, out);
    hipLaunchKernelGGL(wr4, g, b, 0, 0, buf, n);
    hipLaunchKernelGGL(wr4s, g, b, 0, 0, buf, lines);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("bytes touched per kernel: rd4 %zu rd16 %zu rd4s %zu (lines x 128) wr4 %zu wr4s %zu (lines x 128)\n",
              bytes, bytes, lines * 128, bytes, lines * 128);
  hipFree(buf);
  hipFree(out);
  return 0;
}
