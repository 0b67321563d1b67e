// FETCH_SIZE calibration for the access widths the tree kernels use: one
// pass over a buffer of known size with (a) 4 B/lane coalesced dword loads
// (stage_bins' X reads), (b) 16 B/lane loads (the guide's calibrated case).
// Run under: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void read_dword(const float* __restrict__ x, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += x[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}

__global__ void read_dwordx4(const float4* __restrict__ x, size_t n4, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
  const size_t sizes[2] = {112u << 20, 1024u << 20};
  float* out;
  if (hipMalloc(&out, 4096) != hipSuccess) return 1;
  for (size_t bytes : sizes) {
    float* x;
    if (hipMalloc(&x, bytes) != hipSuccess) return 1;
    if (hipMemset(x, 0, bytes) != hipSuccess) return 1;
    const size_t n = bytes / 4;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(read_dword, dim3(4096), dim3(256), 0, 0, x, n, out);
      hipLaunchKernelGGL(read_dwordx4, dim3(4096), dim3(256), 0, 0,
                         reinterpret_cast<const float4*>(x), n / 4, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::printf("bytes %zu\n", bytes);
    (void)hipFree(x);
  }
  (void)hipFree(out);
  return 0;
}
