// Vector-memory cost of a 64-lane gather by access width: every lane loads
// W = 4, 8 or 16 bytes at an independent random address (8 chains per lane)
// in a buffer that stays in L2 / MALL, or with 8 lanes sharing each 128-byte
// line.  Prints ns per wave-instruction and the implied CU cycles (2.4 GHz,
// 256 CUs) -- what one gather of the tree kernels costs the TA/TD path.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int W, bool SHARED>
__global__ void __launch_bounds__(256) gather(const unsigned char* __restrict__ buf, uint32_t mask,
                                              int iters, uint32_t* __restrict__ out) {
  uint32_t st[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) st[c] = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + c * 40503u;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      st[c] = st[c] * 1664525u + 1013904223u;
      uint32_t off;
      if (SHARED) {   // 8 lanes of a wave share a 128-B line
        const uint32_t grp = __builtin_amdgcn_readfirstlane(st[c]) ^ ((threadIdx.x & 63u) >> 3) * 0x9E3779B9u;
        off = ((grp * 128u) & mask) + (threadIdx.x & 7u) * 16u;
      } else {
        off = (st[c] * 16u) & mask;
      }
      if (W == 4) acc += *reinterpret_cast<const uint32_t*>(buf + off);
      if (W == 8) { const uint2 v = *reinterpret_cast<const uint2*>(buf + off); acc += v.x ^ v.y; }
      if (W == 16) { const uint4 v = *reinterpret_cast<const uint4*>(buf + off); acc += v.x ^ v.y ^ v.z ^ v.w; }
    }
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

template <int W, bool SHARED>
void run(const unsigned char* buf, uint32_t mask, uint32_t* out, const char* name, size_t bytes) {
  const int blocks = 256 * 16, iters = 64;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((gather<W, SHARED>), dim3(blocks), dim3(256), 0, 0, buf, mask, iters, out);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((gather<W, SHARED>), dim3(blocks), dim3(256), 0, 0, buf, mask, iters, out);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double insts = 5.0 * blocks * 4 * iters * 8;   // wave-instructions
  const double ns = ms * 1e6 / insts;
  printf("{\"width\": %d, \"lines\": \"%s\", \"buffer_MB\": %zu, \"ns_per_wave_inst\": %.4f, "
         "\"cu_cycles_per_inst\": %.1f}\n", W, name, bytes >> 20, ns, ns * 2.4 * 256);
}

int main() {
  uint32_t* out;
  if (hipMalloc(&out, 4096) != hipSuccess) return 1;
  for (size_t bytes : {size_t(2) << 20, size_t(16) << 20}) {
    unsigned char* buf;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
    const uint32_t mask = static_cast<uint32_t>(bytes - 1) & ~15u;
    run<4, false>(buf, mask, out, "distinct", bytes);
    run<8, false>(buf, mask, out, "distinct", bytes);
    run<16, false>(buf, mask, out, "distinct", bytes);
    run<4, true>(buf, mask, out, "8_per_line", bytes);
    run<8, true>(buf, mask, out, "8_per_line", bytes);
    run<16, true>(buf, mask, out, "8_per_line", bytes);
    (void)hipFree(buf);
  }
  return 0;
}
