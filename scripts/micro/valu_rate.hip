// Issue rate of candidate VALU ops for the tree walk, wave64 on gfx950: 8
// independent chains per lane, 8 waves per SIMD; prints cycles per
// wave-instruction per SIMD at the reported clock.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X X X X X X X X
template <int OP>
__global__ void __launch_bounds__(256) k(unsigned* out, int iters, unsigned m) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, y = m ^ threadIdx.x, z = y * 3u;
  unsigned long long sm = 0;
  asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(y), "v"(z) : "vcc");
  asm volatile("v_cmp_lt_u32 %0, %1, %2" : "=s"(sm) : "v"(y), "v"(z));
  for (int i = 0; i < iters; ++i) {
#define STEP(r)                                                                                  \
    if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(y));                         \
    if (OP == 1) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(y));                          \
    if (OP == 2) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(r));                               \
    if (OP == 3) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(y) : "vcc");        \
    if (OP == 4) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r) : "v"(y), "s"(sm));    \
    if (OP == 5) asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(r), "v"(y) : "vcc");              \
    if (OP == 6) asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(sm) : "v"(r), "v"(y));          \
    if (OP == 7) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(r) : "v"(y)); \
    if (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r) : "v"(z), "v"(y));          \
    if (OP == 9) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r) : "v"(y));                     \
    if (OP == 10) asm volatile("v_mad_u32_u24 %0, %0, 2, %1" : "+v"(r) : "v"(y));                 \
    if (OP == 11) asm volatile("v_lshrrev_b32 %0, 16, %0" : "+v"(r));                             \
    if (OP == 12) asm volatile("v_and_b32 %0, 0x7fff, %0" : "+v"(r));                             \
    if (OP == 13) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(r) :: "vcc");          \
    if (OP == 14) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(y));                   \
    if (OP == 15) asm volatile("v_cmp_lt_u32_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:DWORD" :: "v"(r), "v"(y) : "vcc"); \
    if (OP == 16) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(r) : "v"(y));                \
    if (OP == 17) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(r) : "v"(y));                        \
    if (OP == 18) asm volatile("v_cmp_lt_u16 vcc, %0, %1" :: "v"(r), "v"(y) : "vcc");             \
    if (OP == 19) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(y));                            \
    if (OP == 20) asm volatile("v_max_u32 %0, %0, %1" : "+v"(r) : "v"(y));                        \
    if (OP == 21) asm volatile("v_bfe_u32 %0, %0, 16, 16" : "+v"(r));
    REP8(STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7))
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)sm;
}

template <int OP>
void run(const char* name, unsigned* d, int cus, int wg_per_cu) {
  const int iters = 1000, blocks = cus * wg_per_cu;
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 10, 1u);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  int clk_khz;
  (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double insts_per_simd = (double)blocks * 4 / (cus * 4) * iters * 64;
  const double cycles = ms * 1e-3 * clk_khz * 1e3;
  printf("%-34s waves/SIMD %d  %.2f cycles/wave-instr/SIMD\n", name, wg_per_cu,
         cycles / insts_per_simd);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  unsigned* d;
  (void)hipMalloc(&d, 1 << 26);
  const int c = p.multiProcessorCount;
  for (int w : {8, 2}) {
    run<0>("v_add_u32", d, c, w);
    run<1>("v_or_b32", d, c, w);
    run<2>("v_lshlrev_b32", d, c, w);
    run<3>("v_cndmask_b32 vcc", d, c, w);
    run<4>("v_cndmask_b32_e64 sgpr", d, c, w);
    run<5>("v_cmp_lt_u32 vcc (e32)", d, c, w);
    run<6>("v_cmp_lt_u32_e64 sgpr", d, c, w);
    run<7>("v_add_u32_sdwa WORD_1", d, c, w);
    run<8>("v_and_or_b32", d, c, w);
    run<9>("v_mul_u32_u24", d, c, w);
    run<10>("v_mad_u32_u24", d, c, w);
    run<11>("v_lshrrev_b32", d, c, w);
    run<12>("v_and_b32 literal", d, c, w);
    run<13>("v_addc_co_u32 vcc", d, c, w);
    run<14>("v_add3_u32", d, c, w);
    run<15>("v_cmp_lt_u32_sdwa", d, c, w);
    run<16>("v_lshl_add_u32", d, c, w);
    run<17>("v_sub_u32", d, c, w);
    run<18>("v_cmp_lt_u16 vcc", d, c, w);
    run<19>("v_mov_b32", d, c, w);
    run<20>("v_max_u32", d, c, w);
    run<21>("v_bfe_u32", d, c, w);
  }
  return 0;
}
