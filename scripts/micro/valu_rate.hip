// Issue rate of the VALU instructions the tree walks are made of, wave64 on
// gfx950: 8 independent chains per lane, W waves per SIMD (256-thread
// workgroups = one wave per SIMD each, W workgroups per CU).  Each round of
// the 8 chains is ONE asm statement: hipcc pads hazards only between
// statements (cdna_hip_programming.md 5.7), so nothing but the named
// instructions runs.  Cycles are the chip's own: every workgroup's wave 0
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its
// loop, so the effective clock is d(memtime) / d(memrealtime) x 100 MHz
// (MI355X_MICROARCH.md "DVFS give-back" item 6) and
//   cycles per step per SIMD = d(memtime) / (W x steps per wave)   (stamped)
// The kernel's event time gives the same figure from the whole launch
// (wall x clock x SIMDs / steps), a check on the stamped one.  One JSON line
// per (op, W), medians over workgroups.
//
// The "step" rows time the binned-heap walk steps as the walk issues them
// (independent trees): round 2's 5-VALU step and the fixed-layout 4-VALU
// step, with the compare mask in VCC or in an SGPR pair; their cycles per
// step price bench.py's `peak_mix`.
//
// (The 8-chain asm strings were written out by a throw-away generator.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define ROUND_OPERANDS                                                                          \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(i0), \
    "+v"(i1), "+v"(i2), "+v"(i3), "+v"(i4), "+v"(i5), "+v"(i6), "+v"(i7), "=&v"(z), "+s"(sm)   \
  : "v"(y), "s"(m), "v"(lane)                                                                   \
  : "vcc"

template <int OP>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned long long* stamps, int iters,
                                         unsigned m) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, y = m ^ threadIdx.x, z = y * 3u, lane = threadIdx.x * 4u;
  unsigned i0 = 1, i1 = 2, i2 = 3, i3 = 4, i4 = 5, i5 = 6, i6 = 7, i7 = 8;
  unsigned long long sm = 0;
  asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(y), "v"(z) : "vcc");
  asm volatile("v_cmp_lt_u32 %0, %1, %2" : "=s"(sm) : "v"(y), "v"(z));
  unsigned long long t0, r0;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %18\n\tv_add_u32 %1, %1, %18\n\tv_add_u32 %2, %2, %18\n\tv_add_u32 %3, %3, %18\n\tv_add_u32 %4, %4, %18\n\tv_add_u32 %5, %5, %18\n\tv_add_u32 %6, %6, %18\n\tv_add_u32 %7, %7, %18" ROUND_OPERANDS);
      if (OP == 1) asm volatile("v_or_b32 %0, %0, %18\n\tv_or_b32 %1, %1, %18\n\tv_or_b32 %2, %2, %18\n\tv_or_b32 %3, %3, %18\n\tv_or_b32 %4, %4, %18\n\tv_or_b32 %5, %5, %18\n\tv_or_b32 %6, %6, %18\n\tv_or_b32 %7, %7, %18" ROUND_OPERANDS);
      if (OP == 2) asm volatile("v_lshlrev_b32 %0, 1, %0\n\tv_lshlrev_b32 %1, 1, %1\n\tv_lshlrev_b32 %2, 1, %2\n\tv_lshlrev_b32 %3, 1, %3\n\tv_lshlrev_b32 %4, 1, %4\n\tv_lshlrev_b32 %5, 1, %5\n\tv_lshlrev_b32 %6, 1, %6\n\tv_lshlrev_b32 %7, 1, %7" ROUND_OPERANDS);
      if (OP == 3) asm volatile("v_cndmask_b32 %0, %0, %18, vcc\n\tv_cndmask_b32 %1, %1, %18, vcc\n\tv_cndmask_b32 %2, %2, %18, vcc\n\tv_cndmask_b32 %3, %3, %18, vcc\n\tv_cndmask_b32 %4, %4, %18, vcc\n\tv_cndmask_b32 %5, %5, %18, vcc\n\tv_cndmask_b32 %6, %6, %18, vcc\n\tv_cndmask_b32 %7, %7, %18, vcc" ROUND_OPERANDS);
      if (OP == 4) asm volatile("v_cndmask_b32_e64 %0, %0, %18, %17\n\tv_cndmask_b32_e64 %1, %1, %18, %17\n\tv_cndmask_b32_e64 %2, %2, %18, %17\n\tv_cndmask_b32_e64 %3, %3, %18, %17\n\tv_cndmask_b32_e64 %4, %4, %18, %17\n\tv_cndmask_b32_e64 %5, %5, %18, %17\n\tv_cndmask_b32_e64 %6, %6, %18, %17\n\tv_cndmask_b32_e64 %7, %7, %18, %17" ROUND_OPERANDS);
      if (OP == 5) asm volatile("v_cmp_lt_u32 vcc, %0, %18\n\tv_cmp_lt_u32 vcc, %1, %18\n\tv_cmp_lt_u32 vcc, %2, %18\n\tv_cmp_lt_u32 vcc, %3, %18\n\tv_cmp_lt_u32 vcc, %4, %18\n\tv_cmp_lt_u32 vcc, %5, %18\n\tv_cmp_lt_u32 vcc, %6, %18\n\tv_cmp_lt_u32 vcc, %7, %18" ROUND_OPERANDS);
      if (OP == 6) asm volatile("v_cmp_lt_u32_e64 %17, %0, %18\n\tv_cmp_lt_u32_e64 %17, %1, %18\n\tv_cmp_lt_u32_e64 %17, %2, %18\n\tv_cmp_lt_u32_e64 %17, %3, %18\n\tv_cmp_lt_u32_e64 %17, %4, %18\n\tv_cmp_lt_u32_e64 %17, %5, %18\n\tv_cmp_lt_u32_e64 %17, %6, %18\n\tv_cmp_lt_u32_e64 %17, %7, %18" ROUND_OPERANDS);
      if (OP == 7) asm volatile("v_add_u32_sdwa %0, %0, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %1, %1, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %2, %2, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %3, %3, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %4, %4, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %5, %5, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %6, %6, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\tv_add_u32_sdwa %7, %7, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" ROUND_OPERANDS);
      if (OP == 8) asm volatile("v_and_or_b32 %0, %0, %19, %20\n\tv_and_or_b32 %1, %1, %19, %20\n\tv_and_or_b32 %2, %2, %19, %20\n\tv_and_or_b32 %3, %3, %19, %20\n\tv_and_or_b32 %4, %4, %19, %20\n\tv_and_or_b32 %5, %5, %19, %20\n\tv_and_or_b32 %6, %6, %19, %20\n\tv_and_or_b32 %7, %7, %19, %20" ROUND_OPERANDS);
      if (OP == 9) asm volatile("v_mul_u32_u24 %0, %0, %18\n\tv_mul_u32_u24 %1, %1, %18\n\tv_mul_u32_u24 %2, %2, %18\n\tv_mul_u32_u24 %3, %3, %18\n\tv_mul_u32_u24 %4, %4, %18\n\tv_mul_u32_u24 %5, %5, %18\n\tv_mul_u32_u24 %6, %6, %18\n\tv_mul_u32_u24 %7, %7, %18" ROUND_OPERANDS);
      if (OP == 10) asm volatile("v_lshrrev_b32 %0, 16, %0\n\tv_lshrrev_b32 %1, 16, %1\n\tv_lshrrev_b32 %2, 16, %2\n\tv_lshrrev_b32 %3, 16, %3\n\tv_lshrrev_b32 %4, 16, %4\n\tv_lshrrev_b32 %5, 16, %5\n\tv_lshrrev_b32 %6, 16, %6\n\tv_lshrrev_b32 %7, 16, %7" ROUND_OPERANDS);
      if (OP == 11) asm volatile("v_and_b32 %0, 0x7f8, %0\n\tv_and_b32 %1, 0x7f8, %1\n\tv_and_b32 %2, 0x7f8, %2\n\tv_and_b32 %3, 0x7f8, %3\n\tv_and_b32 %4, 0x7f8, %4\n\tv_and_b32 %5, 0x7f8, %5\n\tv_and_b32 %6, 0x7f8, %6\n\tv_and_b32 %7, 0x7f8, %7" ROUND_OPERANDS);
      if (OP == 12) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc\n\tv_addc_co_u32 %1, vcc, %1, %1, vcc\n\tv_addc_co_u32 %2, vcc, %2, %2, vcc\n\tv_addc_co_u32 %3, vcc, %3, %3, vcc\n\tv_addc_co_u32 %4, vcc, %4, %4, vcc\n\tv_addc_co_u32 %5, vcc, %5, %5, vcc\n\tv_addc_co_u32 %6, vcc, %6, %6, vcc\n\tv_addc_co_u32 %7, vcc, %7, %7, vcc" ROUND_OPERANDS);
      if (OP == 13) asm volatile("v_cmp_lt_u32_sdwa vcc, %0, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %1, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %2, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %3, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %4, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %5, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %6, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cmp_lt_u32_sdwa vcc, %7, %18 src0_sel:WORD_1 src1_sel:DWORD" ROUND_OPERANDS);
      if (OP == 14) asm volatile("v_lshl_add_u32 %0, %0, 3, %18\n\tv_lshl_add_u32 %1, %1, 3, %18\n\tv_lshl_add_u32 %2, %2, 3, %18\n\tv_lshl_add_u32 %3, %3, 3, %18\n\tv_lshl_add_u32 %4, %4, 3, %18\n\tv_lshl_add_u32 %5, %5, 3, %18\n\tv_lshl_add_u32 %6, %6, 3, %18\n\tv_lshl_add_u32 %7, %7, 3, %18" ROUND_OPERANDS);
      if (OP == 15) asm volatile("v_mov_b32 %0, %18\n\tv_mov_b32 %1, %18\n\tv_mov_b32 %2, %18\n\tv_mov_b32 %3, %18\n\tv_mov_b32 %4, %18\n\tv_mov_b32 %5, %18\n\tv_mov_b32 %6, %18\n\tv_mov_b32 %7, %18" ROUND_OPERANDS);
      if (OP == 16) asm volatile("v_bfe_u32 %0, %0, 16, 16\n\tv_bfe_u32 %1, %1, 16, 16\n\tv_bfe_u32 %2, %2, 16, 16\n\tv_bfe_u32 %3, %3, 16, 16\n\tv_bfe_u32 %4, %4, 16, 16\n\tv_bfe_u32 %5, %5, 16, 16\n\tv_bfe_u32 %6, %6, 16, 16\n\tv_bfe_u32 %7, %7, 16, 16" ROUND_OPERANDS);
      if (OP == 17) asm volatile("v_and_or_b32 %16, %0, %19, %20\n\tv_lshl_add_u32 %16, %8, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %0, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %0, %0, %18, vcc\n\tv_addc_co_u32 %8, vcc, %8, %8, vcc\n\tv_and_or_b32 %16, %1, %19, %20\n\tv_lshl_add_u32 %16, %9, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %1, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %1, %1, %18, vcc\n\tv_addc_co_u32 %9, vcc, %9, %9, vcc\n\tv_and_or_b32 %16, %2, %19, %20\n\tv_lshl_add_u32 %16, %10, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %2, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %2, %2, %18, vcc\n\tv_addc_co_u32 %10, vcc, %10, %10, vcc\n\tv_and_or_b32 %16, %3, %19, %20\n\tv_lshl_add_u32 %16, %11, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %3, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %3, %3, %18, vcc\n\tv_addc_co_u32 %11, vcc, %11, %11, vcc\n\tv_and_or_b32 %16, %4, %19, %20\n\tv_lshl_add_u32 %16, %12, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %4, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %4, %4, %18, vcc\n\tv_addc_co_u32 %12, vcc, %12, %12, vcc\n\tv_and_or_b32 %16, %5, %19, %20\n\tv_lshl_add_u32 %16, %13, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %5, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %5, %5, %18, vcc\n\tv_addc_co_u32 %13, vcc, %13, %13, vcc\n\tv_and_or_b32 %16, %6, %19, %20\n\tv_lshl_add_u32 %16, %14, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %6, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %6, %6, %18, vcc\n\tv_addc_co_u32 %14, vcc, %14, %14, vcc\n\tv_and_or_b32 %16, %7, %19, %20\n\tv_lshl_add_u32 %16, %15, 3, %20\n\tv_cmp_lt_u32_sdwa vcc, %7, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %7, %7, %18, vcc\n\tv_addc_co_u32 %15, vcc, %15, %15, vcc" ROUND_OPERANDS);
      if (OP == 18) asm volatile("v_and_or_b32 %16, %0, %19, %20\n\tv_and_b32 %16, 0x7f8, %0\n\tv_cmp_lt_u32_sdwa vcc, %0, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %0, %0, %18, vcc\n\tv_and_or_b32 %16, %1, %19, %20\n\tv_and_b32 %16, 0x7f8, %1\n\tv_cmp_lt_u32_sdwa vcc, %1, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %1, %1, %18, vcc\n\tv_and_or_b32 %16, %2, %19, %20\n\tv_and_b32 %16, 0x7f8, %2\n\tv_cmp_lt_u32_sdwa vcc, %2, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %2, %2, %18, vcc\n\tv_and_or_b32 %16, %3, %19, %20\n\tv_and_b32 %16, 0x7f8, %3\n\tv_cmp_lt_u32_sdwa vcc, %3, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %3, %3, %18, vcc\n\tv_and_or_b32 %16, %4, %19, %20\n\tv_and_b32 %16, 0x7f8, %4\n\tv_cmp_lt_u32_sdwa vcc, %4, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %4, %4, %18, vcc\n\tv_and_or_b32 %16, %5, %19, %20\n\tv_and_b32 %16, 0x7f8, %5\n\tv_cmp_lt_u32_sdwa vcc, %5, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %5, %5, %18, vcc\n\tv_and_or_b32 %16, %6, %19, %20\n\tv_and_b32 %16, 0x7f8, %6\n\tv_cmp_lt_u32_sdwa vcc, %6, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %6, %6, %18, vcc\n\tv_and_or_b32 %16, %7, %19, %20\n\tv_and_b32 %16, 0x7f8, %7\n\tv_cmp_lt_u32_sdwa vcc, %7, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32 %7, %7, %18, vcc" ROUND_OPERANDS);
      if (OP == 19) asm volatile("v_and_or_b32 %16, %0, %19, %20\n\tv_and_b32 %16, 0x7f8, %0\n\tv_cmp_lt_u32_sdwa %17, %0, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %0, %0, %18, %17\n\tv_and_or_b32 %16, %1, %19, %20\n\tv_and_b32 %16, 0x7f8, %1\n\tv_cmp_lt_u32_sdwa %17, %1, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %1, %1, %18, %17\n\tv_and_or_b32 %16, %2, %19, %20\n\tv_and_b32 %16, 0x7f8, %2\n\tv_cmp_lt_u32_sdwa %17, %2, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %2, %2, %18, %17\n\tv_and_or_b32 %16, %3, %19, %20\n\tv_and_b32 %16, 0x7f8, %3\n\tv_cmp_lt_u32_sdwa %17, %3, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %3, %3, %18, %17\n\tv_and_or_b32 %16, %4, %19, %20\n\tv_and_b32 %16, 0x7f8, %4\n\tv_cmp_lt_u32_sdwa %17, %4, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %4, %4, %18, %17\n\tv_and_or_b32 %16, %5, %19, %20\n\tv_and_b32 %16, 0x7f8, %5\n\tv_cmp_lt_u32_sdwa %17, %5, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %5, %5, %18, %17\n\tv_and_or_b32 %16, %6, %19, %20\n\tv_and_b32 %16, 0x7f8, %6\n\tv_cmp_lt_u32_sdwa %17, %6, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %6, %6, %18, %17\n\tv_and_or_b32 %16, %7, %19, %20\n\tv_and_b32 %16, 0x7f8, %7\n\tv_cmp_lt_u32_sdwa %17, %7, %18 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e64 %7, %7, %18, %17" ROUND_OPERANDS);
    }
  }
  unsigned long long t1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)sm ^ i0 ^ i1 ^ i2 ^ i3 ^ i4 ^ i5 ^ i6 ^ i7 ^ z;
  if (threadIdx.x == 0) {   // stamps go to a buffer of their own, never into out
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

template <int OP>
void run(const char* name, int insts_per_step, unsigned* d, unsigned long long* st, int cus, int w) {
  const int iters = 2000, blocks = cus * w;
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, st, 50, 1u);   // warm
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, st, iters, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * blocks);
  (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> cyc, clk;
  for (int b = 0; b < blocks; ++b) {
    cyc.push_back((double)h[2 * b]);
    clk.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);   // GHz (memrealtime: 100 MHz)
  }
  const double steps = (double)iters * 64;   // per wave: 8 rounds x 8 chains per iteration
  const double c_step = median(cyc) / (w * steps);
  const double ghz = median(clk);
  // whole launch: every SIMD ran w waves x steps; cycles = wall x clock
  const double c_wall = ms * 1e-3 * ghz * 1e9 / (w * steps);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"valu_per_step\": %d, "
         "\"cycles_per_step_per_simd\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f, "
         "\"cycles_per_step_per_simd_wall\": %.3f, \"clock_GHz\": %.3f, \"kernel_ms\": %.3f}\n",
         name, w, insts_per_step, c_step, c_step / insts_per_step, c_wall, ghz, ms);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  unsigned* d;
  unsigned long long* st;
  const int c = p.multiProcessorCount;
  (void)hipMalloc(&d, (size_t)c * 8 * 256 * 4);
  (void)hipMalloc(&st, (size_t)c * 8 * 16);
  for (int w : {8, 6, 4, 2}) {
    run<0>("v_add_u32", 1, d, st, c, w);
    run<1>("v_or_b32", 1, d, st, c, w);
    run<2>("v_lshlrev_b32", 1, d, st, c, w);
    run<3>("v_cndmask_b32 vcc", 1, d, st, c, w);
    run<4>("v_cndmask_b32_e64 sgpr", 1, d, st, c, w);
    run<5>("v_cmp_lt_u32 vcc (e32)", 1, d, st, c, w);
    run<6>("v_cmp_lt_u32_e64 sgpr", 1, d, st, c, w);
    run<7>("v_add_u32_sdwa WORD_1", 1, d, st, c, w);
    run<8>("v_and_or_b32 sgpr mask", 1, d, st, c, w);
    run<9>("v_mul_u32_u24", 1, d, st, c, w);
    run<10>("v_lshrrev_b32", 1, d, st, c, w);
    run<11>("v_and_b32 literal", 1, d, st, c, w);
    run<12>("v_addc_co_u32 vcc", 1, d, st, c, w);
    run<13>("v_cmp_lt_u32_sdwa", 1, d, st, c, w);
    run<14>("v_lshl_add_u32", 1, d, st, c, w);
    run<15>("v_mov_b32", 1, d, st, c, w);
    run<16>("v_bfe_u32", 1, d, st, c, w);
    run<17>("step r2 (and_or, lshl_add, cmp_sdwa, cndmask, addc)", 5, d, st, c, w);
    run<18>("step fixed (and_or, and, cmp_sdwa, cndmask)", 4, d, st, c, w);
    run<19>("step fixed sgpr mask (and_or, and, cmp_sdwa e64, cndmask e64)", 4, d, st, c, w);
  }
  return 0;
}
