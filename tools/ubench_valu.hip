// Issue-rate probe for the VALU ops the SAD kernels use (gfx950):
// 8 independent chains per wave, 256-thread blocks, 16 blocks/CU-worth of grid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ unsigned long long g_clk[4];
template <int OP, bool SOP>
__global__ __launch_bounds__(256) void k(uint32_t seed, int iters, uint32_t* out) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t s0 = SOP ? __builtin_amdgcn_readfirstlane(seed * 7 + blockIdx.x) : seed * 7 + threadIdx.x;
  uint32_t s1 = SOP ? __builtin_amdgcn_readfirstlane(seed * 13 + 1) : seed * 13 + threadIdx.x * 3;
  uint32_t r[8], a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { r[j] = (threadIdx.x + 37 * j) * 0x01010101u ^ (j * 0x1f2e3d4c); a[j] = j; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
#pragma unroll
      for (int j = 0; j < 8; j++) {
        uint32_t x = r[(u + j) & 7], y = (j & 1) ? s1 : s0;
        if (OP == 0) a[j] = __builtin_amdgcn_sad_u8(x, y, a[j]);
        if (OP == 1) a[j] = x + a[j] + y;                       // v_add3_u32
        if (OP == 2) a[j] = __builtin_amdgcn_udot4(x, y, a[j], false);
        if (OP == 3) a[j] = __builtin_amdgcn_msad_u8(x, y, a[j]);
        if (OP == 4) a[j] = __builtin_amdgcn_alignbyte(x, a[j], y);
        if (OP == 5) a[j] = __builtin_amdgcn_sad_hi_u8(x, y, a[j]);
        if (OP == 6) a[j] = __builtin_amdgcn_sad_u16(x, y, a[j]);
        if (OP == 7) a[j] = __mul24((int)x, (int)a[j]) ;
        if (OP == 8) a[j] = x ^ a[j];
        if (OP == 9) a[j] = __builtin_amdgcn_qsad_pk_u16_u8(((uint64_t)x << 32) | y, y, a[j]);
        if (OP == 10) asm("v_pk_add_u16 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 11) asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 12) asm("v_add_u32_e64 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 13) asm("v_med3_i32 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 14) asm("v_add_u32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 15) asm("v_cvt_f32_i32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j] ^ x));
        if (OP == 16) asm("v_mul_f32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 17) asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 18) asm("v_pk_lshrrev_b16 %0, 1, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 19) asm("v_bfe_u32 %0, %1, 3, 7" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 20) asm("v_mul_u32_u24_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 21) asm("v_ashrrev_i32_e32 %0, 3, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 22) asm("v_ashrrev_i32_e64 %0, 3, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 23) asm("v_cndmask_b32_e64 %0, %1, %2, s[0:1]" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 24) asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 25) asm("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 26) a[j] = __builtin_amdgcn_lerp(x, a[j], 0u);
        if (OP == 27) asm("v_perm_b32 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(a[j]), "v"(y));
        if (OP == 28) asm("v_cndmask_b32_e32 %0, %1, %2, vcc" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 29) asm("v_add_u32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 30) asm("v_fma_f32 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 31) asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 32) asm("v_min_u32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 33) asm("v_cmp_gt_i32_e64 s[2:3], %1, %2\n v_cndmask_b32_e64 %0, %1, %2, s[2:3]" : "=v"(a[j]) : "v"(x), "v"(a[j]) : "s2", "s3");
        if (OP == 34) asm("v_cvt_i32_f32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j] ^ x));
        if (OP == 35) asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(*(uint64_t*)&a[j & 6]) : "v"(((uint64_t)x << 32) | y), "v"(((uint64_t)y << 32) | x), "v"(*(uint64_t*)&a[j & 6]));
        if (OP == 36) asm("v_lshrrev_b32_e32 %0, 8, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 37) asm("v_sad_u8 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(r[(u + j + 3) & 7]), "v"(a[j]));
        if (OP == 38) asm("v_floor_f32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 39) asm("v_trunc_f32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 40) asm("v_cvt_f32_ubyte1_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 41) asm("v_cvt_pk_u8_f32 %0, %1, 1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 42) asm("v_med3_f32 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 43) asm("v_max_f32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 44) asm("v_add_f32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 45) asm("v_sub_f32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 46) asm("v_rndne_f32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 47) asm("v_cvt_i32_f32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 48) asm("v_cvt_f32_i32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 49) asm("v_and_b32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 50) asm("v_or_b32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 51) asm("v_max_i32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 52) asm("v_dot2c_i32_i16_e32 %0, %1, %2" : "+v"(a[j]) : "v"(x), "v"(y));
        if (OP == 53) asm("v_dot2c_i32_i16_e32 %0, 0xfe27016a, %1" : "+v"(a[j]) : "v"(x));
        if (OP == 54) asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(a[j]) : "v"(x), "v"(y), "v"(a[j]));
        if (OP == 55) asm("v_pk_sub_i16 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 56) asm("v_pk_ashrrev_i16 %0, 1, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 57) asm("v_sat_pk_u8_i16_e32 %0, %1" : "=v"(a[j]) : "v"(a[j] ^ x));
        if (OP == 58) asm("v_mul_lo_u32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 59) asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 60) asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 61) asm("v_mul_i32_i24_e32 %0, 0x16a, %1" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 62) asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 63) asm("v_sub_u32_e32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 64) asm("v_mad_u64_u32 %0, s[2:3], %1, %2, %3" : "=v"(*(uint64_t*)&a[j & 6]) : "v"(x), "v"(a[(j + 1) & 7]), "v"(*(uint64_t*)&a[j & 6]) : "s2", "s3");
        if (OP == 65) asm("v_pk_min_i16 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 66) asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 67) asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 68) asm("v_mul_i32_i24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "=v"(a[j]) : "v"(x), "v"(a[j]));
        if (OP == 69) asm("v_mov_b32_e32 %0, %1" : "=v"(a[j]) : "v"(a[j] ^ x));
        if (OP == 70) asm("v_bfe_i32 %0, %1, 0, 16" : "=v"(a[j]) : "v"(a[j]));
        if (OP == 71) asm("v_mul_hi_u32 %0, %1, %2" : "=v"(a[j]) : "v"(x), "v"(a[j]));
      }
    asm volatile("" : "+v"(r[0]), "+v"(r[3]));
  }
  uint32_t t = 0;
  for (int j = 0; j < 8; j++) t += a[j];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if (blockIdx.x == 17 && threadIdx.x == 0) {
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    g_clk[0] = t1 - t0;
    g_clk[1] = r1 - r0;
  }
}

template <int OP, bool SOP>
void run(const char* name, uint32_t* d) {
  int blocks = 256 * 16, iters = 1000;
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 4; rep++) {
    (void)hipEventRecord(e0);
    k<OP, SOP><<<blocks, 256>>>(1, iters, d);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  double winstr = (double)blocks * 4 * iters * 64;
  double per_simd = winstr / 1024 / (best * 1e-3);
  unsigned long long c[2];
  (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_clk), sizeof c);
  double ghz = (double)c[0] / (double)c[1] * 0.1;
  printf("%-20s %s  %.3f ms  %.3f Twave-instr/s  block clock %.2f GHz  %.2f cycles/instr/SIMD at that clock\n",
         name, SOP ? "sgpr" : "vgpr", best, winstr / best / 1e9, ghz, ghz * 1e9 / per_simd);
}

int main(int argc, char** argv) {
  uint32_t* d; (void)hipMalloc(&d, 256 * 4096 * 4 * 4);
  if (argc > 1) {  // only the later additions (and the PMC calibration pair)
    run<1, false>("v_add3_u32", d);
    run<64, false>("v_mad_u64_u32", d);
    run<65, false>("v_pk_min_i16", d);
    run<66, false>("v_pk_mul_lo_u16", d);
    run<67, false>("v_add_u32_sdwa", d);
    run<68, false>("v_mul_i32_i24_sdwa", d);
    run<69, false>("v_mov_b32+xor", d);
    run<70, false>("v_bfe_i32", d);
    run<71, false>("v_mul_hi_u32", d);
    run<29, false>("v_add_u32_e32", d);
    run<58, false>("v_mul_lo_u32", d);
    return 0;
  }
  run<1, false>("v_add3_u32", d);
  run<0, true>("v_sad_u8", d);
  run<0, false>("v_sad_u8", d);
  run<3, true>("v_msad_u8", d);
  run<5, true>("v_sad_hi_u8", d);
  run<6, true>("v_sad_u16", d);
  run<2, true>("v_dot4_u32_u8", d);
  run<4, false>("v_alignbyte_b32", d);
  run<7, false>("v_mul_i32_i24", d);
  run<8, false>("v_xor_b32", d);
  run<9, true>("v_qsad_pk_u16_u8", d);
  run<10, false>("v_pk_add_u16", d);
  run<11, false>("v_pk_mad_u16", d);
  run<12, false>("v_add_u32_e64", d);
  run<13, false>("v_med3_i32", d);
  run<14, false>("v_add_u32_dpp", d);
  run<15, false>("v_cvt_f32_i32+xor", d);
  run<16, false>("v_mul_f32", d);
  run<17, false>("v_lshl_add_u32", d);
  run<18, false>("v_pk_lshrrev_b16", d);
  run<19, false>("v_bfe_u32", d);
  run<20, false>("v_mul_u32_u24_e32", d);
  run<21, false>("v_ashrrev_i32_e32", d);
  run<22, false>("v_ashrrev_i32_e64", d);
  run<23, false>("v_cndmask_b32_e64", d);
  run<24, false>("v_mad_i32_i24", d);
  run<25, false>("v_mov_b32_dpp", d);
  run<26, false>("v_lerp_u8", d);
  run<27, false>("v_perm_b32", d);
  run<28, false>("v_cndmask_b32_e32", d);
  run<29, false>("v_add_u32_e32", d);
  run<30, false>("v_fma_f32", d);
  run<31, false>("v_bfi_b32", d);
  run<32, false>("v_min_u32_e32", d);
  run<33, false>("cmp_e64+cndmask_e64", d);
  run<34, false>("v_cvt_i32_f32+xor", d);
  run<35, false>("v_pk_fma_f32", d);
  run<36, false>("v_lshrrev_b32_e32", d);
  run<37, false>("v_sad_u8 (3 vgpr)", d);
  run<38, false>("v_floor_f32", d);
  run<39, false>("v_trunc_f32", d);
  run<40, false>("v_cvt_f32_ubyte1", d);
  run<41, false>("v_cvt_pk_u8_f32", d);
  run<42, false>("v_med3_f32", d);
  run<43, false>("v_max_f32", d);
  run<44, false>("v_add_f32", d);
  run<45, false>("v_sub_f32", d);
  run<46, false>("v_rndne_f32", d);
  run<47, false>("v_cvt_i32_f32", d);
  run<48, false>("v_cvt_f32_i32", d);
  run<49, false>("v_and_b32", d);
  run<50, false>("v_or_b32", d);
  run<51, false>("v_max_i32", d);
  run<52, false>("v_dot2c_i32_i16_e32", d);
  run<53, false>("v_dot2c_i32_i16 lit", d);
  run<54, false>("v_dot2_i32_i16 (vop3p)", d);
  run<55, false>("v_pk_sub_i16", d);
  run<56, false>("v_pk_ashrrev_i16", d);
  run<57, false>("v_sat_pk_u8_i16+xor", d);
  run<58, false>("v_mul_lo_u32", d);
  run<59, false>("v_cvt_pk_i16_i32", d);
  run<60, false>("v_lshl_or_b32", d);
  run<61, false>("v_mul_i32_i24 lit", d);
  run<62, false>("v_pk_add_u16 op_sel", d);
  run<63, false>("v_sub_u32_e32", d);
  return 0;
}
