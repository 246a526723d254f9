#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
__global__ __launch_bounds__(256) void k_bfe_i32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_bfe_i32 %0, %0, %8, 8\n\tv_bfe_i32 %1, %1, %8, 8\n\tv_bfe_i32 %2, %2, %8, 8\n\tv_bfe_i32 %3, %3, %8, 8\n\tv_bfe_i32 %4, %4, %8, 8\n\tv_bfe_i32 %5, %5, %8, 8\n\tv_bfe_i32 %6, %6, %8, 8\n\tv_bfe_i32 %7, %7, %8, 8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_u16 %0, %8, %0\n\tv_add_u16 %1, %8, %1\n\tv_add_u16 %2, %8, %2\n\tv_add_u16 %3, %8, %3\n\tv_add_u16 %4, %8, %4\n\tv_add_u16 %5, %8, %5\n\tv_add_u16 %6, %8, %6\n\tv_add_u16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_max_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max_i16 %0, %8, %0\n\tv_max_i16 %1, %8, %1\n\tv_max_i16 %2, %8, %2\n\tv_max_i16 %3, %8, %3\n\tv_max_i16 %4, %8, %4\n\tv_max_i16 %5, %8, %5\n\tv_max_i16 %6, %8, %6\n\tv_max_i16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_sub_u16_e64_clamp(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_sub_u16_e64 %0, %0, %8 clamp\n\tv_sub_u16_e64 %1, %1, %8 clamp\n\tv_sub_u16_e64 %2, %2, %8 clamp\n\tv_sub_u16_e64 %3, %3, %8 clamp\n\tv_sub_u16_e64 %4, %4, %8 clamp\n\tv_sub_u16_e64 %5, %5, %8 clamp\n\tv_sub_u16_e64 %6, %6, %8 clamp\n\tv_sub_u16_e64 %7, %7, %8 clamp" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dot4_i32_i8(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_dot4_i32_i8 %0, %8, %9, %0\n\tv_dot4_i32_i8 %1, %8, %9, %1\n\tv_dot4_i32_i8 %2, %8, %9, %2\n\tv_dot4_i32_i8 %3, %8, %9, %3\n\tv_dot4_i32_i8 %4, %8, %9, %4\n\tv_dot4_i32_i8 %5, %8, %9, %5\n\tv_dot4_i32_i8 %6, %8, %9, %6\n\tv_dot4_i32_i8 %7, %8, %9, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dot4c_i32_i8(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_dot4c_i32_i8 %0, %8, %9\n\tv_dot4c_i32_i8 %1, %8, %9\n\tv_dot4c_i32_i8 %2, %8, %9\n\tv_dot4c_i32_i8 %3, %8, %9\n\tv_dot4c_i32_i8 %4, %8, %9\n\tv_dot4c_i32_i8 %5, %8, %9\n\tv_dot4c_i32_i8 %6, %8, %9\n\tv_dot4c_i32_i8 %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dot2_i32_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_dot2_i32_i16 %0, %8, %9, %0\n\tv_dot2_i32_i16 %1, %8, %9, %1\n\tv_dot2_i32_i16 %2, %8, %9, %2\n\tv_dot2_i32_i16 %3, %8, %9, %3\n\tv_dot2_i32_i16 %4, %8, %9, %4\n\tv_dot2_i32_i16 %5, %8, %9, %5\n\tv_dot2_i32_i16 %6, %8, %9, %6\n\tv_dot2_i32_i16 %7, %8, %9, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dot2c_i32_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_dot2c_i32_i16 %0, %8, %9\n\tv_dot2c_i32_i16 %1, %8, %9\n\tv_dot2c_i32_i16 %2, %8, %9\n\tv_dot2c_i32_i16 %3, %8, %9\n\tv_dot2c_i32_i16 %4, %8, %9\n\tv_dot2c_i32_i16 %5, %8, %9\n\tv_dot2c_i32_i16 %6, %8, %9\n\tv_dot2c_i32_i16 %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dot4_u32_u8(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_dot4_u32_u8 %0, %8, %9, %0\n\tv_dot4_u32_u8 %1, %8, %9, %1\n\tv_dot4_u32_u8 %2, %8, %9, %2\n\tv_dot4_u32_u8 %3, %8, %9, %3\n\tv_dot4_u32_u8 %4, %8, %9, %4\n\tv_dot4_u32_u8 %5, %8, %9, %5\n\tv_dot4_u32_u8 %6, %8, %9, %6\n\tv_dot4_u32_u8 %7, %8, %9, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_i16_opsel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_i16 %0, %0, %8 op_sel:[0,1,0]\n\tv_add_i16 %1, %1, %8 op_sel:[0,1,0]\n\tv_add_i16 %2, %2, %8 op_sel:[0,1,0]\n\tv_add_i16 %3, %3, %8 op_sel:[0,1,0]\n\tv_add_i16 %4, %4, %8 op_sel:[0,1,0]\n\tv_add_i16 %5, %5, %8 op_sel:[0,1,0]\n\tv_add_i16 %6, %6, %8 op_sel:[0,1,0]\n\tv_add_i16 %7, %7, %8 op_sel:[0,1,0]" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_i16 %0, %0, %8\n\tv_add_i16 %1, %1, %8\n\tv_add_i16 %2, %2, %8\n\tv_add_i16 %3, %3, %8\n\tv_add_i16 %4, %4, %8\n\tv_add_i16 %5, %5, %8\n\tv_add_i16 %6, %6, %8\n\tv_add_i16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mad_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_mad_u16 %0, %0, %8, %9\n\tv_mad_u16 %1, %1, %8, %9\n\tv_mad_u16 %2, %2, %8, %9\n\tv_mad_u16 %3, %3, %8, %9\n\tv_mad_u16 %4, %4, %8, %9\n\tv_mad_u16 %5, %5, %8, %9\n\tv_mad_u16 %6, %6, %8, %9\n\tv_mad_u16 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_lshrrev_b16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_lshrrev_b16 %0, %8, %0\n\tv_lshrrev_b16 %1, %8, %1\n\tv_lshrrev_b16 %2, %8, %2\n\tv_lshrrev_b16 %3, %8, %3\n\tv_lshrrev_b16 %4, %8, %4\n\tv_lshrrev_b16 %5, %8, %5\n\tv_lshrrev_b16 %6, %8, %6\n\tv_lshrrev_b16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_lshlrev_b16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_lshlrev_b16 %0, %8, %0\n\tv_lshlrev_b16 %1, %8, %1\n\tv_lshlrev_b16 %2, %8, %2\n\tv_lshlrev_b16 %3, %8, %3\n\tv_lshlrev_b16 %4, %8, %4\n\tv_lshlrev_b16 %5, %8, %5\n\tv_lshlrev_b16 %6, %8, %6\n\tv_lshlrev_b16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mul_lo_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_mul_lo_u16 %0, %8, %0\n\tv_mul_lo_u16 %1, %8, %1\n\tv_mul_lo_u16 %2, %8, %2\n\tv_mul_lo_u16 %3, %8, %3\n\tv_mul_lo_u16 %4, %8, %4\n\tv_mul_lo_u16 %5, %8, %5\n\tv_mul_lo_u16 %6, %8, %6\n\tv_mul_lo_u16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mac_f16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_mac_f16 %0, %8, %9\n\tv_mac_f16 %1, %8, %9\n\tv_mac_f16 %2, %8, %9\n\tv_mac_f16 %3, %8, %9\n\tv_mac_f16 %4, %8, %9\n\tv_mac_f16 %5, %8, %9\n\tv_mac_f16 %6, %8, %9\n\tv_mac_f16 %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_max_f16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max_f16 %0, %8, %0\n\tv_max_f16 %1, %8, %1\n\tv_max_f16 %2, %8, %2\n\tv_max_f16 %3, %8, %3\n\tv_max_f16 %4, %8, %4\n\tv_max_f16 %5, %8, %5\n\tv_max_f16 %6, %8, %6\n\tv_max_f16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_f16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_f16 %0, %8, %0\n\tv_add_f16 %1, %8, %1\n\tv_add_f16 %2, %8, %2\n\tv_add_f16 %3, %8, %3\n\tv_add_f16 %4, %8, %4\n\tv_add_f16 %5, %8, %5\n\tv_add_f16 %6, %8, %6\n\tv_add_f16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_max3_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max3_i16 %0, %0, %8, %9\n\tv_max3_i16 %1, %1, %8, %9\n\tv_max3_i16 %2, %2, %8, %9\n\tv_max3_i16 %3, %3, %8, %9\n\tv_max3_i16 %4, %4, %8, %9\n\tv_max3_i16 %5, %5, %8, %9\n\tv_max3_i16 %6, %6, %8, %9\n\tv_max3_i16 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_u16_sdwa_w1(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_u16_sdwa %0, %8, %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %1, %8, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %2, %8, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %3, %8, %3 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %4, %8, %4 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %5, %8, %5 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %6, %8, %6 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\tv_add_u16_sdwa %7, %8, %7 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_sub_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_sub_u16 %0, %0, %8\n\tv_sub_u16 %1, %1, %8\n\tv_sub_u16 %2, %2, %8\n\tv_sub_u16 %3, %3, %8\n\tv_sub_u16 %4, %4, %8\n\tv_sub_u16 %5, %5, %8\n\tv_sub_u16 %6, %6, %8\n\tv_sub_u16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_min_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_min_u16 %0, %8, %0\n\tv_min_u16 %1, %8, %1\n\tv_min_u16 %2, %8, %2\n\tv_min_u16 %3, %8, %3\n\tv_min_u16 %4, %8, %4\n\tv_min_u16 %5, %8, %5\n\tv_min_u16 %6, %8, %6\n\tv_min_u16 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_xor_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_xor_b32 %0, %8, %0\n\tv_xor_b32 %1, %8, %1\n\tv_xor_b32 %2, %8, %2\n\tv_xor_b32 %3, %8, %3\n\tv_xor_b32 %4, %8, %4\n\tv_xor_b32 %5, %8, %5\n\tv_xor_b32 %6, %8, %6\n\tv_xor_b32 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_dpp_shr1(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %3, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %4, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %5, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %6, %6 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %7, %7 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
typedef void (*kfn)(uint32_t*, int, uint32_t);
int main(int argc, char** argv) {
  uint32_t* dout; if (hipMalloc(&dout, 1 << 26) != hipSuccess) return 1;
  struct { const char* name; kfn f; } ks[] = {{"bfe_i32", k_bfe_i32},
{"add_u16", k_add_u16},
{"max_i16", k_max_i16},
{"sub_u16_e64_clamp", k_sub_u16_e64_clamp},
{"dot4_i32_i8", k_dot4_i32_i8},
{"dot4c_i32_i8", k_dot4c_i32_i8},
{"dot2_i32_i16", k_dot2_i32_i16},
{"dot2c_i32_i16", k_dot2c_i32_i16},
{"dot4_u32_u8", k_dot4_u32_u8},
{"add_i16_opsel", k_add_i16_opsel},
{"add_i16", k_add_i16},
{"mad_u16", k_mad_u16},
{"lshrrev_b16", k_lshrrev_b16},
{"lshlrev_b16", k_lshlrev_b16},
{"mul_lo_u16", k_mul_lo_u16},
{"mac_f16", k_mac_f16},
{"max_f16", k_max_f16},
{"add_f16", k_add_f16},
{"max3_i16", k_max3_i16},
{"add_u16_sdwa_w1", k_add_u16_sdwa_w1},
{"sub_u16", k_sub_u16},
{"min_u16", k_min_u16},
{"xor_b32", k_xor_b32},
{"dpp_shr1", k_dpp_shr1}};
  const int iters = 20000;
  for (auto& k : ks) {
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, 50, 1u); (void)hipDeviceSynchronize();
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0); hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, iters, 1u);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double winst = 2048.0 * 4 * iters * 8;
    printf("%-24s %7.3f ms  %.3f wave-instr/cyc/SIMD@2.4GHz\n", k.name, best, winst / (256 * 4.0 * best * 1e-3 * 2.4e9));
  }
  return 0;
}
