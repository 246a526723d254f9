#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ __launch_bounds__(256) void k_cndmask_e64_sgpr(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[40:41]\n\tv_cndmask_b32_e64 %1, %1, %8, s[40:41]\n\tv_cndmask_b32_e64 %2, %2, %8, s[40:41]\n\tv_cndmask_b32_e64 %3, %3, %8, s[40:41]\n\tv_cndmask_b32_e64 %4, %4, %8, s[40:41]\n\tv_cndmask_b32_e64 %5, %5, %8, s[40:41]\n\tv_cndmask_b32_e64 %6, %6, %8, s[40:41]\n\tv_cndmask_b32_e64 %7, %7, %8, s[40:41]" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_cndmask_e32_vcc_after_cmp(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_cmp_eq_u32_e32 vcc, %8, %9\n\tv_cndmask_b32_e32 %0, %0, %8, vcc\n\tv_cndmask_b32_e32 %1, %1, %8, vcc\n\tv_cndmask_b32_e32 %2, %2, %8, vcc\n\tv_cndmask_b32_e32 %3, %3, %8, vcc\n\tv_cndmask_b32_e32 %4, %4, %8, vcc\n\tv_cndmask_b32_e32 %5, %5, %8, vcc\n\tv_cndmask_b32_e32 %6, %6, %8, vcc\n\tv_cndmask_b32_e32 %7, %7, %8, vcc" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_sub_co_e64(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_sub_co_u32_e64 %0, s[42:43], %0, %8\n\tv_sub_co_u32_e64 %1, s[42:43], %1, %8\n\tv_sub_co_u32_e64 %2, s[42:43], %2, %8\n\tv_sub_co_u32_e64 %3, s[42:43], %3, %8\n\tv_sub_co_u32_e64 %4, s[42:43], %4, %8\n\tv_sub_co_u32_e64 %5, s[42:43], %5, %8\n\tv_sub_co_u32_e64 %6, s[42:43], %6, %8\n\tv_sub_co_u32_e64 %7, s[42:43], %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_co_e64(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_add_co_u32_e64 %0, s[42:43], %0, %8\n\tv_add_co_u32_e64 %1, s[42:43], %1, %8\n\tv_add_co_u32_e64 %2, s[42:43], %2, %8\n\tv_add_co_u32_e64 %3, s[42:43], %3, %8\n\tv_add_co_u32_e64 %4, s[42:43], %4, %8\n\tv_add_co_u32_e64 %5, s[42:43], %5, %8\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_add_co_u32_e64 %7, s[42:43], %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_subrev_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_subrev_u32 %0, %0, %8\n\tv_subrev_u32 %1, %1, %8\n\tv_subrev_u32 %2, %2, %8\n\tv_subrev_u32 %3, %3, %8\n\tv_subrev_u32 %4, %4, %8\n\tv_subrev_u32 %5, %5, %8\n\tv_subrev_u32 %6, %6, %8\n\tv_subrev_u32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_u32_rev(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_add_u32 %0, %8, %0\n\tv_add_u32 %1, %8, %1\n\tv_add_u32 %2, %8, %2\n\tv_add_u32 %3, %8, %3\n\tv_add_u32 %4, %8, %4\n\tv_add_u32 %5, %8, %5\n\tv_add_u32 %6, %8, %6\n\tv_add_u32 %7, %8, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mul_u32_u24(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_mul_u32_u24 %0, %0, %8\n\tv_mul_u32_u24 %1, %1, %8\n\tv_mul_u32_u24 %2, %2, %8\n\tv_mul_u32_u24 %3, %3, %8\n\tv_mul_u32_u24 %4, %4, %8\n\tv_mul_u32_u24 %5, %5, %8\n\tv_mul_u32_u24 %6, %6, %8\n\tv_mul_u32_u24 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mad_u32_u24(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_mad_u32_u24 %0, %0, %8, %9\n\tv_mad_u32_u24 %1, %1, %8, %9\n\tv_mad_u32_u24 %2, %2, %8, %9\n\tv_mad_u32_u24 %3, %3, %8, %9\n\tv_mad_u32_u24 %4, %4, %8, %9\n\tv_mad_u32_u24 %5, %5, %8, %9\n\tv_mad_u32_u24 %6, %6, %8, %9\n\tv_mad_u32_u24 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_cvt_f32_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_cvt_f32_u32 %0, %0\n\tv_cvt_f32_u32 %1, %1\n\tv_cvt_f32_u32 %2, %2\n\tv_cvt_f32_u32 %3, %3\n\tv_cvt_f32_u32 %4, %4\n\tv_cvt_f32_u32 %5, %5\n\tv_cvt_f32_u32 %6, %6\n\tv_cvt_f32_u32 %7, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_lshrrev_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_lshrrev_b32 %0, 1, %0\n\tv_lshrrev_b32 %1, 1, %1\n\tv_lshrrev_b32 %2, 1, %2\n\tv_lshrrev_b32 %3, 1, %3\n\tv_lshrrev_b32 %4, 1, %4\n\tv_lshrrev_b32 %5, 1, %5\n\tv_lshrrev_b32 %6, 1, %6\n\tv_lshrrev_b32 %7, 1, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_ashrrev_i32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_ashrrev_i32 %0, 1, %0\n\tv_ashrrev_i32 %1, 1, %1\n\tv_ashrrev_i32 %2, 1, %2\n\tv_ashrrev_i32 %3, 1, %3\n\tv_ashrrev_i32 %4, 1, %4\n\tv_ashrrev_i32 %5, 1, %5\n\tv_ashrrev_i32 %6, 1, %6\n\tv_ashrrev_i32 %7, 1, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_not_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_not_b32 %0, %0\n\tv_not_b32 %1, %1\n\tv_not_b32 %2, %2\n\tv_not_b32 %3, %3\n\tv_not_b32 %4, %4\n\tv_not_b32 %5, %5\n\tv_not_b32 %6, %6\n\tv_not_b32 %7, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_mov_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_mov_b32 %0, %1\n\tv_mov_b32 %1, %2\n\tv_mov_b32 %2, %3\n\tv_mov_b32 %3, %4\n\tv_mov_b32 %4, %5\n\tv_mov_b32 %5, %6\n\tv_mov_b32 %6, %7\n\tv_mov_b32 %7, %0" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_alignbit_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_alignbit_b32 %0, %0, %8, 1\n\tv_alignbit_b32 %1, %1, %8, 1\n\tv_alignbit_b32 %2, %2, %8, 1\n\tv_alignbit_b32 %3, %3, %8, 1\n\tv_alignbit_b32 %4, %4, %8, 1\n\tv_alignbit_b32 %5, %5, %8, 1\n\tv_alignbit_b32 %6, %6, %8, 1\n\tv_alignbit_b32 %7, %7, %8, 1" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_bfi_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_bfi_b32 %0, %0, %8, %9\n\tv_bfi_b32 %1, %1, %8, %9\n\tv_bfi_b32 %2, %2, %8, %9\n\tv_bfi_b32 %3, %3, %8, %9\n\tv_bfi_b32 %4, %4, %8, %9\n\tv_bfi_b32 %5, %5, %8, %9\n\tv_bfi_b32 %6, %6, %8, %9\n\tv_bfi_b32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_max_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_max_i16 %0, %0, %8\n\tv_max_i16 %1, %1, %8\n\tv_max_i16 %2, %2, %8\n\tv_max_i16 %3, %3, %8\n\tv_max_i16 %4, %4, %8\n\tv_max_i16 %5, %5, %8\n\tv_max_i16 %6, %6, %8\n\tv_max_i16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_add_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_add_u16 %0, %0, %8\n\tv_add_u16 %1, %1, %8\n\tv_add_u16 %2, %2, %8\n\tv_add_u16 %3, %3, %8\n\tv_add_u16 %4, %4, %8\n\tv_add_u16 %5, %5, %8\n\tv_add_u16 %6, %6, %8\n\tv_add_u16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_fmac_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_fmac_f32 %0, %8, %9\n\tv_fmac_f32 %1, %8, %9\n\tv_fmac_f32 %2, %8, %9\n\tv_fmac_f32 %3, %8, %9\n\tv_fmac_f32 %4, %8, %9\n\tv_fmac_f32 %5, %8, %9\n\tv_fmac_f32 %6, %8, %9\n\tv_fmac_f32 %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_min3_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_min3_f32 %0, %0, %8, %9\n\tv_min3_f32 %1, %1, %8, %9\n\tv_min3_f32 %2, %2, %8, %9\n\tv_min3_f32 %3, %3, %8, %9\n\tv_min3_f32 %4, %4, %8, %9\n\tv_min3_f32 %5, %5, %8, %9\n\tv_min3_f32 %6, %6, %8, %9\n\tv_min3_f32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_xad_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_xad_u32 %0, %0, %8, %9\n\tv_xad_u32 %1, %1, %8, %9\n\tv_xad_u32 %2, %2, %8, %9\n\tv_xad_u32 %3, %3, %8, %9\n\tv_xad_u32 %4, %4, %8, %9\n\tv_xad_u32 %5, %5, %8, %9\n\tv_xad_u32 %6, %6, %8, %9\n\tv_xad_u32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_or3_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_or3_b32 %0, %0, %8, %9\n\tv_or3_b32 %1, %1, %8, %9\n\tv_or3_b32 %2, %2, %8, %9\n\tv_or3_b32 %3, %3, %8, %9\n\tv_or3_b32 %4, %4, %8, %9\n\tv_or3_b32 %5, %5, %8, %9\n\tv_or3_b32 %6, %6, %8, %9\n\tv_or3_b32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_readlane(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40","s41");
  for (int i = 0; i < iters; ++i) asm volatile("v_readlane_b32 s44, %0, 5\n\tv_readlane_b32 s45, %1, 5\n\tv_readlane_b32 s46, %2, 5\n\tv_readlane_b32 s47, %3, 5\n\tv_readlane_b32 s48, %4, 5\n\tv_readlane_b32 s49, %5, 5\n\tv_readlane_b32 s50, %6, 5\n\tv_readlane_b32 s51, %7, 5\n\tv_add_f32 %0, s44, %0\n\tv_add_f32 %1, s45, %1\n\tv_add_f32 %2, s46, %2\n\tv_add_f32 %3, s47, %3\n\tv_add_f32 %4, s48, %4\n\tv_add_f32 %5, s49, %5\n\tv_add_f32 %6, s50, %6\n\tv_add_f32 %7, s51, %7" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
typedef void (*kfn)(uint32_t*, int, uint32_t);
int main() {
  uint32_t* dout; hipMalloc(&dout, 1 << 26);
  struct { const char* name; kfn f; int per; } ks[] = { {"cndmask_e64_sgpr", k_cndmask_e64_sgpr, 8},
{"cndmask_e32_vcc_after_cmp", k_cndmask_e32_vcc_after_cmp, 9},
{"sub_co_e64", k_sub_co_e64, 8},
{"add_co_e64", k_add_co_e64, 8},
{"subrev_u32", k_subrev_u32, 8},
{"add_u32_rev", k_add_u32_rev, 8},
{"mul_u32_u24", k_mul_u32_u24, 8},
{"mad_u32_u24", k_mad_u32_u24, 8},
{"cvt_f32_u32", k_cvt_f32_u32, 8},
{"lshrrev_b32", k_lshrrev_b32, 8},
{"ashrrev_i32", k_ashrrev_i32, 8},
{"not_b32", k_not_b32, 8},
{"mov_b32", k_mov_b32, 8},
{"alignbit_b32", k_alignbit_b32, 8},
{"bfi_b32", k_bfi_b32, 8},
{"max_i16", k_max_i16, 8},
{"add_u16", k_add_u16, 8},
{"fmac_f32", k_fmac_f32, 8},
{"min3_f32", k_min3_f32, 8},
{"xad_u32", k_xad_u32, 8},
{"or3_b32", k_or3_b32, 8},
{"readlane", k_readlane, 16} };
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const double clk = prop.clockRate * 1e3;
  const int iters = 20000;
  for (auto& k : ks) {
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, 50, 1u); hipDeviceSynchronize();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0); hipLaunchKernelGGL(k.f, dim3(2048), dim3(256), 0, 0, dout, iters, 1u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double winst = 2048.0 * 4 * iters * k.per;
    printf("%-28s %7.3f ms  %.3f wave-instr/cyc/SIMD@2.4GHz\n", k.name, best, winst / (prop.multiProcessorCount * 4.0 * best * 1e-3 * clk));
  }
  return 0;
}
