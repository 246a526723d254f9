#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ __launch_bounds__(256) void k_v_add_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_sub_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_sub_u32 %0, %0, %8\n\tv_sub_u32 %1, %1, %8\n\tv_sub_u32 %2, %2, %8\n\tv_sub_u32 %3, %3, %8\n\tv_sub_u32 %4, %4, %8\n\tv_sub_u32 %5, %5, %8\n\tv_sub_u32 %6, %6, %8\n\tv_sub_u32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max_i32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_max_i32 %0, %0, %8\n\tv_max_i32 %1, %1, %8\n\tv_max_i32 %2, %2, %8\n\tv_max_i32 %3, %3, %8\n\tv_max_i32 %4, %4, %8\n\tv_max_i32 %5, %5, %8\n\tv_max_i32 %6, %6, %8\n\tv_max_i32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_max_u32 %0, %0, %8\n\tv_max_u32 %1, %1, %8\n\tv_max_u32 %2, %2, %8\n\tv_max_u32 %3, %3, %8\n\tv_max_u32 %4, %4, %8\n\tv_max_u32 %5, %5, %8\n\tv_max_u32 %6, %6, %8\n\tv_max_u32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_min_i32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_min_i32 %0, %0, %8\n\tv_min_i32 %1, %1, %8\n\tv_min_i32 %2, %2, %8\n\tv_min_i32 %3, %3, %8\n\tv_min_i32 %4, %4, %8\n\tv_min_i32 %5, %5, %8\n\tv_min_i32 %6, %6, %8\n\tv_min_i32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_and_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_and_b32 %0, %0, %8\n\tv_and_b32 %1, %1, %8\n\tv_and_b32 %2, %2, %8\n\tv_and_b32 %3, %3, %8\n\tv_and_b32 %4, %4, %8\n\tv_and_b32 %5, %5, %8\n\tv_and_b32 %6, %6, %8\n\tv_and_b32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_or_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_or_b32 %0, %0, %8\n\tv_or_b32 %1, %1, %8\n\tv_or_b32 %2, %2, %8\n\tv_or_b32 %3, %3, %8\n\tv_or_b32 %4, %4, %8\n\tv_or_b32 %5, %5, %8\n\tv_or_b32 %6, %6, %8\n\tv_or_b32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_xor_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_lshlrev_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_lshlrev_b32 %0, %0, %8\n\tv_lshlrev_b32 %1, %1, %8\n\tv_lshlrev_b32 %2, %2, %8\n\tv_lshlrev_b32 %3, %3, %8\n\tv_lshlrev_b32 %4, %4, %8\n\tv_lshlrev_b32 %5, %5, %8\n\tv_lshlrev_b32 %6, %6, %8\n\tv_lshlrev_b32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_add_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_add_f32 %0, %0, %8\n\tv_add_f32 %1, %1, %8\n\tv_add_f32 %2, %2, %8\n\tv_add_f32 %3, %3, %8\n\tv_add_f32 %4, %4, %8\n\tv_add_f32 %5, %5, %8\n\tv_add_f32 %6, %6, %8\n\tv_add_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_sub_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_sub_f32 %0, %0, %8\n\tv_sub_f32 %1, %1, %8\n\tv_sub_f32 %2, %2, %8\n\tv_sub_f32 %3, %3, %8\n\tv_sub_f32 %4, %4, %8\n\tv_sub_f32 %5, %5, %8\n\tv_sub_f32 %6, %6, %8\n\tv_sub_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_mul_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_mul_f32 %0, %0, %8\n\tv_mul_f32 %1, %1, %8\n\tv_mul_f32 %2, %2, %8\n\tv_mul_f32 %3, %3, %8\n\tv_mul_f32 %4, %4, %8\n\tv_mul_f32 %5, %5, %8\n\tv_mul_f32 %6, %6, %8\n\tv_mul_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_max_f32 %0, %0, %8\n\tv_max_f32 %1, %1, %8\n\tv_max_f32 %2, %2, %8\n\tv_max_f32 %3, %3, %8\n\tv_max_f32 %4, %4, %8\n\tv_max_f32 %5, %5, %8\n\tv_max_f32 %6, %6, %8\n\tv_max_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_min_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_min_f32 %0, %0, %8\n\tv_min_f32 %1, %1, %8\n\tv_min_f32 %2, %2, %8\n\tv_min_f32 %3, %3, %8\n\tv_min_f32 %4, %4, %8\n\tv_min_f32 %5, %5, %8\n\tv_min_f32 %6, %6, %8\n\tv_min_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_pk_add_u16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_pk_add_u16 %0, %0, %8\n\tv_pk_add_u16 %1, %1, %8\n\tv_pk_add_u16 %2, %2, %8\n\tv_pk_add_u16 %3, %3, %8\n\tv_pk_add_u16 %4, %4, %8\n\tv_pk_add_u16 %5, %5, %8\n\tv_pk_add_u16 %6, %6, %8\n\tv_pk_add_u16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_pk_max_i16(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_pk_max_i16 %0, %0, %8\n\tv_pk_max_i16 %1, %1, %8\n\tv_pk_max_i16 %2, %2, %8\n\tv_pk_max_i16 %3, %3, %8\n\tv_pk_max_i16 %4, %4, %8\n\tv_pk_max_i16 %5, %5, %8\n\tv_pk_max_i16 %6, %6, %8\n\tv_pk_max_i16 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_pk_add_f32(uint32_t* out, int iters, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {1.f*threadIdx.x, 2.f}, a1=a0*1.1f, a2=a0*1.2f, a3=a0*1.3f, a4=a0*1.4f, a5=a0*1.5f, a6=a0*1.6f, a7=a0*1.7f, b={1.0001f,0.9999f};
  for (int i = 0; i < iters; ++i) asm volatile("v_pk_add_f32 %0, %0, %8\n\tv_pk_add_f32 %1, %1, %8\n\tv_pk_add_f32 %2, %2, %8\n\tv_pk_add_f32 %3, %3, %8\n\tv_pk_add_f32 %4, %4, %8\n\tv_pk_add_f32 %5, %5, %8\n\tv_pk_add_f32 %6, %6, %8\n\tv_pk_add_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = (uint32_t)(a0.x+a1.y+a2.x+a3.y+a4.x+a5.x+a6.x+a7.y);
}
__global__ __launch_bounds__(256) void k_v_pk_mul_f32(uint32_t* out, int iters, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {1.f*threadIdx.x, 2.f}, a1=a0*1.1f, a2=a0*1.2f, a3=a0*1.3f, a4=a0*1.4f, a5=a0*1.5f, a6=a0*1.6f, a7=a0*1.7f, b={1.0001f,0.9999f};
  for (int i = 0; i < iters; ++i) asm volatile("v_pk_mul_f32 %0, %0, %8\n\tv_pk_mul_f32 %1, %1, %8\n\tv_pk_mul_f32 %2, %2, %8\n\tv_pk_mul_f32 %3, %3, %8\n\tv_pk_mul_f32 %4, %4, %8\n\tv_pk_mul_f32 %5, %5, %8\n\tv_pk_mul_f32 %6, %6, %8\n\tv_pk_mul_f32 %7, %7, %8" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = (uint32_t)(a0.x+a1.y+a2.x+a3.y+a4.x+a5.x+a6.x+a7.y);
}
__global__ __launch_bounds__(256) void k_v_mov_b32_dpp_shr(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %3, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %4, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %5, %6 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %6, %7 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %7, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b));
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max3_i32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max3_i32 %0, %0, %8, %9\n\tv_max3_i32 %1, %1, %8, %9\n\tv_max3_i32 %2, %2, %8, %9\n\tv_max3_i32 %3, %3, %8, %9\n\tv_max3_i32 %4, %4, %8, %9\n\tv_max3_i32 %5, %5, %8, %9\n\tv_max3_i32 %6, %6, %8, %9\n\tv_max3_i32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max3_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max3_f32 %0, %0, %8, %9\n\tv_max3_f32 %1, %1, %8, %9\n\tv_max3_f32 %2, %2, %8, %9\n\tv_max3_f32 %3, %3, %8, %9\n\tv_max3_f32 %4, %4, %8, %9\n\tv_max3_f32 %5, %5, %8, %9\n\tv_max3_f32 %6, %6, %8, %9\n\tv_max3_f32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_med3_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_med3_f32 %0, %0, %8, %9\n\tv_med3_f32 %1, %1, %8, %9\n\tv_med3_f32 %2, %2, %8, %9\n\tv_med3_f32 %3, %3, %8, %9\n\tv_med3_f32 %4, %4, %8, %9\n\tv_med3_f32 %5, %5, %8, %9\n\tv_med3_f32 %6, %6, %8, %9\n\tv_med3_f32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_fma_f32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\tv_fma_f32 %3, %3, %8, %9\n\tv_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\tv_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_add3_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_add3_u32 %0, %0, %8, %9\n\tv_add3_u32 %1, %1, %8, %9\n\tv_add3_u32 %2, %2, %8, %9\n\tv_add3_u32 %3, %3, %8, %9\n\tv_add3_u32 %4, %4, %8, %9\n\tv_add3_u32 %5, %5, %8, %9\n\tv_add3_u32 %6, %6, %8, %9\n\tv_add3_u32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_lshl_or_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_lshl_or_b32 %0, %0, 1, %9\n\tv_lshl_or_b32 %1, %1, 1, %9\n\tv_lshl_or_b32 %2, %2, 1, %9\n\tv_lshl_or_b32 %3, %3, 1, %9\n\tv_lshl_or_b32 %4, %4, 1, %9\n\tv_lshl_or_b32 %5, %5, 1, %9\n\tv_lshl_or_b32 %6, %6, 1, %9\n\tv_lshl_or_b32 %7, %7, 1, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_lshl_add_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_lshl_add_u32 %0, %0, 1, %9\n\tv_lshl_add_u32 %1, %1, 1, %9\n\tv_lshl_add_u32 %2, %2, 1, %9\n\tv_lshl_add_u32 %3, %3, 1, %9\n\tv_lshl_add_u32 %4, %4, 1, %9\n\tv_lshl_add_u32 %5, %5, 1, %9\n\tv_lshl_add_u32 %6, %6, 1, %9\n\tv_lshl_add_u32 %7, %7, 1, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_and_or_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_and_or_b32 %0, %0, %8, %9\n\tv_and_or_b32 %1, %1, %8, %9\n\tv_and_or_b32 %2, %2, %8, %9\n\tv_and_or_b32 %3, %3, %8, %9\n\tv_and_or_b32 %4, %4, %8, %9\n\tv_and_or_b32 %5, %5, %8, %9\n\tv_and_or_b32 %6, %6, %8, %9\n\tv_and_or_b32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_bfe_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_bfe_u32 %0, %0, 3, 5\n\tv_bfe_u32 %1, %1, 3, 5\n\tv_bfe_u32 %2, %2, 3, 5\n\tv_bfe_u32 %3, %3, 3, 5\n\tv_bfe_u32 %4, %4, 3, 5\n\tv_bfe_u32 %5, %5, 3, 5\n\tv_bfe_u32 %6, %6, 3, 5\n\tv_bfe_u32 %7, %7, 3, 5" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_perm_b32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_perm_b32 %0, %0, %8, %9\n\tv_perm_b32 %1, %1, %8, %9\n\tv_perm_b32 %2, %2, %8, %9\n\tv_perm_b32 %3, %3, %8, %9\n\tv_perm_b32 %4, %4, %8, %9\n\tv_perm_b32 %5, %5, %8, %9\n\tv_perm_b32 %6, %6, %8, %9\n\tv_perm_b32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_cndmask_vcc(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_cndmask_b32_e32 %0, %0, %8, vcc\n\tv_cndmask_b32_e32 %1, %1, %8, vcc\n\tv_cndmask_b32_e32 %2, %2, %8, vcc\n\tv_cndmask_b32_e32 %3, %3, %8, vcc\n\tv_cndmask_b32_e32 %4, %4, %8, vcc\n\tv_cndmask_b32_e32 %5, %5, %8, vcc\n\tv_cndmask_b32_e32 %6, %6, %8, vcc\n\tv_cndmask_b32_e32 %7, %7, %8, vcc" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_v_max3_u32(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4 = a0*9, a5 = a0*11, a6 = a0*13, a7 = a0*15, b = seed ^ 0x1234, c = seed*77;
  for (int i = 0; i < iters; ++i) asm volatile("v_max3_u32 %0, %0, %8, %9\n\tv_max3_u32 %1, %1, %8, %9\n\tv_max3_u32 %2, %2, %8, %9\n\tv_max3_u32 %3, %3, %8, %9\n\tv_max3_u32 %4, %4, %8, %9\n\tv_max3_u32 %5, %5, %8, %9\n\tv_max3_u32 %6, %6, %8, %9\n\tv_max3_u32 %7, %7, %8, %9" : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) : "v"(b), "v"(c) : "vcc");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ __launch_bounds__(256) void k_cmpf_addc(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile(
    "v_cmp_eq_f32_e64 s[40:41], %0, %4\n\tv_cmp_eq_f32_e64 s[42:43], %1, %4\n\tv_cmp_eq_f32_e64 s[44:45], %2, %4\n\tv_cmp_eq_f32_e64 s[46:47], %3, %4\n\t"
    "v_addc_co_u32_e64 %0, s[40:41], %0, %0, s[40:41]\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %1, s[42:43]\n\tv_addc_co_u32_e64 %2, s[44:45], %2, %2, s[44:45]\n\tv_addc_co_u32_e64 %3, s[46:47], %3, %3, s[46:47]"
    : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3) : "v"(b) : "s40","s41","s42","s43","s44","s45","s46","s47");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3;
}
__global__ __launch_bounds__(256) void k_cmp_only(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, b = seed ^ 0x1234;
  for (int i = 0; i < iters; ++i) asm volatile(
    "v_cmp_eq_u32_e64 s[40:41], %0, %4\n\tv_cmp_eq_u32_e64 s[42:43], %1, %4\n\tv_cmp_eq_u32_e64 s[44:45], %2, %4\n\tv_cmp_eq_u32_e64 s[46:47], %3, %4\n\t"
    "v_cmp_eq_u32_e64 s[48:49], %0, %4\n\tv_cmp_eq_u32_e64 s[50:51], %1, %4\n\tv_cmp_eq_u32_e64 s[52:53], %2, %4\n\tv_cmp_eq_u32_e64 s[54:55], %3, %4"
    : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3) : "v"(b) : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3;
}
__global__ __launch_bounds__(256) void k_addc_only(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0*3, a2 = a0*5, a3 = a0*7, a4=a0*9, a5=a0*11, a6=a0*13, a7=a0*15;
  for (int i = 0; i < iters; ++i) asm volatile(
    "v_addc_co_u32_e64 %0, s[40:41], %0, %0, s[40:41]\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %1, s[42:43]\n\tv_addc_co_u32_e64 %2, s[44:45], %2, %2, s[44:45]\n\tv_addc_co_u32_e64 %3, s[46:47], %3, %3, s[46:47]\n\t"
    "v_addc_co_u32_e64 %4, s[48:49], %4, %4, s[48:49]\n\tv_addc_co_u32_e64 %5, s[50:51], %5, %5, s[50:51]\n\tv_addc_co_u32_e64 %6, s[52:53], %6, %6, s[52:53]\n\tv_addc_co_u32_e64 %7, s[54:55], %7, %7, s[54:55]"
    : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) :: "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
  out[blockIdx.x*blockDim.x+threadIdx.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
typedef void (*kfn)(uint32_t*, int, uint32_t);
int main() {
  uint32_t* dout; hipMalloc(&dout, 1 << 26);
  struct { const char* name; kfn f; } ks[] = { {"v_add_u32", k_v_add_u32},
{"v_sub_u32", k_v_sub_u32},
{"v_max_i32", k_v_max_i32},
{"v_max_u32", k_v_max_u32},
{"v_min_i32", k_v_min_i32},
{"v_and_b32", k_v_and_b32},
{"v_or_b32", k_v_or_b32},
{"v_xor_b32", k_v_xor_b32},
{"v_lshlrev_b32", k_v_lshlrev_b32},
{"v_add_f32", k_v_add_f32},
{"v_sub_f32", k_v_sub_f32},
{"v_mul_f32", k_v_mul_f32},
{"v_max_f32", k_v_max_f32},
{"v_min_f32", k_v_min_f32},
{"v_pk_add_u16", k_v_pk_add_u16},
{"v_pk_max_i16", k_v_pk_max_i16},
{"v_pk_add_f32", k_v_pk_add_f32},
{"v_pk_mul_f32", k_v_pk_mul_f32},
{"v_mov_b32_dpp_shr", k_v_mov_b32_dpp_shr},
{"v_max3_i32", k_v_max3_i32},
{"v_max3_f32", k_v_max3_f32},
{"v_med3_f32", k_v_med3_f32},
{"v_fma_f32", k_v_fma_f32},
{"v_add3_u32", k_v_add3_u32},
{"v_lshl_or_b32", k_v_lshl_or_b32},
{"v_lshl_add_u32", k_v_lshl_add_u32},
{"v_and_or_b32", k_v_and_or_b32},
{"v_bfe_u32", k_v_bfe_u32},
{"v_perm_b32", k_v_perm_b32},
{"v_cndmask_vcc", k_v_cndmask_vcc},
{"v_max3_u32", k_v_max3_u32},
{"cmpf_addc", k_cmpf_addc},
{"cmp_only", k_cmp_only},
{"addc_only", k_addc_only} };
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
    const double winst = 2048.0 * 4 * iters * 8;
    printf("%-22s %7.3f ms  %.3f wave-instr/cyc/SIMD@2.4GHz  %.1f T lane-ops/s\n", k.name, best, winst / (prop.multiProcessorCount * 4.0 * best * 1e-3 * clk), winst * 64 / (best * 1e-3) / 1e12);
  }
  return 0;
}
