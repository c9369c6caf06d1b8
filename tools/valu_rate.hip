// VALU issue rate of packed vs plain f32 mul / add on gfx950 (a microbenchmark for the Gabor kernels' choice of
// v_pk_mul_f32 / v_pk_add_f32).  Each lane runs independent accumulator chains; the same number of f32 operations
// per lane either as plain v_mul_f32 + v_add_f32 (8 chains) or as v_pk_mul_f32 + v_pk_add_f32 (4 packed chains).
// Every CU runs 8 waves per SIMD.  Prints ms per form and the implied cycles per wave-instruction at the clock
// measured with s_memtime.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_plain(float* out, float s, float t, long long* clk) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 1e-3f + i;
  const long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "s"(s));
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "s"(t));
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; i++) r += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) *clk = c1 - c0;
}

__global__ __launch_bounds__(256) void k_packed(float* out, float s, float t, long long* clk) {
  f2 a[4];
#pragma unroll
  for (int i = 0; i < 4; i++) a[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f + i + 4};
  const f2 ss = f2{s, s}, tt = f2{t, t};
  const long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(ss));
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(tt));
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++) r += a[i].x + a[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) *clk = c1 - c0;
}

// the Gabor form: packed mul then packed add on separate product registers (acc += c * pp)
__global__ __launch_bounds__(256) void k_packed_mac(float* out, float s, float t, long long* clk) {
  f2 a[4], p[4];
#pragma unroll
  for (int i = 0; i < 4; i++) a[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f + i + 4};
  const f2 ss = f2{s, t};
  const long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(p[i]) : "v"(a[i]), "v"(ss));
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(p[i]));
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++) r += a[i].x + a[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) *clk = c1 - c0;
}

__global__ __launch_bounds__(256) void k_plain_mac(float* out, float s, float t, long long* clk) {
  float a[8], p[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 1e-3f + i;
  const long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p[i]) : "v"(a[i]), "s"(i & 1 ? s : t));
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(p[i]));
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; i++) r += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) *clk = c1 - c0;
}

int main() {
  const int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
  float* out;
  long long* clk;
  (void)hipMalloc(&out, blocks * 256 * sizeof(float));
  (void)hipMalloc(&clk, sizeof(long long));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[4] = {"plain mul+add (8 chains)", "packed mul+add (4 chains)", "packed mul, add (acc += p)",
                          "plain mul, add (acc += p)"};
  for (int k = 0; k < 4; k++) {
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(e0);
      if (k == 0) k_plain<<<blocks, 256>>>(out, 1.0000001f, 1e-7f, clk);
      if (k == 1) k_packed<<<blocks, 256>>>(out, 1.0000001f, 1e-7f, clk);
      if (k == 2) k_packed_mac<<<blocks, 256>>>(out, 1.0000001f, 1e-7f, clk);
      if (k == 3) k_plain_mac<<<blocks, 256>>>(out, 1.0000001f, 1e-7f, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      long long c;
      (void)hipMemcpy(&c, clk, sizeof c, hipMemcpyDeviceToHost);
      // wave-instructions per SIMD: 8 waves x ITERS x (16 plain or 8 packed)
      const double insts = 8.0 * ITERS * ((k == 0 || k == 3) ? 16 : 8);
      const double lane_ops = (double)blocks * 256 * ITERS * 16;  // f32 operations (mul or add)
      printf("%-30s %.3f ms  %.1f G f32-ops/s  %.2f ns per wave-instruction per SIMD  (wave 0: %lld memtime ticks)\n",
             names[k], ms, lane_ops / ms / 1e6, ms * 1e6 / insts, c);
    }
  }
  return 0;
}
