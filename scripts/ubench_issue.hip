// ubench_issue.hip -- measured VALU issue cost (SIMD cycles per wave64 instruction) of the
// instruction classes the fused kernels issue on gfx950, with 8 waves per SIMD each running 8
// independent chains (throughput, not latency).  One kernel per instruction.
// Relative costs (printed): s_memtime around each wave's loop, cost = wave ticks / (waves per
// SIMD x instructions per wave); s_memtime does not tick at the shader clock on gfx950, so these
// are relative only.
// Absolute costs: run under rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE and let
// scripts/issue_costs.py divide each dispatch's SIMD-cycles (1024 x GRBM_GUI_ACTIVE / 8) by its
// VALU wave-instructions -> profiles/<tag>_issue_costs.json ("calibration": "absolute").
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_issue ubench_issue.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define N_ITER 2048
#define CH 8

#define ASM8(op)                                                                          \
  asm volatile(op : "+v"(a[0]) : "v"(b), "v"(c)); asm volatile(op : "+v"(a[1]) : "v"(b), "v"(c)); \
  asm volatile(op : "+v"(a[2]) : "v"(b), "v"(c)); asm volatile(op : "+v"(a[3]) : "v"(b), "v"(c)); \
  asm volatile(op : "+v"(a[4]) : "v"(b), "v"(c)); asm volatile(op : "+v"(a[5]) : "v"(b), "v"(c)); \
  asm volatile(op : "+v"(a[6]) : "v"(b), "v"(c)); asm volatile(op : "+v"(a[7]) : "v"(b), "v"(c));

#define KERNEL(NAME, T, BT, OP)                                                            \
  __global__ __launch_bounds__(256) void NAME(unsigned long long* cyc, T* sink) {          \
    T a[CH];                                                                               \
    const BT b = (BT)(threadIdx.x + 3), c = (BT)(blockIdx.x + 5);                          \
    for (int i = 0; i < CH; ++i) a[i] = (T)(threadIdx.x * 7 + i);                          \
    __builtin_amdgcn_s_waitcnt(0);                                                         \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                            \
    for (int it = 0; it < N_ITER; ++it) { ASM8(OP) }                                       \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                            \
    T s = a[0];                                                                            \
    for (int i = 1; i < CH; ++i) s += a[i];                                                \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;          \
    if (s == (T)12345) sink[threadIdx.x] = s;                                              \
  }

KERNEL(k_fma_f64, double, double, "v_fma_f64 %0, %0, %1, %2")
KERNEL(k_add_f64, double, double, "v_add_f64 %0, %0, %1")
KERNEL(k_mul_f64, double, double, "v_mul_f64 %0, %0, %1")
KERNEL(k_fma_f32, float, float, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_add_u32, uint32_t, uint32_t, "v_add_u32 %0, %0, %1")
KERNEL(k_bitop3, uint32_t, uint32_t, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_alignbit, uint32_t, uint32_t, "v_alignbit_b32 %0, %0, %1, 12")
KERNEL(k_mul_lo_u32, uint32_t, uint32_t, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul_hi_u32, uint32_t, uint32_t, "v_mul_hi_u32 %0, %0, %1")
KERNEL(k_mad_u64_u32, uint64_t, uint32_t, "v_mad_u64_u32 %0, vcc, %1, %2, %0")
KERNEL(k_lshl_b64, uint64_t, uint32_t, "v_lshlrev_b64 %0, %1, %0")
KERNEL(k_cvt_f64_u32, double, uint32_t, "v_cvt_f64_u32 %0, %1")
KERNEL(k_cvt_f64_i32, double, uint32_t, "v_cvt_f64_i32 %0, %1")
KERNEL(k_rsq_f64, double, double, "v_rsq_f64 %0, %0")
KERNEL(k_rcp_f64, double, double, "v_rcp_f64 %0, %0")
KERNEL(k_ldexp_f64, double, uint32_t, "v_ldexp_f64 %0, %0, %1")
KERNEL(k_max_f64, double, double, "v_max_f64 %0, %0, %1")
KERNEL(k_fract_f64, double, double, "v_fract_f64 %0, %0")
KERNEL(k_cndmask, uint32_t, uint32_t, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_med3_i32, uint32_t, uint32_t, "v_med3_i32 %0, %0, %1, %2")
KERNEL(k_pk_fma_f32, uint64_t, uint64_t, "v_pk_fma_f32 %0, %0, %1, %2")
KERNEL(k_mul_u32_u24, uint32_t, uint32_t, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_pk_sub_u16, uint32_t, uint32_t, "v_pk_sub_u16 %0, %0, %1")
KERNEL(k_pk_min_u16, uint32_t, uint32_t, "v_pk_min_u16 %0, %0, %1")
KERNEL(k_bcnt, uint32_t, uint32_t, "v_bcnt_u32_b32 %0, %0, %1")
KERNEL(k_cvt_f32_f64, uint32_t, double, "v_cvt_f32_f64 %0, %1")
KERNEL(k_cvt_pknorm, uint32_t, uint32_t, "v_cvt_pknorm_u16_f32 %0, %0, %1")
KERNEL(k_min_f64, double, double, "v_min_f64 %0, %0, %1")

typedef void (*Fn)(unsigned long long*, void*);

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu * 8;   // 8 x 4 waves per CU = 8 waves per SIMD
  unsigned long long* cyc;
  void* sink;
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4);
  hipMalloc(&sink, 1 << 16);
  struct { const char* name; Fn fn; } ks[] = {
      {"v_fma_f64", (Fn)k_fma_f64}, {"v_add_f64", (Fn)k_add_f64}, {"v_mul_f64", (Fn)k_mul_f64},
      {"v_fma_f32", (Fn)k_fma_f32}, {"v_add_u32", (Fn)k_add_u32}, {"v_bitop3_b32", (Fn)k_bitop3},
      {"v_alignbit_b32", (Fn)k_alignbit}, {"v_mul_lo_u32", (Fn)k_mul_lo_u32},
      {"v_mul_hi_u32", (Fn)k_mul_hi_u32}, {"v_mad_u64_u32", (Fn)k_mad_u64_u32},
      {"v_lshlrev_b64", (Fn)k_lshl_b64}, {"v_cvt_f64_u32", (Fn)k_cvt_f64_u32},
      {"v_cvt_f64_i32", (Fn)k_cvt_f64_i32}, {"v_rsq_f64", (Fn)k_rsq_f64}, {"v_rcp_f64", (Fn)k_rcp_f64},
      {"v_ldexp_f64", (Fn)k_ldexp_f64}, {"v_max_f64", (Fn)k_max_f64}, {"v_fract_f64", (Fn)k_fract_f64},
      {"v_cndmask_b32", (Fn)k_cndmask}, {"v_med3_i32", (Fn)k_med3_i32},
      {"v_pk_fma_f32", (Fn)k_pk_fma_f32}, {"v_mul_u32_u24", (Fn)k_mul_u32_u24},
      {"v_pk_sub_u16", (Fn)k_pk_sub_u16}, {"v_pk_min_u16", (Fn)k_pk_min_u16},
      {"v_bcnt_u32_b32", (Fn)k_bcnt}, {"v_cvt_f32_f64", (Fn)k_cvt_f32_f64},
      {"v_cvt_pknorm_u16_f32", (Fn)k_cvt_pknorm}, {"v_min_f64", (Fn)k_min_f64}};
  unsigned long long* h = new unsigned long long[blocks * 4];
  printf("{\"waves_per_simd\": 8, \"instructions_per_wave\": %d, \"cycles_per_wave_instruction\": {", N_ITER * CH);
  const int nk = sizeof(ks) / sizeof(ks[0]);
  for (int i = 0; i < nk; ++i) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(ks[i].fn, dim3(blocks), dim3(256), 0, 0, cyc, sink);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int w = 0; w < blocks * 4; ++w) sum += (double)h[w];
    const double per = sum / (blocks * 4) / (8.0 * N_ITER * CH);
    printf("%s\"%s\": %.3f", i ? ", " : "", ks[i].name, per);
  }
  printf("}}\n");
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
