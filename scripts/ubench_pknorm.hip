// Checks that v_cvt_pknorm_u16_f32 (the sign records' code map, dcor_fused.hip code_pair) is
// monotone non-decreasing over every float in [0, 2], that negative floats code as 0, and how
// NaN codes.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_pknorm scripts/ubench_pknorm.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// thread u compares the codes of the floats with bit patterns u and u + 1
__global__ void k_mono(uint32_t ubegin, uint32_t count, uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t u = ubegin + i;
  const float a = __uint_as_float(u), b = __uint_as_float(u + 1u);
  const u16x2 q = __builtin_amdgcn_cvt_pknorm_u16(a, b);
  if (q.x > q.y) bad[0] = u;           // plain vector store; any violating u will do
  const u16x2 n = __builtin_amdgcn_cvt_pknorm_u16(-a, -b);
  if (n.x != 0 || n.y != 0) bad[1] = u;
}

// code resolution: t = (k + f) / 65535 must code as k (f = 0, 0.3) and k + 1 (f = 0.7)
__global__ void k_levels(uint32_t* bad) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 65535u) return;
  const float a = (float)k / 65535.0f, b = ((float)k + 0.3f) / 65535.0f, c = ((float)k + 0.7f) / 65535.0f;
  const u16x2 q = __builtin_amdgcn_cvt_pknorm_u16(a, b);
  const u16x2 r = __builtin_amdgcn_cvt_pknorm_u16(c, c);
  if (q.x != k || q.y != k || r.x != k + 1u) atomicAdd(&bad[0], 1u);
}

__global__ void k_special(uint32_t* out) {
  if (threadIdx.x != 0) return;
  const float nan = __uint_as_float(0x7fc00000u);
  const u16x2 q0 = __builtin_amdgcn_cvt_pknorm_u16(nan, 1.0f);
  const u16x2 q1 = __builtin_amdgcn_cvt_pknorm_u16(0.5f, 32767.0f / 65535.0f);
  out[0] = q0.x; out[1] = q0.y; out[2] = q1.x; out[3] = q1.y;
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 64) != hipSuccess) return 2;
  const uint32_t init[8] = {0xffffffffu, 0xffffffffu, 0, 0, 0, 0, 0, 0};
  hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice);
  const uint32_t top = 0x40000000u;  // 2.0f
  const uint32_t chunk = 1u << 28;
  for (uint32_t b = 0; b < top; b += chunk) {
    const uint32_t cnt = (top - b) < chunk ? (top - b) : chunk;
    hipLaunchKernelGGL(k_mono, dim3((cnt + 255) / 256), dim3(256), 0, 0, b, cnt, d);
  }
  hipLaunchKernelGGL(k_special, dim3(1), dim3(64), 0, 0, d + 2);
  hipLaunchKernelGGL(k_levels, dim3(256), dim3(256), 0, 0, d + 6);
  uint32_t h[8];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  std::printf("monotone violations: %s (first u 0x%08x); negative nonzero: %s\n",
              h[0] == 0xffffffffu ? "none" : "FOUND", h[0], h[1] == 0xffffffffu ? "none" : "FOUND");
  std::printf("code levels off by rounding: %u of 65535\n", h[6]);
  std::printf("pknorm(NaN) = %u, pknorm(1) = %u, pknorm(0.5) = %u, pknorm(32767/65535) = %u\n",
              h[2], h[3], h[4], h[5]);
  hipFree(d);
  return (h[0] == 0xffffffffu && h[1] == 0xffffffffu) ? 0 : 1;
}
