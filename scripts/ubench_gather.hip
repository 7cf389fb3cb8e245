// Microbenchmark: random 16-B gathers from an L2-resident packed panel (the C5-continuous NI
// access pattern), to find what bounds them.  Each replicate row holds k*m int32 sample indices
// (n = 19,433, k*m = 19,432, 8,192 rows as in C5); a thread reads int4 index groups and gathers
// the four 16-B panel entries.  Variants: U index groups in flight per thread, WPE waves per SIMD;
// 'idx' = the index stream alone (no gathers); 'seq' = gathers at sequential addresses (i mod n).
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_gather scripts/ubench_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int iv4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U, int MODE>  // MODE 0 gather, 1 index stream only, 2 sequential gather
__global__ __launch_bounds__(256) void k_gather(const double2* __restrict__ xy, const iv4* __restrict__ perm,
                                               int64_t groups, int n, double* __restrict__ out) {
  double sx = 0, sy = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; g + (U - 1) * stride < groups; g += U * stride) {
    iv4 p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = __builtin_nontemporal_load(perm + g + u * stride);
    if (MODE == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) sx += (double)(p[u].x + p[u].y + p[u].z + p[u].w);
      continue;
    }
    if (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int b = (int)((g + u * stride) * 4 % n);
        p[u] = iv4{b, b + 1 < n ? b + 1 : 0, b + 2 < n ? b + 2 : 0, b + 3 < n ? b + 3 : 0} + (p[u] & 0);
      }
    }
    double2 v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u][0] = xy[p[u].x]; v[u][1] = xy[p[u].y]; v[u][2] = xy[p[u].z]; v[u][3] = xy[p[u].w];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) { sx += v[u][r].x; sy += v[u][r].y; }
  }
  for (; g < groups; g += stride) {
    const iv4 q = perm[g];
    if (MODE == 1) { sx += q.x; continue; }
    sx += xy[q.x].x + xy[q.y].x + xy[q.z].x + xy[q.w].x;
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = sx + sy;
}

template <int U, int MODE>
static float run(const double2* xy, const iv4* perm, int64_t groups, int n, double* out, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_gather<U, MODE>), dim3(grid), dim3(256), 0, 0, xy, perm, groups, n, out);
  CK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i)
    hipLaunchKernelGGL((k_gather<U, MODE>), dim3(grid), dim3(256), 0, 0, xy, perm, groups, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / 5;
}

int main() {
  const int n = 19433, km = 19432, R = 8192;
  const int64_t groups = (int64_t)R * km / 4;
  std::vector<double2> hxy(n);
  for (int i = 0; i < n; ++i) hxy[i] = make_double2(i * 1e-3, -i * 1e-3);
  std::vector<int> hp((size_t)R * km);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < hp.size(); ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    hp[i] = (int)(s % n);
  }
  double2* xy; iv4* perm; double* out;
  CK(hipMalloc(&xy, n * sizeof(double2)));
  CK(hipMalloc(&perm, hp.size() * 4));
  CK(hipMalloc(&out, (size_t)256 * 256 * 64 * 8));
  CK(hipMemcpy(xy, hxy.data(), n * sizeof(double2), hipMemcpyHostToDevice));
  CK(hipMemcpy(perm, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  const double idx_bytes = (double)hp.size() * 4;
  for (int grid : {256 * 8, 256 * 16, 256 * 32}) {
    float t;
    t = run<1, 1>(xy, perm, groups, n, out, grid);
    printf("grid %5d idx-only U1  %.3f ms  %.2f TB/s of indices\n", grid, t, idx_bytes / t / 1e9);
    t = run<4, 1>(xy, perm, groups, n, out, grid);
    printf("grid %5d idx-only U4  %.3f ms  %.2f TB/s of indices\n", grid, t, idx_bytes / t / 1e9);
    t = run<1, 0>(xy, perm, groups, n, out, grid);
    printf("grid %5d gather   U1  %.3f ms  %.2f G gathers/s\n", grid, t, (double)R * km / t / 1e6);
    t = run<2, 0>(xy, perm, groups, n, out, grid);
    printf("grid %5d gather   U2  %.3f ms  %.2f G gathers/s\n", grid, t, (double)R * km / t / 1e6);
    t = run<4, 0>(xy, perm, groups, n, out, grid);
    printf("grid %5d gather   U4  %.3f ms  %.2f G gathers/s\n", grid, t, (double)R * km / t / 1e6);
    t = run<4, 2>(xy, perm, groups, n, out, grid);
    printf("grid %5d seq      U4  %.3f ms  %.2f G gathers/s\n", grid, t, (double)R * km / t / 1e6);
  }
  return 0;
}
