// ubench_rng.hip -- throughput of the fused kernels' building blocks on gfx950:
// Philox4x32-10 (mad_u64 form, xor3 form), Threefry4x32 (20 / 13 rounds), Box-Muller on
// given words, and single instructions.  Each thread runs ITER independent blocks; a
// sink keeps everything live.  Prints blocks/s per GPU and cycles/block/SIMD estimates.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ubench_rng ubench_rng.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../distributed-correlation_amd/csrc/dcor_device.h"

using namespace dcor;
#define ITER 2048

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return a ^ b ^ c;  // gfx950 has no v_xor3_b32
}

__device__ __forceinline__ U4 philox_x3(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0), n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

template <int R>
__device__ __forceinline__ U4 threefry(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                       uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  const uint32_t k4 = 0x1BD11BDAu ^ k0 ^ k1 ^ k2 ^ k3;
  const uint32_t ks[5] = {k0, k1, k2, k3, k4};
  const int rot[8][2] = {{10, 26}, {11, 21}, {13, 27}, {23, 5}, {6, 20}, {17, 11}, {25, 10}, {18, 20}};
  x0 += k0; x1 += k1; x2 += k2; x3 += k3;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & 1) {
      x0 += x3; x3 = rotl(x3, rot[r % 8][0]); x3 ^= x0;
      x2 += x1; x1 = rotl(x1, rot[r % 8][1]); x1 ^= x2;
    } else {
      x0 += x1; x1 = rotl(x1, rot[r % 8][0]); x1 ^= x0;
      x2 += x3; x3 = rotl(x3, rot[r % 8][1]); x3 ^= x2;
    }
    if ((r & 3) == 3) {
      const int s = (r >> 2) + 1;
      x0 += ks[s % 5]; x1 += ks[(s + 1) % 5]; x2 += ks[(s + 2) % 5]; x3 += ks[(s + 3) % 5] + s;
    }
  }
  return U4{x0, x1, x2, x3};
}

template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t* sink, uint32_t k0, uint32_t k1) {
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  double dacc = 0.0;
  for (int it = 0; it < ITER; ++it) {
    U4 w;
    if constexpr (KIND == 0) w = philox(gid, (uint32_t)it, 1u, 0u, k0, k1);
    if constexpr (KIND == 1) w = philox_x3(gid, (uint32_t)it, 1u, 0u, k0, k1);
    if constexpr (KIND == 2) w = threefry<20>(gid, (uint32_t)it, 1u, 0u, k0, k1, 7u, 9u);
    if constexpr (KIND == 3) w = threefry<13>(gid, (uint32_t)it, 1u, 0u, k0, k1, 7u, 9u);
    if constexpr (KIND == 4) {  // Box-Muller only, cheap words
      w = U4{gid * 0x9E3779B9u + it, gid ^ (it * 0x85EBCA6Bu), it * 0xC2B2AE35u + gid, gid + it};
      double a, b;
      normal_pair(w, &a, &b);
      dacc += a + b;
      continue;
    }
    if constexpr (KIND == 5) {  // Philox + Box-Muller (one Gaussian sample of the engine)
      w = philox(gid, (uint32_t)it, 1u, 0u, k0, k1);
      double a, b;
      normal_pair(w, &a, &b);
      dacc += a + b;
      continue;
    }
    if constexpr (KIND == 6) {  // unit Laplace only
      const double u = u53(gid * 0x9E3779B9u + it, gid ^ (it * 0x85EBCA6Bu));
      dacc += unit_laplace(u);
      continue;
    }
    acc ^= w.w0 ^ w.w1 ^ w.w2 ^ w.w3;
  }
  if (acc == 0x12345678u || dacc == 1.2345) sink[gid] = acc + (uint32_t)dacc;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* sink;
  hipMalloc(&sink, 64u << 20);
  const char* names[] = {"philox10 (mad_u64)", "philox10 (dup)", "threefry4x32-20",
                         "threefry4x32-13", "box-muller only", "philox10 + box-muller",
                         "unit laplace only"};
  const int blocks = ncu * 16;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    for (int kind = 0; kind < 7; ++kind) {
      void (*fn)(uint32_t*, uint32_t, uint32_t) = nullptr;
      switch (kind) {
        case 0: fn = k<0>; break; case 1: fn = k<1>; break; case 2: fn = k<2>; break;
        case 3: fn = k<3>; break; case 4: fn = k<4>; break; case 5: fn = k<5>; break;
        default: fn = k<6>;
      }
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, sink, 1u, 2u);
      hipEventRecord(a);
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, sink, 3u, 4u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double items = (double)blocks * 256 * ITER;
      const double per_s = items / (ms * 1e-3);
      // SIMD-cycles per item per wave of 64 at 2.4 GHz nominal: (cycles per SIMD) / (items per SIMD / 64)
      const double cyc = (ms * 1e-3 * 2.4e9) / (items / (ncu * 4.0) / 64.0);
      if (rep == 1) printf("%-24s %8.3f ms  %10.3e items/s  %7.1f wave-cycles/item\n", names[kind], ms, per_s, cyc);
    }
  }
  return 0;
}
