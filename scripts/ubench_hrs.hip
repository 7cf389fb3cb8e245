// ubench_hrs.hip -- where does the C5 (HRS pre-materialised) streaming kernel spend its time?
// Standalone: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/ubench_hrs.hip -o scripts/ubench_hrs
// Variants: 0 full (INT stream + NI gathers), 1 INT stream only, 2 NI gathers only,
// 3 NI with coalesced (identity) batches, 4 HBM streams only (no panel reads).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct DD { double hi, lo; };
__device__ __forceinline__ void ks_acc(DD& acc, double x) {
  const double s = acc.hi + x;
  const double bb = s - acc.hi;
  acc.lo += (acc.hi - (s - bb)) + (x - bb);
  acc.hi = s;
}
__device__ __forceinline__ double clip(double x, double L) { return fmax(fmin(x, L), -L); }

template <int V, int UNR>
__global__ __launch_bounds__(256) void k(int n, int kb, const double* __restrict__ ll,
                                         const int* __restrict__ perm, const double* __restrict__ lx,
                                         const double* __restrict__ ly, const double2* __restrict__ soc,
                                         const double2* __restrict__ xy, double* __restrict__ out) {
  const int rep = blockIdx.x, tid = threadIdx.x;
  const double* l = ll + (size_t)rep * n;
  const int* pm = perm + (size_t)rep * 2 * kb;
  const double* ax = lx + (size_t)rep * kb;
  const double* ay = ly + (size_t)rep * kb;
  DD sU{0, 0}, sU2{0, 0}, sP{0, 0}, sT{0, 0}, sT2{0, 0};
  const double bs = 0.37, lr = 3.0, bx = 0.11, by = 0.13, md = 2.0;
  if (V == 0 || V == 1 || V == 4) {
    int i = tid;
    for (; i + (UNR - 1) * 256 < n; i += UNR * 256) {
      double lv[UNR];
      double2 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        lv[u] = l[i + u * 256];
        v[u] = (V == 4) ? make_double2(1.0, 0.5) : soc[i + u * 256];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const double Uc = clip((v[u].x + bs * lv[u]) * v[u].y, lr);
        ks_acc(sU, Uc);
        ks_acc(sU2, Uc * Uc);
      }
    }
    for (; i < n; i += 256) {
      const double2 v = soc[i];
      const double Uc = clip((v.x + bs * l[i]) * v.y, lr);
      ks_acc(sU, Uc);
      ks_acc(sU2, Uc * Uc);
    }
  }
  if (V == 0 || V == 2 || V == 3 || V == 4) {
    int j = tid;
    for (; j + (UNR - 1) * 256 < kb; j += UNR * 256) {
      int2 pr[UNR];
      double a[UNR], b[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int jj = j + u * 256;
        pr[u] = *reinterpret_cast<const int2*>(pm + 2 * jj);
        if (V == 3) pr[u] = make_int2(2 * jj, 2 * jj + 1);
        a[u] = ax[jj]; b[u] = ay[jj];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        double2 p, q;
        if (V == 4) { p = make_double2(pr[u].x, 1.0); q = make_double2(pr[u].y, 2.0); }
        else { p = xy[pr[u].x]; q = xy[pr[u].y]; }
        const double xt = (p.x + q.x) * 0.5 + bx * a[u];
        const double yt = (p.y + q.y) * 0.5 + by * b[u];
        ks_acc(sP, xt * yt);
        const double T = md * xt * yt;
        ks_acc(sT, T);
        ks_acc(sT2, T * T);
      }
    }
    for (; j < kb; j += 256) {
      const double2 p = xy[pm[2 * j]], q = xy[pm[2 * j + 1]];
      const double xt = (p.x + q.x) * 0.5 + bx * ax[j];
      const double yt = (p.y + q.y) * 0.5 + by * ay[j];
      ks_acc(sP, xt * yt);
      const double T = md * xt * yt;
      ks_acc(sT, T);
      ks_acc(sT2, T * T);
    }
  }
  double s = sU.hi + sU.lo + sU2.hi + sU2.lo + sP.hi + sP.lo + sT.hi + sT.lo + sT2.hi + sT2.lo;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) atomicAdd(out + rep, s);
}

template <int V, int UNR>
float run(int R, int n, int kb, double* ll, int* perm, double* lx, double* ly, double2* soc,
          double2* xy, double* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k<V, UNR><<<R, 256>>>(n, kb, ll, perm, lx, ly, soc, xy, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int it = 5;
  for (int t = 0; t < it; ++t) k<V, UNR><<<R, 256>>>(n, kb, ll, perm, lx, ly, soc, xy, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / it;
}

// Variant 5: LDS-resident panel components.  One rep per 1024-thread workgroup; the clipped
// x column fills LDS, x gathers give xt per batch (registers), then the y column replaces it.
#define LDS_N 19968
#define NT 1024
#define SLOTS 10
__global__ __launch_bounds__(NT) void k_lds(int n, int kb, const double* __restrict__ ll,
                                            const int* __restrict__ perm, const double* __restrict__ lx,
                                            const double* __restrict__ ly, const double2* __restrict__ soc,
                                            const double* __restrict__ xc, const double* __restrict__ yc,
                                            double* __restrict__ out) {
  __shared__ double pan[LDS_N];
  const int rep = blockIdx.x, tid = threadIdx.x;
  const double* l = ll + (size_t)rep * n;
  const int* pm = perm + (size_t)rep * 2 * kb;
  const double* ax = lx + (size_t)rep * kb;
  const double* ay = ly + (size_t)rep * kb;
  DD sU{0, 0}, sU2{0, 0}, sP{0, 0}, sT{0, 0}, sT2{0, 0};
  const double bs = 0.37, lr = 3.0, bx = 0.11, by = 0.13, md = 2.0;
  int2 pr[SLOTS];
  double xt[SLOTS], yv[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int j = tid + s * NT;
    pr[s] = j < kb ? *reinterpret_cast<const int2*>(pm + 2 * j) : make_int2(0, 0);
    xt[s] = j < kb ? ax[j] : 0.0;
  }
  for (int i = tid; i < n; i += NT) pan[i] = xc[i];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int j = tid + s * NT;
    yv[s] = j < kb ? ay[j] : 0.0;
    xt[s] = (pan[pr[s].x] + pan[pr[s].y]) * 0.5 + bx * xt[s];
  }
  __syncthreads();
  for (int i = tid; i < n; i += NT) pan[i] = yc[i];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int j = tid + s * NT;
    if (j < kb) {
      const double yt = (pan[pr[s].x] + pan[pr[s].y]) * 0.5 + by * yv[s];
      ks_acc(sP, xt[s] * yt);
      const double T = md * xt[s] * yt;
      ks_acc(sT, T);
      ks_acc(sT2, T * T);
    }
  }
  {
    int i = tid;
    for (; i + 3 * NT < n; i += 4 * NT) {
      double lv[4];
      double2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { lv[u] = l[i + u * NT]; v[u] = soc[i + u * NT]; }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double Uc = clip((v[u].x + bs * lv[u]) * v[u].y, lr);
        ks_acc(sU, Uc);
        ks_acc(sU2, Uc * Uc);
      }
    }
    for (; i < n; i += NT) {
      const double2 v = soc[i];
      const double Uc = clip((v.x + bs * l[i]) * v.y, lr);
      ks_acc(sU, Uc);
      ks_acc(sU2, Uc * Uc);
    }
  }
  double s = sU.hi + sU.lo + sU2.hi + sU2.lo + sP.hi + sP.lo + sT.hi + sT.lo + sT2.hi + sT2.lo;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) atomicAdd(out + rep, s);
}

float run_lds(int R, int n, int kb, double* ll, int* perm, double* lx, double* ly, double2* soc,
              double* xc, double* yc, double* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k_lds<<<R, NT>>>(n, kb, ll, perm, lx, ly, soc, xc, yc, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int it = 5;
  for (int t = 0; t < it; ++t) k_lds<<<R, NT>>>(n, kb, ll, perm, lx, ly, soc, xc, yc, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / it;
}

int main() {
  const int n = 19433, kb = 9716, R = 4096;
  std::vector<int> hp((size_t)R * 2 * kb);
  srand(1);
  std::vector<int> idx(n);
  for (int r = 0; r < R; ++r) {
    for (int i = 0; i < n; ++i) idx[i] = i;
    for (int t = 0; t < 2 * kb; ++t) {
      int s = t + rand() % (n - t);
      int tmp = idx[t]; idx[t] = idx[s]; idx[s] = tmp;
      hp[(size_t)r * 2 * kb + t] = idx[t];
    }
  }
  double *ll, *lx, *ly, *out;
  int* perm;
  double2 *soc, *xy;
  CK(hipMalloc(&ll, (size_t)R * n * 8));
  CK(hipMalloc(&lx, (size_t)R * kb * 8));
  CK(hipMalloc(&ly, (size_t)R * kb * 8));
  CK(hipMalloc(&perm, (size_t)R * 2 * kb * 4));
  CK(hipMalloc(&soc, (size_t)n * 16));
  CK(hipMalloc(&xy, (size_t)n * 16));
  CK(hipMalloc(&out, (size_t)R * 8));
  CK(hipMemset(ll, 0, (size_t)R * n * 8));
  CK(hipMemset(lx, 0, (size_t)R * kb * 8));
  CK(hipMemset(ly, 0, (size_t)R * kb * 8));
  CK(hipMemset(soc, 0, (size_t)n * 16));
  CK(hipMemset(xy, 0, (size_t)n * 16));
  CK(hipMemset(out, 0, (size_t)R * 8));
  CK(hipMemcpy(perm, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  const double bytes = (double)R * (8.0 * n + 4.0 * 2 * kb + 16.0 * kb);
  const char* names[] = {"full", "INT only", "NI gather only", "NI coalesced", "HBM streams only"};
  float ms[5][2];
  ms[0][0] = run<0, 4>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[1][0] = run<1, 4>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[2][0] = run<2, 4>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[3][0] = run<3, 4>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[4][0] = run<4, 4>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[0][1] = run<0, 8>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[1][1] = run<1, 8>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[2][1] = run<2, 8>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[3][1] = run<3, 8>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  ms[4][1] = run<4, 8>(R, n, kb, ll, perm, lx, ly, soc, xy, out);
  double *xc, *yc;
  CK(hipMalloc(&xc, (size_t)n * 8));
  CK(hipMalloc(&yc, (size_t)n * 8));
  CK(hipMemset(xc, 0, (size_t)n * 8));
  CK(hipMemset(yc, 0, (size_t)n * 8));
  const float mlds = run_lds(R, n, kb, ll, perm, lx, ly, soc, xc, yc, out);
  printf("%-18s       %.3f ms   (full-bytes GB/s: %.0f)\n", "LDS panel", mlds, bytes / (mlds * 1e-3) / 1e9);
  for (int v = 0; v < 5; ++v)
    printf("%-18s UNR4 %.3f ms  UNR8 %.3f ms   (full-bytes GB/s at UNR8: %.0f)\n", names[v], ms[v][0],
           ms[v][1], bytes / (ms[v][1] * 1e-3) / 1e9);
  return 0;
}
