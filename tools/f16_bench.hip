// Microbenchmark of the diagonal kernel's 16x16 factorisation (factor16) variants.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tblup_amd/csrc tools/f16_bench.hip -o tools/f16_bench
// One wave per workgroup factorises an SPD 16x16 block in LDS `reps` times (restoring it
// in between); prints ns per factorisation per variant (0 = previous, 1 = current).
#include "k_chol.hip"
#include <cstdio>
#include <vector>

using namespace tblup;

__device__ __forceinline__ double rdlane0(double x, int lane) {
  const long long bits = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)bits, lane);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ void factor16_v0(double* D, double* X, int l) {
  const int i = l & 15, g = l >> 4;
  double v[NB], e[NB], pv[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    v[c] = (c <= i) ? D[bo(i, c)] : D[bo(c, i)];   // symmetric row from the lower triangle
    e[c] = (c == i) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double piv = rdlane0(v[j], j);
    pv[j] = piv;
    double r[NB], ej[NB];
#pragma unroll
    for (int c = j + 1; c < NB; ++c) r[c] = rdlane0(v[c], j);
#pragma unroll
    for (int c = 0; c < j; ++c) ej[c] = rdlane0(e[c], j);
    const double li = v[j] * recip(piv);
#pragma unroll
    for (int c = j + 1; c < NB; ++c) v[c] = __builtin_fma(-li, r[c], v[c]);
    const bool below = i > j;
#pragma unroll
    for (int c = 0; c < j; ++c) e[c] = below ? __builtin_fma(-li, ej[c], e[c]) : e[c];
    e[j] = below ? -li : e[j];
  }
  // deferred scaling: L_ic = T_ic / sqrt(piv_c), X_ic = E_ic / sqrt(piv_i)
  const double rs_own = 1.0 / sqrt(v[i]);   // v[i] = piv_i
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    double vc = v[0], ec = e[0], pc = pv[0];
#pragma unroll
    for (int cc = 1; cc < NB; ++cc) {
      vc = (c == cc) ? v[cc] : vc;
      ec = (c == cc) ? e[cc] : ec;
      pc = (c == cc) ? pv[cc] : pc;
    }
    X[bo(i, c)] = (i >= c) ? ec * rs_own : 0.0;
    if (i >= c) D[bo(i, c)] = vc * (1.0 / sqrt(pc));
  }
}




template <int V>
__global__ __launch_bounds__(64) void bench_f16(const double* src, double* out, int reps) {
  __shared__ double D[BLKD], X[BLKD];
  const int l = threadIdx.x;
  for (int e = l; e < BLKD; e += 64) D[e] = src[e];
  __syncthreads();
  double acc = 0.0;
  for (int r = 0; r < reps; ++r) {
    if (V == 0) factor16_v0(D, X, l);
    else factor16(D, X, l);
    __syncthreads();
    acc += X[bo(l & 15, 0)];
    for (int e = l; e < BLKD; e += 64) D[e] = src[e];
    __syncthreads();
  }
  for (int e = l; e < BLKD; e += 64) out[blockIdx.x * 2 * BLKD + e] = X[e];
  for (int e = l; e < BLKD; e += 64) out[blockIdx.x * 2 * BLKD + BLKD + e] = D[e];
  if (acc == 1234.5) out[0] = acc;
}

int main() {
  // SPD block A = M M^T + 16 I, stored in the packed-block (bo) layout, lower part used
  std::vector<double> M(256), A(256), Ab(256);
  for (int i = 0; i < 256; ++i) M[i] = ((i * 37) % 17) / 17.0 - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = (i == j) ? 16.0 : 0.0;
      for (int k = 0; k < 16; ++k) s += M[i * 16 + k] * M[j * 16 + k];
      A[i * 16 + j] = s;
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) Ab[bo(i, j)] = A[i * 16 + j];
  double *src, *out;
  const int nwg = 1024, reps = 200;
  hipMalloc(&src, 256 * 8);
  hipMalloc(&out, (size_t)nwg * 2 * BLKD * 8);
  hipMemcpy(src, Ab.data(), 256 * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<double> res[2];
  for (int v = 0; v < 2; ++v) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a, 0);
      if (v == 0) hipLaunchKernelGGL(bench_f16<0>, dim3(nwg), dim3(64), 0, 0, src, out, reps);
      if (v == 1) hipLaunchKernelGGL(bench_f16<1>, dim3(nwg), dim3(64), 0, 0, src, out, reps);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    res[v].resize(2 * BLKD);
    hipMemcpy(res[v].data(), out, 2 * BLKD * 8, hipMemcpyDeviceToHost);
    // nwg one-wave WGs over 256 CUs x 4 SIMDs: 1 wave per SIMD
    printf("variant %d  %.1f ns per factor16 (one wave per SIMD)\n", v, best * 1e6 / reps / ((nwg + 1023) / 1024));
  }
  double md = 0;
  for (int e = 0; e < 2 * BLKD; ++e) md = fmax(md, fabs(res[0][e] - res[1][e]));
  printf("max |v0 - v1| = %g\n", md);
  return 0;
}
