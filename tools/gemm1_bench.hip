// Microbenchmark of the off-diagonal GEMM1 building block (gemm1_tt) in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tblup_amd/csrc tools/gemm1_bench.hip -o tools/gemm1_bench
// Modes: 0 = gemm1_tt<2> (production), 1 = gemm1_tt<3>, 2 = MFMA-only (no memory), 3 = D=2 on an
// L2-resident buffer, 4 = 8-wave workgroups (128 x 16 per wave), 5 = D=2 on a 64-row-block buffer.  Prints TFLOP/s (fp64) over nwg workgroups of J*8 16-row stages.
#include "k_chol.hip"
#include <cstdio>
#include <vector>

using namespace tblup;

template <int D, int OCC>
__global__ __launch_bounds__(256, OCC) void bench_gemm1(const double* L, int64_t rows_per_wg, int64_t wrap, int J,
                                                        double* out) {
  __shared__ __attribute__((aligned(16))) double lds[D * 2 * LTS];
  v4d acc[8][2];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) acc[cb][ib] = v4d{0.0, 0.0, 0.0, 0.0};
  const int64_t g = blockIdx.x;
  const double* ltJ = L + ((g / 4) % wrap) * rows_per_wg;          // shared by 4 WGs (one "individual")
  const double* ltI = L + ((g + 7) % wrap) * rows_per_wg;
  gemm1_tt<D>(ltJ, ltI, J, lds, acc);
  double s = 0.0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) s += acc[cb][ib][0] + acc[cb][ib][1] + acc[cb][ib][2] + acc[cb][ib][3];
  if (s == 12345.678) out[g] = s;
}

// 8-wave variant: wave w owns i rows 16w..16w+15 (acc[8][1]); 512 threads, 2 WGs per CU
template <int D>
__device__ __forceinline__ void gemm1_tt_w8(const double* __restrict__ ltJ, const double* __restrict__ ltI, int J,
                                            double* lds, v4d (&acc)[8]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nst = 8 * J;
  if (nst == 0) return;
  auto issue = [&](int s) {
    double* slot = lds + (s % D) * 2 * LTS;
    const int64_t src = (int64_t)(s >> 3) * TT + (s & 7) * LTS;
    // 16 rows x 1 KiB per operand: 8 waves x 2 rows each, for J then I
    const int k = 2 * (w & 7) + 0;
    const double* srcJ = ltJ + src;
    const double* srcI = ltI + src;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int kk = k + e;
      __builtin_amdgcn_global_load_lds(srcJ + kk * TILE + 2 * (l ^ (8 * (kk & 1))), (lds_ptr_t)(slot + kk * TILE), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(srcI + kk * TILE + 2 * (l ^ (8 * (kk & 1))), (lds_ptr_t)(slot + LTS + kk * TILE), 16, 0, 0);
    }
  };
  for (int s = 0; s < D - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    if (s + D - 2 < nst) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + D - 1 < nst) issue(s + D - 1);
    const double* As = lds + (s % D) * 2 * LTS;
    const double* Bs = As + LTS;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kk + (l >> 4);
      const double bv = Bs[lt_off(k, 16 * w + (l & 15))];
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) acc[cb] = mfma64_nega(As[lt_off(k, 16 * cb + (l & 15))], bv, acc[cb]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int D>
__global__ __launch_bounds__(512, 2) void bench_gemm1_w8(const double* L, int64_t rows_per_wg, int64_t wrap, int J,
                                                         double* out) {
  __shared__ __attribute__((aligned(16))) double lds[D * 2 * LTS];
  v4d acc[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) acc[cb] = v4d{0.0, 0.0, 0.0, 0.0};
  const int64_t g = blockIdx.x;
  const double* ltJ = L + ((g / 4) % wrap) * rows_per_wg;
  const double* ltI = L + ((g + 7) % wrap) * rows_per_wg;
  gemm1_tt_w8<D>(ltJ, ltI, J, lds, acc);
  double s = 0.0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) s += acc[cb][0] + acc[cb][1] + acc[cb][2] + acc[cb][3];
  if (s == 12345.678) out[g] = s;
}

__global__ __launch_bounds__(256, 2) void bench_mfma_only(int J, double* out) {
  const int l = threadIdx.x & 63;
  v4d acc[8][2];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) acc[cb][ib] = v4d{0.0, 0.0, 0.0, 0.0};
  double av = 1.0 + l * 1e-3, bv = 2.0 - l * 1e-3;
  for (int s = 0; s < 8 * J; ++s)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) acc[cb][ib] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[cb][ib], 0, 0, 0);
  double s = 0.0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) s += acc[cb][ib][0];
  if (s == 12345.678) out[blockIdx.x] = s;
}

int main(int argc, char** argv) {
  const int J = argc > 1 ? atoi(argv[1]) : 6;
  const int nwg = argc > 2 ? atoi(argv[2]) : 2048;
  const int64_t rows = (int64_t)J * TT;      // doubles of one Lt block row (J tiles)
  const int64_t wrap_big = 4096, wrap_small = 8;
  double *L, *out;
  hipMalloc(&L, (size_t)wrap_big * rows * 8);
  hipMalloc(&out, (size_t)nwg * 8);
  std::vector<double> h((size_t)rows);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
  for (int64_t r = 0; r < wrap_big; ++r) hipMemcpy(L + r * rows, h.data(), rows * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double flops = (double)nwg * 2.0 * 128 * 128 * 128 * J;
  for (int mode = 0; mode < 6; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a, 0);
      if (mode == 0) hipLaunchKernelGGL((bench_gemm1<2, 2>), dim3(nwg), dim3(256), 0, 0, L, rows, wrap_big, J, out);
      if (mode == 1) hipLaunchKernelGGL((bench_gemm1<3, 1>), dim3(nwg), dim3(256), 0, 0, L, rows, wrap_big, J, out);
      if (mode == 2) hipLaunchKernelGGL(bench_mfma_only, dim3(nwg), dim3(256), 0, 0, J, out);
      if (mode == 3) hipLaunchKernelGGL((bench_gemm1<2, 2>), dim3(nwg), dim3(256), 0, 0, L, rows, wrap_small, J, out);
      if (mode == 4) hipLaunchKernelGGL((bench_gemm1_w8<2>), dim3(nwg), dim3(512), 0, 0, L, rows, wrap_big, J, out);
      if (mode == 5) hipLaunchKernelGGL((bench_gemm1<2, 2>), dim3(nwg), dim3(256), 0, 0, L, rows, (int64_t)64, J, out);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("mode %d  J=%d nwg=%d  %.3f ms  %.1f TFLOP/s\n", mode, J, nwg, best, flops / (best * 1e-3) / 1e12);
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
