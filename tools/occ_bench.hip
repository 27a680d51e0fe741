// Occupancy microbenchmark of the off-diagonal GEMM1 loop (k_chol.hip gemm1_a32: 32-row Lt_J stages
// through a 2 x 32 KiB LDS-DMA ring, each wave's Lt_I columns straight into registers): how fast does
// ONE 8-wave workgroup alone on a CU run it, against two per CU (production), and against one
// 16-wave workgroup whose waves split the tile's row blocks (wave w: columns 16 (w & 7), row blocks
// 4 (w >> 3) .. +3)?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tblup_amd/csrc tools/occ_bench.hip -o tools/occ_bench
//   tools/occ_bench [nL]   -> one JSON line per variant (TFLOP/s over the launch, fp64)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "tblup_internal.h"

using namespace tblup;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int TT = TILE * TILE;

__device__ __forceinline__ v4d mfma64_nega(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
}
__device__ __forceinline__ int lt_off(int k, int x) { return k * TILE + 2 * ((x >> 1) ^ (8 * (k & 1))) + (x & 1); }

template <int NW, int NCB>
__device__ __forceinline__ void gemm1(const double* __restrict__ ltJ, const double* __restrict__ ltI, int nL, double* lds,
                                      v4d (&acc)[NCB]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wc = w & 7, cb0 = (w >> 3) * NCB;
  constexpr int AS = 32 * TILE;
  constexpr int RPW = 32 / NW;   // stage rows issued per wave
  const int nst = 4 * nL;
  auto src_of = [&](int s) { return (int64_t)(s >> 2) * TT + (s & 3) * AS; };
  auto issue_a = [&](int s) {
    double* slot = lds + (s & 1) * AS;
    const int64_t src = src_of(s);
#pragma unroll
    for (int e = 0; e < RPW; ++e) {
      const int k = RPW * w + e;
      glds16_asm(ltJ + src + k * TILE + 2 * (l ^ (8 * (k & 1))), slot + k * TILE);
    }
  };
  const double* bcol = ltI + 16 * wc + (l & 15) + (l >> 4) * TILE;
  double bc[8];
  issue_a(0);
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) bc[kk] = bcol[4 * kk * TILE];
  for (int s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool more = s + 1 < nst;
    if (more) issue_a(s + 1);
    const double* bs = bcol + src_of(more ? s + 1 : s);
    const double* As = lds + (s & 1) * AS;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = 4 * kk + (l >> 4);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[cb] = mfma64_nega(As[lt_off(k, 16 * (cb0 + cb) + (l & 15))], bc[kk], acc[cb]);
      if (more) bc[kk] = bs[4 * kk * TILE];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// T-unit pair: 8 waves, one workgroup per CU (256 VGPRs), wave w holds the 16 columns w of TWO tiles
// (Lt_I and Lt_I2 in registers) against one shared Lt_J stage: 16 MFMAs per 8 LDS A reads
__device__ __forceinline__ void gemm1_pair(const double* __restrict__ ltJ, const double* __restrict__ ltI,
                                           const double* __restrict__ ltI2, int nL, double* lds, v4d (&acc)[8],
                                           v4d (&acc2)[8]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int AS = 32 * TILE;
  const int nst = 4 * nL;
  auto src_of = [&](int s) { return (int64_t)(s >> 2) * TT + (s & 3) * AS; };
  auto issue_a = [&](int s) {
    double* slot = lds + (s & 1) * AS;
    const int64_t src = src_of(s);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * w + e;
      glds16_asm(ltJ + src + k * TILE + 2 * (l ^ (8 * (k & 1))), slot + k * TILE);
    }
  };
  const double* bcol = ltI + 16 * w + (l & 15) + (l >> 4) * TILE;
  const double* bcol2 = ltI2 + 16 * w + (l & 15) + (l >> 4) * TILE;
  double bc[8], bd[8];
  issue_a(0);
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    bc[kk] = bcol[4 * kk * TILE];
    bd[kk] = bcol2[4 * kk * TILE];
  }
  for (int s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool more = s + 1 < nst;
    if (more) issue_a(s + 1);
    const int64_t so = src_of(more ? s + 1 : s);
    const double* As = lds + (s & 1) * AS;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = 4 * kk + (l >> 4);
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const double a = As[lt_off(k, 16 * cb + (l & 15))];
        acc[cb] = mfma64_nega(a, bc[kk], acc[cb]);
        acc2[cb] = mfma64_nega(a, bd[kk], acc2[cb]);
      }
      if (more) {
        bc[kk] = bcol[so + 4 * kk * TILE];
        bd[kk] = bcol2[so + 4 * kk * TILE];
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

__global__ __launch_bounds__(512, 1) void k_pair(const double* L, int rows, int nL, double* out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  v4d acc[8], acc2[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) acc[cb] = acc2[cb] = v4d{0.0, 0.0, 0.0, 0.0};
  const int g = blockIdx.x;
  const double* ltJ = L + (int64_t)(g % rows) * 8 * TT;
  const double* ltI = L + (int64_t)((g * 7 + 3) % rows) * 8 * TT;
  const double* ltI2 = L + (int64_t)((g * 11 + 5) % rows) * 8 * TT;
  gemm1_pair(ltJ, ltI, ltI2, nL, lds, acc, acc2);
  double s = 0.0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) s += acc[cb][0] + acc[cb][1] + acc[cb][2] + acc[cb][3] + acc2[cb][0] + acc2[cb][3];
  if (s == 12345.678) out[g] = s;
}

// every workgroup: GEMM1 of nL terms for one tile, rows of 8 tiles in L (row r = tiles r*8 .. r*8+7)
template <int NW, int NCB, int MINB>
__global__ __launch_bounds__(64 * NW, MINB) void k_bench(const double* L, int rows, int nL, double* out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  v4d acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = v4d{0.0, 0.0, 0.0, 0.0};
  const int g = blockIdx.x;
  const double* ltJ = L + (int64_t)(g % rows) * 8 * TT;
  const double* ltI = L + (int64_t)((g * 7 + 3) % rows) * 8 * TT;
  gemm1<NW, NCB>(ltJ, ltI, nL, lds, acc);
  double s = 0.0;
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) s += acc[cb][0] + acc[cb][1] + acc[cb][2] + acc[cb][3];
  if (s == 12345.678) out[g] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

template <int NW, int NCB, int MINB>
void run(const char* name, const double* L, int rows, int nL, int grid, size_t lds_bytes, double* out) {
  auto k = k_bench<NW, NCB, MINB>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds_bytes, 0, L, rows, nL, out);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds_bytes, 0, L, rows, nL, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double tiles = (double)grid * (NW == 16 ? 1.0 : 1.0);
  const double flops = tiles * nL * 2.0 * 128.0 * 128.0 * 128.0 * reps;
  printf("{\"variant\": \"%s\", \"grid\": %d, \"lds_kb\": %zu, \"nL\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.2f}\n", name,
         grid, lds_bytes / 1024, nL, ms / reps, flops / (ms * 1e-3) / 1e12);
}

void run_pair(const double* L, int rows, int nL, int grid, double* out) {
  const size_t lds_bytes = 64 * 1024;
  CK(hipFuncSetAttribute((const void*)k_pair, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_pair, dim3(grid), dim3(512), lds_bytes, 0, L, rows, nL, out);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_pair, dim3(grid), dim3(512), lds_bytes, 0, L, rows, nL, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double flops = 2.0 * grid * nL * 2.0 * 128.0 * 128.0 * 128.0 * reps;
  printf("{\"variant\": \"w8_pair_one_per_cu\", \"grid\": %d, \"nL\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.2f}\n", grid,
         nL, ms / reps, flops / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
  const int nL = argc > 1 ? atoi(argv[1]) : 6;
  const int rows = 512;   // 512 x 8 tiles x 128 KiB = 512 MiB of Lt tiles (beyond the MALL: HBM-served)
  double *L, *out;
  CK(hipMalloc(&L, (size_t)rows * 8 * TT * 8));
  CK(hipMalloc(&out, 1 << 20));
  std::vector<double> h((size_t)8 * TT);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
  for (int r = 0; r < rows; ++r) CK(hipMemcpy(L + (size_t)r * 8 * TT, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  const size_t base = 64 * 1024;   // the 2 x 32 KiB ring
  for (int rounds : {1, 4}) {
    // production: 8 waves, 72 KiB-class LDS, two workgroups per CU when the grid allows
    run<8, 8, 4>("w8_two_per_cu", L, rows, nL, 512 * rounds, base, out);
    // one 8-wave workgroup per CU (LDS beyond half the CU)
    run<8, 8, 4>("w8_one_per_cu", L, rows, nL, 256 * rounds, 96 * 1024, out);
    // one 16-wave workgroup per CU: waves split the row blocks (4 per wave)
    run<16, 4, 1>("w16_one_per_cu", L, rows, nL, 256 * rounds, base, out);
    run<16, 4, 1>("w16_lds96", L, rows, nL, 256 * rounds, 96 * 1024, out);
    run_pair(L, rows, nL, 256 * rounds, out);
  }
  // L2-resident operands (an individual's Lt rows shared by its tiles): 8 rows only
  for (int rounds : {4}) {
    run<8, 8, 4>("w8_two_per_cu_l2", L, 8, nL, 512 * rounds, base, out);
    run<16, 4, 1>("w16_one_per_cu_l2", L, 8, nL, 256 * rounds, base, out);
    run_pair(L, 8, nL, 256 * rounds, out);
  }
  return 0;
}
