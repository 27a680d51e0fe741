// Microbenchmark of the off-diagonal GRM tile phase (int8 MFMA on 2-bit packed rows) in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tblup_amd/csrc tools/grm_bench.hip -o tools/grm_bench
//   tools/grm_bench [nblk=20] [nwg=2048]
// Modes: 0 = i8_tt8_pk64<4> (production), 1 = same loads / LDS reads without the 2-bit unpack,
// 2 = unpack + MFMA from registers (no memory), 3 = MFMA only.  Rows are gathered at random
// from a 50k-row packed table like the split matrix.  Prints int8 TOPS over nwg tiles.
#include "k_chol.hip"
#include <cstdio>
#include <vector>

using namespace tblup;

template <int MODE>
__device__ __forceinline__ v4i opnd(uint32_t x) {
  if constexpr (MODE == 1 || MODE == 3) return v4i{(int)x, (int)(x ^ 1u), (int)(x ^ 2u), (int)(x ^ 3u)};
  return unpack16(x);
}

template <int D, int MODE>
__device__ __forceinline__ void tile_loop(const uint8_t* sa, const uint8_t* sb, int64_t nblk, uint8_t* lds,
                                          v4i (&cnt)[8]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) cnt[cb] = v4i{0, 0, 0, 0};
  const int64_t nst = (nblk + 3) >> 2;
  constexpr int TB = TILE * 64;
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  if constexpr (MODE >= 2) {
    uint32_t seed = (uint32_t)(l * 2654435761u) ^ (uint32_t)(size_t)sa;
    for (int64_t st = 0; st < nst; ++st) {
      seed = seed * 1664525u + 1013904223u;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const v4i bv = opnd<MODE>(seed + s4);
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
          cnt[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(opnd<MODE>(seed ^ (cb * 77 + s4)), bv, cnt[cb], 0, 0, 0);
      }
    }
    return;
  }
  auto issue = [&](int64_t st) {
    uint8_t* slot = lds + (int)(st % D) * 2 * TB;
    __builtin_amdgcn_global_load_lds(sa + st * 64, (lds_ptr_t)(slot + w * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(sb + st * 64, (lds_ptr_t)(slot + TB + w * 1024), 16, 0, 0);
  };
  for (int64_t st = 0; st < D - 1 && st < nst; ++st) issue(st);
  for (int64_t st = 0; st < nst; ++st) {
    if (st + D - 2 < nst) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 2) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (st + D - 1 < nst) issue(st + D - 1);
    const uint8_t* As = lds + (int)(st % D) * 2 * TB;
    const uint8_t* Bs = As + TB;
    const uint4 bq = *reinterpret_cast<const uint4*>(Bs + i8off_b(16 * w + rho, ch));
    uint4 aq[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) aq[cb] = *reinterpret_cast<const uint4*>(As + i8off_a(16 * cb + prow, ch));
    const uint32_t bw[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const v4i bv = opnd<MODE>(bw[s4]);
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const uint32_t aw = s4 == 0 ? aq[cb].x : s4 == 1 ? aq[cb].y : s4 == 2 ? aq[cb].z : aq[cb].w;
        cnt[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(opnd<MODE>(aw), bv, cnt[cb], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int MODE>
__global__ __launch_bounds__(512, 2) void bench_grm(const uint8_t* gpk, int64_t row_bytes, const int32_t* rows,
                                                    int64_t nblk, int* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * TILE * 64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t g = blockIdx.x;
  const int row = 16 * w + (l >> 2), pos = l & 3;
  const int32_t* rj = rows + (g / 4) * 128;          // 4 tiles share the J panel (same individual)
  const int32_t* ri = rows + (g + 1) * 128;
  const uint8_t* sa = gpk + (int64_t)rj[row] * row_bytes + 16 * (pos ^ ((row >> 2) & 3));
  const uint8_t* sb = gpk + (int64_t)ri[row] * row_bytes + 16 * (pos ^ ((row >> 2) & 2));
  v4i cnt[8];
  if constexpr (MODE == 0) {
    i8_tt8_pk64<4>(sa, sb, nblk, lds, cnt);
  } else {
    tile_loop<4, MODE>(sa, sb, nblk, lds, cnt);
  }
  int s = 0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) s += cnt[cb][0] + cnt[cb][1] + cnt[cb][2] + cnt[cb][3];
  if (s == 123456789) out[g] = s;
}

int main(int argc, char** argv) {
  const int64_t nblk = argc > 1 ? atoi(argv[1]) : 20;
  const int nwg = argc > 2 ? atoi(argv[2]) : 2048;
  const int64_t P = 50000, row_bytes = 16 * (nblk + 4);
  uint8_t* gpk;
  int32_t* rows;
  int* out;
  hipMalloc(&gpk, (size_t)P * row_bytes);
  hipMalloc(&rows, (size_t)(nwg + 2) * 128 * 4);
  hipMalloc(&out, (size_t)nwg * 4);
  std::vector<uint8_t> h((size_t)P * row_bytes);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 13);
  hipMemcpy(gpk, h.data(), h.size(), hipMemcpyHostToDevice);
  std::vector<int32_t> hr((size_t)(nwg + 2) * 128);
  uint64_t st = 88172645463325252ull;
  for (auto& r : hr) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    r = (int32_t)(st % P);
  }
  hipMemcpy(rows, hr.data(), hr.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double ops = (double)nwg * 2.0 * 128 * 128 * 64 * (double)(4 * ((nblk + 3) / 4));
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a, 0);
      if (mode == 0) hipLaunchKernelGGL(bench_grm<0>, dim3(nwg), dim3(512), 0, 0, gpk, row_bytes, rows, nblk, out);
      if (mode == 1) hipLaunchKernelGGL(bench_grm<1>, dim3(nwg), dim3(512), 0, 0, gpk, row_bytes, rows, nblk, out);
      if (mode == 2) hipLaunchKernelGGL(bench_grm<2>, dim3(nwg), dim3(512), 0, 0, gpk, row_bytes, rows, nblk, out);
      if (mode == 3) hipLaunchKernelGGL(bench_grm<3>, dim3(nwg), dim3(512), 0, 0, gpk, row_bytes, rows, nblk, out);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("mode %d  nblk=%ld nwg=%d  %.1f us  %.1f int8 TOPS  %.2f us/tile-round\n", mode, (long)nblk, nwg,
           best * 1e3, ops / (best * 1e-3) / 1e12, best * 1e3 / ((nwg + 511) / 512));
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
