// Microbenchmark of k_sys_tiles' structure (FP4 MFMA system tiles from 2-bit packed rows) in
// isolation: the ring depth D, the bytes per row per stage (SUB x 64 B) and the workgroups per
// CU that the LDS ring leaves, with loads + MFMA, loads only, or MFMA only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tblup_amd/csrc tools/sys_bench.hip -o tools/sys_bench
//   tools/sys_bench [B=256]
// Rows are gathered from a 50k x 512 B table by a random index list per individual (the split
// matrix's shape at config 2: n_T = 1280 -> 320 B per row, 5 x 64 B); 36 tiles per individual.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {   // as tblup_internal.h
  if (nwg <= 8) return orig;
  int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  int64_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}
typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int TILE_ = 128, NSUB = 5, ROWB = 512;

__device__ __forceinline__ v8i fp4_op(uint32_t x0, uint32_t x1) {
  constexpr uint32_t M = 0x66666666u;
  return v8i{(int)((x0 << 1) & M), (int)((x0 >> 1) & M), (int)((x1 << 1) & M), (int)((x1 >> 1) & M), 0, 0, 0, 0};
}

__device__ __forceinline__ v4f mfma_fp4(v8i a, v8i b, v4f c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}
__device__ __forceinline__ void lds_load16(const uint8_t* src, uint8_t* dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)dst, 16, 0, 0);
}

// LDS image of one stage: per operand 128 rows x (SUB x 64 B), row-major, 16-B chunks swizzled
template <int SUB>
__device__ __forceinline__ int off(int row, int c) { return row * 64 * SUB + 16 * (c ^ ((row >> 2) & (4 * SUB - 1))); }

template <int D, int SUB, int MODE, bool RT = false, int WPE = 2>
__global__ __launch_bounds__(256, WPE) void k_bench(const uint8_t* __restrict__ tab, const int32_t* __restrict__ idx,
                                                  int ntri, int* out, int16_t* kc, int nsub_rt = NSUB) {
  constexpr int TB = TILE_ * 64 * SUB;
  __shared__ __attribute__((aligned(16))) uint8_t lds[D * 2 * TB];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, qr = w >> 1, qc = w & 1;
  const int64_t lg = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = lg / ntri;
  const int t = (int)(lg % ntri);
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  const int J = t - I * (I + 1) / 2;
  constexpr int LPR = 4 * SUB;            // lanes per row per instruction
  constexpr int RPI = 64 / LPR;           // rows per instruction
  constexpr int NI = TILE_ / RPI / 4;     // instructions per wave per operand
  const uint8_t* sa[NI];
  const uint8_t* sb[NI];
#pragma unroll
  for (int h = 0; h < NI; ++h) {
    const int row = RPI * (NI * w + h) + l / LPR, pos = l % LPR;
    sa[h] = tab + (int64_t)idx[b * 1024 + J * TILE_ + row] * ROWB + 16 * (pos ^ ((row >> 2) & (LPR - 1)));
    sb[h] = tab + (int64_t)idx[b * 1024 + I * TILE_ + row] * ROWB + 16 * (pos ^ ((row >> 2) & (LPR - 1)));
  }
  const int nst = RT ? (nsub_rt + SUB - 1) / SUB : (NSUB + SUB - 1) / SUB;
#define ISSUE(st_)                                                                                               \
  {                                                                                                              \
    uint8_t* slot = lds + ((st_) % D) * 2 * TB;                                                                  \
    _Pragma("unroll") for (int h = 0; h < NI; ++h) {                                                             \
      lds_load16(sa[h] + (st_) * 64 * SUB, slot + (NI * w + h) * 1024); \
      lds_load16(sb[h] + (st_) * 64 * SUB, slot + TB + (NI * w + h) * 1024); \
    }                                                                                                            \
  }
  v4f cnt[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) cnt[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  if (MODE != 2)
    for (int st = 0; st < D - 1 && st < nst; ++st) ISSUE(st);
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  for (int st = 0; st < nst; ++st) {
    if (MODE != 2) {
      if (st + D - 2 < nst) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 2 * NI) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (st + D - 1 < nst) ISSUE(st + D - 1);
    }
    if (MODE != 1) {
      const uint8_t* As = lds + (st % D) * 2 * TB;
      const uint8_t* Bs = As + TB;
#pragma unroll
      for (int sub = 0; sub < SUB; ++sub) {
        if (st * SUB + sub >= NSUB) break;
        uint4 aq[4], bq[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          aq[m] = *reinterpret_cast<const uint4*>(As + off<SUB>(16 * (4 * qr + m) + prow, 4 * sub + ch));
          bq[m] = *reinterpret_cast<const uint4*>(Bs + off<SUB>(16 * (4 * qc + m) + rho, 4 * sub + ch));
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          v8i av[4], bv[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            av[m] = s2 == 0 ? fp4_op(aq[m].x, aq[m].y) : fp4_op(aq[m].z, aq[m].w);
            bv[m] = s2 == 0 ? fp4_op(bq[m].x, bq[m].y) : fp4_op(bq[m].z, bq[m].w);
          }
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
              cnt[m][n] = mfma_fp4(av[m], bv[n], cnt[m][n]);
        }
      }
    }
  }
  if (MODE == 0 || MODE == 2) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) s += cnt[m][n][0] + cnt[m][n][3];
    if (s == -1.f) out[blockIdx.x] = (int)s;   // keeps the work; never true
  } else if (MODE == 3 || MODE == 4) {   // the production epilogue: every tile's int16 counts (32 KiB)
    int16_t* kt = kc + lg * (128 * 128);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int cb = 4 * qr + m, ib = 4 * qc + n;
        const v4f c = cnt[m][n];
        const int2 packed = {(int)((uint32_t)((int)c[0] & 0xffff) | ((uint32_t)(int)c[1] << 16)),
                             (int)((uint32_t)((int)c[2] & 0xffff) | ((uint32_t)(int)c[3] << 16))};
        if (MODE == 3)
          *reinterpret_cast<int2*>(kt + ((ib * 8 + cb) * 64 + l) * 4) = packed;
        else
          { typedef int v2i_ __attribute__((ext_vector_type(2))); __builtin_nontemporal_store(v2i_{packed.x, packed.y}, reinterpret_cast<v2i_*>(kt + ((ib * 8 + cb) * 64 + l) * 4)); }
      }
  }
}

template <int D, int SUB, int MODE, bool RT = false, int WPE = 2>
void run(const char* name, const uint8_t* tab, const int32_t* idx, int B, int* out, int16_t* kc) {
  const int ntri = 36;
  dim3 g(B * ntri), blk(256);
  for (int i = 0; i < 3; ++i) k_bench<D, SUB, MODE, RT, WPE><<<g, blk>>>(tab, idx, ntri, out, kc, NSUB);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R = 20;
  hipEventRecord(e0);
  for (int i = 0; i < R; ++i) k_bench<D, SUB, MODE, RT, WPE><<<g, blk>>>(tab, idx, ntri, out, kc, NSUB);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / R;
  printf("{\"variant\": \"%s\", \"D\": %d, \"stage_B_per_row\": %d, \"mode\": %d, \"lds_KiB\": %d, \"us\": %.1f}\n", name, D,
         64 * SUB, MODE, D * 2 * TILE_ * 64 * SUB / 1024, us);
}

// Persistent variant: a fixed grid (NPW workgroups per CU) walks its tiles with ONE LDS ring
// across tile boundaries -- stage g of the walk is stage g % 5 of tile g / 5 -- so the ring's
// fill latency is paid once per workgroup instead of once per tile, and a tile's stores overlap
// the next tile's loads.  Tiles of an XCD's individuals stay on that XCD.
template <int D, int STORE>
__global__ __launch_bounds__(256, 2) void k_persist(const uint8_t* __restrict__ tab, const int32_t* __restrict__ idx,
                                                    int ntri, int64_t ntiles, int* out, int16_t* kc) {
  constexpr int TB = TILE_ * 64;
  constexpr int NST = NSUB;
  __shared__ __attribute__((aligned(16))) uint8_t lds[D * 2 * TB];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, qr = w >> 1, qc = w & 1;
  const int64_t xcd = blockIdx.x % 8, slotx = blockIdx.x / 8, nper = gridDim.x / 8;
  const int64_t t0 = xcd * ntiles / 8, t1 = (xcd + 1) * ntiles / 8;   // this XCD's tiles
  // tile k of this workgroup: t0 + slotx + k * nper
  auto tile_of = [&](int64_t k) { return t0 + slotx + k * nper; };
  int64_t ntile_me = 0;
  if (t0 + slotx < t1) ntile_me = (t1 - 1 - (t0 + slotx)) / nper + 1;
  const int64_t nstage = ntile_me * NST;
  const int row0 = 16 * (2 * w) + (l >> 2), pos = l & 3;
  auto ptrs = [&](int64_t lg, const uint8_t* (&pa)[2], const uint8_t* (&pb)[2]) {
    const int64_t b = lg / ntri;
    const int t = (int)(lg % ntri);
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = row0 + 16 * h;
      pa[h] = tab + (int64_t)idx[b * 1024 + J * TILE_ + row] * ROWB + 16 * (pos ^ ((row >> 2) & 3));
      pb[h] = tab + (int64_t)idx[b * 1024 + I * TILE_ + row] * ROWB + 16 * (pos ^ ((row >> 2) & 3));
    }
  };
  const uint8_t* ia[2];
  const uint8_t* ib[2];
  int64_t itile = 0;   // tile the issue pointers belong to
  if (ntile_me > 0) ptrs(tile_of(0), ia, ib);
  auto issue = [&](int64_t g) {
    const int64_t k = g / NST;
    const int st = (int)(g % NST);
    if (k != itile) {
      itile = k;
      ptrs(tile_of(k), ia, ib);
    }
    uint8_t* slot = lds + (int)(g % D) * 2 * TB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      lds_load16(ia[h] + st * 64, slot + (2 * w + h) * 1024);
      lds_load16(ib[h] + st * 64, slot + TB + (2 * w + h) * 1024);
    }
  };
  for (int64_t g = 0; g < D - 1 && g < nstage; ++g) issue(g);
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  v4f cnt[4][4];
  for (int64_t g = 0; g < nstage; ++g) {
    const int st = (int)(g % NST);
    if (st == 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) cnt[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
    }
    if (g + D - 2 < nstage) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (g + D - 1 < nstage) issue(g + D - 1);
    const uint8_t* As = lds + (int)(g % D) * 2 * TB;
    const uint8_t* Bs = As + TB;
    uint4 aq[4], bq[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      aq[m] = *reinterpret_cast<const uint4*>(As + off<1>(16 * (4 * qr + m) + prow, ch));
      bq[m] = *reinterpret_cast<const uint4*>(Bs + off<1>(16 * (4 * qc + m) + rho, ch));
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      v8i av[4], bv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        av[m] = s2 == 0 ? fp4_op(aq[m].x, aq[m].y) : fp4_op(aq[m].z, aq[m].w);
        bv[m] = s2 == 0 ? fp4_op(bq[m].x, bq[m].y) : fp4_op(bq[m].z, bq[m].w);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) cnt[m][n] = mfma_fp4(av[m], bv[n], cnt[m][n]);
    }
    if (st == NST - 1) {
      const int64_t lg = tile_of(g / NST);
      if (STORE) {
        int16_t* kt = kc + lg * (128 * 128);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) {
            const int cb = 4 * qr + m, ib_ = 4 * qc + n;
            const v4f c = cnt[m][n];
            const int2 packed = {(int)((uint32_t)((int)c[0] & 0xffff) | ((uint32_t)(int)c[1] << 16)),
                                 (int)((uint32_t)((int)c[2] & 0xffff) | ((uint32_t)(int)c[3] << 16))};
            *reinterpret_cast<int2*>(kt + ((ib_ * 8 + cb) * 64 + l) * 4) = packed;
          }
      } else {
        float sacc = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) sacc += cnt[m][n][0] + cnt[m][n][3];
        if (sacc == -1.f) out[lg] = 1;
      }
    }
  }
}

template <int D, int STORE>
void run_persist(const char* name, int npc, const uint8_t* tab, const int32_t* idx, int B, int* out, int16_t* kc) {
  const int ntri = 36;
  const int64_t ntiles = (int64_t)B * ntri;
  dim3 g(256 * npc), blk(256);
  for (int i = 0; i < 3; ++i) k_persist<D, STORE><<<g, blk>>>(tab, idx, ntri, ntiles, out, kc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R = 20;
  hipEventRecord(e0);
  for (int i = 0; i < R; ++i) k_persist<D, STORE><<<g, blk>>>(tab, idx, ntri, ntiles, out, kc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("{\"variant\": \"%s\", \"D\": %d, \"wg_per_cu\": %d, \"store\": %d, \"us\": %.1f}\n", name, D, npc, STORE, ms * 1e3 / R);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int P = 50000;
  std::vector<uint8_t> h_tab((size_t)P * ROWB);
  std::mt19937 rng(1);
  for (auto& x : h_tab) x = (uint8_t)(rng() & 0x55);   // genotypes 0/1 in every 2-bit field
  std::vector<int32_t> h_idx((size_t)B * 1024);
  for (int b = 0; b < B; ++b)
    for (int r = 0; r < 1024; ++r) h_idx[(size_t)b * 1024 + r] = (int32_t)(rng() % P);
  uint8_t* tab;
  int32_t* idx;
  int* out;
  hipMalloc(&tab, h_tab.size());
  hipMalloc(&idx, h_idx.size() * 4);
  hipMalloc(&out, (size_t)B * 64 * 4);
  hipMemcpy(tab, h_tab.data(), h_tab.size(), hipMemcpyHostToDevice);
  hipMemcpy(idx, h_idx.data(), h_idx.size() * 4, hipMemcpyHostToDevice);
  int16_t* kc;
  hipMalloc(&kc, (size_t)B * 36 * 128 * 128 * 2);
  run<2, 1, 3, true, 4>("D2 stores, <=128 VGPRs (4 WG/CU)", tab, idx, B, out, kc);
  run<3, 1, 3, true, 3>("D3 stores, <=168 VGPRs", tab, idx, B, out, kc);
  run<2, 1, 0, true, 4>("D2 no stores, <=128 VGPRs", tab, idx, B, out, kc);
  run<3, 1, 0, true, 2>("D3 no stores (ref)", tab, idx, B, out, kc);
  run_persist<3, 0>("persistent", 3, tab, idx, B, out, kc);
  run_persist<3, 1>("persistent + int16 stores", 3, tab, idx, B, out, kc);
  run_persist<4, 1>("persistent D4 + stores", 2, tab, idx, B, out, kc);
  run_persist<3, 1>("persistent + stores, 2 per CU", 2, tab, idx, B, out, kc);
  run_persist<2, 1>("persistent D2 + stores, 4 per CU", 4, tab, idx, B, out, kc);
  run<3, 1, 0>("no stores", tab, idx, B, out, kc);
  run<3, 1, 0, true>("no stores, runtime stage count", tab, idx, B, out, kc);
  run<3, 1, 3, true>("int16 stores, runtime stage count", tab, idx, B, out, kc);
  run<3, 1, 3>("int16 stores (prod)", tab, idx, B, out, kc);
  run<3, 1, 4>("int16 nontemporal stores", tab, idx, B, out, kc);
  run<3, 1, 1>("loads only", tab, idx, B, out, kc);
  run<3, 1, 2>("mfma only", tab, idx, B, out, kc);
  run<2, 1, 3>("D2 stores", tab, idx, B, out, kc);
  run<3, 1, 3>("int16 stores again", tab, idx, B, out, kc);
  run<3, 1, 0>("no stores again", tab, idx, B, out, kc);
  return 0;
}
