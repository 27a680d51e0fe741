// FP4 (e2m1) MFMA probe for exact genotype products: genotype g in {0,1,2} is the e2m1 nibble
// 2g (0, 1.0, 2.0), products and fp32 sums of counts below 2^24 are exact.  Checks
// v_mfma_scale_f32_16x16x128_f8f6f4 (A, B fp4; E8M0 scales 1.0) against integer A B^T with A and
// B given in one layout (lane l: row / column l & 15, 16 bytes = 32 nibbles of k-chunk l >> 4),
// reads back the C layout, and times it beside i8 16x16x64.
//   hipcc --offload-arch=gfx950 -O3 tools/fp4_probe.hip -o tools/fp4_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_check(const uint8_t* A, const uint8_t* B, float* C) {   // A, B: [16][64] bytes
  const int l = threadIdx.x;
  const uint4 a = *reinterpret_cast<const uint4*>(A + (l & 15) * 64 + 16 * (l >> 4));
  const uint4 b = *reinterpret_cast<const uint4*>(B + (l & 15) * 64 + 16 * (l >> 4));
  v8i av = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, 0, 0, 0, 0};
  v8i bv = {(int)b.x, (int)b.y, (int)b.z, (int)b.w, 0, 0, 0, 0};
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 4, 4, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) C[l * 4 + r] = c[r];
}

constexpr int ITER = 4096;
__global__ __launch_bounds__(256) void k_fp4(const int* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  v8i a = {in[l & 63], in[(l + 1) & 63], in[(l + 2) & 63], in[(l + 3) & 63], 0, 0, 0, 0};
  v8i b = {in[64 + (l & 63)], in[64 + ((l + 5) & 63)], in[64 + ((l + 6) & 63)], in[64 + ((l + 7) & 63)], 0, 0, 0, 0};
  v4f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0, 0, 0, (float)i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[i], 4, 4, 0, 127, 0, 127);
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
__global__ __launch_bounds__(256) void k_i8(const int* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  v4i a = {in[l & 63], in[(l + 1) & 63], in[(l + 2) & 63], in[(l + 3) & 63]};
  v4i b = {in[64 + (l & 63)], in[64 + ((l + 5) & 63)], in[64 + ((l + 6) & 63)], in[64 + ((l + 7) & 63)]};
  v4i acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v4i{0, 0, 0, i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_readcyclecounter();
  int s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = (float)s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <class K>
static void timeit(const char* name, K kern, int* din, float* dout, long long* dcyc, int nblk, double ops) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), 0, 0, din, dout, dcyc);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), 0, 0, din, dout, dcyc);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("\"%s\": {\"tops\": %.1f, \"ms\": %.4f}, ", name, (double)nblk * 4 * ITER * 8 * ops / (best * 1e-3) / 1e12, best);
}

int main() {
  // genotypes g[16][128] for A and B; fp4 nibble 2g, k = 2 * byte + (nibble high)
  std::vector<int> ga(16 * 128), gb(16 * 128);
  std::vector<uint8_t> A(16 * 64), B(16 * 64);
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) { ga[i] = rand() % 3; gb[i] = rand() % 3; }
  for (int r = 0; r < 16; ++r)
    for (int m = 0; m < 64; ++m) {
      A[r * 64 + m] = (uint8_t)((2 * ga[r * 128 + 2 * m]) | ((2 * ga[r * 128 + 2 * m + 1]) << 4));
      B[r * 64 + m] = (uint8_t)((2 * gb[r * 128 + 2 * m]) | ((2 * gb[r * 128 + 2 * m + 1]) << 4));
    }
  uint8_t *dA, *dB; float* dC;
  CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dC, 256 * 4));
  CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  std::vector<float> C(256);
  CK(hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost));
  // which (row, col) does lane l, element r hold?  try row = 4 (l >> 4) + r, col = l & 15
  int bad_a = 0, bad_b = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      long ref_a = 0, ref_b = 0;
      const int ra = 4 * (l >> 4) + r, ca = l & 15;       // candidate layout a
      const int rb = (l >> 4) + 4 * r, cb = l & 15;       // candidate layout b
      for (int k = 0; k < 128; ++k) { ref_a += ga[ra * 128 + k] * gb[ca * 128 + k]; ref_b += gb[cb * 128 + k] * ga[rb * 128 + k]; }
      if ((float)ref_a != C[l * 4 + r]) ++bad_a;
      if ((float)ref_b != C[l * 4 + r]) ++bad_b;
    }
  printf("{\"layout_row_4g_plus_r_mismatches\": %d, \"layout_row_g_plus_4r_mismatches\": %d, \"c00\": %.1f, ", bad_a, bad_b, C[0]);
  int* di; float* dout; long long* dcyc;
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int nblk = p.multiProcessorCount * 4;
  CK(hipMalloc(&di, 1024)); CK(hipMalloc(&dout, (size_t)nblk * 256 * 4)); CK(hipMalloc(&dcyc, 8));
  std::vector<int> hi(256); for (auto& x : hi) x = rand() & 0x44444444;
  CK(hipMemcpy(di, hi.data(), 1024, hipMemcpyHostToDevice));
  timeit("i8_16x16x64", k_i8, di, dout, dcyc, nblk, 2.0 * 16 * 16 * 64);
  timeit("fp4_16x16x128", k_fp4, di, dout, dcyc, nblk, 2.0 * 16 * 16 * 128);
  printf("\"ok\": 1}\n");
  return 0;
}
