// Measured MFMA peaks on the box (the microarchitecture guide has no fp64 MFMA row):
// every wave issues back-to-back MFMAs on 8 independent accumulators over random operands
// for ITER iterations; grids of 1, 2, 4 and 8 workgroups of 4 waves per CU.  Prints one
// JSON line with TFLOP/s (TOP/s for int8) per instruction, the per-wave cycles per MFMA
// and (cycle counter / wall time) the clock the chip held when all blocks ran in one round.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int ITER = 4096;

__global__ __launch_bounds__(256) void k_f64(const double* in, double* out, long long* cyc) {
  const int l = threadIdx.x;
  double a = in[l & 63], b = in[64 + (l & 63)];
  v4d acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4d{0, 0, 0, (double)i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_readcyclecounter();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

__global__ __launch_bounds__(256) void k_f32(const float* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  float a = in[l & 63], b = in[64 + (l & 63)];
  v4f acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0, 0, 0, (float)i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

__global__ __launch_bounds__(256) void k_i8(const int* in, int* out, long long* cyc) {
  const int l = threadIdx.x;
  v4i a = {in[l & 63], in[(l + 1) & 63], in[(l + 2) & 63], in[(l + 3) & 63]};
  v4i b = {in[64 + (l & 63)], in[64 + ((l + 5) & 63)], in[64 + ((l + 6) & 63)], in[64 + ((l + 7) & 63)]};
  v4i acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4i{0, 0, 0, i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_readcyclecounter();
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

__global__ __launch_bounds__(256) void k_bf16(const float* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  v8bf a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)in[(l + j) & 63];
    b[j] = (__bf16)in[64 + ((l + 3 * j) & 63)];
  }
  v4f acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0, 0, 0, (float)i};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <typename K, typename T>
static void run(const char* name, K kern, T* din, T* dout, long long* dcyc, int nblk, double flop_per_mfma,
                bool last, int wpb = 4) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(64 * wpb), 0, 0, din, dout, dcyc);   // warm-up
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  long long cyc = 0;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(nblk), dim3(64 * wpb), 0, 0, din, dout, dcyc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) {
      best = ms;
      CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    }
  }
  const double waves = (double)nblk * wpb;
  const double flops = waves * ITER * 8 * flop_per_mfma;
  // cycles per MFMA issue slot on one SIMD: 4 waves share a SIMD when 4 WGs of 4 waves sit on a CU
  const double cyc_per_mfma = (double)cyc / (ITER * 8.0);
  printf("\"%s\": {\"tflops\": %.2f, \"ms\": %.4f, \"wave_cycles_per_mfma\": %.2f, \"mhz_from_counter\": %.0f}%s", name,
         flops / (best * 1e-3) / 1e12, best, cyc_per_mfma, (double)cyc / (best * 1e-3) / 1e6, last ? "" : ", ");
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int nblk = cus * 4;   // 4 workgroups x 4 waves per CU = 4 waves per SIMD
  double* dd;
  long long* dcyc;
  CK(hipMalloc(&dd, (size_t)cus * 8 * 256 * 8 + 1024));
  CK(hipMalloc(&dcyc, 8));
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + (double)rand() / RAND_MAX;
  CK(hipMemcpy(dd, h, sizeof h, hipMemcpyHostToDevice));
  float hf[128];
  for (int i = 0; i < 128; ++i) hf[i] = (float)h[i];
  float* df;
  CK(hipMalloc(&df, (size_t)cus * 8 * 256 * 4 + 1024));
  CK(hipMemcpy(df, hf, sizeof hf, hipMemcpyHostToDevice));
  int hi[128];
  for (int i = 0; i < 128; ++i) hi[i] = rand();
  int* di;
  CK(hipMalloc(&di, (size_t)cus * 8 * 256 * 4 + 1024));
  CK(hipMemcpy(di, hi, sizeof hi, hipMemcpyHostToDevice));
  printf("{\"cus\": %d, \"clock_mhz_prop\": %d, ", cus, p.clockRate / 1000);
  run("f64_16x16x4", k_f64, dd, dd + 128, dcyc, nblk, 2.0 * 16 * 16 * 4, false);
  run("f32_16x16x4", k_f32, df, df + 128, dcyc, nblk, 2.0 * 16 * 16 * 4, false);
  run("bf16_16x16x32", k_bf16, df, df + 128, dcyc, nblk, 2.0 * 16 * 16 * 32, false);
  run("i8_16x16x64", k_i8, di, di + 128, dcyc, nblk, 2.0 * 16 * 16 * 64, false);
  // f64 occupancy sweep: 1, 2 and 8 waves per SIMD
  run("f64_1wave_per_simd", k_f64, dd, dd + 128, dcyc, cus, 2.0 * 16 * 16 * 4, false, 4);
  run("f64_2waves_per_simd", k_f64, dd, dd + 128, dcyc, cus * 2, 2.0 * 16 * 16 * 4, false, 4);
  run("f64_8waves_per_simd", k_f64, dd, dd + 128, dcyc, cus * 8, 2.0 * 16 * 16 * 4, true, 4);
  printf("}\n");
  return 0;
}
