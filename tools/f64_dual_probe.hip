// Does gfx950 run fp64 VALU FMAs beside fp64 MFMAs on the same SIMD?  (The spec sheet gives
// MI355X the same fp64 rate for vector and matrix, 78.6 TFLOP/s.)  One 512-thread workgroup per
// slot, two per CU: waves 0-3 issue v_mfma_f64_16x16x4 on 8 independent accumulators, waves 4-7
// issue v_fma_f64 on 16 independent accumulators (so every SIMD holds one wave of each kind per
// workgroup).  Modes: 0 both, 1 MFMA waves only, 2 VALU waves only.  If the two pipes are
// separate, mode 0 takes max(mode 1, mode 2), not the sum.  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 tools/f64_dual_probe.hip -o tools/f64_dual_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v4d __attribute__((ext_vector_type(4)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int ITER_M = 1024;   // MFMA loop: 8 MFMAs per iteration
constexpr int NV = 16;         // VALU accumulators per lane

__global__ __launch_bounds__(512) void k_dual(const double* in, double* out, int mode, int iter_v) {
  const int l = threadIdx.x, w = l >> 6;
  double s = 0.0;
  if (w < 4) {
    if (mode == 2) return;
    double a = in[l & 63], b = in[64 + (l & 63)];
    v4d acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v4d{0, 0, 0, (double)i};
    for (int it = 0; it < ITER_M; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    if (mode == 1) return;
    double x[NV];
    const double b = in[64 + (l & 63)];
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = in[(l + i) & 63];
    for (int it = 0; it < iter_v; ++it) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = __builtin_fma(x[i], b, 1e-3);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) s += x[i];
  }
  out[blockIdx.x * 512 + l] = s;
}

static float time_mode(double* din, double* dout, int nblk, int mode, int iter_v) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_dual, dim3(nblk), dim3(512), 0, 0, din, dout, mode, iter_v);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_dual, dim3(nblk), dim3(512), 0, 0, din, dout, mode, iter_v);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int nblk = cus * 2;
  double* dd;
  CK(hipMalloc(&dd, (size_t)nblk * 512 * 8 + 1024));
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + (double)rand() / RAND_MAX;
  CK(hipMemcpy(dd, h, sizeof h, hipMemcpyHostToDevice));
  double* dout = dd + 128;
  const double mflop = (double)nblk * 4 * ITER_M * 8 * 2048.0;   // MFMA waves
  printf("{\"cus\": %d, \"rows\": [", cus);
  const int ivs[] = {1024, 2048, 4096, 8192};
  for (int k = 0; k < 4; ++k) {
    const int iv = ivs[k];
    const double vflop = (double)nblk * 4 * 64 * iv * NV * 2.0;   // VALU waves
    const float tb = time_mode(dd, dout, nblk, 0, iv);
    const float tm = time_mode(dd, dout, nblk, 1, iv);
    const float tv = time_mode(dd, dout, nblk, 2, iv);
    printf("%s{\"iter_v\": %d, \"ms_both\": %.4f, \"ms_mfma\": %.4f, \"ms_valu\": %.4f, \"tf_mfma_alone\": %.2f, "
           "\"tf_valu_alone\": %.2f, \"tf_both\": %.2f}",
           k ? ", " : "", iv, tb, tm, tv, mflop / (tm * 1e-3) / 1e12, vflop / (tv * 1e-3) / 1e12,
           (mflop + vflop) / (tb * 1e-3) / 1e12);
  }
  printf("]}\n");
  return 0;
}
