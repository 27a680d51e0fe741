// Differential-evolution generation step on the GPU: mutation + binary crossover
// (+ clip) for every individual of a population, bit-exact to the reference's
// numpy arithmetic and RNG streams.
//
//   DE/rand/1            tblup/evolver.py:103-138   mutant = a + F (b - c)
//   DE/current-to-best/1 tblup/evolver.py:179-221   mutant = x + F (best - x) + F (a - b)
//   binary crossover     tblup/evolver.py:63-82     np.random.rand(L) < cr, forced position `fixed`
//   clip                 np.clip(genome, 0, dimensionality - 1)
//
// One workgroup per individual.  Individual i's uniforms are numpy's legacy
// RandomState doubles (two MT19937 outputs each) at stream offset pos0 + 2Li; the
// workgroup regenerates the sequence that follows the generation's base state in
// LDS, jumps to its own offset by the GF(2) correlation W'[j] = XOR_k p_k x[k+j]
// with its jump polynomial (mt_jump.cpp), and then runs the MT19937 recurrence
// forward in a two-block LDS ring, 312 doubles per 624-word block.  Workgroup `pop`
// produces numpy's (key, pos) after the whole generation's draws.
#include "mt_jump.h"
#include "tblup_internal.h"

namespace tblup {
namespace {

constexpr int MTN = 624;
constexpr int DE_THREADS = 640;                       // one thread per window word in the correlation
constexpr int SEQ_WORDS = MTN + tblup_mt::MT_DEG + MTN - 1;   // base sequence read up to pos0 (<= 624) + 19937 + 623

__device__ __forceinline__ uint32_t mt_twist(uint32_t xt, uint32_t xt1, uint32_t xtm) {
  const uint32_t y = (xt & 0x80000000u) | (xt1 & 0x7fffffffu);
  return xtm ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// next 624 words of the ring (block b into slot b&1 from block b-1 in the other slot):
// three dependency steps of 227 / 227 / 170 words
__device__ __forceinline__ void mt_block(uint32_t* ring, int b, int tid) {
  uint32_t* cur = ring + (b & 1) * MTN;
  const uint32_t* prv = ring + ((b + 1) & 1) * MTN;
  if (tid < 227) cur[tid] = mt_twist(prv[tid], prv[tid + 1], prv[tid + 397]);
  __syncthreads();
  if (tid < 227) {
    const int w = tid + 227;
    cur[w] = mt_twist(prv[w], prv[w + 1], cur[w - 227]);
  }
  __syncthreads();
  if (tid < 170) {
    const int w = tid + 454;
    cur[w] = mt_twist(prv[w], w == MTN - 1 ? cur[0] : prv[w + 1], cur[w - 227]);
  }
  __syncthreads();
}

struct DeArgs {
  const uint32_t* key;     // numpy key[624] at the generation's first draw
  int pos0;                // numpy pos (0..624)
  const uint32_t* polys;   // [pop][624]: row i-1 -> individual i >= 1; row pop-1 -> end state
  int end_jump;            // end window by polys[pop-1] (else the base key itself)
  int end_s, end_pos;      // numpy key = end ring words [end_s, end_s + 624), pos = end_pos
  const double* parent;    // [pop][ldp]
  int64_t ldp;
  const int32_t* donors;   // [pop][3]
  const int64_t* fixed;    // [pop]
  int strategy;            // 0 rand/1, 1 current-to-best/1
  double F, cr;
  int clip;
  double hi;               // clip upper bound (dimensionality - 1)
  int64_t L;               // genome length
  int pop;
  double* child;           // [pop][ldc]
  int64_t ldc;
  uint32_t* key_out;       // [624]
  int32_t* pos_out;
};

__global__ __launch_bounds__(DE_THREADS) void k_de_step(DeArgs a) {
#pragma clang fp contract(off)
  __shared__ uint32_t seq[SEQ_WORDS];
  __shared__ uint32_t ring[2 * MTN];
  const int tid = threadIdx.x;
  const int i = blockIdx.x;
  const bool is_end = i == a.pop;
  const bool jump = is_end ? a.end_jump != 0 : i > 0;

  // 1. the sequence that continues the base window, as far as this workgroup reads it
  for (int t = tid; t < MTN; t += DE_THREADS) seq[t] = a.key[t];
  const int need = jump ? a.pos0 + tblup_mt::MT_DEG + MTN - 1 : (i == 0 ? a.pos0 + MTN : MTN);
  for (int t0 = MTN; t0 < need; t0 += 227) {
    __syncthreads();
    const int t = t0 + tid;
    if (tid < 227 && t < need) seq[t] = mt_twist(seq[t - 624], seq[t - 623], seq[t - 227]);
  }
  __syncthreads();

  // 2. this workgroup's start window: W[j] = XOR_{k: p_k} seq[pos0 + k + j]
  uint32_t w = 0;
  if (tid < MTN) {
    if (jump) {
      const uint32_t* poly = a.polys + (int64_t)(is_end ? a.pop - 1 : i - 1) * MTN;
      const uint32_t* s = seq + a.pos0 + tid;
      uint32_t acc0 = 0, acc1 = 0;
      for (int pw = 0; pw < MTN; ++pw) {
        uint32_t cw = poly[pw];   // uniform: scalar load
        const uint32_t* sp = s + 32 * pw;
        while (cw) {
          const int b0 = __builtin_ctz(cw);
          cw &= cw - 1;
          const uint32_t m1 = cw ? ~0u : 0u;
          const int b1 = cw ? __builtin_ctz(cw) : 0;
          cw &= cw - 1;
          const uint32_t m2 = cw ? ~0u : 0u;
          const int b2 = cw ? __builtin_ctz(cw) : 0;
          cw &= cw - 1;
          const uint32_t m3 = cw ? ~0u : 0u;
          const int b3 = cw ? __builtin_ctz(cw) : 0;
          cw &= cw - 1;
          acc0 ^= sp[b0] ^ (sp[b1] & m1);
          acc1 ^= (sp[b2] & m2) ^ (sp[b3] & m3);
        }
      }
      w = acc0 ^ acc1;
    } else {
      w = seq[(i == 0 ? a.pos0 : 0) + tid];
    }
  }
  if (tid < MTN) ring[tid] = w;   // block 0 in slot 0
  __syncthreads();

  if (is_end) {
    mt_block(ring, 1, tid);
    if (tid < MTN) a.key_out[tid] = ring[a.end_s + tid];
    if (tid == 0) *a.pos_out = a.end_pos;
    return;
  }

  // 3. stream: words [f, f + 2L) of the sequence from this window, one double per word pair
  const int f = i == 0 ? 0 : 2;
  const int64_t L = a.L;
  const double* P = a.parent + (int64_t)i * a.ldp;
  double* C = a.child + (int64_t)i * a.ldc;
  const int d0 = a.donors[3 * i], d1 = a.donors[3 * i + 1], d2 = a.donors[3 * i + 2];
  const double* X0 = a.parent + (int64_t)d0 * a.ldp;
  const double* X1 = a.parent + (int64_t)d1 * a.ldp;
  const double* X2 = a.parent + (int64_t)d2 * a.ldp;
  const int64_t fixed = a.fixed[i];
  const int64_t nblocks = (f + 2 * L + MTN - 1) / MTN;
  for (int64_t b = 0; b < nblocks; ++b) {
    if (b > 0) mt_block(ring, (int)(b & 1), tid);
    const uint32_t* blk = ring + (b & 1) * MTN;
    const int q = tid;
    if (q < MTN / 2 && !(b == 0 && q < f / 2)) {
      const int64_t j = (MTN / 2) * b + q - f / 2;
      if (j < L) {
        const uint32_t hi = mt_temper(blk[2 * q]) >> 5, lo = mt_temper(blk[2 * q + 1]) >> 6;
        const double u = ((double)hi * 67108864.0 + (double)lo) / 9007199254740992.0;
        double v = P[j];
        if (u < a.cr || j == fixed) {
          if (a.strategy == 0) {
            v = X0[j] + a.F * (X1[j] - X2[j]);
          } else {
            const double x = v;
            v = (x + a.F * (X0[j] - x)) + a.F * (X1[j] - X2[j]);
          }
        }
        if (a.clip) {   // numpy's _NPY_CLIP: MIN(MAX(v, 0), hi) with a > b ? a : b, NaN passes through
          v = (v != v || v > 0.0) ? v : 0.0;
          v = (v != v || v < a.hi) ? v : a.hi;
        }
        C[j] = v;
      }
    }
  }
}

}  // namespace

hipError_t launch_de_step(const uint32_t* key, int pos0, const uint32_t* polys, int end_jump, int end_s, int end_pos,
                          const double* parent, int64_t ldp, const int32_t* donors, const int64_t* fixed, int strategy,
                          double F, double cr, int clip, double hi, int64_t L, int pop, double* child, int64_t ldc,
                          uint32_t* key_out, int32_t* pos_out, hipStream_t s) {
  DeArgs a{key, pos0, polys, end_jump, end_s, end_pos, parent, ldp, donors, fixed, strategy, F, cr, clip, hi, L, pop,
           child, ldc, key_out, pos_out};
  hipLaunchKernelGGL(k_de_step, dim3(pop + 1), dim3(DE_THREADS), 0, s, a);
  return hipGetLastError();
}

}  // namespace tblup
