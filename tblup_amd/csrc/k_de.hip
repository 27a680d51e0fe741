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
// produces numpy's (key, pos) after the whole generation's draws.  Populations larger than
// the CU count run the same steps as three launches (k_de_seq / k_de_jump / k_de_mask): the
// 85 KB sequence buffer holds the fused kernel at one workgroup per CU, while the mask
// recurrence -- a chain of barriers -- wants several workgroups per CU to hide each other's.
#include <cstdlib>

#include "mt_jump.h"
#include "tblup_internal.h"

namespace tblup {
namespace {

constexpr int MTN = 624;
constexpr int DE_THREADS = 640;                       // one thread per window word in the correlation
constexpr int SEQ_WORDS = MTN + tblup_mt::MT_DEG + MTN - 1;   // base sequence read up to pos0 (<= 624) + 19937 + 623
constexpr int SEQ_ALLOC = SEQ_WORDS + 64;                       // + alignment shift and the correlation's tail loads
static_assert((DE_THREADS / 64) * MTN <= SEQ_WORDS, "correlation partials must fit the sequence buffer");

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
  int dbg;                 // phase-ablation timing only (env TBLUP_DE_DBG, diagnostic builds; results wrong):
                           // 1 no jump correlation, 2 no mask recurrence, 4 no stream
  // per-individual strategy / F / crossover rate ([pop] each; null: the scalars above) -- SaDE
  // (evolver.py:407-547): each individual's strategy by python's random.random() < p, its own cr
  const int32_t* strat_i;
  const double* F_i;
  const double* cr_i;
};

// 1. the sequence that continues the base window, words [0, need) of sq
__device__ __forceinline__ void de_sequence(const uint32_t* key, uint32_t* sq, int need, int tid) {
  for (int t = tid; t < MTN; t += DE_THREADS) sq[t] = key[t];
  for (int t0 = MTN; t0 < need; t0 += 227) {
    __syncthreads();
    const int t = t0 + tid;
    if (tid < 227 && t < need) sq[t] = mt_twist(sq[t - 624], sq[t - 623], sq[t - 227]);
  }
  __syncthreads();
}

// acc ^= x in place: the tied operand keeps each accumulator in one register across the
// wave-uniform branches (plain ^= left the register allocator copying all R accumulators after
// every bit once the kernel's helpers were split out)
__device__ __forceinline__ void acc_xor(uint32_t& acc, uint32_t x) {
  asm("v_xor_b32 %0, %0, %1" : "+v"(acc) : "v"(x));
}

// 2. workgroup i's start window into ring slot 0: W[j] = XOR_{k: p_k} x[pos0 + k + j].  Wave g
// (of NW) takes poly words [624g/NW, 624(g+1)/NW); lane l < 63 owns outputs 10l .. 10l+9 and holds
// the 42 sequence words they read for one poly word in registers, so a set bit costs 10 register
// XORs (scalar branch on the wave-uniform poly bit); the waves' partial windows are XOR-reduced
// through LDS (seq, reused).  VALU-bound: 624 x ~10k set bits XORs per workgroup.
__device__ __forceinline__ void de_window(const DeArgs& a, uint32_t* seq, const uint32_t* sq, uint32_t* ring, int i,
                                          bool is_end, bool jump, int tid) {
  uint32_t w = 0;
  if (jump && !(a.dbg & 1)) {
    constexpr int NW = DE_THREADS / 64, R = 10, NL = (MTN + R - 1) / R;   // 63 lanes
    // the constant address space: the compiler's uniformity / no-clobber analysis does not carry
    // through the split kernels' helpers, and a vector load of the poly word (+ readfirstlane) costs
    // a vmcnt(0) wait per word -- this keeps it a scalar load
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    cu32* poly = (cu32*)(a.polys + (int64_t)(is_end ? a.pop - 1 : i - 1) * MTN);
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int pw0 = MTN * g / NW, pw1 = MTN * (g + 1) / NW;
    uint32_t acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
    if (lane < NL) {
      const uint32_t* base = sq + a.pos0 + R * lane;
      for (int pw = pw0; pw < pw1; ++pw) {
        const uint32_t cw = poly[pw];   // wave-uniform: scalar load, scalar branches below
        if (!cw) continue;
        uint32_t v[32 + R];
#pragma unroll
        for (int q = 0; q < 32 + R; ++q) v[q] = base[32 * pw + q];
#pragma unroll
        for (int b = 0; b < 32; ++b)
          if ((cw >> b) & 1u) {
#pragma unroll
            for (int r = 0; r < R; ++r) acc_xor(acc[r], v[b + r]);
          }
      }
    }
    __syncthreads();   // every wave is done reading the sequence: reuse it for the partials
    if (lane < NL) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (R * lane + r < MTN) seq[g * MTN + R * lane + r] = acc[r];
    }
    __syncthreads();
    if (tid < MTN) {
#pragma unroll
      for (int gg = 0; gg < NW; ++gg) w ^= seq[gg * MTN + tid];
    }
  } else if (tid < MTN) {
    w = sq[(i == 0 ? a.pos0 : 0) + tid];
  }
  if (tid < MTN) ring[tid] = w;   // block 0 in slot 0
  __syncthreads();
}

// the end workgroup (i = pop): numpy's (key, pos) after the generation's draws
__device__ __forceinline__ void de_end_state(const DeArgs& a, uint32_t* ring, int tid) {
  mt_block(ring, 1, tid);
  if (tid < MTN) a.key_out[tid] = ring[a.end_s + tid];
  if (tid == 0) *a.pos_out = a.end_pos;
}

// 3. crossover mask, then the elementwise mutant / crossover / clip stream, NTHR threads.  The mask
// of a segment of up to MASKW x 32 elements is built in LDS from the MT19937 words [f, f + 2L) of
// the window in ring slot 0, one double per word pair; the segment is then streamed with every
// thread (coalesced loads, many in flight) instead of 312 lanes per block.
template <int NTHR>
__device__ __forceinline__ void de_stream(const DeArgs& a, uint32_t* ring, uint32_t* mask, int maskw, int i, int tid) {
#pragma clang fp contract(off)   // numpy's separate multiply and add (the pragma is scoped: here, not the caller)
  static_assert(NTHR >= MTN / 2, "one thread per word pair of a block");
  const int f = i == 0 ? 0 : 2;
  const int64_t L = a.L;
  const int strategy = a.strat_i ? a.strat_i[i] : a.strategy;
  const double F = a.F_i ? a.F_i[i] : a.F, cr = a.cr_i ? a.cr_i[i] : a.cr;
  const double* P = a.parent + (int64_t)i * a.ldp;
  double* C = a.child + (int64_t)i * a.ldc;
  const int d0 = a.donors[3 * i], d1 = a.donors[3 * i + 1], d2 = a.donors[3 * i + 2];
  const double* X0 = a.parent + (int64_t)d0 * a.ldp;
  const double* X1 = a.parent + (int64_t)d1 * a.ldp;
  const double* X2 = a.parent + (int64_t)d2 * a.ldp;
  const int64_t fixed = a.fixed[i];
  const int64_t SEG = (int64_t)maskw * 32;
  int64_t b = 0;                             // next ring block to consume (block 0 = the window)
  for (int64_t lo = 0; lo < L; lo += SEG) {
    const int64_t hi = lo + SEG < L ? lo + SEG : L;
    __syncthreads();   // previous segment's stream has finished reading the mask
    for (int t = tid; t < maskw; t += NTHR) mask[t] = 0u;
    __syncthreads();
    // element j = 312 b + q - f/2 comes from block b, pair q.  (A one-wave recurrence without
    // s_barrier -- a wave's LDS operations execute in order -- measured slower: 0.42 vs
    // 0.29 ms per step, its passes serialise on the LDS latency.)
    for (; !(a.dbg & 2) && (MTN / 2) * b - f / 2 < hi; ++b) {
      if (b > 0) mt_block(ring, (int)(b & 1), tid);
      const uint32_t* blk = ring + (b & 1) * MTN;
      const int q = tid;
      const int64_t j = (MTN / 2) * b + q - f / 2;
      const bool valid = q < MTN / 2 && !(b == 0 && q < f / 2) && j >= lo && j < hi;
      bool set = false;
      if (valid) {
        const uint32_t w0 = mt_temper(blk[2 * q]) >> 5, w1 = mt_temper(blk[2 * q + 1]) >> 6;
        const double u = ((double)w0 * 67108864.0 + (double)w1) / 9007199254740992.0;
        set = u < cr || j == fixed;
      }
      // a wave's elements are consecutive: one OR per mask word it touches (<= 3), from the word's
      // first lane in the wave, instead of 32 lanes' atomics on one LDS word (bank conflicts)
      const uint64_t bal = __builtin_amdgcn_ballot_w64(set);
      const int lane = tid & 63, bit = (int)((j - lo) & 31);
      if (valid && (bit == 0 || lane == 0)) {
        const uint32_t wb = (uint32_t)(lane >= bit ? bal >> (lane - bit) : bal << (bit - lane));
        if (wb) atomicOr(&mask[(j - lo) >> 5], wb);
      }
      if ((MTN / 2) * (b + 1) - f / 2 > hi) break;   // this block also feeds the next segment
    }
    __syncthreads();
    constexpr int U = 4;
    for (int64_t j0 = lo + tid; !(a.dbg & 4) && j0 < hi; j0 += (int64_t)U * NTHR) {
      double x[U], y0[U], y1[U], y2[U];
      bool m[U];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        const int64_t j = j0 + (int64_t)r * NTHR;
        m[r] = false;
        if (j < hi) {
          x[r] = P[j];
          m[r] = (mask[(j - lo) >> 5] >> ((j - lo) & 31)) & 1u;
          if (m[r]) {
            y0[r] = X0[j];
            y1[r] = X1[j];
            y2[r] = X2[j];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < U; ++r) {
        const int64_t j = j0 + (int64_t)r * NTHR;
        if (j >= hi) continue;
        double v = x[r];
        if (m[r]) {
          if (strategy == 0) v = y0[r] + F * (y1[r] - y2[r]);
          else v = (v + F * (y0[r] - v)) + F * (y1[r] - y2[r]);
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

// One launch per generation (small populations): every workgroup rebuilds the sequence, jumps, and
// streams its child with the sequence buffer as the mask.
__global__ __launch_bounds__(DE_THREADS) void k_de_step(DeArgs a) {
  // sequence buffer, 16-B aligned at word pos0 (sq = seq + sh) so the correlation reads b128s;
  // the slack covers the correlation's trailing loads (bits past degree 19936 are zero)
  __shared__ __attribute__((aligned(16))) uint32_t seq[SEQ_ALLOC];
  __shared__ uint32_t ring[2 * MTN];
  const int tid = threadIdx.x;
  const int i = blockIdx.x;
  const bool is_end = i == a.pop;
  const bool jump = is_end ? a.end_jump != 0 : i > 0;
  uint32_t* sq = seq + ((4 - (a.pos0 & 3)) & 3);
  de_sequence(a.key, sq, jump ? a.pos0 + tblup_mt::MT_DEG + MTN - 1 : (i == 0 ? a.pos0 + MTN : MTN), tid);
  de_window(a, seq, sq, ring, i, is_end, jump, tid);
  if (is_end) {
    de_end_state(a, ring, tid);
    return;
  }
  de_stream<DE_THREADS>(a, ring, seq, SEQ_WORDS, i, tid);
}

// Large populations, three launches: the base sequence once (one workgroup, into gseq), then every
// workgroup's jump (its window into gwin; the sequence buffer keeps these at one per CU), then the
// mask and stream on 320 threads with a small LDS footprint, several workgroups per CU -- the mask
// recurrence is a chain of barriers, so co-resident workgroups hide each other's.  The same
// arithmetic in the same order as k_de_step: the same bits.
__global__ __launch_bounds__(DE_THREADS) void k_de_seq(DeArgs a, uint32_t* __restrict__ gseq) {
  __shared__ __attribute__((aligned(16))) uint32_t seq[SEQ_ALLOC];
  const int tid = threadIdx.x;
  uint32_t* sq = seq + ((4 - (a.pos0 & 3)) & 3);
  const int need = a.pos0 + tblup_mt::MT_DEG + MTN - 1;
  de_sequence(a.key, sq, need, tid);
  for (int t = tid; t < need; t += DE_THREADS) gseq[t] = sq[t];
}

__global__ __launch_bounds__(DE_THREADS) void k_de_jump(DeArgs a, const uint32_t* __restrict__ gseq,
                                                        uint32_t* __restrict__ gwin) {
  __shared__ __attribute__((aligned(16))) uint32_t seq[SEQ_ALLOC];
  __shared__ uint32_t ring[2 * MTN];
  const int tid = threadIdx.x;
  const int i = blockIdx.x;
  const bool is_end = i == a.pop;
  const bool jump = is_end ? a.end_jump != 0 : i > 0;
  uint32_t* sq = seq + ((4 - (a.pos0 & 3)) & 3);
  const int need = jump ? a.pos0 + tblup_mt::MT_DEG + MTN - 1 : (i == 0 ? a.pos0 + MTN : MTN);
  for (int t = tid; t < need; t += DE_THREADS) sq[t] = gseq[t];
  __syncthreads();
  de_window(a, seq, sq, ring, i, is_end, jump, tid);
  if (is_end) {
    de_end_state(a, ring, tid);
    return;
  }
  if (tid < MTN) gwin[(int64_t)i * MTN + tid] = ring[tid];
}

constexpr int DE_MASK_THREADS = 320;
constexpr int DE_MASK_WORDS = 2048;   // 65536 elements per mask segment (8 KiB)
__global__ __launch_bounds__(DE_MASK_THREADS) void k_de_mask(DeArgs a, const uint32_t* __restrict__ gwin) {
  __shared__ uint32_t ring[2 * MTN];
  __shared__ uint32_t mask[DE_MASK_WORDS];
  const int tid = threadIdx.x;
  const int i = blockIdx.x;
  for (int t = tid; t < MTN; t += DE_MASK_THREADS) ring[t] = gwin[(int64_t)i * MTN + t];
  __syncthreads();
  de_stream<DE_MASK_THREADS>(a, ring, mask, DE_MASK_WORDS, i, tid);
}

}  // namespace

hipError_t launch_de_step(const uint32_t* key, int pos0, const uint32_t* polys, int end_jump, int end_s, int end_pos,
                          const double* parent, int64_t ldp, const int32_t* donors, const int64_t* fixed, int strategy,
                          double F, double cr, int clip, double hi, int64_t L, int pop, double* child, int64_t ldc,
                          uint32_t* key_out, int32_t* pos_out, hipStream_t s, const int32_t* strat_i,
                          const double* F_i, const double* cr_i, uint32_t* scratch) {
#ifdef TBLUP_DIAG_BUILD   // phase ablation (results wrong when set): diagnostic builds only
  static const int dbg = getenv("TBLUP_DE_DBG") ? atoi(getenv("TBLUP_DE_DBG")) : 0;
#else
  constexpr int dbg = 0;
#endif
  DeArgs a{key, pos0, polys, end_jump, end_s, end_pos, parent, ldp, donors, fixed, strategy, F, cr, clip, hi, L, pop,
           child, ldc, key_out, pos_out, dbg, strat_i, F_i, cr_i};
  if (scratch == nullptr) {
    hipLaunchKernelGGL(k_de_step, dim3(pop + 1), dim3(DE_THREADS), 0, s, a);
    return hipGetLastError();
  }
  uint32_t* gseq = scratch;
  uint32_t* gwin = scratch + DE_SEQ_SCRATCH;
  hipLaunchKernelGGL(k_de_seq, dim3(1), dim3(DE_THREADS), 0, s, a, gseq);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(k_de_jump, dim3(pop + 1), dim3(DE_THREADS), 0, s, a, gseq, gwin);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(k_de_mask, dim3(pop), dim3(DE_MASK_THREADS), 0, s, a, gwin);
  return hipGetLastError();
}

namespace {
// dst row r (L doubles) = the device row src.p[r]; 16-B loads and stores when L is even and
// the rows are 16-B aligned, else 8-B
__global__ __launch_bounds__(256) void k_gather_rows(double* __restrict__ dst, int64_t ldd, int64_t L, RowPtrs src,
                                                     int vec2) {
  const int64_t r = blockIdx.y;
  const double* sr = src.p[r];
  double* dr = dst + r * ldd;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (vec2) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; 2 * j < L; j += stride)
      reinterpret_cast<v2d*>(dr)[j] = reinterpret_cast<const v2d*>(sr)[j];
  } else {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < L; j += stride) dr[j] = sr[j];
  }
}
}  // namespace

hipError_t launch_gather_rows(double* dst, int64_t ldd, int64_t L, const RowPtrs& src, int nr, hipStream_t s) {
  if (nr <= 0 || L <= 0) return hipSuccess;
  bool vec2 = (L % 2 == 0) && (ldd % 2 == 0) && ((uintptr_t)dst % 16 == 0);
  for (int r = 0; r < nr; ++r) vec2 = vec2 && ((uintptr_t)src.p[r] % 16 == 0);
  const int64_t per = vec2 ? L / 2 : L;
  const int64_t nb = (per + 256 * 4 - 1) / (256 * 4);   // ~4 elements per thread
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)(nb < 256 ? nb : 256), (unsigned)nr), dim3(256), 0, s, dst, ldd, L,
                     src, vec2 ? 1 : 0);
  return hipGetLastError();
}

}  // namespace tblup
