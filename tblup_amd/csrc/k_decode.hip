// RandomKeyIndividual genome decode on the GPU:
//   genome = np.argsort(keys)[-k:]                      tblup/individual.py:154-156
// i.e. the k largest keys, returned in ascending key order.  Ties are resolved as a
// stable argsort does (equal keys keep index order, so the largest indices among a tie
// that straddles the k-th position are the ones selected); numpy's default quicksort
// gives the same set whenever no tie straddles the threshold (continuous keys).
//
// One 1024-thread workgroup per individual:
//   1. MSB-first radix select on the order-preserving uint64 image of the keys, 8 bits
//      per pass, LDS histogram; stops as soon as the boundary bucket is taken whole
//      (random keys: 2-3 passes over the 400 KB row at d = 50k)
//   2. compaction of the selected (key, index) pairs into LDS (ties: backward chunked
//      scan so the largest indices win)
//   3. bitonic sort of the k pairs by (key, index), written out as int64 indices at the
//      individual's offset (k may differ per individual: CoevolutionIndividual lengths)
#include "tblup_internal.h"

namespace tblup {

namespace {

constexpr int DTH = 1024;
constexpr int KSORT_MAX = 8192;   // LDS sort capacity (k <= 8192)

__device__ __forceinline__ uint64_t ord_key(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

}  // namespace

__global__ __launch_bounds__(DTH) void k_decode_topk(const double* __restrict__ keys, int64_t ld, int64_t d,
                                                     const int64_t* __restrict__ off, int64_t* __restrict__ out) {
  __shared__ uint64_t sk[KSORT_MAX];
  __shared__ int32_t si[KSORT_MAX];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t cnt_sh, tie_base_sh;
  __shared__ uint32_t wsum[DTH / 64];
  __shared__ int64_t sel_sh[4];   // prefix, shift, need, exact
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const double* row = keys + b * ld;
  const int64_t k = off[b + 1] - off[b];   // int(length) of this individual (host-checked 1..min(d, 8192))

  // ---- 1. radix select ----
  uint64_t prefix = 0;
  int shift = 64;            // bits below the resolved prefix
  int64_t need = k;          // how many of the elements matching `prefix` are still to take
  bool exact = false;
  for (int pass = 0; pass < 8; ++pass) {
    const int sh = 56 - 8 * pass;
    for (int i = t; i < 256; i += DTH) hist[i] = 0;
    __syncthreads();
    for (int64_t i = t; i < d; i += DTH) {
      const uint64_t u = ord_key(row[i]);
      if (pass == 0 || (u >> shift) == prefix) atomicAdd(&hist[(u >> sh) & 255], 1u);
    }
    __syncthreads();
    if (t == 0) {
      int64_t above = 0;
      int bsel = 0;
      for (int bin = 255; bin >= 0; --bin) {
        if (above + (int64_t)hist[bin] >= need) {
          bsel = bin;
          break;
        }
        above += hist[bin];
      }
      const int64_t nneed = need - above;
      sel_sh[0] = (int64_t)((prefix << 8) | (uint64_t)bsel);
      sel_sh[2] = nneed;
      sel_sh[3] = ((int64_t)hist[bsel] == nneed) ? 1 : 0;
    }
    __syncthreads();
    prefix = (uint64_t)sel_sh[0];
    need = sel_sh[2];
    exact = sel_sh[3] != 0;
    shift = sh;
    __syncthreads();
    if (exact) break;
  }
  // selected = {u >> shift > prefix}  u  (the `need` largest-index elements with u >> shift == prefix)

  // ---- 2. compaction ----
  if (t == 0) cnt_sh = 0;
  __syncthreads();
  for (int64_t i = t; i < d; i += DTH) {
    const uint64_t u = ord_key(row[i]);
    const uint64_t hi = u >> shift;
    if (hi > prefix || (exact && hi == prefix)) {
      const uint32_t pos = atomicAdd(&cnt_sh, 1u);
      sk[pos] = u;
      si[pos] = (int32_t)i;
    }
  }
  __syncthreads();
  if (!exact && need > 0) {
    // a true tie at the full 64-bit key: take the `need` largest indices, scanning
    // 1024-element chunks from the end of the row
    const uint32_t base = cnt_sh;
    if (t == 0) tie_base_sh = 0;
    __syncthreads();
    const int l = t & 63, w = t >> 6;
    for (int64_t c0 = ((d - 1) / DTH) * DTH; c0 >= 0; c0 -= DTH) {
      const int64_t i = c0 + (DTH - 1 - t);   // thread 0 takes the largest index of the chunk
      bool flag = false;
      uint64_t u = 0;
      if (i >= 0 && i < d) {
        u = ord_key(row[i]);
        flag = (u >> shift) == prefix;
      }
      // block-wide exclusive scan of the flags in thread order
      const uint64_t bal = __ballot(flag);
      const uint32_t lane_prefix = __popcll(bal & ((1ull << l) - 1ull));
      if (l == 0) wsum[w] = __popcll(bal);
      __syncthreads();
      uint32_t wbase = 0;
      for (int q = 0; q < w; ++q) wbase += wsum[q];
      const uint32_t rank = tie_base_sh + wbase + lane_prefix;
      if (flag && rank < (uint32_t)need) {
        sk[base + rank] = u;
        si[base + rank] = (int32_t)i;
      }
      __syncthreads();
      if (t == 0) {
        uint32_t tot = 0;
        for (int q = 0; q < DTH / 64; ++q) tot += wsum[q];
        tie_base_sh += tot;
      }
      __syncthreads();
      if (tie_base_sh >= (uint32_t)need) break;
    }
  }
  __syncthreads();

  // ---- 3. bitonic sort by (key, index) ascending over the next power of two ----
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  for (int i = t; i < n2; i += DTH)
    if (i >= k) {
      sk[i] = ~0ull;
      si[i] = 0x7fffffff;
    }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < n2 / 2; i += DTH) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = sk[lo], c = sk[hi];
        const int32_t ia = si[lo], ic = si[hi];
        const bool gt = (a > c) || (a == c && ia > ic);
        if (gt == up) {
          sk[lo] = c;
          sk[hi] = a;
          si[lo] = ic;
          si[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int64_t i = t; i < k; i += DTH) out[off[b] + i] = (int64_t)si[i];
}

hipError_t launch_decode_topk(const double* keys, int64_t B, int64_t d, int64_t ld, const int64_t* off, int64_t* out,
                              hipStream_t s) {
  if (d > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_decode_topk, dim3((unsigned)B), dim3(DTH), 0, s, keys, ld, d, off, out);
  return hipGetLastError();
}

}  // namespace tblup
