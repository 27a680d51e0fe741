// RandomKeyIndividual genome decode on the GPU:
//   genome = np.argsort(keys)[-k:]                      tblup/individual.py:154-156
// i.e. the k largest keys, returned in ascending key order.  Ties are resolved as a
// stable argsort does (equal keys keep index order, so the largest indices among a tie
// that straddles the k-th position are the ones selected); numpy's default quicksort
// gives the same set whenever no tie straddles the threshold (continuous keys).
//
// One 1024-thread workgroup per individual:
//   1. fast path: a strided sample (<= 4096 keys, in runs of 8) in LDS gives a threshold with ~1.25 k
//      keys above it; one pass over the row collects them in LDS; an exact radix select
//      among those candidates picks the k largest (one read of the 400 KB row at d = 50k)
//   2. fallback (candidates < k or > 8192, or a full-key tie at the k-th key): MSB-first
//      radix select on the order-preserving uint64 image of the row, 8 bits per pass,
//      LDS histogram, then compaction (ties: backward chunked scan, largest indices win)
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

// MSB-first radix select, 8 bits per pass, of the `want`-th largest of get(0..n): on return
// the selected set is {u >> shift > prefix} plus, when `exact`, the whole bucket
// {u >> shift == prefix}; otherwise `need` elements of that bucket remain to be chosen.
template <typename Get>
__device__ __forceinline__ void radix_select(Get get, int64_t n, int64_t want, int max_pass, uint32_t* hist,
                                             int64_t* sel_sh, uint64_t& prefix, int& shift, int64_t& need,
                                             bool& exact) {
  const int t = threadIdx.x;
  prefix = 0;
  shift = 64;
  need = want;
  exact = false;
  for (int pass = 0; pass < max_pass; ++pass) {
    const int sh = 56 - 8 * pass;
    for (int i = t; i < 256; i += DTH) hist[i] = 0;
    __syncthreads();
    for (int64_t i = t; i < n; i += DTH) {
      const uint64_t u = get(i);
      if (pass == 0 || (u >> shift) == prefix) atomicAdd(&hist[(u >> sh) & 255], 1u);
    }
    __syncthreads();
    if (t < 64) {
      // boundary bin = the first bin from the top whose inclusive count from the top reaches
      // `need`: lane l holds bins 4l..4l+3, a suffix scan over lanes finds the crossing lane
      uint32_t h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = hist[4 * t + j];
      const uint32_t sl = h[0] + h[1] + h[2] + h[3];
      uint32_t suf = sl;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_down(suf, o);
        if (t + o < 64) suf += v;
      }
      const int64_t excl = (int64_t)(suf - sl);
      if (excl < need && need <= (int64_t)suf) {
        int64_t above = excl;
        int jsel = 0;
#pragma unroll
        for (int j = 3; j >= 0; --j) {
          if (above + (int64_t)h[j] >= need) {
            jsel = j;
            break;
          }
          above += h[j];
        }
        const int64_t nneed = need - above;
        const uint32_t hsel = jsel == 3 ? h[3] : jsel == 2 ? h[2] : jsel == 1 ? h[1] : h[0];
        sel_sh[0] = (int64_t)((prefix << 8) | (uint64_t)(4 * t + jsel));
        sel_sh[2] = nneed;
        sel_sh[3] = ((int64_t)hsel == nneed) ? 1 : 0;
      }
    }
    __syncthreads();
    prefix = (uint64_t)sel_sh[0];
    need = sel_sh[2];
    exact = sel_sh[3] != 0;
    shift = sh;
    __syncthreads();
    if (exact) break;
  }
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

  // ---- 1. fast path: threshold from a strided sample, ONE pass over the row ----
  //   a. the keys at i = s*j (<= 4096 of them) into LDS; tau = lower edge of the 24-bit
  //      bucket holding the sample's r-th largest, r ~ 1.25 k / s (so about 1.25 k keys of
  //      the row are >= tau); b. one pass appends every (key, index) >= tau to LDS;
  //   c. exact radix select of the k-th largest among those candidates in LDS.
  // Falls back to the radix select over the row (section 2) when the candidates do not
  // cover k, overflow the 8192 slots, or the k-th key is tied at full 64 bits.
  __shared__ int fast_sh;
  {
    // the sample: runs of 8 consecutive keys (one 64-B line) every 8 s keys, so it reads about
    // 1/s of the row's lines (a single key every s touched up to one line per sample, more
    // bytes than the row itself at s >= 8); slots past the row hold 0, below every key
    const int64_t s = (d + 4095) / 4096;
    const int64_t ns = 8 * ((d + 8 * s - 1) / (8 * s));
    for (int64_t j = t; j < ns; j += DTH) {
      const int64_t i = (j >> 3) * (8 * s) + (j & 7);
      sk[j] = i < d ? ord_key(row[i]) : 0ull;
    }
    __syncthreads();
    int64_t r = (5 * k) / (4 * s) + 8;
    r = r < ns ? r : ns;
    uint64_t pre;
    int shf;
    int64_t nd;
    bool ex;
    radix_select([&](int64_t i) { return sk[i]; }, ns, r, 3, hist, sel_sh, pre, shf, nd, ex);
    if (t == 0) cnt_sh = 0;
    __syncthreads();
    for (int64_t i = t; i < d; i += DTH) {
      const uint64_t u = ord_key(row[i]);
      if ((u >> shf) >= pre) {
        const uint32_t pos = atomicAdd(&cnt_sh, 1u);
        if (pos < KSORT_MAX) {
          sk[pos] = u;
          si[pos] = (int32_t)i;
        }
      }
    }
    __syncthreads();
    const int64_t c = cnt_sh;
    bool ok = c >= k && c <= KSORT_MAX;
    if (ok) {
      radix_select([&](int64_t i) { return sk[i]; }, c, k, 8, hist, sel_sh, pre, shf, nd, ex);
      ok = ex;
    }
    if (ok) {
      // keep exactly the k selected candidates: registers first, then compact from slot 0
      uint64_t ku[KSORT_MAX / DTH];
      int32_t ki[KSORT_MAX / DTH];
#pragma unroll
      for (int q = 0; q < KSORT_MAX / DTH; ++q) {
        const int64_t e = t + (int64_t)q * DTH;
        ku[q] = e < c ? sk[e] : 0;
        ki[q] = e < c ? si[e] : -1;
      }
      __syncthreads();
      if (t == 0) cnt_sh = 0;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < KSORT_MAX / DTH; ++q) {
        if (ki[q] >= 0 && (ku[q] >> shf) >= pre) {
          const uint32_t pos = atomicAdd(&cnt_sh, 1u);
          sk[pos] = ku[q];
          si[pos] = ki[q];
        }
      }
    }
    if (t == 0) fast_sh = ok ? 1 : 0;
    __syncthreads();
  }

  if (!fast_sh) {
  // ---- 2. fallback: radix select over the row, compaction, full-key ties by index ----
  uint64_t prefix;
  int shift;
  int64_t need;
  bool exact;
  radix_select([&](int64_t i) { return ord_key(row[i]); }, d, k, 8, hist, sel_sh, prefix, shift, need, exact);
  // selected = {u >> shift > prefix}  u  (the `need` largest-index elements with u >> shift == prefix)

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

  }

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
