// MT19937 jump-ahead over GF(2) — host side of the GPU differential-evolution step.
//
// The reference's binary crossover draws `np.random.rand(genome_len)` once per
// individual (tblup/evolver.py:77, numpy's legacy RandomState: two 32-bit MT19937
// outputs per double), so individual i of a generation consumes the global stream
// words [pos0 + 2Li, pos0 + 2L(i+1)).  To draw every individual's uniforms in
// parallel on the GPU, each workgroup starts from the MT19937 state jumped ahead by
// its offset.  The MT19937 sequence x_{t+624} = x_{t+397} ^ twist(x_t, x_{t+1}) is a
// linear recurrence over GF(2) with characteristic polynomial phi (degree 19937), so
// the state window W_{t+J} = p(A) W_t with p = x^J mod phi, and
//     W_{t+J}[j] = XOR_{k : p_k = 1} x_{t+k+j}
// (a GF(2) correlation of the sequence continuing from W_t with p's bits).  This file
// computes phi (Berlekamp-Massey on one output bit), x^J mod phi (carry-less
// multiplication + Barrett reduction), the per-individual polynomials of a DE step,
// and a host jump of a numpy (key, pos) state used by the tests.
//
// p(A)W equals A^J W except in the 31 low bits of the window's first word (those bits
// never influence later words), so jumped windows are always used from word 1 on.
#include "mt_jump.h"

#include <immintrin.h>

#include <cstring>
#include <map>
#include <mutex>
#include <utility>

namespace tblup_mt {
namespace {

constexpr int D = MT_DEG;               // 19937
constexpr int PW = (D + 1 + 63) / 64;   // 312 words: bits 0..D (phi is monic of degree D)

using Poly = std::vector<uint64_t>;

inline uint32_t twist(uint32_t xt, uint32_t xt1, uint32_t xtm) {
  const uint32_t y = (xt & 0x80000000u) | (xt1 & 0x7fffffffu);
  return xtm ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// extend s (first 624 words = a window) to `len` words of the sequence
void extend(std::vector<uint32_t>& s, size_t len) {
  size_t t = s.size();
  s.resize(len);
  for (; t < len; ++t) s[t] = twist(s[t - 624], s[t - 623], s[t - 227]);
}

// ---- carry-less arithmetic ----
__attribute__((target("pclmul,sse4.1"))) inline void clmul(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
  const __m128i r = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)a), _mm_cvtsi64_si128((long long)b), 0);
  lo = (uint64_t)_mm_cvtsi128_si64(r);
  hi = (uint64_t)_mm_extract_epi64(r, 1);
}

inline void clmul_soft(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
  uint64_t l = 0, h = 0;
  for (int i = 0; i < 64; ++i)
    if ((b >> i) & 1) {
      l ^= a << i;
      if (i) h ^= a >> (64 - i);
    }
  lo = l;
  hi = h;
}

bool have_pclmul() {
  static const bool ok = __builtin_cpu_supports("pclmul");
  return ok;
}

// out = a * b (out sized na + nb words)
__attribute__((target("pclmul,sse4.1"))) void mul_hw(const uint64_t* a, size_t na, const uint64_t* b, size_t nb,
                                                      uint64_t* out) {
  std::memset(out, 0, (na + nb) * 8);
  for (size_t i = 0; i < na; ++i) {
    if (!a[i]) continue;
    const __m128i av = _mm_cvtsi64_si128((long long)a[i]);
    for (size_t j = 0; j < nb; ++j) {
      const __m128i r = _mm_clmulepi64_si128(av, _mm_cvtsi64_si128((long long)b[j]), 0);
      out[i + j] ^= (uint64_t)_mm_cvtsi128_si64(r);
      out[i + j + 1] ^= (uint64_t)_mm_extract_epi64(r, 1);
    }
  }
}

void mul(const uint64_t* a, size_t na, const uint64_t* b, size_t nb, uint64_t* out) {
  if (have_pclmul()) return mul_hw(a, na, b, nb, out);
  std::memset(out, 0, (na + nb) * 8);
  for (size_t i = 0; i < na; ++i)
    for (size_t j = 0; j < nb; ++j) {
      uint64_t lo, hi;
      clmul_soft(a[i], b[j], lo, hi);
      out[i + j] ^= lo;
      out[i + j + 1] ^= hi;
    }
}

// floor(P / x^s) into `out` (nout words)
void shr(const uint64_t* P, size_t np, int s, uint64_t* out, size_t nout) {
  const size_t q = (size_t)s >> 6;
  const int r = s & 63;
  for (size_t w = 0; w < nout; ++w) {
    const size_t i = w + q;
    uint64_t v = i < np ? P[i] >> r : 0;
    if (r && i + 1 < np) v |= P[i + 1] << (64 - r);
    out[w] = v;
  }
}

inline void mask_low(uint64_t* p, size_t n, int bits) {  // keep bits [0, bits)
  for (size_t w = 0; w < n; ++w) {
    const int lo = (int)w * 64;
    if (lo >= bits) p[w] = 0;
    else if (bits - lo < 64) p[w] &= (1ull << (bits - lo)) - 1;
  }
}

inline bool bit(const uint64_t* p, int64_t i) { return (p[i >> 6] >> (i & 63)) & 1; }

// ---- Berlekamp-Massey: minimal polynomial of a binary sequence ----
// returns the characteristic polynomial phi(x) = x^L C(1/x) (bit i = coefficient of x^i)
Poly berlekamp_massey(const std::vector<uint8_t>& s, int& L_out) {
  const size_t n = s.size();
  const size_t W = n / 64 + 3;
  std::vector<uint64_t> rs(W, 0);   // reversed sequence: bit (n-1-t) = s_t
  for (size_t t = 0; t < n; ++t)
    if (s[t]) rs[(n - 1 - t) >> 6] |= 1ull << ((n - 1 - t) & 63);
  std::vector<uint64_t> C(W, 0), B(W, 0), T;
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  auto xor_shift = [&](std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, int sh) {
    const int q = sh >> 6, r = sh & 63;
    for (size_t w = 0; w + q < W; ++w) {
      if (!src[w]) continue;
      dst[w + q] ^= src[w] << r;
      if (r && w + q + 1 < W) dst[w + q + 1] ^= src[w] >> (64 - r);
    }
  };
  for (size_t i = 0; i < n; ++i) {
    const size_t base = n - 1 - i;   // sum_j C_j s_{i-j} = sum_j C_j rs[base + j]
    uint64_t acc = 0;
    const int nw = L / 64 + 1;
    for (int w = 0; w < nw; ++w) {
      const size_t b = base + 64 * (size_t)w, q = b >> 6;
      const int r = (int)(b & 63);
      uint64_t v = q < W ? rs[q] >> r : 0;
      if (r && q + 1 < W) v |= rs[q + 1] << (64 - r);
      acc ^= C[w] & v;
    }
    if (!__builtin_parityll(acc)) {
      ++m;
      continue;
    }
    if (2 * L <= (int)i) {
      T = C;
      xor_shift(C, B, m);
      L = (int)i + 1 - L;
      B = T;
      m = 1;
    } else {
      xor_shift(C, B, m);
      ++m;
    }
  }
  L_out = L;
  Poly phi(PW, 0);
  for (int j = 0; j <= L && j <= D; ++j)
    if (bit(C.data(), L - j)) phi[j >> 6] |= 1ull << (j & 63);
  return phi;
}

struct Field {
  Poly phi;   // x^D + ...  (PW words)
  Poly mu;    // floor(x^{2D} / phi), degree D (PW words)
};

const Field& field() {
  static Field F;
  static std::once_flag once;
  std::call_once(once, [] {
    // sequence: bit 31 of x_t from MT19937's init_genrand(5489) key, 2D + 64 terms
    std::vector<uint32_t> x(624);
    x[0] = 5489u;
    for (int i = 1; i < 624; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    const size_t n = 2 * (size_t)D + 64;
    extend(x, n);
    std::vector<uint8_t> s(n);
    for (size_t t = 0; t < n; ++t) s[t] = (uint8_t)(x[t] >> 31);
    int L = 0;
    F.phi = berlekamp_massey(s, L);
    if (L != D) std::abort();   // MT19937's minimal polynomial has degree 19937
    // mu = floor(x^{2D} / phi) by long division
    const int64_t nb = 2 * (int64_t)D + 1;
    std::vector<uint64_t> rem((nb + 63) / 64 + 1, 0), q((D + 1 + 63) / 64 + 1, 0);
    rem[(2 * D) >> 6] |= 1ull << ((2 * D) & 63);
    for (int64_t b = 2 * (int64_t)D; b >= D; --b) {
      if (!bit(rem.data(), b)) continue;
      const int64_t sh = b - D;
      q[sh >> 6] |= 1ull << (sh & 63);
      const int64_t wq = sh >> 6;
      const int r = (int)(sh & 63);
      for (int w = 0; w < PW; ++w) {
        if (!F.phi[w]) continue;
        rem[w + wq] ^= F.phi[w] << r;
        if (r) rem[w + wq + 1] ^= F.phi[w] >> (64 - r);
      }
    }
    F.mu.assign(q.begin(), q.begin() + PW);
  });
  return F;
}

// P (2*PW words, degree < 2D) mod phi -> r (PW words, degree < D): Barrett reduction
// (exact over GF(2)[x]: no correction step).
void reduce(const uint64_t* P, uint64_t* r) {
  const Field& F = field();
  uint64_t q1[PW], t[2 * PW + 2], q[PW], qp[2 * PW];
  shr(P, 2 * PW, D, q1, PW);                 // floor(P / x^D)
  mul(q1, PW, F.mu.data(), PW, t);           // * mu
  shr(t, 2 * PW, D, q, PW);                  // quotient
  mul(q, PW, F.phi.data(), PW, qp);
  for (int w = 0; w < PW; ++w) r[w] = P[w] ^ qp[w];
  mask_low(r, PW, D);
}

void mulmod(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  uint64_t P[2 * PW];
  mul(a, PW, b, PW, P);
  reduce(P, out);
}

// x^J mod phi
Poly powmod_x(uint64_t J) {
  const Field& F = field();
  Poly r(PW, 0);
  r[0] = 1;
  if (J == 0) return r;
  int top = 63;
  while (!((J >> top) & 1)) --top;
  uint64_t P[2 * PW];
  for (int b = top; b >= 0; --b) {
    mul(r.data(), PW, r.data(), PW, P);   // square
    reduce(P, r.data());
    if ((J >> b) & 1) {                   // * x
      const bool carry = bit(r.data(), D - 1);
      for (int w = PW - 1; w > 0; --w) r[w] = (r[w] << 1) | (r[w - 1] >> 63);
      r[0] <<= 1;
      if (carry)
        for (int w = 0; w < PW; ++w) r[w] ^= F.phi[w];
      mask_low(r.data(), PW, D);
    }
  }
  return r;
}

inline void to_words32(const Poly& p, uint32_t* out) {   // little-endian reinterpretation
  for (int w = 0; w < MT_N; ++w) out[w] = (uint32_t)(p[w >> 1] >> (32 * (w & 1)));
}

// window at relative offset `off` of the sequence that starts with `key` (no jump): seq words [off, off+624)
// jumped window: W[j] = XOR_{k: p_k} seq[base + k + j]
void apply_poly(const std::vector<uint32_t>& seq, size_t base, const Poly& p, uint32_t* W) {
  uint32_t acc[MT_N] = {0};
  for (int k = 0; k < D; ++k)
    if (bit(p.data(), k)) {
      const uint32_t* s = seq.data() + base + k;
      for (int j = 0; j < MT_N; ++j) acc[j] ^= s[j];
    }
  std::memcpy(W, acc, sizeof(acc));
}

}  // namespace

void jump_poly(uint64_t J, uint32_t* out) { to_words32(powmod_x(J), out); }

DePolys de_polys(int64_t L, int64_t pop) {
  static std::mutex mu;
  static std::map<std::pair<int64_t, int64_t>, DePolys> cache;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({L, pop});
    if (it != cache.end()) return it->second;
  }
  DePolys out;
  out.words.assign((size_t)pop * MT_N, 0u);
  const uint64_t step = 2 * (uint64_t)L;
  if (pop > 1) {
    Poly p = powmod_x(step - 2);   // individual 1: window at pos0 + 2L - 2
    const Poly q = powmod_x(step);
    Poly nxt(PW);
    for (int64_t i = 1; i < pop; ++i) {
      to_words32(p, &out.words[(size_t)(i - 1) * MT_N]);
      if (i + 1 < pop) {
        mulmod(p.data(), q.data(), nxt.data());
        p.swap(nxt);
      }
    }
  }
  const uint64_t total = step * (uint64_t)pop;
  out.end_jump = total >= 625;
  if (out.end_jump) to_words32(powmod_x(total - 625), &out.words[(size_t)(pop - 1) * MT_N]);
  std::lock_guard<std::mutex> g(mu);
  cache[{L, pop}] = out;
  return out;
}

EndState end_state(int pos0, uint64_t n_words) {
  EndState e;
  const uint64_t r_end = (uint64_t)pos0 + n_words;
  e.o_rel = n_words >= 625 ? (uint64_t)pos0 + n_words - 625 : 0;
  const uint64_t tq = (r_end - 1) / MT_N;
  e.s = (int)(tq * MT_N - e.o_rel);
  e.pos = (int)(r_end - tq * MT_N);
  return e;
}

void jump_state(const uint32_t* key, int pos, uint64_t n_words, uint32_t* key_out, int* pos_out) {
  if (n_words == 0 || (uint64_t)pos + n_words == 0) {
    std::memcpy(key_out, key, MT_N * 4);
    *pos_out = pos;
    return;
  }
  std::vector<uint32_t> seq(key, key + MT_N);
  uint32_t W[MT_N];
  if (n_words >= 625) {
    extend(seq, (size_t)pos + D + MT_N);
    apply_poly(seq, (size_t)pos, powmod_x(n_words - 625), W);
  } else {
    std::memcpy(W, key, sizeof(W));
  }
  std::vector<uint32_t> w(W, W + MT_N);
  extend(w, 2 * MT_N);
  const EndState e = end_state(pos, n_words);
  std::memcpy(key_out, w.data() + e.s, MT_N * 4);
  *pos_out = e.pos;
}

// ---- CPython's `random` (Modules/_randommodule.c of CPython 3.10): the same MT19937
// recurrence, consumed one tempered word at a time from (mt, index); randrange(0, n) is
// _randbelow_with_getrandbits(n): k = n.bit_length(), draw getrandbits(k) = word >> (32 - k)
// until it is < n.  The donor loops restate utils.py:21-36 (exclusive_randrange: first draw,
// then redraw while excluded), evolver.py:118-121 (a, b, c) and :199-203 (a, b beside the
// best), then evolver.py:76 (fixed = randrange(0, L)), in that order per individual.
namespace {

struct PyMT {
  uint32_t* mt;
  int idx;
  uint32_t word() {
    if (idx >= MT_N) {
      for (int k = 0; k < MT_N; ++k) mt[k] = twist(mt[k], mt[(k + 1) % MT_N], mt[(k + 397) % MT_N]);
      idx = 0;
    }
    uint32_t y = mt[idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  uint32_t below(uint64_t n) {   // 1 <= n < 2^32
    const int k = 64 - __builtin_clzll(n);
    uint32_t r = word() >> (32 - k);
    while (r >= n) r = word() >> (32 - k);
    return r;
  }
  // exclusive_randrange(0, n, ex[0..ne))
  uint32_t excluding(uint64_t n, const int64_t* ex, int ne) {
    for (;;) {
      const uint32_t r = below(n);
      bool hit = false;
      for (int j = 0; j < ne; ++j) hit |= (int64_t)r == ex[j];
      if (!hit) return r;
    }
  }
};

}  // namespace

void py_random_donors(uint32_t* mt, int32_t* index, int64_t pop, int64_t L, int32_t best, int32_t* donors,
                      int64_t* fixed) {
  PyMT g{mt, *index};
  for (int64_t i = 0; i < pop; ++i) {
    if (best < 0) {
      int64_t ex[3] = {i, 0, 0};
      ex[1] = g.excluding(pop, ex, 1);
      ex[2] = g.excluding(pop, ex, 2);
      const int64_t c = g.excluding(pop, ex, 3);
      donors[3 * i] = (int32_t)ex[1];
      donors[3 * i + 1] = (int32_t)ex[2];
      donors[3 * i + 2] = (int32_t)c;
    } else {
      int64_t ex[3] = {i, best, 0};
      ex[2] = g.excluding(pop, ex, 2);
      const int64_t b = g.excluding(pop, ex, 3);
      donors[3 * i] = best;
      donors[3 * i + 1] = (int32_t)ex[2];
      donors[3 * i + 2] = (int32_t)b;
    }
    fixed[i] = g.below((uint64_t)L);
  }
  *index = g.idx;
}

}  // namespace tblup_mt
