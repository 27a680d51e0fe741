// MT19937 jump-ahead (host, mt_jump.cpp): polynomials for the GPU DE step and a
// host jump of numpy's legacy RandomState (key[624], pos) state.
#pragma once
#include <cstdint>
#include <vector>

namespace tblup_mt {

constexpr int MT_N = 624;
constexpr int MT_DEG = 19937;

// x^J mod phi, 624 little-endian words (bit k = coefficient of x^k)
void jump_poly(uint64_t J, uint32_t* out624);

// Jump polynomials of one DE generation of `pop` individuals with genome length L
// (2L stream words each): row i-1 (i = 1..pop-1) = x^{2Li-2} (the window whose words
// 2.. are individual i's stream), row pop-1 = x^{2L pop - 625} (the window 625 words
// before the end of the generation's draws) when end_jump.  Cached per (L, pop).
struct DePolys {
  std::vector<uint32_t> words;   // pop x 624
  bool end_jump = false;
};
DePolys de_polys(int64_t L, int64_t pop);

// numpy's (key, pos) after n_words more outputs, taken from the 1248 words that follow the
// window at relative offset o_rel (pos0 + n - 625, or 0 when n < 625): key = words[s .. s+624)
struct EndState {
  uint64_t o_rel;
  int s;
  int pos;
};
EndState end_state(int pos0, uint64_t n_words);

// host jump of a numpy MT19937 state by n_words 32-bit outputs (tests and small cases)
void jump_state(const uint32_t* key, int pos, uint64_t n_words, uint32_t* key_out, int* pos_out);

// One DE generation's python-`random` draws (donors + the crossover's fixed position) on
// CPython's MT19937 state (random.getstate()[1]: mt[624], index); best < 0: DE/rand/1, else
// DE/current-to-best/1 with that best index.  Needs pop >= 4 and 1 <= L < 2^32.
void py_random_donors(uint32_t* mt, int32_t* index, int64_t pop, int64_t L, int32_t best, int32_t* donors,
                      int64_t* fixed);

}  // namespace tblup_mt
