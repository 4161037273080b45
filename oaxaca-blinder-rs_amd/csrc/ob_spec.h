// ob_spec.h -- the OBRS-3 resample stream and the per-replicate row layout, shared by the HIP
// kernels (device) and the host runtime. DESIGN.md §3 is the normative description.
//
// The reference resamples each group with polars `sample_n_literal(n_g, with_replacement=true,
// shuffle=false, seed=None)` (oaxaca_blinder/src/builder.rs:822-827): n_g i.i.d. uniform row
// draws per group, unseeded. OBRS-3 produces the same distribution (an exact multinomial with
// cell probability 1/n_g) from a counter-based stream so that replicate r is reproducible from
// (seed, r) alone on any GPU count:
//   level 1: the tile counts m_j of n_g uniform row draws, by binomial splitting (no per-draw
//            index): over the dyadic tree of 2^D >= T tiles a node holding c draws sends an exact
//            Binomial(c, 1/2) left and the rest right (ob_l1_split_stream: Knuth-Yao samples of
//            B(2^j, 1/2) over the binary digits of c, OBRS-1's popcount of c fair bits for the
//            low 7); children past the last tile and draws a partial last tile rejects (byte >=
//            its rows) are drawn again in further rounds, the last <= 2048 by Lemire's
//            multiply-and-reject over [0, n_g). DESIGN.md §3, oracle orc_level1_counts.
//   level 2: m_j draws inside tile j (S_j rows). Full tiles (S_j = OB_TILE_ROWS = 2^8): Philox
//            call p yields draws 16p..16p+15, draw 16p + 4i + b = byte b (LSB first) of output
//            word i (exactly uniform, independent). The partial last tile: call p yields draws
//            2p, 2p+1, local = mulhi64(u64, S_j) of words (x,y) and (z,w).
// Conditional on the tile counts the level-2 draws are i.i.d. uniform in their tile, so the
// joint law of per-row counts equals that of n_g i.i.d. uniform draws over the group.
// (OBRS-1, rounds 1-2, split a level-1 node by the popcount of c fair bits: ~5.5M bits per group
// and replicate at 500k rows against ~0.5M for OBRS-2, rounds 3-4. OBRS-3, round 5, draws the last
// <= 2048 rejected draws directly instead of <= 256: at configs[1] the third round's ~1,000 draws
// then take four Philox calls a thread instead of a pass over the whole tree, level 1 1.94 -> 1.71 ms.
// Level 2 is the same in all three.)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define OB_HD __host__ __device__ __forceinline__
#else
#define OB_HD static inline
#endif

#define OB_TILE_ROWS 256u
#define OB_TILE_SHIFT 8u
#define OB_TAG_L1T 0x4C310000u /* "L1" + (round << 5) + level: popcount bits of node k (c < 4096), {q, rep, 2k | g} */
#define OB_TAG_L1K 0x4B310000u /* "K1" + (round << 5) + level: KY streams of node k (c >= 4096), {q << 12 | call, rep, 2k | g} */
#ifndef OB_KY_MIN_C
#define OB_KY_MIN_C 4096u      /* a node of at least this many draws splits by Knuth-Yao samples */
#endif
#define OB_TAG_L1S 0x4C530000u /* "LS" + round: partial-tile acceptance bytes, {q, rep, g} */
#define OB_TAG_L1D 0x4C440000u /* "LD" + (j >> 2): direct draw r, attempt j, {r, rep, g} */
#ifndef OB_L1_DIRECT
#define OB_L1_DIRECT 2048u     /* rejected draws at most this many are drawn directly (OBRS-3) */
#endif
#if !defined(OB_TUNING) || !OB_TUNING
/* OBRS-3 fixes both constants: another value is another stream (the oracle and the golden rows
   use 4096 / 2048), so only a tuning build may override them. */
static_assert(OB_L1_DIRECT == 2048u, "OB_L1_DIRECT is part of the OBRS-3 stream");
static_assert(OB_KY_MIN_C == 4096u, "OB_KY_MIN_C is part of the OBRS-3 stream");
#endif
#define OB_TAG_L2 0x4F425232u  /* "OBR2" */

struct ob_u32x4 {
  uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11), Random123 constants.
OB_HD ob_u32x4 ob_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  ob_u32x4 o = {c0, c1, c2, c3};
  return o;
}

// The same function with each three-way xor as one v_bitop3_b32 (truth table 0x96) on gfx950,
// where the compiler otherwise emits two v_xor_b32 per output word. The level-2 count kernel
// draws with it (4.78 -> 4.48 ms at configs[1]), level 1's streams too (OB_L1_PHILOX). Identical
// outputs by construction.
OB_HD uint32_t ob_xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

OB_HD ob_u32x4 ob_philox_x3(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = ob_xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = ob_xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  ob_u32x4 o = {c0, c1, c2, c3};
  return o;
}

// ---- OBRS-2 level-1 split ---------------------------------------------------------------------
#ifndef OB_L1_PHILOX
// the level-1 streams' Philox: ob_philox_x3, the same function with bitop3 xors (2.19 -> 2.03 ms per
// level-1 launch at configs[1], tools/ab_libs.sh; ob_philox measured faster before the level-1
// kernel lost its per-block L2 write-back)
#define OB_L1_PHILOX ob_philox_x3
#endif
// Binomial(c, 1/2) of a node with c < OB_KY_MIN_C draws: the popcount of c fair bits (OBRS-1's
// split, ob_l1_split_bits). From OB_KY_MIN_C up, the sum of exact B(2^j, 1/2) samples over the binary
// digits of c: c >> 12 samples of B(4096), one B(2^j) per set bit j = 11 .. 7, and the popcount of
// c & 127 fair bits.
// B(n = 2^j) is a Knuth-Yao walk (discrete distribution generating tree) over the dyadic
// probabilities p_k = C(n, k) / 2^n: column i = 1 .. n of the tree holds the k whose bit n - i of
// C(n, k) is set, in ascending k (list[off[i] .. off[i+1])); the walk reads one stream bit per
// column, d = 2 d + bit, returns the d-th entry when d < the column's count and subtracts the
// count otherwise. Exact, ~H + 2 ~ 9 bits per sample. Streams, one sample each: q < c >> 12 carries
// B(4096) sample q, the next ones one B(2^j) per set bit j = 11 .. 7 (high to low), the last, when
// c & 127 != 0, the c & 127 popcount bits; bit b of stream q is bit (b & 31) of word ((b >> 5) & 3)
// of Philox({q << 12 | b >> 7, rep, c2, tag}).
#define OB_KY_MIN_LOG 7
#define OB_KY_MAX_LOG 12
#define OB_KY_TABLES (OB_KY_MAX_LOG - OB_KY_MIN_LOG + 1)
#define OB_KY_HOT 9         // columns i0 .. i0 + 8 of each table staged in LDS: a walk ends there with p > 0.99
#define OB_KY_HOT_CAP 2192  // their entries, all tables (2,186 at OB_KY_HOT = 9)

// The tables on the device (built once per process, ob_engine.hip ky_host): table t (n = 2^(t + 7))
// has n + 2 column offsets at off + off_base[t] (positions in its own list) and its list at
// list + list_base[t]; hot = [OB_KY_TABLES][OB_KY_HOT + 1] offsets of the hot columns into the hot
// entries that follow as uint16 pairs.
struct ob_ky_tables {
  const uint32_t* off;
  const uint16_t* list;
  const uint32_t* hot;
  uint32_t off_base[OB_KY_TABLES], list_base[OB_KY_TABLES], i0[OB_KY_TABLES];
  uint32_t hot_entries;
};

// Fair bits [128 q, min(c, 128 q + 128)) of a node's popcount stream, counted (nodes of c < 4096
// draws): bit b is bit (b & 31) of word ((b >> 5) & 3) of Philox({b >> 7, rep, c2, tag}).
OB_HD uint32_t ob_l1_split_bits(uint32_t q, uint32_t c, uint32_t rep, uint32_t c2, uint32_t tag, uint32_t k0,
                                uint32_t k1) {
  const ob_u32x4 u = OB_L1_PHILOX(q, rep, c2, tag, k0, k1);
  const uint32_t r = c - 128u * q;
  const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
  uint32_t s = 0;
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t nb = r > 32u * i ? r - 32u * i : 0u;
    s += (uint32_t)__builtin_popcount(nb >= 32u ? wd[i] : (wd[i] & ((1u << nb) - 1u)));
  }
  return s;
}

// Work items of a node's split: popcount words below OB_KY_MIN_C, else its streams (c >> 12 of
// B(4096), one per set bit 11 .. 7, one for the popcount of c & 127 when nonzero).
OB_HD uint32_t ob_l1_items(uint32_t c) {
  return c < OB_KY_MIN_C ? (c + 127u) >> 7
                         : (c >> 12) + (uint32_t)__builtin_popcount((c >> 7) & 31u) + ((c & 127u) ? 1u : 0u);
}
// Stream i (< the digit streams) after the B(4096) ones: the table exponent j of the i-th set bit of
// c among bits 11 .. 7, high to low.
OB_HD uint32_t ob_l1_digit_log(uint32_t c, uint32_t i) {
  uint32_t j = OB_KY_MAX_LOG - 1;
  for (;; --j)
    if ((c >> j) & 1u) {
      if (i == 0) return j;
      --i;
    }
}

// A node stream: bit b is bit (b & 31) of word ((b >> 5) & 3) of Philox({ctr0 | b >> 7, rep, c2, tag}).
struct ob_bitstream {
  uint32_t ctr0, rep, c2, tag, k0, k1;
  uint32_t pos;
  uint32_t w0, w1, w2, w3;
};

OB_HD uint32_t ob_bs_word(ob_bitstream& s) {  // the 32-bit word holding bit s.pos (refilled per 128 bits)
  if ((s.pos & 127u) == 0) {
    const ob_u32x4 u = OB_L1_PHILOX(s.ctr0 | (s.pos >> 7), s.rep, s.c2, s.tag, s.k0, s.k1);
    s.w0 = u.x;
    s.w1 = u.y;
    s.w2 = u.z;
    s.w3 = u.w;
  }
  const uint32_t q = (s.pos >> 5) & 3u;
  return q == 0 ? s.w0 : q == 1 ? s.w1 : q == 2 ? s.w2 : s.w3;
}

OB_HD uint32_t ob_bs_bit(ob_bitstream& s) {
  const uint32_t b = (ob_bs_word(s) >> (s.pos & 31u)) & 1u;
  ++s.pos;
  return b;
}

// The next m <= 32 stream bits as an integer, the first bit most significant (d = 2 d + bit, m times).
OB_HD uint32_t ob_bs_take_msb(ob_bitstream& s, uint32_t m) {
  uint32_t v = 0;
  while (m) {
    const uint32_t sh = s.pos & 31u, take = m < 32u - sh ? m : 32u - sh;
    const uint32_t w = ob_bs_word(s) >> sh;
    const uint32_t chunk = take == 32u ? w : (w & ((1u << take) - 1u));
    const uint32_t rev = __builtin_bitreverse32(chunk) >> (32u - take);
    v = take == 32u ? rev : ((v << take) | rev);
    s.pos += take;
    m -= take;
  }
  return v;
}

// Popcount of the next m stream bits.
OB_HD uint32_t ob_bs_popcount(ob_bitstream& s, uint32_t m) {
  uint32_t left = 0;
  while (m) {
    const uint32_t sh = s.pos & 31u, take = m < 32u - sh ? m : 32u - sh;
    const uint32_t w = ob_bs_word(s) >> sh;
    left += (uint32_t)__builtin_popcount(take == 32u ? w : (w & ((1u << take) - 1u)));
    s.pos += take;
    m -= take;
  }
  return left;
}
// The walk and the stream split (device, LDS-staged hot columns): ob_engine.hip ky_walk,
// l1_split_stream; restated independently in oracle/ob_oracle.c orc_split_left.

// floor(u * s / 2^64), s < 2^32.
OB_HD uint32_t ob_mulhi64(uint32_t lo, uint32_t hi, uint32_t s) {
  const uint64_t h = (uint64_t)hi * s;
  const uint64_t l = ((uint64_t)lo * s) >> 32;
  return (uint32_t)((h + l) >> 32);
}

// ---- per-replicate result row (also include/oaxaca_boot.h OB_ROW_*) ------------------------
// [0] explained [1] unexplained [2] endowments [3] coefficients [4] interaction [5] total_gap
// [6, 6+Kd) detailed explained  [6+Kd, 6+2Kd) detailed unexplained   (Kd = K + n_base)
// then beta_a[K], beta_b[K], xa_mean[K], xb_mean[K], beta_star[K]
OB_HD int ob_row_len(int k, int n_base) { return 6 + 2 * (k + n_base) + 5 * k; }

// Extended-Gram pair enumeration over v = [1, x_1..x_P, y] (K1 = P + 2 entries):
// e -> (a, b), a <= b, a-major: (0,0),(0,1)..(0,K1-1),(1,1),...  E = K1 (K1 + 1) / 2.
OB_HD int ob_pair_index(int a, int b, int k1) {  // requires a <= b
  return a * k1 - (a * (a - 1)) / 2 + (b - a);
}

// ---- MM-1: the Machado-Mata draws (quantile_decomposition.rs:215-258) ------------------------
// The reference draws from an unseeded thread_rng: `simulations` quantiles tau ~ U(0.01, 0.99)
// shared by both groups, then one random row of X_A and of X_B per successful simulation. MM-1
// draws the same laws from the counter-based stream, so a pass is a pure function of
// (seed, replicate id):
//   tau_s   = 0.01 + 0.98 u, u = (hi27(x) 2^26 + hi26(y)) 2^-53 of Philox({s, rep, 0, MMT1}) (x, y)
//             words, kept below 0.99;
//   pick_i  = exact uniform position on [0, n_g): Lemire on word (j & 3) of
//             Philox({i, rep, g, MMR1 + (j >> 2)}) for attempt j (reject iff low32(w n) < 2^32 mod n).
// A position of a bootstrap sample maps to the row whose cumulative count first exceeds it (the
// sample in row order; any fixed order of a uniform position has the same law). The point
// estimate runs as replicate OB_MM_POINT_REP with every row once.
#define OB_TAG_MMT 0x4D4D5431u /* "MMT1" */
#define OB_TAG_MMR 0x4D4D5231u /* "MMR1" */
#define OB_MM_POINT_REP 0xFFFFFFFFu

OB_HD double ob_mm_tau(uint32_t s, uint32_t rep, uint32_t k0, uint32_t k1) {
  const ob_u32x4 u = ob_philox(s, rep, 0u, OB_TAG_MMT, k0, k1);
  const double v = ((double)(u.x >> 5) * 67108864.0 + (double)(u.y >> 6)) * (1.0 / 9007199254740992.0);
  const double t = 0.01 + 0.98 * v;
  return t < 0.99 ? t : 0.98999999999999999;
}

OB_HD uint32_t ob_mm_pick(uint32_t i, uint32_t rep, uint32_t g, uint32_t n, uint32_t k0, uint32_t k1) {
  const uint32_t thresh = (0u - n) % n;
  for (uint32_t j = 0;; j += 4) {
    const ob_u32x4 u = ob_philox(i, rep, g, OB_TAG_MMR + (j >> 2), k0, k1);
    const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
    for (int h = 0; h < 4; ++h) {
      const uint64_t m = (uint64_t)wd[h] * n;
      if ((uint32_t)m >= thresh) return (uint32_t)(m >> 32);
    }
  }
}
