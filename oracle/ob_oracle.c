/*
 * ob_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference bootstrap path of dot-comma-hyphen/oaxaca-blinder-rs
 * (Rust crate `oaxaca_blinder`, read-only at /root/reference). It is the parity checker for
 * the HIP engine and the timed CPU baseline ("kind": "port") of bench.py. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (oaxaca-blinder-rs_amd/) never links or calls it.
 *
 * Parity pinning: the reference cannot be built here (no cargo/rustc), so this
 * restatement is pinned by the reference's own known-answer tests (tests/test_oracle_kat.py):
 *   ols.rs:151-209, decomposition.rs:129-184, inference.rs:40-57, normalization.rs:58-111,
 *   tests/integration_test.rs:105-163, tests/weights_test.rs, tests/null_handling_test.rs,
 *   tests/rif_test.rs, tests/optimize_budget_test.rs:34 (gap 16).
 * Bootstrap SE/CI/p values are unpinned by the reference (its resampling is unseeded,
 * builder.rs:822-827); they are defined here on the OBRS-1 index stream.
 *
 * Everything is f64 like the reference. Function-level citations are file:line under
 * /root/reference/oaxaca_blinder/src/.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* OBRS-1 resample stream (our spec; the reference uses polars' unseeded sample_n_literal,    */
/* builder.rs:822-827, i.e. n_g i.i.d. uniform draws with replacement per group).            */
/* ------------------------------------------------------------------------------------------ */
#define ORC_TILE 256u
#define ORC_TAG_L2 0x4F425232u /* "OBR2" */

/* Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants). */
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* floor(u * s / 2^64) for s < 2^32: a 64-bit uniform mapped onto [0, s). */
static inline uint32_t orc_mulhi64(uint64_t u, uint32_t s) {
    uint64_t hi = (u >> 32) * (uint64_t)s;
    uint64_t lo = ((u & 0xFFFFFFFFull) * (uint64_t)s) >> 32;
    return (uint32_t)((hi + lo) >> 32);
}

static inline uint64_t orc_draw_u64(const uint32_t w[4], int odd) {
    return odd ? (((uint64_t)w[3] << 32) | w[2]) : (((uint64_t)w[1] << 32) | w[0]);
}

/* Level 1 (OBRS-3): the tile counts m of n i.i.d. uniform row draws over [0, n),
 * drawn by binomial splitting instead of one index per draw. T = ceil(n / 256) tiles, D =
 * ceil(log2 T); the dyadic tree over 2^D tiles (rows [0, 2^(D+8))) has node (l, k) = tiles
 * [k 2^(D-l), (k+1) 2^(D-l)). A round with c_0 draws at the root splits every node (l < D) with
 * count c into its left child L ~ Binomial(c, 1/2) and its right child c - L (orc_split_left).
 * A child starting at tile >= T is padding: its draws are rejected. At the tiles, a partial last
 * tile (S = n - 256 (T-1) < 256 rows) accepts draw i iff byte (i & 3) of word ((i >> 2) & 3) of
 * Philox({i >> 4, rep, g, ORC_TAG_L1S + round}) is < S. Rejected draws R start the next round
 * while R > 2048; the last R <= 2048 (OBRS-2: 256) are direct: draw r is Lemire's
 * multiply-and-reject on word (j & 3) of Philox({r, rep, g, ORC_TAG_L1D + (j >> 2)}), attempt j.
 * Each split is an exact Binomial(c, 1/2), so the accepted draws are i.i.d. uniform over the valid
 * rows.
 *
 * The split (OBRS-2): a node with c < 4096 draws takes OBRS-1's popcount of c fair bits (bit b =
 * bit (b & 31) of word ((b >> 5) & 3) of Philox({b >> 7, rep, (k << 1) | g, ORC_TAG_L1T + rl}),
 * rl = (round << 5) + level). A node with c >= 4096 sums exact Binomial(2^j, 1/2) samples over
 * the binary digits of c -- c >> 12 samples of B(4096), one B(2^j) for each set bit j = 11 .. 7,
 * and the popcount of c & 127 fair bits. Each B(2^j) is a Knuth-Yao walk (discrete distribution
 * generating tree) over the exact dyadic probabilities C(2^j, k) / 2^(2^j): ~9 random bits per
 * sample instead of 2^j. Bits come from per-node streams: stream q has bit b = bit (b & 31) of
 * word ((b >> 5) & 3) of Philox({(q << 12) | (b >> 7), rep, (k << 1) | g, ORC_TAG_L1K + rl});
 * stream q < c >> 12 carries B(4096) sample q; the next streams carry one B(2^j) each, for the set
 * bits j = 11 down to 7 in that order; the last one, when c & 127 != 0, the c & 127 popcount bits.
 * One sample per stream, so the samples of a node are independent work items. (OBRS-1 used the popcount at every node: ~5.5M bits per group and
 * replicate at 500k rows, ~2.5M of them at nodes of 4096 draws or more.) */
#define ORC_TAG_L1T 0x4C310000u /* OBRS-1 "L1" + (round << 5) + level (superseded) */
#define ORC_TAG_L1K 0x4B310000u /* OBRS-2 "K1" + (round << 5) + level */
#define ORC_TAG_L1S 0x4C530000u /* "LS" + round */
#define ORC_TAG_L1D 0x4C440000u /* "LD" + (j >> 2) */
#define ORC_L1_DIRECT 2048u

/* Knuth-Yao tables for B(n, 1/2), n = 2^j: W_k = C(n, k), p_k = W_k / 2^n; column i (1..n) of the
 * DDG tree holds the k whose bit n - i of W_k is set, ascending: list[off[i] .. off[i+1]). */
typedef struct {
    uint32_t n;
    uint32_t* off; /* n + 2 entries */
    uint16_t* list;
} orc_ky;
static orc_ky orc_ky_tab[13];
static pthread_once_t orc_ky_once = PTHREAD_ONCE_INIT;

static void orc_ky_build(orc_ky* t, uint32_t n) {
    const uint32_t L = n / 64 + 1;
    uint64_t* w = (uint64_t*)calloc((size_t)(n + 1) * L, sizeof(uint64_t));
    w[0] = 1;
    for (uint32_t k = 0; k < n; ++k) { /* C(n, k+1) = C(n, k) (n - k) / (k + 1), exact */
        const uint64_t* a = w + (size_t)k * L;
        uint64_t* b = w + (size_t)(k + 1) * L;
        unsigned __int128 carry = 0;
        for (uint32_t i = 0; i < L; ++i) {
            unsigned __int128 v = (unsigned __int128)a[i] * (n - k) + carry;
            b[i] = (uint64_t)v;
            carry = v >> 64;
        }
        unsigned __int128 rem = 0;
        for (uint32_t i = L; i-- > 0;) {
            unsigned __int128 v = (rem << 64) | b[i];
            b[i] = (uint64_t)(v / (k + 1));
            rem = v % (k + 1);
        }
    }
    t->n = n;
    t->off = (uint32_t*)calloc(n + 2, sizeof(uint32_t));
    size_t total = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        t->off[i] = (uint32_t)total;
        const uint32_t bit = n - i;
        for (uint32_t k = 0; k <= n; ++k) total += (w[(size_t)k * L + bit / 64] >> (bit % 64)) & 1u;
    }
    t->off[n + 1] = (uint32_t)total;
    t->list = (uint16_t*)malloc(sizeof(uint16_t) * (total ? total : 1));
    size_t pos = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        const uint32_t bit = n - i;
        for (uint32_t k = 0; k <= n; ++k)
            if ((w[(size_t)k * L + bit / 64] >> (bit % 64)) & 1u) t->list[pos++] = (uint16_t)k;
    }
    free(w);
}

static void orc_ky_init(void) {
    for (uint32_t j = 7; j <= 12; ++j) orc_ky_build(&orc_ky_tab[j], 1u << j);
}

typedef struct {
    uint32_t ctr[4]; /* {(q << 12) | call, rep, c2, tag}; the call word is set per 128 bits */
    const uint32_t* key;
    uint64_t pos;
    uint32_t w[4];
} orc_bits;

static uint32_t orc_bit(orc_bits* s) {
    if ((s->pos & 127u) == 0) {
        uint32_t ctr[4] = {s->ctr[0] | (uint32_t)(s->pos >> 7), s->ctr[1], s->ctr[2], s->ctr[3]};
        orc_philox4x32_10(ctr, s->key, s->w);
    }
    const uint32_t b = (s->w[(s->pos >> 5) & 3u] >> (s->pos & 31u)) & 1u;
    ++s->pos;
    return b;
}

/* One B(2^j, 1/2) sample: the Knuth-Yao walk, one stream bit per tree level. */
static uint32_t orc_ky_sample(orc_bits* s, const orc_ky* t) {
    uint64_t d = 0;
    for (uint32_t i = 1;; ++i) {
        d = 2 * d + orc_bit(s);
        const uint32_t cnt = t->off[i + 1] - t->off[i];
        if (d < cnt) return t->list[t->off[i] + d];
        d -= cnt;
    }
}

/* Binomial(c, 1/2) for node k of a level, group g; rl = (round << 5) + level (OBRS-2, above). */
#define ORC_KY_MIN_C 4096u
static uint32_t orc_split_left(uint32_t c, uint32_t rep, uint32_t g, uint32_t k, uint32_t rl, const uint32_t key[2]) {
    const uint32_t c2 = (k << 1) | g;
    uint32_t left = 0;
    if (c < ORC_KY_MIN_C) { /* OBRS-1: the popcount of c fair bits, 128 per Philox call */
        for (uint32_t q = 0; 128u * q < c; ++q) {
            uint32_t ctr[4] = {q, rep, c2, ORC_TAG_L1T + rl}, w[4];
            orc_philox4x32_10(ctr, key, w);
            uint32_t r = c - 128u * q;
            for (uint32_t i = 0; i < 4; ++i) {
                uint32_t nb = r > 32u * i ? r - 32u * i : 0u;
                uint32_t mask = nb >= 32u ? 0xFFFFFFFFu : ((1u << nb) - 1u);
                left += (uint32_t)__builtin_popcount(w[i] & mask);
            }
        }
        return left;
    }
    pthread_once(&orc_ky_once, orc_ky_init);
    uint32_t q = 0;
    for (; q < (c >> 12); ++q) { /* one B(4096) sample per stream */
        orc_bits s = {{q << 12, rep, c2, ORC_TAG_L1K + rl}, key, 0, {0, 0, 0, 0}};
        left += orc_ky_sample(&s, &orc_ky_tab[12]);
    }
    for (uint32_t j = 11; j >= 7; --j) /* then one stream per set bit j of c, high to low */
        if ((c >> j) & 1u) {
            orc_bits s = {{q++ << 12, rep, c2, ORC_TAG_L1K + rl}, key, 0, {0, 0, 0, 0}};
            left += orc_ky_sample(&s, &orc_ky_tab[j]);
        }
    if (c & 127u) { /* and the popcount of c & 127 fair bits */
        orc_bits s = {{q << 12, rep, c2, ORC_TAG_L1K + rl}, key, 0, {0, 0, 0, 0}};
        for (uint32_t i = 0; i < (c & 127u); ++i) left += orc_bit(&s);
    }
    return left;
}

/* Test hook: one OBRS-2 split of c draws (node k, rl = (round << 5) + level). */
uint32_t orc_binomial_half(uint32_t c, uint64_t seed, uint32_t rep, uint32_t g, uint32_t k, uint32_t rl) {
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    return orc_split_left(c, rep, g, k, rl, key);
}

void orc_level1_counts(uint64_t seed, uint32_t rep, uint32_t g, uint32_t n, uint32_t* m) {
    uint32_t ntiles = (n + ORC_TILE - 1) / ORC_TILE;
    if (ntiles == 0) return;
    memset(m, 0, sizeof(uint32_t) * ntiles);
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t depth = 0;
    while ((1u << depth) < ntiles) ++depth;
    const uint32_t tail = n - (ntiles - 1) * ORC_TILE; /* rows of the last tile */
    uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * ntiles);
    uint32_t* nxt = (uint32_t*)malloc(sizeof(uint32_t) * ntiles);
    uint32_t todo = n;
    for (uint32_t round = 0; round == 0 || todo > ORC_L1_DIRECT; ++round) {
        uint32_t rejected = 0, nodes = 1;
        cur[0] = todo;
        for (uint32_t l = 0; l < depth; ++l) {
            uint32_t span = 1u << (depth - l - 1); /* tiles per child */
            uint32_t nnext = (ntiles + span - 1) / span;
            for (uint32_t k = 0; k < nodes; ++k) {
                uint32_t c = cur[k], left = c ? orc_split_left(c, rep, g, k, (round << 5) + l, key) : 0;
                nxt[2 * k] = left;
                if (2 * k + 1 < nnext) nxt[2 * k + 1] = c - left;
                else rejected += c - left;
            }
            nodes = nnext;
            uint32_t* t = cur; cur = nxt; nxt = t;
        }
        for (uint32_t t = 0; t < ntiles; ++t) {
            uint32_t c = cur[t];
            if (t == ntiles - 1 && tail < ORC_TILE) {
                uint32_t acc = 0;
                for (uint32_t q = 0; 16u * q < c; ++q) {
                    uint32_t ctr[4] = {q, rep, g, ORC_TAG_L1S + round}, w[4];
                    orc_philox4x32_10(ctr, key, w);
                    for (uint32_t i = 0; i < 16 && 16u * q + i < c; ++i)
                        acc += ((w[i >> 2] >> (8u * (i & 3u))) & 0xFFu) < tail;
                }
                rejected += c - acc;
                c = acc;
            }
            m[t] += c;
        }
        todo = rejected;
    }
    const uint32_t thresh = (0u - n) % n;
    for (uint32_t r = 0; r < todo; ++r) {
        uint64_t x = 0;
        for (uint32_t j = 0;; ++j) {
            uint32_t ctr[4] = {r, rep, g, ORC_TAG_L1D + (j >> 2)}, w[4];
            orc_philox4x32_10(ctr, key, w);
            x = (uint64_t)w[j & 3] * n;
            if ((uint32_t)x >= thresh) break;
        }
        m[(uint32_t)(x >> 32) / ORC_TILE]++;
    }
    free(cur);
    free(nxt);
}

/* Full OBRS-1 index list for (seed, rep, group): tiles ascending, draws in q order. */
void orc_resample_indices(uint64_t seed, uint32_t rep, uint32_t g, uint32_t n, uint32_t* idx_out) {
    uint32_t ntiles = (n + ORC_TILE - 1) / ORC_TILE;
    uint32_t* m = (uint32_t*)malloc(sizeof(uint32_t) * (ntiles ? ntiles : 1));
    orc_level1_counts(seed, rep, g, n, m);
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    size_t pos = 0;
    for (uint32_t j = 0; j < ntiles; ++j) {
        uint32_t base = j * ORC_TILE;
        uint32_t s = (n - base < ORC_TILE) ? (n - base) : ORC_TILE;
        if (s == ORC_TILE) { /* full tile: 16 exact 8-bit draws per Philox call,
                                 draw 16p + 4i + b = byte b (LSB first) of word i */
            for (uint32_t p = 0; 16u * p < m[j]; ++p) {
                uint32_t ctr[4] = {p, rep, (j << 1) | g, ORC_TAG_L2}, w[4];
                orc_philox4x32_10(ctr, key, w);
                for (uint32_t d = 0; d < 16 && 16u * p + d < m[j]; ++d)
                    idx_out[pos++] = base + ((w[d >> 2] >> (8u * (d & 3u))) & 0xFFu);
            }
        } else { /* partial tile: 2 draws per call, 64-bit uniform mapped onto [0, s) */
            for (uint32_t p = 0; 2u * p < m[j]; ++p) {
                uint32_t ctr[4] = {p, rep, (j << 1) | g, ORC_TAG_L2}, w[4];
                orc_philox4x32_10(ctr, key, w);
                for (int h = 0; h < 2; ++h) {
                    uint32_t q = 2u * p + (uint32_t)h;
                    if (q >= m[j]) break;
                    idx_out[pos++] = base + orc_mulhi64(orc_draw_u64(w, h), s);
                }
            }
        }
    }
    free(m);
}

/* ------------------------------------------------------------------------------------------ */
/* OLS / WLS exactly as math/ols.rs:44-144 (nalgebra 0.32 Cholesky operation order).          */
/* X is column-major n x k (nalgebra storage, builder.rs:373).                                */
/* ------------------------------------------------------------------------------------------ */
enum { ORC_OK = 0, ORC_E_INSUFFICIENT = 1, ORC_E_CHOLESKY = 2, ORC_E_NEGWEIGHT = 3, ORC_E_GROUP = 4 };

/* nalgebra Cholesky::new (left-looking, column axpy): fails iff a pivot is 0, negative or NaN.
 * a: k x k column-major, lower triangle read; overwritten by L. */
static int orc_cholesky(double* a, int k) {
    for (int j = 0; j < k; ++j) {
        for (int c = 0; c < j; ++c) {
            double factor = -a[j + (size_t)c * k];
            for (int i = j; i < k; ++i) a[i + (size_t)j * k] += factor * a[i + (size_t)c * k];
        }
        double diag = a[j + (size_t)j * k];
        if (!(diag != 0.0 && diag >= 0.0)) return ORC_E_CHOLESKY; /* !is_zero && try_sqrt */
        double denom = sqrt(diag);
        a[j + (size_t)j * k] = denom;
        for (int i = j + 1; i < k; ++i) a[i + (size_t)j * k] /= denom;
    }
    return ORC_OK;
}

/* Cholesky::solve_mut: L y = b (column axpy form), then L^T x = y (dot form). */
static void orc_chol_solve(const double* l, int k, double* b) {
    for (int i = 0; i < k; ++i) {
        double coeff = b[i] / l[i + (size_t)i * k];
        b[i] = coeff;
        for (int r = i + 1; r < k; ++r) b[r] -= coeff * l[r + (size_t)i * k];
    }
    for (int i = k - 1; i >= 0; --i) {
        double dot = 0.0;
        for (int r = i + 1; r < k; ++r) dot += l[r + (size_t)i * k] * b[r];
        b[i] = (b[i] - dot) / l[i + (size_t)i * k];
    }
}

/* ols.rs:44-144. full != 0 also computes residuals/sigma^2/inverse like the reference
 * (bootstrap replicates never read them, but the reference pays for them; ref-cpu keeps them). */
int orc_ols(const double* y, const double* x, int64_t n, int k, const double* w,
            double* beta, double* resid_out, int full) {
    if (w) {
        for (int64_t i = 0; i < n; ++i)
            if (w[i] < 0.0) return ORC_E_NEGWEIGHT; /* ols.rs:60-66 */
    }
    double* xtx = (double*)calloc((size_t)k * k, sizeof(double));
    double* xty = (double*)calloc((size_t)k, sizeof(double));
    const double* xs = x;
    const double* ys = y;
    double* xw = NULL;
    double* yw = NULL;
    if (w) { /* ols.rs:68-78: scale rows by sqrt(w) */
        xw = (double*)malloc(sizeof(double) * (size_t)n * k);
        yw = (double*)malloc(sizeof(double) * (size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            double s = sqrt(w[i]);
            yw[i] = y[i] * s;
            for (int c = 0; c < k; ++c) xw[i + (size_t)c * n] = x[i + (size_t)c * n] * s;
        }
        xs = xw;
        ys = yw;
    }
    /* ols.rs:80-81 / 88-89: X^T X and X^T y (full matrix, as the gemm computes it) */
    for (int a = 0; a < k; ++a) {
        const double* ca = xs + (size_t)a * n;
        for (int b = 0; b < k; ++b) {
            const double* cb = xs + (size_t)b * n;
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += ca[i] * cb[i];
            xtx[a + (size_t)b * k] = s;
        }
        double s = 0.0;
        for (int64_t i = 0; i < n; ++i) s += ca[i] * ys[i];
        xty[a] = s;
    }
    int rc = ORC_OK;
    if ((double)n <= (double)k) rc = ORC_E_INSUFFICIENT; /* ols.rs:98-105 (row count) */
    if (rc == ORC_OK) rc = orc_cholesky(xtx, k);        /* ols.rs:107-111 */
    if (rc == ORC_OK) {
        memcpy(beta, xty, sizeof(double) * (size_t)k); /* ols.rs:115 */
        orc_chol_solve(xtx, k, beta);
        if (full || resid_out) { /* ols.rs:118-137 */
            double sse = 0.0;
            for (int64_t i = 0; i < n; ++i) {
                double yh = 0.0;
                for (int c = 0; c < k; ++c) yh += x[i + (size_t)c * n] * beta[c];
                double e = y[i] - yh;
                if (resid_out) resid_out[i] = e;
                sse += w ? e * (w[i] * e) : e * e;
            }
            double sigma2 = sse / ((double)n - (double)k);
            if (full) {
                double* inv = (double*)calloc((size_t)k * k, sizeof(double));
                for (int c = 0; c < k; ++c) {
                    inv[c + (size_t)c * k] = 1.0;
                    orc_chol_solve(xtx, k, inv + (size_t)c * k);
                }
                volatile double sink = 0.0;
                for (int c = 0; c < k * k; ++c) sink += inv[c] * sigma2;
                (void)sink;
                free(inv);
            }
        }
    }
    free(xtx);
    free(xty);
    free(xw);
    free(yw);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* One decomposition pass (builder.rs:420-699 + estimation.rs:51-111) on prepared matrices.   */
/* ------------------------------------------------------------------------------------------ */
enum { ORC_REF_A = 0, ORC_REF_B = 1, ORC_REF_POOLED = 2, ORC_REF_WEIGHTED = 3 };

typedef struct {
    int k;             /* columns incl. intercept: [intercept, predictors..., dummies...] */
    int pool_pos;      /* 1 + numeric predictors: the pooled group indicator's column */
    int ref_mode;
    int weighted;
    int n_norm;            /* .normalize() vars, in call order (builder.rs:213-220) */
    const int* norm_start; /* per var: offset into norm_idx (length n_norm + 1) */
    const int* norm_idx;   /* columns whose name starts with "{var}_" (normalization.rs:11-16) */
    const int* norm_m;     /* category_counts[var], or -1: matches + 1 (normalization.rs:28-31) */
    const int* pooled_start; /* the same lists on the pooled name list (builder.rs:572-578) */
    const int* pooled_idx;
    const int* has_base;   /* var is a categorical predictor with a base level (builder.rs:636-640) */
} orc_cfg;

int orc_n_base(const orc_cfg* c) {
    int nb = 0;
    for (int v = 0; v < c->n_norm; ++v) nb += c->has_base[v] != 0;
    return nb;
}

/* normalization.rs:5-51 on beta (k entries); returns base coefficient per var. */
static void orc_normalize(double* beta, const orc_cfg* c, const int* starts, const int* idx_lists,
                          double* base) {
    for (int v = 0; v < c->n_norm; ++v) {
        int s = starts[v], e = starts[v + 1];
        base[v] = 0.0;
        if (e == s) continue;
        double sum = 0.0;
        for (int t = s; t < e; ++t) sum += beta[idx_lists[t]];
        int m = c->norm_m[v] >= 0 ? c->norm_m[v] : (e - s) + 1;
        if (m == 0) continue;
        double mean = sum / (double)m;
        base[v] = -mean;
        beta[0] += mean;
        for (int t = s; t < e; ++t) beta[idx_lists[t]] -= mean;
    }
}

static void orc_means(const double* x, int64_t n, int k, const double* w, double* out) {
    if (w) { /* estimation.rs:57-64 */
        double tw = 0.0;
        for (int64_t i = 0; i < n; ++i) tw += w[i];
        for (int c = 0; c < k; ++c) {
            double d = 0.0;
            for (int64_t i = 0; i < n; ++i) d += x[i + (size_t)c * n] * w[i];
            out[c] = d / tw;
        }
    } else { /* row_mean */
        for (int c = 0; c < k; ++c) {
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += x[i + (size_t)c * n];
            out[c] = s / (double)n;
        }
    }
}

/* Row layout shared with the engine (include/oaxaca_boot.h, OB_ROW_*):
 * [0] explained [1] unexplained [2] endowments [3] coefficients [4] interaction [5] total_gap
 * [6, 6+Kd) detailed explained, [6+Kd, 6+2Kd) detailed unexplained (Kd = k + n_norm),
 * then beta_a[k], beta_b[k], xa_mean[k], xb_mean[k], beta_star[k]. */
int orc_row_len(int k, int n_base) { return 6 + 2 * (k + n_base) + 5 * k; }

/* xa/xb: column-major n x k with the intercept column; ya/yb; wa/wb optional. */
int orc_single_pass(const orc_cfg* c, const double* xa, const double* ya, const double* wa, int64_t na,
                    const double* xb, const double* yb, const double* wb, int64_t nb, double* row,
                    double* resid_b, int full) {
    const int k = c->k;
    double* beta_a = (double*)malloc(sizeof(double) * k);
    double* beta_b = (double*)malloc(sizeof(double) * k);
    double* xam = (double*)malloc(sizeof(double) * k);
    double* xbm = (double*)malloc(sizeof(double) * k);
    double* bstar = (double*)malloc(sizeof(double) * (k + 1));
    double base_a[64], base_b[64], base_s[64];
    int rc = ORC_OK;
    if (c->n_norm > 64) return ORC_E_GROUP;
    if (na == 0 || nb == 0) { rc = ORC_E_GROUP; goto done; } /* builder.rs:431-435 */
    rc = orc_ols(ya, xa, na, k, c->weighted ? wa : NULL, beta_a, NULL, full);
    if (rc) goto done;
    rc = orc_ols(yb, xb, nb, k, c->weighted ? wb : NULL, beta_b, resid_b, full);
    if (rc) goto done;
    orc_means(xa, na, k, c->weighted ? wa : NULL, xam);
    orc_means(xb, nb, k, c->weighted ? wb : NULL, xbm);
    for (int v = 0; v < c->n_norm; ++v) base_a[v] = base_b[v] = base_s[v] = 0.0;
    if (c->n_norm) { /* estimation.rs:76-91 */
        orc_normalize(beta_a, c, c->norm_start, c->norm_idx, base_a);
        orc_normalize(beta_b, c, c->norm_start, c->norm_idx, base_b);
    }
    switch (c->ref_mode) { /* builder.rs:536-621 */
    case ORC_REF_A:
        memcpy(bstar, beta_a, sizeof(double) * k);
        memcpy(base_s, base_a, sizeof(double) * c->n_norm);
        break;
    case ORC_REF_B:
        memcpy(bstar, beta_b, sizeof(double) * k);
        memcpy(base_s, base_b, sizeof(double) * c->n_norm);
        break;
    case ORC_REF_POOLED: {
        /* vstack(A, B) with __ob_group_indicator__ = 1[A] inserted after the numeric predictors */
        int kp = k + 1;
        int64_t np = na + nb;
        double* xp = (double*)malloc(sizeof(double) * (size_t)np * kp);
        double* yp = (double*)malloc(sizeof(double) * (size_t)np);
        double* wp = c->weighted ? (double*)malloc(sizeof(double) * (size_t)np) : NULL;
        for (int cc = 0, src = 0; cc < kp; ++cc) {
            double* dst = xp + (size_t)cc * np;
            if (cc == c->pool_pos) {
                for (int64_t i = 0; i < na; ++i) dst[i] = 1.0;
                for (int64_t i = 0; i < nb; ++i) dst[na + i] = 0.0;
                continue;
            }
            memcpy(dst, xa + (size_t)src * na, sizeof(double) * na);
            memcpy(dst + na, xb + (size_t)src * nb, sizeof(double) * nb);
            ++src;
        }
        memcpy(yp, ya, sizeof(double) * na);
        memcpy(yp + na, yb, sizeof(double) * nb);
        if (wp) {
            memcpy(wp, wa, sizeof(double) * na);
            memcpy(wp + na, wb, sizeof(double) * nb);
        }
        double* bp = (double*)malloc(sizeof(double) * kp);
        rc = orc_ols(yp, xp, np, kp, wp, bp, NULL, full);
        if (!rc && c->n_norm) orc_normalize(bp, c, c->pooled_start, c->pooled_idx, base_s);
        for (int cc = 0, dst = 0; cc < kp && !rc; ++cc) /* remove_row(indicator) */
            if (cc != c->pool_pos) bstar[dst++] = bp[cc];
        free(xp); free(yp); free(wp); free(bp);
        if (rc) goto done;
        break;
    }
    case ORC_REF_WEIGHTED: {
        double sa = 0.0, sb = 0.0;
        if (c->weighted) {
            for (int64_t i = 0; i < na; ++i) sa += wa[i];
            for (int64_t i = 0; i < nb; ++i) sb += wb[i];
        } else {
            sa = (double)na;
            sb = (double)nb;
        }
        double tot = sa + sb;
        if (tot == 0.0) { rc = ORC_E_GROUP; goto done; }
        double wA = sa / tot, wB = 1.0 - wA;
        for (int v = 0; v < c->n_norm; ++v) base_s[v] = base_a[v] * wA + base_b[v] * wB;
        for (int j = 0; j < k; ++j) bstar[j] = beta_a[j] * wA + beta_b[j] * wB;
        break;
    }
    default: rc = ORC_E_GROUP; goto done;
    }
    {
        const int kd = k + orc_n_base(c);
        double* dex = row + 6;
        double* dun = row + 6 + kd;
        /* decomposition.rs:56-89 */
        double expl = 0.0, gap2 = 0.0, endow = 0.0, coef = 0.0, inter = 0.0;
        double ta = 0.0, tb = 0.0;
        for (int j = 0; j < k; ++j) {
            double dx = xam[j] - xbm[j], db = beta_a[j] - beta_b[j];
            expl += dx * bstar[j];
            ta += xam[j] * beta_a[j];
            tb += xbm[j] * beta_b[j];
            endow += dx * beta_b[j];
            coef += xbm[j] * db;
            inter += dx * db;
        }
        gap2 = ta - tb;
        double unexpl = gap2 - expl;
        /* decomposition.rs:92-122 */
        for (int j = 0; j < k; ++j) {
            dex[j] = (xam[j] - xbm[j]) * bstar[j];
            dun[j] = xam[j] * (beta_a[j] - bstar[j]) + xbm[j] * (bstar[j] - beta_b[j]);
        }
        /* builder.rs:634-674 base-category terms */
        for (int v = 0, bi = 0; v < c->n_norm; ++v) {
            if (!c->has_base[v]) continue;
            double sa = 0.0, sb = 0.0;
            for (int t = c->norm_start[v]; t < c->norm_start[v + 1]; ++t) {
                sa += xam[c->norm_idx[t]];
                sb += xbm[c->norm_idx[t]];
            }
            double xa0 = 1.0 - sa, xb0 = 1.0 - sb;
            double cu = xa0 * (base_a[v] - base_s[v]) + xb0 * (base_s[v] - base_b[v]);
            double ce = (xa0 - xb0) * base_s[v];
            dun[k + bi] = cu;
            dex[k + bi] = ce;
            ++bi;
            expl += ce;
            unexpl += cu;
        }
        /* builder.rs:676-684 */
        double ma = 0.0, mb = 0.0;
        if (c->weighted) {
            double swa = 0.0, swb = 0.0;
            for (int64_t i = 0; i < na; ++i) { ma += ya[i] * wa[i]; swa += wa[i]; }
            for (int64_t i = 0; i < nb; ++i) { mb += yb[i] * wb[i]; swb += wb[i]; }
            ma /= swa;
            mb /= swb;
        } else {
            for (int64_t i = 0; i < na; ++i) ma += ya[i];
            for (int64_t i = 0; i < nb; ++i) mb += yb[i];
            ma /= (double)na;
            mb /= (double)nb;
        }
        row[0] = expl;
        row[1] = unexpl;
        row[2] = endow;
        row[3] = coef;
        row[4] = inter;
        row[5] = ma - mb;
        double* tail = row + 6 + 2 * kd;
        memcpy(tail, beta_a, sizeof(double) * k);
        memcpy(tail + k, beta_b, sizeof(double) * k);
        memcpy(tail + 2 * k, xam, sizeof(double) * k);
        memcpy(tail + 3 * k, xbm, sizeof(double) * k);
        memcpy(tail + 4 * k, bstar, sizeof(double) * k);
    }
done:
    free(beta_a); free(beta_b); free(xam); free(xbm); free(bstar);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* Bootstrap driver, reference algorithm (builder.rs:816-839): per replicate resample both    */
/* groups (OBRS-1 indices instead of polars), gather every column, re-run the single pass.    */
/* Multithreaded over replicates like the Rayon pool.                                         */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_cfg* cfg;
    const double *xa, *ya, *wa, *xb, *yb, *wb; /* column-major incl. intercept column */
    int64_t na, nb;
    uint64_t seed;
    uint32_t first_rep;
    uint32_t n_reps;
    int full;
    double* rows;
    uint8_t* ok;
    int nthreads, tid;
} orc_boot_job;

static void orc_gather(const double* x, const double* y, const double* w, int64_t n, int k,
                       const uint32_t* idx, double* xs, double* ys, double* ws) {
    for (int c = 0; c < k; ++c) {
        const double* src = x + (size_t)c * n;
        double* dst = xs + (size_t)c * n;
        for (int64_t i = 0; i < n; ++i) dst[i] = src[idx[i]];
    }
    for (int64_t i = 0; i < n; ++i) ys[i] = y[idx[i]];
    if (w)
        for (int64_t i = 0; i < n; ++i) ws[i] = w[idx[i]];
}

static void* orc_boot_worker(void* arg) {
    orc_boot_job* j = (orc_boot_job*)arg;
    const int k = j->cfg->k;
    int rl = orc_row_len(k, orc_n_base(j->cfg));
    uint32_t* ia = (uint32_t*)malloc(sizeof(uint32_t) * (j->na ? j->na : 1));
    uint32_t* ib = (uint32_t*)malloc(sizeof(uint32_t) * (j->nb ? j->nb : 1));
    double* xas = (double*)malloc(sizeof(double) * (size_t)j->na * k);
    double* xbs = (double*)malloc(sizeof(double) * (size_t)j->nb * k);
    double* yas = (double*)malloc(sizeof(double) * j->na);
    double* ybs = (double*)malloc(sizeof(double) * j->nb);
    double* was = j->wa ? (double*)malloc(sizeof(double) * j->na) : NULL;
    double* wbs = j->wb ? (double*)malloc(sizeof(double) * j->nb) : NULL;
    for (uint32_t r = (uint32_t)j->tid; r < j->n_reps; r += (uint32_t)j->nthreads) {
        uint32_t rep = j->first_rep + r;
        orc_resample_indices(j->seed, rep, 0, (uint32_t)j->na, ia);
        orc_resample_indices(j->seed, rep, 1, (uint32_t)j->nb, ib);
        orc_gather(j->xa, j->ya, j->wa, j->na, k, ia, xas, yas, was);
        orc_gather(j->xb, j->yb, j->wb, j->nb, k, ib, xbs, ybs, wbs);
        double* row = j->rows + (size_t)r * rl;
        int rc = orc_single_pass(j->cfg, xas, yas, was, j->na, xbs, ybs, wbs, j->nb, row, NULL, j->full);
        j->ok[r] = (rc == ORC_OK);
        if (rc) for (int t = 0; t < rl; ++t) row[t] = NAN;
    }
    free(ia); free(ib); free(xas); free(xbs); free(yas); free(ybs); free(was); free(wbs);
    return NULL;
}

void orc_boot_ref(const orc_cfg* cfg, const double* xa, const double* ya, const double* wa, int64_t na,
                  const double* xb, const double* yb, const double* wb, int64_t nb, uint64_t seed,
                  uint32_t first_rep, uint32_t n_reps, int full, int nthreads, double* rows, uint8_t* ok) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    orc_boot_job* jobs = (orc_boot_job*)malloc(sizeof(orc_boot_job) * nthreads);
    for (int t = 0; t < nthreads; ++t) {
        orc_boot_job j = {cfg, xa, ya, wa, xb, yb, wb, na, nb, seed, first_rep, n_reps, full, rows, ok, nthreads, t};
        jobs[t] = j;
        pthread_create(&th[t], NULL, orc_boot_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* ------------------------------------------------------------------------------------------ */
/* inference.rs:4-34                                                                          */
/* ------------------------------------------------------------------------------------------ */
static int orc_cmp(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/* out: std_err, p_value, ci_lower, ci_upper */
void orc_bootstrap_stats(const double* v, int64_t n, double* out) {
    if (n == 0) { out[0] = out[1] = out[2] = out[3] = NAN; return; }
    double nf = (double)n, mean = 0.0, ss = 0.0;
    for (int64_t i = 0; i < n; ++i) mean += v[i];
    mean /= nf;
    for (int64_t i = 0; i < n; ++i) ss += (v[i] - mean) * (v[i] - mean);
    out[0] = sqrt(ss / (nf - 1.0));
    int64_t pos = 0, neg = 0;
    for (int64_t i = 0; i < n; ++i) { pos += v[i] >= 0.0; neg += v[i] <= 0.0; }
    double pp = (double)pos / nf, pn = (double)neg / nf;
    double p = 2.0 * (pp < pn ? pp : pn);
    out[1] = p < 1.0 ? p : 1.0;
    double* s = (double*)malloc(sizeof(double) * n);
    memcpy(s, v, sizeof(double) * n);
    qsort(s, (size_t)n, sizeof(double), orc_cmp);
    int64_t lo = (int64_t)floor(0.025 * nf);
    int64_t hi = (int64_t)floor(0.975 * nf);
    if (hi > n - 1) hi = n - 1;
    out[2] = lo < n ? s[lo] : NAN;
    out[3] = s[hi];
    free(s);
}

/* ------------------------------------------------------------------------------------------ */
/* math/rif.rs:14-88                                                                          */
/* ------------------------------------------------------------------------------------------ */
void orc_rif(const double* y, int64_t n, double tau, double* out) {
    if (n < 2) { memcpy(out, y, sizeof(double) * (n > 0 ? n : 0)); return; }
    double nf = (double)n;
    double* s = (double*)malloc(sizeof(double) * n);
    memcpy(s, y, sizeof(double) * n);
    qsort(s, (size_t)n, sizeof(double), orc_cmp);
    double h = (nf - 1.0) * tau, hf = floor(h), hc = ceil(h), frac = h - hf;
    double q = (hf == hc) ? s[(int64_t)hf] : s[(int64_t)hf] + frac * (s[(int64_t)hc] - s[(int64_t)hf]);
    double mean = 0.0;
    for (int64_t i = 0; i < n; ++i) mean += y[i];
    mean /= nf;
    double var = 0.0;
    for (int64_t i = 0; i < n; ++i) var += (y[i] - mean) * (y[i] - mean);
    var /= (nf - 1.0);
    double sd = sqrt(var);
    int64_t i75 = (int64_t)ceil(0.75 * nf); i75 = i75 == 0 ? 0 : i75 - 1;
    int64_t i25 = (int64_t)ceil(0.25 * nf); i25 = i25 == 0 ? 0 : i25 - 1;
    if (i75 > n - 1) i75 = n - 1;
    if (i25 > n - 1) i25 = n - 1;
    double iqr = s[i75] - s[i25];
    double spread = (iqr > 1e-8) ? fmin(sd, iqr / 1.34) : sd;
    if (spread < 1e-8) spread = 1.0;
    double bw = 0.9 * spread * pow(nf, -0.2);
    const double c = 1.0 / sqrt(2.0 * 3.14159265358979323846);
    double dens = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double u = (q - y[i]) / bw;
        dens += c * exp(-0.5 * (u * u));
    }
    dens /= (nf * bw);
    if (dens < 1e-8) dens = 1e-8;
    for (int64_t i = 0; i < n; ++i) out[i] = q + (tau - (y[i] <= q ? 1.0 : 0.0)) / dens;
    free(s);
}
