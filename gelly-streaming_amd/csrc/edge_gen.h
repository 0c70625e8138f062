/*
 * edge_gen.h — deterministic, counter-based synthetic edge streams for the CC benchmark configs.
 *
 * Every generator is a pure function of (params, edge index i), so any rank / GPU / host thread can
 * produce any contiguous slice of a stream with no communication, and the HIP generator kernel and
 * the host generator produce the same bytes (this header is compiled by both hipcc and gcc).
 *
 * Streams:
 *   GCC_GEN_EXAMPLE     ConnectedComponentsExample default data: edge i = (i+1, i+3), i in [0,100),
 *                       event time (i+1)*100 ms (reference: example/ConnectedComponentsExample.java:121-133)
 *   GCC_GEN_RMAT        R-MAT / Graph500-Kronecker, A,B,C,D = 0.57,0.19,0.19,0.05, seeded vertex permutation
 *   GCC_GEN_GNM         uniform G(n,m): endpoints iid uniform in [0,n)
 *   GCC_GEN_ADVERSARIAL shuffled random-permutation path over [0,2^P) + S stars of L ids over [2^P, 2^P+S*L)
 *
 * Edges are written as interleaved u32 pairs (src, dst) — the HBM edge-batch layout of the fold kernel.
 */
#ifndef GELLY_CC_EDGE_GEN_H
#define GELLY_CC_EDGE_GEN_H

#include <stdint.h>

#include "gelly_cc.h" /* gcc_gen_params, GCC_GEN_* */

#if defined(__HIPCC__)
#define GCC_HD __host__ __device__ static inline
#else
#define GCC_HD static inline
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* R-MAT quadrant thresholds as exact integers: floor(p * 2^32) of the cumulative probabilities. */
#define GCC_RMAT_T_A 2448131358u   /* 0.57 */
#define GCC_RMAT_T_AB 3264175144u  /* 0.76 */
#define GCC_RMAT_T_ABC 4080218931u /* 0.95 */

#define GCC_KEY_PERM 0x7065726D75746531ull /* "permute1" */
#define GCC_KEY_PATH 0x706174687065726Dull /* "pathperm" */
#define GCC_KEY_SHUF 0x73687566666C6531ull /* "shuffle1" */
#define GCC_KEY_DIR 0x6469726563746E31ull  /* "directn1" */

GCC_HD uint64_t gcc_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* high 64 bits of a*b, portable (no __int128 on the device side) */
GCC_HD uint64_t gcc_mulhi64(uint64_t a, uint64_t b) {
    uint64_t a_lo = (uint32_t)a, a_hi = a >> 32, b_lo = (uint32_t)b, b_hi = b >> 32;
    uint64_t p0 = a_lo * b_lo, p1 = a_lo * b_hi, p2 = a_hi * b_lo, p3 = a_hi * b_hi;
    uint64_t mid = (p0 >> 32) + (uint32_t)p1 + (uint32_t)p2;
    return p3 + (p1 >> 32) + (p2 >> 32) + (mid >> 32);
}

/* Seeded bijection on [0, 2^bits), bits in [1, 32]: three rounds of (odd multiply, add, xorshift). */
GCC_HD uint32_t gcc_perm_bits(uint64_t x, uint32_t bits, uint64_t key) {
    const uint64_t mask = (bits >= 64) ? ~0ull : ((1ull << bits) - 1ull);
    const uint32_t sh = (bits + 1u) / 2u;
    for (uint32_t r = 0; r < 3; ++r) {
        uint64_t km = gcc_splitmix64(key + 2u * r) | 1ull;
        uint64_t ka = gcc_splitmix64(key + 2u * r + 1u);
        x = (x * km) & mask;
        x = (x + ka) & mask;
        x ^= x >> sh;
    }
    return (uint32_t)x;
}

/* per-edge random base; draw k of edge i = splitmix64(base + k) */
GCC_HD uint64_t gcc_edge_base(uint64_t seed, uint64_t i) { return gcc_splitmix64(seed ^ gcc_splitmix64(i)); }

GCC_HD uint32_t gcc_ceil_log2(uint64_t n) {
    uint32_t b = 0;
    while (b < 63 && (1ull << b) < n) ++b;
    return b;
}

/* number of edges and id-range (V) each generator produces */
GCC_HD uint64_t gcc_gen_num_edges(const gcc_gen_params* p) {
    switch (p->kind) {
    case GCC_GEN_EXAMPLE: return 100;
    case GCC_GEN_RMAT:
    case GCC_GEN_GNM: return p->n_edges;
    case GCC_GEN_ADVERSARIAL:
        return ((1ull << p->scale) - 1ull) + (uint64_t)p->n_stars * (uint64_t)(p->star_size - 1u);
    default: return 0;
    }
}

GCC_HD uint64_t gcc_gen_num_vertices(const gcc_gen_params* p) {
    switch (p->kind) {
    case GCC_GEN_EXAMPLE: return 103; /* ids 1..102 (+ id 0 never seen) */
    case GCC_GEN_RMAT: return 1ull << p->scale;
    case GCC_GEN_GNM: return p->n_vertices;
    case GCC_GEN_ADVERSARIAL: return (1ull << p->scale) + (uint64_t)p->n_stars * p->star_size;
    default: return 0;
    }
}

/* event timestamp in ms of edge i (only EXAMPLE carries reference timestamps; others: 0) */
GCC_HD uint64_t gcc_gen_timestamp(const gcc_gen_params* p, uint64_t i) {
    return p->kind == GCC_GEN_EXAMPLE ? (i + 1u) * 100u : 0u;
}

GCC_HD void gcc_gen_edge(const gcc_gen_params* p, uint64_t i, uint32_t* u_out, uint32_t* v_out) {
    uint32_t u = 0, v = 0;
    switch (p->kind) {
    case GCC_GEN_EXAMPLE:
        u = (uint32_t)(i + 1u);
        v = (uint32_t)(i + 3u);
        break;
    case GCC_GEN_RMAT: {
        const uint64_t base = gcc_edge_base(p->seed, i);
        uint64_t r = 0;
        for (uint32_t lvl = 0; lvl < p->scale; ++lvl) {
            if ((lvl & 1u) == 0) r = gcc_splitmix64(base + (lvl >> 1));
            const uint32_t d = (uint32_t)(r >> (32u * (lvl & 1u)));
            uint32_t bu, bv;
            if (d < GCC_RMAT_T_A) { bu = 0; bv = 0; }
            else if (d < GCC_RMAT_T_AB) { bu = 0; bv = 1; }
            else if (d < GCC_RMAT_T_ABC) { bu = 1; bv = 0; }
            else { bu = 1; bv = 1; }
            u = (u << 1) | bu;
            v = (v << 1) | bv;
        }
        if (p->permute) {
            u = gcc_perm_bits(u, p->scale, p->seed ^ GCC_KEY_PERM);
            v = gcc_perm_bits(v, p->scale, p->seed ^ GCC_KEY_PERM);
        }
        break;
    }
    case GCC_GEN_GNM: {
        const uint64_t base = gcc_edge_base(p->seed, i);
        u = (uint32_t)gcc_mulhi64(gcc_splitmix64(base + 0u), p->n_vertices);
        v = (uint32_t)gcc_mulhi64(gcc_splitmix64(base + 1u), p->n_vertices);
        break;
    }
    case GCC_GEN_ADVERSARIAL: {
        const uint64_t E = gcc_gen_num_edges(p);
        const uint32_t dbits = gcc_ceil_log2(E);
        uint64_t j = gcc_perm_bits(i, dbits, p->seed ^ GCC_KEY_SHUF);
        while (j >= E) j = gcc_perm_bits(j, dbits, p->seed ^ GCC_KEY_SHUF); /* cycle walking */
        const uint64_t n_path = (1ull << p->scale) - 1ull;
        if (j < n_path) {
            u = gcc_perm_bits(j, p->scale, p->seed ^ GCC_KEY_PATH);
            v = gcc_perm_bits(j + 1u, p->scale, p->seed ^ GCC_KEY_PATH);
        } else {
            const uint64_t k = j - n_path;
            const uint64_t leaves = p->star_size - 1u;
            const uint64_t hub = (1ull << p->scale) + (k / leaves) * p->star_size;
            u = (uint32_t)hub;
            v = (uint32_t)(hub + 1u + (k % leaves));
        }
        if (gcc_splitmix64(p->seed ^ GCC_KEY_DIR ^ i) & 1ull) {
            uint32_t t = u; u = v; v = t;
        }
        break;
    }
    default: break;
    }
    *u_out = u;
    *v_out = v;
}

#ifdef __cplusplus
}
#endif

#endif /* GELLY_CC_EDGE_GEN_H */
