/*
 * fa_oracle.c -- scalar CPU restatement of the reference aggregation arithmetic.
 * TEST INFRASTRUCTURE ONLY (see fa_oracle.h for the citation map and rules).
 *
 * Built with -ffp-contract=off so that the only fused operations are the
 * explicit fmaf() calls of the FedAvg chain.
 */
#include "fa_oracle.h"

#include <math.h>
#include <pthread.h>
#include <string.h>

uint64_t fa_oracle_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

float fa_oracle_gen_value(uint64_t seed, uint32_t client, uint64_t idx) {
    uint64_t h = fa_oracle_splitmix64(seed ^ ((uint64_t)client << 40) ^ idx);
    uint32_t u24 = (uint32_t)(h >> 40);
    /* u24 * 2^-23 is exact and so is the subtraction: value in [-1, 1). */
    return (float)u24 * 0x1p-23f - 1.0f;
}

void fa_oracle_fill_f32(uint64_t seed, uint32_t client, uint64_t idx0, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = fa_oracle_gen_value(seed, client, idx0 + i);
}

void fa_oracle_gen_at(uint64_t seed, uint32_t client, const uint64_t* idx, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = fa_oracle_gen_value(seed, client, idx[i]);
}

uint16_t fa_oracle_f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u); /* quiet NaN */
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

float fa_oracle_bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

void fa_oracle_fill_bf16(uint64_t seed, uint32_t client, uint64_t idx0, size_t n, uint16_t* out) {
    for (size_t i = 0; i < n; ++i) out[i] = fa_oracle_f32_to_bf16(fa_oracle_gen_value(seed, client, idx0 + i));
}

void fa_oracle_weights(uint64_t seed, int n_clients, float* w) {
    double total = 0.0;
    for (int k = 0; k < n_clients; ++k) {
        uint64_t nk = 500u + fa_oracle_splitmix64(seed ^ ((uint64_t)k << 32)) % 1001u;
        w[k] = (float)nk; /* exact: nk <= 1500 */
        total += (double)nk;
    }
    for (int k = 0; k < n_clients; ++k) w[k] = (float)((double)w[k] / total);
}

/* ---- FedAvg chain: the per-element order is the client order; the loop nest is
 * client-outer so the compiler vectorises the element loop (same arithmetic). */

typedef struct {
    const void* const* x;
    const float* w;
    int n_clients;
    size_t lo, hi;
    const float* init;
    void* out;
    int in_bf16, out_bf16;
} chain_job;

enum { CHUNK = 4096 };

static void chain_range(const chain_job* j) {
    float acc[CHUNK];
    for (size_t b = j->lo; b < j->hi; b += CHUNK) {
        size_t m = (j->hi - b < CHUNK) ? (j->hi - b) : CHUNK;
        if (j->init) memcpy(acc, j->init + b, m * sizeof(float));
        else for (size_t i = 0; i < m; ++i) acc[i] = 0.0f;
        for (int k = 0; k < j->n_clients; ++k) {
            const float wk = j->w[k];
            if (j->in_bf16) {
                const uint16_t* xk = (const uint16_t*)j->x[k] + b;
                for (size_t i = 0; i < m; ++i) acc[i] = fmaf(fa_oracle_bf16_to_f32(xk[i]), wk, acc[i]);
            } else {
                const float* xk = (const float*)j->x[k] + b;
                for (size_t i = 0; i < m; ++i) acc[i] = fmaf(xk[i], wk, acc[i]);
            }
        }
        if (j->out_bf16) {
            uint16_t* o = (uint16_t*)j->out + b;
            for (size_t i = 0; i < m; ++i) o[i] = fa_oracle_f32_to_bf16(acc[i]);
        } else {
            memcpy((float*)j->out + b, acc, m * sizeof(float));
        }
    }
}

static void* chain_thread(void* p) {
    chain_range((const chain_job*)p);
    return NULL;
}

static void run_chain(const void* const* x, const float* w, int n_clients, size_t n, const float* init,
                      void* out, int in_bf16, int out_bf16, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((size_t)threads > n / CHUNK + 1) threads = (int)(n / CHUNK + 1);
    chain_job jobs[256];
    pthread_t tids[256];
    size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    per = (per + CHUNK - 1) / CHUNK * CHUNK;
    int launched = 0;
    for (int t = 0; t < threads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t] = (chain_job){x, w, n_clients, lo, hi, init, out, in_bf16, out_bf16};
        if (threads == 1) { chain_range(&jobs[t]); launched = 0; break; }
        pthread_create(&tids[t], NULL, chain_thread, &jobs[t]);
        ++launched;
    }
    for (int t = 0; t < launched; ++t) pthread_join(tids[t], NULL);
}

void fa_oracle_fedavg_f32(const float* const* x, const float* w, int n_clients, size_t n,
                          const float* init, float* out, int threads) {
    run_chain((const void* const*)x, w, n_clients, n, init, out, 0, 0, threads);
}

void fa_oracle_fedavg_bf16(const uint16_t* const* x, const float* w, int n_clients, size_t n,
                           const float* init, void* out, int out_bf16, int threads) {
    run_chain((const void* const*)x, w, n_clients, n, init, out, 1, out_bf16, threads);
}

/* aggregator.cpp:75-76: p = p + p (exact doubling unless it overflows), then a
 * correctly rounded division by kTrainSize_10 (libtorch div == '/' bit-for-bit). */
void fa_oracle_literal_f32(const float* x_last, size_t n, float divisor, float* out) {
    for (size_t i = 0; i < n; ++i) {
        float s = x_last[i] + x_last[i];
        out[i] = s / divisor;
    }
}

void fa_oracle_literal_bf16(const uint16_t* x_last, size_t n, float divisor, void* out, int out_bf16) {
    for (size_t i = 0; i < n; ++i) {
        float x = fa_oracle_bf16_to_f32(x_last[i]);
        float r = (x + x) / divisor;
        if (out_bf16) ((uint16_t*)out)[i] = fa_oracle_f32_to_bf16(r);
        else ((float*)out)[i] = r;
    }
}
