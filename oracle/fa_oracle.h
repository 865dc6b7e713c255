/*
 * fa_oracle.h -- CPU restatement of the reference aggregator's reduction.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so.  The product path
 * (libfa.so) never links, calls or falls back to anything in oracle/.
 *
 * What is restated (paths relative to the reference repo root):
 *   - pipeline_simulation/aggregator.cpp:63-88 (and :117-142): per receipt the
 *     module is overwritten by torch::load and every parameter p becomes
 *     fl(fl(p + p) / kTrainSize_10) with kTrainSize_10 = 1000 (:48).  Because
 *     parts and parts_ alias the same modules (systemAPI.cpp:34-37) the value
 *     after D receipts is fl(fl(x_last + x_last) / 1000): fa_oracle_literal_*.
 *   - The intended FedAvg (north star; EdgeSys.pdf Eq. 5-6): out = sum_k w_k x_k
 *     accumulated in client order as libtorch `acc.add_(x_k, w_k)` does on an
 *     FMA host, i.e. an ordered fmaf chain per element: fa_oracle_fedavg_*.
 *   - bf16 variant: bf16 -> f32 exactly, same fp32 chain, round-to-nearest-even
 *     at the end (the libtorch restatement `acc(fp32).add_(x.float(), w)` then
 *     `.to(bf16)`).
 *
 * Parity pin: tests/golden/ holds vectors produced by oracle/_ref/ref_harness,
 * a harness linking the reference's own model builders (models/{resnet,vgg,lenet5}) and
 * libtorch ops (tools/gen_golden.py); tests/test_oracle.py checks this file
 * against them bit-for-bit.
 */
#ifndef FA_ORACLE_H_
#define FA_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Counter-based synthetic input generator shared by oracle, HIP fill kernel
 * and benches: element i of client k = uniform[-1,1) from
 * splitmix64(seed ^ k<<40 ^ i), top 24 bits, exact in fp32. */
uint64_t fa_oracle_splitmix64(uint64_t z);
float fa_oracle_gen_value(uint64_t seed, uint32_t client, uint64_t idx);
void fa_oracle_fill_f32(uint64_t seed, uint32_t client, uint64_t idx0, size_t n, float* out);
void fa_oracle_fill_bf16(uint64_t seed, uint32_t client, uint64_t idx0, size_t n, uint16_t* out);
/* The generator at n arbitrary indices (sampled parity checks at full size). */
void fa_oracle_gen_at(uint64_t seed, uint32_t client, const uint64_t* idx, size_t n, float* out);
/* FedAvg weights w_k = n_k / sum(n), n_k uniform in [500,1500]. */
void fa_oracle_weights(uint64_t seed, int n_clients, float* w);

uint16_t fa_oracle_f32_to_bf16(float f);
float fa_oracle_bf16_to_f32(uint16_t h);

/* Ordered fmaf chain: acc_i = init ? init[i] : +0; acc_i = fmaf(x[k][i], w[k], acc_i)
 * for k = 0..D-1.  threads <= 1 runs scalar; >1 splits the element range. */
void fa_oracle_fedavg_f32(const float* const* x, const float* w, int n_clients, size_t n,
                          const float* init, float* out, int threads);
/* bf16 inputs; out_bf16 != 0 -> uint16 bf16 output (RNE), else fp32 output. */
void fa_oracle_fedavg_bf16(const uint16_t* const* x, const float* w, int n_clients, size_t n,
                           const float* init, void* out, int out_bf16, int threads);
/* Reference-literal: out = fl(fl(x_last + x_last) / divisor). */
void fa_oracle_literal_f32(const float* x_last, size_t n, float divisor, float* out);
void fa_oracle_literal_bf16(const uint16_t* x_last, size_t n, float divisor, void* out, int out_bf16);

#ifdef __cplusplus
}
#endif
#endif
