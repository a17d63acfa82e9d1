// k_chain.hpp — parameters of the persistent batch-1 layer chain (k_chain.hip), shared
// with its caller (engine.hip).
#pragma once
#include <cstdint>

namespace qie {

struct ChainParams {
    const uint16_t* att;                 // [QD] attention output of this layer
    const uint16_t* wo;                  // [H][QD]
    uint16_t* x;                         // [H] residual stream (in / out)
    const uint16_t* ffn_norm;            // [H]
    const uint16_t* wg;                  // [I][H]
    const uint16_t* wu;                  // [I][H]
    uint16_t* h;                         // [I]
    const uint16_t* wd;                  // [H][I]
    const uint16_t* attn_norm;           // next layer [H] (nullptr: no Q phase)
    const uint16_t* wq;                  // next layer [QD][H]
    const uint16_t* wk;                  // [KD][H]
    const uint16_t* wv;                  // [KD][H]
    const uint16_t* bq;                  // biases (nullable)
    const uint16_t* bk;
    const uint16_t* bv;
    uint16_t* qkv;                       // [QD + 2 KD]
    int64_t H, QD, KD, I;
    float eps;
    int numerics;
    unsigned* ctr;                       // kChainCtrWords, zero at rest
    unsigned long long* dbg;             // timing stamps [grid][16] (tools only; nullptr normally)
};


}  // namespace qie
