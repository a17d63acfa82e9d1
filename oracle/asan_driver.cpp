// oracle/asan_driver.cpp — TEST INFRASTRUCTURE ONLY: the CPU oracle under AddressSanitizer
// + UndefinedBehaviorSanitizer (host code only — no GPU code is sanitized).
// `make -C oracle asan` links this driver with qie_oracle.cpp into oracle/_build/asan_driver;
// tests/test_oracle_asan.py runs it.  It drives every oracle entry point the parity tests
// use on tiny models with odd sizes (Qwen2-style with bias, Qwen3-style with qk-norm, both
// numerics modes): a prompt forward, decode steps against the growing KV cache, attention
// with and without the causal mask, sampling (greedy, top-k, top-p) and the RoPE tables.
// Any out-of-bounds access, use of freed memory, or undefined arithmetic aborts with a
// sanitizer report; a clean run prints "asan ok".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/qie/qie_types.h"

typedef uint16_t bf16_t;
extern "C" {
uint16_t or_f2bf(float f);
void or_rope_table_ref(float* cos_out, float* sin_out, int n_pos, int head_dim, float base);
void or_rope_table_hf(float* cos_out, float* sin_out, int n_pos, int head_dim, float base);
void or_set_sum_order(int v);
void or_attention(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, bf16_t* out, int mq, int mkv, int nq, int nkv,
                  int hd, int causal, int q_abs_base, int64_t kv_head_stride, int nthreads);
int or_topk_ref(const bf16_t* logits, int64_t V, int k, int32_t* idx_out, float* val_out);
int or_argmax_ref(const bf16_t* logits, int64_t V);
int or_sample_ref(const bf16_t* logits, int64_t V, int k, float temperature, float top_p, uint64_t seed);
int or_forward(const qie_model_spec* s, const qie_model_weights* w, bf16_t* kcache, bf16_t* vcache, int max_ctx,
               const int32_t* ids, int n, int start_pos, bf16_t* logits_out, bf16_t* final_hidden, int nthreads);
}

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static float urand() {   // xorshift64*, uniform in [-1, 1)
    g_state ^= g_state >> 12;
    g_state ^= g_state << 25;
    g_state ^= g_state >> 27;
    return (float)((g_state * 2685821657736338717ull) >> 40) / (float)(1ull << 23) - 1.0f;
}
static std::vector<bf16_t> rnd(size_t n, float scale, float offset = 0.f) {
    std::vector<bf16_t> v(n);   // exactly n elements: an overrun by the oracle is caught
    for (auto& x : v) x = or_f2bf(offset + scale * urand());
    return v;
}

static int run_model(int L, int H, int nq, int nkv, int hd, int I, int V, int bias, int qkn, int numerics) {
    qie_model_spec s;
    std::memset(&s, 0, sizeof(s));
    s.n_layers = L; s.hidden = H; s.n_heads = nq; s.n_kv_heads = nkv; s.head_dim = hd; s.ffn = I; s.vocab = V;
    s.tie_embeddings = 0; s.qkv_bias = bias; s.qk_norm = qkn; s.rms_eps = 1e-4f; s.rope_theta = 1e6f;
    s.numerics = numerics;
    const int QD = nq * hd, KD = nkv * hd;
    std::vector<std::vector<bf16_t>> keep;
    auto add = [&](size_t n, float sc, float off = 0.f) -> const void* {
        keep.push_back(rnd(n, sc, off));
        return keep.back().data();
    };
    std::vector<qie_layer_weights> layers(L);
    for (auto& lw : layers) {
        std::memset(&lw, 0, sizeof(lw));
        lw.attn_norm = add(H, 0.1f, 1.f);
        lw.wq = add((size_t)QD * H, 0.05f);
        lw.wk = add((size_t)KD * H, 0.05f);
        lw.wv = add((size_t)KD * H, 0.05f);
        if (bias) { lw.bq = add(QD, 0.05f); lw.bk = add(KD, 0.05f); lw.bv = add(KD, 0.05f); }
        if (qkn) { lw.q_norm = add(hd, 0.1f, 1.f); lw.k_norm = add(hd, 0.1f, 1.f); }
        lw.wo = add((size_t)H * QD, 0.05f);
        lw.ffn_norm = add(H, 0.1f, 1.f);
        lw.w_gate = add((size_t)I * H, 0.05f);
        lw.w_up = add((size_t)I * H, 0.05f);
        lw.w_down = add((size_t)H * I, 0.05f);
    }
    qie_model_weights w;
    std::memset(&w, 0, sizeof(w));
    w.embed = add((size_t)V * H, 0.5f);
    w.final_norm = add(H, 0.1f, 1.f);
    w.lm_head = add((size_t)V * H, 0.05f);
    w.n_layers = L;
    w.layers = layers.data();

    const int max_ctx = 23, P = 13;
    std::vector<bf16_t> kc((size_t)L * KD * max_ctx), vc((size_t)L * KD * max_ctx), logits(V), hid(H);
    std::vector<int32_t> ids(P);
    for (int i = 0; i < P; i++) ids[i] = (i * 7919 + 13) % V;
    for (int order = 0; order < 3; order++) {
        or_set_sum_order(order);
        if (or_forward(&s, &w, kc.data(), vc.data(), max_ctx, ids.data(), P, 0, logits.data(), hid.data(), 2)) return 1;
        int tok = or_argmax_ref(logits.data(), V);
        for (int pos = P; pos < max_ctx; pos++) {   // decode up to the last cache row
            if (or_forward(&s, &w, kc.data(), vc.data(), max_ctx, &tok, 1, pos, logits.data(), nullptr, 1)) return 2;
            tok = or_sample_ref(logits.data(), V, 5, 0.7f, 0.9f, 1234 + pos);
            if (tok < 0 || tok >= V) return 3;
        }
    }
    or_set_sum_order(0);
    // attention alone: causal prefill rows against a strided cache, and one decode row
    std::vector<bf16_t> q = rnd((size_t)P * QD, 1.f), out((size_t)P * QD);
    or_attention(q.data(), kc.data(), vc.data(), out.data(), P, P, nq, nkv, hd, 1, 0, max_ctx * (int64_t)hd, 2);
    or_attention(q.data(), kc.data(), vc.data(), out.data(), 1, max_ctx, nq, nkv, hd, 0, max_ctx - 1,
                 max_ctx * (int64_t)hd, 1);
    std::vector<int32_t> ti(7);
    std::vector<float> tv(7);
    if (or_topk_ref(logits.data(), V, 7, ti.data(), tv.data()) < 0) return 4;
    std::vector<float> cs((size_t)max_ctx * (hd / 2)), sn((size_t)max_ctx * (hd / 2));
    or_rope_table_ref(cs.data(), sn.data(), max_ctx, hd, 1e6f);
    or_rope_table_hf(cs.data(), sn.data(), max_ctx, hd, 1e6f);
    return 0;
}

int main() {
    // odd widths on purpose: H not a multiple of 64, a 3-head GQA group, a vocab of 1009
    int rc = run_model(2, 96, 6, 2, 32, 200, 1009, 1, 0, QIE_NUMERICS_REF);
    if (!rc) rc = run_model(2, 128, 4, 1, 64, 144, 517, 0, 1, QIE_NUMERICS_HF);
    if (rc) {
        std::printf("asan driver failed: %d\n", rc);
        return rc;
    }
    std::printf("asan ok\n");
    return 0;
}
