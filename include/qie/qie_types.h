/*
 * qie_types.h — plain-C types shared by the qie C ABI (qie_ops.h, qie_engine.h)
 * and by the CPU oracle (oracle/qie_oracle.cpp).
 *
 * Every tensor crosses the boundary as a raw pointer to little-endian bf16
 * words (uint16_t storage), row-major, PyTorch [out, in] layout for linear
 * weights — exactly the layout of the reference's flat weights.bin
 * (reference: layers/src/tensor_parser.cpp:31-129, model_files/meta_data.txt).
 *
 * The reference hard-codes every dimension (layers/src/utills.cu:8-16,
 * layers/include/iengine.cuh:19-21).  qie replaces those literals with a
 * qie_model_spec so Qwen2 (0.5B/7B/72B) and the reference's own Qwen3-14B run
 * through the same kernels.
 */
#ifndef QIE_TYPES_H
#define QIE_TYPES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Numerics mode.
 *  QIE_NUMERICS_REF: the reference engine's op semantics —
 *    RMSNorm  y = bf16((x / sqrtf(mean(x^2) + eps)) * w)      normalization.cu:5-25
 *    RoPE     interleaved pairs (2j, 2j+1), fp32 cos/sin table  RoPE.cu:6-22, include.cpp:5-16
 *    bf16 rounding after every op, bf16 residual stream.
 *  QIE_NUMERICS_HF: HuggingFace Qwen2/Qwen3 semantics —
 *    RMSNorm  y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps)))
 *    RoPE     rotate_half pairs (j, j + hd/2), bf16 cos/sin, bf16 products.
 */
typedef enum qie_numerics {
    QIE_NUMERICS_REF = 0,
    QIE_NUMERICS_HF = 1
} qie_numerics;

typedef struct qie_model_spec {
    int32_t n_layers;      /* reference: number_of_layers = 40  (utills.cu:8)   */
    int32_t hidden;        /* hidden_dim = 5120                  (utills.cu:10)  */
    int32_t n_heads;       /* num_of_qheads = 40                 (utills.cu:12)  */
    int32_t n_kv_heads;    /* num_of_kvheads = 8                 (utills.cu:13)  */
    int32_t head_dim;      /* head_dim = 128                     (utills.cu:9)   */
    int32_t ffn;           /* up_dim = 17408                     (utills.cu:16)  */
    int32_t vocab;         /* vocab_size = 151936                (utills.cu:15)  */
    int32_t tie_embeddings;/* 1: lm_head is embed_tokens (Qwen2-0.5B)           */
    int32_t qkv_bias;      /* 1: q/k/v projections carry a bias (Qwen2)         */
    int32_t qk_norm;       /* 1: per-head RMSNorm of q and k (Qwen3; qk_norm.cu) */
    float rms_eps;         /* ref mode: 1e-4 (normalization.cu:9, qk_norm.cu:46) */
    float rope_theta;      /* ref mode: 1e6  (include.cpp:7)                     */
    int32_t numerics;      /* qie_numerics                                       */
    int32_t reserved[7];
} qie_model_spec;

/* Per-layer weight pointers (bf16).  Optional tensors are NULL when absent
 * (biases when !qkv_bias, q_norm/k_norm when !qk_norm). */
typedef struct qie_layer_weights {
    const void* attn_norm;   /* input_layernorm.weight           [H]          */
    const void* wq;          /* self_attn.q_proj.weight          [nq*hd, H]   */
    const void* wk;          /* self_attn.k_proj.weight          [nkv*hd, H]  */
    const void* wv;          /* self_attn.v_proj.weight          [nkv*hd, H]  */
    const void* bq;          /* self_attn.q_proj.bias            [nq*hd]      */
    const void* bk;          /* self_attn.k_proj.bias            [nkv*hd]     */
    const void* bv;          /* self_attn.v_proj.bias            [nkv*hd]     */
    const void* q_norm;      /* self_attn.q_norm.weight          [hd]         */
    const void* k_norm;      /* self_attn.k_norm.weight          [hd]         */
    const void* wo;          /* self_attn.o_proj.weight          [H, nq*hd]   */
    const void* ffn_norm;    /* post_attention_layernorm.weight  [H]          */
    const void* w_gate;      /* mlp.gate_proj.weight             [I, H]       */
    const void* w_up;        /* mlp.up_proj.weight               [I, H]       */
    const void* w_down;      /* mlp.down_proj.weight             [H, I]       */
} qie_layer_weights;

typedef struct qie_model_weights {
    const void* embed;       /* embed_tokens.weight  [V, H]                          */
    const void* final_norm;  /* norm.weight          [H]                             */
    const void* lm_head;     /* lm_head.weight (short_name "logits") [V, H]; == embed when tied */
    int32_t n_layers;
    const qie_layer_weights* layers;   /* n_layers entries */
} qie_model_weights;

/* Sampling parameters.  top_k == 1 (or temperature <= 0) is greedy arg-max with
 * the reference's tie rule (logit_decode.cu:15-33).
 * top_k > 1 follows topk_temperature_softmax_sampling_kernel_bf16
 * (logit_decode.cu:149-274): k rounds of masked arg-max (k <= 256), softmax at
 * temperature T, one cuRAND-XORWOW uniform draw seeded (seed, subseq = 0).
 * top_p < 1 additionally truncates the top-k list to the smallest prefix whose
 * probability mass reaches top_p (qie extension; the reference has no top-p). */
typedef struct qie_sampling {
    int32_t top_k;
    float temperature;
    float top_p;
    uint64_t seed;           /* reference: prefill 1234, decode 1234 + step      */
} qie_sampling;

#ifdef __cplusplus
}
#endif

#endif /* QIE_TYPES_H */
