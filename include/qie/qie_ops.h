/*
 * qie_ops.h — operator-level C ABI of libqie.so (MI355X / gfx950 HIP kernels).
 *
 * This replaces the reference's operator API, layers/include/helpers.cuh:45-166
 * (launch_rms, launch_rope, launch_rope_single, launch_qknorm, launch_matmul,
 * proj, launch_attn, launch_act, launch_elem, launch_resadd, sample_topk_bf16,
 * copy_last_vocab_vec, copy_first_token) and the __global__ prototypes of
 * layers/include/layers_include.cuh:15-35.
 *
 * Conventions (differences from the reference are deliberate):
 *   - every pointer is a caller-owned DEVICE pointer unless stated; tensors are
 *     bf16 (uint16_t words), row-major, linear weights in PyTorch [out, in];
 *   - every op takes an explicit hipStream_t (passed as void*; NULL = the
 *     legacy default stream the reference uses) and never synchronises, never
 *     allocates — so every op can be captured into a hipGraph;
 *   - every op returns 0 on success, a positive hipError_t, or a negative QIE
 *     error (-22 = invalid argument); qie_last_error() returns the text.
 *     (The reference returns void and prints to stderr.)
 */
#ifndef QIE_OPS_H
#define QIE_OPS_H

#include "qie_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define QIE_ABI_VERSION 1

const char* qie_last_error(void);
int qie_abi_version(void);
int qie_device_count(int* count);

/* Device memory plumbing for hosts without their own HIP runtime (ctypes tests,
 * FFI bindings).  A process should use ONE HIP runtime: PyTorch wheels ship their
 * own, so Python callers allocate through these rather than torch.cuda. */
int qie_set_device(int device);
int qie_malloc(void** ptr, int64_t bytes);
int qie_free(void* ptr);
int qie_memcpy_h2d(void* dst, const void* src, int64_t bytes);
int qie_memcpy_d2h(void* dst, const void* src, int64_t bytes);
int qie_memset(void* ptr, int value, int64_t bytes);
int qie_synchronize(void);
/* a non-blocking stream of the current device (ops take it as `void* stream`) */
int qie_stream_create(void** stream_out);
int qie_stream_synchronize(void* stream);
int qie_stream_destroy(void* stream);

/* ---------------------------------------------------------------- tables
 * Replaces precompute_cos_sin (layers/src/include.cpp:5-16, called at
 * utills.cu:36-44).  Fills HOST fp32 tables [n_pos][head_dim/2]: the
 * reference's exact table in REF mode, HF's bf16-rounded table in HF mode. */
int qie_rope_table_host(float* cos_out, float* sin_out, int32_t n_pos, int32_t head_dim,
                        float theta, int32_t numerics);

/* ------------------------------------------------------------- embedding
 * Replaces embedding_matrix_func (layers/src/embedded_matrix.cu:5-17, launched
 * utills.cu:51-54 and qwen_main.cu:267).  out[t,:] = E[ids[t],:]. */
int qie_embedding(const void* E, const int32_t* ids, void* out, int64_t n, int64_t H,
                  void* stream);

/* ---------------------------------------------------------------- RMSNorm
 * Replaces launch_rms / rmsNorm (helpers.cuh:45-49, normalization.cu:5-25).
 * y = rmsnorm(x) * w over rows of H; x and y may not alias. */
int qie_rmsnorm(const void* x, const void* w, void* y, int64_t rows, int64_t H, float eps,
                int32_t numerics, void* stream);

/* ----------------------------------------------------------------- linear
 * Replaces launch_matmul / proj (helpers.cuh:81-106, 132-138; matrix_mul.cu:
 * 165-288) with fused epilogues.  y[m, n] = sum_k x[m, k] * W[n, k], fp32
 * accumulation, one bf16 rounding.  W is up to three [rows_i, K] segments
 * concatenated along N (fused QKV without repacking the weights.bin arena).
 * M <= 8 runs the bandwidth-bound GEMV kernel; larger M the MFMA GEMM.
 */
enum {
    QIE_EPI_STORE = 0,     /* y = bf16(acc [+ bias])                                  */
    QIE_EPI_RESIDUAL = 1,  /* y = bf16(y + bf16(acc))   (launch_resadd fused)          */
    QIE_EPI_SWIGLU = 2,    /* segs (gate, up): y[m, j] = bf16(bf16(up) * bf16(silu(bf16(gate))))
                              (SiLU.cu:10-23 + element_add.cu:4-12 fused); N = I      */
    QIE_EPI_F32 = 3        /* y is float [M, N]: y = acc, unrounded (tensor-parallel
                              partial sums, reduced across ranks before the rounding) */
};

typedef struct qie_linear_args {
    const void* x;          /* [M, K] bf16, row stride ldx (elements)                   */
    int64_t ldx;
    const void* w[3];       /* weight segments, each [seg_rows[i], K]                   */
    const void* bias[3];    /* optional per-segment bias [seg_rows[i]] (Qwen2 q/k/v)    */
    int64_t seg_rows[3];
    int64_t M, K, N;        /* N = output columns (sum of seg_rows; I for SWIGLU)       */
    void* y;                /* [M, N] bf16, row stride ldy                              */
    int64_t ldy;
    int32_t epilogue;       /* QIE_EPI_*                                                */
    int32_t numerics;       /* for the fused norm                                       */
    const void* norm_w;     /* optional fused RMSNorm of x (weight [K]); GEMV path only */
    float norm_eps;
    int32_t flags;          /* QIE_LINEAR_FP8: w[i] are fp8 weights (see below); else 0  */
    uint64_t* argmax_keys;  /* optional [M] selection keys, atomically max-merged
                               (fused greedy arg-max, logit_decode.cu:15-33); caller
                               zeroes them before the launch                            */
    int64_t key_col0;       /* global index of output column 0 in the keys (vocab-
                               parallel lm_head shard offset; 0 otherwise)              */
    const uint8_t* x_exps;  /* QIE_LINEAR_ACT_FP8: [M] e8m0 row exponents of x (below)  */
} qie_linear_args;

int qie_linear(const qie_linear_args* args, void* stream);

/* --------------------------------------------- q/k post-projection + KV append
 * Replaces launch_qknorm (helpers.cuh:140-142, qk_norm.cu:43-79), launch_rope /
 * launch_rope_single (helpers.cuh:51-55, 143-147; RoPE.cu:6-22) and
 * kv_copy_layer_to_cache_prefill/decode (include_cuda.cu:165-279) in one pass:
 *   qkv rows [M, (nq + 2*nkv)*hd] (projection output, bias already added)
 *   -> q_out [M, nq*hd] (qk-norm'd, rotated)
 *   -> K cache row (qk-norm'd, rotated) and V cache row at position pos[m].
 * KV cache layout (qie), two forms:
 *   contiguous (block_table == NULL): per sequence [L][nkv][max_ctx][hd] bf16,
 *     sequence s at k + s*seq_stride;
 *   paged (block_table != NULL): a pool of pages of page_tokens tokens (a power
 *     of two, multiple of 128), page p at k + p*seq_stride holding
 *     [L][nkv][page_tokens][hd]; token t of sequence s lives in page
 *     block_table[s*max_pages + t/page_tokens] at row t % page_tokens.
 * Row m belongs to sequence m / rows_per_seq.
 * (The reference's pages are [4 tok][L][kvdim] nodes of a linked list in managed
 * memory, iengine.cu:73-109, walked by include_cuda.cu:165-279; qie replaces the
 * list with a device block table and keeps each (layer, kv head) run of a page
 * contiguous, so a 128-key attention step streams one run of one page.) */
typedef struct qie_kv_cache {
    void* k;                 /* contiguous: sequence 0's K cache; paged: page 0       */
    void* v;
    int64_t seq_stride;      /* elements between sequences (contiguous) / pages (paged) */
    int32_t n_layers, n_kv_heads, head_dim, max_ctx;
    const int32_t* block_table;   /* device [n_seq][max_pages] page ids, or NULL       */
    int32_t page_tokens;          /* paged only                                         */
    int32_t max_pages;            /* paged only: block_table row stride                 */
} qie_kv_cache;

int qie_qkv_post(const void* qkv, int64_t M, const int32_t* pos, int32_t rows_per_seq,
                 const void* q_norm, const void* k_norm, const float* rope_cos,
                 const float* rope_sin, int32_t n_heads, const qie_kv_cache* cache,
                 int32_t layer, float eps, int32_t numerics, void* q_out, void* stream);

/* -------------------------------------------------------------- attention
 * Replaces launch_attn / selfattention (helpers.cuh:121-130,
 * self_attension.cu:10-149): GQA attention of query rows over the cache.
 * Row m attends to positions [0, pos[m]] of sequence m / rows_per_seq
 * (prefill: causal; decode: the whole cache incl. the new token — identical
 * to the reference's causal / mkv = seq_len windows).  Flash-decoding split
 * over the sequence; ws must hold qie_attention_workspace_bytes(). */
int64_t qie_attention_workspace_bytes(int64_t M, int32_t n_heads, int32_t head_dim,
                                      int32_t max_ctx);
int qie_attention(const void* q, int64_t M, const int32_t* pos, int32_t rows_per_seq,
                  const qie_kv_cache* cache, int32_t layer, int32_t n_heads, void* out,
                  void* ws, void* stream);

/* Decode attention with the q/k post-projection fused in (one launch per layer):
 * qkv rows [B][(nq + 2 nkv) hd] straight from the QKV projection; applies qk-norm
 * (q_norm/k_norm non-NULL) and RoPE at pos[m] to q and to the new k, appends the
 * new K/V row of sequence m at pos[m], and attends over [0, pos[m]].  Splits of 128
 * keys are combined in-launch by the last-arriving workgroup.  ws must hold
 * qie_attention_decode_workspace_bytes() and be ZEROED once before first use (it
 * is left zeroed by every call).
 * numerics may carry QIE_ATTN_PREROPED (REF numerics, no qk-norm only): q and the new
 * k in qkv are already rotated (the engine's decode QKV projection applies RoPE in its
 * epilogue), so only the K/V append and the attention run here. */
#define QIE_NUMERICS_MASK 0xff
#define QIE_ATTN_PREROPED 0x100
int64_t qie_attention_decode_workspace_bytes(int64_t B, int32_t n_heads, int32_t n_kv_heads,
                                             int32_t head_dim, int32_t max_ctx);
int qie_attention_decode(const void* qkv, int64_t B, const int32_t* pos, const void* q_norm,
                         const void* k_norm, const float* rope_cos, const float* rope_sin,
                         int32_t n_heads, const qie_kv_cache* cache, int32_t layer, float eps,
                         int32_t numerics, void* out, void* ws, void* stream);

/* Diagnostics: one wave, lane l reads 8 bytes at element 4*l of an LDS array whose
 * element i holds i, through ds_read_b64_tr_b16; out_dev[l*4 + e] receives element e
 * of lane l (pins the transposed-read lane mapping the prefill attention relies on). */
int qie_debug_tr16_probe(int32_t* out_dev);

/* ------------------------------------------- standalone in-place head ops
 * The operator tier of a host that keeps the reference's layer loop
 * (qwen_main.cu:77-241); the engine itself fuses these into qie_qkv_post /
 * qie_attention_decode.  Rows [rows][row_stride] of n_heads heads of head_dim.
 *   qie_qknorm: launch_qknorm / qkNorm (helpers.cuh:140-142, qk_norm.cu:43-79),
 *     in place, the reference's tree summation order (REF); HF = transformers.
 *   qie_rope:   launch_rope / launch_rope_single (helpers.cuh:51-55, 143-147;
 *     RoPE.cu:6-22), in place; row r at position pos[r] (device, may be NULL)
 *     or pos0 + r.  Tables as built by qie_rope_table_host.
 *   qie_kv_write: kv_copy_layer_to_cache_prefill / _decode (include_cuda.cu:
 *     165-279): K and V rows [rows][ld] (n_kv_heads*head_dim used) into layer
 *     `layer` of sequence `seq` at positions pos0 .. pos0+rows-1.  Paged caches
 *     need those pages held (qie_batch_reserve). */
int qie_qknorm(void* x, int64_t rows, int64_t row_stride, int32_t n_heads, int32_t head_dim,
               const void* w, float eps, int32_t numerics, void* stream);
int qie_rope(void* x, int64_t rows, int64_t row_stride, int32_t n_heads, int32_t head_dim,
             const int32_t* pos, int32_t pos0, const float* rope_cos, const float* rope_sin,
             int32_t numerics, void* stream);
int qie_kv_write(const void* k, const void* v, int64_t rows, int64_t ld, int32_t pos0,
                 const qie_kv_cache* cache, int32_t seq, int32_t layer, void* stream);

/* ------------------------------------------------------------- elementwise
 * launch_act + launch_elem (helpers.cuh:108-115) and launch_resadd (:116-119)
 * for callers that do not use the fused linear epilogues: qie_silu_mul fuses the
 * two; qie_silu (activation, SiLU.cu:10-23, in place: x = bf16(x*sigmoid(x))) and
 * qie_mul (element_mul, element_add.cu:4-12: c = bf16(a*b)) are the separate ops.
 * qie_memcpy_d2d: copy_last_vocab_vec / copy_first_token (helpers.cuh:149-155). */
int qie_silu(void* x, int64_t n, void* stream);
int qie_mul(const void* a, const void* b, void* c, int64_t n, void* stream);
int qie_memcpy_d2d(void* dst, const void* src, int64_t bytes, void* stream);
int qie_silu_mul(const void* gate, const void* up, void* h, int64_t n, void* stream);
int qie_residual_add(void* x, const void* y, int64_t n, void* stream);
/* Tensor-parallel residual: x = bf16(x + bf16(sum)) with sum the fp32 all-reduced
 * partials of the row-parallel O / down projection (same rounding as the fused
 * QIE_EPI_RESIDUAL epilogue on one GPU). */
int qie_residual_add_f32(void* x, const float* sum, int64_t n, void* stream);

/* ---------------------------------------------------------------- sampling
 * Replaces sample_topk_bf16 / topk_temperature_softmax_sampling_kernel_bf16
 * (helpers.cuh:157-166, logit_decode.cu:149-274).  Writes the chosen id of each
 * of the M logit rows to out_ids (device).  top_k <= 1 -> greedy arg-max.
 * ws must hold qie_sample_workspace_bytes(). */
int64_t qie_sample_workspace_bytes(int64_t M, int64_t V);
int qie_sample(const void* logits, int64_t M, int64_t V, int64_t ld, const qie_sampling* s,
               const int32_t* step_dev, int32_t* out_ids, void* ws, void* stream);
/* Decode fused arg-max keys (see qie_linear_args.argmax_keys) into ids. */
int qie_keys_to_ids(const uint64_t* keys, int64_t M, int32_t* out_ids, void* stream);

/* ------------------------------------------------------- synthetic weights
 * Deterministic counter-based fill used for synthetic checkpoints (no weights
 * ship in this environment): element i of tensor `tensor_id` is
 *   r = splitmix64(splitmix64(seed*0x9E3779B97F4A7C15 ^ (tensor_id << 32)) + i)
 *   u = ((int32)(r >> 40) - 2^23) * 2^-23          (exact, in [-1, 1))
 *   value = bf16(offset + u * scale)
 * bit-identical on the host (qie_synthetic_fill_host, OpenMP) and the GPU. */
uint32_t qie_tensor_id(const char* name);   /* FNV-1a 32 of the tensor name */
int qie_synthetic_fill(void* dev, int64_t n, uint32_t tensor_id, uint64_t seed, float scale,
                       float offset, void* stream);
int qie_synthetic_fill_host(void* host, int64_t n, uint32_t tensor_id, uint64_t seed,
                            float scale, float offset);
/* ------------------------------------------------------------ fp8 weights
 * A linear weight [rows, cols] in fp8 is rows*cols OCP e4m3 codes followed by rows fp32
 * power-of-two row scales (qie_fp8_weight_bytes); every dequantised value is exactly a
 * bf16.  qie_linear reads such weights when args.flags has QIE_LINEAR_FP8. */
#define QIE_LINEAR_FP8 1
/* Prefill GEMM tile override (tests / tuning; M >= 256, K % 32 == 0): the LDS-DMA kernel
 * with 256x256 (TILE256) or 256x128 (TILE128) block tiles instead of the tile-count choice. */
#define QIE_LINEAR_TILE256 2
#define QIE_LINEAR_TILE128 4
/* ... or the stream-K form of the 256x256 kernel (K % 64 == 0, K >= 256): one workgroup
 * per CU, (tile, k-tile) units in contiguous ranges, shared tiles summed in k order. */
#define QIE_LINEAR_STREAMK 8
int64_t qie_fp8_weight_bytes(int64_t rows, int64_t cols);
int qie_quantize_fp8(const void* w_bf16, int64_t rows, int64_t cols, void* out, void* stream);
int qie_quantize_fp8_host(const void* w_bf16, int64_t rows, int64_t cols, void* out);
/* The inverse, on device: rows x cols bf16 (exact — every dequantised value is a bf16).
 * The engine's fp8 prefill (M >= 256 rows) expands each weight into a scratch with it and
 * runs the bf16 LDS-DMA GEMM: at prefill sizes the GEMM is MFMA-bound and the expansion
 * (1 + 2 bytes per weight) is ~2 % of it. */
int qie_dequantize_fp8(const void* w_fp8, int64_t rows, int64_t cols, void* out_bf16, void* stream);
/* 16-row tiled fp8 layout (QIE_LINEAR_FP8_T16): the codes of rows [16t, 16t + 16) are stored
 * as K/64 consecutive 1-KiB blocks, block j holding row 16t + (l % 16), columns
 * 64j + 16(l / 16) + [0, 16) at bytes [16 l, 16 l + 16) (l = 0..63) — exactly the B fragments
 * of one 64-column unit of the batched-decode MFMA kernel, so each of its 1-KiB wave loads
 * is contiguous (8 whole 128-B lines instead of 16 rows x 64 B); the row scales follow the
 * codes as in the plain layout.  rows % 16 == 0, cols % 64 == 0.  qie_linear reads such
 * weights with args.flags QIE_LINEAR_FP8 | QIE_LINEAR_FP8_T16 (the batched-decode kernel
 * only: M <= 16 rows; the engine tiles its own decode projections, tiled weights are not
 * read by the prefill GEMMs, which take the dequantised bf16 copy). */
#define QIE_LINEAR_FP8_T16 16
/* Block-scaled fp8 ACTIVATIONS — the CDNA4 fp8 MFMA path (v_mfma_scale_f32_16x16x128_
 * f8f6f4), an explicit numerics choice (the engine's qie_engine_opts.prefill_fp8): x holds
 * e4m3 codes [M, K] with row stride ldx BYTES and x_exps their per-row e8m0 exponents, row m
 * standing for 2^(x_exps[m] - 127) * e4m3(code) (qie_quantize_rows_fp8).  The weights must be
 * fp8 (QIE_LINEAR_FP8, plain or QIE_LINEAR_FP8_T16 tiled); their power-of-two row scales are
 * the MFMA's other e8m0 operand.  K % 128 == 0, ldx % 16 == 0, no fused norm / arg-max, any
 * M (the batched-decode row limit of the tiled layout does not apply).  Replaces the
 * reference's matrix_mul (matrix_mul.cu:165-288) for a model whose prefill activations are
 * quantised; the oracle runs the same model (or_set_act_fp8). */
#define QIE_LINEAR_ACT_FP8 32
/* Per-row activation quantisation for QIE_LINEAR_ACT_FP8: s[m] = the smallest power of two
 * with max_k |x[m, k]| / s[m] <= 448 (1 for an all-zero row; e4m3_row_scale), codes
 * q[m, k] = e4m3(x[m, k] / s[m]) rounded to nearest even (|x / s| <= 448: nothing saturates),
 * exps[m] = log2(s[m]) + 127.  x bf16 [rows, cols], row stride ldx elements; q row stride ldq
 * bytes.  cols % 8 == 0, ldx % 8 == 0, ldq % 16 == 0. */
int qie_quantize_rows_fp8(const void* x, int64_t ldx, int64_t rows, int64_t cols, void* q, int64_t ldq,
                          void* exps, void* stream);
int qie_fp8_tile16(const void* w_fp8, int64_t rows, int64_t cols, void* out, void* stream);
/* Test probe: out_dev[i] = the device decode of e4m3 code i (i < 256). */
int qie_debug_fp8_decode(float* out_dev);
/* Test probe: out_dev[i] = the bf16 bits the fp8 MFMA GEMV decodes e4m3 code i to (i < 256). */
int qie_debug_fp8_decode_bf16(uint16_t* out_dev);

/* Tensor-parallel shard of the same synthetic tensor: dev[i][j] = element
 * (row0 + i) * full_cols + col0 + j of the full tensor, rows x cols, row-major. */
int qie_synthetic_fill_slice(void* dev, int64_t rows, int64_t cols, int64_t full_cols, int64_t row0,
                             int64_t col0, uint32_t tensor_id, uint64_t seed, float scale, float offset,
                             void* stream);
/* Rows r of a bf16 [rows, cols] matrix with (row0 + r) % every == 0 multiplied by 2^log2f
 * in place (exact while finite).  Used to give a synthetic lm_head a peaked, trained-model-
 * like top-1 margin for the end-to-end greedy parity runs (tests/parity.py, bench.py). */
int qie_scale_rows_pow2(void* w, int64_t rows, int64_t cols, int64_t row0, int64_t every, int32_t log2f,
                        void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QIE_OPS_H */
