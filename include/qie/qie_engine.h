/*
 * qie_engine.h — engine-level C ABI of libqie.so: weights, KV cache,
 * prefill and hipGraph-captured decode.
 *
 * Replaces the reference's driver / step API:
 *   llm()                               layers/src/qwen_main.cu:64-417, iengine.cuh:51
 *       -> qie_prefill() (state == prefill) / qie_decode_step() (state == decode)
 *   create_new_sequence()               layers/src/iengine.cu:25-47
 *   initialize_model_buffers()          layers/src/utills.cu:4-129
 *   destroy_model_buffers()             layers/src/utills.cu:142-205
 *       -> qie_batch_create() / qie_batch_destroy()
 *   create_page_list / allocate_page_buffers / free_page_list
 *                                       layers/src/iengine.cu:73-109
 *       -> the KV cache owned by qie_batch (contiguous per (layer, kv head))
 *   load_all_weights_to_gpu_chunked()   layers/src/iengine.cu:117-223
 *       -> qie_engine_load_weights_bin()
 *   parsed_tensors / build_indexed_tensors (tensor_parser.cpp:31-165)
 *       -> qie_index_* (reference-compatible weights.bin index)
 *
 * All functions return 0 on success; qie_last_error() (qie_ops.h) has the text.
 */
#ifndef QIE_ENGINE_H
#define QIE_ENGINE_H

#include "qie_types.h"
#include "qie_ops.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qie_engine qie_engine;
typedef struct qie_comm qie_comm;
typedef struct qie_batch qie_batch;
typedef struct qie_index qie_index;

/* ------------------------------------------------------------------ index
 * Reference-compatible tensor index (tensor_parser.hh:204-210):
 * {tensor_name, shape, data_offsets (bytes, re-based into one contiguous
 * weights.bin), layer_index (-1 for globals), short_name}; lm_head.weight
 * has short_name "logits". */
int qie_index_load_meta(const char* meta_data_txt, qie_index** out);   /* meta_data.txt format */
int qie_index_synthetic(const qie_model_spec* spec, qie_index** out);  /* HF names, sorted, one shard */
int qie_index_count(const qie_index* idx);
int qie_index_get(const qie_index* idx, int i, const char** name, const char** short_name,
                  int32_t* layer, int64_t* off0, int64_t* off1, int32_t* ndim, int64_t* shape4);
int64_t qie_index_total_bytes(const qie_index* idx);
int qie_index_write_meta(const qie_index* idx, const char* path);
void qie_index_destroy(qie_index* idx);

/* ----------------------------------------------------------------- engine */
/* ------------------------------------------------------ tensor parallelism
 * One communicator per rank.  RCCL: rank 0 calls qie_comm_unique_id() and ships the
 * QIE_COMM_ID_BYTES bytes to every rank (any host channel), then every rank calls
 * qie_comm_create_rccl() with its device (blocks until all ranks joined).  Local:
 * qie_comm_create_local(world, out[world]) makes `world` ranks of ONE process on one
 * device, driven by one host thread each (test backend; engines on it run without
 * hipGraphs).  Pass the handle as qie_engine_opts.tp_comm; the engine then holds
 * only its shard and every collective call of a step must be made by
 * all ranks (prefill, decode, qie_batch_logits). */
#define QIE_COMM_ID_BYTES 128
int qie_comm_unique_id(void* id_out);
int qie_comm_create_rccl(const void* id, int32_t world, int32_t rank, int32_t device, qie_comm** out);
int qie_comm_create_local(int32_t world, qie_comm** out);
/* Peer backend: every rank's exchange buffer mapped into every rank, one
 * kernel per collective (push + per-block generation flags + rank-ordered reduce, the
 * residual add fused into the row-parallel all-reduce); graph-capturable.  Across
 * processes: qie_comm_create_peer() returns this rank's QIE_COMM_PEER_HANDLE_BYTES IPC
 * handle, the host ships all handles to every rank (handles[r] = rank r's), then
 * qie_comm_peer_connect().  Ranks of one process on one device (world <= 2: the
 * process's hardware queues must give every rank its own):
 * qie_comm_create_peer_local(world, out[world]).  A rank that waited ~10 s for a peer
 * sets the error word qie_comm_peer_error() reads (no kernel waits forever); it then stores
 * no result, the communicator stays poisoned (later exchanges return at once) and the
 * engine's next synchronising call fails. */
#define QIE_COMM_PEER_HANDLE_BYTES 128
int qie_comm_create_peer(int32_t world, int32_t rank, int32_t device, qie_comm** out, void* handle_out);
int qie_comm_peer_connect(qie_comm* c, const void* handles);
int qie_comm_create_peer_local(int32_t world, qie_comm** out);
int qie_comm_peer_error(const qie_comm* c, int32_t* err);
/* Peer backend exchange form, set identically on every rank between steps
 * (a captured decode graph keeps the form it was captured with): tagged = 1 sends
 * row-parallel exchanges of <= 131,072 elements as {generation tag, f32} words that the
 * readers poll directly (no flags, no system fences), 0 the flagged form; push = 1 (with
 * tagged) lets a batch-1 projection's GEMV epilogue write those words itself, so the
 * exchange kernel only waits and reduces.  Results are bit-identical in every form.
 * Defaults: env QIE_PEER_TAGGED / QIE_PEER_PUSH, else 1 / 1. */
int qie_comm_peer_set_mode(qie_comm* c, int32_t tagged, int32_t push);
/* x (bf16 [n]) = bf16(x + bf16(sum over ranks of part)), in place on x (part may be
 * overwritten): the exchange after a row-parallel projection */
int qie_comm_allreduce_residual_bf16(qie_comm* c, const float* part, void* x, int64_t n, void* stream);
/* Measurement: `count` row-parallel exchanges of n elements captured in one hipGraph on
 * `stream` and replayed `reps` times (after one warm replay); *us_out = microseconds per
 * exchange (hipEvents).  form 0: as the engine runs them (the current mode), 1: the flagged
 * form, 2: the flagged form with n = 0 (the synchronisation alone at the same grid).  Every
 * rank must call it with the same arguments. */
int qie_comm_time_exchange(qie_comm* c, const float* part, void* x, int64_t n, int32_t count, int32_t reps,
                           int32_t form, void* stream, float* us_out);
int qie_comm_rank(const qie_comm* c, int32_t* world, int32_t* rank);
int qie_comm_allreduce_sum_f32(qie_comm* c, float* buf, int64_t n, void* stream);
/* in place: element-wise max over ranks of u64 words (the greedy arg-max keys) */
int qie_comm_allreduce_max_u64(qie_comm* c, uint64_t* buf, int64_t n, void* stream);
void qie_comm_destroy(qie_comm* c);

typedef struct qie_engine_opts {
    int32_t device;          /* HIP device ordinal                                   */
    int32_t max_ctx;         /* RoPE table rows (reference CONTEXT_SIZE = 32786)     */
    int32_t use_graph;       /* 1: decode steps replay a captured hipGraph           */
    int32_t tp_rank, tp_size;/* informational; taken from tp_comm when it is set     */
    void* tp_comm;           /* qie_comm* (tensor parallel over its ranks) or NULL   */
    int32_t weight_fp8;      /* 1: linear weights + lm_head quantised to OCP e4m3 with
                                power-of-two row scales after loading (qie_ops.h)     */
    int32_t comm_always;     /* 1: run the exchange steps (row-parallel all-reduces, the
                                greedy key max, the logit gather) through tp_comm even at
                                world 1 — the captured-collective path on one GPU (tests) */
    int32_t prefill_fp8;     /* 1 (with weight_fp8): the prefill projections run on the
                                block-scaled fp8 MFMA (QIE_LINEAR_ACT_FP8) — activations
                                quantised per row to e4m3 before each projection, a
                                different model from the bf16-activation one (numerics flag) */
    int32_t reserved[5];
} qie_engine_opts;

int qie_engine_create(const qie_model_spec* spec, const qie_engine_opts* opts, qie_engine** out);
/* Synthetic checkpoint at real shapes (no weights ship here): reference-layout
 * arena (qie_index_synthetic), every tensor filled by qie_synthetic_fill with
 * tensor_id = qie_tensor_id(name): linear weights offset 0 / scale w_scale,
 * norm weights 1 + norm_scale*u, biases bias_scale*u. */
int qie_engine_init_synthetic(qie_engine* e, uint64_t seed, float w_scale, float norm_scale,
                              float bias_scale);
/* Reference flat weights.bin + meta_data.txt index, read in chunks through a
 * pinned staging buffer (load_all_weights_to_gpu_chunked semantics). */
int qie_engine_load_weights_bin(qie_engine* e, const char* weights_bin, const char* meta_data_txt,
                                int64_t chunk_bytes);
/* Caller-owned device weights (e.g. torch tensors); not freed by qie. */
int qie_engine_set_weights(qie_engine* e, const qie_model_weights* w);
int qie_engine_weights(const qie_engine* e, qie_model_weights* out, const qie_layer_weights** layers);
int qie_engine_spec(const qie_engine* e, qie_model_spec* out);
void* qie_engine_stream(qie_engine* e);
int qie_engine_sync(qie_engine* e);
void qie_engine_destroy(qie_engine* e);

/* ------------------------------------------------------------------ batch
 * B independent sequences decoded together (weights streamed once per step).
 * KV cache [B][L][nkv][max_ctx][hd] bf16; token history [B][max_ctx]. */
int qie_batch_create(qie_engine* e, int32_t batch, int32_t max_ctx, qie_batch** out);
void qie_batch_destroy(qie_batch* b);

/* Paged KV cache with a device block table.  Replaces the
 * reference's per-sequence linked page list — create_page_list /
 * allocate_page_buffers / free_page_list (iengine.cu:73-109) walked by
 * kv_copy_layer_to_cache_prefill/decode (include_cuda.cu:165-279) and the
 * batch_metadata slots (iengine.cuh:27-37).  A pool of n_pages pages of
 * page_tokens tokens (a power of two >= 128; 0 = 128) shared by the B slots;
 * n_pages 0 = enough for every slot at max_ctx.  Pages are taken on demand by
 * qie_prefill / qie_decode* / qie_batch_set_position and returned by
 * qie_batch_release; running out of pages fails the call (-28, nothing launched).
 * Page 0 is a scratch page that idle slots write into. */
int qie_batch_create_paged(qie_engine* e, int32_t batch, int32_t max_ctx, int32_t page_tokens,
                           int32_t n_pages, qie_batch** out);
/* Ends sequence `seq`: its pages go back to the pool (paged) and the slot idles —
 * it still runs through every decode step on the scratch page, its outputs are
 * meaningless — until the next qie_prefill into it.  Any batch. */
int qie_batch_release(qie_batch* b, int32_t seq);
/* Pool state: free pages, pages per slot (host [B], may be NULL), page_tokens. */
int qie_batch_page_stats(qie_batch* b, int32_t* free_pages, int32_t* pages_per_seq, int32_t* page_tokens);
/* The n first block-table entries of `seq` (host copy); paged batches only. */
int qie_batch_block_table(qie_batch* b, int32_t seq, int32_t* host_pages, int32_t n);

/* Prefill sequence `seq` with n prompt ids (host array); writes its KV rows
 * 0..n-1, samples the first generated token (host *next_id, may be NULL) and
 * makes it the sequence's current token at position n. */
int qie_prefill(qie_batch* b, int32_t seq, const int32_t* ids, int32_t n, const qie_sampling* s,
                int32_t* next_id);
/* qie_prefill of n_seqs prompts of len ids each (host [n_seqs][len], laid end to end)
 * into slots seq0 .. seq0+n_seqs-1 in one pass: every projection GEMM runs once over
 * the n_seqs*len rows (the reference prefills one sequence per call, iengine.cu
 * prefill path; this is the batch-admission form of it).  next_ids: host [n_seqs]
 * or NULL.  Paged batches: all-or-nothing on the pool, as qie_prefill. */
int qie_prefill_batch(qie_batch* b, int32_t seq0, int32_t n_seqs, const int32_t* ids, int32_t len,
                      const qie_sampling* s, int32_t* next_ids);
/* One decode step for all B sequences (hipGraph replay when enabled);
 * next_ids: host [B] or NULL (then nothing is synchronised). */
int qie_decode_step(qie_batch* b, const qie_sampling* s, int32_t* next_ids);
/* n_steps decode steps back to back; out_ids host [n_steps][B] (may be NULL). */
int qie_decode(qie_batch* b, int32_t n_steps, const qie_sampling* s, int32_t* out_ids);
/* Last logits of every sequence: host bf16 [B][V]. */
int qie_batch_logits(qie_batch* b, void* host_out);
/* Current positions (host int32 [B]) and token history row of `seq`. */
int qie_batch_positions(qie_batch* b, int32_t* host_pos);
int qie_batch_history(qie_batch* b, int32_t seq, int32_t* host_ids, int32_t n);
/* Rewind/set sequence `seq` to position pos with current token `token`
 * (KV rows >= pos are simply overwritten later). */
int qie_batch_set_position(qie_batch* b, int32_t seq, int32_t pos, int32_t token);
/* Decode structure of the batch's steps: 0 = five launches per layer (the reference path:
 * QKV GEMV, attention, O GEMV, gate/up GEMV, down GEMV, hipGraph-captured); 1 = the whole
 * layer stack as ONE persistent launch (one workgroup per CU, weight streams running ahead of
 * the layer's dependency edges, tagged hand-offs between CUs; bit-identical outputs).  Mode 1
 * covers batch 1, bf16 weights, one device, head_dim 64 or 128 and a contiguous KV cache;
 * other batches return an error (QIE_EINVAL) naming what is not covered.  The next step
 * re-captures the decode graph.  qie_batch_decode_mode returns the current mode.  Mode 1 is
 * SLOWER on MI355X (Qwen2-7B 317.5 vs 370.9 tok/s, Qwen2-0.5B 1,065 vs 1,566: its cross-CU
 * hand-offs cost more than the kernel boundaries they replace); mode 0 is
 * the default and the measured path. */
int qie_batch_set_decode_mode(qie_batch* b, int32_t mode);
int qie_batch_decode_mode(const qie_batch* b);
/* Diagnostics of decode mode 1: enable != 0 makes the persistent step record s_memrealtime
 * stamps (100 MHz, chip-wide) at its phase boundaries, [n_cu][n_layers][12] uint64 (slots:
 * 0 layer start, 1 x gathered, 2 QKV done, 3 attention done (attention CUs), 4 attention
 * output gathered (other CUs), 5 O done, 6 x' gathered + norm, 7 gate/up done, 8 h gathered,
 * 9 down done); host_out (n >= that count) receives the last step's stamps; enable = 0
 * frees the buffer.  Changing it re-captures the decode graph. */
int qie_batch_pk_trace(qie_batch* b, int32_t enable, uint64_t* host_out, int64_t n);
/* Batch geometry: B slots, max_ctx positions per slot. */
int qie_batch_dims(const qie_batch* b, int32_t* batch, int32_t* max_ctx);
/* KV descriptor of slot `seq` for the operator tier (qie_kv_write, qie_attention with
 * sequence index 0): contiguous -> that slot's region; paged -> the pool with the
 * slot's block-table row.  Valid until the batch is destroyed. */
int qie_batch_kv_cache(const qie_batch* b, int32_t seq, qie_kv_cache* out);
/* Operator tier: make slot `seq` a live sequence holding the KV pages for positions
 * [0, n_tokens) (paged: taken from the pool, all-or-nothing; contiguous: a bounds
 * check).  allocate_page_buffers (iengine.cu:90-100) in the reference's terms. */
int qie_batch_reserve(qie_batch* b, int32_t seq, int32_t n_tokens);
/* The engine's weight arena (load_all_weights_to_gpu_chunked's d_base_out /
 * total_bytes_out, iengine.cu:117) and its RoPE tables (fp32 [rows][head_dim/2]). */
int qie_engine_arena(const qie_engine* e, void** base, int64_t* bytes);
int qie_engine_rope_tables(const qie_engine* e, const float** rope_cos, const float** rope_sin,
                           int32_t* rows);
/* Time `iters` launches of one of the decode step's kernels with hipEvents on
 * the engine stream (which: 0 = gate/up GEMV, 1 = down GEMV, 2 = QKV GEMV,
 * 3 = O GEMV, 4 = lm_head GEMV, 5 = attention; the layer GEMVs cycle through
 * layers 1..L-1 so no weight stays cache-resident; 6 = the persistent layer stack of decode
 * mode 1, all layers per launch, the sequence state restored afterwards).  Returns the average
 * microseconds per launch and the algorithmic bytes per launch. */
int qie_batch_time_kernel(qie_batch* b, int32_t which, int32_t iters, double* avg_us,
                          double* bytes);
/* One decode step run eagerly (as qie_decode_step) that also copies the residual stream
 * into host_x: bf16 [2 n_layers + 1][batch][hidden], slot 0 = the step's input row, slot
 * 2l + 1 = after layer l's attention block (O-proj + residual), 2l + 2 = after its MLP
 * block (down-proj + residual).  Parity diagnostics (tools/flip_attrib.py). */
int qie_batch_debug_step(qie_batch* b, const qie_sampling* smp, int32_t* next_ids, void* host_x);

#ifdef __cplusplus
}
#endif

#endif /* QIE_ENGINE_H */
