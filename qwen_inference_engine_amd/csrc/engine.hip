// engine.hip — qie engine: weight arena, per-batch KV cache and activations,
// prefill and hipGraph-captured decode.
//
// Reference driver being replaced: llm() (layers/src/qwen_main.cu:64-417),
// create_new_sequence (iengine.cu:25-47), initialize_model_buffers
// (utills.cu:4-129), load_all_weights_to_gpu_chunked (iengine.cu:117-223),
// page list helpers (iengine.cu:73-109).  Op order per layer follows
// qwen_main.cu:77-217 (prefill) / :271-359 (decode):
//   rms -> q,k,v -> [qk-norm] -> RoPE -> KV write -> attention -> o -> +res ->
//   rms -> up, gate -> silu*up -> down -> +res;  final rms -> lm_head -> sample.
// MI355X design: the decode step is 5 launches per layer
//   [rms+QKV(+bias) GEMV] [qk-norm+RoPE+KV append] [attention(+combine)]
//   [O GEMV + residual] [rms+gate/up GEMV + SwiGLU] [down GEMV + residual]
// plus [rms+lm_head GEMV + fused arg-max] [finalize: id, position, next
// embedding], captured once into a hipGraph; positions and token ids live in
// device memory so the graph replays without host edits.
#include "qie_common.hpp"
#include "../../include/qie/qie_engine.h"
#include "qie_index.hpp"
#include "qie_comm.hpp"

#include <chrono>
#include <cstring>
#include <fstream>
#include <vector>

namespace qie {
int gemv(const qie_linear_args* a, hipStream_t st);
int gemv_rope(const qie_linear_args* a, const int32_t* pos, const float* cs, const float* sn, int hd, int64_t rows,
              hipStream_t st);
int gemm(const qie_linear_args* a, hipStream_t st);
bool dec8_applies(const qie_linear_args* a);
int dec8_reserve(hipStream_t st);
bool persist_supported(const qie_model_spec& s, int B, int tp, bool fp8, bool paged, int ncu, const char** why);
size_t persist_attn_table_bytes(int n_layers);
int persist_attn_table(const qie_model_spec& s, const qie_layer_weights* h_layers, const void* qkv_scratch,
                       const int32_t* pos, const float* rope_cos, const float* rope_sin, const qie_kv_cache* cache,
                       void* dec_ws, void* d_attp, hipStream_t st);
int persist_decode_launch(const qie_model_spec& s, const qie_layer_weights* d_layers, const void* d_attp,
                          uint16_t* x_res, unsigned long long* granules, const unsigned* epoch, unsigned* err,
                          const int32_t* pos, int splits_target, unsigned long long* ts, hipStream_t st);
int64_t persist_granule_count(const qie_model_spec& s);
int persist_ts_slots();
}  // namespace qie


using namespace qie;

// Tensor-parallel shard of one rank (tp = 1: the whole model).  Column-parallel
// QKV (by heads) and gate/up (by I), row-parallel O and down, vocab-parallel lm_head;
// embedding, norms and the residual stream are replicated.
// Heads: n_kv_heads % tp == 0 splits both head kinds evenly; otherwise, when
// tp % n_kv_heads == 0, every kv head is replicated on rep = tp / n_kv_heads ranks and
// the G = n_heads / n_kv_heads q heads of its group are split among those ranks as
// evenly as they go (the first G % rep ranks take one more): Qwen2-7B (28 / 4 heads) at
// TP 8 gives q heads 4,3,4,3,... with one kv head each.  Every q head lives
// on exactly one rank, so the row-parallel O all-reduce still sums each head once.
struct TpShard {
    int tp = 1, rank = 0;
    int nq = 0, nkv = 0, ffn = 0, vocab = 0;   // local counts
    int q0 = 0, kv0 = 0;                        // first global q / kv head of this rank
    int64_t vocab0 = 0;                         // first global vocab row of this rank
};

// Head split of rank `rank` of `tp` (see TpShard); false when the heads do not shard.
static bool shard_heads(int nq, int nkv, int tp, int rank, TpShard& sh) {
    if (nkv % tp == 0 && nq % tp == 0) {
        sh.nq = nq / tp;
        sh.nkv = nkv / tp;
        sh.q0 = rank * sh.nq;
        sh.kv0 = rank * sh.nkv;
        return true;
    }
    if (tp % nkv != 0) return false;
    const int rep = tp / nkv, G = nq / nkv, g = rank / rep, sub = rank % rep;
    if (rep > G) return false;   // a rank without q heads
    const int base = G / rep, extra = G % rep;
    sh.nkv = 1;
    sh.kv0 = g;
    sh.nq = base + (sub < extra ? 1 : 0);
    sh.q0 = g * G + sub * base + std::min(sub, extra);
    return true;
}

struct qie_engine {
    qie_model_spec spec{};   // the full model
    TpShard sh;              // this rank's shard
    qie_comm* comm = nullptr;
    qie_engine_opts opts{};
    hipStream_t stream = nullptr;
    void* arena = nullptr;
    size_t arena_bytes = 0;
    qie_index* index = nullptr;
    std::vector<qie_layer_weights> layers;
    qie_model_weights w{};
    bool have_weights = false;
    bool fp8 = false;            // linear weights are e4m3 + row scales (fp8_arena)
    bool fp8_t16 = false;        // ... and the decode projections in the 16-row tiled layout
    bool fp8_t16_head = false;   // ... and the lm_head too
    // fp8 engines: the same (dequantised) layer weights as bf16, in place in the arena —
    // prefill's MFMA GEMMs read these (compute-bound: the LDS-DMA bf16 kernel), decode's
    // bandwidth-bound GEMVs the fp8 codes; both compute the one dequantised model
    std::vector<qie_layer_weights> layers_pf;
    void* fp8_arena = nullptr;
    float* rope_cos = nullptr;
    float* rope_sin = nullptr;
    int rope_rows = 0;
};

struct qie_batch {
    qie_engine* e = nullptr;
    int B = 0, max_ctx = 0;
    uint16_t* kc = nullptr;
    uint16_t* vc = nullptr;
    int64_t seq_stride = 0;
    int run_pad = 0;             // contiguous: run = max_ctx + run_pad tokens (dev A/B)
    int32_t* d_pos = nullptr;
    float* d_rope_cur = nullptr;   // [B][rope_cur_stride(hd)]: RoPE row of each slot's current position
    int32_t* d_step = nullptr;
    int32_t* d_hist = nullptr;
    int32_t* d_ids = nullptr;
    unsigned long long* d_keys = nullptr;
    uint16_t* x_res = nullptr;
    uint16_t* qkv = nullptr;
    uint16_t* q = nullptr;
    uint16_t* att = nullptr;
    uint16_t* h = nullptr;
    uint16_t* xn = nullptr;     // [B][H] RMS-normed rows feeding the batched (B >= 2) projections
    uint16_t* logits = nullptr;
    void* attn_ws = nullptr;
    void* dec_ws = nullptr;     // fused decode attention: split partials + zeroed counters
    void* samp_ws = nullptr;
    // tensor parallel: fp32 partials of the row-parallel projections, gathered logits
    float* part = nullptr;            // [B][H]
    uint16_t* logits_full = nullptr;  // [B][V]
    uint16_t* gather_tmp = nullptr;   // [tp][B][V/tp]
    float* pf_part = nullptr;         // [pf_rows][H]
    std::vector<int32_t> h_pos;
    // prefill scratch
    int64_t pf_rows = 0;
    uint16_t *pf_x = nullptr, *pf_hn = nullptr, *pf_qkv = nullptr, *pf_q = nullptr, *pf_att = nullptr,
             *pf_h = nullptr;
    int32_t *pf_pos = nullptr, *pf_ids = nullptr;
    uint8_t *pf_q8 = nullptr, *pf_e8 = nullptr;   // fp8 prefill (opts.prefill_fp8): codes [rows][max K], exps [rows]
    void* pf_attn_ws = nullptr;
    int64_t pf_attn_ws_bytes = 0;   // the split workspace depends on n (short prompts split), not on n <= pf_rows
    // paged KV (qie_batch_create_paged): pool pages of page_tokens tokens, block table
    // [B][max_pages] on device and host, free list, pages held per slot
    int page_tokens = 0, max_pages = 0, n_pages = 0;
    int32_t* d_table = nullptr;
    std::vector<int32_t> h_table, free_pages, held;
    std::vector<char> idle;
    bool table_dirty = false;
    // decode graph
    hipGraphExec_t gexec = nullptr;
    qie_sampling gs{};
    bool graph_ok = false;
    // qie_batch_debug_step: while set, the decode enqueue copies the residual stream after every
    // attention block and every MLP block into dbg_x ([2L + 1][B][H] bf16; slot 0 = the input)
    uint16_t* dbg_x = nullptr;
    // decode structure (qie_batch_set_decode_mode): 0 = five launches per layer, 1 = the whole
    // layer stack as one persistent launch (k_persist.hip).  pk_mem: hand-off granules, then the
    // step epoch and the error word (zeroed once; the finalize kernel advances the epoch)
    int decode_mode = 0;
    void* pk_mem = nullptr;
    qie_layer_weights* d_layers = nullptr;
    void* d_attp = nullptr;      // the attention role's parameters per layer (persist_attn_table)
    unsigned long long* pk_ts = nullptr;   // qie_batch_pk_trace: phase timestamps [cu][layer][slots]
};

namespace qie {

// ------------------------------------------------------------ small kernels
// Step finalisation: chosen id -> token history, position + 1, sample step + 1,
// next step's input row x_res[m] = E[id] (embedding_matrix_func, decode branch
// qwen_main.cu:259-268, without the host round trip).
// The RoPE table row of a slot's current position, kept beside the position (tagged with it)
// so that the decode attention's prologue loads need not wait for the position
// (DecodeAttnParams::rc).  Every kernel that sets a position also writes the row.
struct RopeCurArgs {
    float* rc;
    const float* cs;
    const float* sn;
    int hd, rows;
};
__device__ __forceinline__ void write_rope_cur(const RopeCurArgs& r, int m, int p) {
    if (!r.rc) return;
    float* o = r.rc + (int64_t)m * rope_cur_stride(r.hd);
    const bool ok = p >= 0 && p < r.rows;
    const int h2 = r.hd / 2;
    for (int t = threadIdx.x; t < h2; t += blockDim.x) {
        o[8 + t] = ok ? r.cs[(int64_t)p * h2 + t] : 0.f;
        o[8 + h2 + t] = ok ? r.sn[(int64_t)p * h2 + t] : 0.f;
    }
    if (threadIdx.x == 0) o[0] = __int_as_float(ok ? p : -1);
}

__global__ __launch_bounds__(256) void finalize_kernel(int m0, unsigned long long* keys, const int32_t* ids_in,
                                                       int32_t* ids_out, int32_t* pos, int32_t* step,
                                                       int32_t* hist, int hist_stride, const uint4* E,
                                                       uint4* x_res, int64_t H8, int32_t vocab, RopeCurArgs rca,
                                                       unsigned* pk_epoch) {
    const int m = m0 + blockIdx.x;
    // the persistent step's hand-off epoch advances once per step (k_persist.hip tags)
    if (pk_epoch && blockIdx.x == 0 && threadIdx.x == 0) *pk_epoch += 1u;
    int32_t tok = keys ? key_idx(keys[m]) : ids_in[m];
    const int32_t p = pos[m];
    __syncthreads();
    if (tok < 0 || tok >= vocab) tok = 0;
    if (threadIdx.x == 0) {
        if (keys) keys[m] = 0ull;
        if (p + 1 < hist_stride) hist[(int64_t)m * hist_stride + p + 1] = tok;
        pos[m] = p + 1;
        step[m] = step[m] + 1;
        ids_out[m] = tok;
    }
    write_rope_cur(rca, m, p + 1);
    const uint4* src = E + (int64_t)tok * H8;
    uint4* dst = x_res + (int64_t)m * H8;
    for (int64_t i = threadIdx.x; i < H8; i += 256) dst[i] = src[i];
}

__global__ void set_state_kernel(int m, int32_t pos_v, int32_t step_v, int32_t tok, int32_t* pos,
                                 int32_t* step, int32_t* hist, int hist_stride, const uint4* E,
                                 uint4* x_res, int64_t H8, int write_row, RopeCurArgs rca) {
    write_rope_cur(rca, m, pos_v);
    if (threadIdx.x == 0) {
        pos[m] = pos_v;
        step[m] = step_v;
        if (pos_v >= 0 && pos_v < hist_stride) hist[(int64_t)m * hist_stride + pos_v] = tok;
    }
    if (write_row)
        for (int64_t i = threadIdx.x; i < H8; i += blockDim.x) x_res[(int64_t)m * H8 + i] = E[(int64_t)tok * H8 + i];
}

// positions of n_seqs equal-length prompts laid end to end: row i sits at i % len
__global__ void iota_kernel(int32_t* p, int n, int len) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i % len;
}

// prompt z (blockIdx.y) of len ids -> history row z of dst (stride dst_stride)
__global__ void copy_ids_kernel(const int32_t* src, int32_t* dst, int len, int64_t dst_stride) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) dst[blockIdx.y * dst_stride + i] = src[(int64_t)blockIdx.y * len + i];
}

static int dmalloc(void** p, size_t bytes) {
    QIE_HIP(hipMalloc(p, bytes < 16 ? 16 : bytes));
    return 0;
}

static RopeCurArgs rope_cur_args(const qie_batch* b) {
    const qie_engine* e = b->e;
    return RopeCurArgs{b->d_rope_cur, e->rope_cos, e->rope_sin, (int)e->spec.head_dim, e->rope_rows};
}

// KV descriptor of the batch's sequences seq0.. (kernels see them as sequences 0..)
static qie_kv_cache batch_cache(const qie_batch* b, int seq0) {
    const qie_engine* e = b->e;
    qie_kv_cache c{};
    c.n_layers = e->spec.n_layers;
    c.n_kv_heads = e->sh.nkv;
    c.head_dim = e->spec.head_dim;
    c.max_ctx = b->max_ctx + b->run_pad;   // the run length (positions stay below b->max_ctx)
    c.seq_stride = b->seq_stride;
    if (b->d_table) {
        c.k = b->kc;
        c.v = b->vc;
        c.block_table = b->d_table + (int64_t)seq0 * b->max_pages;
        c.page_tokens = b->page_tokens;
        c.max_pages = b->max_pages;
    } else {
        c.k = b->kc + (int64_t)seq0 * b->seq_stride;
        c.v = b->vc + (int64_t)seq0 * b->seq_stride;
    }
    return c;
}

// ------------------------------------------------------------ page pool
// Host-side allocator of the paged batch.  Decisions are deterministic, so the
// tensor-parallel ranks (each holding its own heads' pages) stay in step.
static int ensure_pages(qie_batch* b, int seq, int64_t ntok) {
    if (!b->d_table) return 0;
    const int64_t need = (ntok + b->page_tokens - 1) / b->page_tokens;
    QIE_REQUIRE(need <= b->max_pages, "KV pages: %lld tokens exceed max_ctx %d", (long long)ntok, b->max_ctx);
    int64_t extra = need - b->held[seq];
    QIE_REQUIRE(extra <= (int64_t)b->free_pages.size(), "KV pages: sequence %d needs %lld more pages, %zu free",
                seq, (long long)extra, b->free_pages.size());
    for (; b->held[seq] < need; b->held[seq]++) {
        b->h_table[(int64_t)seq * b->max_pages + b->held[seq]] = b->free_pages.back();
        b->free_pages.pop_back();
        b->table_dirty = true;
    }
    return 0;
}

static void drop_pages(qie_batch* b, int seq) {
    if (!b->d_table) return;
    for (int i = b->held[seq] - 1; i >= 0; i--) {
        int32_t& t = b->h_table[(int64_t)seq * b->max_pages + i];
        b->free_pages.push_back(t);
        t = 0;   // scratch page
    }
    b->held[seq] = 0;
    b->table_dirty = true;
}

// uploads the host table (ordered after everything already on the stream)
static int flush_table(qie_batch* b) {
    if (!b->d_table || !b->table_dirty) return 0;
    // on the engine stream (non-blocking: a legacy-null-stream copy is not ordered before its
    // kernels), complete before the host table may change again
    QIE_HIP(hipMemcpyAsync(b->d_table, b->h_table.data(), b->h_table.size() * 4, hipMemcpyHostToDevice, b->e->stream));
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    b->table_dirty = false;
    return 0;
}


static int build_rope(qie_engine* e) {
    const int hd = e->spec.head_dim, half = hd / 2, rows = e->opts.max_ctx;
    std::vector<float> c((size_t)rows * half), s((size_t)rows * half);
    QIE_TRY(qie_rope_table_host(c.data(), s.data(), rows, hd, e->spec.rope_theta, e->spec.numerics));
    QIE_TRY(dmalloc((void**)&e->rope_cos, c.size() * 4));
    QIE_TRY(dmalloc((void**)&e->rope_sin, s.size() * 4));
    QIE_HIP(hipMemcpyAsync(e->rope_cos, c.data(), c.size() * 4, hipMemcpyHostToDevice, e->stream));
    QIE_HIP(hipMemcpyAsync(e->rope_sin, s.data(), s.size() * 4, hipMemcpyHostToDevice, e->stream));
    QIE_HIP(hipStreamSynchronize(e->stream));   // the host tables go out of scope
    e->rope_rows = rows;
    return 0;
}

static int check_align(const void* p, const char* what, int layer) {
    if (((uintptr_t)p) % 16 != 0)
        return fail(-22, "weight %s (layer %d) is not 16-byte aligned", what, layer);
    return 0;
}

// fp8 weights (opts.weight_fp8): every linear weight and the lm_head are quantised on
// device into a second arena (OCP e4m3 codes + power-of-two row scales, qie_ops.h) and
// the layer pointers switched to it; embeddings, norms and biases stay bf16 in the
// first arena (a tied embedding keeps its bf16 copy for the token gather).
// own_arena: the bf16 weights live in the engine's arena (synthetic init, weights.bin), so
// they may be rewritten with their dequantisation for prefill; caller-owned weights
// (qie_engine_set_weights) are never written — their prefill takes the fp8 GEMM path.
static int quantize_weights_fp8(qie_engine* e, bool own_arena) {
    QIE_REQUIRE(e->sh.tp == 1, "fp8 weights with tensor parallelism are not supported yet");
    const qie_model_spec& s = e->spec;
    const int64_t H = s.hidden, QD = (int64_t)s.n_heads * s.head_dim, KD = (int64_t)s.n_kv_heads * s.head_dim;
    const int64_t I = s.ffn, V = s.vocab;
    QIE_REQUIRE(H % 16 == 0 && QD % 16 == 0 && I % 16 == 0, "fp8 weights need hidden, q dim and ffn % 16 == 0");
    struct Slot { const void** p; int64_t rows, cols; };
    std::vector<Slot> ts;
    for (auto& L : e->layers) {
        ts.push_back({&L.wq, QD, H});
        ts.push_back({&L.wk, KD, H});
        ts.push_back({&L.wv, KD, H});
        ts.push_back({&L.wo, H, QD});
        ts.push_back({&L.w_gate, I, H});
        ts.push_back({&L.w_up, I, H});
        ts.push_back({&L.w_down, H, I});
    }
    ts.push_back({&e->w.lm_head, V, H});
    size_t total = 0;
    for (auto& t : ts) total += (size_t)((qie_fp8_weight_bytes(t.rows, t.cols) + 255) / 256 * 256);
    if (e->fp8_arena) hipFree(e->fp8_arena);
    e->fp8_arena = nullptr;
    QIE_HIP(hipMalloc(&e->fp8_arena, total));
    char* dst = (char*)e->fp8_arena;
    e->layers_pf.clear();
    if (own_arena) e->layers_pf = e->layers;   // bf16 arena pointers, rewritten below with the dequantised values
    for (auto& t : ts) {
        const void* src = *t.p;
        QIE_TRY(qie_quantize_fp8(src, t.rows, t.cols, dst, e->stream));
        // layer weights: the arena copy becomes the exact dequantisation (prefill reads it);
        // the lm_head is left alone (a tied one is also the embedding table)
        if (own_arena && t.p != &e->w.lm_head)
            QIE_TRY(qie_dequantize_fp8(dst, t.rows, t.cols, const_cast<void*>(src), e->stream));
        *t.p = dst;
        dst += (qie_fp8_weight_bytes(t.rows, t.cols) + 255) / 256 * 256;
    }
    QIE_HIP(hipStreamSynchronize(e->stream));
    e->w.layers = e->layers.data();
    e->fp8 = true;
    e->fp8_t16 = e->fp8_t16_head = false;
    // The decode projections go to the 16-row tiled layout (qie_fp8_tile16: every 1-KiB wave
    // load of the batched-decode kernel contiguous) when that kernel takes every one of them
    // at any batch (it is then their only reader; prefill reads the dequantised bf16 copy, so
    // the engine must own its arena).  QIE_FP8_T16=0 (dev) keeps the plain layout.
    if (own_arena && dev_env("QIE_FP8_T16", 1) != 0) {
        auto ok = [&](int64_t K, int64_t N, int64_t s0, int64_t s1, int64_t s2, bool norm, int epi) {
            qie_linear_args a;
            std::memset(&a, 0, sizeof(a));
            a.flags = QIE_LINEAR_FP8 | QIE_LINEAR_FP8_T16;
            a.M = 1; a.K = K; a.N = N; a.ldx = K;
            a.seg_rows[0] = s0; a.seg_rows[1] = s1; a.seg_rows[2] = s2;
            a.norm_w = norm ? (const void*)e : nullptr;   // (only tested for presence)
            a.epilogue = epi;
            return dec8_applies(&a);
        };
        const bool all = ok(H, QD + 2 * KD, QD, KD, KD, true, QIE_EPI_STORE) && ok(QD, H, H, 0, 0, false, QIE_EPI_RESIDUAL) &&
                         ok(H, I, I, I, 0, true, QIE_EPI_SWIGLU) && ok(I, H, H, 0, 0, false, QIE_EPI_RESIDUAL);
        // the vocabulary projection too: its readers (the decode step's and the prefill's
        // last-row heads, <= 8 rows) run the skinny kernel, which reads the tiled layout
        // (through the batched-decode kernel instead — one 7-wave block per CU, ~37 tiles
        // each — config 4's lm_head took 168.9 vs 119-120 µs plain); dev QIE_FP8_T16_HEAD=0
        // keeps it plain
        const bool head = all && dev_env("QIE_FP8_T16_HEAD", 1) != 0 && H % 64 == 0 && V % 16 == 0 &&
                          (size_t)8 * (H + 8) * 2 <= 120 * 1024;
        if (all) {
            size_t big = 0;
            for (auto& t : ts)
                if (t.p != &e->w.lm_head || head) big = std::max<size_t>(big, (size_t)qie_fp8_weight_bytes(t.rows, t.cols));
            void* tmp = nullptr;
            QIE_TRY(dmalloc(&tmp, big));
            int rc = 0;
            for (auto& t : ts) {
                if (t.p == &e->w.lm_head && !head) continue;
                const size_t nb = (size_t)qie_fp8_weight_bytes(t.rows, t.cols);
                rc = qie_fp8_tile16(*t.p, t.rows, t.cols, tmp, e->stream);
                if (rc) break;
                if (hipMemcpyAsync(const_cast<void*>(*t.p), tmp, nb, hipMemcpyDeviceToDevice, e->stream) != hipSuccess) {
                    rc = fail(-5, "fp8 tiling: copy failed");
                    break;
                }
            }
            if (!rc && hipStreamSynchronize(e->stream) != hipSuccess) rc = fail(-5, "fp8 tiling: synchronize failed");
            hipFree(tmp);
            if (rc) return rc;
            e->fp8_t16 = true;
            e->fp8_t16_head = head;
        }
    }
    return 0;
}

// Resolve role pointers from the reference index (short_name, layer) ->
// arena + data_offsets[0]  (assign_weight_pointer, helpers.cuh:19-30).
static int bind_from_index(qie_engine* e) {
    const qie_model_spec& s = e->spec;
    char* base = (char*)e->arena;
    auto get = [&](const char* sn, int layer, const void** out, bool required) -> int {
        const qie_index_entry* t = index_find(e->index, sn, layer);
        if (!t) {
            if (required) return fail(-22, "tensor %s (layer %d) missing from index", sn, layer);
            *out = nullptr;
            return 0;
        }
        *out = base + t->off0;
        return check_align(*out, sn, layer);
    };
    e->layers.assign(s.n_layers, qie_layer_weights{});
    for (int l = 0; l < s.n_layers; l++) {
        qie_layer_weights& L = e->layers[l];
        QIE_TRY(get("input_layernorm.weight", l, &L.attn_norm, true));
        QIE_TRY(get("self_attn.q_proj.weight", l, &L.wq, true));
        QIE_TRY(get("self_attn.k_proj.weight", l, &L.wk, true));
        QIE_TRY(get("self_attn.v_proj.weight", l, &L.wv, true));
        QIE_TRY(get("self_attn.q_proj.bias", l, &L.bq, s.qkv_bias != 0));
        QIE_TRY(get("self_attn.k_proj.bias", l, &L.bk, s.qkv_bias != 0));
        QIE_TRY(get("self_attn.v_proj.bias", l, &L.bv, s.qkv_bias != 0));
        QIE_TRY(get("self_attn.q_norm.weight", l, &L.q_norm, s.qk_norm != 0));
        QIE_TRY(get("self_attn.k_norm.weight", l, &L.k_norm, s.qk_norm != 0));
        QIE_TRY(get("self_attn.o_proj.weight", l, &L.wo, true));
        QIE_TRY(get("post_attention_layernorm.weight", l, &L.ffn_norm, true));
        QIE_TRY(get("mlp.gate_proj.weight", l, &L.w_gate, true));
        QIE_TRY(get("mlp.up_proj.weight", l, &L.w_up, true));
        QIE_TRY(get("mlp.down_proj.weight", l, &L.w_down, true));
    }
    QIE_TRY(get("embed_tokens.weight", -1, &e->w.embed, true));
    QIE_TRY(get("norm.weight", -1, &e->w.final_norm, true));
    if (s.tie_embeddings && e->sh.tp == 1) e->w.lm_head = e->w.embed;
    else QIE_TRY(get("logits", -1, &e->w.lm_head, true));
    e->w.n_layers = s.n_layers;
    e->w.layers = e->layers.data();
    e->have_weights = true;
    return e->opts.weight_fp8 ? quantize_weights_fp8(e, true) : 0;
}

// ------------------------------------------------------------- enqueue helpers
// every weight linear of the engine: fp8 weights when the engine quantised them
static qie_linear_args lin_base(const qie_engine* e) {
    qie_linear_args a;
    std::memset(&a, 0, sizeof(a));
    a.flags = e->fp8 ? QIE_LINEAR_FP8 : 0;
    return a;
}
// the layer projections (QKV, O, gate/up, down): + the tiled-layout flag where they are tiled
static qie_linear_args lin_proj(const qie_engine* e) {
    qie_linear_args a = lin_base(e);
    if (e->fp8_t16) a.flags |= QIE_LINEAR_FP8_T16;
    return a;
}

// The exchange steps go through the communicator under tensor parallelism, and at world 1
// when the engine was asked to (opts.comm_always: the captured-collective path on one GPU).
static bool use_comm(const qie_engine* e) { return e->comm && (e->sh.tp > 1 || e->opts.comm_always); }

// Device -> host on the engine stream (then wait): never the legacy null stream, whose
// implicit ordering against every blocking stream HIP refuses while ANY thread of the process
// captures a graph (the TP ranks of one process capture their decode graphs concurrently).
static hipError_t d2h(const qie_engine* e, void* dst, const void* src, size_t bytes) {
    hipError_t he = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    return he;
}

// After a stream synchronisation: a device-side exchange failure (the peer backend's bounded
// wait) makes the call fail instead of returning ids computed from a partial exchange.
static int comm_check(const qie_engine* e, const char* who) {
    if (!use_comm(e)) return 0;
    const int err = e->comm->error_state(e->stream);
    if (err) return fail(-7, "%s: tensor-parallel exchange failed on the device (error word %d: a peer rank did "
                             "not arrive within the bounded wait); the communicator is unusable", who, err);
    return 0;
}

// Row-parallel projection epilogue under tensor parallelism: fp32 partials -> all-reduce
// -> x = bf16(x + bf16(sum)); the single-GPU path fuses the residual into the GEMV/GEMM.
static int row_parallel(qie_batch* b, qie_linear_args& a, uint16_t* x, float* part, int64_t rows) {
    qie_engine* e = b->e;
    if (!use_comm(e)) {
        a.y = x;
        a.epilogue = QIE_EPI_RESIDUAL;
        return qie_linear(&a, e->stream);
    }
    a.y = part;
    a.epilogue = QIE_EPI_F32;
    const int64_t n = rows * e->spec.hidden;
    // peer backend, one row: the GEMV's epilogue pushes each finished output straight into
    // every rank's tagged exchange slot (the send overlaps the projection's tail), and the
    // exchange kernel only waits, reduces and adds (comm.hip peer_tag_kernel)
    PeerPush pp;
    if (rows == 1 && e->comm->peer_push(&pp, n)) {
        set_gemv_push(&pp);
        const int rc = qie_linear(&a, e->stream);
        const bool taken = gemv_push_taken();
        set_gemv_push(nullptr);
        QIE_TRY(rc);
        if (taken) return e->comm->allreduce_residual_pushed(x, n, e->stream);
        return e->comm->allreduce_residual_bf16(part, x, n, e->stream);
    }
    QIE_TRY(qie_linear(&a, e->stream));
    return e->comm->allreduce_residual_bf16(part, x, n, e->stream);   // one kernel on the peer backend
}

// Batched rows (2 <= M <= 16, the skinny MFMA kernel): RMSNorm the M rows once into b->xn
// (qie_rmsnorm, normalization.cu:5-25 semantics) and feed the projection plain rows.  The
// skinny kernel's fused norm prologue recomputed every row's norm in every workgroup and
// cost 13-16 us per launch at B = 8 (tools/ubench_b8.py, QIE_SKINNY_DBG); M = 1 keeps the
// GEMV's fused x-first prologue.  QIE_PRENORM=0 restores the fused form (A/B).
static int prenorm(qie_batch* b, qie_linear_args& a, int64_t M) {
    static const int on = dev_env("QIE_PRENORM", 1);
    if (!on || M < 2 || M > 16 || !a.norm_w) return 0;
    if (dec8_applies(&a) && dev_env("QIE_DEC8_PRENORM", 0) == 0) return 0;   // the fp8 batched-decode kernel fuses the norm
    QIE_TRY(qie_rmsnorm(a.x, a.norm_w, b->xn, M, a.K, a.norm_eps, a.numerics, b->e->stream));
    a.x = b->xn;
    a.ldx = a.K;
    a.norm_w = nullptr;
    return 0;
}

// batch 1, REF numerics, no qk-norm (Qwen2): the decode QKV projection's epilogue rotates q
// and k (gemv_rope), so the attention's critical path loses the position -> RoPE-table round
// trip (QIE_ATTN_PREROPED)
static bool rope_in_projection(const qie_batch* b) {
    const qie_model_spec& s = b->e->spec;
    return b->B == 1 && !s.qk_norm && s.numerics == QIE_NUMERICS_REF && dev_env("QIE_ROPE_IN_PROJ", 0) != 0;
}

// qie_batch_debug_step: residual stream snapshot `slot` (eager step only, never captured)
static int dbg_snap(qie_batch* b, int slot) {
    if (!b->dbg_x) return 0;
    const int64_t n = (int64_t)b->B * b->e->spec.hidden;
    QIE_HIP(hipMemcpyAsync(b->dbg_x + slot * n, b->x_res, (size_t)n * 2, hipMemcpyDeviceToDevice, b->e->stream));
    return 0;
}

static int enqueue_layer_decode(qie_batch* b, int l) {
    qie_engine* e = b->e;
    const qie_model_spec& s = e->spec;
    const qie_layer_weights& L = e->layers[l];
    hipStream_t st = e->stream;
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)e->sh.nq * hd, KD = (int64_t)e->sh.nkv * hd;
    const int64_t QKVD = QD + 2 * KD, I = e->sh.ffn, B = b->B;
    const qie_kv_cache cache = batch_cache(b, 0);

    qie_linear_args a = lin_proj(e);
    a.x = b->x_res; a.ldx = H;
    a.w[0] = L.wq; a.w[1] = L.wk; a.w[2] = L.wv;
    a.bias[0] = L.bq; a.bias[1] = L.bk; a.bias[2] = L.bv;
    a.seg_rows[0] = QD; a.seg_rows[1] = KD; a.seg_rows[2] = KD;
    a.M = B; a.K = H; a.N = QKVD;
    a.y = b->qkv; a.ldy = QKVD;
    a.epilogue = QIE_EPI_STORE;
    a.norm_w = L.attn_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
    QIE_TRY(prenorm(b, a, B));
    const bool rope_in_proj = rope_in_projection(b);
    if (rope_in_proj) QIE_TRY(gemv_rope(&a, b->d_pos, e->rope_cos, e->rope_sin, (int)hd, QD + KD, st));
    else QIE_TRY(gemv(&a, st));

    set_decode_rope_cur(b->d_rope_cur);
    const int arc = qie_attention_decode(b->qkv, B, b->d_pos, L.q_norm, L.k_norm, e->rope_cos, e->rope_sin, e->sh.nq,
                                         &cache, l, s.rms_eps, s.numerics | (rope_in_proj ? QIE_ATTN_PREROPED : 0),
                                         b->att, b->dec_ws, st);
    set_decode_rope_cur(nullptr);
    QIE_TRY(arc);
    a = lin_proj(e);
    a.x = b->att; a.ldx = QD;
    a.w[0] = L.wo; a.seg_rows[0] = H;
    a.M = B; a.K = QD; a.N = H;
    a.ldy = H;
    QIE_TRY(row_parallel(b, a, b->x_res, b->part, B));
    QIE_TRY(dbg_snap(b, 2 * l + 1));

    a = lin_proj(e);
    a.x = b->x_res; a.ldx = H;
    a.w[0] = L.w_gate; a.w[1] = L.w_up; a.seg_rows[0] = I; a.seg_rows[1] = I;
    a.M = B; a.K = H; a.N = I;
    a.y = b->h; a.ldy = I;
    a.epilogue = QIE_EPI_SWIGLU;
    a.norm_w = L.ffn_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
    QIE_TRY(prenorm(b, a, B));
    QIE_TRY(gemv(&a, st));

    a = lin_proj(e);
    a.x = b->h; a.ldx = I;
    a.w[0] = L.w_down; a.seg_rows[0] = H;
    a.M = B; a.K = I; a.N = H;
    a.ldy = H;
    QIE_TRY(row_parallel(b, a, b->x_res, b->part, B));
    return dbg_snap(b, 2 * l + 2);
}

static bool is_greedy(const qie_sampling* s) { return !s || s->top_k <= 1 || !(s->temperature > 0.f); }

// tmp[r][i][j] (rank r's logit shard of row i) -> full[m0 + i][r * Vl + j]
__global__ void unshard_rows_kernel(const uint16_t* __restrict__ tmp, uint16_t* __restrict__ full, int tp, int M,
                                    int64_t Vl, int64_t V, int m0) {
    const int64_t n = (int64_t)tp * M * Vl;
    for (int64_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
        const int64_t j = k % Vl, i = (k / Vl) % M, r = k / (Vl * M);
        full[(m0 + i) * V + r * Vl + j] = tmp[k];
    }
}

// all-gather of the vocab-parallel logits of rows [m0, m0 + M) into logits_full
static int gather_logits(qie_batch* b, int m0, int M) {
    qie_engine* e = b->e;
    const int64_t Vl = e->sh.vocab;
    QIE_TRY(e->comm->allgather(b->logits + (int64_t)m0 * Vl, b->gather_tmp, (int64_t)M * Vl * 2, e->stream));
    const int64_t n = (int64_t)e->sh.tp * M * Vl;
    hipLaunchKernelGGL(unshard_rows_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                       e->stream, b->gather_tmp, b->logits_full, e->sh.tp, M, Vl, (int64_t)e->spec.vocab, m0);
    QIE_LAUNCH_CHECK();
    return 0;
}

// the persistent step's words behind its granules: [0] step epoch, [1] error word
static unsigned* pk_epoch_ptr(const qie_batch* b) {
    return (unsigned*)((unsigned long long*)b->pk_mem + persist_granule_count(b->e->spec));
}

// lm_head over rows [m0, m0+M) of x (already the residual stream), then the
// sampler; leaves ids in d_keys (greedy) or d_ids.
static int enqueue_head(qie_batch* b, const uint16_t* x, int64_t ldx, int m0, int M, const qie_sampling* smp) {
    qie_engine* e = b->e;
    const qie_model_spec& s = e->spec;
    hipStream_t st = e->stream;
    const int64_t Vl = e->sh.vocab;
    qie_linear_args a = lin_base(e);
    if (e->fp8_t16_head) a.flags |= QIE_LINEAR_FP8_T16;
    a.x = x; a.ldx = ldx;
    a.w[0] = e->w.lm_head; a.seg_rows[0] = Vl;
    a.M = M; a.K = s.hidden; a.N = Vl;
    a.y = b->logits + (int64_t)m0 * Vl; a.ldy = Vl;
    a.epilogue = QIE_EPI_STORE;
    a.norm_w = e->w.final_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
    QIE_TRY(prenorm(b, a, M));
    const bool greedy = is_greedy(smp);
    if (greedy) {
        a.argmax_keys = (uint64_t*)(b->d_keys + m0);
        a.key_col0 = e->sh.vocab0;   // keys carry global vocab ids
    }
    QIE_TRY(gemv(&a, st));
    if (greedy && use_comm(e)) QIE_TRY(e->comm->allreduce_max_u64((uint64_t*)(b->d_keys + m0), M, st));
    if (!greedy) {
        const uint16_t* lg = b->logits + (int64_t)m0 * Vl;
        if (use_comm(e)) {   // every rank samples the same draw from the gathered row
            QIE_TRY(gather_logits(b, m0, M));
            lg = b->logits_full + (int64_t)m0 * s.vocab;
        }
        QIE_TRY(qie_sample(lg, M, s.vocab, s.vocab, smp, b->d_step + m0, b->d_ids + m0, b->samp_ws, st));
    }
    hipLaunchKernelGGL(finalize_kernel, dim3(M), dim3(256), 0, st, m0, greedy ? b->d_keys : nullptr,
                       b->d_ids, b->d_ids, b->d_pos, b->d_step, b->d_hist, b->max_ctx,
                       (const uint4*)e->w.embed, (uint4*)b->x_res, (int64_t)s.hidden / 8, s.vocab, rope_cur_args(b),
                       b->pk_mem ? pk_epoch_ptr(b) : nullptr);
    QIE_LAUNCH_CHECK();
    return 0;
}

static bool pk_on(const qie_batch* b) { return b->decode_mode == 1 && b->pk_mem && !b->dbg_x; }

// the split target of the batch-1 decode attention (qie_attention_decode's rule at B = 1)
static int pk_splits_target(const qie_batch* b) { (void)b; return 32; }

static int enqueue_layers_persistent(qie_batch* b) {
    qie_engine* e = b->e;
    return persist_decode_launch(e->spec, b->d_layers, b->d_attp, b->x_res, (unsigned long long*)b->pk_mem,
                                 pk_epoch_ptr(b), pk_epoch_ptr(b) + 1, b->d_pos, pk_splits_target(b), b->pk_ts,
                                 e->stream);
}

static int enqueue_decode(qie_batch* b, const qie_sampling* smp) {
    if (pk_on(b)) QIE_TRY(enqueue_layers_persistent(b));
    else
        for (int l = 0; l < b->e->spec.n_layers; l++) QIE_TRY(enqueue_layer_decode(b, l));
    return enqueue_head(b, b->x_res, b->e->spec.hidden, 0, b->B, smp);
}

// opts.prefill_fp8 (numerics flag): the prefill projections on the block-scaled fp8 MFMA
// GEMM (QIE_LINEAR_ACT_FP8) — fp8 weights in the engine's arena, every projection input
// quantised per row (qie_quantize_rows_fp8), K of each a multiple of 128 — qie_engine_create
// refuses the flag where that does not hold, so it is never dropped silently here
static bool prefill_mx(const qie_engine* e) {
    return e->fp8 && e->opts.prefill_fp8;
}

static int ensure_prefill_scratch(qie_batch* b, int64_t n) {
    if (n <= b->pf_rows) {
        // rows fit; the attention workspace is not monotone in n (<= 8 rows run the split
        // kernel with partials, longer prompts need none), so size it for this n
        const qie_model_spec& s = b->e->spec;
        const int64_t ws = qie_attention_workspace_bytes(n, b->e->sh.nq, s.head_dim, b->max_ctx);
        if (ws > b->pf_attn_ws_bytes) {
            hipFree(b->pf_attn_ws);
            b->pf_attn_ws = nullptr;
            b->pf_attn_ws_bytes = 0;
            QIE_TRY(dmalloc(&b->pf_attn_ws, (size_t)ws));
            b->pf_attn_ws_bytes = ws;
        }
        return 0;
    }
    const qie_model_spec& s = b->e->spec;
    const TpShard& sh = b->e->sh;
    const int64_t H = s.hidden, QD = (int64_t)sh.nq * s.head_dim, KD = (int64_t)sh.nkv * s.head_dim;
    void** olds[] = {(void**)&b->pf_x, (void**)&b->pf_hn, (void**)&b->pf_qkv, (void**)&b->pf_q, (void**)&b->pf_att,
                     (void**)&b->pf_h, (void**)&b->pf_pos, (void**)&b->pf_ids, &b->pf_attn_ws, (void**)&b->pf_part,
                     (void**)&b->pf_q8, (void**)&b->pf_e8};
    for (void** p : olds) {   // nulled as freed: a failed re-allocation below leaves nothing dangling
        if (*p) hipFree(*p);
        *p = nullptr;
    }
    b->pf_rows = 0;
    if (use_comm(b->e)) QIE_TRY(dmalloc((void**)&b->pf_part, n * H * 4));
    QIE_TRY(dmalloc((void**)&b->pf_x, n * H * 2));
    QIE_TRY(dmalloc((void**)&b->pf_hn, n * H * 2));
    QIE_TRY(dmalloc((void**)&b->pf_qkv, n * (QD + 2 * KD) * 2));
    QIE_TRY(dmalloc((void**)&b->pf_q, n * QD * 2));
    QIE_TRY(dmalloc((void**)&b->pf_att, n * QD * 2));
    QIE_TRY(dmalloc((void**)&b->pf_h, n * (int64_t)sh.ffn * 2));
    if (prefill_mx(b->e)) {
        const int64_t kmax = std::max<int64_t>(std::max<int64_t>(H, QD), sh.ffn);
        QIE_TRY(dmalloc((void**)&b->pf_q8, n * kmax));
        QIE_TRY(dmalloc((void**)&b->pf_e8, std::max<int64_t>(n, 16)));
    }
    QIE_TRY(dmalloc((void**)&b->pf_pos, n * 4));
    QIE_TRY(dmalloc((void**)&b->pf_ids, n * 4));
    b->pf_attn_ws = nullptr;
    b->pf_attn_ws_bytes = 0;
    int64_t ws = qie_attention_workspace_bytes(n, sh.nq, s.head_dim, b->max_ctx);
    QIE_TRY(dmalloc(&b->pf_attn_ws, (size_t)ws));
    b->pf_attn_ws_bytes = ws;
    b->pf_rows = n;
    return 0;
}

// The ids and (tensor parallel, peer backend) the exchange error word come back in ONE
// stream-ordered batch with one synchronisation — not a second blocking round trip per token
// (ADVICE r05); a backend without the word keeps comm_check's own read.
// The persistent step's error word (a bounded hand-off wait that gave up): the step's outputs
// are garbage and the call fails loudly (never a hang; k_persist.hip)
static int pk_fail(unsigned w) {
    return fail(-8, "decode: the persistent decode step gave up on a hand-off wait (error word 0x%x: a CU never "
                    "published its part within the bound); outputs of this step are invalid", w);
}
static int pk_check(qie_batch* b) {
    if (!b->pk_mem) return 0;
    unsigned w = 0;
    QIE_HIP(hipMemcpyAsync(&w, pk_epoch_ptr(b) + 1, 4, hipMemcpyDeviceToHost, b->e->stream));
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    return w ? pk_fail(w) : 0;
}

static int sync_ids(qie_batch* b, int32_t* next_ids) {
    if (!next_ids) return pk_check(b);
    qie_engine* e = b->e;
    QIE_HIP(hipMemcpyAsync(next_ids, b->d_ids, b->B * 4, hipMemcpyDeviceToHost, e->stream));
    const unsigned* ew = use_comm(e) ? e->comm->error_word() : nullptr;
    unsigned err = 0, pkw = 0;
    if (ew) QIE_HIP(hipMemcpyAsync(&err, ew, sizeof(err), hipMemcpyDeviceToHost, e->stream));
    if (b->pk_mem) QIE_HIP(hipMemcpyAsync(&pkw, pk_epoch_ptr(b) + 1, 4, hipMemcpyDeviceToHost, e->stream));
    QIE_HIP(hipStreamSynchronize(e->stream));
    if (pkw) return pk_fail(pkw);
    if (ew) {
        if (err) return fail(-7, "decode: tensor-parallel exchange failed on the device (error word %u: a peer rank "
                                 "did not arrive within the bounded wait); the communicator is unusable", err);
        return 0;
    }
    return comm_check(e, "decode");
}

}  // namespace qie

extern "C" {

int qie_engine_create(const qie_model_spec* spec, const qie_engine_opts* opts, qie_engine** out) {
    QIE_REQUIRE(spec && out, "qie_engine_create: bad arguments");
    const qie_model_spec& s = *spec;
    QIE_REQUIRE(s.n_layers > 0 && s.hidden > 0 && s.n_heads > 0 && s.n_kv_heads > 0 && s.head_dim > 0 &&
                    s.ffn > 0 && s.vocab > 0 && s.n_heads % s.n_kv_heads == 0,
                "qie_engine_create: invalid model spec");
    QIE_REQUIRE(s.hidden % 8 == 0 && s.ffn % 8 == 0 && (s.head_dim == 64 || s.head_dim == 128),
                "qie_engine_create: hidden/ffn must be multiples of 8 and head_dim 64 or 128");
    qie_comm* comm = opts ? (qie_comm*)opts->tp_comm : nullptr;
    const int tp = comm ? comm->world : 1;
    TpShard probe;
    QIE_REQUIRE(shard_heads(s.n_heads, s.n_kv_heads, tp, 0, probe) && s.ffn % tp == 0 && (s.ffn / tp) % 8 == 0 &&
                    s.vocab % tp == 0,
                "qie_engine_create: tensor parallel %d needs n_kv_heads divisible by it (or dividing it, with at "
                "most n_heads / n_kv_heads ranks per kv head), vocab divisible by it and ffn / tp a multiple of 8 "
                "(use replicas for this model at this size)", tp);
    // prefill_fp8 is a numerics choice (every projection input quantised to e4m3): refuse it
    // where the engine could not honour it, instead of silently running bf16 activations
    // against a caller (and an oracle) that expects the fp8-activation model
    if (opts && opts->prefill_fp8) {
        const int64_t qd = (int64_t)probe.nq * s.head_dim, ffl = s.ffn / tp;
        QIE_REQUIRE(opts->weight_fp8, "qie_engine_create: prefill_fp8 needs weight_fp8 (fp8 weights are the "
                                      "block-scaled MFMA's second operand)");
        QIE_REQUIRE(s.hidden % 128 == 0 && qd % 128 == 0 && ffl % 128 == 0,
                    "qie_engine_create: prefill_fp8 needs hidden (%lld), this rank's q width (%lld) and ffn / tp "
                    "(%lld) to be multiples of 128 (the fp8 MFMA's k block)",
                    (long long)s.hidden, (long long)qd, (long long)ffl);
    }
    qie_engine* e = new qie_engine();
    e->spec = s;
    if (opts) e->opts = *opts;
    if (e->opts.max_ctx <= 0) e->opts.max_ctx = 32786;   // reference CONTEXT_SIZE (iengine.cuh:19)
    e->comm = comm;
    e->sh.tp = tp;
    e->sh.rank = comm ? comm->rank : 0;
    shard_heads(s.n_heads, s.n_kv_heads, tp, e->sh.rank, e->sh);
    e->sh.ffn = s.ffn / tp;
    e->sh.vocab = s.vocab / tp;
    e->sh.vocab0 = (int64_t)e->sh.rank * e->sh.vocab;
    e->opts.tp_size = tp;
    e->opts.tp_rank = e->sh.rank;
    if (comm && !comm->graph_capturable()) e->opts.use_graph = 0;
    hipError_t he = hipSetDevice(e->opts.device);
    if (he != hipSuccess) {
        delete e;
        return fail((int)he, "hipSetDevice(%d): %s", opts ? opts->device : 0, hipGetErrorString(he));
    }
    he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        delete e;
        return fail((int)he, "hipStreamCreate: %s", hipGetErrorString(he));
    }
    int rc = build_rope(e);
    if (rc) {
        qie_engine_destroy(e);
        return rc;
    }
    *out = e;
    return 0;
}

static int alloc_arena_synthetic(qie_engine* e) {
    if (e->index) qie_index_destroy(e->index);
    e->index = nullptr;
    QIE_TRY(qie_index_synthetic(&e->spec, &e->index));
    e->arena_bytes = (size_t)qie_index_total_bytes(e->index);
    if (e->arena) hipFree(e->arena);
    e->arena = nullptr;
    QIE_HIP(hipMalloc(&e->arena, e->arena_bytes));
    return 0;
}

// This rank's part of one full tensor: rows [row0, row0 + rows) x cols [col0, col0 + cols)
// of the row-major [full_rows, full_cols] tensor `src` (1-D tensors are one row).
struct ShardSlice {
    const qie_index_entry* src = nullptr;
    int64_t rows = 0, cols = 0, full_cols = 0, row0 = 0, col0 = 0;
};

static ShardSlice plan_slice(const qie_index_entry& t, const qie_model_spec& s, const TpShard& sh) {
    ShardSlice x;
    x.src = &t;
    const int64_t d0 = t.shape.empty() ? 1 : t.shape[0];
    const int64_t d1 = t.shape.size() >= 2 ? t.shape[1] : 1;
    const bool two_d = t.shape.size() >= 2;
    x.rows = two_d ? d0 : 1;
    x.cols = two_d ? d1 : d0;
    x.full_cols = x.cols;
    const int64_t hd = s.head_dim;
    const std::string& n = t.short_name;
    auto rows_part = [&](int64_t local, int64_t first) { x.rows = local; x.row0 = first; };
    auto cols_part = [&](int64_t local, int64_t first) { x.cols = local; x.col0 = first; };
    if (sh.tp == 1) return x;
    const int64_t qn = sh.nq * hd, q0 = (int64_t)sh.q0 * hd, kn = sh.nkv * hd, k0 = (int64_t)sh.kv0 * hd;
    if (n == "self_attn.q_proj.weight") rows_part(qn, q0);                              // column-parallel
    else if (n == "self_attn.k_proj.weight" || n == "self_attn.v_proj.weight") rows_part(kn, k0);
    else if (n == "self_attn.q_proj.bias") cols_part(qn, q0);
    else if (n == "self_attn.k_proj.bias" || n == "self_attn.v_proj.bias") cols_part(kn, k0);
    else if (n == "self_attn.o_proj.weight") cols_part(qn, q0);                         // row-parallel
    else if (n == "mlp.gate_proj.weight" || n == "mlp.up_proj.weight") rows_part(sh.ffn, (int64_t)sh.rank * sh.ffn);
    else if (n == "mlp.down_proj.weight") cols_part(sh.ffn, (int64_t)sh.rank * sh.ffn);
    else if (n == "logits") rows_part(sh.vocab, (int64_t)sh.rank * sh.vocab);          // vocab-parallel
    return x;
}

// Shard index: same names / roles as the full index, local shapes and arena offsets
// (256-B aligned).  A tied lm_head becomes a vocab slice of the embedding under tp > 1.
static int build_shard_index(qie_engine* e, const qie_index* full, qie_index** out, std::vector<ShardSlice>& sl) {
    qie_index* idx = new qie_index();
    sl.clear();
    int64_t off = 0;
    auto add = [&](const qie_index_entry& src, const ShardSlice& x, const char* short_name) {
        qie_index_entry le;
        le.name = src.name;
        le.short_name = short_name ? short_name : src.short_name;
        le.layer = src.layer;
        le.shape = src.shape.size() >= 2 ? std::vector<int64_t>{x.rows, x.cols} : std::vector<int64_t>{x.cols};
        le.off0 = off;
        le.off1 = off + x.rows * x.cols * 2;
        off = (le.off1 + 255) / 256 * 256;
        idx->t.push_back(le);
        sl.push_back(x);
    };
    for (const auto& t : full->t) add(t, plan_slice(t, e->spec, e->sh), nullptr);
    if (e->spec.tie_embeddings && e->sh.tp > 1) {
        const qie_index_entry* emb = index_find(full, "embed_tokens.weight", -1);
        if (!emb) {
            delete idx;
            return fail(-22, "tied lm_head: embed_tokens.weight missing from index");
        }
        qie_index_entry as_logits = *emb;
        as_logits.short_name = "logits";
        ShardSlice x = plan_slice(as_logits, e->spec, e->sh);
        x.src = emb;
        add(*emb, x, "logits");
    }
    *out = idx;
    return 0;
}

static int init_synthetic_sharded(qie_engine* e, uint64_t seed, float w_scale, float norm_scale, float bias_scale) {
    qie_index* full = nullptr;
    QIE_TRY(qie_index_synthetic(&e->spec, &full));
    std::vector<ShardSlice> sl;
    qie_index* local = nullptr;
    int rc = build_shard_index(e, full, &local, sl);
    if (!rc) {
        if (e->index) qie_index_destroy(e->index);
        e->index = local;
        e->arena_bytes = (size_t)(local->t.empty() ? 16 : local->t.back().off1);
        if (e->arena) hipFree(e->arena);
        e->arena = nullptr;
        hipError_t he = hipMalloc(&e->arena, e->arena_bytes);
        if (he != hipSuccess) rc = fail((int)he, "weight arena (%zu bytes): %s", e->arena_bytes, hipGetErrorString(he));
    }
    for (size_t i = 0; !rc && i < sl.size(); i++) {
        const qie_index_entry& le = local->t[i];
        const ShardSlice& x = sl[i];
        const std::string& sn = x.src->short_name;
        float scale = w_scale, offset = 0.f;
        if (sn.find("norm") != std::string::npos) { scale = norm_scale; offset = 1.0f; }
        else if (sn.find("bias") != std::string::npos) { scale = bias_scale; }
        rc = qie_synthetic_fill_slice((char*)e->arena + le.off0, x.rows, x.cols, x.full_cols, x.row0, x.col0,
                                      qie_tensor_id(x.src->name.c_str()), seed, scale, offset, e->stream);
    }
    qie_index_destroy(full);   // slices point into it only during the fill
    if (rc) return rc;
    QIE_HIP(hipStreamSynchronize(e->stream));
    return bind_from_index(e);
}

int qie_engine_init_synthetic(qie_engine* e, uint64_t seed, float w_scale, float norm_scale, float bias_scale) {
    QIE_REQUIRE(e, "qie_engine_init_synthetic: null engine");
    if (e->sh.tp > 1) return init_synthetic_sharded(e, seed, w_scale, norm_scale, bias_scale);
    QIE_TRY(alloc_arena_synthetic(e));
    const int n = qie_index_count(e->index);
    for (int i = 0; i < n; i++) {
        const char *name, *sn;
        int32_t layer, nd;
        int64_t o0, o1, shp[4];
        qie_index_get(e->index, i, &name, &sn, &layer, &o0, &o1, &nd, shp);
        const std::string sname(sn);
        float scale = w_scale, offset = 0.f;
        if (sname.find("norm") != std::string::npos) { scale = norm_scale; offset = 1.0f; }
        else if (sname.find("bias") != std::string::npos) { scale = bias_scale; }
        QIE_TRY(qie_synthetic_fill((char*)e->arena + o0, (o1 - o0) / 2, qie_tensor_id(name), seed, scale, offset,
                                   e->stream));
    }
    QIE_HIP(hipStreamSynchronize(e->stream));
    return bind_from_index(e);
}

// Tensor-parallel load: each rank reads only its slices of weights.bin (row slices in
// one read, column slices row by row) — 1/tp of the bytes per rank for the big tensors.
static int load_weights_sharded(qie_engine* e, const char* weights_bin, const char* meta) {
    qie_index* full = nullptr;
    QIE_TRY(qie_index_load_meta(meta, &full));
    std::vector<ShardSlice> sl;
    qie_index* local = nullptr;
    int rc = build_shard_index(e, full, &local, sl);
    if (rc) {
        qie_index_destroy(full);
        return rc;
    }
    if (e->index) qie_index_destroy(e->index);
    e->index = local;
    e->arena_bytes = (size_t)(local->t.empty() ? 16 : local->t.back().off1);
    if (e->arena) hipFree(e->arena);
    e->arena = nullptr;
    std::ifstream f(weights_bin, std::ios::binary);
    if (!f.good()) rc = fail(-2, "cannot open %s", weights_bin);
    if (!rc) {
        hipError_t he = hipMalloc(&e->arena, e->arena_bytes);
        if (he != hipSuccess) rc = fail((int)he, "weight arena: %s", hipGetErrorString(he));
    }
    std::vector<uint16_t> host;
    for (size_t i = 0; !rc && i < sl.size(); i++) {
        const ShardSlice& x = sl[i];
        host.resize((size_t)(x.rows * x.cols));
        if (x.cols == x.full_cols) {
            f.seekg(x.src->off0 + x.row0 * x.full_cols * 2);
            f.read((char*)host.data(), x.rows * x.cols * 2);
            if (!f) rc = fail(-5, "short read of %s (%s)", weights_bin, x.src->name.c_str());
        } else {
            for (int64_t r = 0; r < x.rows && !rc; r++) {
                f.seekg(x.src->off0 + ((x.row0 + r) * x.full_cols + x.col0) * 2);
                f.read((char*)(host.data() + r * x.cols), x.cols * 2);
                if (!f) rc = fail(-5, "short read of %s (%s)", weights_bin, x.src->name.c_str());
            }
        }
        if (!rc) {
            // stream-ordered before the engine's kernels (its stream is non-blocking: a copy on the
            // legacy null stream is not), complete before the staging vector is refilled
            hipError_t he = hipMemcpyAsync((char*)e->arena + local->t[i].off0, host.data(),
                                           (size_t)(x.rows * x.cols * 2), hipMemcpyHostToDevice, e->stream);
            if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
            if (he != hipSuccess) rc = fail((int)he, "H2D: %s", hipGetErrorString(he));
        }
    }
    qie_index_destroy(full);
    if (rc) return rc;
    return bind_from_index(e);
}

int qie_engine_load_weights_bin(qie_engine* e, const char* weights_bin, const char* meta, int64_t chunk_bytes) {
    QIE_REQUIRE(e && weights_bin && meta, "qie_engine_load_weights_bin: bad arguments");
    if (e->sh.tp > 1) return load_weights_sharded(e, weights_bin, meta);
    if (e->index) qie_index_destroy(e->index);
    e->index = nullptr;
    QIE_TRY(qie_index_load_meta(meta, &e->index));
    std::ifstream f(weights_bin, std::ios::binary | std::ios::ate);
    QIE_REQUIRE(f.good(), "cannot open %s", weights_bin);
    const int64_t file_bytes = (int64_t)f.tellg();
    f.seekg(0);
    const int64_t need = qie_index_total_bytes(e->index);
    QIE_REQUIRE(file_bytes >= need, "%s is %lld bytes, index needs %lld", weights_bin, (long long)file_bytes,
                (long long)need);
    e->arena_bytes = (size_t)need;
    if (e->arena) hipFree(e->arena);
    e->arena = nullptr;
    QIE_HIP(hipMalloc(&e->arena, e->arena_bytes));
    if (chunk_bytes <= 0) chunk_bytes = (int64_t)1 << 28;
    // Two pinned staging buffers: file read of chunk i+1 overlaps H2D of chunk i.
    void* stage[2] = {nullptr, nullptr};
    hipEvent_t done[2];
    QIE_HIP(hipHostMalloc(&stage[0], chunk_bytes, hipHostMallocDefault));
    QIE_HIP(hipHostMalloc(&stage[1], chunk_bytes, hipHostMallocDefault));
    QIE_HIP(hipEventCreate(&done[0]));
    QIE_HIP(hipEventCreate(&done[1]));
    int64_t off = 0;
    int which = 0;
    bool pending[2] = {false, false};
    int rc = 0;
    while (off < need) {
        const int64_t n = std::min<int64_t>(chunk_bytes, need - off);
        if (pending[which]) {
            hipEventSynchronize(done[which]);
            pending[which] = false;
        }
        f.read((char*)stage[which], n);
        if (f.gcount() != n) { rc = fail(-5, "short read of %s at %lld", weights_bin, (long long)off); break; }
        hipError_t he = hipMemcpyAsync((char*)e->arena + off, stage[which], n, hipMemcpyHostToDevice, e->stream);
        if (he != hipSuccess) { rc = fail((int)he, "H2D: %s", hipGetErrorString(he)); break; }
        hipEventRecord(done[which], e->stream);
        pending[which] = true;
        off += n;
        which ^= 1;
    }
    hipStreamSynchronize(e->stream);
    hipEventDestroy(done[0]);
    hipEventDestroy(done[1]);
    hipHostFree(stage[0]);
    hipHostFree(stage[1]);
    if (rc) return rc;
    return bind_from_index(e);
}

int qie_engine_set_weights(qie_engine* e, const qie_model_weights* w) {
    QIE_REQUIRE(e && w && w->layers && w->n_layers == e->spec.n_layers && w->embed && w->final_norm && w->lm_head,
                "qie_engine_set_weights: bad arguments");
    e->layers.assign(w->layers, w->layers + w->n_layers);
    for (int l = 0; l < w->n_layers; l++) {
        const qie_layer_weights& L = e->layers[l];
        QIE_REQUIRE(L.attn_norm && L.wq && L.wk && L.wv && L.wo && L.ffn_norm && L.w_gate && L.w_up && L.w_down,
                    "qie_engine_set_weights: layer %d incomplete", l);
        QIE_REQUIRE(!e->spec.qkv_bias || (L.bq && L.bk && L.bv), "layer %d: q/k/v bias missing", l);
        QIE_REQUIRE(!e->spec.qk_norm || (L.q_norm && L.k_norm), "layer %d: q/k norm missing", l);
        const void* ps[] = {L.attn_norm, L.wq, L.wk, L.wv, L.wo, L.ffn_norm, L.w_gate, L.w_up, L.w_down};
        for (const void* p : ps) QIE_TRY(check_align(p, "weight", l));
    }
    e->w = *w;
    e->w.layers = e->layers.data();
    e->have_weights = true;
    return e->opts.weight_fp8 ? quantize_weights_fp8(e, false) : 0;
}

int qie_engine_weights(const qie_engine* e, qie_model_weights* out, const qie_layer_weights** layers) {
    QIE_REQUIRE(e && e->have_weights, "qie_engine_weights: no weights");
    if (out) *out = e->w;
    if (layers) *layers = e->layers.data();
    return 0;
}

int qie_engine_spec(const qie_engine* e, qie_model_spec* out) {
    QIE_REQUIRE(e && out, "qie_engine_spec: bad arguments");
    *out = e->spec;
    return 0;
}

void* qie_engine_stream(qie_engine* e) { return e ? (void*)e->stream : nullptr; }

int qie_engine_sync(qie_engine* e) {
    QIE_REQUIRE(e, "qie_engine_sync: null");
    QIE_HIP(hipStreamSynchronize(e->stream));
    return comm_check(e, "qie_engine_sync");
}

void qie_engine_destroy(qie_engine* e) {
    if (!e) return;
    if (e->stream) hipStreamSynchronize(e->stream);
    if (e->arena) hipFree(e->arena);
    if (e->fp8_arena) hipFree(e->fp8_arena);
    if (e->rope_cos) hipFree(e->rope_cos);
    if (e->rope_sin) hipFree(e->rope_sin);
    if (e->index) qie_index_destroy(e->index);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
}

static int batch_create(qie_engine* e, int32_t batch, int32_t max_ctx, int32_t page_tokens, int32_t n_pages,
                        qie_batch** out) {
    QIE_REQUIRE(e && out && batch > 0 && batch <= 8 && max_ctx > 1, "qie_batch_create: bad arguments (B <= 8)");
    QIE_REQUIRE(e->have_weights, "qie_batch_create: engine has no weights");
    QIE_REQUIRE(max_ctx <= e->rope_rows, "qie_batch_create: max_ctx %d > engine max_ctx %d", max_ctx, e->rope_rows);
    const qie_model_spec& s = e->spec;
    qie_batch* b = new qie_batch();
    b->e = e;
    b->B = batch;
    b->max_ctx = max_ctx;
    const TpShard& sh = e->sh;
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)sh.nq * hd, KD = (int64_t)sh.nkv * hd;
    int64_t n_runs = batch;   // sequences (contiguous) or pages (paged) in the K and V pools
    if (page_tokens > 0) {
        b->page_tokens = page_tokens;
        b->max_pages = (max_ctx + page_tokens - 1) / page_tokens;
        b->n_pages = n_pages > 0 ? n_pages : batch * b->max_pages + 1;
        b->seq_stride = (int64_t)s.n_layers * sh.nkv * page_tokens * hd;   // elements per page
        n_runs = b->n_pages;
        b->h_table.assign((size_t)batch * b->max_pages, 0);
        for (int p = b->n_pages - 1; p >= 1; p--) b->free_pages.push_back(p);   // page 1 handed out first
        b->held.assign(batch, 0);
        b->table_dirty = true;
    } else {
        b->run_pad = dev_env("QIE_KV_RUN_PAD", 0);   // dev A/B: tokens of padding per (layer, head) run
        b->seq_stride = (int64_t)s.n_layers * sh.nkv * (max_ctx + b->run_pad) * hd;   // this rank's kv heads only
    }
    // Slots start idle: a slot runs as a live sequence only after a prefill or
    // set_position, so unused slots never take pool pages (they run on scratch page 0)
    // and are rewound before they would pass max_ctx (prepare_steps).
    b->idle.assign(batch, 1);
    int rc = 0;
    auto A = [&](void** p, size_t bytes) {
        if (!rc) rc = dmalloc(p, bytes);
    };
    A((void**)&b->kc, (size_t)n_runs * b->seq_stride * 2);
    A((void**)&b->vc, (size_t)n_runs * b->seq_stride * 2);
    if (page_tokens > 0) A((void**)&b->d_table, b->h_table.size() * 4);
    A((void**)&b->d_pos, batch * 4);
    A((void**)&b->d_rope_cur, (size_t)batch * rope_cur_stride((int)hd) * 4);
    A((void**)&b->d_step, batch * 4);
    A((void**)&b->d_hist, (size_t)batch * max_ctx * 4);
    A((void**)&b->d_ids, batch * 4);
    A((void**)&b->d_keys, batch * 8);
    A((void**)&b->x_res, batch * H * 2);
    A((void**)&b->qkv, batch * (QD + 2 * KD) * 2);
    A((void**)&b->q, batch * QD * 2);
    A((void**)&b->att, batch * QD * 2);
    A((void**)&b->h, batch * (int64_t)sh.ffn * 2);
    A((void**)&b->xn, batch * H * 2);
    A((void**)&b->logits, batch * (int64_t)sh.vocab * 2);
    A(&b->attn_ws, (size_t)qie_attention_workspace_bytes(batch, sh.nq, s.head_dim, max_ctx));
    A(&b->samp_ws, (size_t)qie_sample_workspace_bytes(batch, s.vocab));
    const int64_t dec_ws = qie_attention_decode_workspace_bytes(batch, sh.nq, sh.nkv, s.head_dim, max_ctx);
    A(&b->dec_ws, (size_t)dec_ws);
    if (use_comm(e)) {
        A((void**)&b->part, batch * H * 4);
        A((void**)&b->logits_full, batch * (int64_t)s.vocab * 2);
        A((void**)&b->gather_tmp, batch * (int64_t)s.vocab * 2);
    }
    if (!rc) {
        hipMemsetAsync(b->dec_ws, 0, (size_t)dec_ws, e->stream);
        hipMemsetAsync(b->kc, 0, (size_t)n_runs * b->seq_stride * 2, e->stream);
        hipMemsetAsync(b->vc, 0, (size_t)n_runs * b->seq_stride * 2, e->stream);
        hipMemsetAsync(b->d_keys, 0, batch * 8, e->stream);
        hipMemsetAsync(b->d_pos, 0, batch * 4, e->stream);
        hipMemsetAsync(b->d_rope_cur, 0xff, (size_t)batch * rope_cur_stride((int)hd) * 4, e->stream);   // tags -1
        hipMemsetAsync(b->d_step, 0, batch * 4, e->stream);
        hipMemsetAsync(b->d_ids, 0, batch * 4, e->stream);
        hipMemsetAsync(b->d_hist, 0, (size_t)batch * max_ctx * 4, e->stream);
        hipMemsetAsync(b->x_res, 0, batch * H * 2, e->stream);
        hipError_t he = hipStreamSynchronize(e->stream);
        if (he != hipSuccess) rc = fail((int)he, "batch init: %s", hipGetErrorString(he));
    }
    if (rc) {
        qie_batch_destroy(b);
        return rc;
    }
    b->h_pos.assign(batch, 0);
    if (!rc) rc = flush_table(b);
    // the fp8 batched-decode split-K workspace of this stream, before any graph capture
    if (!rc && e->fp8 && (batch >= 2 || e->fp8_t16)) rc = dec8_reserve(e->stream);
    if (rc) {
        qie_batch_destroy(b);
        return rc;
    }
    *out = b;
    return 0;
}

int qie_batch_create(qie_engine* e, int32_t batch, int32_t max_ctx, qie_batch** out) {
    return batch_create(e, batch, max_ctx, 0, 0, out);
}

int qie_batch_create_paged(qie_engine* e, int32_t batch, int32_t max_ctx, int32_t page_tokens, int32_t n_pages,
                           qie_batch** out) {
    if (page_tokens == 0) page_tokens = 128;
    QIE_REQUIRE(page_tokens >= 128 && (page_tokens & (page_tokens - 1)) == 0,
                "qie_batch_create_paged: page_tokens %d must be a power of two >= 128", page_tokens);
    QIE_REQUIRE(n_pages >= 0, "qie_batch_create_paged: bad n_pages");
    QIE_REQUIRE(n_pages == 0 || n_pages >= 2, "qie_batch_create_paged: need the scratch page and one more");
    return batch_create(e, batch, max_ctx, page_tokens, n_pages, out);
}

int qie_batch_release(qie_batch* b, int32_t seq) {
    QIE_REQUIRE(b && seq >= 0 && seq < b->B, "qie_batch_release: bad arguments");
    drop_pages(b, seq);
    b->idle[seq] = 1;
    QIE_TRY(flush_table(b));
    qie_engine* e = b->e;
    hipLaunchKernelGGL(set_state_kernel, dim3(1), dim3(256), 0, e->stream, seq, 0, 0, 0, b->d_pos, b->d_step, b->d_hist,
                       b->max_ctx, (const uint4*)e->w.embed, (uint4*)b->x_res, (int64_t)e->spec.hidden / 8, 1, rope_cur_args(b));
    QIE_LAUNCH_CHECK();
    QIE_HIP(hipStreamSynchronize(e->stream));
    b->h_pos[seq] = 0;
    return 0;
}

int qie_batch_page_stats(qie_batch* b, int32_t* free_pages, int32_t* pages_per_seq, int32_t* page_tokens) {
    QIE_REQUIRE(b, "qie_batch_page_stats: null batch");
    if (free_pages) *free_pages = (int32_t)b->free_pages.size();
    if (pages_per_seq)
        for (int m = 0; m < b->B; m++) pages_per_seq[m] = b->d_table ? b->held[m] : 0;
    if (page_tokens) *page_tokens = b->page_tokens;
    return 0;
}

int qie_batch_block_table(qie_batch* b, int32_t seq, int32_t* host_pages, int32_t n) {
    QIE_REQUIRE(b && b->d_table && host_pages && seq >= 0 && seq < b->B && n >= 0 && n <= b->max_pages,
                "qie_batch_block_table: bad arguments (paged batch, n <= max_pages)");
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    QIE_HIP(d2h(b->e, host_pages, b->d_table + (int64_t)seq * b->max_pages, (size_t)n * 4));
    return 0;
}

void qie_batch_destroy(qie_batch* b) {
    if (!b) return;
    if (b->e && b->e->stream) hipStreamSynchronize(b->e->stream);
    if (b->gexec) hipGraphExecDestroy(b->gexec);
    void* ps[] = {b->kc, b->vc, b->d_table, b->d_pos, b->d_rope_cur, b->d_step, b->d_hist, b->d_ids, b->d_keys, b->x_res, b->qkv, b->q,
                  b->att, b->h, b->logits, b->attn_ws, b->dec_ws, b->samp_ws, b->pf_x, b->pf_hn, b->pf_qkv, b->pf_q,
                  b->pf_att, b->pf_h, b->pf_pos, b->pf_ids, b->pf_attn_ws, b->part, b->logits_full,
                  b->gather_tmp, b->pf_part, b->xn, b->pf_q8, b->pf_e8, b->pk_mem, b->d_layers, b->d_attp, b->pk_ts};
    for (void* p : ps)
        if (p) hipFree(p);
    delete b;
}

// Prefill of n_seqs prompts of len ids each into slots seq0 .. seq0+n_seqs-1 (ids laid end
// to end): every GEMM runs once over all n_seqs * len rows, attention and the KV append see
// the prompts as sequences of rows_per_seq = len, and the head samples the n_seqs last rows
// in one launch.  n_seqs = 1 is qie_prefill.
static int prefill_rows(qie_batch* b, int seq0, int n_seqs, const int32_t* ids, int len, const qie_sampling* smp,
                        int32_t* next_ids, const char* who) {
    QIE_REQUIRE(b && ids && len > 0 && n_seqs > 0 && seq0 >= 0 && seq0 + n_seqs <= b->B, "%s: bad arguments", who);
    QIE_REQUIRE(len < b->max_ctx, "%s: prompt of %d tokens does not fit max_ctx %d", who, len, b->max_ctx);
    qie_engine* e = b->e;
    const qie_model_spec& s = e->spec;
    const int64_t n = (int64_t)n_seqs * len;   // rows
    QIE_REQUIRE(n <= INT32_MAX, "%s: %lld rows", who, (long long)n);
    for (int64_t i = 0; i < n; i++)
        QIE_REQUIRE(ids[i] >= 0 && ids[i] < s.vocab, "%s: token id %d out of range", who, ids[i]);
    hipStream_t st = e->stream;
    QIE_TRY(ensure_prefill_scratch(b, n));
    if (b->d_table) {   // all-or-nothing: the slots' own pages count, nothing is dropped on failure
        const int64_t need = ((int64_t)len + b->page_tokens - 1) / b->page_tokens * n_seqs;
        int64_t held = 0;
        for (int z = 0; z < n_seqs; z++) held += b->held[seq0 + z];
        QIE_REQUIRE(need <= (int64_t)b->free_pages.size() + held,
                    "%s: KV pool exhausted (%lld pages needed, %zu free + %lld held by slots %d..%d)", who,
                    (long long)need, b->free_pages.size(), (long long)held, seq0, seq0 + n_seqs - 1);
    }
    // a prefill starts a new sequence in each slot: every target slot's pages go back to
    // the pool BEFORE any slot draws, so the check above (free + held) is exactly what the
    // draws below can use and none of them can fail part way
    for (int z = 0; z < n_seqs; z++) drop_pages(b, seq0 + z);
    for (int z = 0; z < n_seqs; z++) {
        QIE_TRY(ensure_pages(b, seq0 + z, len));
        b->idle[seq0 + z] = 0;
    }
    QIE_TRY(flush_table(b));
    const TpShard& sh = e->sh;
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)sh.nq * hd, KD = (int64_t)sh.nkv * hd;
    const int64_t QKVD = QD + 2 * KD, I = sh.ffn;
    QIE_HIP(hipMemcpyAsync(b->pf_ids, ids, (size_t)n * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, b->pf_pos, (int)n, len);
    hipLaunchKernelGGL(copy_ids_kernel, dim3((len + 255) / 256, n_seqs), dim3(256), 0, st, b->pf_ids,
                       b->d_hist + (int64_t)seq0 * b->max_ctx, len, (int64_t)b->max_ctx);
    QIE_TRY(qie_embedding(e->w.embed, b->pf_ids, b->pf_x, n, H, st));
    const qie_kv_cache cache = batch_cache(b, seq0);
    // fp8 engine, >= 256 rows: the GEMMs run on the dequantised bf16 copy (layers_pf); with
    // tiled fp8 projections (readable by the batched-decode kernel only) every prefill of more
    // than 16 rows does
    const bool pf16 = e->fp8 && !e->layers_pf.empty() && (n >= 256 || (e->fp8_t16 && n > 16));
    auto pf_base = [&]() {
        qie_linear_args a = lin_proj(e);
        if (pf16) a.flags &= ~(QIE_LINEAR_FP8 | QIE_LINEAR_FP8_T16);
        return a;
    };
    const bool mx = prefill_mx(e);
    // fp8 activations: quantise the projection input x [n][K] (bf16) into pf_q8 / pf_e8 and
    // point the linear at the codes
    auto mx_in = [&](qie_linear_args& a, const uint16_t* x, int64_t K) -> int {
        QIE_TRY(qie_quantize_rows_fp8(x, K, n, K, b->pf_q8, K, b->pf_e8, st));
        a.x = b->pf_q8; a.ldx = K; a.x_exps = b->pf_e8;
        a.flags |= QIE_LINEAR_ACT_FP8;
        return 0;
    };
    for (int l = 0; l < s.n_layers; l++) {
        if (mx) {   // every projection on fp8 codes x fp8 weights (e->layers: the fp8 arena)
            const qie_layer_weights& L = e->layers[l];
            QIE_TRY(qie_rmsnorm(b->pf_x, L.attn_norm, b->pf_hn, n, H, s.rms_eps, s.numerics, st));
            qie_linear_args a = lin_proj(e);
            QIE_TRY(mx_in(a, b->pf_hn, H));
            a.w[0] = L.wq; a.w[1] = L.wk; a.w[2] = L.wv;
            a.bias[0] = L.bq; a.bias[1] = L.bk; a.bias[2] = L.bv;
            a.seg_rows[0] = QD; a.seg_rows[1] = KD; a.seg_rows[2] = KD;
            a.M = n; a.K = H; a.N = QKVD; a.y = b->pf_qkv; a.ldy = QKVD; a.epilogue = QIE_EPI_STORE;
            QIE_TRY(qie_linear(&a, st));
            QIE_TRY(qie_qkv_post(b->pf_qkv, n, b->pf_pos, len, L.q_norm, L.k_norm, e->rope_cos, e->rope_sin, sh.nq,
                                 &cache, l, s.rms_eps, s.numerics, b->pf_q, st));
            QIE_TRY(qie_attention(b->pf_q, n, b->pf_pos, len, &cache, l, sh.nq, b->pf_att, b->pf_attn_ws, st));
            a = lin_proj(e);
            QIE_TRY(mx_in(a, b->pf_att, QD));
            a.w[0] = L.wo; a.seg_rows[0] = H;
            a.M = n; a.K = QD; a.N = H; a.ldy = H;
            QIE_TRY(row_parallel(b, a, b->pf_x, b->pf_part, n));
            QIE_TRY(qie_rmsnorm(b->pf_x, L.ffn_norm, b->pf_hn, n, H, s.rms_eps, s.numerics, st));
            a = lin_proj(e);
            QIE_TRY(mx_in(a, b->pf_hn, H));
            a.w[0] = L.w_gate; a.w[1] = L.w_up; a.seg_rows[0] = I; a.seg_rows[1] = I;
            a.M = n; a.K = H; a.N = I; a.y = b->pf_h; a.ldy = I; a.epilogue = QIE_EPI_SWIGLU;
            QIE_TRY(qie_linear(&a, st));
            a = lin_proj(e);
            QIE_TRY(mx_in(a, b->pf_h, I));
            a.w[0] = L.w_down; a.seg_rows[0] = H;
            a.M = n; a.K = I; a.N = H; a.ldy = H;
            QIE_TRY(row_parallel(b, a, b->pf_x, b->pf_part, n));
            continue;
        }
        const qie_layer_weights& L = pf16 ? e->layers_pf[l] : e->layers[l];
        QIE_TRY(qie_rmsnorm(b->pf_x, L.attn_norm, b->pf_hn, n, H, s.rms_eps, s.numerics, st));
        qie_linear_args a = pf_base();
        a.x = b->pf_hn; a.ldx = H;
        a.w[0] = L.wq; a.w[1] = L.wk; a.w[2] = L.wv;
        a.bias[0] = L.bq; a.bias[1] = L.bk; a.bias[2] = L.bv;
        a.seg_rows[0] = QD; a.seg_rows[1] = KD; a.seg_rows[2] = KD;
        a.M = n; a.K = H; a.N = QKVD; a.y = b->pf_qkv; a.ldy = QKVD; a.epilogue = QIE_EPI_STORE;
        QIE_TRY(qie_linear(&a, st));
        QIE_TRY(qie_qkv_post(b->pf_qkv, n, b->pf_pos, len, L.q_norm, L.k_norm, e->rope_cos, e->rope_sin, sh.nq,
                             &cache, l, s.rms_eps, s.numerics, b->pf_q, st));
        QIE_TRY(qie_attention(b->pf_q, n, b->pf_pos, len, &cache, l, sh.nq, b->pf_att, b->pf_attn_ws, st));
        a = pf_base();
        a.x = b->pf_att; a.ldx = QD; a.w[0] = L.wo; a.seg_rows[0] = H;
        a.M = n; a.K = QD; a.N = H; a.ldy = H;
        QIE_TRY(row_parallel(b, a, b->pf_x, b->pf_part, n));
        QIE_TRY(qie_rmsnorm(b->pf_x, L.ffn_norm, b->pf_hn, n, H, s.rms_eps, s.numerics, st));
        a = pf_base();
        a.x = b->pf_hn; a.ldx = H; a.w[0] = L.w_gate; a.w[1] = L.w_up; a.seg_rows[0] = I; a.seg_rows[1] = I;
        a.M = n; a.K = H; a.N = I; a.y = b->pf_h; a.ldy = I; a.epilogue = QIE_EPI_SWIGLU;
        QIE_TRY(qie_linear(&a, st));
        a = pf_base();
        a.x = b->pf_h; a.ldx = I; a.w[0] = L.w_down; a.seg_rows[0] = H;
        a.M = n; a.K = I; a.N = H; a.ldy = H;
        QIE_TRY(row_parallel(b, a, b->pf_x, b->pf_part, n));
    }
    // position of each last prompt token; finalize advances it to len (the new token).
    for (int z = 0; z < n_seqs; z++) {
        hipLaunchKernelGGL(set_state_kernel, dim3(1), dim3(64), 0, st, seq0 + z, len - 1, 0,
                           ids[(int64_t)z * len + len - 1], b->d_pos, b->d_step, b->d_hist, b->max_ctx,
                           (const uint4*)e->w.embed, (uint4*)b->x_res, (int64_t)H / 8, 0, rope_cur_args(b));
        QIE_LAUNCH_CHECK();
    }
    const uint16_t* last = b->pf_x + (int64_t)(len - 1) * H;
    if (n_seqs > 1) {   // the last rows, packed (the head's pre-norm reads contiguous rows)
        QIE_HIP(hipMemcpy2DAsync(b->pf_hn, (size_t)H * 2, last, (size_t)len * H * 2, (size_t)H * 2, n_seqs,
                                 hipMemcpyDeviceToDevice, st));
        last = b->pf_hn;
    }
    QIE_TRY(enqueue_head(b, last, H, seq0, n_seqs, smp));
    for (int z = 0; z < n_seqs; z++) b->h_pos[seq0 + z] = len;
    if (next_ids) {
        QIE_HIP(hipMemcpyAsync(next_ids, b->d_ids + seq0, (size_t)n_seqs * 4, hipMemcpyDeviceToHost, st));
        QIE_HIP(hipStreamSynchronize(st));
        QIE_TRY(comm_check(e, who));
    }
    return 0;
}

int qie_prefill(qie_batch* b, int32_t seq, const int32_t* ids, int32_t n, const qie_sampling* smp, int32_t* next_id) {
    return prefill_rows(b, seq, 1, ids, n, smp, next_id, "qie_prefill");
}

int qie_prefill_batch(qie_batch* b, int32_t seq0, int32_t n_seqs, const int32_t* ids, int32_t len,
                      const qie_sampling* smp, int32_t* next_ids) {
    return prefill_rows(b, seq0, n_seqs, ids, len, smp, next_ids, "qie_prefill_batch");
}

static bool same_sampling(const qie_sampling& a, const qie_sampling* b) {
    qie_sampling g{1, 0.f, 1.f, 0};
    const qie_sampling& bb = b ? *b : g;
    return a.top_k == bb.top_k && a.temperature == bb.temperature && a.top_p == bb.top_p && a.seed == bb.seed;
}

static int launch_step(qie_batch* b, const qie_sampling* smp) {
    qie_engine* e = b->e;
    if (!e->opts.use_graph) return enqueue_decode(b, smp);
    if (!b->graph_ok || !same_sampling(b->gs, smp)) {
        if (b->gexec) hipGraphExecDestroy(b->gexec);
        b->gexec = nullptr;
        b->graph_ok = false;
        hipGraph_t g = nullptr;
        QIE_HIP(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        int rc = enqueue_decode(b, smp);
        hipError_t he = hipStreamEndCapture(e->stream, &g);
        if (rc) {
            if (g) hipGraphDestroy(g);
            return rc;
        }
        if (he != hipSuccess) return fail((int)he, "graph capture: %s", hipGetErrorString(he));
        if (dev_env("QIE_GRAPH_DUMP", 0)) {   // dev: every node of the decode graph (type, grid, block, LDS)
            size_t n = 0;
            hipGraphGetNodes(g, nullptr, &n);
            std::vector<hipGraphNode_t> nodes(n);
            hipGraphGetNodes(g, nodes.data(), &n);
            size_t max_shm = 0;
            for (size_t i = 0; i < n; i++) {
                hipGraphNodeType t;
                hipGraphNodeGetType(nodes[i], &t);
                if (t == hipGraphNodeTypeKernel) {
                    hipKernelNodeParams kp{};
                    hipGraphKernelNodeGetParams(nodes[i], &kp);
                    max_shm = std::max(max_shm, (size_t)kp.sharedMemBytes);
                    fprintf(stderr, "graph node %zu: kernel %p grid %u,%u,%u block %u,%u,%u dyn_lds %u\n", i, kp.func,
                            kp.gridDim.x, kp.gridDim.y, kp.gridDim.z, kp.blockDim.x, kp.blockDim.y, kp.blockDim.z,
                            kp.sharedMemBytes);
                } else {
                    fprintf(stderr, "graph node %zu: type %d\n", i, (int)t);
                }
            }
            fprintf(stderr, "graph: %zu nodes, max dynamic LDS %zu B\n", n, max_shm);
        }
        he = hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (he != hipSuccess) return fail((int)he, "graph instantiate: %s", hipGetErrorString(he));
        b->gs = smp ? *smp : qie_sampling{1, 0.f, 1.f, 0};
        b->graph_ok = true;
    }
    QIE_HIP(hipGraphLaunch(b->gexec, e->stream));
    return 0;
}

// Before n_steps decode steps: every live sequence fits max_ctx and holds the pages the
// steps write (positions h_pos .. h_pos + n_steps - 1); idle slots are rewound to
// position 0 when they would run past max_ctx.  Nothing is launched on failure.
static int prepare_steps(qie_batch* b, int n_steps, const char* who) {
    QIE_REQUIRE(n_steps < b->max_ctx, "%s: %d steps exceed max_ctx %d", who, n_steps, b->max_ctx);
    for (int m = 0; m < b->B; m++)
        if (!b->idle[m])
            QIE_REQUIRE(b->h_pos[m] + n_steps < b->max_ctx, "%s: sequence %d would exceed max_ctx %d", who, m,
                        b->max_ctx);
    if (b->d_table) {
        int64_t need = 0;
        for (int m = 0; m < b->B; m++)
            if (!b->idle[m])
                need += std::max<int64_t>(0, (b->h_pos[m] + n_steps + b->page_tokens - 1) / b->page_tokens - b->held[m]);
        QIE_REQUIRE(need <= (int64_t)b->free_pages.size(), "%s: KV pool exhausted (%lld pages needed, %zu free)", who,
                    (long long)need, b->free_pages.size());
        for (int m = 0; m < b->B; m++)
            if (!b->idle[m]) QIE_TRY(ensure_pages(b, m, b->h_pos[m] + n_steps));
        QIE_TRY(flush_table(b));
    }
    qie_engine* e = b->e;
    for (int m = 0; m < b->B; m++)
        if (b->idle[m] && b->h_pos[m] + n_steps >= b->max_ctx) {
            hipLaunchKernelGGL(set_state_kernel, dim3(1), dim3(256), 0, e->stream, m, 0, 0, 0, b->d_pos, b->d_step,
                               b->d_hist, b->max_ctx, (const uint4*)e->w.embed, (uint4*)b->x_res,
                               (int64_t)e->spec.hidden / 8, 1, rope_cur_args(b));
            QIE_LAUNCH_CHECK();
            b->h_pos[m] = 0;
        }
    return 0;
}

int qie_decode_step(qie_batch* b, const qie_sampling* smp, int32_t* next_ids) {
    QIE_REQUIRE(b, "qie_decode_step: null batch");
    QIE_TRY(prepare_steps(b, 1, "qie_decode_step"));
    QIE_TRY(launch_step(b, smp));
    for (int m = 0; m < b->B; m++) b->h_pos[m] += 1;
    return sync_ids(b, next_ids);
}

int qie_decode(qie_batch* b, int32_t n_steps, const qie_sampling* smp, int32_t* out_ids) {
    QIE_REQUIRE(b && n_steps >= 0, "qie_decode: bad arguments");
    QIE_TRY(prepare_steps(b, n_steps, "qie_decode"));
    std::vector<int32_t> p0 = b->h_pos;
    for (int i = 0; i < n_steps; i++) {
        QIE_TRY(launch_step(b, smp));
        for (int m = 0; m < b->B; m++) b->h_pos[m] += 1;
    }
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    QIE_TRY(comm_check(b->e, "qie_decode"));
    QIE_TRY(pk_check(b));
    if (out_ids && n_steps > 0) {
        std::vector<int32_t> row(b->max_ctx);
        for (int m = 0; m < b->B; m++) {
            QIE_HIP(d2h(b->e, row.data(), b->d_hist + (int64_t)m * b->max_ctx, (size_t)b->max_ctx * 4));
            for (int i = 0; i < n_steps; i++) out_ids[(int64_t)i * b->B + m] = row[p0[m] + 1 + i];
        }
    }
    return 0;
}

int qie_batch_logits(qie_batch* b, void* host_out) {
    QIE_REQUIRE(b && host_out, "qie_batch_logits: bad arguments");
    const uint16_t* src = b->logits;
    if (use_comm(b->e)) {   // collective: every rank calls this at the same point
        QIE_TRY(gather_logits(b, 0, b->B));
        src = b->logits_full;
    }
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    QIE_TRY(comm_check(b->e, "qie_batch_logits"));
    QIE_TRY(pk_check(b));
    QIE_HIP(d2h(b->e, host_out, src, (size_t)b->B * b->e->spec.vocab * 2));
    return 0;
}

int qie_batch_positions(qie_batch* b, int32_t* host_pos) {
    QIE_REQUIRE(b && host_pos, "qie_batch_positions: bad arguments");
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    QIE_HIP(d2h(b->e, host_pos, b->d_pos, (size_t)b->B * 4));
    return 0;
}

int qie_batch_history(qie_batch* b, int32_t seq, int32_t* host_ids, int32_t n) {
    QIE_REQUIRE(b && host_ids && seq >= 0 && seq < b->B && n >= 0 && n <= b->max_ctx,
                "qie_batch_history: bad arguments");
    QIE_HIP(hipStreamSynchronize(b->e->stream));
    QIE_HIP(d2h(b->e, host_ids, b->d_hist + (int64_t)seq * b->max_ctx, (size_t)n * 4));
    return 0;
}

int qie_batch_set_position(qie_batch* b, int32_t seq, int32_t pos, int32_t token) {
    QIE_REQUIRE(b && seq >= 0 && seq < b->B && pos >= 0 && pos + 1 < b->max_ctx && token >= 0 &&
                    token < b->e->spec.vocab,
                "qie_batch_set_position: bad arguments");
    QIE_TRY(ensure_pages(b, seq, (int64_t)pos + 1));
    QIE_TRY(flush_table(b));
    b->idle[seq] = 0;
    qie_engine* e = b->e;
    hipLaunchKernelGGL(set_state_kernel, dim3(1), dim3(256), 0, e->stream, seq, pos, pos, token, b->d_pos, b->d_step,
                       b->d_hist, b->max_ctx, (const uint4*)e->w.embed, (uint4*)b->x_res,
                       (int64_t)e->spec.hidden / 8, 1, rope_cur_args(b));
    QIE_LAUNCH_CHECK();
    QIE_HIP(hipStreamSynchronize(e->stream));
    b->h_pos[seq] = pos;
    return 0;
}

int qie_batch_set_decode_mode(qie_batch* b, int32_t mode) {
    QIE_REQUIRE(b && (mode == 0 || mode == 1), "qie_batch_set_decode_mode: bad arguments (mode 0 or 1)");
    qie_engine* e = b->e;
    if (mode == 1) {
        const char* why = "";
        QIE_REQUIRE(persist_supported(e->spec, b->B, e->sh.tp, e->fp8, b->d_table != nullptr, device_cu_count(), &why),
                    "qie_batch_set_decode_mode: the persistent decode step does not cover this batch (%s)", why);
        if (!b->pk_mem || !b->d_layers || !b->d_attp) {
            // all three or none: a failed allocation leaves the batch in mode 0 with nothing held
            const size_t gb = (size_t)persist_granule_count(e->spec) * 8 + 64;
            hipFree(b->pk_mem);
            hipFree(b->d_layers);
            hipFree(b->d_attp);
            b->pk_mem = nullptr;
            b->d_layers = nullptr;
            b->d_attp = nullptr;
            void *pk = nullptr, *dl = nullptr, *ap = nullptr;
            if (dmalloc(&pk, gb) || dmalloc(&dl, sizeof(qie_layer_weights) * e->layers.size()) ||
                dmalloc(&ap, persist_attn_table_bytes((int)e->layers.size()))) {
                hipFree(pk);
                hipFree(dl);
                hipFree(ap);
                return fail(-2, "qie_batch_set_decode_mode: device allocation failed: %s", qie_last_error());
            }
            b->pk_mem = pk;
            b->d_layers = (qie_layer_weights*)dl;
            b->d_attp = ap;
            QIE_HIP(hipMemsetAsync(b->pk_mem, 0, gb, e->stream));
            QIE_HIP(hipMemcpyAsync(b->d_layers, e->layers.data(), sizeof(qie_layer_weights) * e->layers.size(),
                                   hipMemcpyHostToDevice, e->stream));
            const qie_kv_cache cache = batch_cache(b, 0);
            set_decode_rope_cur(b->d_rope_cur);
            const int rc = persist_attn_table(e->spec, e->layers.data(), b->qkv, b->d_pos, e->rope_cos, e->rope_sin,
                                              &cache, b->dec_ws, b->d_attp, e->stream);
            set_decode_rope_cur(nullptr);
            QIE_TRY(rc);
            QIE_HIP(hipStreamSynchronize(e->stream));
        }
    }
    if (mode != b->decode_mode) b->graph_ok = false;   // re-captured at the next step
    b->decode_mode = mode;
    return 0;
}

int qie_batch_decode_mode(const qie_batch* b) { return b ? b->decode_mode : -22; }

int qie_batch_pk_trace(qie_batch* b, int32_t enable, uint64_t* host_out, int64_t n) {
    QIE_REQUIRE(b, "qie_batch_pk_trace: null batch");
    qie_engine* e = b->e;
    const int64_t need = (int64_t)device_cu_count() * e->spec.n_layers * persist_ts_slots();
    if (enable && !b->pk_ts) {
        QIE_TRY(dmalloc((void**)&b->pk_ts, (size_t)need * 8));
        QIE_HIP(hipMemsetAsync(b->pk_ts, 0, (size_t)need * 8, e->stream));
        b->graph_ok = false;
    }
    if (host_out) {
        QIE_REQUIRE(b->pk_ts && n >= need, "qie_batch_pk_trace: tracing off or n < %lld", (long long)need);
        QIE_HIP(hipStreamSynchronize(e->stream));
        QIE_HIP(d2h(e, host_out, b->pk_ts, (size_t)need * 8));
    }
    if (!enable && b->pk_ts) {
        QIE_HIP(hipStreamSynchronize(e->stream));
        hipFree(b->pk_ts);
        b->pk_ts = nullptr;
        b->graph_ok = false;
    }
    return 0;
}

int qie_batch_dims(const qie_batch* b, int32_t* batch, int32_t* max_ctx) {
    QIE_REQUIRE(b, "qie_batch_dims: null batch");
    if (batch) *batch = b->B;
    if (max_ctx) *max_ctx = b->max_ctx;
    return 0;
}

int qie_batch_kv_cache(const qie_batch* b, int32_t seq, qie_kv_cache* out) {
    QIE_REQUIRE(b && out && seq >= 0 && seq < b->B, "qie_batch_kv_cache: bad arguments");
    *out = batch_cache(b, seq);
    return 0;
}

int qie_batch_reserve(qie_batch* b, int32_t seq, int32_t n_tokens) {
    QIE_REQUIRE(b && seq >= 0 && seq < b->B && n_tokens >= 0, "qie_batch_reserve: bad arguments");
    QIE_REQUIRE(n_tokens <= b->max_ctx, "qie_batch_reserve: %d tokens exceed max_ctx %d", n_tokens, b->max_ctx);
    QIE_TRY(ensure_pages(b, seq, n_tokens));
    QIE_TRY(flush_table(b));
    b->idle[seq] = 0;
    return 0;
}

int qie_engine_arena(const qie_engine* e, void** base, int64_t* bytes) {
    QIE_REQUIRE(e && e->have_weights, "qie_engine_arena: engine has no weights");
    if (base) *base = e->arena;
    if (bytes) *bytes = (int64_t)e->arena_bytes;
    return 0;
}

int qie_engine_rope_tables(const qie_engine* e, const float** rope_cos, const float** rope_sin, int32_t* rows) {
    QIE_REQUIRE(e, "qie_engine_rope_tables: null engine");
    if (rope_cos) *rope_cos = e->rope_cos;
    if (rope_sin) *rope_sin = e->rope_sin;
    if (rows) *rows = e->rope_rows;
    return 0;
}

// Live per-kernel timing (bench.py's roofline line).  The launches cycle through layers
// 1 .. L-1 (layer 0 where L == 1), as the decode step does: replaying ONE layer's weights
// back to back would leave a ~272 MB gate/up working set largely in the 256 MiB Infinity
// Cache and time a cache hit rate no decode step sees (round-1 verdict).  lm_head (which 4)
// has one weight; its 1.09 GB stream cannot stay resident.
// which == 6: the persistent layer stack (k_persist.hip) alone, `iters` back-to-back launches at
// the current position.  Each launch gets its own hand-off epoch (a device array of fresh
// values, so no kernel runs between the timed launches); the residual row is restored and the
// real epoch advanced past them afterwards, and the KV rows the launches wrote at the current
// position are rewritten by the next real step.  Bytes: every layer weight read once plus the
// K / V rows the attention reads.
static int time_persistent(qie_batch* b, int iters, double* avg_us, double* bytes) {
    qie_engine* e = b->e;
    const qie_model_spec& s = e->spec;
    QIE_REQUIRE(b->decode_mode == 1 && b->pk_mem, "qie_batch_time_kernel: which 6 needs decode mode 1");
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)s.n_heads * hd, KD = (int64_t)s.n_kv_heads * hd,
                  I = s.ffn;
    int32_t pos = 0;
    unsigned ep = 0;
    QIE_HIP(d2h(e, &pos, b->d_pos, 4));
    QIE_HIP(d2h(e, &ep, pk_epoch_ptr(b), 4));
    const int n = iters + 4;
    std::vector<unsigned> eps(n);
    for (int i = 0; i < n; i++) eps[i] = ep + 1 + (unsigned)i;
    unsigned* d_eps = nullptr;
    uint16_t* xsave = nullptr;
    QIE_TRY(dmalloc((void**)&d_eps, n * 4));
    QIE_TRY(dmalloc((void**)&xsave, H * 2));
    QIE_HIP(hipMemcpyAsync(d_eps, eps.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    QIE_HIP(hipMemcpyAsync(xsave, b->x_res, H * 2, hipMemcpyDeviceToDevice, e->stream));
    // launches back to back on the same input: x_res is only read at layer 0 and written at the
    // last layer, so each launch sees a row of the same magnitude (restored afterwards)
    auto run = [&](int i) {
        return persist_decode_launch(s, b->d_layers, b->d_attp, b->x_res, (unsigned long long*)b->pk_mem, d_eps + i,
                                     pk_epoch_ptr(b) + 1, b->d_pos, pk_splits_target(b), nullptr, e->stream);
    };
    hipEvent_t t0, t1;
    QIE_HIP(hipEventCreate(&t0));
    QIE_HIP(hipEventCreate(&t1));
    for (int i = 0; i < 4; i++) QIE_TRY(run(i));
    QIE_HIP(hipEventRecord(t0, e->stream));
    for (int i = 0; i < iters; i++) QIE_TRY(run(4 + i));
    QIE_HIP(hipEventRecord(t1, e->stream));
    QIE_HIP(hipEventSynchronize(t1));
    float ms = 0;
    QIE_HIP(hipEventElapsedTime(&ms, t0, t1));
    hipEventDestroy(t0);
    hipEventDestroy(t1);
    const unsigned ep_after = ep + (unsigned)n + 1;
    QIE_HIP(hipMemcpyAsync(b->x_res, xsave, H * 2, hipMemcpyDeviceToDevice, e->stream));
    QIE_HIP(hipMemcpyAsync(pk_epoch_ptr(b), &ep_after, 4, hipMemcpyHostToDevice, e->stream));
    QIE_HIP(hipStreamSynchronize(e->stream));
    hipFree(d_eps);
    hipFree(xsave);
    QIE_TRY(pk_check(b));
    const double per_layer = (double)(QD + 2 * KD) * H * 2 + (double)(QD + 2 * KD) * 2 * (s.qkv_bias ? 1 : 0) +
                             (double)H * QD * 2 + 2.0 * I * H * 2 + (double)H * I * 2 + 2.0 * H * 2 +
                             (double)(pos + 1) * KD * 2 * 2;
    *bytes = per_layer * s.n_layers;
    *avg_us = ms * 1000.0 / iters;
    return 0;
}

int qie_batch_time_kernel(qie_batch* b, int32_t which, int32_t iters, double* avg_us, double* bytes) {
    QIE_REQUIRE(b && iters > 0 && avg_us && bytes && which >= 0 && which <= 6, "qie_batch_time_kernel: bad arguments");
    qie_engine* e = b->e;
    if (which == 6) return time_persistent(b, iters, avg_us, bytes);
    const qie_model_spec& s = e->spec;
    const TpShard& sh = e->sh;   // this rank's shard sizes
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)sh.nq * hd, KD = (int64_t)sh.nkv * hd;
    const int64_t I = sh.ffn, B = b->B, V = sh.vocab;
    // scratch output so timing never disturbs the sequence state
    uint16_t* scratch = nullptr;
    QIE_TRY(dmalloc((void**)&scratch,
                    (size_t)B * std::max<int64_t>(std::max(I, V), QD + 2 * KD) * 2 + B * 8 + 64));
    const double wb = e->fp8 ? 1.0 : 2.0;   // weight bytes per element (fp8 row scales: negligible)
    const bool batched_norm = B >= 2 && dev_env("QIE_PRENORM", 1) != 0;
    auto args_for = [&](int l, double* by) {
        const qie_layer_weights& L = e->layers[l];
        qie_linear_args a = which == 4 ? lin_base(e) : lin_proj(e);
        if (which == 4 && e->fp8_t16_head) a.flags |= QIE_LINEAR_FP8_T16;
        if (which == 0) {
            a.x = b->x_res; a.ldx = H; a.w[0] = L.w_gate; a.w[1] = L.w_up; a.seg_rows[0] = I; a.seg_rows[1] = I;
            a.M = B; a.K = H; a.N = I; a.y = scratch; a.ldy = I; a.epilogue = QIE_EPI_SWIGLU;
            a.norm_w = L.ffn_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
            *by = 2.0 * I * H * wb + B * H * 2 + H * 2 + B * I * 2;
        } else if (which == 1) {
            a.x = b->h; a.ldx = I; a.w[0] = L.w_down; a.seg_rows[0] = H;
            a.M = B; a.K = I; a.N = H; a.y = scratch; a.ldy = H; a.epilogue = QIE_EPI_STORE;
            *by = (double)H * I * wb + B * I * 2 + B * H * 2;
        } else if (which == 2) {
            a.x = b->x_res; a.ldx = H; a.w[0] = L.wq; a.w[1] = L.wk; a.w[2] = L.wv;
            a.bias[0] = L.bq; a.bias[1] = L.bk; a.bias[2] = L.bv;
            a.seg_rows[0] = QD; a.seg_rows[1] = KD; a.seg_rows[2] = KD;
            a.M = B; a.K = H; a.N = QD + 2 * KD; a.y = scratch; a.ldy = QD + 2 * KD; a.epilogue = QIE_EPI_STORE;
            a.norm_w = L.attn_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
            *by = (double)(QD + 2 * KD) * H * wb + B * H * 2 + B * (QD + 2 * KD) * 2;
        } else if (which == 3) {
            a.x = b->att; a.ldx = QD; a.w[0] = L.wo; a.seg_rows[0] = H;
            a.M = B; a.K = QD; a.N = H; a.y = scratch; a.ldy = H; a.epilogue = QIE_EPI_STORE;
            *by = (double)H * QD * wb + B * QD * 2 + B * H * 2;
        } else if (which == 4) {
            a.x = b->x_res; a.ldx = H; a.w[0] = e->w.lm_head; a.seg_rows[0] = V;
            a.M = B; a.K = H; a.N = V; a.y = scratch; a.ldy = V; a.epilogue = QIE_EPI_STORE;
            a.norm_w = e->w.final_norm; a.norm_eps = s.rms_eps; a.numerics = s.numerics;
            a.argmax_keys = (uint64_t*)(((uintptr_t)(scratch + B * V) + 7) & ~(uintptr_t)7);   // as the greedy step runs it
            *by = (double)V * H * wb + B * H * 2 + B * (double)V * 2;
        }
        // as prenorm() decides for the real step: the fp8 batched-decode kernel keeps its fused norm
        const bool fused8 = dec8_applies(&a) && dev_env("QIE_DEC8_PRENORM", 0) == 0;
        if (batched_norm && a.norm_w && !fused8) {
            a.x = b->xn;   // as the batched step runs it: rows normed once by prenorm(), plain GEMV
            a.ldx = a.K;
            a.norm_w = nullptr;
        }
        return a;
    };
    double by = 0;
    if (which == 5) {
        std::vector<int32_t> pos(B);
        QIE_HIP(d2h(e, pos.data(), b->d_pos, B * 4));
        for (int m = 0; m < B; m++) by += (double)(pos[m] + 1) * KD * 2 * 2;
        by += (double)B * QD * 2 * 2;
    }
    const qie_kv_cache cache = batch_cache(b, 0);
    const int nl = s.n_layers;
    auto layer_of = [&](int i) { return which == 4 || nl == 1 ? 0 : 1 + i % (nl - 1); };
    auto run = [&](int i) -> int {
        const int l = layer_of(i);
        const qie_layer_weights& L = e->layers[l];
        const bool rp = rope_in_projection(b);
        if (which == 5) {
            set_decode_rope_cur(b->d_rope_cur);
            const int rc = qie_attention_decode(b->qkv, B, b->d_pos, L.q_norm, L.k_norm, e->rope_cos, e->rope_sin,
                                                sh.nq, &cache, l, s.rms_eps, s.numerics | (rp ? QIE_ATTN_PREROPED : 0),
                                                scratch, b->dec_ws, e->stream);
            set_decode_rope_cur(nullptr);
            return rc;
        }
        double lb = 0;
        qie_linear_args a = args_for(l, &lb);
        if (which == 2 && rp)   // as the step runs it
            return gemv_rope(&a, b->d_pos, e->rope_cos, e->rope_sin, (int)s.head_dim, QD + KD, e->stream);
        return qie_linear(&a, e->stream);
    };
    if (which != 5) args_for(0, &by);
    hipEvent_t t0, t1;
    QIE_HIP(hipEventCreate(&t0));
    QIE_HIP(hipEventCreate(&t1));
    for (int i = 0; i < std::min(nl, 4); i++) QIE_TRY(run(i));   // warm-up
    QIE_HIP(hipEventRecord(t0, e->stream));
    for (int i = 0; i < iters; i++) QIE_TRY(run(i));
    QIE_HIP(hipEventRecord(t1, e->stream));
    QIE_HIP(hipEventSynchronize(t1));
    float ms = 0;
    QIE_HIP(hipEventElapsedTime(&ms, t0, t1));
    hipEventDestroy(t0);
    hipEventDestroy(t1);
    hipFree(scratch);
    *avg_us = ms * 1000.0 / iters;
    *bytes = by;
    return 0;
}

int qie_batch_debug_step(qie_batch* b, const qie_sampling* smp, int32_t* next_ids, void* host_x) {
    QIE_REQUIRE(b && host_x, "qie_batch_debug_step: bad arguments");
    qie_engine* e = b->e;
    const int64_t n = (int64_t)b->B * e->spec.hidden, slots = 2 * (int64_t)e->spec.n_layers + 1;
    QIE_TRY(prepare_steps(b, 1, "qie_batch_debug_step"));
    QIE_TRY(dmalloc((void**)&b->dbg_x, (size_t)(slots * n * 2)));
    int rc = dbg_snap(b, 0);
    if (!rc) rc = enqueue_decode(b, smp);   // eager: the graph (if any) is left as it is
    hipError_t he = hipStreamSynchronize(e->stream);
    if (!rc && he == hipSuccess) he = d2h(e, host_x, b->dbg_x, (size_t)(slots * n * 2));
    hipFree(b->dbg_x);
    b->dbg_x = nullptr;
    QIE_TRY(rc);
    QIE_HIP(he);
    for (int m = 0; m < b->B; m++) b->h_pos[m] += 1;
    return sync_ids(b, next_ids);
}

int qie_linear(const qie_linear_args* a, void* stream) {
    QIE_REQUIRE(a && a->x && a->y && a->w[0] && a->M > 0 && a->K > 0 && a->N > 0, "qie_linear: bad arguments");
    QIE_REQUIRE(a->K % 8 == 0 && a->ldx >= a->K && a->ldx % 8 == 0, "qie_linear: K and ldx must be multiples of 8");
    QIE_REQUIRE(((uintptr_t)a->x % 16) == 0, "qie_linear: x must be 16-byte aligned");
    for (int i = 0; i < 3; i++)
        QIE_REQUIRE(((uintptr_t)a->w[i] % 16) == 0, "qie_linear: weight segment %d must be 16-byte aligned", i);
    if (a->epilogue == QIE_EPI_SWIGLU) {
        QIE_REQUIRE(a->w[1] && a->seg_rows[0] == a->N && a->seg_rows[1] == a->N && a->ldy >= a->N,
                    "qie_linear: SWIGLU needs w[0]=gate, w[1]=up with N rows each");
    } else {
        QIE_REQUIRE(a->seg_rows[0] + a->seg_rows[1] + a->seg_rows[2] == a->N && a->ldy >= a->N,
                    "qie_linear: seg_rows must sum to N");
        QIE_REQUIRE(a->seg_rows[1] == 0 || a->w[1], "qie_linear: missing weight segment 1");
        QIE_REQUIRE(a->seg_rows[2] == 0 || a->w[2], "qie_linear: missing weight segment 2");
    }
    QIE_REQUIRE(a->epilogue >= 0 && a->epilogue <= 3, "qie_linear: bad epilogue");
    QIE_REQUIRE(a->epilogue != QIE_EPI_F32 || (a->bias[0] == nullptr && a->bias[1] == nullptr && a->bias[2] == nullptr),
                "qie_linear: F32 (partial-sum) epilogue takes no bias");
    QIE_REQUIRE(a->argmax_keys == nullptr || a->epilogue == QIE_EPI_STORE, "qie_linear: arg-max needs STORE");
    const bool act_fp8 = (a->flags & QIE_LINEAR_ACT_FP8) != 0;
    hipStream_t st = (hipStream_t)stream;
    if (act_fp8) return gemm(a, st);   // fp8 activations: the block-scaled MFMA GEMM at every M
    QIE_REQUIRE(!(a->flags & QIE_LINEAR_FP8_T16) ||
                    ((a->flags & QIE_LINEAR_FP8) && a->M >= 1 && a->M <= 16 && a->K % 64 == 0 &&
                     (a->epilogue == QIE_EPI_SWIGLU ? a->N % 16 == 0
                                                    : a->seg_rows[0] % 16 == 0 && a->seg_rows[1] % 16 == 0 &&
                                                          a->seg_rows[2] % 16 == 0)),
                "qie_linear: 16-row tiled fp8 weights are read by the batched-decode kernels only (M <= 16, K %% 64 == 0, "
                "segments of whole 16-row tiles) and, with fp8 activations, the block-scaled GEMM");
    if (a->M <= 16) return gemv(a, st);   // GEMV (M = 1..8) or the skinny MFMA kernel (2..16)
    return gemm(a, st);
}

}  // extern "C"
