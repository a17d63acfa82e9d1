// compat.hpp — the reference engine's host entry points, by name, over the qie C ABI.
//
// A host driver written against Rafae1130/qwen_inference_engine's C++ API keeps its
// shape: parsed_tensors / build_indexed_tensors (layers/src/tensor_parser.cpp:31-165),
// load_all_weights_to_gpu_chunked (layers/src/iengine.cu:117-223), create_new_sequence
// (iengine.cu:25-47), llm (layers/src/qwen_main.cu:64-417) with batch_metadata.state
// selecting prefill or ONE decode step, and the caller advancing step /
// generated_token / state exactly like iengine.cu:419-421.
//
// Two forms of the driver tier:
//   * the reference's own argument lists (iengine.cuh:51-55, iengine.cu:25,117,
//     tensor_parser.hh:216-219): llm(seq, tensors, weights, kv_head, page_size,
//     g_gpu_weights_buffer), create_new_sequence(id, ids, len, tensors, weights),
//     create_page_list(n), allocate_page_buffers(node, elems),
//     load_all_weights_to_gpu_chunked(all, ifstream, h_host, chunk, d_base&, total&),
//     parsed_tensors(), build_indexed_tensors() — a host written against iengine.cu:226-456
//     compiles against this header unchanged (csrc/tools/ref_driver.cpp is one);
//   * qie-native overloads taking a qie_batch slot explicitly (llm(seq, sampling), ...).
// Differences (deliberate):
//   * bf16 is uint16_t storage (no __nv_bfloat16); device memory comes from qie_malloc.
//   * the model is config().spec (default: the reference's Qwen3-14B literals,
//     utills.cu:8-16), not compiled-in constants; parsed_tensors() reads the
//     meta_data.txt index at config().meta_path (the reference re-parses safetensors
//     shards at hard-coded /mnt/data paths, tensor_parser.cpp:37-46).
//   * the KV cache lives in a qie_batch the first llm() call binds to the sequence; the
//     page list only records capacity (no per-node device buffers).
//   * llm() returns 0 on error like the reference (qwen_main.cu:135 ...), the text in
//     qie_last_error() and the code in config().error.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "qie_engine.h"

namespace qie_compat {

using bf16 = uint16_t;
struct ModelBuffers;

// Settings the reference compiles in: the model (utills.cu:8-16), eps (normalization.cu:19),
// context (iengine.cuh:19), index path (tensor_parser.cpp:34), sampling (qwen_main.cu).
inline qie_model_spec reference_spec() {   // Qwen3-14B (utills.cu:8-16, iengine.cuh:19-21)
    qie_model_spec s;
    std::memset(&s, 0, sizeof(s));
    s.n_layers = 40; s.hidden = 5120; s.n_heads = 40; s.n_kv_heads = 8; s.head_dim = 128;
    s.ffn = 17408; s.vocab = 151936; s.tie_embeddings = 0; s.qkv_bias = 0; s.qk_norm = 1;
    s.rms_eps = 1e-4f; s.rope_theta = 1e6f; s.numerics = QIE_NUMERICS_REF;
    return s;
}

struct Config {
    float rms_eps = 1e-4f;
    float qk_eps = 1e-4f;
    int32_t numerics = QIE_NUMERICS_REF;
    void* stream = nullptr;
    int error = 0;        // last non-zero qie return code seen by a compat wrapper
    // driver tier (reference-signature form)
    qie_model_spec spec = reference_spec();
    int32_t max_ctx = 32786;                            // CONTEXT_SIZE, iengine.cuh:19
    int32_t device = 0;                                 // iengine.cu:238-240
    std::string meta_path = "../model_files/meta_data.txt";   // tensor_parser.cpp:34
    int greedy = 0;       // 1: llm() decodes greedily instead of the reference's top-k schedule
};
inline Config& config() {
    static Config c;
    return c;
}
// the arena the last reference-form load_all_weights_to_gpu_chunked call filled (the
// reference-form initialize_model_buffers binds the engine to it)
inline bf16*& loaded_arena_() {
    static bf16* p = nullptr;
    return p;
}
inline void check_(int rc, const char* who) {
    if (rc != 0) {
        config().error = rc;
        std::fprintf(stderr, "%s: %s\n", who, qie_last_error());
    }
}

struct tensor {                       // tensor_parser.hh:204-210
    std::string tensor_name;
    std::vector<size_t> shape;
    std::vector<size_t> data_offsets;
    int layer_index = -1;
    std::string short_name;
};
using TensorTable = std::unordered_map<std::string, std::vector<tensor>>;

typedef enum { prefill, decode } State;   // iengine.cuh:23

// iengine.cuh:27-37 field for field (plain data: the reference mallocs and frees it), plus
// the qie slot that holds the sequence's KV cache and state.
struct batch_metadata {
    int sequence_id;
    bf16* k_ptr;          // the slot's K / V cache base once bound (qie_batch_kv_cache)
    bf16* v_ptr;
    State state;
    int sequence_len;
    int generated_token;
    int step;
    ModelBuffers* buffer;
    qie_batch* batch;     // qie: bound by the first llm() (reference form) or given
    int slot;
    int last_token;       // qie: the engine's last output (a different generated_token is fed back)
};

// Reference sampling schedule, qwen_main.cu:241 (prefill) and :381-388 (decode).
inline qie_sampling reference_sampling(State s) {
    qie_sampling q;
    q.top_k = 50;
    q.temperature = s == prefill ? 1.0f : 0.7f;
    q.top_p = 1.0f;
    q.seed = 1234;        // + per-sequence step on device (1234 + step, as the reference)
    return q;
}
constexpr int32_t kRefEos = 151645;   // qwen_main.cu:257

inline std::vector<tensor> parsed_tensors(const char* meta_data_txt) {
    std::vector<tensor> out;
    qie_index* idx = nullptr;
    if (qie_index_load_meta(meta_data_txt, &idx) != 0) return out;
    const int n = qie_index_count(idx);
    for (int i = 0; i < n; i++) {
        const char *name, *sn;
        int32_t layer, nd;
        int64_t o0, o1, shp[4];
        qie_index_get(idx, i, &name, &sn, &layer, &o0, &o1, &nd, shp);
        tensor t;
        t.tensor_name = name;
        t.short_name = sn;
        t.layer_index = layer;
        t.data_offsets = {(size_t)o0, (size_t)o1};
        for (int k = 0; k < nd; k++) t.shape.push_back((size_t)shp[k]);
        out.push_back(t);
    }
    qie_index_destroy(idx);
    return out;
}

inline TensorTable build_indexed_tensors(const std::vector<tensor>& all) {
    TensorTable idx;
    for (const auto& t : all) {
        auto& v = idx[t.short_name];
        const size_t li = t.layer_index >= 0 ? (size_t)t.layer_index : 0;
        if (v.size() <= li) v.resize(li + 1);
        v[li] = t;
    }
    return idx;
}

// Reference forms (tensor_parser.hh:216-219): no arguments, the index at config().meta_path.
inline std::vector<tensor> parsed_tensors() { return parsed_tensors(config().meta_path.c_str()); }
inline TensorTable build_indexed_tensors() { return build_indexed_tensors(parsed_tensors()); }

// load_all_weights_to_gpu_chunked, reference form (iengine.cu:117-223): one device
// allocation of min(max data_offsets[1], file size) bytes, filled from the open binary
// stream in chunk_bytes pieces staged through the caller's h_host; d_base_out is the arena
// (pass it to llm() as g_gpu_weights_buffer), total_bytes_out the bytes uploaded.
inline bool load_all_weights_to_gpu_chunked(const std::vector<tensor>& all_tensors, std::ifstream& f, void* h_host,
                                            size_t chunk_bytes, bf16*& d_base_out, size_t& total_bytes_out) {
    d_base_out = nullptr;
    total_bytes_out = 0;
    if (!f.is_open() || !h_host || chunk_bytes == 0) {
        std::fprintf(stderr, "load_all_weights_to_gpu_chunked: stream not open or no staging buffer\n");
        return false;
    }
    size_t max_end = 0;
    for (const auto& t : all_tensors)
        if (t.data_offsets.size() >= 2 && t.data_offsets[1] > max_end) max_end = t.data_offsets[1];
    f.clear();
    f.seekg(0, std::ios::end);
    const std::streamoff fsz = f.tellg();
    if (max_end == 0 || fsz <= 0) {
        std::fprintf(stderr, "load_all_weights_to_gpu_chunked: empty index or file\n");
        return false;
    }
    const size_t total = max_end < (size_t)fsz ? max_end : (size_t)fsz;
    void* d = nullptr;
    if (qie_set_device(config().device) != 0 || qie_malloc(&d, (int64_t)total) != 0) {
        check_(-12, "load_all_weights_to_gpu_chunked");
        return false;
    }
    f.clear();
    f.seekg(0, std::ios::beg);
    size_t off = 0;
    while (off < total) {
        const size_t want = chunk_bytes < total - off ? chunk_bytes : total - off;
        f.read(static_cast<char*>(h_host), (std::streamsize)want);
        const std::streamsize got = f.gcount();
        if (got <= 0 || qie_memcpy_h2d(static_cast<char*>(d) + off, h_host, (int64_t)got) != 0) {
            std::fprintf(stderr, "load_all_weights_to_gpu_chunked: read / copy failed at %zu\n", off);
            qie_free(d);
            return false;
        }
        off += (size_t)got;
        if ((size_t)got < want) break;   // short read before the end
    }
    d_base_out = static_cast<bf16*>(d);
    total_bytes_out = off;
    loaded_arena_() = d_base_out;
    return true;
}

// Loads weights.bin into the engine's single device arena in chunk_bytes pieces.
inline bool load_all_weights_to_gpu_chunked(qie_engine* e, const char* weights_bin, const char* meta_data_txt,
                                            size_t chunk_bytes) {
    return qie_engine_load_weights_bin(e, weights_bin, meta_data_txt, (int64_t)chunk_bytes) == 0;
}

inline batch_metadata* new_sequence_(int sequence_id, const int* h_token_ids, int sequence_len);

// qie-native form: the sequence lives in slot `slot` of an existing batch.
inline batch_metadata* create_new_sequence(int sequence_id, const int* h_token_ids, int sequence_len,
                                           qie_batch* batch, int slot) {
    batch_metadata* s = new_sequence_(sequence_id, h_token_ids, sequence_len);
    if (s) {
        s->batch = batch;
        s->slot = slot;
    }
    return s;
}

inline int llm_step_(batch_metadata* seq, const qie_sampling* sampling);

// One call = prefill (state == prefill) or ONE decode step (state == decode); returns
// the sampled token id, or 0 on error (the reference's convention, qwen_main.cu:135;
// qie_last_error() / config().error say what failed).  Greedy callers pass a qie_sampling
// with top_k = 1; nullptr follows the reference's schedule (reference_sampling).
inline int llm(batch_metadata* seq, const qie_sampling* sampling = nullptr) { return llm_step_(seq, sampling); }

inline void destroy_model_buffers(ModelBuffers& buf);
inline void destroy_sequence(batch_metadata* s);

// Page list (iengine.cuh:39-49, iengine.cu:73-109).  The reference gives each sequence a
// linked list of 4-token pages in managed memory (create_page_list, then
// allocate_page_buffers per node as the sequence grows, free_page_list at the end).  In
// qie every slot of a batch (paged: qie_batch_create_paged) draws pages from one pool
// behind a device block table, so a page_table here is the slot's handle:
// create_page_list reserves nothing up front, allocate_page_buffers grows the slot by
// one reference page's worth of positions, free_page_list returns the slot's pages.
// The reference-form list (create_page_list(n) + allocate_page_buffers(node, elems)) keeps
// the reference's nodes and fields; its K/V storage is the qie batch the sequence's first
// llm() binds, so k_page_ptr / v_page_ptr stay NULL and a node only counts capacity.
struct page_table {
    bf16* k_page_ptr = nullptr;          // iengine.cuh:42-48
    bf16* v_page_ptr = nullptr;
    int page_allocated = 0;
    page_table* ptr_to_next_page = nullptr;
    qie_batch* batch = nullptr;          // qie-native form: the slot this handle reserves in
    int slot = 0;
    int tokens = 0;   // positions reserved so far (allocate_page_buffers / kv writes)
    size_t elems = 0; // reference form: elements of this node (page_size * L * hidden_kv)
};

inline page_table* create_page_list(qie_batch* batch, int slot) {
    auto* p = new page_table();
    p->batch = batch;
    p->slot = slot;
    return p;
}

// create_page_list (iengine.cu:73-89): a list of pages_required unallocated nodes
inline page_table* create_page_list(int pages_required) {
    page_table* head = nullptr;
    page_table** cur = &head;
    for (int i = 0; i < pages_required; ++i) {
        *cur = new page_table();
        cur = &(*cur)->ptr_to_next_page;
    }
    return head;
}

// allocate_page_buffers (iengine.cu:90-100), reference form: marks the node allocated
inline void allocate_page_buffers(page_table* node, size_t elems_per_page) {
    if (!node) return;
    node->elems = elems_per_page;
    node->page_allocated = 1;
}

// free_page_list (iengine.cu:101-109): the whole list; a qie-native handle's pages
// return to its batch's pool
inline void free_page_list(page_table* head) {
    while (head) {
        page_table* next = head->ptr_to_next_page;
        if (head->batch && qie_batch_release(head->batch, head->slot) != 0)
            std::fprintf(stderr, "free_page_list: %s\n", qie_last_error());
        delete head;
        head = next;
    }
}

// ===================================================================== operator tier
// The reference's per-op host API (helpers.cuh:45-166, include_cuda.cu:165-279,
// utills.cu:4-205) over qie_ops.h, so a host that keeps the reference's own layer loop
// (qwen_main.cu:77-241 prefill, :271-359 decode) can be re-pointed op by op.
//   * bf16 tensors are device pointers to bf16 bits (uint16_t); no CUDA types.
//   * every launch goes to config().stream (default: the null stream, the reference's
//     legacy default-stream ordering); failures print qie_last_error() to stderr like
//     the reference's launch checks and set config().error.
//   * the reference hard-codes eps 1e-4 for rmsNorm and qkNorm (normalization.cu:19,
//     qk_norm.cu:70) and its model constants (utills.cu:8-16); here eps and numerics
//     come from config() (defaults: 1e-4, REF) and dims from the engine's spec.

// Device scratch the reference's launch helpers allocate per call (d_token in
// sample_topk_bf16, smem in launch_attn): positions, attention / sampling workspace.
struct Scratch {
    void* p = nullptr;
    int64_t bytes = 0;
    void* get(int64_t n) {   // never NULL on success (a zero-byte request still gets 256 B)
        n = n < 256 ? 256 : n;
        if (n > bytes) {
            if (p) qie_free(p);
            p = nullptr;
            bytes = 0;
            if (qie_malloc(&p, n) != 0) return nullptr;
            bytes = n;
        }
        return p;
    }
    ~Scratch() {
        if (p) qie_free(p);
    }
};
inline Scratch& scratch(int which) {
    static Scratch s[3];   // 0: positions, 1: attention ws, 2: sampling ws + token
    return s[which];
}

// assign_weight_pointer / load_weight (helpers.cuh:19-35): W = arena + data_offsets[0],
// nothing copied.  The ifstream and host staging pointer are kept for signature parity.
template <class T>
void assign_weight_pointer(const tensor& t, T*& d, bf16* g_gpu_weights_buffer) {
    d = reinterpret_cast<T*>(reinterpret_cast<char*>(g_gpu_weights_buffer) + t.data_offsets[0]);
}
template <class T>
void load_weight(const tensor& t, std::ifstream&, T*, T*& d, size_t, bf16* g_gpu_weights_buffer) {
    assign_weight_pointer(t, d, g_gpu_weights_buffer);
}

// load_all_weights_to_gpu_chunked (iengine.cu:117-223) in the reference's output form.
inline bool load_all_weights_to_gpu_chunked(qie_engine* e, const char* weights_bin, const char* meta_data_txt,
                                            size_t chunk_bytes, bf16*& d_base_out, size_t& total_bytes_out) {
    if (qie_engine_load_weights_bin(e, weights_bin, meta_data_txt, (int64_t)chunk_bytes) != 0) return false;
    void* base = nullptr;
    int64_t n = 0;
    if (qie_engine_arena(e, &base, &n) != 0) return false;
    d_base_out = (bf16*)base;
    total_bytes_out = (size_t)n;
    return true;
}

// launch_rms (helpers.cuh:45-49, normalization.cu:5-25): y = rmsnorm(x) * w, seqlen rows
inline void launch_rms(bf16* x, bf16* w, bf16* y, size_t hidden, size_t seqlen) {
    check_(qie_rmsnorm(x, w, y, (int64_t)seqlen, (int64_t)hidden, config().rms_eps, config().numerics,
                       config().stream), "launch_rms");
}

// launch_rope (helpers.cuh:51-55, RoPE.cu:6-22): rows 0..seqlen-1 at positions 0..seqlen-1,
// in place; hidden_dim is the row stride, nheads heads of head_dim
inline void launch_rope(float* cos_d, float* sin_d, bf16* x, size_t seqlen, size_t head_dim, size_t hidden_dim,
                        size_t nheads) {
    check_(qie_rope(x, (int64_t)seqlen, (int64_t)hidden_dim, (int32_t)nheads, (int32_t)head_dim, nullptr, 0, cos_d,
                    sin_d, config().numerics, config().stream), "launch_rope");
}

// launch_rope_single (helpers.cuh:143-147): one row at position pos
inline void launch_rope_single(float* cos_d, float* sin_d, bf16* x, size_t pos, size_t head_dim, int hidden_dim,
                               int nheads) {
    check_(qie_rope(x, 1, hidden_dim, nheads, (int32_t)head_dim, nullptr, (int32_t)pos, cos_d, sin_d,
                    config().numerics, config().stream), "launch_rope_single");
}

// launch_qknorm (helpers.cuh:140-142, qk_norm.cu:43-79): in place, hidden = row stride
inline void launch_qknorm(bf16* X, bf16* w, int head_dim, int seqlen, int hidden, int nheads) {
    check_(qie_qknorm(X, seqlen, hidden, nheads, head_dim, w, config().qk_eps, config().numerics, config().stream),
           "launch_qknorm");
}

// launch_matmul (helpers.cuh:81-106, matrix_mul.cu:165-288): C[M][K] = A[M][N] . W[K][N]^T
// (W in PyTorch [out, in] layout; the reference names the inner dimension N and the
// output dimension K)
inline void launch_matmul(bf16* A, bf16* W, bf16* Cout, int M, int N, int K) {
    qie_linear_args a;
    std::memset(&a, 0, sizeof(a));
    a.x = A; a.ldx = N;
    a.w[0] = W; a.seg_rows[0] = K;
    a.M = M; a.K = N; a.N = K;
    a.y = Cout; a.ldy = K;
    a.epilogue = QIE_EPI_STORE;
    a.numerics = config().numerics;
    check_(qie_linear(&a, config().stream), "launch_matmul");
}

// proj (helpers.cuh:132-138): resolve the weight from the arena, then launch_matmul
inline void proj(const tensor& t, std::ifstream& f, bf16* w_h, bf16* w_d, size_t w_elems, bf16* x, bf16* y, int m,
                 int n, int k, bf16* g_gpu_weights_buffer) {
    load_weight(t, f, w_h, w_d, w_elems, g_gpu_weights_buffer);
    launch_matmul(x, w_d, y, m, n, k);
}

// launch_act / launch_elem / launch_resadd (helpers.cuh:108-119)
inline void launch_act(bf16* x, size_t n) { check_(qie_silu(x, (int64_t)n, config().stream), "launch_act"); }
inline void launch_elem(bf16* a, bf16* b, bf16* out, int n) {
    check_(qie_mul(a, b, out, n, config().stream), "launch_elem");
}
inline void launch_resadd(bf16* x, bf16* y, size_t n) {
    check_(qie_residual_add(x, y, (int64_t)n, config().stream), "launch_resadd");
}

// copy_last_vocab_vec / copy_first_token (helpers.cuh:149-155)
inline void copy_last_vocab_vec(bf16* seq, bf16* dst, int hidden, int seqlen) {
    check_(qie_memcpy_d2d(dst, seq + (int64_t)(seqlen - 1) * hidden, (int64_t)hidden * 2, config().stream),
           "copy_last_vocab_vec");
}
inline void copy_first_token(bf16* seq, bf16* dst, int hidden) {
    check_(qie_memcpy_d2d(dst, seq, (int64_t)hidden * 2, config().stream), "copy_first_token");
}

// sample_topk_bf16 (helpers.cuh:157-166, logit_decode.cu:149-274): k rounds of arg-max,
// softmax(v / T), one XORWOW draw from curand_init(seed, subsequence = step, 0).  Only
// subsequence 0 is implemented (every call site in the reference passes 0 and moves the
// seed instead, qwen_main.cu:241,388).  Returns the token, or -1 on error.
inline int sample_topk_bf16(bf16* logits_d, int vocab, float temperature, int topk, unsigned long long seed,
                            int step) {
    if (step != 0) {
        std::fprintf(stderr, "sample_topk_bf16: cuRAND subsequence %d not supported (only 0)\n", step);
        config().error = -22;
        return -1;
    }
    const int64_t ws = qie_sample_workspace_bytes(1, vocab);
    char* p = (char*)scratch(2).get(ws + 256);
    if (!p) return -1;
    qie_sampling s;
    s.top_k = topk;
    s.temperature = temperature;
    s.top_p = 1.0f;
    s.seed = seed;
    int32_t* d_tok = (int32_t*)(p + (ws + 255) / 256 * 256);
    int rc = qie_sample(logits_d, 1, vocab, vocab, &s, nullptr, d_tok, p, config().stream);
    check_(rc, "sample_topk_bf16");
    int32_t h = -1;
    if (rc == 0) check_(qie_memcpy_d2h(&h, d_tok, 4), "sample_topk_bf16");
    return h;
}

// allocate_page_buffers (iengine.cu:90-100): the reference allocates one page node of
// elems_per_page = page_size * L * hidden_kv elements; here the slot grows by the
// positions those elements hold (elems / (L * hidden_kv)), taken from the pool.
inline void allocate_page_buffers(page_table* node, size_t elems_per_page, size_t n_layers, size_t hidden_dim_kv) {
    node->tokens += (int)(elems_per_page / (n_layers * hidden_dim_kv));
    check_(qie_batch_reserve(node->batch, node->slot, node->tokens), "allocate_page_buffers");
}

// ModelBuffers (utils.hh:14-88): per-sequence activations and dims.  Weight pointer
// slots are bound by load_weight into the engine arena; RoPE tables are the engine's.
struct ModelBuffers {
    int* d_token_ids = nullptr;
    size_t sequence_len = 0;
    size_t number_of_layers = 0, head_dim = 0, hidden_dim = 0, hidden_dim_kv = 0, num_of_qheads = 0,
           num_of_kvheads = 0, context_size = 0, vocab_size = 0, up_dim = 0;
    bf16* embeddings_h = nullptr;     // (the reference's pinned host copy; unused)
    bf16* embeddings_d = nullptr;     // E [V][H] (engine arena)
    bf16* embeddings_out = nullptr;   // residual stream [rows][H]
    float* cos_values_h = nullptr;
    float* sin_values_h = nullptr;
    float* cos_values_d = nullptr;
    float* sin_values_d = nullptr;
    bf16* k_cache = nullptr;          // driver form: the sequence's slot K / V base once bound
    bf16* v_cache = nullptr;
    bf16 *norm_weights_h = nullptr, *norm_weights_d = nullptr, *rms_out = nullptr;
    bf16 *qk_norm_weights_h = nullptr, *qk_norm_weights_d = nullptr;
    bf16 *q_proj_weights_h = nullptr, *q_proj_weights_d = nullptr, *Q = nullptr;
    size_t q_proj_size = 0;
    bf16 *kv_proj_weights_h = nullptr, *kv_proj_weights_d = nullptr, *K = nullptr, *V = nullptr;
    size_t kv_proj_size = 0;
    bf16* atten_out = nullptr;
    bf16 *o_proj_weights_h = nullptr, *o_proj_weights_d = nullptr, *out_proj = nullptr;
    size_t o_proj_size = 0;
    bf16 *mlp_up_proj_weights_h = nullptr, *mlp_up_proj_weights_d = nullptr, *MLP_UP = nullptr, *MLP_GATE = nullptr,
         *MLP_GATE_OUT = nullptr, *MLP_DOWN = nullptr;
    size_t mlp_up_proj_size = 0;
    bf16 *last_x = nullptr, *prefill_output_d = nullptr, *logits_weights_h = nullptr, *logits_weights_d = nullptr;
    bf16 *O = nullptr, *test_out = nullptr;
    size_t logtis_shape = 0;   // (sic, utils.hh:87)
    size_t rows = 0;           // activation rows allocated (max prompt length)
    // qie: the prompt (driver tier) and the batch the reference-form llm() bound (freed here)
    std::vector<int32_t> h_token_ids;
    qie_batch* owned_batch = nullptr;
};

// initialize_model_buffers (utills.cu:4-129): dims from the engine's spec, activations
// for `sequence_len` rows, the prompt ids on device and embedded into embeddings_out
// (embedding_matrix_func, embedded_matrix.cu:5-17).  Returns false on error.
inline bool initialize_model_buffers(ModelBuffers& buf, const int* h_token_ids, TensorTable&, qie_engine* e,
                                     size_t sequence_len) {
    qie_model_spec s;
    if (qie_engine_spec(e, &s) != 0) return false;
    qie_model_weights w;
    if (qie_engine_weights(e, &w, nullptr) != 0) return false;
    int32_t rope_rows = 0;
    const float *cs = nullptr, *sn = nullptr;
    if (qie_engine_rope_tables(e, &cs, &sn, &rope_rows) != 0) return false;
    buf.sequence_len = sequence_len;
    buf.rows = sequence_len;
    buf.number_of_layers = (size_t)s.n_layers;
    buf.head_dim = (size_t)s.head_dim;
    buf.num_of_qheads = (size_t)s.n_heads;
    buf.num_of_kvheads = (size_t)s.n_kv_heads;
    buf.hidden_dim = (size_t)s.hidden;
    buf.hidden_dim_kv = (size_t)s.n_kv_heads * s.head_dim;
    buf.context_size = (size_t)rope_rows;
    buf.vocab_size = (size_t)s.vocab;
    buf.up_dim = (size_t)s.ffn;
    buf.embeddings_d = (bf16*)w.embed;
    buf.cos_values_d = (float*)cs;
    buf.sin_values_d = (float*)sn;
    const int64_t R = (int64_t)sequence_len, H = s.hidden, QD = (int64_t)s.n_heads * s.head_dim;
    const int64_t KD = (int64_t)buf.hidden_dim_kv, I = s.ffn;
    bool ok = true;
    auto A = [&](bf16** p, int64_t elems) {
        void* q = nullptr;
        if (ok && qie_malloc(&q, elems * 2) == 0) *p = (bf16*)q;
        else ok = false;
    };
    A(&buf.embeddings_out, R * H);
    A(&buf.rms_out, R * H);
    A(&buf.Q, R * QD);
    A(&buf.K, R * KD);
    A(&buf.V, R * KD);
    A(&buf.atten_out, R * QD);
    A(&buf.out_proj, R * H);
    A(&buf.MLP_UP, R * I);
    A(&buf.MLP_GATE, R * I);
    A(&buf.MLP_GATE_OUT, R * I);
    A(&buf.MLP_DOWN, R * H);
    A(&buf.last_x, H);
    A(&buf.prefill_output_d, s.vocab);
    void* ids = nullptr;
    if (ok && qie_malloc(&ids, R * 4) == 0) buf.d_token_ids = (int*)ids;
    else ok = false;
    buf.q_proj_size = (size_t)(QD * H);
    buf.kv_proj_size = (size_t)(KD * H);
    buf.o_proj_size = (size_t)(H * QD);
    buf.mlp_up_proj_size = (size_t)(I * H);
    buf.logtis_shape = (size_t)s.vocab * H;
    if (ok) ok = qie_memcpy_h2d(buf.d_token_ids, h_token_ids, R * 4) == 0;
    if (ok) ok = qie_embedding(buf.embeddings_d, buf.d_token_ids, buf.embeddings_out, R, H, config().stream) == 0;
    if (!ok) std::fprintf(stderr, "initialize_model_buffers: %s\n", qie_last_error());
    return ok;
}

// destroy_model_buffers (utils.hh:105, utills.cu:142-205): frees the activations
// (weights and RoPE tables belong to the engine)
inline void destroy_model_buffers(ModelBuffers& buf) {
    bf16* ps[] = {buf.embeddings_out, buf.rms_out, buf.Q, buf.K, buf.V, buf.atten_out, buf.out_proj, buf.MLP_UP,
                  buf.MLP_GATE, buf.MLP_GATE_OUT, buf.MLP_DOWN, buf.last_x, buf.prefill_output_d};
    for (bf16* p : ps)
        if (p) qie_free(p);
    if (buf.d_token_ids) qie_free(buf.d_token_ids);
    if (buf.owned_batch) qie_batch_destroy(buf.owned_batch);
    buf = ModelBuffers();
}

// ===================================================================== driver tier bodies
inline void fill_dims_(ModelBuffers& b, const qie_model_spec& s, int sequence_len) {
    b.sequence_len = (size_t)sequence_len;
    b.number_of_layers = (size_t)s.n_layers;
    b.head_dim = (size_t)s.head_dim;
    b.hidden_dim = (size_t)s.hidden;
    b.hidden_dim_kv = (size_t)s.n_kv_heads * s.head_dim;
    b.num_of_qheads = (size_t)s.n_heads;
    b.num_of_kvheads = (size_t)s.n_kv_heads;
    b.context_size = (size_t)config().max_ctx;
    b.vocab_size = (size_t)s.vocab;
    b.up_dim = (size_t)s.ffn;
}

inline batch_metadata* new_sequence_(int sequence_id, const int* h_token_ids, int sequence_len) {
    auto* s = static_cast<batch_metadata*>(std::malloc(sizeof(batch_metadata)));
    if (!s) return nullptr;
    std::memset(s, 0, sizeof(*s));
    s->sequence_id = sequence_id;
    s->state = prefill;
    s->sequence_len = sequence_len;
    s->last_token = -1;
    s->buffer = new ModelBuffers();
    fill_dims_(*s->buffer, config().spec, sequence_len);
    s->buffer->h_token_ids.assign(h_token_ids, h_token_ids + sequence_len);
    return s;
}

inline void initialize_model_buffers(ModelBuffers& buf, int* h_token_ids, TensorTable& tensors,
                                     std::ifstream& weights, size_t sequence_len);

// create_new_sequence, reference form (iengine.cu:25-47): the sequence's buffers (dims from
// config().spec, the prompt); its KV slot is bound by its first llm() call.
inline batch_metadata* create_new_sequence(int sequence_id, int* h_token_ids, int sequence_len, TensorTable tensors,
                                           std::ifstream& weights) {
    batch_metadata* s = new_sequence_(sequence_id, h_token_ids, sequence_len);
    // as iengine.cu:25-47: the sequence's model buffers, once weights have been loaded
    if (s && loaded_arena_()) initialize_model_buffers(*s->buffer, h_token_ids, tensors, weights, (size_t)sequence_len);
    return s;
}

inline void destroy_sequence(batch_metadata* s) {
    if (!s) return;
    if (s->buffer) {
        destroy_model_buffers(*s->buffer);
        delete s->buffer;
    }
    std::free(s);
}

inline int llm_step_(batch_metadata* seq, const qie_sampling* sampling) {
    auto bad = [](int rc, const char* who) {
        check_(rc ? rc : -22, who);
        return 0;
    };
    config().error = 0;   // per call: an earlier failure must not mark this call failed
    if (!seq || !seq->batch || !seq->buffer) return bad(-22, "llm: sequence has no batch slot");
    int32_t tok = -1;
    if (seq->state == prefill) {
        qie_sampling s = sampling ? *sampling : reference_sampling(prefill);
        const auto& ids = seq->buffer->h_token_ids;
        const int rc = qie_prefill(seq->batch, seq->slot, ids.data(), (int32_t)ids.size(), &s, &tok);
        if (rc) return bad(rc, "llm(prefill)");
        seq->last_token = tok;
        return tok;
    }
    // qie_decode_step advances every slot of the batch; the reference's llm steps only
    // `seq`, so a B > 1 batch would silently skip tokens of its other sequences.
    int32_t nb = 0;
    if (qie_batch_dims(seq->batch, &nb, nullptr) != 0 || nb != 1) {
        std::fprintf(stderr, "llm(decode): needs a batch of one slot (got %d); step B > 1 batches with "
                             "qie_decode_step, which returns every slot's token\n", nb);
        return bad(-22, "llm(decode)");
    }
    // the decode input is seq->generated_token (qwen_main.cu:259-261); the graph already
    // holds the engine's own last output, anything else is written in first
    if (seq->generated_token != seq->last_token) {
        const int rc = qie_batch_set_position(seq->batch, seq->slot, seq->sequence_len, seq->generated_token);
        if (rc) return bad(rc, "llm(decode)");
    }
    qie_sampling s = sampling ? *sampling : reference_sampling(decode);
    int32_t ids[8] = {0};
    const int rc = qie_decode_step(seq->batch, &s, ids);
    if (rc) return bad(rc, "llm(decode)");
    seq->sequence_len += 1;
    seq->buffer->sequence_len = (size_t)seq->sequence_len;
    seq->last_token = ids[seq->slot];
    return ids[seq->slot];
}

// The engine behind the reference-form llm(): bound to the caller's weight arena
// (g_gpu_weights_buffer) through the index, exactly as assign_weight_pointer resolves
// every weight (helpers.cuh:19-30): base + data_offsets[0]; nothing is copied.
struct Driver {
    qie_engine* engine = nullptr;
    const void* base = nullptr;
    std::vector<qie_layer_weights> layers;
    ~Driver() {
        if (engine) qie_engine_destroy(engine);
    }
};
inline Driver& driver() {
    static Driver d;
    return d;
}
// destroy the bound engine (before the caller frees the weight arena).  The arena the engine
// was bound to is forgotten too: a sequence created after the caller freed it must not bind
// a new engine to freed device memory (create_new_sequence then skips the binding and the
// next llm() binds to the arena it is given).
inline void release_engine() {
    Driver& d = driver();
    if (d.engine) qie_engine_destroy(d.engine);
    if (d.base && loaded_arena_() == d.base) loaded_arena_() = nullptr;
    d.engine = nullptr;
    d.base = nullptr;
}
// frees an arena load_all_weights_to_gpu_chunked returned (the reference's cudaFree of
// g_gpu_weights_buffer, iengine.cu:464-475), releasing the engine bound to it first
inline void free_weight_arena(bf16* arena) {
    if (!arena) return;
    if (driver().base == arena) release_engine();
    if (loaded_arena_() == arena) loaded_arena_() = nullptr;
    qie_free(arena);
}

inline int bind_engine_(const TensorTable& tensors, bf16* base) {
    Driver& d = driver();
    if (d.engine && d.base == base) return 0;
    release_engine();
    const qie_model_spec& s = config().spec;
    auto ptr = [&](const char* sn, int layer, bool required, const void** out) -> bool {
        *out = nullptr;
        auto it = tensors.find(sn);
        const size_t li = layer < 0 ? 0 : (size_t)layer;
        if (it == tensors.end() || it->second.size() <= li || it->second[li].data_offsets.size() < 2 ||
            it->second[li].short_name.empty())
            return !required;
        *out = reinterpret_cast<const char*>(base) + it->second[li].data_offsets[0];
        return true;
    };
    d.layers.assign((size_t)s.n_layers, qie_layer_weights{});
    bool ok = true;
    for (int l = 0; l < s.n_layers && ok; l++) {
        qie_layer_weights& L = d.layers[(size_t)l];
        ok = ptr("input_layernorm.weight", l, true, &L.attn_norm) && ptr("self_attn.q_proj.weight", l, true, &L.wq) &&
             ptr("self_attn.k_proj.weight", l, true, &L.wk) && ptr("self_attn.v_proj.weight", l, true, &L.wv) &&
             ptr("self_attn.q_proj.bias", l, s.qkv_bias != 0, &L.bq) &&
             ptr("self_attn.k_proj.bias", l, s.qkv_bias != 0, &L.bk) &&
             ptr("self_attn.v_proj.bias", l, s.qkv_bias != 0, &L.bv) &&
             ptr("self_attn.q_norm.weight", l, s.qk_norm != 0, &L.q_norm) &&
             ptr("self_attn.k_norm.weight", l, s.qk_norm != 0, &L.k_norm) &&
             ptr("self_attn.o_proj.weight", l, true, &L.wo) &&
             ptr("post_attention_layernorm.weight", l, true, &L.ffn_norm) &&
             ptr("mlp.gate_proj.weight", l, true, &L.w_gate) && ptr("mlp.up_proj.weight", l, true, &L.w_up) &&
             ptr("mlp.down_proj.weight", l, true, &L.w_down);
    }
    qie_model_weights w;
    std::memset(&w, 0, sizeof(w));
    ok = ok && ptr("embed_tokens.weight", -1, true, &w.embed) && ptr("norm.weight", -1, true, &w.final_norm);
    if (ok) {
        if (s.tie_embeddings) w.lm_head = w.embed;
        else ok = ptr("logits", -1, true, &w.lm_head);
    }
    if (!ok) {
        std::fprintf(stderr, "llm: the tensor table lacks a tensor config().spec needs\n");
        config().error = -22;
        return -22;
    }
    w.n_layers = s.n_layers;
    w.layers = d.layers.data();
    qie_engine_opts o;
    std::memset(&o, 0, sizeof(o));
    o.device = config().device;
    o.max_ctx = config().max_ctx;
    o.use_graph = 1;
    int rc = qie_engine_create(&s, &o, &d.engine);
    if (!rc) rc = qie_engine_set_weights(d.engine, &w);
    if (rc) {
        check_(rc, "llm: engine");
        release_engine();
        return rc;
    }
    d.base = base;
    return 0;
}

// initialize_model_buffers, reference form (utils.hh:90-92, utills.cu:4-129): the sequence's
// buffers over the engine bound to the arena that load_all_weights_to_gpu_chunked filled last
// (the reference re-reads the embedding and norm tensors from `weights`; here they are in that
// arena already).  Returns void as the reference does: failures set config().error.
inline void initialize_model_buffers(ModelBuffers& buf, int* h_token_ids, TensorTable& tensors,
                                     std::ifstream& weights, size_t sequence_len) {
    (void)weights;
    bf16* base = loaded_arena_();
    if (!base) {
        std::fprintf(stderr, "initialize_model_buffers: no weights loaded (load_all_weights_to_gpu_chunked first)\n");
        config().error = -22;
        return;
    }
    if (bind_engine_(tensors, base) != 0) return;   // reported by bind_engine_
    if (!initialize_model_buffers(buf, h_token_ids, tensors, driver().engine, sequence_len)) config().error = -22;
}

// llm, reference form (iengine.cuh:51, qwen_main.cu:64-417): prefill when
// seq->state == prefill, else ONE decode step fed seq->generated_token; the caller
// advances step / generated_token / state (iengine.cu:419-421).  The first call binds the
// engine to g_gpu_weights_buffer through `tensors` and the sequence to its own KV slot.
// Sampling follows the reference's schedule unless config().greedy.  Returns the token,
// or 0 on error (the reference's convention).
inline int llm(batch_metadata* seq, TensorTable tensors, std::ifstream& weights, page_table* kv_cache_seq1,
               int page_size, bf16* g_gpu_weights_buffer) {
    (void)weights;
    config().error = 0;   // per call (0 is also a token id: callers read config().error)
    if (!seq || !seq->buffer || !kv_cache_seq1 || page_size <= 0 || !g_gpu_weights_buffer) {
        check_(-22, "llm: bad arguments");
        return 0;
    }
    if (bind_engine_(tensors, g_gpu_weights_buffer) != 0) return 0;
    if (!seq->batch) {
        qie_batch* b = nullptr;
        const int rc = qie_batch_create(driver().engine, 1, config().max_ctx, &b);
        if (rc) {
            check_(rc, "llm: KV slot");
            return 0;
        }
        seq->batch = b;
        seq->slot = 0;
        seq->buffer->owned_batch = b;
        qie_kv_cache c;
        if (qie_batch_kv_cache(b, 0, &c) == 0) {
            seq->k_ptr = seq->buffer->k_cache = (bf16*)c.k;
            seq->v_ptr = seq->buffer->v_cache = (bf16*)c.v;
        }
    }
    qie_sampling g;
    g.top_k = 1;
    g.temperature = 1.f;
    g.top_p = 1.f;
    g.seed = 1234;
    return llm_step_(seq, config().greedy ? &g : nullptr);
}

// embedding_matrix_func launch (embedded_matrix.cu:5-17; decode: qwen_main.cu:259-268):
// rows 0..n-1 of `out` = E[ids]; ids on the host
inline void embed_tokens(ModelBuffers& buf, const int* h_ids, size_t n) {
    check_(qie_memcpy_h2d(buf.d_token_ids, h_ids, (int64_t)n * 4), "embed_tokens");
    check_(qie_embedding(buf.embeddings_d, buf.d_token_ids, buf.embeddings_out, (int64_t)n, (int64_t)buf.hidden_dim,
                         config().stream), "embed_tokens");
}

// kv_copy_layer_to_cache_prefill (include_cuda.cu:165-228): K/V rows 0..sequence_len-1
// of layer i into positions 0..sequence_len-1 of the page table's slot
inline void kv_copy_layer_to_cache_prefill(ModelBuffers* buffer, int i, page_table* kv, int /*page_size*/) {
    const int n = (int)buffer->sequence_len;
    if (kv->tokens < n) {
        kv->tokens = n;
        check_(qie_batch_reserve(kv->batch, kv->slot, n), "kv_copy_layer_to_cache_prefill");
    }
    qie_kv_cache c;
    check_(qie_batch_kv_cache(kv->batch, kv->slot, &c), "kv_copy_layer_to_cache_prefill");
    check_(qie_kv_write(buffer->K, buffer->V, n, (int64_t)buffer->hidden_dim_kv, 0, &c, 0, i, config().stream),
           "kv_copy_layer_to_cache_prefill");
}

// kv_copy_layer_to_cache_decode (include_cuda.cu:233-279): row 0 of K/V of layer i into
// position sequence_len - 1 (a missing page is taken from the pool, as the reference
// allocates one)
inline void kv_copy_layer_to_cache_decode(ModelBuffers* buffer, int i, page_table* kv, int /*page_size*/) {
    const int pos = (int)buffer->sequence_len - 1;
    if (kv->tokens < pos + 1) {
        kv->tokens = pos + 1;
        check_(qie_batch_reserve(kv->batch, kv->slot, pos + 1), "kv_copy_layer_to_cache_decode");
    }
    qie_kv_cache c;
    check_(qie_batch_kv_cache(kv->batch, kv->slot, &c), "kv_copy_layer_to_cache_decode");
    check_(qie_kv_write(buffer->K, buffer->V, 1, (int64_t)buffer->hidden_dim_kv, pos, &c, 0, i, config().stream),
           "kv_copy_layer_to_cache_decode");
}

// launch_attn (helpers.cuh:121-130, self_attension.cu:10-149): mq query rows of Q
// ([mq][hidden]) over the first mkv cached positions of the slot's layer `layer_id`.
// causal: row r sees positions <= q_abs_base + r; otherwise every row sees all mkv.
inline void launch_attn(bf16* Q, bf16* out, size_t mq, size_t mkv, size_t head_dim, size_t hidden, size_t hidden_kv,
                        int causal, size_t q_abs_base, int layer_id, page_table* kv, int /*page_size*/) {
    qie_kv_cache c;
    if (qie_batch_kv_cache(kv->batch, kv->slot, &c) != 0) return check_(-22, "launch_attn");
    std::vector<int32_t> pos(mq);
    for (size_t r = 0; r < mq; r++) pos[r] = causal ? (int32_t)(q_abs_base + r) : (int32_t)mkv - 1;
    int32_t* dpos = (int32_t*)scratch(0).get((int64_t)mq * 4);
    const int32_t nq = (int32_t)(hidden / head_dim);
    void* ws = scratch(1).get(qie_attention_workspace_bytes((int64_t)mq, nq, (int32_t)head_dim, c.max_ctx));
    // every call site in the reference is causal prefill or mq = 1 decode (qwen_main.cu:123,300)
    if (!dpos || !ws || hidden_kv != (size_t)c.n_kv_heads * c.head_dim || (!causal && mq != 1))
        return check_(-22, "launch_attn");
    check_(qie_memcpy_h2d(dpos, pos.data(), (int64_t)mq * 4), "launch_attn");
    check_(qie_attention(Q, (int64_t)mq, dpos, (int32_t)mq, &c, layer_id, nq, out, ws, config().stream),
           "launch_attn");
}

}  // namespace qie_compat
