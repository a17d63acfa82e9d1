// compat.hpp — the reference engine's host entry points, by name, over the qie C ABI.
//
// A host driver written against Rafae1130/qwen_inference_engine's C++ API keeps its
// shape: parsed_tensors / build_indexed_tensors (layers/src/tensor_parser.cpp:31-165),
// load_all_weights_to_gpu_chunked (layers/src/iengine.cu:117-223), create_new_sequence
// (iengine.cu:25-47), llm (layers/src/qwen_main.cu:64-417) with batch_metadata.state
// selecting prefill or ONE decode step, and the caller advancing step /
// generated_token / state exactly like iengine.cu:419-421.
//
// Differences (deliberate):
//   * CUDA types are gone: the weight arena, KV cache and streams are owned by a
//     qie_engine / qie_batch; no std::ifstream or __nv_bfloat16* crosses the API.
//   * parsed_tensors reads the meta_data.txt index (the reference re-parses the
//     safetensors shards at hard-coded /mnt/data paths, tensor_parser.cpp:37-46).
//   * llm() returns -1 (not 0) on error, with qie_last_error() holding the text.
//   * the model is a qie_model_spec, not the Qwen3-14B literals of utills.cu:8-16.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "qie_engine.h"

namespace qie_compat {

struct tensor {                       // tensor_parser.hh:204-210
    std::string tensor_name;
    std::vector<size_t> shape;
    std::vector<size_t> data_offsets;
    int layer_index = -1;
    std::string short_name;
};
using TensorTable = std::unordered_map<std::string, std::vector<tensor>>;

typedef enum { prefill, decode } State;   // iengine.cuh:23

struct batch_metadata {               // iengine.cuh:27-37 (buffer -> qie_batch slot)
    int sequence_id = 0;
    State state = prefill;
    int sequence_len = 0;
    int generated_token = 0;
    int step = 0;
    qie_batch* batch = nullptr;
    int slot = 0;
    std::vector<int32_t> prompt;
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

// Loads weights.bin into the engine's single device arena in chunk_bytes pieces.
inline bool load_all_weights_to_gpu_chunked(qie_engine* e, const char* weights_bin, const char* meta_data_txt,
                                            size_t chunk_bytes) {
    return qie_engine_load_weights_bin(e, weights_bin, meta_data_txt, (int64_t)chunk_bytes) == 0;
}

inline batch_metadata* create_new_sequence(int sequence_id, const int* h_token_ids, int sequence_len,
                                           qie_batch* batch, int slot) {
    auto* s = new batch_metadata();
    s->sequence_id = sequence_id;
    s->state = prefill;
    s->sequence_len = sequence_len;
    s->batch = batch;
    s->slot = slot;
    s->prompt.assign(h_token_ids, h_token_ids + sequence_len);
    return s;
}

// One call = prefill (state == prefill) or ONE decode step (state == decode); returns
// the sampled token id.  Greedy callers pass a qie_sampling with top_k = 1.
inline int llm(batch_metadata* seq, const qie_sampling* sampling = nullptr) {
    int32_t tok = -1;
    if (seq->state == prefill) {
        qie_sampling s = sampling ? *sampling : reference_sampling(prefill);
        if (qie_prefill(seq->batch, seq->slot, seq->prompt.data(), (int32_t)seq->prompt.size(), &s, &tok) != 0) {
            std::fprintf(stderr, "llm(prefill): %s\n", qie_last_error());
            return -1;
        }
        return tok;
    }
    qie_sampling s = sampling ? *sampling : reference_sampling(decode);
    std::vector<int32_t> ids(64);
    if (qie_decode_step(seq->batch, &s, ids.data()) != 0) {
        std::fprintf(stderr, "llm(decode): %s\n", qie_last_error());
        return -1;
    }
    seq->sequence_len += 1;
    return ids[seq->slot];
}

inline void destroy_sequence(batch_metadata* s) { delete s; }

// Page list (iengine.cuh:39-49, iengine.cu:73-109).  The reference gives each sequence a
// linked list of 4-token pages in managed memory (create_page_list, then
// allocate_page_buffers per node as the sequence grows, free_page_list at the end).  In
// qie every slot of a paged batch (qie_batch_create_paged) draws pages on demand from
// one pool behind a device block table, so a page_table here is only the slot's handle:
// create_page_list reserves nothing up front, free_page_list returns the slot's pages.
struct page_table {
    qie_batch* batch = nullptr;
    int slot = 0;
};

inline page_table* create_page_list(qie_batch* paged_batch, int slot) {
    auto* p = new page_table();
    p->batch = paged_batch;
    p->slot = slot;
    return p;
}

inline void free_page_list(page_table* head) {
    if (!head) return;
    if (qie_batch_release(head->batch, head->slot) != 0) std::fprintf(stderr, "free_page_list: %s\n", qie_last_error());
    delete head;
}

}  // namespace qie_compat
