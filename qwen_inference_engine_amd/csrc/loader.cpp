// loader.cpp — reference-compatible tensor index for the flat weights.bin.
//
// Semantics of parsed_tensors / build_indexed_tensors
// (layers/src/tensor_parser.cpp:31-165):
//   * safetensors headers are parsed into an ordered map, so each shard's keys
//     are visited in sorted (byte-lexicographic) order;
//   * keys starting with "model." are kept; "model.layers.N.<rest>" gives
//     layer_index N and short_name <rest>, other "model.<rest>" give
//     layer_index -1 and short_name <rest>;
//   * keys starting with "lm_" are kept with short_name "logits";
//   * each kept tensor's data is re-based into ONE contiguous weights.bin:
//     offsets = [global, global + (end - begin)], global advancing in
//     (shard order, sorted key order).
// The on-disk index is the reference's meta_data.txt text format
// (operator<< at tensor_parser.cpp:19-28).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/qie/qie_engine.h"
#include "qie_common.hpp"
#include "qie_index.hpp"


namespace qie {

// Reference key classification (tensor_parser.cpp:69-116).  Returns false if
// the key is skipped.
static bool classify(const std::string& key, qie_index_entry& e) {
    e.name = key;
    if (key.rfind("model.", 0) == 0) {
        size_t lp = key.find("layers.");
        if (lp != std::string::npos) {
            size_t dot = key.find('.', lp + 7);
            e.layer = std::stoi(key.substr(lp + 7, dot - (lp + 7)));
            e.short_name = key.substr(dot + 1);
        } else {
            e.layer = -1;
            e.short_name = key.substr(6);
        }
        return true;
    }
    if (key.rfind("lm_", 0) == 0) {
        e.layer = -1;
        e.short_name = "logits";
        return true;
    }
    return false;
}

static void hf_names(const qie_model_spec& s, std::vector<std::pair<std::string, std::vector<int64_t>>>& out) {
    const int64_t H = s.hidden, hd = s.head_dim, QD = (int64_t)s.n_heads * hd, KD = (int64_t)s.n_kv_heads * hd;
    const int64_t I = s.ffn, V = s.vocab;
    out.push_back({"model.embed_tokens.weight", {V, H}});
    out.push_back({"model.norm.weight", {H}});
    if (!s.tie_embeddings) out.push_back({"lm_head.weight", {V, H}});
    for (int l = 0; l < s.n_layers; l++) {
        std::string p = "model.layers." + std::to_string(l) + ".";
        out.push_back({p + "input_layernorm.weight", {H}});
        out.push_back({p + "post_attention_layernorm.weight", {H}});
        out.push_back({p + "self_attn.q_proj.weight", {QD, H}});
        out.push_back({p + "self_attn.k_proj.weight", {KD, H}});
        out.push_back({p + "self_attn.v_proj.weight", {KD, H}});
        out.push_back({p + "self_attn.o_proj.weight", {H, QD}});
        if (s.qkv_bias) {
            out.push_back({p + "self_attn.q_proj.bias", {QD}});
            out.push_back({p + "self_attn.k_proj.bias", {KD}});
            out.push_back({p + "self_attn.v_proj.bias", {KD}});
        }
        if (s.qk_norm) {
            out.push_back({p + "self_attn.q_norm.weight", {hd}});
            out.push_back({p + "self_attn.k_norm.weight", {hd}});
        }
        out.push_back({p + "mlp.gate_proj.weight", {I, H}});
        out.push_back({p + "mlp.up_proj.weight", {I, H}});
        out.push_back({p + "mlp.down_proj.weight", {H, I}});
    }
}

const qie_index_entry* index_find(const qie_index* idx, const char* short_name, int layer) {
    for (const auto& e : idx->t)
        if (e.layer == layer && e.short_name == short_name) return &e;
    return nullptr;
}

}  // namespace qie

using namespace qie;

extern "C" {

int qie_index_synthetic(const qie_model_spec* spec, qie_index** out) {
    QIE_REQUIRE(spec && out, "qie_index_synthetic: bad arguments");
    std::vector<std::pair<std::string, std::vector<int64_t>>> names;
    hf_names(*spec, names);
    // One virtual shard; header keys visited in sorted order like nlohmann::json's std::map.
    std::sort(names.begin(), names.end(),
              [](const auto& a, const auto& b) { return a.first < b.first; });
    qie_index* idx = new qie_index();
    int64_t global = 0;
    for (auto& nm : names) {
        qie_index_entry e;
        if (!classify(nm.first, e)) continue;
        int64_t numel = 1;
        for (auto d : nm.second) numel *= d;
        e.shape = nm.second;
        e.off0 = global;
        e.off1 = global + numel * 2;
        global = e.off1;
        idx->t.push_back(std::move(e));
    }
    *out = idx;
    return 0;
}

int qie_index_load_meta(const char* path, qie_index** out) {
    QIE_REQUIRE(path && out, "qie_index_load_meta: bad arguments");
    std::ifstream f(path);
    QIE_REQUIRE(f.good(), "qie_index_load_meta: cannot open %s", path);
    qie_index* idx = new qie_index();
    std::string line;
    qie_index_entry cur;
    bool open = false;
    auto trim = [](std::string s) {
        size_t a = s.find_first_not_of(" \t\r");
        size_t b = s.find_last_not_of(" \t\r");
        return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
    };
    auto nums = [](const std::string& s) {
        std::vector<int64_t> v;
        std::string t;
        for (char c : s) {
            if ((c >= '0' && c <= '9') || c == '-') t.push_back(c);
            else if (!t.empty()) { v.push_back(std::stoll(t)); t.clear(); }
        }
        if (!t.empty()) v.push_back(std::stoll(t));
        return v;
    };
    while (std::getline(f, line)) {
        std::string s = trim(line);
        if (s.rfind("Tensor:", 0) == 0) {
            if (open) idx->t.push_back(cur);
            cur = qie_index_entry();
            cur.name = trim(s.substr(7));
            open = true;
        } else if (s.rfind("layer:", 0) == 0) {
            cur.layer = (int32_t)std::stol(trim(s.substr(6)));
        } else if (s.rfind("short_name:", 0) == 0) {
            cur.short_name = trim(s.substr(11));
        } else if (s.rfind("shape:", 0) == 0) {
            cur.shape = nums(s.substr(6));
        } else if (s.rfind("offsets:", 0) == 0) {
            auto v = nums(s.substr(8));
            if (v.size() == 2) { cur.off0 = v[0]; cur.off1 = v[1]; }
        }
    }
    if (open) idx->t.push_back(cur);
    if (idx->t.empty()) {
        delete idx;
        return fail(-22, "qie_index_load_meta: no tensors in %s", path);
    }
    *out = idx;
    return 0;
}

int qie_index_count(const qie_index* idx) { return idx ? (int)idx->t.size() : 0; }

int qie_index_get(const qie_index* idx, int i, const char** name, const char** short_name,
                  int32_t* layer, int64_t* off0, int64_t* off1, int32_t* ndim, int64_t* shape4) {
    QIE_REQUIRE(idx && i >= 0 && i < (int)idx->t.size(), "qie_index_get: bad index");
    const auto& e = idx->t[i];
    if (name) *name = e.name.c_str();
    if (short_name) *short_name = e.short_name.c_str();
    if (layer) *layer = e.layer;
    if (off0) *off0 = e.off0;
    if (off1) *off1 = e.off1;
    if (ndim) *ndim = (int32_t)e.shape.size();
    if (shape4)
        for (size_t k = 0; k < 4; k++) shape4[k] = k < e.shape.size() ? e.shape[k] : 0;
    return 0;
}

int64_t qie_index_total_bytes(const qie_index* idx) {
    int64_t m = 0;
    if (!idx) return 0;
    for (const auto& e : idx->t) m = std::max(m, e.off1);
    return m;
}

int qie_index_write_meta(const qie_index* idx, const char* path) {
    QIE_REQUIRE(idx && path, "qie_index_write_meta: bad arguments");
    std::ofstream f(path);
    QIE_REQUIRE(f.good(), "qie_index_write_meta: cannot open %s", path);
    for (const auto& e : idx->t) {
        f << "Tensor: " << e.name << "\n";
        f << "  layer: " << e.layer << "\n";
        f << "  short_name: " << e.short_name << "\n";
        f << "  shape: [ ";
        for (auto s : e.shape) f << s << " ";
        f << "]\n";
        f << "  offsets: [ " << e.off0 << ", " << e.off1 << " ]\n";
        f << "\n";
    }
    return 0;
}

void qie_index_destroy(qie_index* idx) { delete idx; }

}  // extern "C"
