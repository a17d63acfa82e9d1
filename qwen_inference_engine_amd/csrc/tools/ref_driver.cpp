// ref_driver.cpp — a host driver written against the reference's own driver-tier
// signatures (layers/include/iengine.cuh:51-55, layers/src/iengine.cu:25,117,
// tensor_parser.hh:216-219), following main()'s call sequence (iengine.cu:226-456):
//
//   build_indexed_tensors() -> ifstream weights.bin -> parsed_tensors() -> malloc staging
//   -> load_all_weights_to_gpu_chunked(all, ifs, h_host, chunk, d_base, total)
//   -> create_new_sequence(0, ids, len, tensors, ifs) -> create_page_list(pages_required)
//   -> allocate_page_buffers(node, page_size * L * hidden_kv) for every node
//   -> loop { tok = llm(seq, tensors, ifs, kv, page_size, d_base); step++;
//             generated_token = tok; state = decode }
//   -> free_page_list, destroy_model_buffers, free(seq), free staging, free the arena.
//
// Only what the reference hard-codes is taken from the command line instead: the model
// (utills.cu:8-16), the weights / index paths (iengine.cu:232, tensor_parser.cpp:34), the
// prompt ids (iengine.cu:325), and a step count in place of the getchar() loop.
//
//   ref_driver --weights W.bin --meta meta.txt --spec L,H,nq,nkv,hd,I,V,tie,bias,qkn[,eps,theta]
//              [--prompt 151643,785,...] [--gen N] [--greedy] [--max-ctx N]
// Prints one line: "tokens: t0 t1 ..." (the prefill token first).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/qie/compat.hpp"

using namespace qie_compat;

static std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    while (a <= s.size()) {
        size_t b = s.find(',', a);
        if (b == std::string::npos) b = s.size();
        if (b > a) out.push_back(s.substr(a, b - a));
        a = b + 1;
    }
    return out;
}

int main(int argc, char** argv) {
    std::string wpath, spec;
    std::vector<int> ids = {151643, 785, 4767, 315, 279, 3639, 4180, 374};   // iengine.cu:325
    int gen = 8;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : std::string(); };
        if (a == "--weights") wpath = next();
        else if (a == "--meta") config().meta_path = next();
        else if (a == "--spec") spec = next();
        else if (a == "--gen") gen = std::atoi(next().c_str());
        else if (a == "--greedy") config().greedy = 1;
        else if (a == "--max-ctx") config().max_ctx = std::atoi(next().c_str());
        else if (a == "--prompt") {
            ids.clear();
            for (const auto& t : split(next())) ids.push_back(std::atoi(t.c_str()));
        } else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    if (!spec.empty()) {
        const auto f = split(spec);
        if (f.size() < 10) {
            std::fprintf(stderr, "--spec needs L,H,nq,nkv,hd,I,V,tie,bias,qkn[,eps,theta]\n");
            return 2;
        }
        qie_model_spec& s = config().spec;
        s.n_layers = std::atoi(f[0].c_str()); s.hidden = std::atoi(f[1].c_str());
        s.n_heads = std::atoi(f[2].c_str()); s.n_kv_heads = std::atoi(f[3].c_str());
        s.head_dim = std::atoi(f[4].c_str()); s.ffn = std::atoi(f[5].c_str()); s.vocab = std::atoi(f[6].c_str());
        s.tie_embeddings = std::atoi(f[7].c_str()); s.qkv_bias = std::atoi(f[8].c_str());
        s.qk_norm = std::atoi(f[9].c_str());
        if (f.size() > 10) s.rms_eps = (float)std::atof(f[10].c_str());
        if (f.size() > 11) s.rope_theta = (float)std::atof(f[11].c_str());
    }

    // ---- iengine.cu:228-283
    auto tensors = build_indexed_tensors();
    std::ifstream weights(wpath, std::ios::binary);
    if (!weights) {
        std::printf("Failed to open weights.bin\n");
        return 1;
    }
    auto tensors_nomap = parsed_tensors();
    size_t chunk_bytes = 64ull << 20;
    void* h_host = std::malloc(chunk_bytes);
    if (!h_host) return 1;
    bf16* g_gpu_weights_buffer = nullptr;
    size_t total_bytes = 0;
    bool ok = load_all_weights_to_gpu_chunked(tensors_nomap, weights, h_host, chunk_bytes, g_gpu_weights_buffer,
                                              total_bytes);
    if (!ok) return 1;

    // ---- iengine.cu:325-360
    int seq_len_1 = (int)ids.size();
    batch_metadata* new_seq_1 = create_new_sequence(0, ids.data(), seq_len_1, tensors, weights);
    int page_size = 4;
    int pages_required = ((seq_len_1 + page_size - 1) / page_size) + 1;
    page_table* kv_cache_seq1 = create_page_list(pages_required);
    int elements_per_page = page_size * new_seq_1->buffer->number_of_layers * (size_t)new_seq_1->buffer->hidden_dim_kv;
    for (page_table* p = kv_cache_seq1; p; p = p->ptr_to_next_page) allocate_page_buffers(p, elements_per_page);
    new_seq_1->buffer->k_cache = kv_cache_seq1->k_page_ptr;
    new_seq_1->buffer->v_cache = kv_cache_seq1->v_page_ptr;

    // ---- iengine.cu:384-421 (gen steps instead of the getchar() loop)
    std::vector<int> out;
    for (int i = 0; i < gen; i++) {
        int out_token_1 = llm(new_seq_1, tensors, weights, kv_cache_seq1, page_size, g_gpu_weights_buffer);
        if (config().error) {
            std::fprintf(stderr, "llm failed: %s\n", qie_last_error());
            return 1;
        }
        out.push_back(out_token_1);
        new_seq_1->step = new_seq_1->step + 1;
        new_seq_1->generated_token = out_token_1;
        new_seq_1->state = decode;
    }
    std::printf("tokens:");
    for (int t : out) std::printf(" %d", t);
    std::printf("\n");

    // ---- iengine.cu:460-475
    if (weights.is_open()) weights.close();
    free_page_list(kv_cache_seq1);
    destroy_model_buffers(*new_seq_1->buffer);
    delete new_seq_1->buffer;
    free(new_seq_1);
    std::free(h_host);
    free_weight_arena(g_gpu_weights_buffer);
    return 0;
}
