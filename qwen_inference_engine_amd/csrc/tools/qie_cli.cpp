// qie_cli — native driver replacing the reference's `layers/engine` executable
// (main: layers/src/iengine.cu:226-481), written against include/qie/compat.hpp so
// it exercises the same entry points a reference-style driver uses.
//
//   qie_cli [--model Qwen2-7B|Qwen2-0.5B|Qwen2-72B|Qwen3-14B] [--numerics ref|hf]
//           [--weights weights.bin --meta meta_data.txt | --synthetic SEED]
//           [--prompt 151643,785,... | --prompt-file ids.txt] [--gen N] [--greedy] [--device D]
//           [--no-graph] [--stream] [--page-tokens T]
//
// --prompt-file: token ids separated by commas / whitespace (the reference hard-codes them,
// iengine.cu:325, after tokenising with temp.py:4); --stream prints each id as it is
// generated (the reference prints per step, qwen_main.cu:392-398); --page-tokens runs on a
// paged KV cache (qie_batch_create_paged).
//
// Defaults follow the reference: Qwen3-14B dims, prompt ids
// {151643,785,4767,315,279,3639,4180,374} (iengine.cu:325), reference sampling
// schedule (k=50; T=1.0 prefill, 0.7 decode; seed 1234+step), stop at EOS 151645
// (qwen_main.cu:257) or after --gen tokens.  Unlike the reference there is no
// getchar() between steps and the loop ends.
#include <chrono>
#include <cstdio>
#include <fstream>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/qie/compat.hpp"

using namespace qie_compat;

static qie_model_spec preset(const std::string& name, bool hf) {
    qie_model_spec s;
    std::memset(&s, 0, sizeof(s));
    auto set = [&](int L, int H, int nq, int nkv, int hd, int I, int V, int tie, int bias, int qkn, float eps) {
        s.n_layers = L; s.hidden = H; s.n_heads = nq; s.n_kv_heads = nkv; s.head_dim = hd; s.ffn = I;
        s.vocab = V; s.tie_embeddings = tie; s.qkv_bias = bias; s.qk_norm = qkn;
        s.rms_eps = hf ? eps : 1e-4f;      // normalization.cu:9
        s.rope_theta = 1e6f;               // include.cpp:7
        s.numerics = hf ? QIE_NUMERICS_HF : QIE_NUMERICS_REF;
    };
    if (name == "Qwen2-0.5B") set(24, 896, 14, 2, 64, 4864, 151936, 1, 1, 0, 1e-6f);
    else if (name == "Qwen2-7B") set(28, 3584, 28, 4, 128, 18944, 152064, 0, 1, 0, 1e-6f);
    else if (name == "Qwen2-72B") set(80, 8192, 64, 8, 128, 29568, 152064, 0, 1, 0, 1e-5f);
    else set(40, 5120, 40, 8, 128, 17408, 151936, 0, 0, 1, 1e-6f);   // Qwen3-14B (reference)
    return s;
}

int main(int argc, char** argv) {
    std::string model = "Qwen3-14B", weights, meta, numerics = "ref";
    std::vector<int> prompt = {151643, 785, 4767, 315, 279, 3639, 4180, 374};
    long seed = -1;
    int gen = 32, device = 0, greedy = 0, graph = 1, stream = 0, page_tokens = 0;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--model") model = next();
        else if (a == "--numerics") numerics = next();
        else if (a == "--weights") weights = next();
        else if (a == "--meta") meta = next();
        else if (a == "--synthetic") seed = std::atol(next().c_str());
        else if (a == "--gen") gen = std::atoi(next().c_str());
        else if (a == "--device") device = std::atoi(next().c_str());
        else if (a == "--greedy") greedy = 1;
        else if (a == "--no-graph") graph = 0;
        else if (a == "--stream") stream = 1;
        else if (a == "--page-tokens") page_tokens = std::atoi(next().c_str());
        else if (a == "--prompt-file") {
            std::ifstream f(next());
            if (!f) { std::fprintf(stderr, "cannot read %s\n", argv[i]); return 2; }
            prompt.clear();
            std::string tokstr;
            char c;
            auto flush = [&]() { if (!tokstr.empty()) prompt.push_back(std::atoi(tokstr.c_str())); tokstr.clear(); };
            while (f.get(c)) {
                if (c >= '0' && c <= '9') tokstr += c;
                else flush();
            }
            flush();
            if (prompt.empty()) { std::fprintf(stderr, "no token ids in %s\n", argv[i]); return 2; }
        }
        else if (a == "--prompt") {
            prompt.clear();
            std::string p = next();
            for (size_t s = 0; s < p.size();) {
                size_t e = p.find(',', s);
                prompt.push_back(std::atoi(p.substr(s, e - s).c_str()));
                if (e == std::string::npos) break;
                s = e + 1;
            }
        } else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    qie_model_spec spec = preset(model, numerics == "hf");
    qie_engine_opts opts;
    std::memset(&opts, 0, sizeof(opts));
    opts.device = device;
    opts.max_ctx = (int)prompt.size() + gen + 8;
    opts.use_graph = graph;
    opts.tp_size = 1;
    qie_engine* e = nullptr;
    if (qie_engine_create(&spec, &opts, &e)) { std::fprintf(stderr, "%s\n", qie_last_error()); return 1; }
    auto t0 = std::chrono::steady_clock::now();
    if (!weights.empty()) {
        std::vector<tensor> all = parsed_tensors(meta.c_str());
        TensorTable tt = build_indexed_tensors(all);
        std::printf("index: %zu tensors, %zu short names\n", all.size(), tt.size());
        if (!load_all_weights_to_gpu_chunked(e, weights.c_str(), meta.c_str(), (size_t)1 << 30)) {
            std::fprintf(stderr, "load: %s\n", qie_last_error());
            return 1;
        }
    } else {
        if (qie_engine_init_synthetic(e, seed < 0 ? 0 : (uint64_t)seed, 0.0346f, 0.f, 0.0346f)) {
            std::fprintf(stderr, "%s\n", qie_last_error());
            return 1;
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    std::printf("weights ready in %.2f s (%s)\n", std::chrono::duration<double>(t1 - t0).count(),
                weights.empty() ? "synthetic" : weights.c_str());
    qie_batch* b = nullptr;
    const int brc = page_tokens > 0 ? qie_batch_create_paged(e, 1, opts.max_ctx, page_tokens, 0, &b)
                                    : qie_batch_create(e, 1, opts.max_ctx, &b);
    if (brc) { std::fprintf(stderr, "%s\n", qie_last_error()); return 1; }
    batch_metadata* seq = create_new_sequence(0, prompt.data(), (int)prompt.size(), b, 0);
    qie_sampling g{1, 1.0f, 1.0f, 0};
    std::vector<int> out;
    auto tp0 = std::chrono::steady_clock::now();
    int tok = llm(seq, greedy ? &g : nullptr);
    auto tp1 = std::chrono::steady_clock::now();
    if (config().error) return 1;
    out.push_back(tok);
    if (stream) { std::printf("%d\n", tok); std::fflush(stdout); }
    seq->step++;                 // iengine.cu:419-421
    seq->generated_token = tok;
    seq->state = decode;
    while ((int)out.size() < gen && tok != kRefEos) {
        tok = llm(seq, greedy ? &g : nullptr);
        if (config().error) return 1;
        out.push_back(tok);
        if (stream) { std::printf("%d\n", tok); std::fflush(stdout); }
        seq->step++;
        seq->generated_token = tok;
    }
    auto tp2 = std::chrono::steady_clock::now();
    std::printf("tokens:");
    for (int t : out) std::printf(" %d", t);
    std::printf("\nprefill %zu tok: %.3f ms; decode %zu steps: %.3f ms/step\n", prompt.size(),
                std::chrono::duration<double, std::milli>(tp1 - tp0).count(), out.size() - 1,
                out.size() > 1 ? std::chrono::duration<double, std::milli>(tp2 - tp1).count() / (out.size() - 1) : 0.0);
    destroy_sequence(seq);
    qie_batch_destroy(b);
    qie_engine_destroy(e);
    return 0;
}
