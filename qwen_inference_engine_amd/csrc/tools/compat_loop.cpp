// compat_loop — the reference's own layer loop, op by op, written ONLY against the
// operator tier of include/qie/compat.hpp (launch_rms, proj, launch_qknorm, launch_rope,
// kv_copy_layer_to_cache_prefill/decode, launch_attn, launch_resadd, launch_act,
// launch_elem, copy_last_vocab_vec / copy_first_token, launch_matmul, sample_topk_bf16,
// initialize_model_buffers / destroy_model_buffers, page lists).  Prefill follows
// layers/src/qwen_main.cu:77-241 and each decode step :250-405, in the same order.
// Used by tests/test_gpu_compat.py: the logits of every step are checked against the
// CPU oracle.  Weights are the engine's synthetic init (reachable through the index
// exactly as the reference reaches weights.bin: arena + data_offsets[0]).
//
//   compat_loop OUT.bin L H NQ NKV HD I V EPS THETA SEED PAGED G  P id0 .. id{P-1}  F f0 .. f{F-1}
//
// OUT.bin: for each of the G + 1 sampled tokens, int32 token then V bf16 logits.  The
// F forced ids (teacher forcing; F may be 0) replace the sampled token as the next
// step's input where given.  Greedy (sample_topk_bf16 with k = 1).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../../include/qie/compat.hpp"

using namespace qie_compat;

int main(int argc, char** argv) {
    if (argc < 16) {
        std::fprintf(stderr, "usage: compat_loop OUT L H NQ NKV HD I V EPS THETA SEED PAGED G P ids.. F ids..\n");
        return 2;
    }
    int ai = 1;
    const char* out_path = argv[ai++];
    qie_model_spec s;
    std::memset(&s, 0, sizeof(s));
    s.n_layers = atoi(argv[ai++]);
    s.hidden = atoi(argv[ai++]);
    s.n_heads = atoi(argv[ai++]);
    s.n_kv_heads = atoi(argv[ai++]);
    s.head_dim = atoi(argv[ai++]);
    s.ffn = atoi(argv[ai++]);
    s.vocab = atoi(argv[ai++]);
    s.rms_eps = (float)atof(argv[ai++]);
    s.rope_theta = (float)atof(argv[ai++]);
    s.qk_norm = 1;   // the reference's model family (Qwen3: qk-norm, no q/k/v bias)
    s.numerics = QIE_NUMERICS_REF;
    const long seed = atol(argv[ai++]);
    const int paged = atoi(argv[ai++]);
    const int G = atoi(argv[ai++]);
    const int P = atoi(argv[ai++]);
    std::vector<int> prompt;
    for (int i = 0; i < P; i++) prompt.push_back(atoi(argv[ai++]));
    const int F = ai < argc ? atoi(argv[ai++]) : 0;
    std::vector<int> forced;
    for (int i = 0; i < F && ai < argc; i++) forced.push_back(atoi(argv[ai++]));

    const int max_ctx = P + G + 8;
    qie_engine_opts o;
    std::memset(&o, 0, sizeof(o));
    o.max_ctx = max_ctx;
    o.use_graph = 0;
    qie_engine* e = nullptr;
    if (qie_engine_create(&s, &o, &e) || qie_engine_init_synthetic(e, (uint64_t)seed, 0.08f, 0.25f, 0.05f)) {
        std::fprintf(stderr, "engine: %s\n", qie_last_error());
        return 1;
    }
    qie_batch* kvb = nullptr;
    if ((paged ? qie_batch_create_paged(e, 1, max_ctx, 128, 0, &kvb) : qie_batch_create(e, 1, max_ctx, &kvb)) != 0) {
        std::fprintf(stderr, "batch: %s\n", qie_last_error());
        return 1;
    }
    // the reference reaches every weight as arena + data_offsets[0] through the index
    qie_index* idx = nullptr;
    const std::string meta = std::string(out_path) + ".meta";
    if (qie_index_synthetic(&s, &idx) || qie_index_write_meta(idx, meta.c_str())) {
        std::fprintf(stderr, "index: %s\n", qie_last_error());
        return 1;
    }
    qie_index_destroy(idx);
    std::vector<tensor> all = parsed_tensors(meta.c_str());
    TensorTable tensors = build_indexed_tensors(all);
    void* arena = nullptr;
    int64_t arena_bytes = 0;
    qie_engine_arena(e, &arena, &arena_bytes);
    bf16* g_gpu_weights_buffer = (bf16*)arena;
    std::ifstream weights;   // unused: weights are resident (signature parity only)

    config().rms_eps = s.rms_eps;
    config().qk_eps = s.rms_eps;
    page_table* kv_cache_seq1 = create_page_list(kvb, 0);
    const int page_size = 128;
    ModelBuffers bufs;
    ModelBuffers* buffer = &bufs;
    if (!initialize_model_buffers(bufs, prompt.data(), tensors, e, (size_t)P)) return 1;
    FILE* out = std::fopen(out_path, "wb");
    std::vector<uint16_t> lg(s.vocab);
    auto emit = [&](int tok) {
        qie_memcpy_d2h(lg.data(), buffer->prefill_output_d, (int64_t)s.vocab * 2);
        std::fwrite(&tok, 4, 1, out);
        std::fwrite(lg.data(), 2, lg.size(), out);
    };

    // ------------------------------------------------------------- prefill (:77-241)
    for (size_t i = 0; i < buffer->number_of_layers; i++) {
        load_weight(tensors["input_layernorm.weight"][i], weights, buffer->norm_weights_h, buffer->norm_weights_d,
                    buffer->hidden_dim, g_gpu_weights_buffer);
        launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim,
                   buffer->sequence_len);
        proj(tensors["self_attn.q_proj.weight"][i], weights, buffer->q_proj_weights_h, buffer->q_proj_weights_d,
             buffer->q_proj_size, buffer->rms_out, buffer->Q, buffer->sequence_len, buffer->hidden_dim,
             buffer->num_of_qheads * buffer->head_dim, g_gpu_weights_buffer);
        proj(tensors["self_attn.k_proj.weight"][i], weights, buffer->kv_proj_weights_h, buffer->kv_proj_weights_d,
             buffer->kv_proj_size, buffer->rms_out, buffer->K, buffer->sequence_len, buffer->hidden_dim,
             buffer->hidden_dim_kv, g_gpu_weights_buffer);
        proj(tensors["self_attn.v_proj.weight"][i], weights, buffer->kv_proj_weights_h, buffer->kv_proj_weights_d,
             buffer->kv_proj_size, buffer->rms_out, buffer->V, buffer->sequence_len, buffer->hidden_dim,
             buffer->hidden_dim_kv, g_gpu_weights_buffer);
        load_weight(tensors["self_attn.q_norm.weight"][i], weights, buffer->qk_norm_weights_h,
                    buffer->qk_norm_weights_d, buffer->head_dim, g_gpu_weights_buffer);
        launch_qknorm(buffer->Q, buffer->qk_norm_weights_d, buffer->head_dim, buffer->sequence_len,
                      buffer->num_of_qheads * buffer->head_dim, buffer->num_of_qheads);
        load_weight(tensors["self_attn.k_norm.weight"][i], weights, buffer->qk_norm_weights_h,
                    buffer->qk_norm_weights_d, buffer->head_dim, g_gpu_weights_buffer);
        launch_qknorm(buffer->K, buffer->qk_norm_weights_d, buffer->head_dim, buffer->sequence_len,
                      buffer->hidden_dim_kv, buffer->num_of_kvheads);
        launch_rope(buffer->cos_values_d, buffer->sin_values_d, buffer->Q, buffer->sequence_len, buffer->head_dim,
                    buffer->num_of_qheads * buffer->head_dim, buffer->num_of_qheads);
        launch_rope(buffer->cos_values_d, buffer->sin_values_d, buffer->K, buffer->sequence_len, buffer->head_dim,
                    buffer->hidden_dim_kv, buffer->num_of_kvheads);
        kv_copy_layer_to_cache_prefill(buffer, (int)i, kv_cache_seq1, page_size);
        launch_attn(buffer->Q, buffer->atten_out, buffer->sequence_len, buffer->sequence_len, buffer->head_dim,
                    buffer->num_of_qheads * buffer->head_dim, buffer->hidden_dim_kv, /*causal=*/1, 0, (int)i,
                    kv_cache_seq1, page_size);
        proj(tensors["self_attn.o_proj.weight"][i], weights, buffer->o_proj_weights_h, buffer->o_proj_weights_d,
             buffer->o_proj_size, buffer->atten_out, buffer->out_proj, buffer->sequence_len,
             buffer->num_of_qheads * buffer->head_dim, buffer->hidden_dim, g_gpu_weights_buffer);
        launch_resadd(buffer->embeddings_out, buffer->out_proj, buffer->sequence_len * buffer->hidden_dim);
        load_weight(tensors["post_attention_layernorm.weight"][i], weights, buffer->norm_weights_h,
                    buffer->norm_weights_d, buffer->hidden_dim, g_gpu_weights_buffer);
        launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim,
                   buffer->sequence_len);
        proj(tensors["mlp.up_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h, buffer->mlp_up_proj_weights_d,
             buffer->mlp_up_proj_size, buffer->rms_out, buffer->MLP_UP, buffer->sequence_len, buffer->hidden_dim,
             buffer->up_dim, g_gpu_weights_buffer);
        proj(tensors["mlp.gate_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h,
             buffer->mlp_up_proj_weights_d, buffer->mlp_up_proj_size, buffer->rms_out, buffer->MLP_GATE,
             buffer->sequence_len, buffer->hidden_dim, buffer->up_dim, g_gpu_weights_buffer);
        launch_act(buffer->MLP_GATE, buffer->sequence_len * buffer->up_dim);
        launch_elem(buffer->MLP_UP, buffer->MLP_GATE, buffer->MLP_GATE_OUT, buffer->sequence_len * buffer->up_dim);
        proj(tensors["mlp.down_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h,
             buffer->mlp_up_proj_weights_d, buffer->mlp_up_proj_size, buffer->MLP_GATE_OUT, buffer->MLP_DOWN,
             buffer->sequence_len, buffer->up_dim, buffer->hidden_dim, g_gpu_weights_buffer);
        launch_resadd(buffer->embeddings_out, buffer->MLP_DOWN, buffer->sequence_len * buffer->hidden_dim);
    }
    load_weight(tensors["norm.weight"][0], weights, buffer->norm_weights_h, buffer->norm_weights_d,
                buffer->hidden_dim, g_gpu_weights_buffer);
    launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim,
               buffer->sequence_len);
    load_weight(tensors["logits"][0], weights, buffer->logits_weights_h, buffer->logits_weights_d,
                buffer->logtis_shape, g_gpu_weights_buffer);
    copy_last_vocab_vec(buffer->rms_out, buffer->last_x, buffer->hidden_dim, buffer->sequence_len);
    launch_matmul(buffer->last_x, buffer->logits_weights_d, buffer->prefill_output_d, 1, buffer->hidden_dim,
                  buffer->vocab_size);
    int tok = sample_topk_bf16(buffer->prefill_output_d, buffer->vocab_size, 1.0f, /*greedy*/ 1, 1234ULL, 0);
    emit(tok);

    // ---------------------------------------------------- decode steps (:250-405)
    for (int step = 1; step <= G && config().error == 0; step++) {
        const int in_tok = step - 1 < (int)forced.size() ? forced[step - 1] : tok;
        const size_t q1 = 1;
        buffer->sequence_len = buffer->sequence_len + 1;
        embed_tokens(bufs, &in_tok, 1);
        for (size_t i = 0; i < buffer->number_of_layers; i++) {
            load_weight(tensors["input_layernorm.weight"][i], weights, buffer->norm_weights_h,
                        buffer->norm_weights_d, buffer->hidden_dim, g_gpu_weights_buffer);
            launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim, q1);
            proj(tensors["self_attn.q_proj.weight"][i], weights, buffer->q_proj_weights_h, buffer->q_proj_weights_d,
                 buffer->q_proj_size, buffer->rms_out, buffer->Q, q1, buffer->hidden_dim,
                 buffer->num_of_qheads * buffer->head_dim, g_gpu_weights_buffer);
            proj(tensors["self_attn.k_proj.weight"][i], weights, buffer->kv_proj_weights_h,
                 buffer->kv_proj_weights_d, buffer->kv_proj_size, buffer->rms_out, buffer->K, q1, buffer->hidden_dim,
                 buffer->hidden_dim_kv, g_gpu_weights_buffer);
            proj(tensors["self_attn.v_proj.weight"][i], weights, buffer->kv_proj_weights_h,
                 buffer->kv_proj_weights_d, buffer->kv_proj_size, buffer->rms_out, buffer->V, q1, buffer->hidden_dim,
                 buffer->hidden_dim_kv, g_gpu_weights_buffer);
            load_weight(tensors["self_attn.q_norm.weight"][i], weights, buffer->qk_norm_weights_h,
                        buffer->qk_norm_weights_d, buffer->head_dim, g_gpu_weights_buffer);
            launch_qknorm(buffer->Q, buffer->qk_norm_weights_d, buffer->head_dim, q1,
                          buffer->num_of_qheads * buffer->head_dim, buffer->num_of_qheads);
            load_weight(tensors["self_attn.k_norm.weight"][i], weights, buffer->qk_norm_weights_h,
                        buffer->qk_norm_weights_d, buffer->head_dim, g_gpu_weights_buffer);
            launch_qknorm(buffer->K, buffer->qk_norm_weights_d, buffer->head_dim, q1, buffer->hidden_dim_kv,
                          buffer->num_of_kvheads);
            launch_rope_single(buffer->cos_values_d, buffer->sin_values_d, buffer->Q, buffer->sequence_len - 1,
                               buffer->head_dim, buffer->num_of_qheads * buffer->head_dim, buffer->num_of_qheads);
            launch_rope_single(buffer->cos_values_d, buffer->sin_values_d, buffer->K, buffer->sequence_len - 1,
                               buffer->head_dim, buffer->hidden_dim_kv, buffer->num_of_kvheads);
            kv_copy_layer_to_cache_decode(buffer, (int)i, kv_cache_seq1, page_size);
            const int q_abs = (int)buffer->sequence_len - 1;
            launch_attn(buffer->Q, buffer->atten_out, q1, buffer->sequence_len, buffer->head_dim,
                        buffer->num_of_qheads * buffer->head_dim, buffer->hidden_dim_kv, /*causal=*/0, q_abs, (int)i,
                        kv_cache_seq1, page_size);
            proj(tensors["self_attn.o_proj.weight"][i], weights, buffer->o_proj_weights_h, buffer->o_proj_weights_d,
                 buffer->o_proj_size, buffer->atten_out, buffer->out_proj, q1,
                 buffer->num_of_qheads * buffer->head_dim, buffer->hidden_dim, g_gpu_weights_buffer);
            launch_resadd(buffer->embeddings_out, buffer->out_proj, q1 * buffer->hidden_dim);
            load_weight(tensors["post_attention_layernorm.weight"][i], weights, buffer->norm_weights_h,
                        buffer->norm_weights_d, buffer->hidden_dim, g_gpu_weights_buffer);
            launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim, q1);
            proj(tensors["mlp.up_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h,
                 buffer->mlp_up_proj_weights_d, buffer->mlp_up_proj_size, buffer->rms_out, buffer->MLP_UP, q1,
                 buffer->hidden_dim, buffer->up_dim, g_gpu_weights_buffer);
            proj(tensors["mlp.gate_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h,
                 buffer->mlp_up_proj_weights_d, buffer->mlp_up_proj_size, buffer->rms_out, buffer->MLP_GATE, q1,
                 buffer->hidden_dim, buffer->up_dim, g_gpu_weights_buffer);
            launch_act(buffer->MLP_GATE, q1 * buffer->up_dim);
            launch_elem(buffer->MLP_UP, buffer->MLP_GATE, buffer->MLP_GATE_OUT, q1 * buffer->up_dim);
            proj(tensors["mlp.down_proj.weight"][i], weights, buffer->mlp_up_proj_weights_h,
                 buffer->mlp_up_proj_weights_d, buffer->mlp_up_proj_size, buffer->MLP_GATE_OUT, buffer->MLP_DOWN, q1,
                 buffer->up_dim, buffer->hidden_dim, g_gpu_weights_buffer);
            launch_resadd(buffer->embeddings_out, buffer->MLP_DOWN, q1 * buffer->hidden_dim);
        }
        load_weight(tensors["norm.weight"][0], weights, buffer->norm_weights_h, buffer->norm_weights_d,
                    buffer->hidden_dim, g_gpu_weights_buffer);
        launch_rms(buffer->embeddings_out, buffer->norm_weights_d, buffer->rms_out, buffer->hidden_dim, q1);
        load_weight(tensors["logits"][0], weights, buffer->logits_weights_h, buffer->logits_weights_d,
                    buffer->logtis_shape, g_gpu_weights_buffer);
        copy_first_token(buffer->rms_out, buffer->last_x, buffer->hidden_dim);
        launch_matmul(buffer->last_x, buffer->logits_weights_d, buffer->prefill_output_d, 1, buffer->hidden_dim,
                      buffer->vocab_size);
        tok = sample_topk_bf16(buffer->prefill_output_d, buffer->vocab_size, 0.7f, /*greedy*/ 1, 1234ULL + step, 0);
        emit(tok);
    }
    std::fclose(out);
    std::remove(meta.c_str());
    destroy_model_buffers(bufs);
    free_page_list(kv_cache_seq1);
    qie_batch_destroy(kvb);
    qie_engine_destroy(e);
    if (config().error) {
        std::fprintf(stderr, "compat_loop: a launch failed (rc %d)\n", config().error);
        return 1;
    }
    return 0;
}
