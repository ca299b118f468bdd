/*
 * asan_driver.c -- runs CPU-oracle functions (oracle/wf_oracle.c, compiled into this executable)
 * on inputs the caller wrote as raw little-endian files, under -fsanitize=address,undefined
 * (SURVEY.md §5 "race detection / sanitizers"; tests/test_sanitizers_cpu.py builds and drives it).
 * TEST INFRASTRUCTURE ONLY: the product library never links this.
 *
 *   asan_driver quant    n x.f32 q.i8 s.f64
 *   asan_driver qrows    M K x.f32 q.i8 s.f64
 *   asan_driver gemm     M N K scale w.u8 a.i8 y.f32
 *   asan_driver packs    N K w.f32 i2s.u8 tq.u8 back.u8          (I2_S pack, TQ pack, TQ unpack)
 *   asan_driver linear   N K ws x.u16 w.u8 y.u16
 *   asan_driver attn     Hq Hkv D Smax S mode q.u16 k.u16 v.u16 out.u16   (mode 0 exact, 1 SDPA)
 *   asan_driver decode   dir steps attn_mode                       (dir/<array>.bin, dir/cfg.txt,
 *                                                                    dir/tokens.i32 -> dir/logits.u16)
 * Every command exits 0 on success, 2 on an oracle argument error, 3 on an I/O error.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wf_oracle.h"

static void* rd(const char* path, size_t bytes) {
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "open %s\n", path); exit(3); }
    void* p = malloc(bytes ? bytes : 1);
    if (fread(p, 1, bytes, f) != bytes) { fprintf(stderr, "short read %s\n", path); exit(3); }
    fclose(f);
    return p;
}
static void wr(const char* path, const void* p, size_t bytes) {
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(p, 1, bytes, f) != bytes) { fprintf(stderr, "write %s\n", path); exit(3); }
    fclose(f);
}
static void ck(int rc) {
    if (rc) { fprintf(stderr, "oracle rejected its arguments\n"); exit(2); }
}
static char* cat(const char* dir, const char* name) {
    static char buf[4096];
    snprintf(buf, sizeof buf, "%s/%s", dir, name);
    return buf;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const char* cmd = argv[1];
    if (!strcmp(cmd, "quant") && argc == 6) {
        long n = atol(argv[2]);
        float* x = rd(argv[3], 4 * n);
        int8_t* q = malloc(n);
        double s;
        ck(orc_quantize_i8(x, n, q, &s));
        wr(argv[4], q, n);
        wr(argv[5], &s, 8);
        free(x); free(q);
    } else if (!strcmp(cmd, "qrows") && argc == 7) {
        int M = atoi(argv[2]), K = atoi(argv[3]);
        float* x = rd(argv[4], 4 * (size_t)M * K);
        int8_t* q = malloc((size_t)M * K);
        double* s = malloc(8 * (size_t)M);
        ck(orc_quantize_i8_rows(x, M, K, q, s));
        wr(argv[5], q, (size_t)M * K);
        wr(argv[6], s, 8 * (size_t)M);
        free(x); free(q); free(s);
    } else if (!strcmp(cmd, "gemm") && argc == 9) {
        int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]);
        float sc = (float)atof(argv[5]);
        uint8_t* w = rd(argv[6], (size_t)N * K / 4);
        int8_t* a = rd(argv[7], (size_t)M * K);
        float* y = malloc(4 * (size_t)M * N);
        ck(orc_gemm_i2s(w, a, sc, M, N, K, y));
        wr(argv[8], y, 4 * (size_t)M * N);
        free(w); free(a); free(y);
    } else if (!strcmp(cmd, "packs") && argc == 8) {
        int N = atoi(argv[2]), K = atoi(argv[3]);
        float* w = rd(argv[4], 4 * (size_t)N * K);
        uint8_t* p = malloc((size_t)N * K / 4);
        ck(orc_pack_i2s(w, N, K, p));
        wr(argv[5], p, (size_t)N * K / 4);
        const size_t tb = (size_t)N * (size_t)orc_tq_row_bytes(K);
        uint8_t* t = malloc(tb);
        uint8_t* back = malloc((size_t)N * K / 4);
        ck(orc_pack_tq(p, N, K, t));
        ck(orc_unpack_tq(t, N, K, back));
        wr(argv[6], t, tb);
        wr(argv[7], back, (size_t)N * K / 4);
        free(w); free(p); free(t); free(back);
    } else if (!strcmp(cmd, "linear") && argc == 8) {
        int N = atoi(argv[2]), K = atoi(argv[3]);
        float ws = (float)atof(argv[4]);
        uint16_t* x = rd(argv[5], 2 * (size_t)K);
        uint8_t* w = rd(argv[6], (size_t)N * K / 4);
        uint16_t* y = malloc(2 * (size_t)N);
        ck(orc_bitnet_linear_bf16(x, w, ws, N, K, y));
        wr(argv[7], y, 2 * (size_t)N);
        free(x); free(w); free(y);
    } else if (!strcmp(cmd, "attn") && argc == 12) {
        int Hq = atoi(argv[2]), Hkv = atoi(argv[3]), D = atoi(argv[4]), Smax = atoi(argv[5]), S = atoi(argv[6]);
        int mode = atoi(argv[7]);
        uint16_t* q = rd(argv[8], 2 * (size_t)Hq * D);
        uint16_t* k = rd(argv[9], 2 * (size_t)Hkv * Smax * D);
        uint16_t* v = rd(argv[10], 2 * (size_t)Hkv * Smax * D);
        uint16_t* o = malloc(2 * (size_t)Hq * D);
        if (mode) ck(orc_attention_sdpa_cpu_bf16(q, k, v, Hq, Hkv, D, Smax, S, o));
        else ck(orc_attention_gqa_bf16(q, k, v, Hq, Hkv, D, Smax, S, 1.0f / sqrtf((float)D), o));
        wr(argv[11], o, 2 * (size_t)Hq * D);
        free(q); free(k); free(v); free(o);
    } else if (!strcmp(cmd, "decode") && argc == 5) {
        const char* dir = argv[2];
        int steps = atoi(argv[3]);
        orc_model m;
        memset(&m, 0, sizeof m);
        FILE* f = fopen(cat(dir, "cfg.txt"), "r");
        if (!f || fscanf(f, "%d %d %d %d %d %d %d %d %f", &m.hidden, &m.layers, &m.n_heads, &m.n_kv_heads,
                         &m.head_dim, &m.inter, &m.vocab, &m.max_seq, &m.eps) != 9) return 3;
        fclose(f);
        const size_t H = m.hidden, L = m.layers, I = m.inter, V = m.vocab, D = m.head_dim, S = m.max_seq;
        const size_t KV = (size_t)m.n_kv_heads * D;
        m.embed = rd(cat(dir, "embed.bin"), 2 * V * H);
        m.final_norm = rd(cat(dir, "final_norm.bin"), 2 * H);
        m.rope_cos = rd(cat(dir, "rope_cos.bin"), 2 * S * (D / 2));
        m.rope_sin = rd(cat(dir, "rope_sin.bin"), 2 * S * (D / 2));
        m.ln_in = rd(cat(dir, "ln_in.bin"), 2 * L * H);
        m.ln_post = rd(cat(dir, "ln_post.bin"), 2 * L * H);
        m.attn_sub = rd(cat(dir, "attn_sub.bin"), 2 * L * H);
        m.ffn_sub = rd(cat(dir, "ffn_sub.bin"), 2 * L * I);
        m.wq = rd(cat(dir, "wq.bin"), L * H * H / 4);
        m.wk = rd(cat(dir, "wk.bin"), L * KV * H / 4);
        m.wv = rd(cat(dir, "wv.bin"), L * KV * H / 4);
        m.wo = rd(cat(dir, "wo.bin"), L * H * H / 4);
        m.wg = rd(cat(dir, "wg.bin"), L * I * H / 4);
        m.wu = rd(cat(dir, "wu.bin"), L * I * H / 4);
        m.wd = rd(cat(dir, "wd.bin"), L * H * I / 4);
        m.wscale = rd(cat(dir, "wscale.bin"), 4 * L * 7);
        m.k_cache = calloc(L * KV * S, 2);
        m.v_cache = calloc(L * KV * S, 2);
        m.attn_mode = atoi(argv[4]);
        int32_t* tokens = rd(cat(dir, "tokens.i32"), 4 * (size_t)steps);
        uint16_t* logits = malloc(2 * V * (size_t)steps);
        for (int i = 0; i < steps; ++i) {
            int nxt;
            ck(orc_decode_step(&m, tokens[i], i, logits + (size_t)i * V, &nxt));
        }
        wr(cat(dir, "logits.u16"), logits, 2 * V * (size_t)steps);
        free((void*)m.embed); free((void*)m.final_norm); free((void*)m.rope_cos); free((void*)m.rope_sin);
        free((void*)m.ln_in); free((void*)m.ln_post); free((void*)m.attn_sub); free((void*)m.ffn_sub);
        free((void*)m.wq); free((void*)m.wk); free((void*)m.wv); free((void*)m.wo); free((void*)m.wg);
        free((void*)m.wu); free((void*)m.wd); free((void*)m.wscale); free(m.k_cache); free(m.v_cache);
        free(tokens); free(logits);
    } else {
        fprintf(stderr, "unknown command or argument count: %s\n", cmd);
        return 2;
    }
    return 0;
}
