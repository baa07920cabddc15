// C launch API of the mxllm gfx950 kernels (csrc/kernels/*.hip).
// All functions return 0 on success, a hipError_t (>0) or -1 on bad arguments.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {
// rmsnorm.hip
int mx_rmsnorm_fwd(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* y,
                   uint16_t* h_out, float* rstd, int T, int H, int ldy, float eps, hipStream_t stream);
int mx_rmsnorm_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* w, const float* rstd,
                   const uint16_t* dres, uint16_t* dx, float* dwp, int T, int H, int ldr, int ldx, int rpb,
                   hipStream_t stream);
int mx_colsum_f32(const float* p, float* out, int nblk, int H, hipStream_t stream);

// misc.hip
int mx_segmented_mean_i32(const int32_t* codes, const int64_t* offs, float* out, int nseg,
                          hipStream_t stream);
int mx_sqnorm(const void* x, int bf16, int64_t n, float* out, float* work, hipStream_t stream);
int mx_copy2d_batched(const int64_t* desc, int n, int64_t total_blocks, hipStream_t stream);
int mx_prefetch(const void* p, int64_t bytes, int wgs, hipStream_t stream);
int mx_transpose16(const void* in, void* out, int64_t R, int64_t C, int64_t ld_in, int64_t ld_out,
                   const float* scale, hipStream_t stream);
}

extern "C" {
// elementwise.hip
int mx_swiglu_fwd(const uint16_t* gu, uint16_t* m, int64_t T, int F, int64_t ldm, hipStream_t stream);
int mx_swiglu_bwd(const uint16_t* dm, const uint16_t* gu, uint16_t* dgu, int64_t T, int F, int64_t ldg,
                  hipStream_t stream, uint16_t* m = nullptr);
int mx_ce_inv_count(const int64_t* labels, int64_t T, int64_t ignore, float* inv_n, hipStream_t stream);
int mx_ce_chunk(uint16_t* logits, const int64_t* labels, float* losses, const float* inv_n, int64_t T, int V,
                int64_t ignore, hipStream_t stream);
int mx_ce_chunk_f32(const float* logits, uint16_t* dl, const int64_t* labels, float* losses, const float* inv_n,
                    int64_t T, int V, int64_t ignore, hipStream_t stream);
int mx_gemm8(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc, void* C,
             int64_t ldc, int out_f32, int M, int N, int K, float beta, const float* alpha_t, float alpha_f,
             int ph, hipStream_t stream);
int mx_gemm8_stamps(unsigned long long* host);
// layout of csrc/kernels/gemm8.hip G8Epi (fused forward epilogues)
struct MxG8Epi {
  uint16_t* q;
  uint16_t* k;
  uint16_t* v;
  const float* cosb;
  const float* sinb;
  int S, Hq, Hkv;
  uint16_t* m;
  int64_t ldm;
  int F;
  const uint16_t* gu;
  int64_t ldg;
  float* sq;
};
int mx_gemm8_epi(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, uint16_t* C, int64_t ldc, int M,
                 int N, int K, int mode, MxG8Epi ep, hipStream_t stream);
int mx_gemm8_sq(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc, uint16_t* C,
                int64_t ldc, int M, int N, int K, const float* alpha_t, float alpha_f, float* sq, hipStream_t stream);
int mx_gemm8_tail(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc, uint16_t* C,
                  int64_t ldc, int M, int N, int K, int rows, int at, float* ws, int ph, hipStream_t stream,
                  float* sq = nullptr);
int mx_gemm8_rope_tail(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M, int N, int K, int at,
                       float* ws, MxG8Epi ep, hipStream_t stream);
int mx_adamw(float* p, void* g, int grad_bf16, float* m, float* v, uint16_t* lowp, int16_t* lo, int64_t n,
             float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, const float* scale_t,
             float scale_f, int zero_grad, hipStream_t stream);
int mx_split_master(const float* x, uint16_t* hi, int16_t* lo, int64_t n, hipStream_t stream);
int mx_join_master(const uint16_t* hi, const int16_t* lo, float* x, int64_t n, hipStream_t stream);
int mx_embedding_fwd(const int64_t* ids, const uint16_t* w, uint16_t* out, int64_t T, int H, int64_t V,
                     hipStream_t stream);
int mx_embedding_bwd_sorted(const uint16_t* dy, const int64_t* sid, const int64_t* perm, int64_t T, int H,
                            int64_t V, void* out, int out_f32, float* ws, hipStream_t stream);
int mx_embedding_bwd(const int64_t* ids, const uint16_t* dy, float* dw, int64_t T, int H, int64_t V,
                     hipStream_t stream);
// cross_entropy.hip
int mx_ce_fwd_bwd(uint16_t* logits, const int64_t* labels, float* losses, float* inv_n, float* loss_out, int64_t T,
                  int V, int64_t ignore, hipStream_t stream);
// rope.hip
int mx_rope_split(const uint16_t* qkv, const float* cosb, const float* sinb, const int32_t* positions, uint16_t* q,
                  uint16_t* k, uint16_t* v, int B, int S, int Hq, int Hkv, int D, hipStream_t stream);
int mx_rope_merge_bwd(const float* dq, const float* dkp, const float* dvp, const float* cosb, const float* sinb,
                      uint16_t* dqkv, int B, int S, int Hq, int Hkv, int kv_heads_in, int D, int64_t ldq,
                      hipStream_t stream, int head0);
// attn_fwd.hip / attn_bwd.hip
int mx_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse, int B, int Hq,
                int Hkv, int S, int Sk, int D, int causal, float scale, int ldo, hipStream_t stream);
int mx_attn_bwd_partial_heads(int B, int Hq, int Hkv, int S, int Sk, int D, int dq_mode);
int mx_attn_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o, const uint16_t* dout,
                const float* lse, float* delta, float* dq, float* dkp, float* dvp, int B, int Hq, int Hkv, int S,
                int Sk, int D, int causal, float scale, int dq_mode, void* work, int64_t ldo, hipStream_t stream,
                uint16_t* dqkv, int64_t ldq, const float* cosb, const float* sinb);
}

extern "C" {
// decode.hip
int mx_rope_append(const uint16_t* qkv, const float* cosb, const float* sinb, const int32_t* pos, const int32_t* slots,
                   uint16_t* q, uint16_t* kc, uint16_t* vc, int B, int Hq, int Hkv, int D, int max_seq,
                   const int32_t* bt, int maxb, hipStream_t stream);
int mx_decode_attn(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* lens, int len_off,
                   const int32_t* slots, float* part_ml, float* part_o, uint16_t* out, int B, int Hq, int Hkv, int D,
                   int max_seq, int nsplit, float scale, const int32_t* bt, int maxb, unsigned int* cnt,
                   hipStream_t stream);
int64_t mx_sample_ws_floats(int B);
int mx_sample(const void* logits, int is_bf16, int64_t* out, int B, int V, float temperature, uint32_t seed,
              uint32_t step, float* ws, hipStream_t stream);
int mx_sample_temp_rows(const void* logits, int is_bf16, int64_t* out, int B, int V, const float* temps,
                        const int64_t* seeds, const int32_t* steps, float* ws, hipStream_t stream);
// sampling.hip
int mx_sample_rows(const void* logits, int is_bf16, int64_t* out, int B, int V, const float* temps,
                   const float* top_ps, const int32_t* top_ks, const int64_t* seeds, const int32_t* steps,
                   hipStream_t stream);
}

extern "C" {
// fp8_gemm.hip
int mx_skinny_gemm(const uint16_t* x, int64_t ldx, const uint16_t* w, int64_t ldw, uint16_t* y, int64_t ldy,
                   int M, int N, int K, hipStream_t stream);
int mx_skinny_gemm_swiglu(const uint16_t* x, int64_t ldx, const uint16_t* w, int64_t ldw, uint16_t* y,
                          int64_t ldy, int M, int F, int K, hipStream_t stream);
int mx_skinny_rope_gemm(const uint16_t* h, int64_t ldh, int norm, const uint16_t* delta, int64_t ldd,
                        const uint16_t* gamma, float eps, uint16_t* h_out, const uint16_t* w, int64_t ldw,
                        const float* cosb, const float* sinb, const int32_t* pos, const int32_t* slots, uint16_t* q,
                        uint16_t* kc, uint16_t* vc, int Hq, int Hkv, int max_seq, const int32_t* bt, int maxb, int M, int K, hipStream_t stream);
int mx_skinny_merge_gemm(const float* ml, const float* po, int nsplit, const uint16_t* w, int64_t ldw, uint16_t* y,
                         int64_t ldy, int M, int N, int K, hipStream_t stream);
int mx_skinny_norm_gemm(const uint16_t* h, int64_t ldh, const uint16_t* delta, int64_t ldd, const uint16_t* gamma,
                        float eps, uint16_t* h_out, const uint16_t* w, int64_t ldw, uint16_t* y, int64_t ldy, int M,
                        int N, int K, int swiglu, hipStream_t stream);
int mx_w8a16_gemm(const uint16_t* x, int64_t ldx, const uint8_t* q, const float* scale, uint16_t* y, int64_t ldy,
                  int M, int N, int K, hipStream_t stream);
int mx_w8_dequant(const uint8_t* q, const float* scale, uint16_t* w, int64_t N, int K, hipStream_t stream);
int mx_quant_rows_e4m3(const uint16_t* x, int64_t ldx, uint8_t* q, float* s, int64_t M, int K, hipStream_t stream);
int64_t mx_lora_xwt_ws(int M, int K, int rows);
int64_t mx_lora_xtg_ws(int ntiles, int T);
int mx_lora_xwt(const uint16_t* X, int64_t ldx, const uint16_t* V, int64_t ldv, int Vrows, uint16_t* out, int64_t ldo,
                float* ws, int M, int K, float alpha, int rows, hipStream_t stream);
int64_t mx_swiglu_lora_ws(int T, int F, int nrb);
int mx_swiglu_lora(int bwd, const uint16_t* gu, const uint16_t* dm, uint16_t* out, int64_t ldo, const uint16_t* V,
                   int64_t ldv, int nrb, int pad, float alpha, float* ws, int T, int F, hipStream_t stream);
int mx_lora_xtg(const int64_t* desc, int np, int T, float alpha, int accumulate, float* ws, hipStream_t stream);
}
