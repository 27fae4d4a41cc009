// smsgate_amd — native launch sequences for the work that is NOT graph-captured.
//
// The decode steps replay hipGraphs, but a prefill's shape (tokens, sequences,
// longest prompt) changes with every admission, so its 30-layer forward used to be
// launched op by op from Python: 150 launches per half batch, each through the
// Python wrapper's shape checks, tile lookup, pointer extraction and a ctypes
// call (~20-30 us of host time apiece).  At the headline's rate the rank process
// then spent ~11 ms of each ~28 ms engine step inside admission, close enough to
// the GPU's time per step that every host hiccup left the GPU idle.
// sg_prefill_forward runs the same kernels in the same order from one C call:
// per layer the QKV+RoPE+KV-write GEMM, the varlen prefill attention, the o-proj
// residual GEMM, the SwiGLU gate/up GEMM and the down-proj residual GEMM (the
// sequence of ExtractionEngine._layers_fused, serving/engine.py), every launch on the
// caller's stream.  The tile configs are chosen by the caller (ops.gemm_cfg).
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

int sg_gemm(const void* A, int lda, const void* W, void* C, int ldc, const void* R, int ldr, int M, int N, int K,
            int epi, int norm, float eps, int cfg, const float* ssin, float* ssout, int ss_ld, hipStream_t stream);
int sg_gemm_qkv_rope(const void* A, int lda, const void* W, int M, int K, float eps, int cfg, const int* pos,
                     const int* slot, const void* cos_sin, void* q_out, void* k_cache, void* vt_cache, int nh, int nkv,
                     int Lmax, int p0, const float* ssin, int ss_ld, hipStream_t stream);
int sg_attn_prefill(const void* q, const int* cu_q, const int* q_start, const int* slot, const void* k_cache,
                    const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int nseq,
                    int max_q, int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream);

// Per-layer pointers are arrays of L device addresses (weights in the fused serving
// layout: norm folded in, gate/up interleaved; the layer's K cache / blocked V^T cache /
// shared-prefix K and V^T).  x [T, H] is the residual stream, updated in place; q
// [T, nh, D], a [T, nh*D] and act [T, I] are scratch; ss [16][ss_ld] the producer-norm
// row partials (zeroed by the caller; null: every norm GEMM accumulates x² itself).
// Returns 0, or the first failing launch's code + 1000 * (5 * layer + op).
int sg_prefill_forward(int L, const int64_t* w_qkv, const int64_t* w_o, const int64_t* w_gu, const int64_t* w_down,
                       const int64_t* k_cache, const int64_t* vt_cache, const int64_t* pk, const int64_t* pvt,
                       void* x, int T, int H, int I, int nh, int nkv, int D, int Lmax, int P0, int P0pad,
                       const int* pos, const int* slot, const void* cos_sin, int p0, const int* cu_q,
                       const int* q_start, const int* seq_slot, int nseq, int max_q, float scale, void* q, void* a,
                       void* act, float* ss, int ss_ld, float eps, int cfg_qkv, int cfg_o, int cfg_gu, int cfg_down,
                       hipStream_t stream) {
  if (L <= 0 || T <= 0) return 0;
  const int HA = nh * D;
  auto P = [](int64_t v) { return reinterpret_cast<void*>(static_cast<intptr_t>(v)); };
  for (int i = 0; i < L; ++i) {
    int rc = sg_gemm_qkv_rope(x, H, P(w_qkv[i]), T, H, eps, cfg_qkv, pos, slot, cos_sin, q, P(k_cache[i]),
                              P(vt_cache[i]), nh, nkv, Lmax, p0, i > 0 ? ss : nullptr, ss_ld, stream);
    if (rc) return rc + 1000 * (5 * i);
    rc = sg_attn_prefill(q, cu_q, q_start, seq_slot, P(k_cache[i]), P(vt_cache[i]), P(pk[i]), P(pvt[i]), P0, P0pad, a,
                         nseq, max_q, nh, nkv, D, Lmax, scale, stream);
    if (rc) return rc + 1000 * (5 * i + 1);
    rc = sg_gemm(a, HA, P(w_o[i]), x, H, x, H, T, H, HA, /*epi resid*/ 1, /*norm*/ 0, 0.f, cfg_o, nullptr, ss, ss_ld,
                 stream);
    if (rc) return rc + 1000 * (5 * i + 2);
    rc = sg_gemm(x, H, P(w_gu[i]), act, I, nullptr, 0, T, 2 * I, H, /*epi swiglu*/ 2, ss ? 2 : 1, eps, cfg_gu, ss,
                 nullptr, ss_ld, stream);
    if (rc) return rc + 1000 * (5 * i + 3);
    rc = sg_gemm(act, I, P(w_down[i]), x, H, x, H, T, H, I, /*epi resid*/ 1, /*norm*/ 0, 0.f, cfg_down, nullptr, ss,
                 ss_ld, stream);
    if (rc) return rc + 1000 * (5 * i + 4);
  }
  return 0;
}

}  // extern "C"
