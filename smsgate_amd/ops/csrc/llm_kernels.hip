// smsgate_amd — HIP/CDNA4 (gfx950) kernels for the local extraction LM.
//
// Plain C ABI (extern "C"), launched on a caller-supplied hipStream_t so every
// launch is capturable into a hipGraph by torch.cuda.CUDAGraph; no allocation,
// no synchronisation inside a launch function (cdna_hip_programming.md G9).
//
// Kernels (all bf16 storage, fp32 math):
//   sg_rmsnorm_residual  residual += x (optional); out = rmsnorm(residual) * w
//   sg_silu_mul          out = silu(gu[:, :I]) * gu[:, I:]
//   sg_rope_qkv_cache    RoPE(q,k) + write K rows / V^T columns into the KV cache
//   sg_attn_prefill      varlen causal attention over [shared prefix | own keys],
//                        MFMA 16x16x32 bf16, one wave per 16 query rows
//   sg_attn_decode       one query token per sequence, GQA group per workgroup
//   sg_fsm_sample        schema-FSM masked argmax / Gumbel sampling + FSM step
//
// KV layout (memory sized for 288 GB HBM: every slot owns its rows, no paging):
//   K   [slots][nkv][Lmax][D]   (a key row is 128 contiguous bytes at D = 64)
//   V^T [slots][nkv][D][Lmax]   (transposed so 8 consecutive keys of one dim are
//                                one 16-byte load: the MFMA B operand of P·V)
// Key index space of a sequence = [prefix keys 0..P0pad) ++ [own keys]:
// the shared system-prompt prefix lives once in pk/pvt (zero padded to a
// multiple of 32 keys), own keys live in the slot, RoPE position = P0 + own offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

static __device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
static __device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 on gfx950: RNE, NaN stays NaN
  return __builtin_bit_cast(uint16_t, b);
}
static __device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
static __device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}

// ---------------------------------------------------------------------------
// RMSNorm (+ residual add). One wave per row, 4 rows per 256-thread block.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) rmsnorm_residual_kernel(const uint16_t* __restrict__ x_in,
                                                               uint16_t* __restrict__ residual,
                                                               const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ out, int T, int H,
                                                               float eps) {
  // The row stays in registers (<= RMS_MAXV chunks of 8 per lane, H <= 2048):
  // one read of residual/x, one write of residual and out — no second pass.
  constexpr int RMS_MAXV = 4;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nvec = H >> 3;
  uint4* r4 = reinterpret_cast<uint4*>(residual + (size_t)row * H);
  const uint4* x4 = x_in ? reinterpret_cast<const uint4*>(x_in + (size_t)row * H) : nullptr;
  uint4 rv[RMS_MAXV], xv[RMS_MAXV];
#pragma unroll
  for (int k = 0; k < RMS_MAXV; ++k) {
    const int c = lane + k * WAVE;
    if (c < nvec) {
      rv[k] = r4[c];
      if (x4) xv[k] = x4[c];
    }
  }
  float ss = 0.f;
  float a[RMS_MAXV][8];
#pragma unroll
  for (int k = 0; k < RMS_MAXV; ++k) {
    const int c = lane + k * WAVE;
    if (c < nvec) {
      unpack8(rv[k], a[k]);
      if (x4) {
        float b[8];
        unpack8(xv[k], b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[k][j] = bf2f(f2bf(a[k][j] + b[j]));  // residual stream stays bf16
        r4[c] = pack8(a[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += a[k][j] * a[k][j];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  const uint4* w4 = reinterpret_cast<const uint4*>(w);
  uint4* o4 = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
  for (int k = 0; k < RMS_MAXV; ++k) {
    const int c = lane + k * WAVE;
    if (c < nvec) {
      float g[8];
      unpack8(w4[c], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = a[k][j] * r * g[j];
      o4[c] = pack8(g);
    }
  }
}

// ---------------------------------------------------------------------------
// SwiGLU activation: out[t, i] = silu(gu[t, i]) * gu[t, I + i]; 8 elements/thread.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                       int T, int I) {
  const int nv = I >> 3;
  const long total = (long)T * nv;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long t = idx / nv;
    const int c = (int)(idx - t * nv);
    const uint4* row = reinterpret_cast<const uint4*>(gu + (size_t)t * 2 * I);
    float g[8], u[8];
    unpack8(row[c], g);
    unpack8(row[nv + c], u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    reinterpret_cast<uint4*>(out + (size_t)t * I)[c] = pack8(g);
  }
}

// ---------------------------------------------------------------------------
// RoPE on q and k (rotate-half convention) + KV-cache write. One block/token.
//   qkv    [T][(nh + 2 nkv) D]    (GEMM output)
//   pos    [T] own offset of the token; RoPE position = p0 + pos
//   slot   [T] cache slot
//   cs     [max_pos][D/2] float2 (cos, sin)
// ---------------------------------------------------------------------------
// One wave per token, 4 tokens per block. V goes to the *blocked* V^T layout
// [slot][kvh][Lmax/8][D][8]: one token's 64 values land in one 1 KiB block (8
// cache lines) instead of 64 rows, and a P·V reader gets 8 keys of one dim as
// one 16-byte load with the 64 lanes of a wave reading 1 KiB contiguously.
__global__ void __launch_bounds__(256) rope_qkv_cache_kernel(const uint16_t* __restrict__ qkv, const int* __restrict__ pos,
                                                             const int* __restrict__ slot, const float2* __restrict__ cs,
                                                             uint16_t* __restrict__ q_out, uint16_t* __restrict__ k_cache,
                                                             uint16_t* __restrict__ vt_cache, int T, int nh, int nkv,
                                                             int D, int Lmax, int p0) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const int half = D >> 1;
  const int p = pos[t];
  const int s = slot[t];
  const float2* cst = cs + (size_t)(p0 + p) * half;
  const uint16_t* src = qkv + (size_t)t * (nh + 2 * nkv) * D;
  const int nrot = (nh + nkv) * half;
  for (int it = lane; it < nrot; it += WAVE) {
    const int h = it / half;
    const int i = it - h * half;
    const float2 c = cst[i];
    const float x1 = bf2f(src[h * D + i]);
    const float x2 = bf2f(src[h * D + i + half]);
    const float y1 = x1 * c.x - x2 * c.y;
    const float y2 = x2 * c.x + x1 * c.y;
    if (h < nh) {
      uint16_t* q = q_out + ((size_t)t * nh + h) * D;
      q[i] = f2bf(y1);
      q[i + half] = f2bf(y2);
    } else {
      const int kh = h - nh;
      uint16_t* k = k_cache + (((size_t)s * nkv + kh) * Lmax + p) * D;
      k[i] = f2bf(y1);
      k[i + half] = f2bf(y2);
    }
  }
  const uint16_t* v = src + (nh + nkv) * D;
  const int nb = Lmax >> 3;
  for (int it = lane; it < nkv * D; it += WAVE) {
    const int kh = it / D;
    const int d = it - kh * D;
    vt_cache[((((size_t)s * nkv + kh) * nb + (p >> 3)) * D + d) * 8 + (p & 7)] = v[it];
  }
}

// ---------------------------------------------------------------------------
// Prefill attention (varlen, causal), D = 64, MFMA 16x16x32 bf16.
// grid = (ceil(max_q / 16), nseq, nh); block = one wave.
//   S = Q K^T   : A = Q (lane: row l&15, dims 8(l>>4)+j+32s), B = K^T (lane: key l&15)
//                 acc: S[q = 4(l>>4)+i][key = l&15]
//   O += P V    : A = P (via LDS, lane: row l&15, keys 8(l>>4)+j),
//                 B = V (lane: keys 8(l>>4)+j, dim l&15 (+16n)) = one 16-B load of V^T
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) attn_prefill_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ q_start,
    const int* __restrict__ slot, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad, uint16_t* __restrict__ out,
    int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int tile = blockIdx.x, b = blockIdx.y, h = blockIdx.z;
  const int l = threadIdx.x;
  const int qbeg = cu_q[b];
  const int qlen = cu_q[b + 1] - qbeg;
  if (tile * 16 >= qlen) return;
  const int G = nh / nkv;
  const int kh = h / G;
  const int g4 = l >> 4, r16 = l & 15;
  const int qs = q_start[b];
  const int sl = slot[b];

  __shared__ __attribute__((aligned(16))) uint16_t P_lds[16 * 32];

  // Q fragments (two k-steps of 32 dims)
  bf16x8 qa[2];
  {
    const int row = tile * 16 + r16;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < qlen) v = *reinterpret_cast<const uint4*>(q + ((size_t)(qbeg + row) * nh + h) * D + 8 * g4 + 32 * s);
      qa[s] = __builtin_bit_cast(bf16x8, v);
    }
  }
  // own offsets of the 4 query rows this lane accumulates (S/O layout)
  int qoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) qoff[i] = qs + tile * 16 + 4 * g4 + i;
  const int last_row = min(tile * 16 + 15, qlen - 1);
  const int own_keys = qs + last_row + 1;  // own keys needed by this tile
  const int nkeys = P0pad + own_keys;

  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], lsum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -INFINITY; lsum[i] = 0.f; }

  for (int kt = 0; kt < nkeys; kt += 32) {
    const bool pre = kt < P0pad;  // tiles never straddle: P0pad % 32 == 0
    f32x4 sacc[2];
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;
      sacc[hs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint4 kv = make_uint4(0, 0, 0, 0);
        if (key < nkeys) {
          const uint16_t* krow = pre ? (kpre + (size_t)key * D) : (kself + (size_t)(key - P0pad) * D);
          kv = *reinterpret_cast<const uint4*>(krow + 8 * g4 + 32 * s);
        }
        sacc[hs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[s], __builtin_bit_cast(bf16x8, kv), sacc[hs], 0, 0, 0);
      }
    }
    // mask + scale, tile row max
    float sv[2][4];
    float tmax[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) tmax[i] = -INFINITY;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool ok;
        if (pre) ok = key < P0;
        else ok = (key - P0pad) <= qoff[i];
        const float v = ok ? sacc[hs][i] * scale_log2 : -INFINITY;
        sv[hs][i] = v;
        tmax[i] = fmaxf(tmax[i], v);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) tmax[i] = fmaxf(tmax[i], __shfl_xor(tmax[i], o2, WAVE));
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mn = fmaxf(m[i], tmax[i]);
      alpha[i] = (mn == -INFINITY) ? 1.f : exp2f(m[i] - mn);
      m[i] = mn;
      rs[i] = 0.f;
    }
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = (m[i] == -INFINITY) ? 0.f : exp2f(sv[hs][i] - m[i]);
        rs[i] += p;
        P_lds[(4 * g4 + i) * 32 + 16 * hs + r16] = f2bf(p);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs[i] += __shfl_xor(rs[i], o2, WAVE);
      lsum[i] = lsum[i] * alpha[i] + rs[i];
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha[i];
    }
    __syncthreads();
    const bf16x8 pa = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&P_lds[r16 * 32 + 8 * g4]));
    const int kk = kt + 8 * g4;  // first of this lane's 8 keys
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int d = 16 * n + r16;
      uint4 vv = make_uint4(0, 0, 0, 0);
      if (kk < nkeys) {
        // blocked V^T: 8 keys of dim d = one 16-byte chunk at ((key/8) * D + d) * 8
        const uint16_t* vrow = pre ? (vpre + ((size_t)(kk >> 3) * D + d) * 8)
                                   : (vself + ((size_t)((kk - P0pad) >> 3) * D + d) * 8);
        vv = *reinterpret_cast<const uint4*>(vrow);
      }
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, vv), o[n], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = tile * 16 + 4 * g4 + i;
    if (row >= qlen) continue;
    const float inv = lsum[i] > 0.f ? 1.f / lsum[i] : 0.f;
    uint16_t* orow = out + ((size_t)(qbeg + row) * nh + h) * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) orow[16 * n + r16] = f2bf(o[n][i] * inv);
  }
}

// ---------------------------------------------------------------------------
// Prefill attention, multi-tile (opt-in "multi"): same wave decomposition and layouts as
// attn_prefill_kernel, but the K and V tiles of NT key tiles (a whole short
// sequence: the shared prefix + ~54 own keys is 3 tiles) are loaded up front,
// all at once, and the softmax runs once per chunk of NT tiles instead of once per
// tile.  The per-tile kernel walks its tiles as a chain of dependent cold loads
// (K tile -> scores -> V tile -> next K tile): at the engine's prefill batches every
// wave is latency-bound and the kernel ran at ~0.5 TB/s (profiles/r03_bench_grid_hist.csv:
// 32 us per 8 k-token call).  Longer sequences take several chunks (online softmax
// across chunks).
// ---------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(64) attn_prefill_mt_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ q_start,
    const int* __restrict__ slot, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad, uint16_t* __restrict__ out,
    int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int tile = blockIdx.x, b = blockIdx.y, h = blockIdx.z;
  const int l = threadIdx.x;
  const int qbeg = cu_q[b];
  const int qlen = cu_q[b + 1] - qbeg;
  if (tile * 16 >= qlen) return;
  const int kh = h / (nh / nkv);
  const int g4 = l >> 4, r16 = l & 15;
  const int qs = q_start[b];
  const int sl = slot[b];

  __shared__ __attribute__((aligned(16))) uint16_t P_lds[NT][16 * 32];

  bf16x8 qa[2];
  {
    const int row = tile * 16 + r16;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < qlen) v = *reinterpret_cast<const uint4*>(q + ((size_t)(qbeg + row) * nh + h) * D + 8 * g4 + 32 * s);
      qa[s] = __builtin_bit_cast(bf16x8, v);
    }
  }
  int qoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) qoff[i] = qs + tile * 16 + 4 * g4 + i;
  const int last_row = min(tile * 16 + 15, qlen - 1);
  const int nkeys = P0pad + qs + last_row + 1;

  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], lsum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -INFINITY; lsum[i] = 0.f; }

  for (int kc = 0; kc < nkeys; kc += NT * 32) {
    // ---- every load of the chunk first (K: 4 x 16 B, V: 4 x 16 B per lane and tile)
    uint4 kv[NT][2][2], vv[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int kt = kc + 32 * t;
      const bool pre = kt < P0pad;  // tiles never straddle: P0pad % 32 == 0
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const int key = kt + 16 * hs + r16;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          kv[t][hs][s] = make_uint4(0, 0, 0, 0);
          if (key < nkeys) {
            const uint16_t* krow = pre ? (kpre + (size_t)key * D) : (kself + (size_t)(key - P0pad) * D);
            kv[t][hs][s] = *reinterpret_cast<const uint4*>(krow + 8 * g4 + 32 * s);
          }
        }
      }
      const int kk = kt + 8 * g4;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int d = 16 * n + r16;
        vv[t][n] = make_uint4(0, 0, 0, 0);
        if (kk < nkeys) {
          const uint16_t* vrow = pre ? (vpre + ((size_t)(kk >> 3) * D + d) * 8)
                                     : (vself + ((size_t)((kk - P0pad) >> 3) * D + d) * 8);
          vv[t][n] = *reinterpret_cast<const uint4*>(vrow);
        }
      }
    }
    // ---- scores of the chunk, masked and scaled; chunk row max
    float sv[NT][2][4];
    float cmax[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cmax[i] = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int kt = kc + 32 * t;
      const bool pre = kt < P0pad;
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[s], __builtin_bit_cast(bf16x8, kv[t][hs][s]), acc, 0, 0, 0);
        const int key = kt + 16 * hs + r16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = key < nkeys && (pre ? key < P0 : (key - P0pad) <= qoff[i]);
          const float v = ok ? acc[i] * scale_log2 : -INFINITY;
          sv[t][hs][i] = v;
          cmax[i] = fmaxf(cmax[i], v);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) cmax[i] = fmaxf(cmax[i], __shfl_xor(cmax[i], o2, WAVE));
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mn = fmaxf(m[i], cmax[i]);
      alpha[i] = (mn == -INFINITY) ? 1.f : exp2f(m[i] - mn);
      m[i] = mn;
      rs[i] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int hs = 0; hs < 2; ++hs)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = (m[i] == -INFINITY) ? 0.f : exp2f(sv[t][hs][i] - m[i]);
          rs[i] += p;
          P_lds[t][(4 * g4 + i) * 32 + 16 * hs + r16] = f2bf(p);
        }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs[i] += __shfl_xor(rs[i], o2, WAVE);
      lsum[i] = lsum[i] * alpha[i] + rs[i];
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha[i];
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 pa = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&P_lds[t][r16 * 32 + 8 * g4]));
#pragma unroll
      for (int n = 0; n < 4; ++n)
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, vv[t][n]), o[n], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = tile * 16 + 4 * g4 + i;
    if (row >= qlen) continue;
    const float inv = lsum[i] > 0.f ? 1.f / lsum[i] : 0.f;
    uint16_t* orow = out + ((size_t)(qbeg + row) * nh + h) * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) orow[16 * n + r16] = f2bf(o[n][i] * inv);
  }
}

// ---------------------------------------------------------------------------
// Prefill attention, GQA-shared (K/V loaded once per GQA group): one wave per (16-query tile,
// sequence, KV head) computes all G query heads of the group from ONE load of
// each K/V tile (the per-head kernel above re-reads K/V G times), and the K tile
// of step kt+1 and the V tile of step kt are in flight while the scores of step
// kt are computed (register double buffering: the per-head kernel waited on a
// cold load at every step).  Same masking, rounding and online softmax as the
// per-head kernel; numerics are checked against the same fp32 reference.
// KS > 1 (key split): KS waves per block deal the 32-key tiles round-robin, each
// with its own online-softmax state, merged by wave 0 through LDS — KS times the
// waves for the same bytes (the kernel runs at 2 waves per SIMD: 194 VGPRs).
// ---------------------------------------------------------------------------
template <int G, int KS>
__global__ void __launch_bounds__(64 * KS) attn_prefill_gqa_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ q_start,
    const int* __restrict__ slot, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad, uint16_t* __restrict__ out,
    int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int tile = blockIdx.x, b = blockIdx.y, kh = blockIdx.z;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qbeg = cu_q[b];
  const int qlen = cu_q[b + 1] - qbeg;
  if (tile * 16 >= qlen) return;  // block-uniform
  const int g4 = l >> 4, r16 = l & 15;
  const int qs = q_start[b];
  const int sl = slot[b];

  // ONE __shared__ array: per-wave P tiles, then (KS > 1) the merge area
  constexpr int PSZ = G * 16 * 32;                                 // bf16 elements per wave
  constexpr int RED = KS > 1 ? KS * 64 * G * 24 * 2 : 0;           // fp32 state as bf16-sized units
  __shared__ __attribute__((aligned(16))) uint16_t smem_pf[(KS * PSZ > RED ? KS * PSZ : RED)];
  uint16_t (*P_lds)[16 * 32] = reinterpret_cast<uint16_t (*)[16 * 32]>(smem_pf + w * PSZ);

  bf16x8 qa[G][2];
  {
    const int row = tile * 16 + r16;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (row < qlen)
          v = *reinterpret_cast<const uint4*>(q + ((size_t)(qbeg + row) * nh + kh * G + g) * D + 8 * g4 + 32 * s);
        qa[g][s] = __builtin_bit_cast(bf16x8, v);
      }
  }
  int qoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) qoff[i] = qs + tile * 16 + 4 * g4 + i;
  const int last_row = min(tile * 16 + 15, qlen - 1);
  const int nkeys = P0pad + qs + last_row + 1;

  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  auto load_k = [&](int kt, uint4 (&kv)[2][2]) {
    const bool pre = kt < P0pad;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        kv[hs][s] = make_uint4(0, 0, 0, 0);
        if (key < nkeys) {
          const uint16_t* krow = pre ? (kpre + (size_t)key * D) : (kself + (size_t)(key - P0pad) * D);
          kv[hs][s] = *reinterpret_cast<const uint4*>(krow + 8 * g4 + 32 * s);
        }
      }
    }
  };

  f32x4 o[G][4];
  float m[G][4], lsum[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      m[g][i] = -INFINITY;
      lsum[g][i] = 0.f;
    }

  uint4 kc[2][2];
  load_k(32 * w, kc);
  for (int kt = 32 * w; kt < nkeys; kt += 32 * KS) {
    const bool pre = kt < P0pad;  // tiles never straddle: P0pad % 32 == 0
    // V tile of this step and K tile of the next step: in flight during the scores
    uint4 vv[4];
    const int kk = kt + 8 * g4;  // first of this lane's 8 keys
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int d = 16 * n + r16;
      vv[n] = make_uint4(0, 0, 0, 0);
      if (kk < nkeys) {
        const uint16_t* vrow = pre ? (vpre + ((size_t)(kk >> 3) * D + d) * 8)
                                   : (vself + ((size_t)((kk - P0pad) >> 3) * D + d) * 8);
        vv[n] = *reinterpret_cast<const uint4*>(vrow);
      }
    }
    uint4 kn[2][2];
    load_k(kt + 32 * KS, kn);  // guarded by key < nkeys: past the end it loads nothing

    bool okm[2][4];
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) okm[hs][i] = pre ? (key < P0) : ((key - P0pad) <= qoff[i]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4 sacc[2];
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        sacc[hs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s)
          sacc[hs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[g][s], __builtin_bit_cast(bf16x8, kc[hs][s]),
                                                             sacc[hs], 0, 0, 0);
      }
      float sv[2][4], tmax[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) tmax[i] = -INFINITY;
#pragma unroll
      for (int hs = 0; hs < 2; ++hs)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = okm[hs][i] ? sacc[hs][i] * scale_log2 : -INFINITY;
          sv[hs][i] = v;
          tmax[i] = fmaxf(tmax[i], v);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o2 = 8; o2 > 0; o2 >>= 1) tmax[i] = fmaxf(tmax[i], __shfl_xor(tmax[i], o2, WAVE));
      float alpha[4], rs[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float mn = fmaxf(m[g][i], tmax[i]);
        alpha[i] = (mn == -INFINITY) ? 1.f : exp2f(m[g][i] - mn);
        m[g][i] = mn;
        rs[i] = 0.f;
      }
#pragma unroll
      for (int hs = 0; hs < 2; ++hs)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = (m[g][i] == -INFINITY) ? 0.f : exp2f(sv[hs][i] - m[g][i]);
          rs[i] += p;
          P_lds[g][(4 * g4 + i) * 32 + 16 * hs + r16] = f2bf(p);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o2 = 8; o2 > 0; o2 >>= 1) rs[i] += __shfl_xor(rs[i], o2, WAVE);
        lsum[g][i] = lsum[g][i] * alpha[i] + rs[i];
      }
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[g][n][i] *= alpha[i];
    }
    // P tiles are private to the wave (waves of a KS block run different trip
    // counts, so no block barrier here): LDS ops of one wave complete in order
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bf16x8 pa = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&P_lds[g][r16 * 32 + 8 * g4]));
#pragma unroll
      for (int n = 0; n < 4; ++n)
        o[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, vv[n]), o[g][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR: next step rewrites P_lds
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int hs = 0; hs < 2; ++hs)
#pragma unroll
      for (int s = 0; s < 2; ++s) kc[hs][s] = kn[hs][s];
  }
  if constexpr (KS > 1) {
    // merge the KS partial softmax states (per lane: head g, rows 4·g4 + i)
    float* red = reinterpret_cast<float*>(smem_pf);
    __syncthreads();  // every wave is done with its P tile
    float* mine = red + ((size_t)w * 64 + l) * (G * 24);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int n = 0; n < 4; ++n) mine[g * 24 + n * 4 + i] = o[g][n][i];
        mine[g * 24 + 16 + i] = m[g][i];
        mine[g * 24 + 20 + i] = lsum[g][i];
      }
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float M = -INFINITY;
#pragma unroll
        for (int v = 0; v < KS; ++v) M = fmaxf(M, red[((size_t)v * 64 + l) * (G * 24) + g * 24 + 16 + i]);
        float L = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < KS; ++v) {
          const float* src = red + ((size_t)v * 64 + l) * (G * 24) + g * 24;
          const float mv = src[16 + i];
          if (mv == -INFINITY) continue;  // no valid key in this wave's tiles
          const float f = exp2f(mv - M);
          L += f * src[20 + i];
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[n] += f * src[n * 4 + i];
        }
        m[g][i] = M;
        lsum[g][i] = L;
#pragma unroll
        for (int n = 0; n < 4; ++n) o[g][n][i] = acc[n];
      }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = tile * 16 + 4 * g4 + i;
      if (row >= qlen) continue;
      const float inv = lsum[g][i] > 0.f ? 1.f / lsum[g][i] : 0.f;
      uint16_t* orow = out + ((size_t)(qbeg + row) * nh + kh * G + g) * D;
#pragma unroll
      for (int n = 0; n < 4; ++n) orow[16 * n + r16] = f2bf(o[g][n][i] * inv);
    }
}

// ---------------------------------------------------------------------------
// Decode attention: one query token per sequence; grid = (B, nkv), ONE wave per
// (sequence, kv head) computing its G = nh/nkv query heads, so every K/V byte is
// read once per GQA group. Finished rows exit immediately (done[b] != 0).
// Score index space: [prefix 0..P0pad) ++ [own 0..own8) with padding p = 0.
//   phase 1  8 lanes per key row (16 B each), 16 keys in flight per iteration
//   phase 2  softmax per head (lane-strided over the scores in LDS)
//   phase 3  lane = dim; blocked V^T gives 8 keys of the lane's dim per 16-B
//            load, the wave reading 1 KiB contiguously per chunk
// ---------------------------------------------------------------------------
#define DEC_MAXCTX 512
#define DEC_MAXG 4
__global__ void __launch_bounds__(64) attn_decode_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int b = blockIdx.x, kh = blockIdx.y;
  const int lane = threadIdx.x;
  if (done != nullptr && done[b]) return;
  const int G = nh / nkv;
  const int own = pos[b] + 1;              // own keys 0..pos inclusive
  const int own8 = (own + 7) & ~7;
  const int sl = slot[b];
  const int ns = P0pad + own8;             // padded score count
  __shared__ __attribute__((aligned(16))) float sc[DEC_MAXG][DEC_MAXCTX];

  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  // phase 1 ------------------------------------------------------------------
  const int dc = lane & 7, kr = lane >> 3;
  float qf[DEC_MAXG][8];
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g) {
    if (g < G) unpack8(*reinterpret_cast<const uint4*>(q + ((size_t)b * nh + kh * G + g) * D + 8 * dc), qf[g]);
  }
  // Latency, not bandwidth, bounds this kernel (~140 keys per wave): every
  // round issues DEC_UNR independent 16-B loads per lane before consuming any.
  constexpr int DEC_UNR = 4;
  auto score_rows = [&](const uint16_t* base, int nkeys, int sbase) {
    for (int k0 = 0; k0 < nkeys; k0 += 8 * DEC_UNR) {
      uint4 kv[DEC_UNR];
#pragma unroll
      for (int u = 0; u < DEC_UNR; ++u) {
        const int k = k0 + 8 * u + kr;
        kv[u] = (k < nkeys) ? *reinterpret_cast<const uint4*>(base + (size_t)k * D + 8 * dc) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < DEC_UNR; ++u) {
        const int k = k0 + 8 * u + kr;
        float f[8];
        unpack8(kv[u], f);
#pragma unroll
        for (int g = 0; g < DEC_MAXG; ++g) {
          if (g < G) {
            float sa = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) sa += qf[g][j] * f[j];
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) sa += __shfl_xor(sa, o, WAVE);
            if (dc == 0 && k < nkeys) sc[g][sbase + k] = sa * scale_log2;
          }
        }
      }
    }
  };
  score_rows(kpre, P0, 0);
  score_rows(kself, own, P0pad);
  __syncthreads();
  // phase 2 ------------------------------------------------------------------
  float inv_sum[DEC_MAXG];
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g) {
    inv_sum[g] = 0.f;
    if (g >= G) continue;
    float mx = -INFINITY;
    for (int i = lane; i < ns; i += WAVE) {
      const bool ok = (i < P0) || (i >= P0pad && i - P0pad < own);
      if (ok) mx = fmaxf(mx, sc[g][i]);
    }
    mx = wave_max(mx);
    float sm = 0.f;
    for (int i = lane; i < ns; i += WAVE) {
      const bool ok = (i < P0) || (i >= P0pad && i - P0pad < own);
      const float p = ok ? exp2f(sc[g][i] - mx) : 0.f;
      sc[g][i] = p;
      sm += p;
    }
    inv_sum[g] = 1.f / wave_sum(sm);
  }
  __syncthreads();
  // phase 3 ------------------------------------------------------------------
  const int d = lane;
  float acc[DEC_MAXG];
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g) acc[g] = 0.f;
  auto pv_chunks = [&](const uint16_t* vbase, int nchunks, int sbase) {
    for (int c0 = 0; c0 < nchunks; c0 += DEC_UNR) {
      uint4 vv[DEC_UNR];
#pragma unroll
      for (int u = 0; u < DEC_UNR; ++u)
        vv[u] = (c0 + u < nchunks) ? *reinterpret_cast<const uint4*>(vbase + ((size_t)(c0 + u) * D + d) * 8)
                                   : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < DEC_UNR; ++u) {
        const int c = c0 + u;
        if (c >= nchunks) break;
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int g = 0; g < DEC_MAXG; ++g) {
          if (g < G) {
            const float4 p0 = *reinterpret_cast<const float4*>(&sc[g][sbase + 8 * c]);
            const float4 p1 = *reinterpret_cast<const float4*>(&sc[g][sbase + 8 * c + 4]);
            acc[g] += p0.x * vf[0] + p0.y * vf[1] + p0.z * vf[2] + p0.w * vf[3] +
                      p1.x * vf[4] + p1.y * vf[5] + p1.z * vf[6] + p1.w * vf[7];
          }
        }
      }
    }
  };
  pv_chunks(vpre, P0pad >> 3, 0);
  pv_chunks(vself, own8 >> 3, P0pad);
#pragma unroll
  for (int g = 0; g < DEC_MAXG; ++g)
    if (g < G) out[((size_t)b * nh + kh * G + g) * D + d] = f2bf(acc[g] * inv_sum[g]);
}

// ---------------------------------------------------------------------------
// MFMA decode attention (the production decode path). grid = (B, nkv), one wave.
// The G query heads that share a KV head are the rows of one 16-row MFMA tile
// (rows >= G carry q = 0 and are never stored), so S = Q·K^T and O += P·V are
// two and four mfma_f32_16x16x32_bf16 per 32-key tile — the arithmetic is free
// and the kernel reduces to streaming K/V once per GQA group. Tile t+1's K/V
// (8 × 16-B loads per lane) is issued before tile t is consumed, and finished
// rows exit at once. Layouts and the prefix/own key spaces as in prefill.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) attn_decode_mfma_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int b = blockIdx.x, kh = blockIdx.y, l = threadIdx.x;
  if (done != nullptr && done[b]) return;
  const int G = nh / nkv;
  const int g4 = l >> 4, r16 = l & 15;
  const int own = pos[b] + 1;
  const int sl = slot[b];
  __shared__ __attribute__((aligned(16))) uint16_t P_lds[16 * 32];

  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  bf16x8 qa[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r16 < G) v = *reinterpret_cast<const uint4*>(q + ((size_t)b * nh + kh * G + r16) * D + 8 * g4 + 32 * s);
    qa[s] = __builtin_bit_cast(bf16x8, v);
  }
  const int npre = P0pad >> 5;
  const int ntiles = npre + ((own + 31) >> 5);

  // Tile loads are UNconditional: every key index of a tile is < roundup(own, 32)
  // <= Lmax (resp. P0pad), inside the slot's rows, and cache rows past the valid
  // length hold finite stale values (the caches are zero-initialised and only
  // ever receive finite K/V), which the score mask turns into p = 0.  A per-lane
  // guarded load would compile to a branch + vmcnt(0) and serialise the prefetch.
  auto load_tile = [&](int t, uint4 (&kv)[2][2], uint4 (&vv)[4]) {
    const bool pre = t < npre;
    const int kt = pre ? t * 32 : (t - npre) * 32;
    const uint16_t* kb = pre ? kpre : kself;
    const uint16_t* vb = pre ? vpre : vself;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;
#pragma unroll
      for (int s = 0; s < 2; ++s) kv[hs][s] = *reinterpret_cast<const uint4*>(kb + (size_t)key * D + 8 * g4 + 32 * s);
    }
    const int kk = kt + 8 * g4;
#pragma unroll
    for (int n = 0; n < 4; ++n)
      vv[n] = *reinterpret_cast<const uint4*>(vb + ((size_t)(kk >> 3) * D + 16 * n + r16) * 8);
  };

  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], lsum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -INFINITY; lsum[i] = 0.f; }

  // Ping-pong K/V register sets, loop unrolled by 2 (a `cur = next` copy at the end
  // of an iteration makes the compiler wait for the prefetch right there).  An odd
  // tile count is padded with one fully-masked tile (its keys are >= own).
  auto process = [&](int t, const uint4 (&kc)[2][2], const uint4 (&vc)[4]) {
    const bool pre = t < npre;
    const int kt = pre ? t * 32 : (t - npre) * 32;
    const int nval = pre ? P0 : own;
    f32x4 sacc[2];
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      sacc[hs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s)
        sacc[hs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[s], __builtin_bit_cast(bf16x8, kc[hs][s]), sacc[hs],
                                                           0, 0, 0);
    }
    float sv[2][4], tmax[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) tmax[i] = -INFINITY;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const bool ok = (kt + 16 * hs + r16) < nval;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = ok ? sacc[hs][i] * scale_log2 : -INFINITY;
        sv[hs][i] = v;
        tmax[i] = fmaxf(tmax[i], v);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) tmax[i] = fmaxf(tmax[i], __shfl_xor(tmax[i], o2, WAVE));
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mn = fmaxf(m[i], tmax[i]);
      alpha[i] = (mn == -INFINITY) ? 1.f : exp2f(m[i] - mn);
      m[i] = mn;
      rs[i] = 0.f;
    }
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = (m[i] == -INFINITY) ? 0.f : exp2f(sv[hs][i] - m[i]);
        rs[i] += p;
        P_lds[(4 * g4 + i) * 32 + 16 * hs + r16] = f2bf(p);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs[i] += __shfl_xor(rs[i], o2, WAVE);
      lsum[i] = lsum[i] * alpha[i] + rs[i];
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha[i];
    }
    // one-wave block: LDS ops of a wave execute in order, so the P transpose needs
    // no barrier (a __syncthreads() would also drain the K/V prefetch: vmcnt(0))
    asm volatile("" ::: "memory");
    const bf16x8 pa = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&P_lds[r16 * 32 + 8 * g4]));
#pragma unroll
    for (int n = 0; n < 4; ++n)
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, vc[n]), o[n], 0, 0, 0);
    asm volatile("" ::: "memory");
  };
  uint4 ka[2][2], va[4], kb2[2][2], vb2[4];
  load_tile(0, ka, va);
  const int nt2 = (ntiles + 1) & ~1;
  for (int t = 0; t < nt2; t += 2) {
    load_tile(min(t + 1, ntiles - 1), kb2, vb2);
    process(t, ka, va);
    load_tile(min(t + 2, ntiles - 1), ka, va);
    process(t + 1, kb2, vb2);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * g4 + i;
    if (row >= G) continue;
    const float inv = 1.f / lsum[i];
    uint16_t* orow = out + ((size_t)b * nh + kh * G + row) * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) orow[16 * n + r16] = f2bf(o[n][i] * inv);
  }
}

// ---------------------------------------------------------------------------
// Transposed MFMA decode attention (production path).  grid = (B, nkv), one wave.
//
//   S^T = K · Q^T   (A = 16 keys × 32 dims from the K cache, B = Q^T: the G query
//                    heads of the GQA group are the 16 columns, cols >= G are 0)
//   O^T = V^T · P^T (A = 16 dims × 32 keys straight from the blocked V^T cache,
//                    B = P^T, which is exactly the S^T accumulator after exp2)
//
// Each lane owns ONE query column (q = lane & 15) and 8 of the tile's 32 keys
// (4·(lane>>4)+i and 16+4·(lane>>4)+i), so the online-softmax max/sum are 7
// in-lane ops + 2 cross-lane shuffles, the rescale of O^T is lane-local, and P
// never leaves registers: its k-order (the MFMA's 8·(lane>>4)+j) is defined as
// that same key set, and the V^T fragment is read in the same order (two 8-byte
// pieces of the [key/8][D][8] blocks).  vs attn_decode_mfma_kernel: no LDS, 4
// instead of 32 shuffles per 32-key tile.  K/V tiles are double-buffered in
// registers (ping-pong, unrolled by 2) and loaded unconditionally (all key
// indices < roundup(own, 32) <= Lmax; requires Lmax % 32 == 0).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) attn_decode_st_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int b = blockIdx.x, kh = blockIdx.y, l = threadIdx.x;
  if (done != nullptr && done[b]) return;
  const int G = nh / nkv;
  const int g4 = l >> 4, r16 = l & 15;
  const int own = pos[b] + 1;
  const int sl = slot[b];
  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;

  // B operand Q^T: lane holds Q[q = r16][dims 8·g4 + j (+32 s)]
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r16 < G) v = *reinterpret_cast<const uint4*>(q + ((size_t)b * nh + kh * G + r16) * D + 8 * g4 + 32 * s2);
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  const int npre = P0pad >> 5;
  const int ntiles = npre + ((own + 31) >> 5);

  auto load_tile = [&](int t, uint4 (&kv)[2][2], uint4 (&vv)[4]) {
    const bool pre = t < npre;
    const int kt = pre ? t * 32 : (t - npre) * 32;
    const uint16_t* kb = pre ? kpre : kself;
    const uint16_t* vb = pre ? vpre : vself;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      const int key = kt + 16 * hs + r16;  // A operand row
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        kv[hs][s2] = *reinterpret_cast<const uint4*>(kb + (size_t)key * D + 8 * g4 + 32 * s2);
    }
    // V^T A operand: row = dim 16n + r16, k-slots j<4 -> keys kt+4g4+j, j>=4 -> kt+16+4g4+j-4
    const int k_lo = kt + 4 * g4, k_hi = kt + 16 + 4 * g4;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int dim = 16 * n + r16;
      const uint2 lo = *reinterpret_cast<const uint2*>(vb + ((size_t)(k_lo >> 3) * D + dim) * 8 + (k_lo & 7));
      const uint2 hi = *reinterpret_cast<const uint2*>(vb + ((size_t)(k_hi >> 3) * D + dim) * 8 + (k_hi & 7));
      vv[n] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  };

  f32x4 o[4];  // O^T: lane holds O[q = r16][dim 16n + 4g4 + i]
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;

  auto process = [&](int t, const uint4 (&kc)[2][2], const uint4 (&vc)[4]) {
    const bool pre = t < npre;
    const int kt = pre ? t * 32 : (t - npre) * 32;
    const int nval = pre ? P0 : own;
    f32x4 st[2];
#pragma unroll
    for (int hs = 0; hs < 2; ++hs) {
      st[hs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        st[hs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kc[hs][s2]), qb[s2], st[hs], 0, 0,
                                                         0);
    }
    // lane: st[hs][i] = score(query r16, key kt + 16hs + 4g4 + i)
    float sv[2][4], tmax = -INFINITY;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = (kt + 16 * hs + 4 * g4 + i) < nval;
        sv[hs][i] = ok ? st[hs][i] * scale_log2 : -INFINITY;
        tmax = fmaxf(tmax, sv[hs][i]);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, WAVE));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, WAVE));
    const float mn = fmaxf(m, tmax);
    const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
    m = mn;
    float p[8], rs = 0.f;
#pragma unroll
    for (int hs = 0; hs < 2; ++hs)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = (mn == -INFINITY) ? 0.f : exp2f(sv[hs][i] - mn);
        p[4 * hs + i] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 16, WAVE);
    rs += __shfl_xor(rs, 32, WAVE);
    lsum = lsum * alpha + rs;
    uint4 pw;
    pw.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
    pw.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
    pw.z = (uint32_t)f2bf(p[4]) | ((uint32_t)f2bf(p[5]) << 16);
    pw.w = (uint32_t)f2bf(p[6]) | ((uint32_t)f2bf(p[7]) << 16);
    const bf16x8 pb = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha;
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vc[n]), pb, o[n], 0, 0, 0);
    }
  };

  uint4 ka[2][2], va[4], kb2[2][2], vb2[4];
  load_tile(0, ka, va);
  const int nt2 = (ntiles + 1) & ~1;  // odd counts: one fully-masked pad tile (keys >= own)
  for (int t = 0; t < nt2; t += 2) {
    load_tile(min(t + 1, ntiles - 1), kb2, vb2);
    process(t, ka, va);
    load_tile(min(t + 2, ntiles - 1), ka, va);
    process(t + 1, kb2, vb2);
  }
  if (r16 < G) {
    const float inv = 1.f / lsum;
    uint16_t* orow = out + ((size_t)b * nh + kh * G + r16) * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[n][0] * inv) | ((uint32_t)f2bf(o[n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[n][2] * inv) | ((uint32_t)f2bf(o[n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Cascade decode attention = shared-prefix pass + own-key pass (production).
//
// Every decode row attends to the same P0 system-prompt keys.  Reading them once
// per (row, kv head) made the L2 traffic of the prefix larger than the HBM
// traffic of the rows' own keys.  Pass 1 (attn_prefix_kernel) packs 16 query
// rows of ANY sequences of one kv head into the 16 MFMA columns, so the prefix
// K/V are read once per 16 rows, and writes the normalised prefix output O_pre
// (fp32) and its log-sum-exp (log2 domain).  Pass 2 (attn_own_kernel) starts its
// online softmax from the exact state (m = lse, l = 1, o = O_pre) and streams
// only the row's own keys.  Both use the transposed formulation of
// attn_decode_st_kernel (S^T = K·Q^T, O^T = V^T·P^T; one query per lane column).
// ---------------------------------------------------------------------------
// `full` = false: only the first 16 keys of the tile can be valid (the sequence
// ends in the first half) -> the second half's K rows / V^T pieces are not read
// (zeros; their scores are masked), i.e. 16-key granularity on the last tile.
__device__ __forceinline__ void st_load_tile(const uint16_t* __restrict__ kb, const uint16_t* __restrict__ vb, int kt,
                                             int g4, int r16, bool full, uint4 (&kv)[2][2], uint4 (&vv)[4]) {
  constexpr int D = 64;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    kv[0][s2] = *reinterpret_cast<const uint4*>(kb + (size_t)(kt + r16) * D + 8 * g4 + 32 * s2);
  const int k_lo = kt + 4 * g4, k_hi = kt + 16 + 4 * g4;
  uint2 lo[4], hi[4];
#pragma unroll
  for (int n = 0; n < 4; ++n)
    lo[n] = *reinterpret_cast<const uint2*>(vb + ((size_t)(k_lo >> 3) * D + 16 * n + r16) * 8 + (k_lo & 7));
  if (full) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      kv[1][s2] = *reinterpret_cast<const uint4*>(kb + (size_t)(kt + 16 + r16) * D + 8 * g4 + 32 * s2);
#pragma unroll
    for (int n = 0; n < 4; ++n)
      hi[n] = *reinterpret_cast<const uint2*>(vb + ((size_t)(k_hi >> 3) * D + 16 * n + r16) * 8 + (k_hi & 7));
  } else {
    kv[1][0] = kv[1][1] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int n = 0; n < 4; ++n) hi[n] = make_uint2(0, 0);
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) vv[n] = make_uint4(lo[n].x, lo[n].y, hi[n].x, hi[n].y);
}

// One 32-key tile of the transposed online softmax (state per lane = its query).
__device__ __forceinline__ void st_tile(const bf16x8 (&qb)[2], const uint4 (&kc)[2][2], const uint4 (&vc)[4],
                                        int kt, int nval, int g4, float scale_log2, float& m, float& lsum,
                                        f32x4 (&o)[4], bool col_ok = true) {
  f32x4 st[2];
#pragma unroll
  for (int hs = 0; hs < 2; ++hs) {
    st[hs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      st[hs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kc[hs][s2]), qb[s2], st[hs], 0, 0, 0);
  }
  float sv[2][4], tmax = -INFINITY;
#pragma unroll
  for (int hs = 0; hs < 2; ++hs)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // col_ok = false: this lane's query column does not own these keys (grouped
      // kernel) -> -inf scores leave its softmax state (m, l, o) untouched
      const bool ok = col_ok && (kt + 16 * hs + 4 * g4 + i) < nval;
      sv[hs][i] = ok ? st[hs][i] * scale_log2 : -INFINITY;
      tmax = fmaxf(tmax, sv[hs][i]);
    }
  tmax = fmaxf(tmax, __shfl_xor(tmax, 16, WAVE));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32, WAVE));
  const float mn = fmaxf(m, tmax);
  const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
  m = mn;
  float p[8], rs = 0.f;
#pragma unroll
  for (int hs = 0; hs < 2; ++hs)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = (mn == -INFINITY) ? 0.f : exp2f(sv[hs][i] - mn);
      p[4 * hs + i] = e;
      rs += e;
    }
  rs += __shfl_xor(rs, 16, WAVE);
  rs += __shfl_xor(rs, 32, WAVE);
  lsum = lsum * alpha + rs;
  uint4 pw;
  pw.x = (uint32_t)f2bf(p[0]) | ((uint32_t)f2bf(p[1]) << 16);
  pw.y = (uint32_t)f2bf(p[2]) | ((uint32_t)f2bf(p[3]) << 16);
  pw.z = (uint32_t)f2bf(p[4]) | ((uint32_t)f2bf(p[5]) << 16);
  pw.w = (uint32_t)f2bf(p[6]) | ((uint32_t)f2bf(p[7]) << 16);
  const bf16x8 pb = __builtin_bit_cast(bf16x8, pw);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[n][i] *= alpha;
    o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vc[n]), pb, o[n], 0, 0, 0);
  }
}

// Pass 1: grid = (ceil(B*G / 16), nkv), one wave; column c <-> query row
// r = 16·blockIdx.x + c of kv head kh, i.e. sequence r / G, head kh·G + r % G.
// Merged key stream (g_attn_merge): the shared prefix's P0 keys and the slot's own keys
// form ONE sequence of 32-key tiles -- key k < P0 is prefix row k, key k >= P0 own key
// k - P0 -- instead of a prefix tile padded to 32 followed by own tiles starting at 0.
// A row with P0 + own keys then walks ceil((P0 + own) / 32) tiles, not
// 1 + ceil(own / 32) (P0 = 20: 0.6 tiles fewer per row on average).  P0 % 4 == 0 keeps
// every lane's 4-key V^T piece inside one of the two sources.  Rows past the slot's
// Lmax (the last tile of a full slot) are clamped; their scores are masked.
// Only keys below nk are fetched (per lane: a K row is one 128-B line pair, a 4-key V^T
// piece shares 64-B lines with its 8-key block): the tail tile of a row reads its valid
// keys, not 16 or 32 — the verify kernel is HBM-bound, so bytes are its time.
__device__ __forceinline__ void st_load_tile_m(const uint16_t* __restrict__ kpre, const uint16_t* __restrict__ vpre,
                                               const uint16_t* __restrict__ kself,
                                               const uint16_t* __restrict__ vself, int P0, int Lmax, int kt, int g4,
                                               int r16, int nk, uint4 (&kv)[2][2], uint4 (&vv)[4]) {
  constexpr int D = 64;
  const int ka = kt + r16, kb = kt + 16 + r16;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  const uint16_t* kra = ka < P0 ? kpre + (size_t)ka * D : kself + (size_t)min(ka - P0, Lmax - 1) * D;
  kv[0][0] = kv[0][1] = z4;
  if (ka < nk) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) kv[0][s2] = *reinterpret_cast<const uint4*>(kra + 8 * g4 + 32 * s2);
  }
  const int k_lo = kt + 4 * g4, k_hi = kt + 16 + 4 * g4;
  const bool plo = k_lo < P0;
  const uint16_t* vlo = plo ? vpre : vself;
  const int kl = plo ? k_lo : min(k_lo - P0, Lmax - 4);
  uint2 lo[4], hi[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) lo[n] = make_uint2(0, 0);
  if (k_lo < nk) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
      lo[n] = *reinterpret_cast<const uint2*>(vlo + ((size_t)(kl >> 3) * D + 16 * n + r16) * 8 + (kl & 7));
  }
  if (kt + 16 < nk) {
    const uint16_t* krb = kb < P0 ? kpre + (size_t)kb * D : kself + (size_t)min(kb - P0, Lmax - 1) * D;
    kv[1][0] = kv[1][1] = z4;
    if (kb < nk) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) kv[1][s2] = *reinterpret_cast<const uint4*>(krb + 8 * g4 + 32 * s2);
    }
    const bool phi = k_hi < P0;
    const uint16_t* vhi = phi ? vpre : vself;
    const int kh2 = phi ? k_hi : min(k_hi - P0, Lmax - 4);
#pragma unroll
    for (int n = 0; n < 4; ++n) hi[n] = make_uint2(0, 0);
    if (k_hi < nk) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
        hi[n] = *reinterpret_cast<const uint2*>(vhi + ((size_t)(kh2 >> 3) * D + 16 * n + r16) * 8 + (kh2 & 7));
    }
  } else {
    kv[1][0] = kv[1][1] = z4;
#pragma unroll
    for (int n = 0; n < 4; ++n) hi[n] = make_uint2(0, 0);
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) vv[n] = make_uint4(lo[n].x, lo[n].y, hi[n].x, hi[n].y);
}

__global__ void __launch_bounds__(64) attn_prefix_kernel(const uint16_t* __restrict__ q,
                                                         const uint16_t* __restrict__ pk,
                                                         const uint16_t* __restrict__ pvt, int P0, int P0pad,
                                                         float* __restrict__ pre_o, float* __restrict__ pre_lse,
                                                         int B, int nh, int nkv, float scale_log2) {
  constexpr int D = 64;
  const int kh = blockIdx.y, l = threadIdx.x, g4 = l >> 4, r16 = l & 15;
  const int G = nh / nkv;
  const int r = blockIdx.x * 16 + r16;
  const bool valid = r < B * G;
  const size_t qrow = valid ? (size_t)(r / G) * nh + kh * G + (r % G) : 0;
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const uint4 v = *reinterpret_cast<const uint4*>(q + qrow * D + 8 * g4 + 32 * s2);  // row 0 when !valid
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  const uint16_t* kb = pk + (size_t)kh * P0pad * D;
  const uint16_t* vb = pvt + (size_t)kh * D * P0pad;
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  for (int kt = 0; kt < P0pad; kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kb, vb, kt, g4, r16, kt + 16 < P0, kc, vc);
    st_tile(qb, kc, vc, kt, P0, g4, scale_log2, m, lsum, o);
  }
  if (valid) {
    const float inv = 1.f / lsum;
    float* orow = pre_o + qrow * D;
#pragma unroll
    for (int n = 0; n < 4; ++n)
      *reinterpret_cast<float4*>(orow + 16 * n + 4 * g4) =
          make_float4(o[n][0] * inv, o[n][1] * inv, o[n][2] * inv, o[n][3] * inv);
    if (g4 == 0) pre_lse[qrow] = m + __log2f(lsum);
  }
}

// Pass 2: grid = (B, nkv), one wave; the row's own keys, seeded with the prefix state.
__global__ void __launch_bounds__(64) attn_own_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const float* __restrict__ pre_o, const float* __restrict__ pre_lse, uint16_t* __restrict__ out, int nh, int nkv,
    int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int b = blockIdx.x, kh = blockIdx.y, l = threadIdx.x;
  if (done != nullptr && done[b]) return;
  const int G = nh / nkv;
  const int g4 = l >> 4, r16 = l & 15;
  const int own = pos[b] + 1;
  const int sl = slot[b];
  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const size_t qrow = (size_t)b * nh + kh * G + (r16 < G ? r16 : 0);
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 v = *reinterpret_cast<const uint4*>(q + qrow * D + 8 * g4 + 32 * s2);
    if (r16 >= G) v = make_uint4(0, 0, 0, 0);
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 o[4];
  float m = -INFINITY, lsum = 0.f;
  if (pre_o != nullptr && r16 < G) {  // exact prefix state: sum of 2^(s - lse) = 1
    m = pre_lse[qrow];
    lsum = 1.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const float4 v = *reinterpret_cast<const float4*>(pre_o + qrow * D + 16 * n + 4 * g4);
      o[n] = (f32x4){v.x, v.y, v.z, v.w};
    }
  } else {
#pragma unroll
    for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // plain loop: with ~4 resident waves per SIMD the load latency is covered by
  // the other waves (a register ping-pong measured no faster and costs VGPRs)
  for (int kt = 0; kt < own; kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kself, vself, kt, g4, r16, kt + 16 < own, kc, vc);
    st_tile(qb, kc, vc, kt, own, g4, scale_log2, m, lsum, o);
  }
  if (r16 < G) {
    const float inv = 1.f / lsum;
    uint16_t* orow = out + qrow * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[n][0] * inv) | ((uint32_t)f2bf(o[n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[n][2] * inv) | ((uint32_t)f2bf(o[n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Grouped decode attention (production): one wave = SPW = 16 / G sequences of one
// kv head.  MFMA column c <-> (sequence c / G, query head c % G).  The shared
// prefix tiles are multiplied once for all 16 columns (15 useful at G = 3); then
// each sequence's own tiles run with a per-column mask, so the other sequences'
// softmax states are untouched.  vs the cascade pair: no fp32 scratch round
// trip, one launch, prefix K/V read once per SPW sequences.
// grid = (ceil(B / SPW), nkv), one wave.
// ---------------------------------------------------------------------------
// HOIST: lanes 0..SPW-1 load their sequence's (done, pos, slot) at kernel entry, so
// the loads overlap the prefix pass and each own-key loop reads them with
// v_readlane instead of a dependent scalar load before its first K/V tile.
template <int MINW, bool HOIST = false>  // MINW: min waves per SIMD (1 = compiler's choice, 6 = VGPR cap 80)
__global__ void __launch_bounds__(64, MINW) attn_grouped_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int B, int nh, int nkv, int Lmax, float scale_log2, int merge) {
  constexpr int D = 64;
  const int kh = blockIdx.y, l = threadIdx.x, g4 = l >> 4, r16 = l & 15;
  const int G = nh / nkv, SPW = 16 / G;
  const int b0 = blockIdx.x * SPW;
  const int j = r16 / G, g = r16 % G;  // this lane's column: sequence j of the group, head g
  const int bj = b0 + j;
  const bool col_valid = j < SPW && bj < B && (done == nullptr || done[bj] == 0);
  const size_t qrow = (size_t)(col_valid ? bj : 0) * nh + kh * G + g;
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 v = *reinterpret_cast<const uint4*>(q + qrow * D + 8 * g4 + 32 * s2);
    if (!col_valid) v = make_uint4(0, 0, 0, 0);
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  int h_done = 1, h_pos = 0, h_slot = 0;
  if (HOIST && l < SPW && b0 + l < B) {
    h_done = done != nullptr ? done[b0 + l] : 0;
    h_pos = pos[b0 + l];
    h_slot = slot[b0 + l];
  }
  // shared prefix: all columns
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;
  // (merged key stream: the prefix is walked per sequence inside its own stream -- the
  // same tiles in the same order as attn_spec_kernel's, so spec and plain decode agree)
  for (int kt = 0; kt < (merge ? 0 : P0); kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kpre, vpre, kt, g4, r16, kt + 16 < P0, kc, vc);
    st_tile(qb, kc, vc, kt, P0, g4, scale_log2, m, lsum, o);
  }
  // own keys, one sequence at a time (wave-uniform loop; masked columns)
  for (int jj = 0; jj < SPW; ++jj) {
    const int b = b0 + jj;
    if (b >= B) break;
    int own, sl;
    if constexpr (HOIST) {
      if (__builtin_amdgcn_readlane(h_done, jj)) continue;
      own = __builtin_amdgcn_readlane(h_pos, jj) + 1;
      sl = __builtin_amdgcn_readlane(h_slot, jj);
    } else {
      if (done != nullptr && done[b]) continue;
      own = pos[b] + 1;
      sl = slot[b];
    }
    const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
    const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
    const bool mine = (j == jj);
    if (merge) {
      const int nk = P0 + own;
      for (int kt = 0; kt < nk; kt += 32) {
        uint4 kc[2][2], vc[4];
        st_load_tile_m(kpre, vpre, kself, vself, P0, Lmax, kt, g4, r16, nk, kc, vc);
        st_tile(qb, kc, vc, kt, nk, g4, scale_log2, m, lsum, o, mine);
      }
      continue;
    }
    for (int kt = 0; kt < own; kt += 32) {
      uint4 kc[2][2], vc[4];
      st_load_tile(kself, vself, kt, g4, r16, kt + 16 < own, kc, vc);
      st_tile(qb, kc, vc, kt, own, g4, scale_log2, m, lsum, o, mine);
    }
  }
  if (col_valid) {
    const float inv = 1.f / lsum;
    uint16_t* orow = out + qrow * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[n][0] * inv) | ((uint32_t)f2bf(o[n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[n][2] * inv) | ((uint32_t)f2bf(o[n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Speculative-verify attention: one wave = ONE row's pseudo-rows (its current
// token + nd <= 16·NCB/G - 1 drafts, contiguous at row_start[r]) of one kv head.
// MFMA column c <-> (pseudo-row i = c / G, query head g = c % G).  All pseudo-rows
// of a row read the same slot, pseudo-row i seeing keys [0, pos + i]: the row's
// key tiles are loaded and multiplied ONCE for every draft (attn_grouped_kernel
// walks them once per pseudo-row), each column masked at its own length.  A
// column's arithmetic is the grouped kernel's (same tiles in the same order; the
// extra tiles past its length are exact no-ops), so outputs are bit-identical.
// grid = (rows, nkv), one wave; finished rows (row_nd < 0) are skipped.
// ---------------------------------------------------------------------------
// NCB column blocks of 16 (NCB = 2: up to 32 / G pseudo-rows, e.g. 1 + 8 drafts at
// G = 3) share every K/V tile load; block cb holds columns 16·cb .. 16·cb + 15.
template <int NCB>
__global__ void __launch_bounds__(64) attn_spec_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ row_start, const int* __restrict__ row_nd,
    const int* __restrict__ x_pos, const int* __restrict__ x_slot, const int* __restrict__ x_done,
    const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache, const uint16_t* __restrict__ pk,
    const uint16_t* __restrict__ pvt, int P0, int P0pad, uint16_t* __restrict__ out, int nh, int nkv, int Lmax,
    float scale_log2, int merge) {
  constexpr int D = 64;
  const int r = blockIdx.x, kh = blockIdx.y, l = threadIdx.x, g4 = l >> 4, r16 = l & 15;
  const int G = nh / nkv, QPW = 16 * NCB / G;
  const int nd = row_nd[r];
  if (nd < 0) return;  // finished row: no pseudo-rows (sg_spec_plan)
  const int st = row_start[r];
  const int nq = min(nd + 1, QPW);  // the host guarantees (1 + spec_k) * G <= 16 * NCB
  const int p = x_pos[st], sl = x_slot[st];
  bf16x8 qb[NCB][2];
  f32x4 o[NCB][4];
  float m[NCB], lsum[NCB];
  int own[NCB];
  bool col_valid[NCB];
  size_t qrow[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int c = 16 * cb + r16, i = c / G, g = c % G;
    col_valid[cb] = i < nq;
    own[cb] = p + i + 1;  // per-lane length (invalid columns: masked by q = 0 and no store)
    qrow[cb] = (size_t)(st + (col_valid[cb] ? i : 0)) * nh + kh * G + g;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint4 v = *reinterpret_cast<const uint4*>(q + qrow[cb] * D + 8 * g4 + 32 * s2);
      if (!col_valid[cb]) v = make_uint4(0, 0, 0, 0);
      qb[cb][s2] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) o[cb][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    m[cb] = -INFINITY;
    lsum[cb] = 0.f;
  }
  // column blocks holding a valid column (wave-uniform): a row with 1 + nd <= 16 / G
  // pseudo-rows (most rows: ~2.3 per row at the bench's draft budget) skips the second
  // block's MFMAs and softmax; the valid columns' arithmetic is unchanged
  const int live = (nq * G + 15) >> 4;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;
  if (merge) {  // one stream of prefix + own keys (st_load_tile_m)
    const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
    const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
    const int nk = P0 + p + nq;
    for (int kt = 0; kt < nk; kt += 32) {
      uint4 kc[2][2], vc[4];
      st_load_tile_m(kpre, vpre, kself, vself, P0, Lmax, kt, g4, r16, nk, kc, vc);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        if (cb < live)
          st_tile(qb[cb], kc, vc, kt, P0 + own[cb], g4, scale_log2, m[cb], lsum[cb], o[cb], col_valid[cb]);
    }
  }
  for (int kt = 0; kt < (merge ? 0 : P0); kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kpre, vpre, kt, g4, r16, kt + 16 < P0, kc, vc);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
      if (cb < live) st_tile(qb[cb], kc, vc, kt, P0, g4, scale_log2, m[cb], lsum[cb], o[cb]);
  }
  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const int own_max = merge ? 0 : p + nq;
  for (int kt = 0; kt < own_max; kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kself, vself, kt, g4, r16, kt + 16 < own_max, kc, vc);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
      if (cb < live) st_tile(qb[cb], kc, vc, kt, own[cb], g4, scale_log2, m[cb], lsum[cb], o[cb], col_valid[cb]);
  }
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    if (!col_valid[cb]) continue;
    const float inv = 1.f / lsum[cb];
    uint16_t* orow = out + qrow[cb] * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[cb][n][0] * inv) | ((uint32_t)f2bf(o[cb][n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[cb][n][2] * inv) | ((uint32_t)f2bf(o[cb][n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Prefill attention in the transposed register formulation (impl "st", default).
// One wave = QPW = 16·NCB/G consecutive queries of ONE sequence and one kv head, all
// G query heads: MFMA column c <-> (query i = c / G, head g = c % G), exactly the
// verify kernel's decomposition with the row's drafts replaced by a prompt chunk.
// S^T = K·Q^T and O^T = V^T·P^T (st_tile): the softmax state stays in the lane that
// owns the column, P never leaves registers — no LDS round trip, no barrier and two
// shuffles per reduction, where the per-head kernel (S = Q·K^T) staged P through LDS
// with eight 2-byte stores and two __syncthreads per 32-key tile and spent its time
// on that VALU / LDS work (prefill_bench: it scales with tokens, not with latency).
// K/V tiles are loaded once for the G heads of the group.  Causal: column i sees own
// keys [0, q_start + i]; the tile loop runs to the wave's last query.
// grid = (ceil(max_q / QPW), nseq, nkv), one wave.  PF = 1 (merged stream only): the
// loads of key tile t+1 are issued before the MFMAs of tile t (one-tile register prefetch).
// ---------------------------------------------------------------------------
template <int NCB, int PF = 0>
__global__ void __launch_bounds__(64) attn_prefill_st_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ q_start,
    const int* __restrict__ slot, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad, uint16_t* __restrict__ out,
    int nh, int nkv, int Lmax, float scale_log2, int merge) {
  constexpr int D = 64;
  const int tile = blockIdx.x, b = blockIdx.y, kh = blockIdx.z, l = threadIdx.x, g4 = l >> 4, r16 = l & 15;
  const int G = nh / nkv, QPW = 16 * NCB / G;
  const int qbeg = cu_q[b], qlen = cu_q[b + 1] - qbeg;
  const int q0 = tile * QPW;
  if (q0 >= qlen) return;
  const int qs = q_start[b], sl = slot[b];
  const int nq = min(QPW, qlen - q0);
  bf16x8 qb[NCB][2];
  f32x4 o[NCB][4];
  float m[NCB], lsum[NCB];
  int own[NCB];
  bool col_valid[NCB];
  size_t qrow[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int c = 16 * cb + r16, i = c / G, g = c % G;
    col_valid[cb] = i < nq;
    own[cb] = qs + q0 + i + 1;  // causal length over own keys
    qrow[cb] = (size_t)(qbeg + q0 + (col_valid[cb] ? i : 0)) * nh + kh * G + g;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint4 v = *reinterpret_cast<const uint4*>(q + qrow[cb] * D + 8 * g4 + 32 * s2);
      if (!col_valid[cb]) v = make_uint4(0, 0, 0, 0);
      qb[cb][s2] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) o[cb][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    m[cb] = -INFINITY;
    lsum[cb] = 0.f;
  }
  const int live = (nq * G + 15) >> 4;  // column blocks with a valid column (a sequence's last chunk)
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;
  if (merge) {  // one stream of prefix + own keys (st_load_tile_m)
    const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
    const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
    const int nk = P0 + qs + q0 + nq;
    if constexpr (PF) {
      uint4 kc[2][2], vc[4];
      st_load_tile_m(kpre, vpre, kself, vself, P0, Lmax, 0, g4, r16, nk, kc, vc);
      for (int kt = 0; kt < nk; kt += 32) {
        uint4 kn[2][2], vn[4];
        const bool more = kt + 32 < nk;
        if (more) st_load_tile_m(kpre, vpre, kself, vself, P0, Lmax, kt + 32, g4, r16, nk, kn, vn);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          if (cb < live)
            st_tile(qb[cb], kc, vc, kt, P0 + own[cb], g4, scale_log2, m[cb], lsum[cb], o[cb], col_valid[cb]);
        if (more) {
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            kc[a][0] = kn[a][0];
            kc[a][1] = kn[a][1];
          }
#pragma unroll
          for (int n = 0; n < 4; ++n) vc[n] = vn[n];
        }
      }
    } else {
      for (int kt = 0; kt < nk; kt += 32) {
        uint4 kc[2][2], vc[4];
        st_load_tile_m(kpre, vpre, kself, vself, P0, Lmax, kt, g4, r16, nk, kc, vc);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          if (cb < live)
            st_tile(qb[cb], kc, vc, kt, P0 + own[cb], g4, scale_log2, m[cb], lsum[cb], o[cb], col_valid[cb]);
      }
    }
  }
  for (int kt = 0; kt < (merge ? 0 : P0); kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kpre, vpre, kt, g4, r16, kt + 16 < P0, kc, vc);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
      if (cb < live) st_tile(qb[cb], kc, vc, kt, P0, g4, scale_log2, m[cb], lsum[cb], o[cb]);
  }
  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const int own_max = merge ? 0 : qs + q0 + nq;
  for (int kt = 0; kt < own_max; kt += 32) {
    uint4 kc[2][2], vc[4];
    st_load_tile(kself, vself, kt, g4, r16, kt + 16 < own_max, kc, vc);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
      if (cb < live) st_tile(qb[cb], kc, vc, kt, own[cb], g4, scale_log2, m[cb], lsum[cb], o[cb], col_valid[cb]);
  }
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    if (!col_valid[cb]) continue;
    const float inv = 1.f / lsum[cb];
    uint16_t* orow = out + qrow[cb] * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[cb][n][0] * inv) | ((uint32_t)f2bf(o[cb][n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[cb][n][2] * inv) | ((uint32_t)f2bf(o[cb][n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Grouped decode attention with a one-tile register prefetch: the same work as
// attn_grouped_kernel, but the wave walks ONE flattened stream of 32-key tiles
// (shared prefix, then each live sequence's own keys) and issues the loads of
// tile t+1 before the MFMAs of tile t.  At a 4096-row half batch there are only
// ~2.4 of these waves per SIMD, too few to cover a cold HBM load with other
// waves, so the latency has to be covered inside the wave.
// ---------------------------------------------------------------------------
struct TileCur {
  int jj, kt, nval;  // jj = -1: shared prefix; SPW: end of stream
  const uint16_t* kb;
  const uint16_t* vb;
};

__global__ void __launch_bounds__(64) attn_grouped_pf_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int B, int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  const int kh = blockIdx.y, l = threadIdx.x, g4 = l >> 4, r16 = l & 15;
  const int G = nh / nkv, SPW = 16 / G;
  const int b0 = blockIdx.x * SPW;
  const int j = r16 / G, g = r16 % G;
  const int bj = b0 + j;
  const bool col_valid = j < SPW && bj < B && (done == nullptr || done[bj] == 0);
  const size_t qrow = (size_t)(col_valid ? bj : 0) * nh + kh * G + g;
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 v = *reinterpret_cast<const uint4*>(q + qrow * D + 8 * g4 + 32 * s2);
    if (!col_valid) v = make_uint4(0, 0, 0, 0);
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;
  // move c to the first tile at or after (c.jj, c.kt) (wave-uniform)
  auto seek = [&](TileCur& c) {
    while (c.jj < SPW) {
      if (c.jj < 0) {
        if (c.kt < P0) {
          c.nval = P0;
          c.kb = kpre;
          c.vb = vpre;
          return;
        }
      } else {
        const int b = b0 + c.jj;
        if (b >= B) break;
        if (done == nullptr || done[b] == 0) {
          c.nval = pos[b] + 1;
          if (c.kt < c.nval) {
            const int sl = slot[b];
            c.kb = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
            c.vb = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
            return;
          }
        }
      }
      ++c.jj;
      c.kt = 0;
    }
    c.jj = SPW;
  };
  TileCur cur{-1, 0, 0, kpre, vpre};
  seek(cur);
  uint4 kc[2][2], vc[4], kn[2][2], vn[4];
  if (cur.jj < SPW) st_load_tile(cur.kb, cur.vb, cur.kt, g4, r16, cur.kt + 16 < cur.nval, kc, vc);
  while (cur.jj < SPW) {
    TileCur nxt = cur;
    nxt.kt += 32;
    seek(nxt);
    if (nxt.jj < SPW) st_load_tile(nxt.kb, nxt.vb, nxt.kt, g4, r16, nxt.kt + 16 < nxt.nval, kn, vn);
    st_tile(qb, kc, vc, cur.kt, cur.nval, g4, scale_log2, m, lsum, o, cur.jj < 0 || j == cur.jj);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) kc[a][s2] = kn[a][s2];
#pragma unroll
    for (int n = 0; n < 4; ++n) vc[n] = vn[n];
    cur = nxt;
  }
  if (col_valid) {
    const float inv = 1.f / lsum;
    uint16_t* orow = out + qrow * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[n][0] * inv) | ((uint32_t)f2bf(o[n][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[n][2] * inv) | ((uint32_t)f2bf(o[n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// Key-split decode attention (small batches): NWV waves per (row, kv head) deal
// the row's 32-key tiles — shared prefix first, then its own keys — round-robin;
// each wave keeps its own online-softmax state and wave 0 merges the NWV states
// through LDS.  At a few hundred rows the grouped kernel launches too few waves
// and each walks ~15 dependent tiles; here each wave walks ceil(tiles / NWV),
// so the step latency shrinks with NWV while the bytes read stay the same.
// grid = (B, nkv), NWV waves per block.
// ---------------------------------------------------------------------------
template <int NWV>
__global__ void __launch_bounds__(NWV * 64) attn_split_kernel(
    const uint16_t* __restrict__ q, const int* __restrict__ pos, const int* __restrict__ slot,
    const int* __restrict__ done, const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ vt_cache,
    const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pvt, int P0, int P0pad,
    uint16_t* __restrict__ out, int nh, int nkv, int Lmax, float scale_log2) {
  constexpr int D = 64;
  __shared__ float red[NWV][64][18];  // per wave and lane: o[16], m, l
  const int b = blockIdx.x, kh = blockIdx.y, tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  if (done != nullptr && done[b]) return;  // block-uniform, before any barrier
  const int G = nh / nkv, g4 = l >> 4, r16 = l & 15;
  const int own = pos[b] + 1;
  const int sl = slot[b];
  const uint16_t* kself = k_cache + ((size_t)sl * nkv + kh) * Lmax * D;
  const uint16_t* vself = vt_cache + ((size_t)sl * nkv + kh) * D * Lmax;
  const uint16_t* kpre = pk + (size_t)kh * P0pad * D;
  const uint16_t* vpre = pvt + (size_t)kh * D * P0pad;
  const size_t qrow = (size_t)b * nh + kh * G + (r16 < G ? r16 : 0);
  bf16x8 qb[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 v = *reinterpret_cast<const uint4*>(q + qrow * D + 8 * g4 + 32 * s2);
    if (r16 >= G) v = make_uint4(0, 0, 0, 0);
    qb[s2] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;
  const int npre = (P0 + 31) >> 5, ntiles = npre + ((own + 31) >> 5);
  for (int t = w; t < ntiles; t += NWV) {
    const bool pre = t < npre;
    const int kt = (pre ? t : t - npre) * 32, nval = pre ? P0 : own;
    uint4 kc[2][2], vc[4];
    st_load_tile(pre ? kpre : kself, pre ? vpre : vself, kt, g4, r16, kt + 16 < nval, kc, vc);
    st_tile(qb, kc, vc, kt, nval, g4, scale_log2, m, lsum, o);
  }
  float* mine = red[w][l];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i) mine[4 * n + i] = o[n][i];
  mine[16] = m;
  mine[17] = lsum;
  __syncthreads();
  if (w != 0 || r16 >= G) return;
  float M = -INFINITY;
#pragma unroll
  for (int v = 0; v < NWV; ++v) M = fmaxf(M, red[v][l][16]);
  float acc[16], L = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
  for (int v = 0; v < NWV; ++v) {
    const float mv = red[v][l][16];
    if (mv == -INFINITY) continue;  // this wave saw no valid key
    const float f = exp2f(mv - M);
    L += f * red[v][l][17];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] += f * red[v][l][j];
  }
  const float inv = 1.f / L;
  uint16_t* orow = out + qrow * D;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    uint2 wv;
    wv.x = (uint32_t)f2bf(acc[4 * n] * inv) | ((uint32_t)f2bf(acc[4 * n + 1] * inv) << 16);
    wv.y = (uint32_t)f2bf(acc[4 * n + 2] * inv) | ((uint32_t)f2bf(acc[4 * n + 3] * inv) << 16);
    *reinterpret_cast<uint2*>(orow + 16 * n + 4 * g4) = wv;
  }
}

// ---------------------------------------------------------------------------
// Schema-FSM constrained sampling + FSM transition, fully on the GPU (so many
// decode steps can be replayed from one captured graph without a host sync).
// One 256-thread block per sequence row.
// ---------------------------------------------------------------------------
static __device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

__global__ void __launch_bounds__(256) fsm_sample_kernel(
    const uint16_t* __restrict__ logits, int ldl, const uint32_t* __restrict__ masks, const int* __restrict__ state_mask,
    int* __restrict__ state, const int* __restrict__ next_sep, const int* __restrict__ next_tok,
    const int* __restrict__ enum_tok, const int* __restrict__ enum_next, int E, int sep_token, int done_state,
    int* __restrict__ tok_io, int* __restrict__ out_buf, int* __restrict__ out_len, int* __restrict__ done,
    int* __restrict__ pos, const int* __restrict__ slot_id, const int* __restrict__ row_map, int max_out, int V,
    float inv_temp, uint32_t seed, const int* __restrict__ copy_kind, const uint32_t* __restrict__ row_masks) {
  const int lr = blockIdx.x;                      // logits row
  const int b = row_map ? row_map[lr] : lr;       // state row
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ float bv[4];
  __shared__ int bi[4];
  if (done[b]) return;  // block-uniform
  const int s = state[b];
  // copy state: the row's own mask (ops.copy_masks, one mask row per logits row)
  const uint32_t* mrow = (copy_kind != nullptr && copy_kind[s]) ? row_masks + (size_t)lr * (V >> 5)
                                                                 : masks + (size_t)state_mask[s] * (V >> 5);
  const uint16_t* lrow = logits + (size_t)lr * ldl;
  const uint32_t rseed = hash3(seed, (uint32_t)slot_id[b], (uint32_t)out_len[b]);
  float best = -INFINITY;
  int besti = 0x7fffffff;
  const int nvec = V >> 3;
  for (int c = tid; c < nvec; c += 256) {
    const uint32_t bits = (mrow[c >> 2] >> ((c & 3) * 8)) & 0xffu;
    if (!bits) continue;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(lrow + 8 * c), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (bits & (1u << j)) {
        const int idx = 8 * c + j;
        float v = f[j];
        if (inv_temp > 0.f) {
          const uint32_t hsh = hash3(rseed, (uint32_t)idx, 0x51ED270Bu);
          const float u = ((hsh >> 8) + 0.5f) * (1.0f / 16777216.0f);
          v = v * inv_temp - __logf(-__logf(u));
        }
        if (v > best || (v == best && idx < besti)) { best = v; besti = idx; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, WAVE);
    const int oi = __shfl_xor(besti, o, WAVE);
    if (ov > best || (ov == best && oi < besti)) { best = ov; besti = oi; }
  }
  if (lane == 0) { bv[wid] = best; bi[wid] = besti; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (bv[w] > best || (bv[w] == best && bi[w] < besti)) { best = bv[w]; besti = bi[w]; }
    int tok = (besti == 0x7fffffff) ? sep_token : besti;
    int ns;
    if (tok == sep_token) {
      ns = next_sep[s];
    } else {
      ns = next_tok[s];
      if (E > 0 && ns == -2) {  // enum/trie state: sparse transition list
        ns = -1;
        for (int e = 0; e < E; ++e)
          if (enum_tok[s * E + e] == tok) { ns = enum_next[s * E + e]; break; }
      }
    }
    const int len = out_len[b];
    out_buf[(size_t)b * max_out + len] = tok;
    out_len[b] = len + 1;
    tok_io[b] = tok;
    state[b] = ns < 0 ? done_state : ns;
    if (ns < 0 || ns == done_state || len + 1 >= max_out) {
      done[b] = 1;
    } else {
      pos[b] = pos[b] + 1;
    }
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int g_prefill_impl = 2;  // sg_set_prefill_impl
static int g_attn_merge = 1;    // sg_set_attn_merge: merged prefix + own key stream (st kernels)
static inline int attn_merge(int P0) { return g_attn_merge && P0 % 4 == 0 ? 1 : 0; }
static int g_prefill_ks = 1;    // sg_set_prefill_split

// ---------------------------------------------------------------------------
// Message-start template reuse (serving/engine.py): copy own offsets 0..k-1 of a
// template slot's keys (k rows of 128 B per layer and kv head) and the V^T blocks
// holding them (8 keys per 1 KiB block; a partial last block carries template
// padding that the message's own prefill overwrites from offset k on) into a
// message's slot, every layer.  grid = (items, layers), 256 threads, 16-B copies.
// ---------------------------------------------------------------------------
// Embedding rows for int32 token ids (the decode / verify step's input): out[i] =
// table[ids[i]], 16-B chunks, one thread per chunk.  F.embedding needs int64 ids, i.e. a
// cast kernel plus a gather kernel per step; ids outside [0, V) give a zero row.
__global__ void __launch_bounds__(256) embed_rows_kernel(const int* __restrict__ ids, const uint16_t* __restrict__ table,
                                                         uint16_t* __restrict__ out, int T, int H, int V) {
  const int cpr = H >> 3;  // 16-B chunks per row
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long long)T * cpr) return;
  const int i = (int)(q / cpr), c = (int)(q % cpr);
  const int t = ids[i];
  uint4 v = make_uint4(0, 0, 0, 0);
  if (t >= 0 && t < V) v = *reinterpret_cast<const uint4*>(table + (size_t)t * H + 8 * c);
  *reinterpret_cast<uint4*>(out + (size_t)i * H + 8 * c) = v;
}

// span-format prompt rows: table[ids[i]] + table[base + pos[i]] in one pass (the token's
// row plus the row of pointer `pos[i]`), the sum rounded to bf16 like torch's bf16 add
// (fp32 add, RNE).  Replaces a cast, two gathers and an add per prefill.
__global__ void __launch_bounds__(256) embed_rows_add_kernel(const int* __restrict__ ids, const int* __restrict__ pos,
                                                             const uint16_t* __restrict__ table,
                                                             uint16_t* __restrict__ out, int T, int H, int V, int base) {
  const int cpr = H >> 3;
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long long)T * cpr) return;
  const int i = (int)(q / cpr), c = (int)(q % cpr);
  const int t = ids[i], p = base + pos[i];
  float a[8], b[8];
  uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
  if (t >= 0 && t < V) va = *reinterpret_cast<const uint4*>(table + (size_t)t * H + 8 * c);
  if (p >= 0 && p < V) vb = *reinterpret_cast<const uint4*>(table + (size_t)p * H + 8 * c);
  unpack8(va, a);
  unpack8(vb, b);
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w[k] = (uint32_t)f2bf(a[2 * k] + b[2 * k]) | ((uint32_t)f2bf(a[2 * k + 1] + b[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(out + (size_t)i * H + 8 * c) = make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(256) kv_copy_prefix_kernel(uint16_t* __restrict__ k_cache,
                                                             uint16_t* __restrict__ vt_cache,
                                                             const int* __restrict__ items, int n, int S_kv,
                                                             int nkv, int Lmax) {
  constexpr int D = 64;
  const int i = blockIdx.x, layer = blockIdx.y;
  const int src = items[i], dst = items[n + i], k = items[2 * n + i];
  const size_t slot_elems = (size_t)nkv * Lmax * D;  // K and V^T: the same elements per slot
  const size_t lbase = (size_t)layer * S_kv * slot_elems;
  const uint4* ks = reinterpret_cast<const uint4*>(k_cache + lbase + (size_t)src * slot_elems);
  uint4* kd = reinterpret_cast<uint4*>(k_cache + lbase + (size_t)dst * slot_elems);
  const uint4* vs = reinterpret_cast<const uint4*>(vt_cache + lbase + (size_t)src * slot_elems);
  uint4* vd = reinterpret_cast<uint4*>(vt_cache + lbase + (size_t)dst * slot_elems);
  const int head16 = Lmax * D / 8;        // uint4 per kv head (K rows or V^T blocks)
  const int krow16 = k * (D / 8);         // K: k rows x 8 chunks
  const int vblk16 = ((k + 7) >> 3) * D;  // V^T: whole 8-key blocks, 64 chunks each
  for (int q = threadIdx.x; q < nkv * krow16; q += 256) {
    const int h = q / krow16, c = q - h * krow16;
    kd[h * head16 + c] = ks[h * head16 + c];
  }
  for (int q = threadIdx.x; q < nkv * vblk16; q += 256) {
    const int h = q / vblk16, c = q - h * vblk16;
    vd[h * head16 + c] = vs[h * head16 + c];
  }
}

extern "C" {

int sg_rmsnorm_residual(const void* x_in, void* residual, const void* w, void* out, int T, int H, float eps,
                        hipStream_t stream) {
  if (H % 8 || H > 2048) return -1;
  if (T == 0) return 0;
  dim3 grid((T + 3) / 4);
  hipLaunchKernelGGL(rmsnorm_residual_kernel, grid, dim3(256), 0, stream, (const uint16_t*)x_in, (uint16_t*)residual,
                     (const uint16_t*)w, (uint16_t*)out, T, H, eps);
  return (int)hipGetLastError();
}

int sg_silu_mul(const void* gu, void* out, int T, int I, hipStream_t stream) {
  if (I % 8) return -1;
  if (T == 0) return 0;
  long total = (long)T * (I / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(blocks), dim3(256), 0, stream, (const uint16_t*)gu, (uint16_t*)out, T, I);
  return (int)hipGetLastError();
}

int sg_embed_rows(const int* ids, const void* table, void* out, int T, int H, int V, hipStream_t stream) {
  if (H % 8) return -1;
  if (T == 0) return 0;
  const long long n = (long long)T * (H >> 3);
  hipLaunchKernelGGL(embed_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ids,
                     (const uint16_t*)table, (uint16_t*)out, T, H, V);
  return (int)hipGetLastError();
}

int sg_embed_rows_add(const int* ids, const int* pos, const void* table, void* out, int T, int H, int V, int base,
                      hipStream_t stream) {
  if (H % 8) return -1;
  if (T == 0) return 0;
  const long long n = (long long)T * (H >> 3);
  hipLaunchKernelGGL(embed_rows_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ids, pos,
                     (const uint16_t*)table, (uint16_t*)out, T, H, V, base);
  return (int)hipGetLastError();
}

// items: int32 [3][n] = template slot, message slot, k (0 < k <= Lmax) per item
int sg_kv_copy_prefix(void* k_cache, void* vt_cache, const int* items, int n, int layers, int S_kv, int nkv, int D,
                      int Lmax, hipStream_t stream) {
  if (D != 64 || Lmax % 8) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(kv_copy_prefix_kernel, dim3(n, layers), dim3(256), 0, stream, (uint16_t*)k_cache,
                     (uint16_t*)vt_cache, items, n, S_kv, nkv, Lmax);
  return (int)hipGetLastError();
}

int sg_rope_qkv_cache(const void* qkv, const int* pos, const int* slot, const void* cos_sin, void* q_out,
                      void* k_cache, void* vt_cache, int T, int nh, int nkv, int D, int Lmax, int p0,
                      hipStream_t stream) {
  if (D % 2) return -1;
  if (T == 0) return 0;
  if (Lmax % 8) return -1;
  hipLaunchKernelGGL(rope_qkv_cache_kernel, dim3((T + 3) / 4), dim3(256), 0, stream, (const uint16_t*)qkv, pos, slot,
                     (const float2*)cos_sin, (uint16_t*)q_out, (uint16_t*)k_cache, (uint16_t*)vt_cache, T, nh, nkv,
                     D, Lmax, p0);
  return (int)hipGetLastError();
}

int sg_attn_prefill(const void* q, const int* cu_q, const int* q_start, const int* slot, const void* k_cache,
                    const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int nseq,
                    int max_q, int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || (P0pad % 32) || (Lmax % 8) || nh % nkv) return -1;
  if (nseq == 0 || max_q == 0) return 0;
  const float sl2 = scale * 1.4426950408889634f;
  const int G = nh / nkv;
  // auto: the per-head kernel launches G x the waves, which wins while the batch is
  // too small to fill the chip (prefill_bench: 12.6 vs 17.2 us at 32 sequences,
  // 32 vs 38 us at 190); the GQA kernel's single K/V load wins at 800 (98 vs 112 us)
  // auto (default) = the transposed register kernel with 32 columns: 14.0 / 20.8 / 42.1 us
  // at 150 / 300 / 800 sequences vs 23.3 / 33.6 / 81.3 for the per-head kernel and 20.8 /
  // 32.6 / 70.2 for the GQA one (profiles/r03_prefill_st.jsonl); bench 29 350 vs 26 698 /
  // 27 508 msgs/s (per-head / GQA auto, profiles/r03_ab_prefill_st.jsonl)
  if ((g_prefill_impl == 2 || g_prefill_impl >= 4) && G <= 16) {
    // st64 (impl 6): 64 columns, half the waves re-read a sequence's keys; st32pf (impl 7):
    // st32 with the one-tile register prefetch; stpf (impl 8): st with it
    // auto = st32 at every batch size: round 5 picked st64 from 1 024 sequences on a
    // microbench (103.4 / 198.7 vs 110.0 / 210.0 us, profiles/r05_prefill_qa.jsonl); the
    // engine itself runs faster with st32 (69.6 vs 69.2 k msgs/s, three identical reps
    // each, interleaved, profiles/r06n_engine_prefill_attn_ab.jsonl)
    const bool wide = g_prefill_impl == 6 || g_prefill_impl == 9;
    const int ncb = (g_prefill_impl == 4 || g_prefill_impl == 8) ? 1 : wide ? 4 : 2, qpw = 16 * ncb / G;
    dim3 grid((max_q + qpw - 1) / qpw, nseq, nkv);
#define SG_PST(NC, PFV)                                                                                             \
  hipLaunchKernelGGL((attn_prefill_st_kernel<NC, PFV>), grid, dim3(64), 0, stream, (const uint16_t*)q, cu_q, q_start, \
                     slot, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,             \
                     (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2, attn_merge(P0))
    if (g_prefill_impl == 7) SG_PST(2, 1);
    else if (g_prefill_impl == 8) SG_PST(1, 1);
    else if (g_prefill_impl == 9) SG_PST(4, 1);  // st64 with the register prefetch (A/B)
    else if (ncb == 2) SG_PST(2, 0);
    else if (ncb == 4) SG_PST(4, 0);
    else SG_PST(1, 0);
#undef SG_PST
    return (int)hipGetLastError();
  }
  if (g_prefill_impl == 3) {  // multi-tile per-head kernel
    dim3 grid((max_q + 15) / 16, nseq, nh);
    hipLaunchKernelGGL((attn_prefill_mt_kernel<3>), grid, dim3(64), 0, stream, (const uint16_t*)q, cu_q, q_start, slot,
                       (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk, (const uint16_t*)pvt,
                       P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2);
    return (int)hipGetLastError();
  }
  const bool gqa = g_prefill_impl == 0 || (g_prefill_impl == 2 && nseq > 384);
  if (gqa && G >= 1 && G <= 4) {
    dim3 grid((max_q + 15) / 16, nseq, nkv);
#define SG_PF(GG, KS)                                                                                          \
  hipLaunchKernelGGL((attn_prefill_gqa_kernel<GG, KS>), grid, dim3(64 * KS), 0, stream, (const uint16_t*)q, cu_q, \
                     q_start, slot, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,     \
                     (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2)
    if (g_prefill_ks == 2) {
      if (G == 1) SG_PF(1, 2);
      else if (G == 2) SG_PF(2, 2);
      else if (G == 3) SG_PF(3, 2);
      else SG_PF(4, 2);
    } else {
      if (G == 1) SG_PF(1, 1);
      else if (G == 2) SG_PF(2, 1);
      else if (G == 3) SG_PF(3, 1);
      else SG_PF(4, 1);
    }
#undef SG_PF
    return (int)hipGetLastError();
  }
  dim3 grid((max_q + 15) / 16, nseq, nh);
  hipLaunchKernelGGL(attn_prefill_kernel, grid, dim3(64), 0, stream, (const uint16_t*)q, cu_q, q_start, slot,
                     (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk, (const uint16_t*)pvt,
                     P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2);
  return (int)hipGetLastError();
}

// 0 = GQA-shared prefetching kernel, 1 = per-head kernel, 2 = auto (5; if G > 16: 0 / 1 by
// batch size), 3 = multi-tile per-head kernel, 4 / 5 = transposed register kernel, 16 / 32 columns
void sg_set_prefill_impl(int impl) { g_prefill_impl = impl; }

// 1 (default): the st attention kernels (verify, grouped decode, prefill st/st32) walk the
// shared prefix and the own keys as one tile stream when P0 % 4 == 0; 0: prefix tiles first
void sg_set_attn_merge(int on) { g_attn_merge = on ? 1 : 0; }

// key split of the GQA prefill kernel: 1 (one wave per tile) or 2 (two waves share the keys)
void sg_set_prefill_split(int ks) { g_prefill_ks = ks == 2 ? 2 : 1; }

int sg_attn_decode(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                   const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B, int nh,
                   int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  // unconditional 32-key tile loads: Lmax and P0pad must be multiples of 32
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(attn_decode_st_kernel, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, pos, slot, done,
                     (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk, (const uint16_t*)pvt, P0,
                     P0pad, (uint16_t*)out, nh, nkv, Lmax, scale * 1.4426950408889634f);
  return (int)hipGetLastError();
}

// Cascade decode attention (production): prefix pass + own-key pass.  pre_o
// [B, nh, D] fp32 and pre_lse [B, nh] fp32 are caller-provided scratch.
int sg_attn_decode_cascade(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                           const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                           int nh, int nkv, int D, int Lmax, float scale, void* pre_o, void* pre_lse,
                           hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (P0 > 0 && (pre_o == nullptr || pre_lse == nullptr)) return -2;
  if (B == 0) return 0;
  const float sl2 = scale * 1.4426950408889634f;
  const int G = nh / nkv;
  if (P0 > 0)
    hipLaunchKernelGGL(attn_prefix_kernel, dim3((B * G + 15) / 16, nkv), dim3(64), 0, stream, (const uint16_t*)q,
                       (const uint16_t*)pk, (const uint16_t*)pvt, P0, P0pad, (float*)pre_o, (float*)pre_lse, B, nh, nkv,
                       sl2);
  hipLaunchKernelGGL(attn_own_kernel, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, pos, slot, done,
                     (const uint16_t*)k_cache, (const uint16_t*)vt_cache, P0 > 0 ? (const float*)pre_o : nullptr,
                     (const float*)pre_lse, (uint16_t*)out, nh, nkv, Lmax, sl2);
  return (int)hipGetLastError();
}

// Grouped decode attention: 16/G sequences per wave, shared prefix once (no scratch).
int sg_attn_decode_grouped(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                           const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                           int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  const int spw = 16 / (nh / nkv);
  hipLaunchKernelGGL(attn_grouped_kernel<1>, dim3((B + spw - 1) / spw, nkv), dim3(64), 0, stream, (const uint16_t*)q,
                     pos, slot, done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,
                     (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, B, nh, nkv, Lmax, scale * 1.4426950408889634f, attn_merge(P0));
  return (int)hipGetLastError();
}

// Speculative-verify attention over B rows' pseudo-rows (row_start / row_nd from sg_spec_plan).
int sg_attn_spec(const void* q, const int* row_start, const int* row_nd, const int* x_pos, const int* x_slot,
                 const int* x_done, const void* k_cache, const void* vt_cache, const void* pk, const void* pvt, int P0,
                 int P0pad, void* out, int B, int nh, int nkv, int D, int Lmax, float scale, int max_q,
                 hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || max_q < 1 || max_q * (nh / nkv) > 32 || (P0pad % 32) || (Lmax % 32) ||
      P0 > P0pad)
    return -1;
  if (B == 0) return 0;
  const float sl2 = scale * 1.4426950408889634f;
  if (max_q * (nh / nkv) <= 16)
    hipLaunchKernelGGL(attn_spec_kernel<1>, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, row_start, row_nd,
                       x_pos, x_slot, x_done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,
                       (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2, attn_merge(P0));
  else
    hipLaunchKernelGGL(attn_spec_kernel<2>, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, row_start, row_nd,
                       x_pos, x_slot, x_done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,
                       (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, sl2, attn_merge(P0));
  return (int)hipGetLastError();
}

// Grouped decode attention with the per-sequence (done, pos, slot) loads hoisted to entry.
int sg_attn_decode_grouped_h(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                             const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out,
                             int B, int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  const int spw = 16 / (nh / nkv);
  hipLaunchKernelGGL((attn_grouped_kernel<1, true>), dim3((B + spw - 1) / spw, nkv), dim3(64), 0, stream,
                     (const uint16_t*)q, pos, slot, done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache,
                     (const uint16_t*)pk, (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, B, nh, nkv, Lmax,
                     scale * 1.4426950408889634f, attn_merge(P0));
  return (int)hipGetLastError();
}

// Grouped decode attention built for 6 resident waves per SIMD (VGPRs capped at 80).
int sg_attn_decode_grouped6(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                            const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                            int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  const int spw = 16 / (nh / nkv);
  hipLaunchKernelGGL(attn_grouped_kernel<6>, dim3((B + spw - 1) / spw, nkv), dim3(64), 0, stream, (const uint16_t*)q,
                     pos, slot, done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,
                     (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, B, nh, nkv, Lmax, scale * 1.4426950408889634f, attn_merge(P0));
  return (int)hipGetLastError();
}

// Grouped decode attention with a one-tile register prefetch (A/B against grouped).
int sg_attn_decode_grouped_pf(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                              const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out,
                              int B, int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  const int spw = 16 / (nh / nkv);
  hipLaunchKernelGGL(attn_grouped_pf_kernel, dim3((B + spw - 1) / spw, nkv), dim3(64), 0, stream,
                     (const uint16_t*)q, pos, slot, done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache,
                     (const uint16_t*)pk, (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, B, nh, nkv, Lmax,
                     scale * 1.4426950408889634f);
  return (int)hipGetLastError();
}

// Key-split decode attention (small batches): nwv waves per (row, kv head).
int sg_attn_decode_split(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                         const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                         int nh, int nkv, int D, int Lmax, float scale, int nwv, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
#define SG_SPLIT(N)                                                                                                \
  hipLaunchKernelGGL(attn_split_kernel<N>, dim3(B, nkv), dim3(N * 64), 0, stream, (const uint16_t*)q, pos, slot, \
                     done, (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk,             \
                     (const uint16_t*)pvt, P0, P0pad, (uint16_t*)out, nh, nkv, Lmax, scale * 1.4426950408889634f)
  if (nwv == 2) SG_SPLIT(2);
  else if (nwv == 4) SG_SPLIT(4);
  else if (nwv == 8) SG_SPLIT(8);
  else return -1;
#undef SG_SPLIT
  return (int)hipGetLastError();
}

// Previous MFMA formulation (S = Q·K^T, P through LDS) — kept for A/B (kbench).
int sg_attn_decode_v1(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                      const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                      int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > 16 || (P0pad % 32) || (Lmax % 32) || P0 > P0pad) return -1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(attn_decode_mfma_kernel, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, pos, slot, done,
                     (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk, (const uint16_t*)pvt, P0,
                     P0pad, (uint16_t*)out, nh, nkv, Lmax, scale * 1.4426950408889634f);
  return (int)hipGetLastError();
}

// VALU reference implementation (kept for A/B measurement: scripts/kbench.py).
int sg_attn_decode_valu(const void* q, const int* pos, const int* slot, const int* done, const void* k_cache,
                        const void* vt_cache, const void* pk, const void* pvt, int P0, int P0pad, void* out, int B,
                        int nh, int nkv, int D, int Lmax, float scale, hipStream_t stream) {
  if (D != 64 || nh % nkv || nh / nkv > DEC_MAXG || P0pad + Lmax > DEC_MAXCTX || (P0pad % 8) || (Lmax % 8) ||
      P0 > P0pad)
    return -1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(attn_decode_kernel, dim3(B, nkv), dim3(64), 0, stream, (const uint16_t*)q, pos, slot, done,
                     (const uint16_t*)k_cache, (const uint16_t*)vt_cache, (const uint16_t*)pk, (const uint16_t*)pvt, P0,
                     P0pad, (uint16_t*)out, nh, nkv, Lmax, scale * 1.4426950408889634f);
  return (int)hipGetLastError();
}

int sg_fsm_sample(const void* logits, int ldl, const void* masks, const int* state_mask, int* state,
                  const int* next_sep, const int* next_tok, const int* enum_tok, const int* enum_next, int E,
                  int sep_token, int done_state, int* tok_io, int* out_buf, int* out_len, int* done, int* pos,
                  const int* slot_id, const int* row_map, int max_out, int V, int B, float inv_temp,
                  unsigned int seed, const int* copy_kind, const void* row_masks, hipStream_t stream) {
  if (V % 32 || ldl % 8 || (copy_kind != nullptr && row_masks == nullptr)) return -1;
  if (B == 0) return 0;
  hipLaunchKernelGGL(fsm_sample_kernel, dim3(B), dim3(256), 0, stream, (const uint16_t*)logits, ldl,
                     (const uint32_t*)masks, state_mask, state, next_sep, next_tok, enum_tok, enum_next, E, sep_token,
                     done_state, tok_io, out_buf, out_len, done, pos, slot_id, row_map, max_out, V, inv_temp, seed,
                     copy_kind, (const uint32_t*)row_masks);
  return (int)hipGetLastError();
}

int sg_version() { return 1; }

}  // extern "C"
