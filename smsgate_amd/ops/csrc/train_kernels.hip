// smsgate_amd — fused elementwise kernels of the extractor's TRAINING step (gfx950).
//
// The training forward (models/train_ops.py) is plain PyTorch around hipBLASLt GEMMs
// and the SDPA flash kernels, but its elementwise glue was ~45 small kernels per layer
// (RMSNorm as pow / mean / rsqrt / mul / mul / cast, rotate-half RoPE as slices / mul /
// neg / cat per q and k, SiLU then mul), forward and backward: at the bench recipe
// (128 x ~60 tokens) over half of a step's GPU time went to re-reading the same
// activations between launches (scripts/train_step_profile.py).  These kernels do each
// group in one pass, forward and backward:
//
//   rms_fwd     y = bf16(x * rsqrt(mean(x^2) + eps) * w), rstd saved      (fp32 x, w)
//   rms_bwd     dx = r*(g) - x * r^3/H * sum(g*x) with g = dy*w;  dw partials per block
//   rope_split  qkv [R, (nh+2nkv)*D] -> q [B,nh,T,D], k, v [B,nkv,T,D] (rotate-half RoPE on
//               q and k in fp32 from the caller's cos / sin tables; optionally k / v
//               expanded to nh heads), and its adjoint (rotation by -theta, expanded
//               copies summed) from dq / dk / dv back to dqkv
//   swiglu      a = bf16(silu(g) * u) on gu = [gate | up], and dgu from da
//   attn_train  causal grouped-query attention over one training batch (T <= 192 rows,
//               D = 64): forward with the per-row log-sum-exp saved, backward in two
//               passes that recompute the probabilities (query rows -> dQ; key rows ->
//               dK / dV summed over the group's query heads).  SDPA's kernels made one
//               synchronous host-to-device copy per call (63 per step, the host could not
//               run ahead of the GPU: scripts/train_step_profile.py); these make none.
//
// One wave (64 lanes) per row for the norms (H <= 1024: 4 float4 per lane in
// registers); 8 bf16 per thread (16-B accesses) for SwiGLU; one lane per output element
// for RoPE.  fp32 arithmetic throughout, one rounding per stored bf16.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ float tk_bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t tk_f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

constexpr int RMS_MAXC = 4;  // float4 chunks per lane: H <= 64 * 4 * 4 = 1024

__global__ void __launch_bounds__(256) rms_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      uint16_t* __restrict__ y, float* __restrict__ rstd, int R,
                                                      int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const int nc = H >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * H);
  float4 v[RMS_MAXC];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < RMS_MAXC; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < nc ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    ss = fmaf(v[i].x, v[i].x, fmaf(v[i].y, v[i].y, fmaf(v[i].z, v[i].z, fmaf(v[i].w, v[i].w, ss))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float r = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd[row] = r;
  const float4* wr = reinterpret_cast<const float4*>(w);
  uint2* yr = reinterpret_cast<uint2*>(y + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < RMS_MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nc) {
      const float4 g = wr[c];
      yr[c] = make_uint2((uint32_t)tk_f2bf(v[i].x * r * g.x) | ((uint32_t)tk_f2bf(v[i].y * r * g.y) << 16),
                         (uint32_t)tk_f2bf(v[i].z * r * g.z) | ((uint32_t)tk_f2bf(v[i].w * r * g.w) << 16));
    }
  }
}

// Rows [blockIdx.x * rpb, +rpb) of dx; the block's dw partial (sum over its rows of
// dy * x * r) into dw_part[blockIdx.x][H].
__global__ void __launch_bounds__(256) rms_bwd_kernel(const uint16_t* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ w, const float* __restrict__ rstd,
                                                      float* __restrict__ dx, float* __restrict__ dw_part, int R,
                                                      int H, int rpb) {
  __shared__ float4 red[4][64 * RMS_MAXC];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nc = H >> 2;
  const float4* wr = reinterpret_cast<const float4*>(w);
  float4 wv[RMS_MAXC], acc[RMS_MAXC];
#pragma unroll
  for (int i = 0; i < RMS_MAXC; ++i) {
    const int c = lane + 64 * i;
    wv[i] = c < nc ? wr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  for (int row = r0 + wave; row < r1; row += 4) {
    const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * H);
    const uint2* dr = reinterpret_cast<const uint2*>(dy + (size_t)row * H);
    const float r = rstd[row];
    float4 xv[RMS_MAXC], gv[RMS_MAXC];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < RMS_MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
        xv[i] = xr[c];
        const uint2 u = dr[c];
        const float d0 = tk_bf2f((uint16_t)(u.x & 0xffffu)), d1 = tk_bf2f((uint16_t)(u.x >> 16));
        const float d2 = tk_bf2f((uint16_t)(u.y & 0xffffu)), d3 = tk_bf2f((uint16_t)(u.y >> 16));
        gv[i] = make_float4(d0 * wv[i].x, d1 * wv[i].y, d2 * wv[i].z, d3 * wv[i].w);
        dot = fmaf(gv[i].x, xv[i].x, fmaf(gv[i].y, xv[i].y, fmaf(gv[i].z, xv[i].z, fmaf(gv[i].w, xv[i].w, dot))));
        acc[i].x = fmaf(d0 * r, xv[i].x, acc[i].x);
        acc[i].y = fmaf(d1 * r, xv[i].y, acc[i].y);
        acc[i].z = fmaf(d2 * r, xv[i].z, acc[i].z);
        acc[i].w = fmaf(d3 * r, xv[i].w, acc[i].w);
      } else {
        xv[i] = gv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
    const float k = r * r * r * dot / (float)H;
    float4* dxr = reinterpret_cast<float4*>(dx + (size_t)row * H);
#pragma unroll
    for (int i = 0; i < RMS_MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nc)
        dxr[c] = make_float4(r * gv[i].x - k * xv[i].x, r * gv[i].y - k * xv[i].y, r * gv[i].z - k * xv[i].z,
                             r * gv[i].w - k * xv[i].w);
    }
  }
#pragma unroll
  for (int i = 0; i < RMS_MAXC; ++i) red[wave][lane + 64 * i] = acc[i];
  __syncthreads();
  float4* dp = reinterpret_cast<float4*>(dw_part + (size_t)blockIdx.x * H);
  for (int c = threadIdx.x; c < nc; c += 256) {
    const float4 a = red[0][c], b = red[1][c], e = red[2][c], f = red[3][c];
    dp[c] = make_float4((a.x + b.x) + (e.x + f.x), (a.y + b.y) + (e.y + f.y), (a.z + b.z) + (e.z + f.z),
                        (a.w + b.w) + (e.w + f.w));
  }
}

// One block of 64 x 4 threads per (row, 4 heads): lane j of a wave is output element j
// of head (blockIdx.y * 4 + wave) of row blockIdx.x.  dir = +1 forward (qkv -> q/k/v),
// -1 the adjoint (dq/dk/dv -> dqkv).  rep > 1 writes k / v expanded to nh heads (each kv
// head `rep` times: SDPA backends without grouped-query support), whose adjoint sums
// the rep copies' gradients.
template <int DIR>
__global__ void __launch_bounds__(256) rope_split_kernel(uint16_t* __restrict__ qkv, uint16_t* __restrict__ q,
                                                         uint16_t* __restrict__ k, uint16_t* __restrict__ v,
                                                         const float* __restrict__ cos_t,
                                                         const float* __restrict__ sin_t, int T, int nh, int nkv,
                                                         int rep) {
  constexpr int D = 64, HD = 32;
  const int row = blockIdx.x, wave = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int hh = blockIdx.y * 4 + wave;
  const int NH = nh + 2 * nkv;
  if (hh >= NH) return;
  const int b = row / T, t = row - b * T;
  uint16_t* src = qkv + (size_t)row * NH * D + hh * D;
  const int kvh = nkv * rep;  // heads of the k / v outputs
  uint16_t* dst;
  size_t hstride = (size_t)T * D;  // between consecutive heads of one batch row
  int copies = 1;
  bool rot = true;
  if (hh < nh) {
    dst = q + (((size_t)b * nh + hh) * T + t) * D;
  } else if (hh < nh + nkv) {
    dst = k + (((size_t)b * kvh + (hh - nh) * rep) * T + t) * D;
    copies = rep;
  } else {
    dst = v + (((size_t)b * kvh + (hh - nh - nkv) * rep) * T + t) * D;
    copies = rep;
    rot = false;
  }
  const int jj = j & (HD - 1);
  if (DIR > 0) {
    float o;
    if (rot) {
      const float c = cos_t[t * HD + jj], s = sin_t[t * HD + jj];
      const float x1 = tk_bf2f(src[jj]), x2 = tk_bf2f(src[jj + HD]);
      o = j < HD ? x1 * c - x2 * s : x2 * c + x1 * s;
    } else {
      o = tk_bf2f(src[j]);
    }
    const uint16_t ob = tk_f2bf(o);
    for (int r = 0; r < copies; ++r) dst[r * hstride + j] = ob;
  } else {  // adjoint: sum of the copies' gradients, then rotation by -theta
    if (rot) {
      const float c = cos_t[t * HD + jj], s = sin_t[t * HD + jj];
      float d1 = 0.f, d2 = 0.f;
      for (int r = 0; r < copies; ++r) {
        d1 += tk_bf2f(dst[r * hstride + jj]);
        d2 += tk_bf2f(dst[r * hstride + jj + HD]);
      }
      src[j] = tk_f2bf(j < HD ? d1 * c + d2 * s : d2 * c - d1 * s);
    } else {
      float d = 0.f;
      for (int r = 0; r < copies; ++r) d += tk_bf2f(dst[r * hstride + j]);
      src[j] = tk_f2bf(d);
    }
  }
}

__device__ __forceinline__ float tk_sigmoid(float g) { return __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// gu [R, 2I] = [gate | up]; 8 elements per thread
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ a,
                                                         int R, int I) {
  const int per_row = I >> 3;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)R * per_row) return;
  const int row = (int)(idx / per_row), c = (int)(idx - (long)row * per_row);
  const uint4 g4 = *reinterpret_cast<const uint4*>(gu + (size_t)row * 2 * I + 8 * c);
  const uint4 u4 = *reinterpret_cast<const uint4*>(gu + (size_t)row * 2 * I + I + 8 * c);
  const uint32_t gw[4] = {g4.x, g4.y, g4.z, g4.w}, uw[4] = {u4.x, u4.y, u4.z, u4.w};
  uint32_t ow[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float g0 = tk_bf2f((uint16_t)(gw[e] & 0xffffu)), g1 = tk_bf2f((uint16_t)(gw[e] >> 16));
    const float u0 = tk_bf2f((uint16_t)(uw[e] & 0xffffu)), u1 = tk_bf2f((uint16_t)(uw[e] >> 16));
    ow[e] = (uint32_t)tk_f2bf(g0 * tk_sigmoid(g0) * u0) | ((uint32_t)tk_f2bf(g1 * tk_sigmoid(g1) * u1) << 16);
  }
  *reinterpret_cast<uint4*>(a + (size_t)row * I + 8 * c) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const uint16_t* __restrict__ da,
                                                         const uint16_t* __restrict__ gu,
                                                         uint16_t* __restrict__ dgu, int R, int I) {
  const int per_row = I >> 3;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)R * per_row) return;
  const int row = (int)(idx / per_row), c = (int)(idx - (long)row * per_row);
  const uint4 g4 = *reinterpret_cast<const uint4*>(gu + (size_t)row * 2 * I + 8 * c);
  const uint4 u4 = *reinterpret_cast<const uint4*>(gu + (size_t)row * 2 * I + I + 8 * c);
  const uint4 d4 = *reinterpret_cast<const uint4*>(da + (size_t)row * I + 8 * c);
  const uint32_t gw[4] = {g4.x, g4.y, g4.z, g4.w}, uw[4] = {u4.x, u4.y, u4.z, u4.w}, dw[4] = {d4.x, d4.y, d4.z, d4.w};
  uint32_t og[4], ou[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float gg[2], uu[2], dd[2], rg[2], ru[2];
    gg[0] = tk_bf2f((uint16_t)(gw[e] & 0xffffu)); gg[1] = tk_bf2f((uint16_t)(gw[e] >> 16));
    uu[0] = tk_bf2f((uint16_t)(uw[e] & 0xffffu)); uu[1] = tk_bf2f((uint16_t)(uw[e] >> 16));
    dd[0] = tk_bf2f((uint16_t)(dw[e] & 0xffffu)); dd[1] = tk_bf2f((uint16_t)(dw[e] >> 16));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float s = tk_sigmoid(gg[h]);
      rg[h] = dd[h] * uu[h] * s * (1.f + gg[h] * (1.f - s));
      ru[h] = dd[h] * gg[h] * s;
    }
    og[e] = (uint32_t)tk_f2bf(rg[0]) | ((uint32_t)tk_f2bf(rg[1]) << 16);
    ou[e] = (uint32_t)tk_f2bf(ru[0]) | ((uint32_t)tk_f2bf(ru[1]) << 16);
  }
  *reinterpret_cast<uint4*>(dgu + (size_t)row * 2 * I + 8 * c) = make_uint4(og[0], og[1], og[2], og[3]);
  *reinterpret_cast<uint4*>(dgu + (size_t)row * 2 * I + I + 8 * c) = make_uint4(ou[0], ou[1], ou[2], ou[3]);
}

// ---- training attention ------------------------------------------------------
// q [B, nh, T, 64], k / v [B, nkv, T, 64] (bf16, rope_split's layout), o [B, T, nh*64]
// (the o-proj GEMM's input layout: no transpose copy), lse [B, nh, T] fp32.  Query head h
// reads kv head h / (nh / nkv).  One thread per row (T <= 256 = the block), the group's
// K and V staged in LDS as bf16 and read by every lane of a wave at the same address
// (LDS broadcast).  fp32 math; the causal mask is the loop bound.
constexpr int AT_D = 64;
constexpr int AT_MAXT = 192;

__device__ __forceinline__ void at_row_f32(const uint16_t* p, float* out) {
#pragma unroll
  for (int c = 0; c < AT_D / 8; ++c) {
    const uint4 u = reinterpret_cast<const uint4*>(p)[c];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      out[8 * c + 2 * e] = tk_bf2f((uint16_t)(w[e] & 0xffffu));
      out[8 * c + 2 * e + 1] = tk_bf2f((uint16_t)(w[e] >> 16));
    }
  }
}

__device__ __forceinline__ float at_dot(const float* a, const uint16_t* b_lds) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < AT_D / 8; ++c) {
    const uint4 u = reinterpret_cast<const uint4*>(b_lds)[c];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s = fmaf(a[8 * c + 2 * e], tk_bf2f((uint16_t)(w[e] & 0xffffu)), s);
      s = fmaf(a[8 * c + 2 * e + 1], tk_bf2f((uint16_t)(w[e] >> 16)), s);
    }
  }
  return s;
}

__device__ __forceinline__ void at_axpy(float* y, float a, const uint16_t* x_lds) {
#pragma unroll
  for (int c = 0; c < AT_D / 8; ++c) {
    const uint4 u = reinterpret_cast<const uint4*>(x_lds)[c];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      y[8 * c + 2 * e] = fmaf(a, tk_bf2f((uint16_t)(w[e] & 0xffffu)), y[8 * c + 2 * e]);
      y[8 * c + 2 * e + 1] = fmaf(a, tk_bf2f((uint16_t)(w[e] >> 16)), y[8 * c + 2 * e + 1]);
    }
  }
}

__device__ __forceinline__ void at_store_bf16(uint16_t* p, const float* v, float scale) {
#pragma unroll
  for (int c = 0; c < AT_D / 8; ++c) {
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)tk_f2bf(v[8 * c + 2 * e] * scale) | ((uint32_t)tk_f2bf(v[8 * c + 2 * e + 1] * scale) << 16);
    reinterpret_cast<uint4*>(p)[c] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// stage `rows` rows of 64 bf16 (row stride `ld` elements) into LDS
__device__ __forceinline__ void at_stage(uint16_t* dst, const uint16_t* src, int rows, size_t ld) {
  for (int i = threadIdx.x; i < rows * (AT_D / 8); i += blockDim.x) {
    const int r = i / (AT_D / 8), c = i % (AT_D / 8);
    reinterpret_cast<uint4*>(dst + r * AT_D)[c] = reinterpret_cast<const uint4*>(src + (size_t)r * ld)[c];
  }
}

__global__ void __launch_bounds__(256) attn_train_fwd_kernel(const uint16_t* __restrict__ q,
                                                             const uint16_t* __restrict__ k,
                                                             const uint16_t* __restrict__ v, uint16_t* __restrict__ o,
                                                             float* __restrict__ lse, int T, int nh, int nkv,
                                                             float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t ks[AT_MAXT * AT_D];
  __shared__ __attribute__((aligned(16))) uint16_t vs[AT_MAXT * AT_D];
  const int b = blockIdx.x / nh, h = blockIdx.x % nh, g = h / (nh / nkv);
  const size_t kvo = ((size_t)b * nkv + g) * T * AT_D;
  at_stage(ks, k + kvo, T, AT_D);
  at_stage(vs, v + kvo, T, AT_D);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= T) return;
  float qr[AT_D], acc[AT_D];
  at_row_f32(q + (((size_t)b * nh + h) * T + t) * AT_D, qr);
#pragma unroll
  for (int d = 0; d < AT_D; ++d) {
    qr[d] *= scale;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j <= t; ++j) {
    const float sc = at_dot(qr, ks + j * AT_D);
    if (sc > m) {
      const float corr = __expf(m - sc);
      l *= corr;
#pragma unroll
      for (int d = 0; d < AT_D; ++d) acc[d] *= corr;
      m = sc;
    }
    const float p = __expf(sc - m);
    l += p;
    at_axpy(acc, p, vs + j * AT_D);
  }
  at_store_bf16(o + ((size_t)b * T + t) * nh * AT_D + h * AT_D, acc, 1.f / l);
  lse[((size_t)b * nh + h) * T + t] = m + __logf(l);
}

// Backward, two kernels (one thread per row each; splitting them keeps every thread's
// live set under the VGPR file: a fused pass spilled).  ds_tj = p_tj (do_t . v_j - D_t),
// D_t = do_t . o_t, p_tj = exp(scale q_t . k_j - lse_t).
// A (block = batch x query head, thread = query row t): dq_t = scale sum_j ds_tj k_j, and
//   D_t into dsum [B, nh, T] for B.
__global__ void __launch_bounds__(256) attn_train_bwd_q_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const uint16_t* __restrict__ o, const float* __restrict__ lse, const uint16_t* __restrict__ dout,
    uint16_t* __restrict__ dq, float* __restrict__ dsum, int T, int nh, int nkv, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t ks[AT_MAXT * AT_D];
  __shared__ __attribute__((aligned(16))) uint16_t vs[AT_MAXT * AT_D];
  const int b = blockIdx.x / nh, h = blockIdx.x % nh, g = h / (nh / nkv);
  const size_t kvo = ((size_t)b * nkv + g) * T * AT_D;
  at_stage(ks, k + kvo, T, AT_D);
  at_stage(vs, v + kvo, T, AT_D);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= T) return;
  const size_t row = ((size_t)b * nh + h) * T + t;  // [B, nh, T] index
  const size_t orow = ((size_t)b * T + t) * nh * AT_D + h * AT_D;
  float qt[AT_D], dt[AT_D], acc[AT_D];
  at_row_f32(o + orow, acc);  // o_t (scratch for D_t)
  at_row_f32(dout + orow, dt);
  float D = 0.f;
#pragma unroll
  for (int d = 0; d < AT_D; ++d) D = fmaf(dt[d], acc[d], D);
  dsum[row] = D;
  at_row_f32(q + row * AT_D, qt);
#pragma unroll
  for (int d = 0; d < AT_D; ++d) {
    qt[d] *= scale;
    acc[d] = 0.f;
  }
  const float L = lse[row];
  for (int j = 0; j <= t; ++j) {
    const float p = __expf(at_dot(qt, ks + j * AT_D) - L);
    const float ds = p * (at_dot(dt, vs + j * AT_D) - D);
    at_axpy(acc, ds, ks + j * AT_D);
  }
  at_store_bf16(dq + row * AT_D, acc, scale);
}

// B (block = batch x kv head, thread = key row j): over the group's query heads,
// dv_j += sum_{t>=j} p_tj do_t and dk_j += scale sum_{t>=j} ds_tj q_t.  k_j / v_j stay
// packed bf16 in registers, q / dO / lse / D of the current head in LDS (broadcast reads).
__global__ void __launch_bounds__(256) attn_train_bwd_kv_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const float* __restrict__ lse, const float* __restrict__ dsum, const uint16_t* __restrict__ dout,
    uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, int T, int nh, int nkv, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t qs[AT_MAXT * AT_D];
  __shared__ __attribute__((aligned(16))) uint16_t dos[AT_MAXT * AT_D];
  __shared__ float ls[AT_MAXT], Ds[AT_MAXT];
  const int b = blockIdx.x / nkv, g = blockIdx.x % nkv, rep = nh / nkv;
  const size_t kvo = ((size_t)b * nkv + g) * T * AT_D;
  const int j = threadIdx.x;
  uint32_t kp[AT_D / 2], vp[AT_D / 2];
  float dkj[AT_D], dvj[AT_D];
  if (j < T) {
#pragma unroll
    for (int c = 0; c < AT_D / 8; ++c) {
      const uint4 ku = reinterpret_cast<const uint4*>(k + kvo + (size_t)j * AT_D)[c];
      const uint4 vu = reinterpret_cast<const uint4*>(v + kvo + (size_t)j * AT_D)[c];
      kp[4 * c] = ku.x; kp[4 * c + 1] = ku.y; kp[4 * c + 2] = ku.z; kp[4 * c + 3] = ku.w;
      vp[4 * c] = vu.x; vp[4 * c + 1] = vu.y; vp[4 * c + 2] = vu.z; vp[4 * c + 3] = vu.w;
    }
  }
#pragma unroll
  for (int d = 0; d < AT_D; ++d) dkj[d] = dvj[d] = 0.f;
  for (int r = 0; r < rep; ++r) {
    const int h = g * rep + r;
    const size_t qo = ((size_t)b * nh + h) * T;
    __syncthreads();  // the previous head's rows are no longer read
    at_stage(qs, q + qo * AT_D, T, AT_D);
    at_stage(dos, dout + (size_t)b * T * nh * AT_D + h * AT_D, T, (size_t)nh * AT_D);
    for (int i = threadIdx.x; i < T; i += blockDim.x) {
      ls[i] = lse[qo + i];
      Ds[i] = dsum[qo + i];
    }
    __syncthreads();
    if (j >= T) continue;
    for (int t = j; t < T; ++t) {
      const uint16_t* qr = qs + t * AT_D;
      const uint16_t* dr = dos + t * AT_D;
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int c = 0; c < AT_D / 8; ++c) {
        const uint4 qu = reinterpret_cast<const uint4*>(qr)[c];
        const uint4 du = reinterpret_cast<const uint4*>(dr)[c];
        const uint32_t qw[4] = {qu.x, qu.y, qu.z, qu.w}, dw[4] = {du.x, du.y, du.z, du.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t kk = kp[4 * c + e], vv = vp[4 * c + e];
          s = fmaf(tk_bf2f((uint16_t)(qw[e] & 0xffffu)), tk_bf2f((uint16_t)(kk & 0xffffu)), s);
          s = fmaf(tk_bf2f((uint16_t)(qw[e] >> 16)), tk_bf2f((uint16_t)(kk >> 16)), s);
          dpv = fmaf(tk_bf2f((uint16_t)(dw[e] & 0xffffu)), tk_bf2f((uint16_t)(vv & 0xffffu)), dpv);
          dpv = fmaf(tk_bf2f((uint16_t)(dw[e] >> 16)), tk_bf2f((uint16_t)(vv >> 16)), dpv);
        }
      }
      const float p = __expf(scale * s - ls[t]);
      const float ds = p * (dpv - Ds[t]) * scale;
#pragma unroll
      for (int c = 0; c < AT_D / 8; ++c) {
        const uint4 qu = reinterpret_cast<const uint4*>(qr)[c];
        const uint4 du = reinterpret_cast<const uint4*>(dr)[c];
        const uint32_t qw[4] = {qu.x, qu.y, qu.z, qu.w}, dw[4] = {du.x, du.y, du.z, du.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dvj[8 * c + 2 * e] = fmaf(p, tk_bf2f((uint16_t)(dw[e] & 0xffffu)), dvj[8 * c + 2 * e]);
          dvj[8 * c + 2 * e + 1] = fmaf(p, tk_bf2f((uint16_t)(dw[e] >> 16)), dvj[8 * c + 2 * e + 1]);
          dkj[8 * c + 2 * e] = fmaf(ds, tk_bf2f((uint16_t)(qw[e] & 0xffffu)), dkj[8 * c + 2 * e]);
          dkj[8 * c + 2 * e + 1] = fmaf(ds, tk_bf2f((uint16_t)(qw[e] >> 16)), dkj[8 * c + 2 * e + 1]);
        }
      }
    }
  }
  if (j < T) {
    at_store_bf16(dk + kvo + (size_t)j * AT_D, dkj, 1.f);
    at_store_bf16(dv + kvo + (size_t)j * AT_D, dvj, 1.f);
  }
}

}  // namespace

extern "C" {

int sg_rms_fwd(const void* x, const void* w, void* y, void* rstd, int R, int H, float eps, hipStream_t st) {
  if (H % 4 || H > 64 * 4 * RMS_MAXC || R <= 0) return 1;
  rms_fwd_kernel<<<dim3((R + 3) / 4), dim3(256), 0, st>>>((const float*)x, (const float*)w, (uint16_t*)y,
                                                          (float*)rstd, R, H, eps);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_rms_bwd(const void* dy, const void* x, const void* w, const void* rstd, void* dx, void* dw_part, int R,
               int H, int rpb, hipStream_t st) {
  if (H % 4 || H > 64 * 4 * RMS_MAXC || R <= 0 || rpb <= 0) return 1;
  rms_bwd_kernel<<<dim3((R + rpb - 1) / rpb), dim3(256), 0, st>>>(
      (const uint16_t*)dy, (const float*)x, (const float*)w, (const float*)rstd, (float*)dx, (float*)dw_part, R, H,
      rpb);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_rope_split(int dir, void* qkv, void* q, void* k, void* v, const void* cos_t, const void* sin_t, int B, int T,
                  int nh, int nkv, int D, int rep, hipStream_t st) {
  if (D != 64 || B <= 0 || T <= 0 || rep < 1) return 1;
  const dim3 grid(B * T, (nh + 2 * nkv + 3) / 4);
  if (dir > 0)
    rope_split_kernel<1><<<grid, dim3(256), 0, st>>>((uint16_t*)qkv, (uint16_t*)q, (uint16_t*)k, (uint16_t*)v,
                                                     (const float*)cos_t, (const float*)sin_t, T, nh, nkv, rep);
  else
    rope_split_kernel<-1><<<grid, dim3(256), 0, st>>>((uint16_t*)qkv, (uint16_t*)q, (uint16_t*)k, (uint16_t*)v,
                                                      (const float*)cos_t, (const float*)sin_t, T, nh, nkv, rep);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_swiglu_fwd(const void* gu, void* a, int R, int I, hipStream_t st) {
  if (I % 8 || R <= 0) return 1;
  const long n = (long)R * (I / 8);
  swiglu_fwd_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>((const uint16_t*)gu, (uint16_t*)a, R, I);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_swiglu_bwd(const void* da, const void* gu, void* dgu, int R, int I, hipStream_t st) {
  if (I % 8 || R <= 0) return 1;
  const long n = (long)R * (I / 8);
  swiglu_bwd_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>((const uint16_t*)da,
                                                                             (const uint16_t*)gu, (uint16_t*)dgu, R, I);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_attn_train_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int T, int nh, int nkv,
                      float scale, hipStream_t st) {
  if (T <= 0 || T > AT_MAXT || B <= 0 || nkv <= 0 || nh % nkv) return 1;
  attn_train_fwd_kernel<<<dim3(B * nh), dim3(256), 0, st>>>((const uint16_t*)q, (const uint16_t*)k,
                                                            (const uint16_t*)v, (uint16_t*)o, (float*)lse, T, nh, nkv,
                                                            scale);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int sg_attn_train_bwd(const void* q, const void* k, const void* v, const void* o, const void* lse, const void* dout,
                      void* dq, void* dk, void* dv, void* dsum, int B, int T, int nh, int nkv, float scale,
                      hipStream_t st) {
  if (T <= 0 || T > AT_MAXT || B <= 0 || nkv <= 0 || nh % nkv) return 1;
  attn_train_bwd_q_kernel<<<dim3(B * nh), dim3(256), 0, st>>>(
      (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)o, (const float*)lse,
      (const uint16_t*)dout, (uint16_t*)dq, (float*)dsum, T, nh, nkv, scale);
  if (hipGetLastError() != hipSuccess) return 2;
  attn_train_bwd_kv_kernel<<<dim3(B * nkv), dim3(256), 0, st>>>(
      (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const float*)lse, (const float*)dsum,
      (const uint16_t*)dout, (uint16_t*)dk, (uint16_t*)dv, T, nh, nkv, scale);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
